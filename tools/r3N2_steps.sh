# round-3 session 2: the sparse form's reload distance (CPK_SP_BPF step pairs ahead)
V=build/variants
tools/gpu_steps.sh \
 "200|r3N2_bpf|QB_N=131072 QB_CFG=4 timeout -k 10 180 python tools/quick_bench.py $V/cur.so@5 $V/bpf1.so@5 $V/bpf3.so@5 $V/bpf4.so@5 $V/cur.so@5 $V/bpf3.so@5 $V/bpf4.so@5"
