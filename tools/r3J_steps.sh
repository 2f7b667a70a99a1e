# round-3 session 2: ablations of the single pass's B phase (timing only; output wrong by design)
V=build/variants
tools/gpu_steps.sh \
 "300|r3J_abl|QB_N=131072 QB_CFG=2,3 timeout -k 10 280 python tools/quick_bench.py $V/cur.so@0 $V/abl1.so@0 $V/abl2.so@0 $V/abl4.so@0 $V/abl8.so@0 $V/abl15.so@0 $V/cur.so@0"
