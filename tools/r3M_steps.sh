# round-3 session 2: decoder ablations (timing only; output wrong by design): no stores, no expansion, no map walk
V=build/variants
tools/gpu_steps.sh \
 "300|r3M_dabl|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/cur.so@5 $V/dabl1.so@5:CPK_DECODER=1 $V/dabl2.so@5:CPK_DECODER=1 $V/dabl4.so@5:CPK_DECODER=1 $V/dabl6.so@5:CPK_DECODER=1 $V/cur.so@5:CPK_DECODER=1"
