# round-3: encoder B -- selectors read a pair ahead (CPK_SP_LUTPF), puts for every lane (CPK_SP_PUTALL)
V=build/variants
tools/gpu_steps.sh \
 "300|r3g_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/pf0.so@0 $V/pf1.so@0 $V/pf1all.so@0 $V/pf0.so@0 $V/pf1.so@0 $V/pf1all.so@0"
