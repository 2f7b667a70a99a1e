# round-3: encoder B re-reading its words (CPK_SP_RELOAD) for a 4-workgroup register budget (CPK_SP_WPE=4)
V=build/variants
tools/gpu_steps.sh \
 "300|r3k_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/r0w3.so@0 $V/r0w4.so@0 $V/r1w4.so@0 $V/r1w4d1.so@0 $V/r1w3.so@0 $V/r0w3.so@0 $V/r1w4.so@0"
