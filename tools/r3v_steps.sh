# round-3: single pass with 4096-word chunks (units) at 4 workgroups per CU (CPK_SP_CS=64, CPK_SP_WPE=4)
V=build/variants
tools/gpu_steps.sh \
 "300|r3v_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/c128.so@5 $V/c64w4.so@5 $V/c128.so@5 $V/c64w4.so@5" \
 "200|r3v_big|QB_W=65536 QB_N=16384 QB_CFG=2 timeout -k 10 180 python tools/quick_bench.py $V/c128.so@5 $V/c64w4.so@5"
