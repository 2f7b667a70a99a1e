# round-3 session 2: next unit's ticket taken mid-B by wave 0 and its lines touched into L2 (CPK_SP_L2PF)
V=build/variants
tools/gpu_steps.sh \
 "300|r3K_ab|QB_N=131072 QB_CFG=2,4,3 timeout -k 10 280 python tools/quick_bench.py $V/cur.so@0 $V/pf16.so@0 $V/pf8.so@0 $V/pf24.so@0 $V/pf16n.so@0 $V/cur.so@0 $V/pf16.so@0"
