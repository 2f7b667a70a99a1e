# round-3 session 2: upcoming units' lines touched into L2 from a separate slice counter (CPK_SP_L2PF=2, no reservation)
V=build/variants
tools/gpu_steps.sh \
 "300|r3L_ab|QB_N=131072 QB_CFG=2,4,3 timeout -k 10 280 python tools/quick_bench.py $V/cur.so@0 $V/pg16.so@0 $V/pg4.so@0 $V/pg28.so@0 $V/cur.so@0 $V/pg16.so@0"
