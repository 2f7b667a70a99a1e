# round-3 session 2: the look-back run by the first wave that needs the offset (CPK_SP_LBANY)
V=build/variants
tools/gpu_steps.sh \
 "200|r3U_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 180 python tools/quick_bench.py $V/cur.so@0 $V/lb1.so@0 $V/cur.so@0 $V/lb1.so@0"
