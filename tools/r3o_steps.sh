# round-3: encoder look-back's first poll issued before B (CPK_SP_LBPF)
V=build/variants
tools/gpu_steps.sh \
 "200|r3o_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 180 python tools/quick_bench.py $V/lb0.so@0 $V/lb1.so@0 $V/lb0.so@0 $V/lb1.so@0" \
 "200|r3o_big|QB_W=65536 QB_N=16384 QB_CFG=2 timeout -k 10 180 python tools/quick_bench.py $V/lb0.so@0 $V/lb1.so@0"
