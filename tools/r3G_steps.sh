# round-3 session 2: a short chunk's steps spread over the four waves (CPK_SP_EVEN), mixed 4-256 KiB pieces
V=build/variants
tools/gpu_steps.sh \
 "300|r3G_mixed|QB_MIXED=1 QB_N=65536 QB_CFG=3,2 timeout -k 10 280 python tools/quick_bench.py $V/sp_head.so@4 $V/sp_head.so@0 $V/sp_even.so@0 $V/sp_even.so@4 $V/sp_head.so@0 $V/sp_even.so@0" \
 "200|r3G_small|QB_W=1024 QB_N=524288 QB_CFG=2,3 timeout -k 10 180 python tools/quick_bench.py $V/sp_head.so@0 $V/sp_even.so@0 $V/sp_head.so@4" \
 "200|r3G_uni|QB_N=131072 QB_CFG=2,3 timeout -k 10 180 python tools/quick_bench.py $V/sp_head.so@0 $V/sp_even.so@0 $V/sp_head.so@0 $V/sp_even.so@0"
