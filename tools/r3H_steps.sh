# round-3 session 2: single pass vs two passes by piece size (the device gate's threshold), 1 GiB per batch
V=build/variants
tools/gpu_steps.sh \
 "120|r3H_w2048|QB_W=2048 QB_N=65536 QB_CFG=2,3 timeout -k 10 110 python tools/quick_bench.py $V/sp_head.so@4 $V/sp_head.so@0 $V/sp_even.so@0" \
 "120|r3H_w4096|QB_W=4096 QB_N=32768 QB_CFG=2,3 timeout -k 10 110 python tools/quick_bench.py $V/sp_head.so@4 $V/sp_head.so@0 $V/sp_even.so@0" \
 "120|r3H_w8192|QB_W=8192 QB_N=16384 QB_CFG=2,3 timeout -k 10 110 python tools/quick_bench.py $V/sp_head.so@4 $V/sp_head.so@0 $V/sp_even.so@0" \
 "120|r3H_w16384|QB_W=16384 QB_N=8192 QB_CFG=2,3 timeout -k 10 110 python tools/quick_bench.py $V/sp_head.so@4 $V/sp_head.so@0 $V/sp_even.so@0" \
 "120|r3H_w8192b|QB_W=8192 QB_N=131072 QB_CFG=2,3 timeout -k 10 110 python tools/quick_bench.py $V/sp_head.so@4 $V/sp_head.so@0"
