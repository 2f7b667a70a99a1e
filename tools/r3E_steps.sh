# round-3 session 2: 8 waves x 16 steps per chunk (a wave's output fits a 4 KiB ring), reload form at 6 waves/SIMD
V=build/variants
tools/gpu_steps.sh \
 "300|r3E_ab|QB_N=131072 QB_CFG=2,4,3 timeout -k 10 280 python tools/quick_bench.py $V/sp_base.so@0 $V/sp_w8r3.so@0 $V/sp_w8r3g8.so@0 $V/sp_w8k2.so@0 $V/sp_rl6.so@0 $V/sp_base.so@0 $V/sp_w8r3.so@0"
