# round-3 session 2: dynamic offset fetch (CPK_SP_DYN) with and without the reload form; phase shares
V=build/variants
tools/gpu_steps.sh \
 "300|r3C_ab|QB_N=131072 QB_CFG=2,4,3 timeout -k 10 280 python tools/quick_bench.py $V/sp_base.so@0 $V/sp_dyn.so@0 $V/sp_rl6y.so@0 $V/sp_rl5y.so@0 $V/sp_rl6.so@0 $V/sp_base.so@0 $V/sp_rl6y.so@0" \
 "200|r3C_phase|python tools/phase_stats.py 2 65536 $V/stats.so && python tools/phase_stats.py 2 65536 $V/stats_rl6y.so"
