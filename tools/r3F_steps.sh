# round-3 session 2: next unit's ticket + words taken at the end of B (CPK_SP_PF)
V=build/variants
tools/gpu_steps.sh \
 "300|r3F_ab|QB_N=131072 QB_CFG=2,4,3 timeout -k 10 280 python tools/quick_bench.py $V/sp_head.so@0 $V/sp_base2.so@0 $V/sp_pf.so@0 $V/sp_head.so@0 $V/sp_pf.so@0" \
 "200|r3F_big|QB_W=65536 QB_N=16384 QB_CFG=2,3 timeout -k 10 180 python tools/quick_bench.py $V/sp_head.so@0 $V/sp_pf.so@0"
