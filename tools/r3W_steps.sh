# round-3: config-4 bench line with the sparse form's masked reload; smoke
tools/gpu_steps.sh \
 "200|r3W_bench_config4|python bench.py --config 4 --steps 10 --warmup 2" \
 "200|r3W_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
V=build/variants
tools/gpu_steps.sh \
 "200|r3W_dec8|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 180 python tools/quick_bench.py $V/gate2.so@5:CPK_DECODER=1 $V/d8.so@5:CPK_DECODER=1 $V/d7r768.so@5:CPK_DECODER=1 $V/gate2.so@5:CPK_DECODER=1 $V/d8.so@5:CPK_DECODER=1"
