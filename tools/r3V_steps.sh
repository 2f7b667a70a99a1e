# round-3 session 2: the two-pass encoder's size pass with the roles as scalar mask algebra (CPK_E4_MASKROLES)
V=build/variants
tools/gpu_steps.sh \
 "200|r3V_ab|QB_N=131072 QB_CFG=3,2,4 timeout -k 10 180 python tools/quick_bench.py $V/mr0.so@4 $V/mr1.so@4 $V/mr0.so@4 $V/mr1.so@4" \
 "200|r3V_mixed|QB_MIXED=1 QB_N=65536 QB_CFG=3,2 timeout -k 10 180 python tools/quick_bench.py $V/mr0.so@5 $V/mr1.so@5 $V/mr0.so@5 $V/mr1.so@5" \
 "400|r3V_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r3V_bench_config3|python bench.py --config 3 --steps 10 --warmup 2 --no-cpu"
