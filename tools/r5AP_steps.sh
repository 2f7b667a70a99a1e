# round-5 final tree (one-path expansion, LDS-address reads, odd-block stores, plain 8-byte stores, rotated visited bits, 32-bit tags): GPU suite, bench lines configs 2/3/4, kernel stats +
# HBM traffic, SQ counters of the config-2 kernels (rocprofv3)
B="python3 bench.py --steps 3 --warmup 1 --no-cpu"
tools/gpu_steps.sh \
 "400|r5AP_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r5AP_bench_config2|python bench.py --config 2 --steps 10 --warmup 2" \
 "200|r5AP_bench_config3|python bench.py --config 3 --steps 10 --warmup 2" \
 "200|r5AP_bench_config4|python bench.py --config 4 --steps 10 --warmup 2" \
 "300|r5AP_prof2|tools/profile.sh r5AP_c2 sq -- $B --config 2" \
 "300|r5AP_prof3|tools/profile.sh r5AP_c3 -- $B --config 3" \
 "300|r5AP_prof4|tools/profile.sh r5AP_c4 -- $B --config 4"
