# round-5 tree after message batches went back to the plain block map: GPU
# suite, config-3 bench line, config-3 kernel stats + HBM traffic
B="python3 bench.py --steps 3 --warmup 1 --no-cpu"
tools/gpu_steps.sh \
 "400|r5F2_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r5F2_bench_config3|python bench.py --config 3 --steps 10 --warmup 2" \
 "300|r5F2_prof3|tools/profile.sh r5F2_c3 -- $B --config 3"
