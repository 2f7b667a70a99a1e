# round-3 session 2: device cpk_decode_batch of a few large pieces via the parallel stream decoder
V=build/variants
tools/gpu_steps.sh \
 "300|r3P_gpu_tests_new|python -u -m pytest tests/test_gpu_parity.py -k 'few_large' -x -q --timeout 150 --timeout-method thread" \
 "400|r3P_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r3P_one_piece|timeout -k 10 180 python tools/one_piece_host_bench.py $V/hp2.so $V/fl.so" \
 "200|r3P_bench_default|python bench.py --no-cpu"
