# round-3 session 2: one large piece through the host forms (single-chunk transfers pipelined; few large pieces decoded as a stream)
V=build/variants
tools/gpu_steps.sh \
 "200|r3Q_one_piece|timeout -k 10 180 python tools/one_piece_host_bench.py $V/cur.so $V/hp.so $V/cur.so $V/hp.so" \
 "300|r3Q_gpu_tests_host|python -u -m pytest tests/test_gpu_parity.py -k 'few_large or host' -x -q --timeout 150 --timeout-method thread"
