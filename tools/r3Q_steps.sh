# round-3 session 2: one large piece through the host forms (single-chunk transfers pipelined; few large pieces decoded as a stream)
V=build/variants
tools/gpu_steps.sh \
 "300|r3Q_gpu_tests_all|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "300|r3Q_gpu_tests_host|python -u -m pytest tests/test_gpu_parity.py -k 'few_large or host or large_message' -x -q --timeout 150 --timeout-method thread"
