# round-3 session 2: single-slot host forms with pipelined copies (read_message_host, decode_stream_host)
tools/gpu_steps.sh \
 "200|r3T_read_message|timeout -k 10 180 python tools/msg_read_bench.py 1 4 16 64 256" \
 "300|r3T_gpu_tests_host|python -u -m pytest tests/test_gpu_read_message.py tests/test_gpu_stream.py tests/test_cpp_mirror.py -x -q --timeout 150 --timeout-method thread" \
 "400|r3T_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread"
