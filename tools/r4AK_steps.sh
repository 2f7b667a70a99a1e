# round-4 late tree (emit pass on the size pass's rows): message-encode
# parity, bench line config 3, config-3 kernel stats + HBM traffic (rocprofv3)
B="python3 bench.py --steps 3 --warmup 1 --no-cpu"
tools/gpu_steps.sh \
 "200|r4AK_msg_tests|python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k encode_messages" \
 "200|r4AK_bench_config3|python bench.py --config 3 --steps 10 --warmup 2" \
 "300|r4AK_prof3|tools/profile.sh r4AK_c3 -- $B --config 3"
