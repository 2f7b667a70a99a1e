# round-3: the device gate sends like-sized pieces over one chunk to the single pass (units)
L=capnproto-java_amd/lib/libcapnp_packed_hip.so
tools/gpu_steps.sh \
 "400|r3m_tests|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r3m_big|QB_W=65536 QB_N=16384 QB_CFG=2,3,4 timeout -k 10 180 python tools/quick_bench.py $L@5 $L@4 $L@0 $L@5" \
 "200|r3m_ab|QB_N=131072 QB_CFG=2,4 timeout -k 10 180 python tools/quick_bench.py $L@5 $L@4 $L@0"
