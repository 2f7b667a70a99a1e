# round-3 A/B: units encoder with early exit-state publication (large pieces,
# 64 KiB pieces), single-message write/read latency probe
tools/gpu_steps.sh \
 "200|r3d_big|QB_W=65536 QB_N=16384 QB_CFG=2,3 timeout -k 10 180 python tools/quick_bench.py build/variants/base.so@0 capnproto-java_amd/lib/libcapnp_packed_hip.so@0 capnproto-java_amd/lib/libcapnp_packed_hip.so@4" \
 "200|r3d_ab|tools/ab.sh 2,4 build/variants/base.so@0 capnproto-java_amd/lib/libcapnp_packed_hip.so@0" \
 "120|r3d_probe|g++ -O2 -std=c++17 -pthread -Iinclude tools/threshold_probe.cpp oracle/packed_oracle.c -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,$PWD/capnproto-java_amd/lib -o gpurun_out/probe && gpurun_out/probe" \
 "300|r3d_tests|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_shapes.py tests/test_gpu_read_message.py -m gpu -q --timeout 150 --timeout-method thread"
