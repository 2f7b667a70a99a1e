# round-3: mixed piece sizes (config-3 segment sizes) single pass with units
# vs two passes; message read threshold
tools/gpu_steps.sh \
 "200|r3e_mixed|QB_MIXED=1 QB_N=131072 QB_CFG=2,3 timeout -k 10 180 python tools/quick_bench.py capnproto-java_amd/lib/libcapnp_packed_hip.so@0 capnproto-java_amd/lib/libcapnp_packed_hip.so@4 capnproto-java_amd/lib/libcapnp_packed_hip.so@0" \
 "120|r3e_probe|g++ -O2 -std=c++17 -pthread -Iinclude tools/threshold_probe.cpp oracle/packed_oracle.c -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,$PWD/capnproto-java_amd/lib -o gpurun_out/probe && gpurun_out/probe" \
 "200|r3e_rm|python -u -m pytest tests/test_gpu_read_message.py tests/test_cpp_mirror.py -m gpu -q --timeout 150 --timeout-method thread"
