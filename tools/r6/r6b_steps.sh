#!/bin/bash
# round 6: GPU suite (capacity guard, dense-window counters, lost-flag count),
# passByBytes replay with the host phase trace, small-decode launch overhead
tools/gpu_steps.sh \
 "600|r6b_gpu_tests|python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread" \
 "200|r6b_pbb|g++ -O2 -std=c++17 -pthread -Iinclude tests/cpp/pass_by_bytes.cpp oracle/packed_oracle.c -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,\$PWD/capnproto-java_amd/lib -o gpurun_out/pbb && CPK_HOST_TRACE=1 gpurun_out/pbb 8192 50" \
 "200|r6b_launch|python tools/r6/launch_overhead.py"
