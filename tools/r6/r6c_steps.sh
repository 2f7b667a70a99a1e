#!/bin/bash
# round 6: single-message host path after the gate fix (huge pieces -> single
# pass), one-workgroup reader bound A/B; GPU suite
g++ -O2 -std=c++17 -pthread -Iinclude tests/cpp/pass_by_bytes.cpp oracle/packed_oracle.c -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,$PWD/capnproto-java_amd/lib -o gpurun_out/pbb || exit 1
tools/gpu_steps.sh \
 "200|r6c_pbb|CPK_HOST_TRACE=1 gpurun_out/pbb 8192 50" \
 "200|r6c_pbb_mw256|CPK_RM_MW_MAX_KB=256 gpurun_out/pbb 8192 50" \
 "200|r6c_pbb_mw128|CPK_RM_MW_MAX_KB=128 gpurun_out/pbb 8192 50" \
 "600|r6c_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread"
tools/gpu_steps.sh "300|r6c_mall_pipe|python tools/r6/mall_pipeline.py"
