#!/bin/bash
# round 6: cpk_ctx_take_error through the pinned read-back (the host encode
# paths call it once per call): GPU suite, then the passByBytes replay with
# the library before (build/before) and after, interleaved
g++ -O2 -std=c++17 -pthread -Iinclude tests/cpp/pass_by_bytes.cpp oracle/packed_oracle.c -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,$PWD/capnproto-java_amd/lib -o gpurun_out/pbb || exit 1
tools/gpu_steps.sh \
 "600|r6z11_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r6z11_pbb_before1|LD_LIBRARY_PATH=$PWD/build/before gpurun_out/pbb 8192 50" \
 "200|r6z11_pbb_after1|gpurun_out/pbb 8192 50" \
 "200|r6z11_pbb_before2|LD_LIBRARY_PATH=$PWD/build/before gpurun_out/pbb 8192 50" \
 "200|r6z11_pbb_after2|gpurun_out/pbb 8192 50"
