#!/bin/bash
# round 6: decoder with two walks per lane (chunk walk: w2; chunk + block-map
# walks: w22) against the tree, full size, three runs per arm interleaved;
# passByBytes with the host read bound at 128 KiB; GPU suite
V=build/variants
g++ -O2 -std=c++17 -pthread -Iinclude tests/cpp/pass_by_bytes.cpp oracle/packed_oracle.c -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,$PWD/capnproto-java_amd/lib -o gpurun_out/pbb || exit 1
tools/gpu_steps.sh \
 "400|r6d_w2_ab|QB_N=1048576 QB_CFG=2,3,4 python tools/quick_bench.py $V/base6.so@5 $V/w2.so@5 $V/w22.so@5 $V/base6.so@5 $V/w2.so@5 $V/w22.so@5 $V/base6.so@5 $V/w2.so@5 $V/w22.so@5" \
 "200|r6d_pbb|CPK_HOST_TRACE=1 gpurun_out/pbb 8192 50" \
 "600|r6d_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread"
