#!/bin/bash
# round 6: GPU suite on the tree, bench lines configs 2/3/4, passByBytes
g++ -O2 -std=c++17 -pthread -Iinclude tests/cpp/pass_by_bytes.cpp oracle/packed_oracle.c -Lcapnproto-java_amd/lib -lcapnp_packed_hip -Wl,-rpath,$PWD/capnproto-java_amd/lib -o gpurun_out/pbb || exit 1
tools/gpu_steps.sh \
 "600|r6g_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r6g_bench_config2|python bench.py --config 2 --steps 10 --warmup 2" \
 "200|r6g_bench_config3|python bench.py --config 3 --steps 10 --warmup 2" \
 "200|r6g_bench_config4|python bench.py --config 4 --steps 10 --warmup 2" \
 "200|r6g_pbb|gpurun_out/pbb 8192 50"
