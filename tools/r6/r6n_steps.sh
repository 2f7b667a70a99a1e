#!/bin/bash
# round 6: the fused encoder at 8 waves per SIMD (fz8: 12 VGPRs spilled)
# against the two passes, and FETCH_SIZE of the fused launch against the two
# passes' (does the emit's re-read hit the caches?)
V=build/variants
export TMPDIR=/tmp
F="CPK_E4_FUSED=1"
tools/gpu_steps.sh \
 "400|r6n_ab_like|QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/fz8.so@4:$F,CPK_E4F_WG=8,CPK_E4F_DEPTH=2 $V/fz8.so@4:$F,CPK_E4F_WG=8,CPK_E4F_DEPTH=4 $V/cur8.so@4 $V/fz8.so@4:$F,CPK_E4F_WG=8,CPK_E4F_DEPTH=8" \
 "200|r6n_fetch_2p|QB_N=262144 QB_CFG=3 timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6n_f2 -o f2 --output-format csv -- python3 tools/quick_bench.py $V/cur8.so@4" \
 "200|r6n_fetch_fz|QB_N=262144 QB_CFG=3 timeout -k 10 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6n_ff -o ff --output-format csv -- python3 tools/quick_bench.py $V/fz8.so@4:$F,CPK_E4F_WG=8,CPK_E4F_DEPTH=4"
