#!/bin/bash
# round 6 A/B: decoder lane-chunk skew (CPK_DEC_SKEW 0 / 4), full size, three
# runs per arm interleaved in one process; then the SQ LDS counters per arm
V=build/variants
export QB_N=1048576
tools/gpu_steps.sh \
 "400|r6a_skew_ab|QB_CFG=2,3,4 python tools/quick_bench.py $V/dsk0.so@5 $V/dsk4.so@5 $V/dsk0.so@5 $V/dsk4.so@5 $V/dsk0.so@5 $V/dsk4.so@5" \
 "200|r6a_pmc_dsk0|QB_N=262144 tools/pmc_sq.sh dsk0 decode_kernel -- python3 tools/quick_bench.py $V/dsk0.so@5" \
 "200|r6a_pmc_dsk4|QB_N=262144 tools/pmc_sq.sh dsk4 decode_kernel -- python3 tools/quick_bench.py $V/dsk4.so@5"
