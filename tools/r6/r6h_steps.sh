#!/bin/bash
# round 6: the expansion's 8-byte reads as two ds_read_b64 (r64), zero-run
# words' reads at one address (zb), both (zb64), against the tree (cur6b),
# three runs per arm interleaved; SQ LDS counters per arm
V=build/variants
tools/gpu_steps.sh \
 "500|r6h_r64_ab|QB_N=1048576 QB_CFG=2,3,4 python tools/quick_bench.py $V/cur6b.so@5 $V/r64.so@5 $V/zb.so@5 $V/zb64.so@5 $V/cur6b.so@5 $V/r64.so@5 $V/zb.so@5 $V/zb64.so@5 $V/cur6b.so@5 $V/r64.so@5 $V/zb.so@5 $V/zb64.so@5" \
 "200|r6h_pmc_cur|QB_N=262144 tools/pmc_sq.sh cur6b decode_kernel -- python3 tools/quick_bench.py $V/cur6b.so@5" \
 "200|r6h_pmc_r64|QB_N=262144 tools/pmc_sq.sh r64 decode_kernel -- python3 tools/quick_bench.py $V/r64.so@5" \
 "200|r6h_pmc_zb|QB_N=262144 tools/pmc_sq.sh zb decode_kernel -- python3 tools/quick_bench.py $V/zb.so@5"
