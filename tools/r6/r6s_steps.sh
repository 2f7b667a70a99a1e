#!/bin/bash
# round 6: the two-pass emit's ring put as encode_sp.hip's (four v_perm, no
# per-dword wrap, one overhang line: e4p) against the tree (cur8)
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400|r6s_parity|CPK_LIB=$PWD/$V/e4p.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_bench_shapes.py -x -q --timeout 150 --timeout-method thread" \
 "500|r6s_ab|QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/e4p.so@4 $V/cur8.so@4 $V/e4p.so@4 $V/cur8.so@4 $V/e4p.so@4" \
 "500|r6s_ab_mixed|QB_MIXED=1 QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/e4p.so@4 $V/cur8.so@4 $V/e4p.so@4 $V/cur8.so@4 $V/e4p.so@4"
