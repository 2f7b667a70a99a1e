#!/bin/bash
# round 6: e4p + the emit step's strings in the single pass's form (e4s)
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400|r6t_parity|CPK_LIB=$PWD/$V/e4s.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_bench_shapes.py -x -q --timeout 150 --timeout-method thread" \
 "500|r6t_ab|QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/e4s.so@4 $V/cur8.so@4 $V/e4s.so@4 $V/cur8.so@4 $V/e4s.so@4" \
 "500|r6t_ab_mixed|QB_MIXED=1 QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/e4s.so@4 $V/cur8.so@4 $V/e4s.so@4 $V/cur8.so@4 $V/e4s.so@4"
