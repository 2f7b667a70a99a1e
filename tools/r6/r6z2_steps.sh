#!/bin/bash
# round 6: the sparse form skips a pair of steps with no bytes (all zero
# words, no head: inside a zero run) before building its strings (skp)
V=build/variants
tools/gpu_steps.sh \
 "400|r6z2_parity|CPK_LIB=$PWD/$V/skp.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_bench_shapes.py -x -q --timeout 150 --timeout-method thread" \
 "500|r6z2_ab|QB_N=1048576 QB_CFG=4 python tools/quick_bench.py $V/cur9.so@5 $V/skp.so@5 $V/cur9.so@5 $V/skp.so@5 $V/cur9.so@5 $V/skp.so@5" \
 "300|r6z2_ab_forced|QB_N=1048576 QB_CFG=2 python tools/quick_bench.py $V/cur9.so@5:CPK_SP_FORM=s $V/skp.so@5:CPK_SP_FORM=s"
