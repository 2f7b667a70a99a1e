#!/bin/bash
# round 6: the sparse form builds no strings for a step of zero words and no
# head (tags from the A1 stash, one ballot) and skips a pair of them whole
# (skp2) against the tree (cur10, with the decode2 change)
V=build/variants
tools/gpu_steps.sh \
 "400|r6z6_parity|CPK_LIB=$PWD/$V/skp2.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_bench_shapes.py -x -q --timeout 150 --timeout-method thread" \
 "500|r6z6_ab|QB_N=1048576 QB_CFG=4 python tools/quick_bench.py $V/cur10.so@5 $V/skp2.so@5 $V/cur10.so@5 $V/skp2.so@5 $V/cur10.so@5 $V/skp2.so@5"
