#!/bin/bash
# round 6: the two passes take a wave's next ticket as it starts a piece
# (etk) against the tree (cur9): parity, config-3 bench shape x3 interleaved,
# like-sized config-3-density pieces
V=build/variants
A="python bench.py --config 3 --steps 10 --warmup 2 --no-cpu"
tools/gpu_steps.sh \
 "400|r6x_parity|CPK_LIB=$PWD/$V/etk.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_bench_shapes.py -x -q --timeout 150 --timeout-method thread" \
 "200|r6x_c3_old1|CPK_LIB=$PWD/$V/cur9.so $A" "200|r6x_c3_new1|CPK_LIB=$PWD/$V/etk.so $A" \
 "200|r6x_c3_old2|CPK_LIB=$PWD/$V/cur9.so $A" "200|r6x_c3_new2|CPK_LIB=$PWD/$V/etk.so $A" \
 "200|r6x_c3_old3|CPK_LIB=$PWD/$V/cur9.so $A" "200|r6x_c3_new3|CPK_LIB=$PWD/$V/etk.so $A" \
 "400|r6x_ab_like|QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur9.so@4 $V/etk.so@4 $V/cur9.so@4 $V/etk.so@4"
