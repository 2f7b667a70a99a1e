#!/bin/bash
# round 6: the decoder's next window prefetched into L2 (one dword per
# 128-byte line at the window's start, l2pf) against the tree (cur9)
V=build/variants
A="python bench.py --config 3 --steps 10 --warmup 2 --no-cpu"
tools/gpu_steps.sh \
 "500|r6y_parity|CPK_LIB=$PWD/$V/l2pf.so python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "600|r6y_ab|QB_N=1048576 QB_CFG=2,4 python tools/quick_bench.py $V/cur9.so@5 $V/l2pf.so@5 $V/cur9.so@5 $V/l2pf.so@5 $V/cur9.so@5 $V/l2pf.so@5" \
 "200|r6y_c3_old1|CPK_LIB=$PWD/$V/cur9.so $A" "200|r6y_c3_new1|CPK_LIB=$PWD/$V/l2pf.so $A" \
 "200|r6y_c3_old2|CPK_LIB=$PWD/$V/cur9.so $A" "200|r6y_c3_new2|CPK_LIB=$PWD/$V/l2pf.so $A"
