#!/bin/bash
# round 6: decode2's expansion skips the byte reads and LUT of a group of 64
# words that are all zero-run words (zsk), config 4 (and config 2 unaffected)
V=build/variants
tools/gpu_steps.sh \
 "400|r6z5_parity|CPK_LIB=$PWD/$V/zsk.so python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k 'decode or parity or stream or read or sparse or bench'" \
 "500|r6z5_ab|QB_N=1048576 QB_CFG=4 python tools/quick_bench.py $V/cur9.so@5 $V/zsk.so@5 $V/cur9.so@5 $V/zsk.so@5 $V/cur9.so@5 $V/zsk.so@5"
