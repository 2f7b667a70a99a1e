#!/bin/bash
# round 6: the current tree against the round-5 final library on one box
# (pieces through quick_bench, messages through bench.py --config 3), three
# runs per arm interleaved
V=build/variants
B="python bench.py --steps 6 --warmup 2 --no-cpu"
tools/gpu_steps.sh \
 "400|r6e_vs_r5_pieces|QB_N=1048576 QB_CFG=2,3,4 python tools/quick_bench.py $V/r5final.so@5 $V/base6.so@5 $V/r5final.so@5 $V/base6.so@5 $V/r5final.so@5 $V/base6.so@5" \
 "120|r6e_c3_r5a|CPK_LIB=$V/r5final.so $B --config 3" \
 "120|r6e_c3_r6a|CPK_LIB=$V/base6.so $B --config 3" \
 "120|r6e_c3_r5b|CPK_LIB=$V/r5final.so $B --config 3" \
 "120|r6e_c3_r6b|CPK_LIB=$V/base6.so $B --config 3" \
 "120|r6e_c3_r5c|CPK_LIB=$V/r5final.so $B --config 3" \
 "120|r6e_c3_r6c|CPK_LIB=$V/base6.so $B --config 3"
