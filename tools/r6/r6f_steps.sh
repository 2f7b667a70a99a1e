#!/bin/bash
# round 6: dense decoder forms after moving their counters to a fixed LDS
# address (cur6) against round 5 (r5final); config-3 messages with the
# two-pass encoder's segments largest first (cur6) or in order (CPK_E4_ORDER=0)
V=build/variants
B="python bench.py --steps 6 --warmup 2 --no-cpu --config 3"
tools/gpu_steps.sh \
 "300|r6f_pieces|QB_N=1048576 QB_CFG=3,2 python tools/quick_bench.py $V/r5final.so@5 $V/cur6.so@5 $V/r5final.so@5 $V/cur6.so@5 $V/r5final.so@5 $V/cur6.so@5" \
 "120|r6f_c3_r5a|CPK_LIB=$V/r5final.so $B" \
 "120|r6f_c3_ordA|CPK_LIB=$V/cur6.so $B" \
 "120|r6f_c3_noordA|CPK_E4_ORDER=0 CPK_LIB=$V/cur6.so $B" \
 "120|r6f_c3_r5b|CPK_LIB=$V/r5final.so $B" \
 "120|r6f_c3_ordB|CPK_LIB=$V/cur6.so $B" \
 "120|r6f_c3_noordB|CPK_E4_ORDER=0 CPK_LIB=$V/cur6.so $B" \
 "120|r6f_c3_r5c|CPK_LIB=$V/r5final.so $B" \
 "120|r6f_c3_ordC|CPK_LIB=$V/cur6.so $B" \
 "120|r6f_c3_noordC|CPK_E4_ORDER=0 CPK_LIB=$V/cur6.so $B"
