#!/bin/bash
# round 6: the emit pass's words (and rows) 6 / 8 steps ahead instead of 4,
# now that the rows come a group ahead too (epf6 / epf8), config-3 bench
# shape interleaved, parity through epf8
V=build/variants
A="python bench.py --config 3 --steps 10 --warmup 2 --no-cpu"
tools/gpu_steps.sh \
 "300|r6z10_parity|CPK_LIB=$PWD/$V/epf8.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'message or random or literal or large or capacity or synthetic'" \
 "200|r6z10_c3_cur1|CPK_LIB=$PWD/$V/cur11.so $A" "200|r6z10_c3_e6_1|CPK_LIB=$PWD/$V/epf6.so $A" "200|r6z10_c3_e8_1|CPK_LIB=$PWD/$V/epf8.so $A" \
 "200|r6z10_c3_cur2|CPK_LIB=$PWD/$V/cur11.so $A" "200|r6z10_c3_e6_2|CPK_LIB=$PWD/$V/epf6.so $A" "200|r6z10_c3_e8_2|CPK_LIB=$PWD/$V/epf8.so $A" \
 "200|r6z10_c3_cur3|CPK_LIB=$PWD/$V/cur11.so $A" "200|r6z10_c3_e6_3|CPK_LIB=$PWD/$V/epf6.so $A" "200|r6z10_c3_e8_3|CPK_LIB=$PWD/$V/epf8.so $A"
