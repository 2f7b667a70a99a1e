#!/bin/bash
# round 6: (1) the dense single pass with rings that hold a wave's whole
# output at config-3 density (17.5 KiB, 2 workgroups per CU: sp2) against the
# tree's (11 KiB, 3 per CU) and the two passes; (2) the ring put's fourth
# dword OR skipped for the wave when no string reaches it (or3), config 2
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300|r6o_parity|CPK_LIB=$PWD/$V/sp2.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'synthetic or gate or capacity or random or literal or large'" \
 "300|r6o_parity_or3|CPK_LIB=$PWD/$V/or3.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'synthetic or gate or sparse or capacity or random or literal or large'" \
 "400|r6o_sp2_c3|QB_N=1048576 QB_CFG=3,2 python tools/quick_bench.py $V/cur8.so@4 $V/cur8.so@0 $V/sp2.so@0 $V/cur8.so@0 $V/sp2.so@0" \
 "400|r6o_or3_c2|QB_N=1048576 QB_CFG=2,4 python tools/quick_bench.py $V/cur8.so@5 $V/or3.so@5 $V/cur8.so@5 $V/or3.so@5 $V/cur8.so@5 $V/or3.so@5"
