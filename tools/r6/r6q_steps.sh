#!/bin/bash
# round 6: the single pass's wave 0 runs the unit's look-back after half its
# steps (w0e) instead of after all of them, so waves 1-3 find the offset out
# when they finish B (phase stats: 8.8 % of wave time waiting for it)
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300|r6q_parity|CPK_LIB=$PWD/$V/w0e.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'synthetic or gate or sparse or capacity or random or literal or large'" \
 "500|r6q_ab|QB_N=1048576 QB_CFG=2,4 python tools/quick_bench.py $V/cur8.so@5 $V/w0e.so@5 $V/cur8.so@5 $V/w0e.so@5 $V/cur8.so@5 $V/w0e.so@5"
