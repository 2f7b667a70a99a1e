#!/bin/bash
# round 6: the single pass's next unit loaded ahead (CPK_SP_PF): its ticket
# taken by wave 1 once it has laid out its steps and every wave's words
# loaded before the flush -- pf0: waves 1-3 before the offset wait, wave 0
# after its look-back; pf1: all waves after the offset -- against the tree
# (cur8; pfoff = this source without the knob: same code as cur8)
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300|r6r_parity_pf0|CPK_LIB=$PWD/$V/pf0.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'synthetic or gate or sparse or capacity or random or literal or large or message'" \
 "300|r6r_parity_pf1|CPK_LIB=$PWD/$V/pf1.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'synthetic or gate or sparse or capacity or random or literal or large or message'" \
 "600|r6r_ab|QB_N=1048576 QB_CFG=2 python tools/quick_bench.py $V/cur8.so@5 $V/pf0.so@5 $V/pf1.so@5 $V/pfoff.so@5 $V/cur8.so@5 $V/pf0.so@5 $V/pf1.so@5 $V/cur8.so@5 $V/pf0.so@5 $V/pf1.so@5"
