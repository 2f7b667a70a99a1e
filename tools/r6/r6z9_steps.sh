#!/bin/bash
# round 6: the sparse form's reload issues no load for a step without a
# nonzero word (ldwb) against the tree (cur11)
V=build/variants
tools/gpu_steps.sh \
 "300|r6z9_parity|CPK_LIB=$PWD/$V/ldwb.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'sparse or gate or synthetic or capacity or random'" \
 "500|r6z9_ab|QB_N=1048576 QB_CFG=4 python tools/quick_bench.py $V/cur11.so@5 $V/ldwb.so@5 $V/cur11.so@5 $V/ldwb.so@5 $V/cur11.so@5 $V/ldwb.so@5"
