#!/bin/bash
# round 6: the emit pass's step rows loaded a group ahead by one vector load
# (e4r), and with the put / string forms (e4rs), against the tree (cur8)
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400|r6u_parity|CPK_LIB=$PWD/$V/e4rs.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py tests/test_gpu_bench_shapes.py -x -q --timeout 150 --timeout-method thread" \
 "300|r6u_parity_r|CPK_LIB=$PWD/$V/e4r.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'synthetic or random or literal or large or message or capacity'" \
 "600|r6u_ab|QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/e4r.so@4 $V/e4rs.so@4 $V/cur8.so@4 $V/e4r.so@4 $V/e4rs.so@4 $V/cur8.so@4 $V/e4r.so@4 $V/e4rs.so@4" \
 "600|r6u_ab_mixed|QB_MIXED=1 QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/e4r.so@4 $V/e4rs.so@4 $V/cur8.so@4 $V/e4r.so@4 $V/e4rs.so@4 $V/cur8.so@4 $V/e4r.so@4 $V/e4rs.so@4"
