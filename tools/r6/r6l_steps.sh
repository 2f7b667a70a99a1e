#!/bin/bash
# round 6: the reload form's B in reverse step order for waves whose output
# fits the ring (rev) against the tree (cur8): config 4, three runs per arm;
# encode FETCH_SIZE per arm; parity subset through the rev library
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "400|r6l_ab|QB_N=1048576 QB_CFG=4,2 python tools/quick_bench.py $V/cur8.so@5 $V/rev.so@5 $V/cur8.so@5 $V/rev.so@5 $V/cur8.so@5 $V/rev.so@5" \
 "300|r6l_parity|CPK_LIB=$PWD/$V/rev.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread -k 'synthetic or gate or sparse or capacity or random or literal or large'" \
 "200|r6l_fetch_cur|QB_N=262144 QB_CFG=4 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6l_fc -o fc --output-format csv -- python3 tools/quick_bench.py $V/cur8.so@5" \
 "200|r6l_fetch_rev|QB_N=262144 QB_CFG=4 timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r6l_fr -o fr --output-format csv -- python3 tools/quick_bench.py $V/rev.so@5"
