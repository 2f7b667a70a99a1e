#!/bin/bash
# round 6: the single pass's line stores plain instead of nontemporal (pst):
# config-2 encode writes 35.1 GB for 32.6 GB of packed bytes (the lines sit at
# any byte alignment); time and WRITE_SIZE
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "500|r6z3_ab|QB_N=1048576 QB_CFG=2,4 python tools/quick_bench.py $V/cur9.so@5 $V/pst.so@5 $V/cur9.so@5 $V/pst.so@5 $V/cur9.so@5 $V/pst.so@5" \
 "200|r6z3_w_cur|QB_N=262144 QB_CFG=2 timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r6z3_wc -o wc --output-format csv -- python3 tools/quick_bench.py $V/cur9.so@5" \
 "200|r6z3_w_pst|QB_N=262144 QB_CFG=2 timeout -k 10 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r6z3_wp -o wp --output-format csv -- python3 tools/quick_bench.py $V/pst.so@5"
