#!/bin/bash
# round 6: pipe utilisation of the two-pass encoder's kernels (config-3
# density pieces, 262,144 x 64 KiB): where the size pass's 78 % of read peak goes
V=build/variants
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "300|r6p_sq_size|QB_N=262144 QB_CFG=3 tools/pmc_sq.sh e4size e4_size -- python3 tools/quick_bench.py $V/cur8.so@4" \
 "300|r6p_sq_emit|QB_N=262144 QB_CFG=3 tools/pmc_sq.sh e4emit e4_emit -- python3 tools/quick_bench.py $V/cur8.so@4" \
 "200|r6p_grbm|QB_N=262144 QB_CFG=3 timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/r6p_g -o g --output-format csv -- python3 tools/quick_bench.py $V/cur8.so@4"
