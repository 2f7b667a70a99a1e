#!/bin/bash
# round 6: the fused encoder (size sweep a few pieces ahead of the emit in one
# launch, encode_fused.hip) -- parity through the two-pass paths with it on,
# then A/B against the tree's two passes (cur8) on config-3-density pieces,
# like-sized and mixed (config-3 segment sizes), over workgroups per CU and
# pending depth
V=build/variants
export TMPDIR=/tmp
F="CPK_E4_FUSED=1"
tools/gpu_steps.sh \
 "400|r6m_parity|CPK_E4_FUSED=1 CPK_LIB=$PWD/$V/fz.so python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capacity.py -x -q --timeout 150 --timeout-method thread" \
 "400|r6m_ab_like|QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/fz.so@4:CPK_E4_FUSED=0 $V/fz.so@4:$F,CPK_E4F_WG=6,CPK_E4F_DEPTH=1 $V/fz.so@4:$F,CPK_E4F_WG=6,CPK_E4F_DEPTH=2 $V/fz.so@4:$F,CPK_E4F_WG=6,CPK_E4F_DEPTH=4 $V/fz.so@4:$F,CPK_E4F_WG=4,CPK_E4F_DEPTH=2 $V/fz.so@4:$F,CPK_E4F_WG=4,CPK_E4F_DEPTH=4 $V/fz.so@4:$F,CPK_E4F_WG=2,CPK_E4F_DEPTH=2 $V/fz.so@4:$F,CPK_E4F_WG=2,CPK_E4F_DEPTH=4" \
 "400|r6m_ab_mixed|QB_MIXED=1 QB_N=1048576 QB_CFG=3 python tools/quick_bench.py $V/cur8.so@4 $V/fz.so@4:CPK_E4_FUSED=0 $V/fz.so@4:$F,CPK_E4F_WG=6,CPK_E4F_DEPTH=2 $V/fz.so@4:$F,CPK_E4F_WG=6,CPK_E4F_DEPTH=4 $V/fz.so@4:$F,CPK_E4F_WG=6,CPK_E4F_DEPTH=8 $V/fz.so@4:$F,CPK_E4F_WG=4,CPK_E4F_DEPTH=4 $V/fz.so@4:$F,CPK_E4F_WG=2,CPK_E4F_DEPTH=8"
