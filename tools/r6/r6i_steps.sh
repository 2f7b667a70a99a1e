#!/bin/bash
# round 6: the single pass's reload (sparse) form with larger rings at 4-5
# workgroups per CU (m1: 7.5 KiB / 4, m2h: 5.5 KiB / 5 + head counts on every
# step, m1h: 7.5 KiB / 4 + head counts), forced on config 2 (CPK_SP_FORM=s)
# against the dense form, and as the sparse form on config 4; three runs per arm
V=build/variants
S=CPK_SP_FORM=s
tools/gpu_steps.sh \
 "500|r6i_c2|QB_N=1048576 QB_CFG=2 python tools/quick_bench.py $V/cur7.so@5 $V/m1.so@5:$S $V/m1h.so@5:$S $V/m2h.so@5:$S $V/cur7.so@5 $V/m1.so@5:$S $V/m1h.so@5:$S $V/m2h.so@5:$S $V/cur7.so@5 $V/m1.so@5:$S $V/m1h.so@5:$S $V/m2h.so@5:$S" \
 "300|r6i_c4|QB_N=1048576 QB_CFG=4 python tools/quick_bench.py $V/cur7.so@5 $V/m1.so@5 $V/m1h.so@5 $V/m2h.so@5 $V/cur7.so@5 $V/m1.so@5 $V/m1h.so@5 $V/m2h.so@5"
