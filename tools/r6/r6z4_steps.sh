#!/bin/bash
# round 6: same-box re-check of round 5's smallest decoder keep (r5AO, the
# walks' tag kept 32-bit): the tree (cur9) against it undone (no32)
V=build/variants
tools/gpu_steps.sh \
 "500|r6z4_ab|QB_N=1048576 QB_CFG=2 python tools/quick_bench.py $V/cur9.so@5 $V/no32.so@5 $V/cur9.so@5 $V/no32.so@5 $V/cur9.so@5 $V/no32.so@5"
