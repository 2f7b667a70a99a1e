#!/bin/bash
# round 6: config-3 messages, segments largest first in both passes (1), the
# emit pass only (2), neither (0); three runs per arm interleaved
B="python bench.py --steps 6 --warmup 2 --no-cpu --config 3"
tools/gpu_steps.sh \
 "120|r6k_o1a|CPK_E4_ORDER=1 $B" "120|r6k_o2a|CPK_E4_ORDER=2 $B" "120|r6k_o0a|CPK_E4_ORDER=0 $B" \
 "120|r6k_o1b|CPK_E4_ORDER=1 $B" "120|r6k_o2b|CPK_E4_ORDER=2 $B" "120|r6k_o0b|CPK_E4_ORDER=0 $B" \
 "120|r6k_o1c|CPK_E4_ORDER=1 $B" "120|r6k_o2c|CPK_E4_ORDER=2 $B" "120|r6k_o0c|CPK_E4_ORDER=0 $B"
