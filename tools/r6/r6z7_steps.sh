#!/bin/bash
# round 6: decode_batch_impl's extent probe through pinned memory (one small
# kernel) instead of four copies into pageable memory: the GPU suite, then
# the per-call overhead probe (profiles/r6b_small_decode_launch_overhead.txt
# before)
tools/gpu_steps.sh \
 "600|r6z7_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r6z7_overhead|python tools/r6/launch_overhead.py"
