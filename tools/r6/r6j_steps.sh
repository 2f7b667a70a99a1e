#!/bin/bash
# round 6: GPU suite, smoke, default bench line on the tree
tools/gpu_steps.sh \
 "600|r6j_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r6j_smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|r6j_bench_default|python bench.py"
