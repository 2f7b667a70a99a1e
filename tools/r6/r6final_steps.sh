#!/bin/bash
# round 6 end: GPU suite, smoke, the default bench line, and the default
# bench under rocprofv3 --kernel-trace --stats (the judged profile)
tools/gpu_steps.sh \
 "600|r6final_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r6final_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200|r6final_bench|python bench.py" \
 "300|r6final_prof|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && timeout -k 10 250 rocprofv3 --kernel-trace --stats -d gpurun_out/r6final_prof -o prof --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu"
