#!/bin/bash
# round 6 end, after the config-4 changes (decode2 zero groups, sparse empty
# steps): GPU suite, smoke, default bench, config-4 bench, config-4 kernel
# stats and HBM traffic
B="python3 bench.py --steps 3 --warmup 1 --no-cpu"
tools/gpu_steps.sh \
 "600|r6final2_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r6final2_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200|r6final2_bench|python bench.py" \
 "200|r6final2_bench_config4|python bench.py --config 4 --steps 10 --warmup 2" \
 "300|r6final2_prof4|tools/profile.sh r6final2_c4 -- $B --config 4"
