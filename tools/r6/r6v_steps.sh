#!/bin/bash
# round 6 tree after the emit-step change: GPU suite, smoke, bench lines
# (default = config 2, configs 3 and 4), config-3 kernel stats and HBM traffic
B="python3 bench.py --steps 3 --warmup 1 --no-cpu"
tools/gpu_steps.sh \
 "600|r6v_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r6v_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200|r6v_bench_default|python bench.py" \
 "200|r6v_bench_config3|python bench.py --config 3 --steps 10 --warmup 2" \
 "200|r6v_bench_config4|python bench.py --config 4 --steps 10 --warmup 2" \
 "300|r6v_prof3|tools/profile.sh r6v_c3 -- $B --config 3"
