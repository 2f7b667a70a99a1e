#!/bin/bash
# round 6 end state: smoke and the three bench lines
tools/gpu_steps.sh \
 "200|r6end_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200|r6end_bench|python bench.py" \
 "200|r6end_bench_config3|python bench.py --config 3 --steps 10 --warmup 2" \
 "200|r6end_bench_config4|python bench.py --config 4 --steps 10 --warmup 2"
