#!/bin/bash
# round 6 final tree: kernel stats + HBM traffic (+ SQ counters and the
# effective clock for config 2) per config, bench-shaped runs
B="python3 bench.py --steps 3 --warmup 1 --no-cpu"
tools/gpu_steps.sh \
 "400|r6z_prof2|tools/profile.sh r6z_c2 sq -- $B --config 2" \
 "300|r6z_prof3|tools/profile.sh r6z_c3 -- $B --config 3" \
 "300|r6z_prof4|tools/profile.sh r6z_c4 -- $B --config 4"
