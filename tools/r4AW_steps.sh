# round-4 final tree: config-3 kernel stats + HBM traffic (rocprofv3)
B="python3 bench.py --steps 3 --warmup 1 --no-cpu"
tools/gpu_steps.sh "300|r4AW_prof3|tools/profile.sh r4AW_c3 -- $B --config 3"
