# round-3 final tree: SQ counters (VALU / LDS / waits) of the config-2 kernels and the config-4 sparse form
tools/gpu_steps.sh \
 "400|r3O_sq2|tools/profile.sh r3O_c2 sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu --config 2" \
 "400|r3O_sq4|tools/profile.sh r3O_c4 sq -- python3 bench.py --steps 2 --warmup 1 --no-cpu --config 4"
