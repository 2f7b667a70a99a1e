# round-3 session 2: the sparse form's B reloads only nonzero words (masked loads); config-4 traffic
V=build/variants
tools/gpu_steps.sh \
 "200|r3X_ab|QB_N=131072 QB_CFG=4,2 timeout -k 10 180 python tools/quick_bench.py $V/gate.so@5 $V/gate2.so@5 $V/gate.so@5 $V/gate2.so@5" \
 "300|r3X_prof4|tools/profile.sh r3X_c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu --config 4"
