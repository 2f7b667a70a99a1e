# round-3 session 2: the single pass's sparse form chosen on the device (>= 85 % sampled zero words; hashed sample positions)
V=build/variants
tools/gpu_steps.sh \
 "200|r3N_ab|QB_N=131072 QB_CFG=4,2,3 timeout -k 10 180 python tools/quick_bench.py $V/cur.so@5 $V/gate.so@5 $V/cur.so@5 $V/gate.so@5" \
 "200|r3N_ab16k|QB_N=16384 QB_W=65536 QB_CFG=4,2 timeout -k 10 180 python tools/quick_bench.py $V/cur.so@5 $V/gate.so@5" \
 "400|r3N_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r3N_bench_config4|python bench.py --config 4 --steps 10 --warmup 2" \
 "200|r3N_bench_config2|python bench.py --config 2 --steps 10 --warmup 2 --no-cpu"
