# round-3 session 2: encoder reload-form A/B, then the restored tree's GPU suite and default bench line
V=build/variants
tools/gpu_steps.sh \
 "300|r3B_ab|QB_N=131072 QB_CFG=2,4,3 timeout -k 10 280 python tools/quick_bench.py $V/sp_base.so@0 $V/sp_rl5.so@0 $V/sp_rl6.so@0 $V/sp_rl7.so@0 $V/sp_rl6d.so@0 $V/sp_base.so@0 $V/sp_rl6.so@0" \
 "400|r3A_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r3A_bench_default|python bench.py"
