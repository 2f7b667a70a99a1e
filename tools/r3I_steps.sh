# round-3 session 2: steps spread over the waves (default) and the gate at 4 Ki words: auto choice by piece size, GPU suite, bench
V=build/variants
tools/gpu_steps.sh \
 "120|r3I_w2048|QB_W=2048 QB_N=65536 QB_CFG=2,3 timeout -k 10 110 python tools/quick_bench.py $V/sp_head.so@5 $V/sp_new.so@5" \
 "120|r3I_w4096|QB_W=4096 QB_N=32768 QB_CFG=2,3 timeout -k 10 110 python tools/quick_bench.py $V/sp_head.so@5 $V/sp_new.so@5" \
 "400|r3I_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r3I_bench_default|python bench.py"
