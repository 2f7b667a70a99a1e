# round-4 final tree (after the size pass NT loads): GPU suite, smoke, default bench line, config-3 bench line
tools/gpu_steps.sh \
 "500|r4AU_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r4AU_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "200|r4AU_bench_default|python bench.py" \
 "200|r4AU_bench_config3|python bench.py --config 3 --steps 10 --warmup 2"
