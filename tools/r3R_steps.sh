# round-3 final check: GPU suite, default bench line, smoke on the final tree
tools/gpu_steps.sh \
 "400|r3R_gpu_tests|python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
 "200|r3R_bench_default|python bench.py" \
 "200|r3R_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
