# round-3: per-phase cycle shares of the single pass (stats build) on the current tree
tools/gpu_steps.sh \
 "200|r3w_phase|python tools/phase_stats.py 2 65536 && python tools/phase_stats.py 3 65536 && python tools/phase_stats.py 4 65536"
