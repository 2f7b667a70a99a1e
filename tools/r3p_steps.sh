# round-3: encoder compaction selectors from a global constant table (CPK_SP_GLUT)
V=build/variants
tools/gpu_steps.sh \
 "200|r3p_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 180 python tools/quick_bench.py $V/gl0.so@0 $V/gl1.so@0 $V/gl0.so@0 $V/gl1.so@0"
