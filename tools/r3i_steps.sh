# round-3: decoder expansion reads a record's first 12 bytes as four LDS dwords (CPK_DEC_EXP4)
V=build/variants
tools/gpu_steps.sh \
 "300|r3i_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/exp0.so@0:CPK_DECODER=1 $V/exp1.so@0:CPK_DECODER=1 $V/exp0.so@0:CPK_DECODER=1 $V/exp1.so@0:CPK_DECODER=1"
