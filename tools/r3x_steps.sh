# round-3: decoder 2-word blocks (one contiguous 16-byte store per lane with nontemporal stores)
V=build/variants
tools/gpu_steps.sh \
 "300|r3x_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/d4.so@5:CPK_DECODER=1 $V/d2r640.so@5:CPK_DECODER=1 $V/d2.so@5:CPK_DECODER=1 $V/d4.so@5:CPK_DECODER=1"
