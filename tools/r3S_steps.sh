# round-3 session 2: the single pass's dense vs sparse form by zero-word fraction (the gate's density threshold)
V=build/variants
tools/gpu_steps.sh \
 "400|r3S_density|for z in 0.6 0.7 0.75 0.8 0.85 0.9 0.95; do for lz in 4 16 64; do echo \"== z=\$z lz=\$lz\"; QB_Z=\$z QB_LZ=\$lz QB_N=65536 QB_CFG=2 timeout -k 10 60 python tools/quick_bench.py $V/cur.so@5:CPK_SP_FORM=dense $V/cur.so@5:CPK_SP_FORM=sparse $V/cur.so@5:CPK_SP_FORM=auto || exit 1; done; done"
