# round-3: nontemporal window loads in the decoders (CPK_DEC_NTLD), in the two-pass encoder's emit pass (CPK_E4_NTST / NTLD2)
V=build/variants
tools/gpu_steps.sh \
 "300|r3s_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/b0.so@5 $V/dntld.so@5 $V/b0.so@4 $V/e4st.so@4 $V/e4ld.so@4 $V/e4both.so@4 $V/b0.so@5 $V/dntld.so@5"
