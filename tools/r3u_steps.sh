# round-3: wave priority (s_setprio) around the encoder's A1 loads / wave 0's B + look-back, the decoder's window loads
V=build/variants
tools/gpu_steps.sh \
 "300|r3u_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/p0.so@5 $V/pa1.so@5 $V/plb.so@5 $V/pboth.so@5 $V/dprio.so@5 $V/p0.so@5"
