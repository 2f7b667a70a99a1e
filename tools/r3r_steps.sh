# round-3: nontemporal loads / stores in the encoder (CPK_SP_NTLD / NTST) and decoders (CPK_DEC_NT)
V=build/variants
tools/gpu_steps.sh \
 "300|r3r_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/nt0.so@5 $V/ntld.so@5 $V/ntst.so@5 $V/ntdec.so@5 $V/ntboth.so@5 $V/nt0.so@5 $V/ntboth.so@5"
