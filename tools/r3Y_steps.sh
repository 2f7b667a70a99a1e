# round-3 session 2: size-pass load depth (CPK_E4_PF) on config-3-shaped messages and mixed pieces
V=build/variants
tools/gpu_steps.sh \
 "200|r3Y_mixed|QB_MIXED=1 QB_N=65536 QB_CFG=3 timeout -k 10 180 python tools/quick_bench.py $V/gate.so@4 $V/e4pf2.so@4 $V/e4pf6.so@4 $V/e4pf8.so@4 $V/gate.so@4 $V/e4pf8.so@4" \
 "200|r3Y_msg|for L in gate e4pf8 e4pf6; do echo == \$L; MB_LIB=$V/\$L.so MB_MAXW=32768 timeout -k 10 60 python tools/msg_bench.py 32768 || exit 1; done"
