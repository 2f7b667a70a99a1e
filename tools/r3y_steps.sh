# round-3: encoder look-back polled between step pairs (CPK_SP_LBINC, distance CPK_SP_LBINC_D)
V=build/variants
tools/gpu_steps.sh \
 "300|r3y_ab|QB_N=131072 QB_CFG=2,3,4 timeout -k 10 280 python tools/quick_bench.py $V/li0.so@5 $V/li4.so@5 $V/li2.so@5 $V/li8.so@5 $V/li0.so@5 $V/li4.so@5" \
 "200|r3y_big|QB_W=65536 QB_N=16384 QB_CFG=2,3 timeout -k 10 180 python tools/quick_bench.py $V/li0.so@5 $V/li4.so@5"
