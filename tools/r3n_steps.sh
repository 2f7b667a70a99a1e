# round-3: gate overhead after the min/max reduction fix (auto vs forced single pass)
L=capnproto-java_amd/lib/libcapnp_packed_hip.so
tools/gpu_steps.sh \
 "200|r3n_ab|QB_N=131072 QB_CFG=2,4 timeout -k 10 180 python tools/quick_bench.py $L@5 $L@0 $L@5 $L@0" \
 "300|r3n_trace|cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_prof -o r3n --output-format csv -- python3 tools/prof_run.py 4 131072 3"
