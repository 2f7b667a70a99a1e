# round-3 A/B session: encoder units / register budget / head-count branch,
# large pieces, config-3 messages, then the GPU test suite
tools/gpu_steps.sh \
 "200|r3c_ab|tools/ab.sh 2,3,4 build/variants/base.so@0 capnproto-java_amd/lib/libcapnp_packed_hip.so@0 build/variants/wpe4.so@0 build/variants/hcbr.so@0" \
 "200|r3c_big|QB_W=65536 QB_N=16384 QB_CFG=2,3 timeout -k 10 180 python tools/quick_bench.py build/variants/base.so@0 capnproto-java_amd/lib/libcapnp_packed_hip.so@0 capnproto-java_amd/lib/libcapnp_packed_hip.so@4" \
 "200|r3c_cfg3_sp|CPK_ENCODER=0 python bench.py --config 3 --segments 65536 --no-cpu --steps 5 --warmup 1" \
 "200|r3c_cfg3_e4|python bench.py --config 3 --segments 65536 --no-cpu --steps 5 --warmup 1" \
 "480|r3c_tests|python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread"
