#!/bin/bash
# round 6: re-check of the emit-step keep on the config-3 bench shape (256 Ki
# messages): tree library against cur8 (before it), three runs each, interleaved
V=build/variants
T=capnproto-java_amd/lib/libcapnp_packed_hip.so
A="python bench.py --config 3 --steps 10 --warmup 2 --no-cpu"
tools/gpu_steps.sh \
 "200|r6w_c3_old1|CPK_LIB=$PWD/$V/cur8.so $A" "200|r6w_c3_new1|CPK_LIB=$PWD/$T $A" \
 "200|r6w_c3_old2|CPK_LIB=$PWD/$V/cur8.so $A" "200|r6w_c3_new2|CPK_LIB=$PWD/$T $A" \
 "200|r6w_c3_old3|CPK_LIB=$PWD/$V/cur8.so $A" "200|r6w_c3_new3|CPK_LIB=$PWD/$T $A"
