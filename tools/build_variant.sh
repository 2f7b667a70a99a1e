#!/bin/bash
# Builds a variant of the codec library with extra -D flags for A/B timing:
#   tools/build_variant.sh NAME -DFOO=1 ...  ->  build/variants/NAME.so
set -e
name=$1; shift
mkdir -p build/variants
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Wno-unused-value \
  -Wno-unused-result "$@" -o build/variants/$name.so capnproto-java_amd/csrc/packed_codec.hip
echo build/variants/$name.so
