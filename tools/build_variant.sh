#!/bin/bash
# Build an A/B variant of the library: bash tools/build_variant.sh NAME [-DFLAG ...] -> jeromq_amd/libcz_NAME.so
cd "$(dirname "$0")/../jeromq_amd/csrc" || exit 1
name=$1; shift
exec /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o ../libcz_$name.so "$@" \
  cz_kernels.hip cz_x25519.hip cz_host.cpp cz_mechanism.cpp cz_wire.cpp cz_engine.cpp cz_handshake.cpp cz_curve_hs.cpp
