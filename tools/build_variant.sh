#!/bin/bash
# Build an A/B variant of the library: bash tools/build_variant.sh NAME [-DFLAG ...] -> jeromq_amd/libcz_NAME.so
# (jeromq_amd/build.py: sources compiled in parallel, the linked library gated on the ISA hazard scan)
cd "$(dirname "$0")/.." || exit 1
name=$1; shift
CZ_EXTRA_FLAGS="$*" CZ_LIB_OUT=$PWD/jeromq_amd/libcz_$name.so python3 -c \
  "from jeromq_amd.build import build_library; build_library(force=True, verbose=False)"
