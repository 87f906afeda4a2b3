#!/bin/bash
# Build a variant of libpnp_amd.so into dune-pnp_amd/ab/lib_<name>.so with extra compile flags
# (own object dir), for the interleaved A/Bs of tools/ab_lib*.sh.
# usage: tools/build_ab.sh <name> "<extra flags>"
set -eu
cd "$(dirname "$0")/../dune-pnp_amd"
mkdir -p ab
make -s -j16 BUILD=ab/build_$1 LIB=ab/lib_$1.so \
  CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value $2" \
  ab/lib_$1.so
