#!/bin/bash
# round 5, lease rb: ILU(0) factors rounded to 11 (half) / 8 (bfloat16) significant bits in f32
# storage (ab/lib_r11.so, ab/lib_r8.so) against HEAD: PNP Newton BiCGSTAB counts at config 3 over
# one-ulp perturbations of x0 (tools/tts_spread.py), i.e. what a 16-bit factor format would cost
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5rb; mkdir -p $O
for lib in dune-pnp_amd/libpnp_amd.so dune-pnp_amd/ab/lib_r11.so dune-pnp_amd/ab/lib_r8.so; do
  n=$(basename $lib .so)
  PNP_AMD_LIB=$PWD/$lib timeout -k 10 400 python -u tools/tts_spread.py 4 > $O/$n.log 2>&1; rc=$?
  echo "$n rc=$rc: $(tail -1 $O/$n.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
