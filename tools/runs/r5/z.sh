#!/bin/bash
# round 5, lease z: plain (allocating) assembly block stores (ab/lib_splain.so) against the
# non-temporal default, warm / in situ / Newton order, interleaved (tools/ab_newton_asm.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5z; mkdir -p $O
for rep in 1 2; do
  for lib in dune-pnp_amd/libpnp_amd.so dune-pnp_amd/ab/lib_splain.so; do
    echo "== $lib" >> $O/ab.log
    PNP_AMD_LIB=$PWD/$lib timeout -k 10 300 python -u tools/ab_newton_asm.py >> $O/ab.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 $O/ab.log; exit $rc; }
  done
done
cat $O/ab.log
exit 0
