#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
for lib in kl16 kl32; do
  PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests_$lib.log 2>&1; echo "nat tests $lib rc=$?"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_seq_order.py -x -q -k driver --timeout 250 --timeout-method thread -s > $O/driver_ref_order.log 2>&1; echo "driver test rc=$?"
bash tools/ab_nat_libs.sh r4f/ab - kl16 kl32 pd2 pd4
