#!/bin/bash
# natural SSOR dataflow: lanes per row (8 / 16 / 32) and polls in flight (1 / 2 / 4), bitwise + A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4f; mkdir -p $O
for lib in kl16 kl32 pd2; do
  PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests_$lib.log 2>&1; echo "nat tests $lib rc=$?"
done
bash tools/ab_nat_libs.sh r4f/ab - kl16 kl32 pd2 pd4
