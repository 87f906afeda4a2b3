#!/bin/bash
# natural SSOR: poll backoff (1 / 4 / 16 / 64 s_sleep periods at most) in the pipelined head and the
# chain kernel, interleaved twice; bitwise tests with the largest
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4v; mkdir -p $O
export TMPDIR=/tmp
PNP_AMD_LIB=dune-pnp_amd/ab/lib_bo64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests_bo64.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for lib in - bo4 bo16 bo64; do
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    echo "== $lib round $i" >> $O/ab.log
    env $libenv timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/ab.log 2>&1 || exit $?
  done
done
