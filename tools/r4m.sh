#!/bin/bash
# natural SSOR: two levels per hop (bitwise test, timing against the default)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssor_chain.py -x -v -k two_levels --timeout 550 --timeout-method thread > $O/recomp_tests.log 2>&1; rc=$?; echo "recomp tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
for i in 1 2; do
  for R in 0 1; do
    echo "== recomp $R" >> $O/recomp_ab.log
    PNP_NAT_RECOMP=$R timeout -k 10 200 python tools/bench_ssor_natural.py 3 4 >> $O/recomp_ab.log 2>&1 || exit $?
  done
done
