#!/bin/bash
# natural SSOR: chain tails (bitwise test, threshold sweep)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ssor_chain.py -x -v --timeout 550 --timeout-method thread > $O/chain_tests.log 2>&1; rc=$?; echo "chain tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
for T in 0 4096 16384 32768; do
  echo "== chain $T" >> $O/chain_sweep.log
  PNP_NAT_CHAIN=$T timeout -k 10 200 python tools/bench_ssor_natural.py 3 4 >> $O/chain_sweep.log 2>&1 || exit $?
done
