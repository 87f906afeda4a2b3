#!/bin/bash
# natural SSOR: the software-pipelined one-wave chain kernel -- bitwise tests, then a threshold sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4o; mkdir -p $O
export TMPDIR=/tmp
PNP_NAT_CHAIN=2048 timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests_chain.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
for T in 0 512 1024 2048 4096 8192; do
  echo "== chain $T" >> $O/chain_sweep.log
  PNP_NAT_CHAIN=$T timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/chain_sweep.log 2>&1 || exit $?
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_ssor_chain.py -x -q --timeout 800 --timeout-method thread > $O/chain_tests.log 2>&1; echo "chain tests rc=$?"
