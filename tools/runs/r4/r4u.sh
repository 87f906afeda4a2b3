#!/bin/bash
# natural SSOR: the software-pipelined head (k_ssor_nat_pipe) -- bitwise tests, then A/B against
# the unpipelined flow head (PNP_NAT_PIPE=0), with the default chains and with units only
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4u; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_ssor_chain.py -x -q --timeout 800 --timeout-method thread > $O/chain_tests.log 2>&1; rc=$?; echo "chain tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for P in 1 0; do
    for C in default 0; do
      if [ "$C" = "default" ]; then cenv=""; else cenv="PNP_NAT_CHAIN=$C"; fi
      echo "== pipe $P chain $C round $i" >> $O/ab.log
      env PNP_NAT_PIPE=$P $cenv timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/ab.log 2>&1 || exit $?
    done
  done
done
