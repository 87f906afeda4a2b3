#!/bin/bash
# natural SSOR: the sparse tail grid (PNP_NAT_TAIL_WPC) -- bitwise tests with it on, then a sweep of
# tail threshold x waves per CU, and the round-4 lanes-per-row / poll-depth library A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4n; mkdir -p $O
export TMPDIR=/tmp
PNP_NAT_TAIL=1024 PNP_NAT_TAIL_WPC=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_ssor_natural.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests_tailgrid.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
for cfg in "0 0" "512 1" "1024 1" "2048 1" "4096 1" "1024 2" "2048 2" "1024 4" "8192 1"; do
  set -- $cfg
  echo "== tail $1 wpc $2" >> $O/tail_grid.log
  PNP_NAT_TAIL=$1 PNP_NAT_TAIL_WPC=$2 timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/tail_grid.log 2>&1 || exit $?
done
bash tools/ab_nat_libs.sh r4n/ab - kl16 kl32 pd2 pd4
