#!/bin/bash
# round 4: natural SSOR with single-workgroup tails (tests, threshold sweep); graph replay count probe
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4e; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ssor_natural.py tests/test_gpu_seq_order.py -x -q --timeout 200 --timeout-method thread > $O/nat_tests.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
for T in 0 512 1024 2048 4096; do
  echo "== tail $T" >> $O/tail_sweep.log
  PNP_NAT_TAIL=$T timeout -k 10 200 python tools/bench_ssor_natural.py 3 4 >> $O/tail_sweep.log 2>&1 || exit $?
done
