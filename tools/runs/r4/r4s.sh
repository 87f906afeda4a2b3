#!/bin/bash
# chain kernel: threshold around the resident-group capacity x head workgroups per CU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4s; mkdir -p $O
export TMPDIR=/tmp
for W in 4 2 8; do
  for T in 6144 8192 10240 12288; do
    echo "== wg $W chain $T" >> $O/sweep.log
    PNP_NAT_FLOW_WG_PER_CU=$W PNP_NAT_CHAIN=$T timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/sweep.log 2>&1 || exit $?
  done
done
