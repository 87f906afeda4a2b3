#!/bin/bash
# natural SSOR at the defaults: head workgroups per CU (3 / 4 / 5) x chain threshold (default / 10240)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4aa; mkdir -p $O
for i in 1 2; do
  for W in 3 4 5; do
    for C in default 10240; do
      if [ "$C" = "default" ]; then cenv=""; else cenv="PNP_NAT_CHAIN=$C"; fi
      echo "== wg $W chain $C round $i" >> $O/ab.log
      env PNP_NAT_FLOW_WG_PER_CU=$W $cenv timeout -k 10 200 python tools/bench_ssor_natural.py 4 >> $O/ab.log 2>&1 || exit $?
    done
  done
done
