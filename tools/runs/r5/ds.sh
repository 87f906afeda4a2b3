#!/bin/bash
# round 5, lease ds: one block-Jacobi sweep (instead of 2) on the AMG levels below level 1
# (PNP_AMG_DEEP_SWEEPS=1) against the default, interleaved: iteration wall time and Newton solves
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5ds; mkdir -p $O
for rep in 1 2; do
  for d in 0 1; do
    PNP_AMG_DEEP_SWEEPS=$d timeout -k 10 300 python -u tools/prof_amg.py run 40 > $O/it_$d.$rep.log 2>&1 || exit 1
    echo "deep=$d rep $rep: $(cat $O/it_$d.$rep.log)"
    PNP_AMG_DEEP_SWEEPS=$d timeout -k 10 300 python -u tools/bench_amg.py > $O/amg_$d.$rep.log 2>&1 || exit 1
    grep "AMG" $O/amg_$d.$rep.log | cut -c1-200
  done
done
exit 0
