#!/bin/bash
# round 5, lease y: the in-situ assembly walk at HEAD, interleaved (PNP_ASM_COLD_HINT 1 = LDS walk
# after a solve, the default; 0 = the direct walk), tools/ab_newton_asm.py
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5y; mkdir -p $O
for rep in 1 2; do
  for h in 1 0; do
    PNP_ASM_COLD_HINT=$h timeout -k 10 300 python -u tools/ab_newton_asm.py >> $O/ab.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "rc=$rc"; tail -5 $O/ab.log; exit $rc; }
  done
done
cat $O/ab.log
exit 0
