#!/bin/bash
# round 5, lease q: the spread of the PNP time to solution's BiCGSTAB count under one-ulp
# perturbations of the Boltzmann state (tools/tts_spread.py)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5q; mkdir -p $O
timeout -k 10 400 python -u tools/tts_spread.py 6 > $O/tts_spread.log 2>&1; rc=$?; echo "spread rc=$rc"; cat $O/tts_spread.log | tail -9
exit 0
