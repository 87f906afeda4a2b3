#!/bin/bash
# round 5, lease ga: hipGraph replay of the BiCGSTAB blocks at config 3 against eager launches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5ga; mkdir -p $O
timeout -k 10 300 python -u tools/ab_graph.py 3 > $O/ab_graph.log 2>&1; rc=$?; echo "rc=$rc"; tail -3 $O/ab_graph.log
exit $rc
