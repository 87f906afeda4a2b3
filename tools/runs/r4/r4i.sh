#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ilu_flow.py -x -q --timeout 200 --timeout-method thread > $O/flow_tests.log 2>&1; rc=$?; echo "flow tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
for m in 2 1; do
  PNP_ILU_FLOW_MODE=$m timeout -k 10 300 python -u tools/bench_ilu_flow.py 3 5 > $O/bench_ilu_flow_mode$m.log 2>&1 || exit $?
done
