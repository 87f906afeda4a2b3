#!/bin/bash
# round 4: one-launch ILU(0) application (bitwise tests, A/B timing), natural-SSOR single-lane poll A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ilu_flow.py -x -v --timeout 200 --timeout-method thread > $O/flow_tests.log 2>&1; rc=$?; echo "flow tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u tools/bench_ilu_flow.py 3 5 > $O/bench_ilu_flow.log 2>&1; rc=$?; echo "bench flow rc=$rc"
[ $rc -ne 0 ] && exit $rc
bash tools/ab_nat_libs.sh r4c/nat - poll0
