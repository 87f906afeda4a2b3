#!/bin/bash
# round 4: FETCH_SIZE calibration, then the natural-SSOR / reference-order tests and timings
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_run.sh r4b calib || exit $?
O=gpurun_out/r4b
timeout -k 10 400 python -u -m pytest tests/test_gpu_ssor_natural.py -x -v --timeout 120 --timeout-method thread > $O/nat.log 2>&1; rc=$?; echo "nat tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/bench_ssor_natural.py 3 4 > $O/bench_flow.log 2>&1 || exit $?
PNP_NAT_FLOW=0 timeout -k 10 200 python -u tools/bench_ssor_natural.py 4 > $O/bench_levels.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_seq_order.py -v --timeout 200 --timeout-method thread > $O/seq.log 2>&1; rc=$?; echo "seq tests rc=$rc"
exit 0
