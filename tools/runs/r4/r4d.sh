#!/bin/bash
# round 4: graph capture under rocprofv3 (verdict item 4), natural-SSOR flow occupancy sweep
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 tools/micro/graph_capture_prof 100 680 1000 2000 4000 > $O/graph_plain.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/graph_prof -o run -- tools/micro/graph_capture_prof 100 680 1000 2000 4000 > $O/graph_prof.log 2>&1; echo "graph prof rc=$?"
PNP_NAT_FLOW=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nat_levels_prof -o run -- python3 tools/bench_ssor_natural.py 3 > $O/nat_levels_prof.log 2>&1; echo "nat levels prof rc=$?"
for w in 1 2 4; do
  PNP_NAT_FLOW_WG_PER_CU=$w timeout -k 10 200 python tools/bench_ssor_natural.py 4 > $O/nat_wg$w.log 2>&1 || exit $?
done
timeout -k 10 300 python -u tools/bench_ilu_flow.py 3 5 > $O/bench_ilu_flow.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_ilu_flow.py -x -v --timeout 200 --timeout-method thread > $O/flow_tests.log 2>&1; echo "flow tests rc=$?"
