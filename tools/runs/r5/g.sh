#!/bin/bash
# round 5, lease g: natural SSOR -- d read at internal positions, gather after; A/B of the
# 32-entry flow head (PNP_NAT_FLOW_KS4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5g; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for k in 1 0 1 0; do
  PNP_NAT_FLOW_KS4=$k timeout -k 10 200 python -u tools/bench_ssor_natural.py 4 > $O/nat_ks4_$k.log 2>&1; rc=$?; echo "nat ks4=$k rc=$rc"; cat $O/nat_ks4_$k.log
  fatal $rc && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_ssor_natural.py 4 > $O/trace.log 2>&1; rc=$?; echo "trace rc=$rc"
fatal $rc && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ssor_natural.py tests/test_gpu_ssor_chain.py tests/test_gpu_seq_order.py tests/test_gpu_rccl.py tests/test_gpu_graph.py tests/test_gpu.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
exit 0
