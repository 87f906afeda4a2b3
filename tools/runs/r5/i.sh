#!/bin/bash
# round 5, lease i: the two-process host-transport test (tight Newton), the graph-cache test with
# and without the 32-entry flow head, then the natural-SSOR and RCCL suites
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5i; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 250 --timeout-method thread tests/test_gpu_dist_host.py > $O/dist_host.log 2>&1; rc=$?; echo "dist host rc=$rc"; grep -o '{"ranks.*' $O/dist_host.log | head -2; tail -3 $O/dist_host.log
fatal $rc && exit $rc
for k in 0 1; do
PNP_NAT_FLOW_KS4=$k timeout -k 10 200 python -u -m pytest -x -v --timeout 150 --timeout-method thread "tests/test_gpu_ssor_natural.py::test_graph_cache_survives_csr_pattern_switch" > $O/graph_ks4_$k.log 2>&1; rc=$?; echo "graph test ks4=$k rc=$rc"; grep -n "^E  \|passed\|failed" $O/graph_ks4_$k.log | head -8
fatal $rc && exit $rc
done
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_ssor_natural.py tests/test_gpu_ssor_chain.py tests/test_gpu_seq_order.py tests/test_gpu_rccl.py tests/test_gpu_graph.py tests/test_gpu_asm_lds.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log
exit 0
