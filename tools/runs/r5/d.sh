#!/bin/bash
# round 5, lease d: natural SSOR, plain loads in the flow head only; A/B of PNP_NAT_SPEC
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5d; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for sp in 0 1 0 1; do
  PNP_NAT_SPEC=$sp timeout -k 10 200 python -u tools/bench_ssor_natural.py 4 > $O/nat_spec$sp.log 2>&1; rc=$?; echo "nat spec=$sp rc=$rc"; cat $O/nat_spec$sp.log
  fatal $rc && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_ssor_natural.py 4 > $O/trace.log 2>&1; rc=$?; echo "trace rc=$rc"
fatal $rc && exit $rc
PNP_NAT_SPEC=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ssor_natural.py tests/test_gpu_ssor_chain.py > $O/tests_spec1.log 2>&1; rc=$?; echo "tests spec1 rc=$rc"; tail -2 $O/tests_spec1.log
fatal $rc && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ssor_natural.py tests/test_gpu_ssor_chain.py tests/test_gpu_seq_order.py tests/test_gpu_rccl.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log
exit 0
