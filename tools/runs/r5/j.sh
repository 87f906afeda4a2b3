#!/bin/bash
# round 5, lease j: natural SSOR timing with the unit-major ELL, kernel trace, and the PNP head's
# cache counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/${TAG:-r5j}; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ssor_natural.py tests/test_gpu_ssor_chain.py tests/test_gpu_seq_order.py tests/test_gpu_rccl.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
fatal $rc && exit $rc
for i in 1 2; do
timeout -k 10 200 python -u tools/bench_ssor_natural.py 4 > $O/nat$i.log 2>&1; rc=$?; echo "nat rc=$rc"; cat $O/nat$i.log
fatal $rc && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/bench_ssor_natural.py 4 > $O/trace.log 2>&1; rc=$?; echo "trace rc=$rc"
fatal $rc && exit $rc
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_mem -o run -- python3 tools/bench_ssor_natural.py 4 > $O/pmc_mem.log 2>&1; rc=$?; echo "pmc_mem rc=$rc"
exit 0
