#!/bin/bash
# round 5, lease a: stream ceilings, the new flow-path tests, BiCGSTAB per-config trace,
# natural-SSOR head counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5a; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'.'); import bench, json
print(json.dumps(bench.measured_stream_gbs(0)))" > $O/stream.log 2>&1; rc=$?; echo "stream rc=$rc"; cat $O/stream.log
fatal $rc && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_ilu_flow.py tests/test_gpu_ssor_natural.py tests/test_gpu_ssor_chain.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
fatal $rc && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 tools/prof_bicg.py 20 3,5 > $O/prof_bicg.log 2>&1; rc=$?; echo "trace rc=$rc"
fatal $rc && exit $rc
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/pmc_sq -o run -- python3 tools/bench_ssor_natural.py 4 > $O/pmc_sq.log 2>&1; rc=$?; echo "pmc_sq rc=$rc"
fatal $rc && exit $rc
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc_mem -o run -- python3 tools/bench_ssor_natural.py 4 > $O/pmc_mem.log 2>&1; rc=$?; echo "pmc_mem rc=$rc"
exit 0
