#!/bin/bash
# round 5, lease b: stream shapes, natural-SSOR pipe for PNP (KS=4) tests + timing, RCCL flow test
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5b; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 120 python -c "
import sys; sys.path.insert(0,'.'); import bench, json
print(json.dumps(bench.measured_stream_gbs(0)))" > $O/stream.log 2>&1; rc=$?; echo "stream rc=$rc"; cat $O/stream.log
fatal $rc && exit $rc
timeout -k 10 200 python -u tools/bench_ssor_natural.py 4 > $O/nat.log 2>&1; rc=$?; echo "nat rc=$rc"; cat $O/nat.log
fatal $rc && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_rccl.py tests/test_gpu_ssor_natural.py tests/test_gpu_ssor_chain.py tests/test_gpu_ilu_flow.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
exit 0
