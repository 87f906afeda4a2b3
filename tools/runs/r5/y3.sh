#!/bin/bash
# round 5, lease y3: the single-precision forward intermediate (PNP_OPT_ILU_F32 = 3) -- the ILU(0)
# tests that cover it, the interleaved 2 / 3 A/B, and the per-config BiCGSTAB trace split with 3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5y3; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -rf tests/test_gpu.py -k "ilu0" tests/test_gpu_ilu_lds.py tests/test_gpu_xdefer.py tests/test_gpu_ilu_flow.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log
fatal $rc && exit $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_ilu_bf16.py 3 2,3 > $O/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cut -c1-600 $O/ab.log
fatal $rc && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/bicg -o run -- python3 tools/prof_bicg.py 20 3,5 > $O/prof_bicg.log 2>&1; rc=$?; echo "prof_bicg rc=$rc"
fatal $rc && exit $rc
python tools/bicg_split.py $O/bicg/run_kernel_trace.csv $O/prof_bicg.log $O/bicg_split.json > $O/bicg_split.txt 2>&1
head -4 $O/bicg_split.txt; sed -n 21,24p $O/bicg_split.txt
gzip -f $O/bicg/run_kernel_trace.csv
rm -f $O/bicg/run_agent_info.csv
exit 0
