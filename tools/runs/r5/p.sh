#!/bin/bash
# round 5, lease p: the AMG V-cycle without the x0 memset and with the row-major coarsest GEMV,
# PB with per-vertex e^{u/5}: AMG / PB / assembly GPU tests, the AMG iteration trace split
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5p; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 900 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_amg.py tests/test_gpu_multirank.py tests/test_gpu_graph.py tests/test_config4.py tests/test_gpu.py tests/test_gpu_asm_lds.py tests/test_gpu_fans.py tests/test_equilibrium.py tests/test_gpu_boundary.py tests/test_gpu_pk.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
fatal $rc && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/prof_amg.py run 40 > $O/run.log 2>&1; rc=$?; echo "prof rc=$rc"; grep iters $O/run.log
fatal $rc && exit $rc
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); echo "trace: $f"
python3 tools/prof_amg.py split "$f" 40 > $O/split.txt 2>&1; head -40 $O/split.txt
gzip -c "$f" > $O/trace.csv.gz; rm -rf $O/prof
timeout -k 10 300 python -u tools/bench_amg.py > $O/bench_amg.log 2>&1; rc=$?; echo "bench_amg rc=$rc"; cat $O/bench_amg.log | tail -6
exit 0
