#!/bin/bash
# round 5, lease s: the AMG's coarsest inverse in single precision too (PNP_AMG_F32): AMG tests
# both ways, interleaved wall A/B of the iteration, bench_amg
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5s; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_amg.py tests/test_gpu_multirank.py tests/test_config4.py tests/test_gpu_pk.py > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log
fatal $rc && exit $rc
PNP_AMG_F32=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread -m gpu tests/test_gpu_amg.py > $O/tests_f64.log 2>&1; rc=$?; echo "tests f64 rc=$rc"; tail -2 $O/tests_f64.log
fatal $rc && exit $rc
for rep in 1 2; do
  for f in 0 1; do
    PNP_AMG_F32=$f timeout -k 10 300 python -u tools/prof_amg.py run 40 > $O/ab_$f.$rep.log 2>&1; rc=$?
    echo "f32=$f rep $rep: $(cat $O/ab_$f.$rep.log)"; fatal $rc && exit $rc
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/prof_amg.py run 40 > $O/run.log 2>&1; rc=$?; echo "prof rc=$rc"
fatal $rc && exit $rc
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/prof_amg.py split "$f" 40 > $O/split.txt 2>&1; head -10 $O/split.txt; grep coarse $O/split.txt
gzip -c "$f" > $O/trace.csv.gz; rm -rf $O/prof
timeout -k 10 300 python -u tools/bench_amg.py > $O/bench_amg.log 2>&1; rc=$?; echo "bench_amg rc=$rc"; tail -3 $O/bench_amg.log
exit 0
