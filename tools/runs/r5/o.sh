#!/bin/bash
# round 5, lease o: where a BiCGSTAB + AMG(ILU(0)) iteration's time goes at config 3 (kernel trace)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5o; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/prof_amg.py run 40 > $O/run.log 2>&1; rc=$?; echo "prof rc=$rc"; tail -2 $O/run.log
[ $rc -ne 0 ] && exit $rc
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); echo "trace: $f"
python3 tools/prof_amg.py split "$f" 40 > $O/split.txt 2>&1; head -50 $O/split.txt
s=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$s" $O/kernel_stats.csv
gzip -c "$f" > $O/trace.csv.gz; rm -rf $O/prof
exit 0
