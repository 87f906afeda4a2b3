#!/bin/bash
# round 5: the whole GPU suite, smoke, the default bench line, the bench's kernel trace (assembly
# regimes, natural-SSOR split) and the per-config BiCGSTAB trace split; raw traces are summarised
# on the box and kept gzipped (gpurun copies back at most 64 MiB).  TAG names the output directory;
# NOTESTS=1 skips the suite, NOPROF=1 the profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/${TAG:-r5full}; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
if [ "${NOTESTS:-0}" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log
fatal $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
fatal $rc && exit $rc
fi
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 400 $O/bench.log
fatal $rc && exit $rc
[ "${NOPROF:-0}" = 1 ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-per-config > $O/prof.log 2>&1; rc=$?; echo "prof rc=$rc"
fatal $rc && exit $rc
python tools/asm_regimes.py $O/prof/run_kernel_trace.csv 353561080 $O/asm_regimes_config3.json "k_assemble_ga<0, 1, 3, 9, 6" 738048 > $O/asm_regimes.log 2>&1
python tools/nat_split.py $O/prof/run_kernel_trace.csv > $O/nat_split.log 2>&1
gzip -f $O/prof/run_kernel_trace.csv
rm -f $O/prof/run_agent_info.csv
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/bicg -o run -- python3 tools/prof_bicg.py 20 3,5 > $O/prof_bicg.log 2>&1; rc=$?; echo "prof_bicg rc=$rc"
fatal $rc && exit $rc
python tools/bicg_split.py $O/bicg/run_kernel_trace.csv $O/prof_bicg.log $O/bicg_split.json > $O/bicg_split.txt 2>&1
gzip -f $O/bicg/run_kernel_trace.csv
rm -f $O/bicg/run_agent_info.csv
du -sh $O
exit 0
