#!/bin/bash
# round 4 validation at HEAD: full GPU suite, smoke, bench (default contract run)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1; echo "bench rc=$?"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/gprof -o run -- python3 tools/graph_prof_check.py > $O/graph_prof_check.log 2>&1; echo "graph prof check rc=$?"
