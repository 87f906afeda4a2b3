#!/bin/bash
# round 4 validation at HEAD (chains and the pipelined head by default): full GPU suite, smoke, bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4_val; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread -rf > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc"
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"
