#!/bin/bash
# round 6, final: the whole GPU suite, smoke and the default bench line at HEAD
set -u
O=gpurun_out/$1; mkdir -p "$O"
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > "$O/tests.log" 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 "$O/tests.log"; fatal $rc && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 "$O/smoke.log"; fatal $rc && exit $rc
timeout -k 10 500 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"; rc=$?; echo "bench rc=$rc"
exit $rc
