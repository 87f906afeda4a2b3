#!/bin/bash
# round 5, lease bf: bfloat16 ILU(0) factors (PNP_OPT_ILU_F32 = 2) -- apply time A/B, the config-3
# Newton count spread, the whole bench line and the GPU suite with bf16 as the default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5bf; mkdir -p $O
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
timeout -k 10 300 python -u tools/ab_ilu_bf16.py 3 > $O/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; cat $O/ab.log | cut -c1-400
fatal $rc && exit $rc
PNP_ILU_F32=2 timeout -k 10 400 python -u tools/tts_spread.py 6 > $O/spread_bf16.log 2>&1; rc=$?; echo "spread rc=$rc: $(tail -1 $O/spread_bf16.log)"
fatal $rc && exit $rc
PNP_ILU_F32=2 timeout -k 10 600 python -u bench.py --no-cpu > $O/bench_bf16.log 2>&1; rc=$?; echo "bench rc=$rc"
fatal $rc && exit $rc
PNP_ILU_F32=2 timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > $O/tests_bf16.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -8 $O/tests_bf16.log
exit 0
