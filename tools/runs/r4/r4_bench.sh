#!/bin/bash
# the default bench at HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4_bench; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench.log 2>&1; echo "bench rc=$?"
