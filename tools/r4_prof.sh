#!/bin/bash
# round 4 final: rocprofv3 kernel trace + stats of the default bench at HEAD
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4_prof; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu > $O/bench_prof.log 2>&1; echo "prof rc=$?"
