#!/bin/bash
# natural SSOR split per launch (head / chains) at the defaults: kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 tools/bench_ssor_natural.py 4 > $O/bench.log 2>&1
