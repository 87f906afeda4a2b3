#!/bin/bash
# chain kernel: kernel trace of the natural SSOR applications (head / chain split, spread per launch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4q; mkdir -p $O
export TMPDIR=/tmp
for T in 8192 16384; do
  PNP_NAT_CHAIN=$T timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_$T -o run -- python3 tools/bench_ssor_natural.py 4 > $O/bench_$T.log 2>&1 || exit $?
  f=$(ls $O/prof_$T/*/run_kernel_trace.csv 2>/dev/null | head -n 1); [ -z "$f" ] && f=$(ls $O/prof_$T/run_kernel_trace.csv)
  python3 tools/nat_split.py $f > $O/split_$T.txt 2>&1
done
