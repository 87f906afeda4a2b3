#!/bin/bash
# rocprofv3 --kernel-trace on hipGraph replays: is it the node count of one graph or the count of
# graph-launched kernels? (verdict round 3 item 4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r4g; mkdir -p $O
export TMPDIR=/tmp
for spec in "100:200" "3000:1" "4000:1" "2000:6"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/p_${spec/:/_} -o run -- tools/micro/graph_capture_prof $spec > $O/prof_${spec/:/_}.log 2>&1; echo "$spec rc=$?" | tee -a $O/summary.txt
done
