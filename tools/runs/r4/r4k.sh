#!/bin/bash
# round 4 measurement: PMC FETCH/WRITE passes on the profiling target (10 assemblies, 10 BiCGSTAB
# ILU(0) iterations), then the bench under rocprofv3 kernel trace + stats (regime split source)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_run.sh r4k pmcf pmcw || exit $?
O=gpurun_out/r4k
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu --no-solve --steps 20 > $O/prof.log 2>&1; echo "prof rc=$?"
