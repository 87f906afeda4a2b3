#!/bin/bash
# round 5, lease pmc: the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_run.sh (config 3, 10
# assemblies, 10 BiCGSTAB + ILU(0) iterations) at HEAD's defaults (bf16 factors), summarised into
# the per-kernel traffic the bench line's roofline `traffic` and BLAS bytes read
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5pmc
bash tools/gpu_run.sh r5pmc pmcf pmcw; rc=$?; echo "pmc rc=$rc"
[ $rc -ne 0 ] && exit $rc
F=$(ls $O/pmc_fetch/*counter_collection.csv | head -1); W=$(ls $O/pmc_write/*counter_collection.csv | head -1)
python tools/pmc_summary.py "$F" "$W" $O/pmc_summary.json 10 > $O/summary.log 2>&1; rc=$?; echo "summary rc=$rc"
gzip -f "$F" "$W"
rm -f $O/pmc_fetch/*agent_info.csv $O/pmc_write/*agent_info.csv
exit $rc
