#!/bin/bash
# round 5, lease ye: PNP_OPT_ILU_F32 = 3 against 2 on the config-5 system where 3 stalled
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5ye; mkdir -p $O
timeout -k 10 500 python -u tools/ilu_y32_err.py > $O/err.log 2>&1; rc=$?; echo "err rc=$rc"; cut -c1-3000 $O/err.log
exit $rc
