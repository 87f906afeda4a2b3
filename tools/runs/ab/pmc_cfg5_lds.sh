#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE passes (one counter per run) of the config-5 assembly with the direct
# and the LDS-staged walk (tools/prof_cfg5.py k=6, 10 launches).  usage: tools/pmc_cfg5_lds.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
for lds in 0 1; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    PNP_ASM_LDS=$lds timeout -s KILL 150 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$OUT/lds${lds}_$ctr" -o run -- python3 tools/prof_cfg5.py 6 10 > "$OUT/lds${lds}_$ctr.log" 2>&1 \
      || { echo "fail lds=$lds $ctr rc=$?"; exit 1; }
    echo "done lds=$lds $ctr"
  done
done
