#!/bin/bash
# Interleaved A/B of the assembly walk on config 2 (cylinder k=6, 1.11M rows: just past the
# auto threshold of the LDS walk): PNP_ASM_LDS=0 (direct) vs unset (auto).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab.log"
for i in 1 2; do
  for v in 0 auto; do
    echo "PNP_ASM_LDS=$v:" >> "$OUT/ab.log"
    if [ $v = auto ]; then
      timeout -k 10 200 python tools/bench_configs.py 2 >> "$OUT/ab.log" 2>&1 || exit 1
    else
      PNP_ASM_LDS=$v timeout -k 10 200 python tools/bench_configs.py 2 >> "$OUT/ab.log" 2>&1 || exit 1
    fi
  done
done
