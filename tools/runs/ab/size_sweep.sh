#!/bin/bash
# Assembly time vs mesh size: config-5 geometry k=4..6 and pore_pnp (config 3 geometry) k=4,5,
# plus FETCH/WRITE PMC passes at config 5 k=6.  usage: tools/size_sweep.sh <tag>
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/sweep.log"
for k in 4 5 6; do
  timeout -k 10 200 python tools/prof_cfg5.py $k 20 >> "$OUT/sweep.log" 2>&1 || exit 1
done
for k in 4 5; do
  timeout -k 10 200 python tools/ab_asm.py $k >> "$OUT/sweep.log" 2>&1 || exit 1
done
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 tools/prof_cfg5.py 6 10 > "$OUT/pmcf.log" 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run -- python3 tools/prof_cfg5.py 6 10 > "$OUT/pmcw.log" 2>&1 || exit 1
cat "$OUT/sweep.log"
