#!/bin/bash
# round 6: the config-5 FETCH_SIZE / WRITE_SIZE passes at HEAD (separate runs, program after --),
# per-kernel means by tools/pmc_kernels.py; merged into profiles/r06/pmc_config5.json on the host
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; [ "$1" -gt 128 ] && return 0; return 1; }
for set in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d "$OUT/pmc5_$set" -o run -- python3 tools/prof_bicg.py 10 5 > "$OUT/pmc5_$set.log" 2>&1; rc=$?; echo "pmc $set=$rc"; fatal $rc && exit 1
done
python tools/pmc_kernels.py "$(ls "$OUT"/pmc5_FETCH_SIZE/*counter_collection.csv | head -1)" "" "$OUT/pmc5_fetch.json" > /dev/null
python tools/pmc_kernels.py "$(ls "$OUT"/pmc5_WRITE_SIZE/*counter_collection.csv | head -1)" "" "$OUT/pmc5_write.json" > /dev/null
find "$OUT" -name "*.csv" -size +1M -exec gzip -f {} \;
exit 0
