#!/bin/bash
# A/B of AMG knobs on bench_amg's PNP legs
OUT=gpurun_out/$1; shift; mkdir -p $OUT; : > $OUT/ab.log
for v in "$@"; do
  echo "== $v" >> $OUT/ab.log
  env $v timeout -k 10 200 python tools/bench_amg.py 4 2>&1 | grep "PNP newton BiCGSTAB+AMG" >> $OUT/ab.log || exit 1
done
cat $OUT/ab.log
