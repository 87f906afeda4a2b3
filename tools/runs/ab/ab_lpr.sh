#!/bin/bash
# A/B of the sweep kernels' shape (PNP_SWEEP = lanes-per-row x slot batch) on config 3
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; : > "$OUT/ab_sweep.log"
run() {  # prec cfg
  PNP_SWEEP=$2 timeout -k 10 200 python bench.py --no-cpu --no-solve --steps 10 --prec $1 > "$OUT/sw_$1_$2.log" 2>&1
  local rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc prec=$1 cfg=$2" >> "$OUT/ab_sweep.log"; return $rc; }
  python - "$OUT/sw_$1_$2.log" $1 $2 >> "$OUT/ab_sweep.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["event_timers_ms"]
print(sys.argv[2], sys.argv[3], "ms/it %.4f" % d["bicgstab_ms_per_iter"],
      "prec_us/apply %.1f" % (1e3 * t["prec_ms"] / max(1, t["prec_launches"])),
      "frac_it %.3f" % d["roofline_bicgstab"]["frac"])
PY
}
for cfg in ${CFGS:-1x1 1x2 1x4 1x8 2x1 2x2 2x4 4x2}; do run ilu0 $cfg || exit $?; done
for cfg in ${SSOR_CFGS:-1x4 2x2}; do run ssor $cfg || exit $?; done
