#!/bin/bash
# Sweep shape A/B (PNP_SWEEP = lanes per row x slot batch) on the bench line, with the PNP Newton
# time to solution (the shape changes the summation order, hence the BiCGSTAB trajectory).
# usage: tools/ab_sweep_shape.sh <tag> <shapes...>
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; : > "$OUT/ab_sweep.log"
for round in 1 2; do
  for sh in "$@"; do
    PNP_SWEEP=$sh timeout -k 10 300 python bench.py --no-cpu --no-strong --no-amg --steps 10 > "$OUT/b_$sh.json" 2>&1 || exit $?
    python - "$OUT/b_$sh.json" "$sh" >> "$OUT/ab_sweep.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["event_timers_ms"]; n = d["pnp_newton_time_to_solution"]
print(sys.argv[2], "ms/it %.4f" % d["bicgstab_ms_per_iter"], "prec_us %.1f" % (1e3 * t["prec_ms"] / max(1, t["prec_launches"])),
      "newton %.2f s %d lin" % (n["seconds"], n["linear_iterations"]))
PY
  done
done
