#!/bin/bash
# A/B: colouring (PNP_COLORING=greedy vs smallest-last + balancing), bench incl. time to solution
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_coloring.log"
for prec in ${PRECS:-ilu0 ssor}; do
  for c in sl greedy; do
    PNP_COLORING=$c timeout -k 10 300 python bench.py --no-cpu --steps 10 --prec $prec > "$OUT/col_${prec}_$c.log" 2>&1 || exit $?
    python - "$OUT/col_${prec}_$c.log" $prec $c >> "$OUT/ab_coloring.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["event_timers_ms"]; n = d["pnp_newton_time_to_solution"]
print(sys.argv[2], sys.argv[3], "colors", d["config"]["colors"], "ms/it %.4f" % d["bicgstab_ms_per_iter"],
      "prec_us/apply %.1f" % (1e3 * t["prec_ms"] / max(1, t["prec_launches"])), "asm_us %.1f" % d["roofline"]["avg_launch_us"],
      "newton", n["iterations"], n["linear_iterations"], "%.2fs" % n["seconds"], "conv", n["converged"])
PY
  done
done
