#!/bin/bash
# Generic bench A/B over one environment knob:
#   bash tools/ab_env.sh <tag> <VAR> "<values>" [prec...]
# runs bench.py (no CPU leg) per value and prints ms/iteration, preconditioner time per apply,
# assembly time and the PB->PNP time to solution.
set -u
OUT=gpurun_out/$1; VAR=$2; VALS=$3; shift 3
PRECS=${*:-ilu0}
mkdir -p "$OUT"; LOG="$OUT/ab_${VAR}.log"; : > "$LOG"
for prec in $PRECS; do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu --steps 10 --prec "$prec" > "$OUT/ab_${VAR}_${prec}_$v.log" 2>&1 || exit $?
    python - "$OUT/ab_${VAR}_${prec}_$v.log" "$prec" "$VAR=$v" >> "$LOG" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["event_timers_ms"]; n = d["pnp_newton_time_to_solution"]
print(sys.argv[2], sys.argv[3], "colors", d["config"]["colors"], "ms/it %.4f" % d["bicgstab_ms_per_iter"],
      "prec_us/apply %.1f" % (1e3 * t["prec_ms"] / max(1, t["prec_launches"])), "asm_us %.1f" % d["roofline"]["avg_launch_us"],
      "newton", n["iterations"], n["linear_iterations"], "%.2fs" % n["seconds"], "conv", n["converged"])
PY
  done
done
