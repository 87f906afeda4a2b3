#!/bin/bash
# A/B of two library builds on the bench line (BiCGStab ms/iter, time to solution), interleaved
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_lib_bench.log"
for i in 1 2; do
  for v in new base; do
    PNP_AMD_LIB=dune-pnp_amd/ab/lib_$v.so timeout -k 10 300 python bench.py --no-cpu --steps 10 > "$OUT/ab_lb_$v.log" 2>&1 || exit $?
    python - "$OUT/ab_lb_$v.log" "$v" >> "$OUT/ab_lib_bench.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
t = d["event_timers_ms"]; n = d["pnp_newton_time_to_solution"]
print(sys.argv[2], "ms/it %.4f" % d["bicgstab_ms_per_iter"], "blas_ms/it %.4f" % (t["blas_ms"] / 10),
      "prec_us %.1f" % (1e3 * t["prec_ms"] / max(1, t["prec_launches"])), "asm_us %.1f" % d["roofline"]["avg_launch_us"],
      "newton", n["iterations"], n["linear_iterations"], "%.2fs" % n["seconds"], "conv", n["converged"])
PY
  done
done
