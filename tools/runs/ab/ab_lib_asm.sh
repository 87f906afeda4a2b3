#!/bin/bash
# A/B of two library builds (dune-pnp_amd/ab/lib_new.so vs lib_base.so) on the assembly timings of
# the bench line (warm / cache-cold / in situ) and the BiCGStab iteration, interleaved, 2 rounds.
# usage: tools/ab_lib_asm.sh <tag> [extra bench args]
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; : > "$OUT/ab_lib_asm.log"
for i in 1 2; do
  for v in new base; do
    PNP_AMD_LIB=dune-pnp_amd/ab/lib_$v.so timeout -k 10 300 python bench.py --no-cpu --no-strong --no-amg --steps 10 "$@" > "$OUT/ab_la_$v.log" 2>&1 || exit $?
    python - "$OUT/ab_la_$v.log" "$v" >> "$OUT/ab_lib_asm.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
n = d["pnp_newton_time_to_solution"] or {}
print(sys.argv[2], "asm %.1f cold %.1f in-situ %.1f us" % (d["roofline"]["avg_launch_us"], d["roofline_cold"]["avg_launch_us"],
      d["roofline_in_situ"]["avg_launch_us"]), "bicg %.1f us/it" % (1e3 * d["bicgstab_ms_per_iter"]),
      "newton", n.get("iterations"), n.get("linear_iterations"), "%.2fs" % n.get("seconds", 0))
PY
  done
done
cat "$OUT/ab_lib_asm.log"
