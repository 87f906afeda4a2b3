#!/bin/bash
# hipGraph replay A/B (PNP_GRAPH): config 4 as specified (test/pore.msh, launch-bound) and the
# config-3 bench line (GPU-bound), interleaved.  usage: tools/ab_graph.sh <tag>
set -u
OUT=gpurun_out/$1; mkdir -p "$OUT"; : > "$OUT/ab_graph.log"
for i in 1 2; do
  for g in 1 0; do
    echo "== PNP_GRAPH=$g round $i" >> "$OUT/ab_graph.log"
    PNP_GRAPH=$g timeout -k 10 200 python tools/bench_configs.py 4 >> "$OUT/ab_graph.log" 2>&1 || exit $?
    PNP_GRAPH=$g timeout -k 10 300 python bench.py --no-cpu --no-strong --no-amg --steps 10 > "$OUT/b_$g.json" 2>&1 || exit $?
    python - "$OUT/b_$g.json" >> "$OUT/ab_graph.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
n = d["pnp_newton_time_to_solution"]
print("config3 bicg ms/it %.4f" % d["bicgstab_ms_per_iter"], "newton %.3f s %d lin" % (n["seconds"], n["linear_iterations"]))
PY
  done
done
