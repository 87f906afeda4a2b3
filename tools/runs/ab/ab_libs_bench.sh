#!/bin/bash
# A/B of library builds on the bench line incl. the config-5 leg (no CPU baseline, AMG or RCCL
# self-check), one run per build, interleaved twice.  usage: tools/ab_libs_bench.sh <tag> <lib>...
# (lib "-" = in-tree, else dune-pnp_amd/ab/lib_<lib>.so)
set -u
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; : > "$OUT/ab.log"
for i in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then libenv=""; else libenv="PNP_AMD_LIB=dune-pnp_amd/ab/lib_$lib.so"; fi
    env $libenv timeout -k 10 400 python bench.py --no-cpu --no-amg --no-parity > /tmp/abl_line.json 2>/tmp/abl_err.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "$lib rc=$rc" >> "$OUT/ab.log"; tail -5 /tmp/abl_err.log >> "$OUT/ab.log"; exit $rc; fi
    python - "$lib" >> "$OUT/ab.log" <<'PY'
import json, sys
d = json.loads([l for l in open("/tmp/abl_line.json") if l.startswith("{")][-1])
t = d["event_timers_ms"]; S = d["strong_scaling"]; n = d["pnp_newton_time_to_solution"]
print(f"{sys.argv[1]:6s} cfg3 asm {d['roofline']['avg_launch_us']:.1f} in-situ {d['roofline_in_situ']['avg_launch_us']:.1f} | "
      f"bicg {d['bicgstab_ms_per_iter']*1e3:.1f} us prec/apply {t['prec_ms']/max(1,t['prec_launches'])*1e3:.1f} | "
      f"newton {n['linear_iterations']} {n['seconds']:.2f}s | cfg5 bicg {S['bicgstab_ms_per_iter']*1e3:.1f} "
      f"ilu {S['ilu0_apply_stored']['seconds']*1e6:.1f} asm {S['roofline_assembly_warm']['seconds']*1e6:.1f}")
PY
  done
done
cat "$OUT/ab.log"
