#!/bin/bash
# A/B of an environment knob on the bench line (config 3): alternates the settings, 2 rounds.
# usage: tools/ab_env_bench.sh <out.log> "<VAR=a>" "<VAR=b>" [extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; A=$2; B=$3; shift 3
: > "$OUT"
for round in 1 2; do
  for setting in "$A" "$B"; do
    echo "== $setting round $round" >> "$OUT"
    env $setting timeout -k 10 300 python bench.py --no-cpu --no-strong --no-amg "$@" > /tmp/ab_line.json 2>/tmp/ab_err.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc" >> "$OUT"; tail -5 /tmp/ab_err.log >> "$OUT"; exit $rc; fi
    python - >> "$OUT" <<'PY'
import json
d = json.loads(open("/tmp/ab_line.json").read())
t = d["event_timers_ms"]
n = d["pnp_newton_time_to_solution"]
situ = d.get("roofline_in_situ") or {}
msg = (f"asm {d['roofline']['avg_launch_us']:.1f} us cold {d['roofline_cold']['avg_launch_us']:.1f} us "
       f"in-situ {situ.get('avg_launch_us', float('nan')):.1f} us | "
       f"bicg {d['bicgstab_ms_per_iter']*1e3:.1f} us/it  prec/apply {t['prec_ms']/max(1,t['prec_launches'])*1e3:.1f} us "
       f"spmv {t['spmv_ms']/max(1,t['spmv_launches'])*1e3:.1f} us blas/it {t['blas_ms']/20*1e3:.1f} us")
if n:
    msg += (f" | newton {n['seconds']:.2f} s {n['iterations']} its {n['linear_iterations']} lin "
            f"conv {n['converged']}")
print(msg)
PY
  done
done
cat "$OUT"
