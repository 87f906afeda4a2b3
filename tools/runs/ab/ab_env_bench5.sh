#!/bin/bash
# A/B of an environment knob on the bench line including the config-5 strong leg (no CPU
# baseline, AMG or RCCL self-check), alternating the settings, 2 rounds.
# usage: tools/ab_env_bench5.sh <out.log> "<VAR=a>" "<VAR=b>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1; A=$2; B=$3
: > "$OUT"
for round in 1 2; do
  for setting in "$A" "$B"; do
    echo "== $setting round $round" >> "$OUT"
    env $setting timeout -k 10 400 python bench.py --no-cpu --no-amg --no-parity > /tmp/ab5_line.json 2>/tmp/ab5_err.log
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc" >> "$OUT"; tail -5 /tmp/ab5_err.log >> "$OUT"; exit $rc; fi
    python - >> "$OUT" <<'PY'
import json
d = json.loads(open("/tmp/ab5_line.json").read())
t = d["event_timers_ms"]; S = d["strong_scaling"]
print(f"cfg3 asm {d['roofline']['avg_launch_us']:.1f} in-situ {d['roofline_in_situ']['avg_launch_us']:.1f} "
      f"cold {d['roofline_cold']['avg_launch_us']:.1f} us | bicg {d['bicgstab_ms_per_iter']*1e3:.1f} us "
      f"spmv {t['spmv_ms']/max(1,t['spmv_launches'])*1e3:.1f} | cfg5 asm {S['roofline_assembly_warm']['seconds']*1e6:.1f} "
      f"in-situ {S['roofline_assembly_in_situ']['seconds']*1e6:.1f} us bicg {S['bicgstab_ms_per_iter']*1e3:.1f} us "
      f"spmv {S['spmv_stored']['seconds']*1e6:.1f} ilu {S['ilu0_apply_stored']['seconds']*1e6:.1f}")
PY
  done
done
cat "$OUT"
