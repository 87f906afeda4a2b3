#!/bin/bash
# round 5, lease bb: the LDS sweeps' slot batch with bf16 factors (PNP_ILU_LDS_B 2 / 3 / 4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5bb; mkdir -p $O
for rep in 1 2; do
  for b in 2 3 4; do
    PNP_ILU_LDS_B=$b timeout -k 10 300 python -u tools/ab_ilu_bf16.py 2 > $O/b$b.$rep.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.load(open('$O/b$b.$rep.log')); print('B=$b rep $rep', 'bf16', round(d['bf16']['apply_us_median'],2), round(d['bf16']['iter_ms_median'],4), 'f32', round(d['f32']['apply_us_median'],2))"
  done
done
exit 0
