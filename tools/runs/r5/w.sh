#!/bin/bash
# round 5, lease w: the N = 2 bench rehearsal through the host-staged transport at HEAD (AMG f32,
# PB exps, rccl_parity at 1e-8 linear solves)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --transport host --steps 3 --warmup 1 --bicg-iters 5 --no-cpu > $O/bench2.log 2>&1; rc=$?; echo "bench N=2 host rc=$rc"
python3 - <<'PY'
import json
d=[json.loads(l) for l in open("gpurun_out/r5w/bench2.log") if l.startswith("{")]
if d:
    d=d[-1]; r=d.get("rccl_parity") or {}
    print("value", d["value"], "n_gpus", d["n_gpus"], "parity", r.get("pass"), r.get("solution_rel_err"), r.get("transport"))
    print("nat", json.dumps(d.get("bicgstab_ssork_natural", {}).get("pnp", {}))[:300])
PY
exit $rc
