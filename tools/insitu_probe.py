"""What the config-3 Jacobian assembly's in-situ penalty depends on: the launch timed
alone (HIP event pair, median of 10 after one untimed) after different predecessors --
  warm          another assembly;
  in_situ       20 BiCGSTAB + ILU(0) iterations (bench.py's `roofline`);
  sleep5ms      the same, then 5 ms of idle GPU (clocks / power state);
  scrub64/512   the same, then a read-only pass over 64 / 512 MiB of scratch (clean lines replace
                what the solve left in the Infinity Cache);
  ilu_only      20 ILU(0) applications through pnp_prec_apply (no SpMV, no vector updates);
  cold          a 1 GiB read-only scrub alone.
One JSON line.  usage: python tools/insitu_probe.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PNP)
rng = np.random.default_rng(20261017)
nv = mesh.nv
x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                    0.06 * rng.uniform(0.5, 1.5, nv)])
ctx.state_set(x)
ctx.assemble_state(2)
ctx.bicgstab_iterations(2, P.PREC_ILU0)
d = rng.uniform(-1, 1, 3 * nv)


def pre(mode):
    if mode == "warm":
        ctx.assemble_state(1)
        return
    if mode == "cold":
        ctx.cache_scrub(1 << 30)
        return
    if mode == "ilu_only":
        for _ in range(20):
            ctx.prec_apply(d, P.PREC_ILU0)
        return
    ctx.bicgstab_iterations(20, P.PREC_ILU0)
    if mode == "sleep5ms":
        time.sleep(0.005)
    elif mode == "scrub64":
        ctx.cache_scrub(64 << 20)
    elif mode == "scrub512":
        ctx.cache_scrub(512 << 20)


out = {}
modes = ("warm", "in_situ", "sleep5ms", "scrub64", "scrub512", "ilu_only", "cold")
for rnd in range(2):  # two interleaved rounds
    for mode in modes:
        ts = []
        for rep in range(11):
            pre(mode)
            ts.append(ctx.assemble_state_timed(1) * 1e6)
        out.setdefault(mode + "_us", []).append(round(float(np.median(ts[1:])), 2))
ctx.close()
print(json.dumps(out), flush=True)
