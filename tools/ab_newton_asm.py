"""The Jacobian assembly as PDELab's Newton issues it, config 3, one MI355X: after a BiCGSTAB solve
(20 iterations of BiCGSTAB + ILU(0)) the line search assembles the residual at the new state, and
only then does the next Newton step assemble the Jacobian.  Times (HIP events, one launch each,
median of 10) the Jacobian launch in that order ("newton"), directly after the solve (bench.py's
roofline_in_situ, "in_situ") and back to back ("warm").  Run with PNP_ASM_COLD_HINT=0/1 to A/B
the walk an assembly after a solve takes.  usage: python tools/ab_newton_asm.py"""
import json
import os
import sys

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
out = {"hint": os.environ.get("PNP_ASM_COLD_HINT", "default")}
for mode in ("warm", "in_situ", "newton"):
    ts = []
    for rep in range(11):
        if mode != "warm":
            ctx.bicgstab_iterations(20, P.PREC_ILU0)
        if mode == "newton":
            ctx.assemble_state(-1)  # the line search's residual at the new state
        ts.append(ctx.assemble_state_timed(1) * 1e6)
    out[mode + "_us"] = float(np.median(ts[1:]))
print(json.dumps(out), flush=True)
