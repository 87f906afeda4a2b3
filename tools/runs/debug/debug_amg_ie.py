"""Config 4 (instationary PNP, implicit Euler) first steps with AMG variants: which converge."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
phi, _ = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=P.PREC_SSOR)
u0 = ctx.initial_state(phi)
dt = cfg.system["tau"]
# step 0 with ILU0 -> state u1 (the failing system is step 1's)
ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=u0)
u1, r0 = ctx.newton(u0, reduction=1e-8, abs_limit=1e-9, prec=P.PREC_ILU0)
print(json.dumps({"step0_ilu0": {k_: r0[k_] for k_ in ("converged", "iterations", "linear_iterations", "status")}}), flush=True)
ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=u1)
J = ctx.jacobian(u1, export=False)
r = ctx.residual(u1)
for label, prec, kw in [("ilu0", P.PREC_ILU0, {}), ("amg w1", P.PREC_AMG, dict(omega=1.0)),
                        ("amg w0.8", P.PREC_AMG, dict(omega=0.8)),
                        ("amg w0.5", P.PREC_AMG, dict(omega=0.5)),
                        ("amg ssor w0.8", P.PREC_AMG, dict(omega=0.8, smoother=P.PREC_SSOR))]:
    if prec == P.PREC_AMG:
        kw.setdefault("smoother", P.PREC_ILU0)
        ctx.amg_configure(**kw)
    for red in (1e-4, 1e-8):
        z, res = ctx.linear_solve(r, prec=prec, reduction=red, maxit=3000)
        print(json.dumps({"step1": label, "reduction": red, **{k_: res[k_] for k_ in ("converged", "iterations", "breakdown", "reduction")}}), flush=True)
