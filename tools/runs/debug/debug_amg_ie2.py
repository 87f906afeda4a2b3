"""Config 4 with AMG(ILU0) from step 0, as tools/bench_configs.py runs it; stops at a failure."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
om = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
phi, _ = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=P.PREC_SSOR)
u = ctx.initial_state(phi)
dt = cfg.system["tau"]
for i in range(4):
    ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=u)
    ctx.amg_configure(smoother=P.PREC_ILU0, omega=om)
    u, res = ctx.newton(u, reduction=1e-8, abs_limit=1e-9, prec=P.PREC_AMG, linear_maxit=3000)
    print(json.dumps({"step": i, **{k_: res[k_] for k_ in ("converged", "iterations", "linear_iterations", "status", "first_defect", "defect")}}), flush=True)
    if not res["converged"]:
        break
