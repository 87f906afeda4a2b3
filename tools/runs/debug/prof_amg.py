"""Profiling target: AMG V-cycles (PNP, ILU0 smoother and PB, SSOR smoother) at config 3."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
phi, _ = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_SSOR)
ctx.jacobian(phi, export=False)
for _ in range(10):
    ctx.prec_apply(np.ones(mesh.nv), P.PREC_AMG)
x0 = ctx.initial_state(phi)
ctx.set_operator(P.OP_PNP)
ctx.amg_configure(smoother=P.PREC_ILU0)
ctx.jacobian(x0, export=False)
for _ in range(10):
    ctx.prec_apply(np.ones(3 * mesh.nv), P.PREC_AMG)
ctx.close()
