"""Hashes of ILU(0) results with bf16 factors (the default mode) on the golden pore system and the
config-3 system -- one application, a BiCGSTAB solve (iterate hash and count), an AMG solve with
the ILU(0) smoother -- for comparing two library builds bit for bit (PNP_AMD_LIB selects one).
usage: python tools/ilu_hash.py"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import conftest  # noqa: E402,F401  (puts the package on the path)
import pnp_amd as P  # noqa: E402
from test_gpu import golden  # noqa: E402


def h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


out = {}
z, mesh, par, orc = golden("pore_small_k0")
x = z["newton_pnp_x0"]
ctx = P.Context(mesh, par)
ctx.set_operator(P.OP_PNP)
ctx.jacobian(x, export=False)
rhs = ctx.residual(x)
out["apply"] = h(ctx.prec_apply(rhs, P.PREC_ILU0))
sol, res = ctx.linear_solve(rhs, prec=P.PREC_ILU0, reduction=1e-10, maxit=20000)
out["solve"] = [h(sol), res["iterations"]]
ctx.amg_configure(smoother=P.PREC_ILU0)
sol, res = ctx.linear_solve(rhs, prec=P.PREC_AMG, reduction=1e-10, maxit=20000)
out["amg"] = [h(sol), res["iterations"]]
ctx.close()
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
m3 = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
ctx = P.Context(m3, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PNP)
rng = np.random.default_rng(20261018)
nv = m3.nv
x3 = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                     0.06 * rng.uniform(0.5, 1.5, nv)])
ctx.jacobian(x3, export=False)
r3 = ctx.residual(x3)
out["apply3"] = h(ctx.prec_apply(r3, P.PREC_ILU0))
sol, res = ctx.linear_solve(r3, prec=P.PREC_ILU0, reduction=1e-6, maxit=2000)
out["solve3"] = [h(sol), res["iterations"]]
ctx.close()
print(json.dumps(out), flush=True)
