"""Per-iteration BiCGSTAB trace of a Jacobi solve (PNP_DEBUG_BICGSTAB=1) next to the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import test_gpu as T  # noqa: E402
import pnp_amd as P  # noqa: E402
import oracle_py as O  # noqa: E402

z, mesh, par, orc = T.golden("pore_small_k0")
ctx = P.Context(mesh, par)
op = T.set_ops(z, ctx, orc, "pnp")
x = z["pnp_x"]
J = ctx.jacobian(x)
rhs = ctx.residual(x)
for prec in (P.PREC_JACOBI, P.PREC_NONE):
    sol, res = ctx.linear_solve(rhs, prec=prec, reduction=1e-10, maxit=60, check_every=1)
    print("gpu", prec, res, flush=True)
    xo, ro = O.bicgstab(orc.jacobian(op, x), rhs, prec=prec, reduction=1e-10, maxit=60)
    print("oracle", prec, ro.converged, ro.iterations, ro.breakdown, ro.defect, flush=True)
