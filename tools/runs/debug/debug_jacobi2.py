"""Debug helper (GPU): export candidate test systems (J, r) for offline robustness checks."""
import os, sys
import numpy as np
import scipy.sparse as sp
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P
from test_gpu import golden
OUT = os.path.join(ROOT, "gpurun_out")
for name, key in (("cylinder_k0", "newton_pnp_x0"), ("pore_small_k0", "newton_pnp_x0")):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    x = z[key]
    J = ctx.jacobian(x)
    r = ctx.residual(x)
    sp.save_npz(os.path.join(OUT, f"{name}_J0.npz"), J.tocsr())
    np.save(os.path.join(OUT, f"{name}_r0.npy"), r)
    for prec in (P.PREC_NONE, P.PREC_JACOBI):
        zz, res = ctx.linear_solve(r, prec=prec, reduction=1e-8, maxit=20000)
        print(name, "prec", prec, {k: res[k] for k in ("converged", "iterations", "breakdown")}, flush=True)
    u, res = ctx.newton(x, prec=P.PREC_NONE)
    print(name, "newton NOPREC", {k: res[k] for k in ("converged", "status", "iterations", "linear_iterations")}, flush=True)
