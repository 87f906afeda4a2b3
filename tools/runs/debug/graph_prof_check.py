"""Under rocprofv3 --kernel-trace: the environment the profiler gives this process (ROCPROF_*) and
a BiCGSTAB run that would replay hipGraphs (pore_small, graph auto) for more than 20,000 kernels,
which crashed the profiler before graph replay turned itself off under it."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pnp_amd as P  # noqa: E402
from test_gpu import golden  # noqa: E402

print("ROCPROF env:", sorted(k for k in os.environ if k.startswith("ROCPROF")), flush=True)
z, mesh, par, orc = golden("pore_small_k0")
ctx = P.Context(mesh, par)
ctx.set_operator(P.OP_PNP)
ctx.jacobian(z["newton_pnp_x0"], export=False)
rhs = ctx.residual(z["newton_pnp_x0"])
for _ in range(12):  # ~12 x 200 iterations x ~10 kernels
    sol, res = ctx.linear_solve(rhs, prec=P.PREC_ILU0, reduction=1e-30, maxit=200)
print("done", res["iterations"], flush=True)
