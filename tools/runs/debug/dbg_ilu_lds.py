import hashlib, json, sys, os
import numpy as np
sys.path.insert(0, "tests")
import conftest  # noqa
from test_gpu import golden
import pnp_amd as P
out = {}
def h(a): return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()[:10]
z, mesh, par, orc = golden("pore_small_k0")
ctx = P.Context(mesh, par)
ctx.set_operator(P.OP_PB)
J = ctx.jacobian(np.zeros(mesh.nv), export=False)
rhs = ctx.residual(np.zeros(mesh.nv))
out["pb_apply"] = h(ctx.prec_apply(rhs, P.PREC_ILU0))
sol, res = ctx.linear_solve(rhs, prec=P.PREC_ILU0, reduction=1e-10, maxit=2000)
out["pb_solve"] = [h(sol), res["it_half"]]
phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0)
out["pb_newton"] = [h(phi), rpb["linear_iterations"]]
x0 = ctx.initial_state(phi)
ctx.set_operator(P.OP_PNP)
J = ctx.jacobian(x0, export=False)
r0 = ctx.residual(x0)
out["pnp_apply_x0"] = h(ctx.prec_apply(r0, P.PREC_ILU0))
sol, res = ctx.linear_solve(r0, prec=P.PREC_ILU0, reduction=1e-8, maxit=20000)
out["pnp_solve_x0"] = [h(sol), res["it_half"]]
u, res = ctx.newton(x0, prec=P.PREC_ILU0)
out["pnp_newton"] = [h(u), res["linear_iterations"], list(ctx.newton_history()[0].tolist())]
ctx2 = P.Context(mesh, par); ctx2.set_operator(P.OP_PNP)
u2, res2 = ctx2.newton(x0, prec=P.PREC_ILU0)
out["pnp_newton_fresh"] = [h(u2), res2["linear_iterations"], list(ctx2.newton_history()[0].tolist())]
print(json.dumps(out))
