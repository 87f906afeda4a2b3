"""Why BiCGSTAB + AMG diverged on config-4 systems in round 1.

Runs config 4 (implicit Euler, pore_pnp k=3) with the round-1 AMG shape (coarsest level <= 64
blocks, omega 1.0, post-smoothing only) until the first step whose AMG solve fails, then on that
Newton system compares the round-1 hierarchy with the current default (coarsest <= 1024 blocks,
dense LU):
  * per coarse level, the spectral radius of the damped block-Jacobi iteration matrix
    I - omega D^-1 A_c (the coarse smoother; > 1 means a sweep amplifies some error modes);
  * the eigenvalues of the AMG-preconditioned operator A B with the smallest real parts (ARPACK
    on A B, B = one V-cycle through pnp_prec_apply, A = the exported Jacobian).
usage: python tools/amg_c4_analyse.py [k]"""
import json
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
nv = mesh.nv
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
phi, _ = ctx.newton(np.zeros(nv), reduction=1e-9, prec=P.PREC_SSOR)
u = ctx.initial_state(phi)
dt = cfg.system["tau"]
R1 = dict(smoother=P.PREC_ILU0, coarse_target=64, omega=1.0, level0_presmooth=-1)
NOW = dict(smoother=P.PREC_ILU0, coarse_target=1024, omega=0.8, level0_presmooth=-1)
fail = None
for i in range(20):
    ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=u)
    ctx.amg_configure(**R1)
    u_prev = u.copy()
    u, res = ctx.newton(u, reduction=1e-8, abs_limit=1e-9, prec=P.PREC_AMG)
    if res["linear_fallbacks"]:
        fail = (i, u_prev)
        break
print(json.dumps({"first_failing_step": None if fail is None else fail[0]}), flush=True)
if fail is None:
    sys.exit(0)
i, uf = fail
ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=uf)
# the first Newton system of that step whose AMG solve fails: walk the step's Newton iterates
x = uf.copy()
for it in range(10):
    J = ctx.jacobian(x)
    b = ctx.residual(x)
    ctx.amg_configure(**R1)
    z, r = ctx.linear_solve(b, prec=P.PREC_AMG, reduction=1e-8, maxit=3000)
    if r["breakdown"] or not r["converged"]:
        break
    x = x - z
print(json.dumps({"newton_iterate": it, "r1_solve": r}), flush=True)
perm = np.array([f * nv + v for v in range(nv) for f in range(3)])
Ai = J[perm][:, perm].tocsr()  # vertex-interleaved


def levels(opts):
    ctx.amg_configure(**opts)
    ctx.prec_apply(b, P.PREC_AMG)  # builds the hierarchy
    info = ctx.amg_info()
    aggs = [ctx.amg_aggregates(l) for l in range(info["levels"] - 1)]
    aggs[0] = aggs[0][np.arange(nv)]  # level 0 by global vertex (one rank: all owned)
    As, cur = [Ai], Ai
    for a in aggs:
        n = cur.shape[0] // 3
        Pv = sp.csr_matrix((np.ones(n), (np.arange(n), a)), shape=(n, int(a.max()) + 1))
        Pm = sp.kron(Pv, sp.identity(3), format="csr")
        cur = (Pm.T @ cur @ Pm).tocsr()
        As.append(cur)
    return info, As


def bj_radius(A, omega):
    nb = A.shape[0] // 3
    C = A.tocoo()
    m = (C.row // 3) == (C.col // 3)
    D = np.zeros((nb, 3, 3))
    np.add.at(D, (C.row[m] // 3, C.row[m] % 3, C.col[m] % 3), C.data[m])
    Di = np.linalg.inv(D)
    Dm = sp.block_diag([sp.csr_matrix(Di[q]) for q in range(nb)], format="csr")
    G = sp.identity(A.shape[0], format="csr") - omega * (Dm @ A)
    if A.shape[0] <= 3000:
        return float(np.max(np.abs(np.linalg.eigvals(G.toarray()))))
    return float(np.max(np.abs(spla.eigs(G, k=3, which="LM", return_eigenvectors=False,
                                         maxiter=3000, tol=1e-6))))


out = {}
for name, opts in (("round1", R1), ("default", NOW)):
    info, As = levels(opts)
    rad = {f"level{l}_{As[l].shape[0] // 3}blocks": bj_radius(As[l], opts["omega"])
           for l in range(1, len(As) - 1)}
    ctx.amg_configure(**opts)
    n = Ai.shape[0]
    AB = spla.LinearOperator((n, n), matvec=lambda v: J @ ctx.prec_apply(v, P.PREC_AMG),
                             dtype=np.float64)
    ev = spla.eigs(AB, k=6, which="SR", return_eigenvectors=False, maxiter=400, tol=1e-4)
    z, r = ctx.linear_solve(b, prec=P.PREC_AMG, reduction=1e-8, maxit=3000)
    out[name] = {"rows": info["rows"], "coarse_block_jacobi_spectral_radius": rad,
                 "AB_smallest_real_eigs": [[float(e.real), float(e.imag)] for e in ev],
                 "bicgstab": {k_: r[k_] for k_ in ("converged", "iterations", "breakdown",
                                                  "reduction")}}
    print(json.dumps({name: out[name]}), flush=True)
