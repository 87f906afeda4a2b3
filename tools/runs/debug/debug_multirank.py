"""Debug helper (GPU): partitioned vs single-rank PB -> PNP on a refined mesh."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import meshio
import oracle_py as O
import pnp_amd as P
from test_gpu_multirank import run_ranks

KEYS = ("converged", "status", "iterations", "linear_iterations", "first_defect", "defect")


def case(cfgname, k, prec, nranks):
    cfg = P.read_config(os.path.join(ROOT, "data", cfgname))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
    par = P.Params.from_config(cfg)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    opb = orc.operator(O.OP_PB, flux=orc.flux(), mask=orc.mask(1))

    def f(ctx, r):
        ctx.set_operator(P.OP_PB)
        phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=prec)
        phi = ctx.sync_vector(phi, 1)
        x0 = ctx.initial_state(phi)
        ctx.set_operator(P.OP_PNP)
        u, res = ctx.newton(x0, prec=prec)
        return phi, x0, ctx.sync_vector(u), res, rpb
    if nranks == 1:
        ctx = P.Context(mesh, par)
        out = [f(ctx, 0)]
    else:
        out = run_ranks(nranks, mesh, par, f)
    phi, x0, u, res, rpb = out[0]
    print(cfgname, k, "prec", prec, "ranks", nranks, flush=True)
    print("  PB ", {q: rpb[q] for q in KEYS}, "oracle |R_pb(phi)|", np.linalg.norm(orc.residual(opb, phi)))
    print("  PNP", {q: res[q] for q in KEYS})
    print("  oracle |R(x0)|", np.linalg.norm(orc.residual(op, x0)), "|R(u)|", np.linalg.norm(orc.residual(op, u)), flush=True)
    return phi, x0, u


for cfgname, k, prec in [("cylinder_config.cfg", 1, P.PREC_SSOR), ("pore_pnp/pore.cfg", 0, P.PREC_ILU0),
                         ("pore_pnp/pore.cfg", 1, P.PREC_ILU0)]:
    a = case(cfgname, k, prec, 1)
    b = case(cfgname, k, prec, 4)
    for nm, x, y in zip(("phi", "x0", "u"), a, b):
        print("  diff", nm, np.max(np.abs(x - y)), flush=True)
