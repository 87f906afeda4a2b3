"""Debug helper (GPU): BiCGStab traces on the first PNP Newton system of cylinder k=1, fresh
context vs after a PB Newton in the same context (PNP_DEBUG_BICGSTAB=1 prints the scalars)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P
cfg = P.read_config(os.path.join(ROOT, "data", "cylinder_config.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(1)
x0 = np.load(os.path.join(ROOT, "tests", "_dbg_cyl1_x0.npy"))


def probe(ctx, tag):
    ctx.set_operator(P.OP_PNP)
    ctx.jacobian(x0, export=False)
    r = ctx.residual(x0)
    print("=== " + tag, flush=True); sys.stderr.flush()
    z, info = ctx.linear_solve(r, prec=P.PREC_SSOR, reduction=1e-8, maxit=12, check_every=1)
    sys.stderr.flush()
    print(tag, "solve", info, flush=True)


probe(P.Context(mesh, P.Params.from_config(cfg)), "fresh")
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
print("=== PB", flush=True)
phi, _ = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_SSOR)
probe(ctx, "afterPB")
probe(P.Context(mesh, P.Params.from_config(cfg)), "fresh2")
