"""PNP_OPT_ILU_F32 = 3 (single-precision forward intermediate) against 2 on the system where it
stalled BiCGSTAB (tests/test_gpu_scaling_iters.py: pore_without_dna scale 0.85 refined k=4, PNP
Jacobian at the Boltzmann state after the PB Newton): the relative difference of one ILU(0)
application per field, for a random vector and for the residual, and the BiCGSTAB count of one
linear solve at the Newton's first-step reduction with each mode.  DESIGN.md §0.13.
usage: python tools/ilu_y32_err.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def main():
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_without_dna", "pore.cfg"))
    mesh = P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(4)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PB)
    phi, _ = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0, reduction=1e-10)
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    ctx.jacobian(x0, export=False)
    r = ctx.residual(x0)
    nv = mesh.nv
    d = np.random.default_rng(3).standard_normal(3 * nv)
    out = {"dofs": 3 * nv}
    v = {}
    for m in (2, 3):
        ctx.set_option(P.OPT_ILU_F32, m)
        v[m] = (ctx.prec_apply(d, P.PREC_ILU0), ctx.prec_apply(r, P.PREC_ILU0))
        sols = {}
        for red in (1e-5, 1e-8):
            sol, res = ctx.linear_solve(r, prec=P.PREC_ILU0, reduction=red, maxit=5000)
            sols[str(red)] = {"converged": res["converged"], "iterations": res["iterations"]}
        out[f"solve_mode{m}"] = sols
    for k, name in ((0, "random"), (1, "residual")):
        a, b = v[2][k], v[3][k]
        per = []
        for f in range(3):
            af, bf = a[f * nv:(f + 1) * nv], b[f * nv:(f + 1) * nv]
            per.append({"max_rel": float(np.max(np.abs(bf - af)) / max(np.max(np.abs(af)), 1e-300)),
                        "l2_rel": float(np.linalg.norm(bf - af) / max(np.linalg.norm(af), 1e-300)),
                        "max_abs_v": float(np.max(np.abs(af)))})
        out[f"apply_{name}"] = per
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
