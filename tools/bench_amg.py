"""AMG (PNP_PREC_AMG) vs the single-level preconditioners on SURVEY config 3 (pore_pnp k=4):
PB Newton (CG_AMG_SSOR vs the bench's BiCGSTAB+SSOR) and PNP Newton from the Boltzmann state
(BiCGSTAB + AMG(ILU0 smoother) vs BiCGSTAB + ILU0).  One JSON line per run.

usage: python tools/bench_amg.py [refine=4]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def run(ctx, label, u0, prec, method=0, reduction=1e-9, minlin=1e-8, **amg):
    if prec == P.PREC_AMG:
        ctx.amg_configure(**amg)
    ctx.timers(enable=True, reset=True)
    t0 = time.perf_counter()
    u, r = ctx.newton(u0, reduction=reduction, min_linear_reduction=minlin, prec=prec,
                      method=method, maxit=10)
    dt = time.perf_counter() - t0
    tm = ctx.timers(enable=False)
    out = {"run": label, "seconds": round(dt, 4), "converged": r["converged"],
           "newton_its": r["iterations"], "linear_its": r["linear_iterations"],
           "defect": r["defect"], "solve_s": round(r["solve_seconds"], 4),
           "prec_us_per_apply": round(tm["prec_ms"] / max(1, tm["prec_launches"]) * 1e3, 1),
           "setup_ms_total": round(tm["factor_ms"], 2)}
    if prec == P.PREC_AMG:
        info = ctx.amg_info()
        out["amg_rows"] = info["rows"]
    print(json.dumps(out), flush=True)
    return u


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    print(json.dumps({"mesh": f"pore_pnp k={k}", "nv": mesh.nv}), flush=True)
    ctx.set_operator(P.OP_PB)
    z = np.zeros(mesh.nv)
    run(ctx, "PB warmup", z, P.PREC_SSOR)
    phi = run(ctx, "PB newton BiCGSTAB+SSOR", z, P.PREC_SSOR)
    run(ctx, "PB newton CG+SSOR", z, P.PREC_SSOR, method=P.METHOD_CG)
    run(ctx, "PB newton CG+AMG(SSOR) = CG_AMG_SSOR", z, P.PREC_AMG, method=P.METHOD_CG,
        smoother=P.PREC_SSOR)
    run(ctx, "PB newton BiCGSTAB+AMG(SSOR)", z, P.PREC_AMG, smoother=P.PREC_SSOR)
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    run(ctx, "PNP newton BiCGSTAB+ILU0", x0, P.PREC_ILU0)
    run(ctx, "PNP newton BiCGSTAB+AMG(ILU0)", x0, P.PREC_AMG, smoother=P.PREC_ILU0)
    run(ctx, "PNP newton BiCGSTAB+AMG(ILU0) omega=1", x0, P.PREC_AMG, smoother=P.PREC_ILU0,
        omega=1.0)
    ctx.close()


if __name__ == "__main__":
    main()
