"""PNP Newton (config 3) with BiCGSTAB + AMG under several AMG options, one process.
usage: python tools/ab_amg_opts.py [refine=4]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
phi, _ = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=P.PREC_SSOR)
x0 = ctx.initial_state(phi)
ctx.set_operator(P.OP_PNP)
variants = [dict(omega=1.0, coarse_sweeps=2), dict(omega=0.8, coarse_sweeps=2),
            dict(omega=0.8, coarse_sweeps=1), dict(omega=1.0, coarse_sweeps=1),
            dict(omega=0.8, coarse_sweeps=3), dict(omega=0.67, coarse_sweeps=2),
            dict(omega=1.0, coarse_sweeps=2, coarse_target=16),
            dict(omega=1.0, coarse_sweeps=2, smoother=P.PREC_SSOR)]
for rep in range(2):
    for v in variants:
        kw = dict(smoother=P.PREC_ILU0)
        kw.update(v)
        ctx.amg_configure(**kw)
        ctx.timers(enable=True, reset=True)
        t0 = time.perf_counter()
        u, r = ctx.newton(x0, reduction=1e-9, min_linear_reduction=1e-8, prec=P.PREC_AMG, maxit=10)
        dt = time.perf_counter() - t0
        tm = ctx.timers(enable=False)
        print(json.dumps({"opts": {k_: (v_ if not isinstance(v_, float) else round(v_, 2)) for k_, v_ in kw.items()},
                          "seconds": round(dt, 3), "linear_its": r["linear_iterations"],
                          "fallbacks": r["linear_fallbacks"], "converged": r["converged"],
                          "prec_us": round(tm["prec_ms"] / max(1, tm["prec_launches"]) * 1e3, 1)}),
              flush=True)
ctx.close()
