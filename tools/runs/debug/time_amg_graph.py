"""PNP Newton with BiCGSTAB + aggregation AMG (ILU(0) smoother, the bench's configuration) on
config 3, eager launches against hipGraph block replay (PNP_OPT_GRAPH 0 / -1), interleaved twice.
Prints one JSON line per run.  usage: python tools/time_amg_graph.py"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
phi, _ = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_SSOR)
x0 = ctx.initial_state(phi)
ctx.set_operator(P.OP_PNP)
ctx.amg_configure(smoother=P.PREC_ILU0, coarse_sweeps=2, omega=0.8)
for g in (0, -1, 0, -1):
    ctx.set_option(P.OPT_GRAPH, g)
    t = time.perf_counter()
    u, res = ctx.newton(x0, prec=P.PREC_AMG, reduction=1e-9, min_linear_reduction=1e-8)
    dt = time.perf_counter() - t
    print(json.dumps({"graph": g, "seconds": dt, "newton_steps": res["iterations"],
                      "linear_iterations": res["linear_iterations"],
                      "converged": res["converged"], "u_sha1": hashlib.sha1(u.tobytes()).hexdigest()[:16]}), flush=True)
