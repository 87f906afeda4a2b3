"""hipGraph replay of the BiCGSTAB blocks at config 3 (PNP_OPT_GRAPH 1) against eager launches
(0, the default above 131,072 rows), interleaved: wall time per iteration of 400 BiCGSTAB + ILU(0)
iterations (no convergence stop) on the Jacobian at a random admissible state.  The kernel trace
shows 7-11 % of an iteration's event time between kernels; replay removes the host's part of it.
usage: python tools/ab_graph.py [reps=3]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PNP)
    rng = np.random.default_rng(20261018)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ctx.state_set(x)
    ctx.assemble_state(1)
    n = 400
    out = {"graph": [], "eager": []}
    for r in range(reps):
        for g in (1, 0):
            ctx.set_option(P.OPT_GRAPH, g)
            ctx.bicgstab_iterations(16, P.PREC_ILU0)  # capture / warm
            t0 = time.perf_counter()
            ctx.bicgstab_iterations(n, P.PREC_ILU0)
            out["graph" if g else "eager"].append(1e3 * (time.perf_counter() - t0) / n)
    out["graph_ms_per_iter"] = float(np.median(out["graph"]))
    out["eager_ms_per_iter"] = float(np.median(out["eager"]))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
