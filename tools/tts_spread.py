"""How chaotic the bench's PNP time to solution is: the 24 V pore system's BiCGSTAB + ILU(0)
trajectory depends on the last bits of its inputs.  Config 3, the bench's setup (PB Newton ->
Boltzmann state, pore.cfg's Newton tolerances, bench.py make_context / time to solution); the PNP
Newton runs from x0 and from x0 with a one-ulp relative perturbation per entry (seeded signs),
printing the linear iteration counts and seconds of each.  A spread across the perturbed runs as
wide as a change between two builds says that change moved the count by chance, not by design.
usage: python tools/tts_spread.py [n_perturbed=6]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def main():
    nrun = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PB)
    phi, _ = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=P.PREC_SSOR, linear_maxit=20000)
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    s = cfg.system
    kw = dict(reduction=s["newtonReduction"], min_linear_reduction=s["newtonMinLinearReduction"],
              prec=P.PREC_ILU0, linear_maxit=int(s["linearSolverIterations"]), maxit=10)
    counts = []
    for k in range(-1, nrun):
        if k < 0:
            x = x0
        else:
            sgn = np.random.default_rng(k).choice([-1.0, 1.0], x0.size)
            x = x0 * (1.0 + sgn * 2.0 ** -52)
        t0 = time.perf_counter()
        _, r = ctx.newton(x, **kw)
        dt = time.perf_counter() - t0
        counts.append(r["linear_iterations"])
        print(json.dumps({"perturbation": "none" if k < 0 else f"1 ulp, seed {k}",
                          "changed_entries": int(np.count_nonzero(x != x0)),
                          "converged": r["converged"], "newton_steps": r["iterations"],
                          "linear_iterations": r["linear_iterations"], "seconds": dt}), flush=True)
    c = np.array(counts)
    print(json.dumps({"linear_iterations_min": int(c.min()), "max": int(c.max()),
                      "median": float(np.median(c)), "spread_over_median": float(
                          (c.max() - c.min()) / np.median(c))}), flush=True)


if __name__ == "__main__":
    main()
