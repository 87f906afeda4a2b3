"""Time to solution with the reference's default linear solver, BCGS_SSORk (BiCGSTAB + SeqSSOR in
the reference's DOF order, PNP_PREC_SSOR_NATURAL), at config 3 on one MI355X: the PB Newton from
zero (the md driver's first solve) and the PNP Newton from the Boltzmann state, the config's
reductions, beside the same Newtons with ILU(0).  Prints one JSON line per solve.
usage: python tools/newton_ssork.py [refine]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402
import bench  # noqa: E402


def main():
    refine = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(refine)
    ctx, x0, _, _ = bench.make_context(mesh, cfg, 0, 1, 0, None)
    red, linred = cfg.system["newtonReduction"], cfg.system["newtonMinLinearReduction"]
    maxit = int(cfg.system["linearSolverIterations"])
    for name, prec in (("ssork_natural", P.PREC_SSOR_NATURAL), ("ilu0", P.PREC_ILU0)):
        ctx.set_operator(P.OP_PB)
        t0 = time.perf_counter()
        _, r = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=prec, linear_maxit=20000)
        pb = {"solve": "PB Newton from zero", "prec": name, "seconds": time.perf_counter() - t0,
              "converged": r["converged"], "iterations": r["iterations"],
              "linear_iterations": r["linear_iterations"], "defect": r["defect"]}
        print(json.dumps(pb), flush=True)
        ctx.set_operator(P.OP_PNP)
        t0 = time.perf_counter()
        _, r = ctx.newton(x0, reduction=red, min_linear_reduction=linred, prec=prec,
                          linear_maxit=maxit, maxit=10)
        pnp = {"solve": "PNP Newton from the Boltzmann state", "prec": name,
               "seconds": time.perf_counter() - t0, "converged": r["converged"],
               "iterations": r["iterations"], "linear_iterations": r["linear_iterations"],
               "defect": r["defect"], "dofs": 3 * mesh.nv}
        print(json.dumps(pnp), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
