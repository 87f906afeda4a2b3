"""BiCGSTAB + ILU(0) timing of the library build in use (PNP_AMD_LIB selects an A/B build, see
tools/build_ab.sh), for interleaved A/Bs: per config (3: pore_pnp k=4, 2.2 M DOF; 5: pore_without_dna
.geo scale 0.85 k=6, 8.87 M DOF) on the Jacobian at a seeded random admissible state, the ILU(0)
application's event time per apply and the BiCGSTAB wall time per iteration (nit iterations, no
convergence stop, after 5 untimed).  One JSON line per config.
usage: python tools/time_bicg.py [configs=3] [nit=200]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def system(c):
    if c == 3:
        cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
        return cfg, P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_without_dna", "pore.cfg"))
    return cfg, P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(6)


def main():
    configs = [int(c) for c in (sys.argv[1] if len(sys.argv) > 1 else "3").split(",")]
    nit = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    for c in configs:
        cfg, mesh = system(c)
        ctx = P.Context(mesh, P.Params.from_config(cfg))
        ctx.set_operator(P.OP_PNP)
        rng = np.random.default_rng(20261018)
        nv = mesh.nv
        x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                            0.06 * rng.uniform(0.5, 1.5, nv)])
        ctx.state_set(x)
        ctx.assemble_state(1)
        ctx.bicgstab_iterations(5, P.PREC_ILU0)
        t0 = time.perf_counter()
        ctx.bicgstab_iterations(nit, P.PREC_ILU0)
        wall = (time.perf_counter() - t0) / nit
        ctx.timers(enable=True, reset=True)
        ctx.bicgstab_iterations(40, P.PREC_ILU0)
        tm = ctx.timers(enable=False)
        ctx.close()
        print(json.dumps({"config": c, "lib": os.environ.get("PNP_AMD_LIB", "in-tree"),
                          "bicgstab_ms_per_iter": wall * 1e3,
                          "ilu_us_per_apply": 1e3 * tm["prec_ms"] / max(1, tm["prec_launches"]),
                          "spmv_us": 1e3 * tm["spmv_ms"] / max(1, tm["spmv_launches"]),
                          "blas_us_per_iter": 1e3 * tm["blas_ms"] / 40}), flush=True)


if __name__ == "__main__":
    main()
