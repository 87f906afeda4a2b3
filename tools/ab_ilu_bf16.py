"""PNP_OPT_ILU_F32 modes against each other at config 3, interleaved (default: bfloat16 factors, 2,
against single precision, 1; 3 = bfloat16 factors with the single-precision forward intermediate):
the ILU(0) application's event time per apply and the BiCGSTAB wall time per iteration, 200
iterations (no convergence stop) on the Jacobian at a random admissible state.
usage: python tools/ab_ilu_bf16.py [reps=3] [modes=1,2]"""
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
    modes = [int(m) for m in (sys.argv[2] if len(sys.argv) > 2 else "1,2").split(",")]
    names = {0: "f64", 1: "f32", 2: "bf16", 3: "bf16_y32"}
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
    n = 200
    out = {m: {"apply_us": [], "iter_ms": []} for m in modes}
    for _ in range(reps):
        for f in modes:
            ctx.set_option(P.OPT_ILU_F32, f)
            ctx.bicgstab_iterations(8, P.PREC_ILU0)  # factorisation in this precision, warm
            ctx.timers(enable=True, reset=True)
            ctx.bicgstab_iterations(n, P.PREC_ILU0)
            tm = ctx.timers(enable=False)
            out[f]["apply_us"].append(1e3 * tm["prec_ms"] / tm["prec_launches"])
            t0 = time.perf_counter()
            ctx.bicgstab_iterations(n, P.PREC_ILU0)
            out[f]["iter_ms"].append(1e3 * (time.perf_counter() - t0) / n)
    res = {names[f]: {"apply_us_median": float(np.median(v["apply_us"])),
                                           "iter_ms_median": float(np.median(v["iter_ms"])),
                                           **v} for f, v in out.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
