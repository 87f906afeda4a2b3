"""ILU(0) application: one dataflow launch (PNP_OPT_ILU_FLOW=1) against the colour launches (0), on
one MI355X, interleaved.  Config 3 (pore_pnp k=4, 2.2 M DOF) and config 5 (pore_without_dna .geo,
scale 0.85, k=6, 8.87 M DOF) at a random PNP state; per setting: BiCGSTAB ILU(0) iterations timed
by the wall clock and by the library's device timers (prec_ms / prec_launches = one application).
Prints one JSON line per (case, setting, round).  usage: python tools/bench_ilu_flow.py [3] [5]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def make(case):
    if case == "3":
        cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
        mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    else:
        cfg = P.read_config(os.path.join(ROOT, "data", "pore_without_dna", "pore.cfg"))
        mesh = P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(6)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    rng = np.random.default_rng(20261015)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ctx.set_operator(P.OP_PNP)
    ctx.state_set(x)
    ctx.assemble_state(1)
    return ctx, 3 * nv


def main():
    cases = sys.argv[1:] or ["3", "5"]
    nit = 20
    for case in cases:
        ctx, n = make(case)
        for flow in (0, 1):  # warm-up: factors, split storage, the flow's dependency lists
            ctx.set_option(P.OPT_ILU_FLOW, flow)
            ctx.bicgstab_iterations(4, P.PREC_ILU0)
        for rnd in range(3):
            for flow in (0, 1):
                ctx.set_option(P.OPT_ILU_FLOW, flow)
                ctx.bicgstab_iterations(2, P.PREC_ILU0)
                t0 = time.perf_counter()
                ctx.bicgstab_iterations(nit, P.PREC_ILU0)
                wall = (time.perf_counter() - t0) / nit
                ctx.timers(enable=True, reset=True)
                ctx.bicgstab_iterations(nit, P.PREC_ILU0)
                tm = ctx.timers(enable=False)
                print(json.dumps({"case": f"config {case} ({n} DOF)", "flow": flow, "round": rnd,
                                  "us_per_iter_wall": wall * 1e6,
                                  "us_per_apply": 1e3 * tm["prec_ms"] / max(1, tm["prec_launches"]),
                                  "apply_launches_timed": tm["prec_launches"]}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
