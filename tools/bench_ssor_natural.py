"""BiCGSTAB + SeqSSOR in the reference's DOF order (PNP_PREC_SSOR_NATURAL) against the multicolour
SSOR, on one MI355X: the PB operator (scalar, the md driver's first solve) on pore_pnp refined r
times and the PNP operator on config 3.  Per case: fixed BiCGSTAB iterations timed with the
device timers (prec_ms / prec_launches = one preconditioner application), ms per iteration.
Prints one JSON line per case.  usage: python tools/bench_ssor_natural.py [refine ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def case(ctx, x, name, nit=20):
    ctx.state_set(x)
    ctx.assemble_state(1)
    out = {"case": name}
    for prec_name, prec in (("ssor_natural", P.PREC_SSOR_NATURAL), ("ssor", P.PREC_SSOR)):
        ctx.bicgstab_iterations(2, prec)  # warm-up: level schedule, split storage
        t0 = time.perf_counter()
        ctx.bicgstab_iterations(nit, prec)
        wall = (time.perf_counter() - t0) / nit
        ctx.timers(enable=True, reset=True)
        ctx.bicgstab_iterations(nit, prec)
        tm = ctx.timers(enable=False)
        out[prec_name] = {"ms_per_iter_wall": wall * 1e3,
                          "prec_ms_per_apply": tm["prec_ms"] / max(1, tm["prec_launches"]),
                          "spmv_ms": tm["spmv_ms"] / max(1, tm["spmv_launches"])}
    return out


def main():
    refines = [int(a) for a in sys.argv[1:]] or [3, 4]
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    par = P.Params.from_config(cfg)
    rng = np.random.default_rng(7)
    for r in refines:
        mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(r)
        nv = mesh.nv
        ctx = P.Context(mesh, par)
        ctx.set_operator(P.OP_PB)
        o = case(ctx, rng.uniform(-1, 1, nv), f"PB pore_pnp k={r} ({nv} DOF)")
        print(json.dumps(o), flush=True)
        ctx.set_operator(P.OP_PNP)
        x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                            0.06 * rng.uniform(0.5, 1.5, nv)])
        o = case(ctx, x, f"PNP pore_pnp k={r} ({3 * nv} DOF)")
        print(json.dumps(o), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
