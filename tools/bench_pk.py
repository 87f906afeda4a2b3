"""P_k (PDEGREE 1, 2, 3) rates on one MI355X: the operator-split driver's scalar operators on the
Lagrange space of degree k (src/instationary_pnp_from_pb_md.hh:26-28, 125, 245-247), on
test/pore_pnp/pore.msh refined r times (default 3: 185K vertices, 367K triangles).
Per degree: DOF nodes, residual + Jacobian assembly time (HIP events) of PoissonOperator and
PBOperator, and the two-pass Jacobian kernels' algorithmic bytes (pk_assemble.hip):
  element pass: reads nl node indices (4 B) + nl node values and nl per frozen field (8 B each) and
                the 3 vertex coordinates (16 B); writes nl records of W = nl + 2 rounded to even
                doubles (the matrix row, the residual entry, padding)
  gather pass : per incidence (ne * nl of them) the code (4 B), the slot bytes (4 B per 4 nodes)
                and the record (8 W B); per row the count, load vector, mask and residual
                (4 + 8 + 1 + 8 B); one value per SELL slot written (8 B)
A PoissonOperator BiCGSTAB solve (ILU(0) for P1/P2, no preconditioner for P3: Q10) is timed too.
Prints one JSON object per degree.  usage: python tools/bench_pk.py [refine] [degrees...]   (PNP_PK_NO_SOLVE=1: assembly only)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

DATA = os.path.join(ROOT, "data")


def timed_assembly(ctx, n=10):
    ctx.assemble_state(2)
    ctx.timers(enable=True, reset=True)
    ctx.assemble_state(n)
    tm = ctx.timers(enable=False)
    ctx.assemble_state(-2)
    ctx.timers(enable=True, reset=True)
    ctx.assemble_state(-n)
    tr = ctx.timers(enable=False)
    return (tm["assemble_ms"] / tm["assemble_launches"] * 1e3,
            tr["assemble_ms"] / tr["assemble_launches"] * 1e3)


def main():
    refine = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    degrees = [int(a) for a in sys.argv[2:]] or [1, 2, 3]
    cfg = P.read_config(os.path.join(DATA, "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(refine)
    par = P.Params.from_config(cfg)
    for k in degrees:
        t0 = time.perf_counter()
        ctx = P.Context(mesh, par, degree=k)
        setup = time.perf_counter() - t0
        info = ctx.info()
        nn = ctx.nn
        nl = (k + 1) * (k + 2) // 2
        rng = np.random.default_rng(1)
        out = {"degree": k, "mesh": f"pore_pnp k={refine}", "vertices": mesh.nv,
               "triangles": mesh.nt, "nodes": nn, "sell_slots": info["nslots"],
               "blocks": info["nblocks"], "colors": info["ncolors"], "setup_s": setup}
        for name, kind in (("poisson", P.OP_POISSON), ("pb", P.OP_PB)):
            if kind == P.OP_POISSON:
                ctx.set_operator(kind, cp=rng.uniform(0, 0.1, nn), cm=rng.uniform(0, 0.1, nn))
            else:
                ctx.set_operator(kind)
            ctx.state_set(rng.uniform(-1, 1, nn))
            us, us_res = timed_assembly(ctx)
            out[name] = {"assemble_us": us, "residual_only_us": us_res,
                         "assembled_dofs_per_s": nn / (us * 1e-6)}
        if k > 1:
            ne = mesh.nt  # one rank: every element is local
            aux = 2  # Poisson: c+ and c- frozen
            W = (nl + 2) & ~1
            elem = ne * (nl * 4 + nl * (1 + aux) * 8 + 3 * 16 + nl * W * 8)
            gather = ne * nl * (4 + 4 * ((nl + 3) // 4) + 8 * W) + nn * 21 + info["nslots"] * 8
            out["poisson"]["bytes_element_pass"] = elem
            out["poisson"]["bytes_gather_pass"] = gather
            out["poisson"]["achieved_gbs"] = (elem + gather) / (out["poisson"]["assemble_us"] * 1e-6) / 1e9
        # a PoissonOperator solve (StationaryLinearProblemSolver, reduction 1e-10)
        if os.environ.get("PNP_PK_NO_SOLVE") == "1":
            print(json.dumps(out), flush=True)
            ctx.close()
            continue
        ctx.set_operator(P.OP_POISSON, cp=rng.uniform(0, 0.1, nn), cm=rng.uniform(0, 0.1, nn))
        x = np.zeros(nn)
        ctx.jacobian(x, export=False)
        r = ctx.residual(x)
        prec = P.PREC_ILU0 if k < 3 else P.PREC_NONE
        t0 = time.perf_counter()
        z, res = ctx.linear_solve(r, prec=prec, reduction=1e-10, maxit=50000)
        ts = time.perf_counter() - t0
        out["poisson_solve"] = {"prec": "ilu0" if k < 3 else "none", "seconds": ts,
                                "iterations": res["iterations"], "converged": res["converged"],
                                "ms_per_iter": ts / max(1, res["iterations"]) * 1e3}
        print(json.dumps(out), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
