"""Config 4 (implicit Euler, dt = tau, pore_pnp k) with BiCGSTAB + AMG(ILU0), the default AMG
options: per step Newton iterations, BiCGSTAB iterations and linear_fallbacks (solves where the
AMG-preconditioned BiCGSTAB failed and the smoother alone was used).  With --dump, the first
failing step's Newton system (Jacobian, right-hand side, level-0 aggregates) is written to
gpurun_out/amg_fail_k<k>.npz.  AMG options from the environment: AMG_COARSE (coarse_target),
AMG_OMEGA, AMG_PRE (level0_presmooth), AMG_SWEEPS (coarse_sweeps).
usage: python tools/amg_config4_scan.py k nsteps [--dump]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
nsteps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
dump = "--dump" in sys.argv
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
phi, _ = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=P.PREC_SSOR)
u = ctx.initial_state(phi)
dt = cfg.system["tau"]
tot = {"newton": 0, "linear": 0, "fallbacks": 0}
for i in range(nsteps):
    ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=u)
    ctx.amg_configure(smoother=P.PREC_ILU0,
                      coarse_target=int(os.environ.get("AMG_COARSE", "1024")),
                      omega=float(os.environ.get("AMG_OMEGA", "0.8")),
                      level0_presmooth=int(os.environ.get("AMG_PRE", "-1")),
                      coarse_sweeps=int(os.environ.get("AMG_SWEEPS", "2")))
    u_prev = u.copy()
    u, res = ctx.newton(u, reduction=1e-8, abs_limit=1e-9, prec=P.PREC_AMG)
    tot["newton"] += res["iterations"]
    tot["linear"] += res["linear_iterations"]
    tot["fallbacks"] += res["linear_fallbacks"]
    print(json.dumps({"step": i, **{k_: res[k_] for k_ in ("converged", "iterations",
                                                         "linear_iterations", "linear_fallbacks",
                                                         "first_defect", "defect")}}), flush=True)
    if res["linear_fallbacks"] and dump:
        # replay the step's first Newton system and save it
        ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=u_prev)
        J = ctx.jacobian(u_prev)
        b = ctx.residual(u_prev)
        z, r = ctx.linear_solve(b, prec=P.PREC_AMG, reduction=1e-8, maxit=3000)
        agg = ctx.amg_aggregates(0)
        print(json.dumps({"replay_first_system": r}), flush=True)
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"amg_fail_k{k}.npz"),
                            indptr=J.indptr, indices=J.indices, data=J.data, b=b, u=u_prev,
                            agg0=agg, step=i)
        break
    if not res["converged"]:
        break
print(json.dumps({"total": tot}), flush=True)
