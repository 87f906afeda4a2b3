"""One rank of the two-process host-transport test (tests/test_gpu_dist_host.py): NOT a test
module.  Started as its own OS process (before it touches the GPU), it joins a gloo process group,
creates its rank's context with the host-staged transport (pnp_comm.host: halo and reductions
through gloo, staged in pinned host memory) and runs the reference driver's sequence on the
pore_pnp mesh: PB Newton -> BCExtension initial state -> PNP Newton with BiCGSTAB + ILU(0)
(src/stationary_pnp_from_pb.hh:105-369; the reference's multi-rank run, src/pnp_solver_main.cc:
93-108).  Rank 0 then runs the same on a one-rank context and writes both results to a JSON file.
usage: python tests/dist_host_worker.py <rank> <world> <port> <out.json> [refine]"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402


def driver(ctx, mesh, cfg):
    s = cfg.system
    ctx.set_operator(P.OP_PB)
    phi, pb = ctx.newton(np.zeros(mesh.nv), reduction=1e-10, prec=P.PREC_ILU0)
    phi = ctx.sync_vector(phi, 1)
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    r0 = ctx.sync_vector(ctx.residual(x0))
    # converged to the rounding floor (the two preconditioners -- block Jacobi ILU(0) across the
    # ranks, ILU(0) on one -- take different paths there, so only tight solutions agree tightly)
    u, res = ctx.newton(x0, reduction=1e-13, abs_limit=1e-15, min_linear_reduction=1e-10,
                        prec=P.PREC_ILU0, linear_maxit=int(s["linearSolverIterations"]))
    u = ctx.sync_vector(u)
    return {"phi": phi, "r0": r0, "u": u, "pb": pb, "pnp": res,
            "flux": np.asarray(ctx.ion_flux(u), dtype=float)}


def main():
    rank, world, port, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    refine = int(sys.argv[5]) if len(sys.argv) > 5 else 2
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(refine)
    par = P.Params.from_config(cfg)
    tr = P.TorchDistTransport(dist)
    t0 = time.perf_counter()
    ctx = P.Context(mesh, par, device=0, rank=rank, size=world, host_transport=tr)
    info = ctx.info()
    d = driver(ctx, mesh, cfg)
    t_dist = time.perf_counter() - t0
    ctx.close()
    dist.barrier()
    if rank == 0:
        c1 = P.Context(mesh, par, device=0)
        d1 = driver(c1, mesh, cfg)
        c1.close()
        rel = lambda a, b: float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))  # noqa
        rep = {"ranks": world, "dofs": 3 * mesh.nv, "transport": info["transport"],
               "nv_owned_rank0": info["nv_owned"], "nv_ghost_rank0": info["nv_ghost"],
               "host_calls_rank0": tr.calls, "seconds_distributed": t_dist,
               "pb_newton": [d["pb"]["iterations"], d1["pb"]["iterations"]],
               "pnp_newton": [d["pnp"]["iterations"], d1["pnp"]["iterations"]],
               "pnp_converged": [d["pnp"]["converged"], d1["pnp"]["converged"]],
               "bicgstab_iterations": [d["pnp"]["linear_iterations"], d1["pnp"]["linear_iterations"]],
               "phi_pb_rel_err": rel(d["phi"], d1["phi"]),
               "residual_x0_rel_err": rel(d["r0"], d1["r0"]),
               "solution_rel_err": rel(d["u"], d1["u"]),
               "ion_flux_rel_err": rel(d["flux"], d1["flux"])}
        with open(out, "w") as f:
            json.dump(rep, f)
        print(json.dumps(rep), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
