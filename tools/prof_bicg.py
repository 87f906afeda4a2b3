"""Profiling target for the per-kernel BiCGSTAB split: the bench's own
systems and event-timed pass, once per config, each phase bracketed by a small k_scrub launch as a
marker so that tools/bicg_split.py can attribute every traced kernel to its config.

Per phase (config 3: pore_pnp k=4, 2.2 M DOF; config 5: pore_without_dna k=6, 8.87 M DOF), as
bench.py measure() runs it: Boltzmann initial state, one assembly, two untimed BiCGSTAB iterations
(ILU(0), f32 factors), then `nit` iterations with the library's event timers on (eager launches,
as under the profiler) between two markers.  Prints one JSON line per phase with the event
timers and the stored-format byte models, which bicg_split.py joins with the trace.
usage: python tools/prof_bicg.py [nit] [configs, e.g. 3,5] [prec]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench as B  # noqa: E402

P = B.P
MARK = 64 << 20  # marker scrub: 64 MiB read, k_scrub's fixed 4096-workgroup grid


def main():
    nit = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    configs = [int(c) for c in (sys.argv[2] if len(sys.argv) > 2 else "3,5").split(",")]
    prec = P.PREC_BY_NAME[sys.argv[3] if len(sys.argv) > 3 else "ilu0"]
    for c in configs:
        if c == 3:
            cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
            mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
        else:
            cfg, mesh = B.strong_mesh(6)
        ctx, x0, _, _ = B.make_context(mesh, cfg, 0, 1, 0, None)
        info = ctx.info()
        ctx.assemble_state(1)
        ctx.bicgstab_iterations(2, prec)
        ctx.cache_scrub(MARK)
        ctx.timers(enable=True, reset=True)
        ctx.bicgstab_iterations(nit, prec)
        tm = ctx.timers(enable=False)
        ctx.cache_scrub(MARK)
        N = 3 * info["nv_owned"]
        T = mesh.nt
        bm = B.byte_models(info, 3, N, T, prec)
        print(json.dumps({"config": c, "dofs": N, "iterations": nit, "timers": tm,
                          "bytes": {k: bm[k] for k in ("spmv_stored", "ilu_stored", "blas")},
                          "blas_source": bm["blas_source"]}), flush=True)
        ctx.close()


if __name__ == "__main__":
    main()
