#!/usr/bin/env python
"""Benchmark: assembled DOFs/s + BiCGSTAB iterations/s, 3-species PNP on pore.msh refined.

Workload (BASELINE.json configs[2]): test/pore_pnp/pore.msh refined
k=4 (V = 738,033, N = 2,214,099 DOFs), test/pore_pnp/pore.cfg (cylindrical), PnpOperator.
State: the Boltzmann initial state of the reference's driver (PB Newton on the GPU, then the
BCExtension interpolation, src/stationary_pnp_from_pb.hh:105-282); the Jacobian at that state
and R(x0) are the linear system (SURVEY.md §8(d) "Synthetic inputs").

One step = one full residual + Jacobian assembly of the device-resident state (the headline
`value`, assembled DOFs/s), timed over K steps bracketed by barrier + device sync.  A second
timed region runs K x --bicg-iters BiCGSTAB iterations (ILU0 = multicolour ILU(0) by default) on
the assembled system and reports BiCGSTAB iterations/s.  Roofline numbers come from HIP events
recorded on the library's own stream around every assembly launch; `roofline.traffic` is the
HBM-side byte count per launch of the same kernel from rocprofv3 PMC passes (FETCH_SIZE x2 +
WRITE_SIZE, tools/pmc_summary.py), read from the committed profiles/<round>/pmc_summary.json.

Beside the warm (back-to-back) assembly the line carries a cache-cold one: 1 GiB of scratch is
read between launches, so the matrix is not re-dirtied inside the 256 MiB Infinity Cache
(`roofline_cold`).  The BiCGSTAB line carries two byte models: the contract's CSR bytes
 and the bytes the stored formats move (k-form SELL values + one column index
per slot, split L/U factors), per kernel class, so every `frac` is <= 1 on its own model.

Multi-GPU (torch.distributed.run, one rank per GPU):
  * the primary line (`--scaling weak`, the default): the mesh is N mirrored copies of the pore
    glued at their outflow/inflow planes, partitioned by RCB (one copy per GPU), with RCCL halo
    exchange per SpMV and allreduce per BiCGSTAB reduction;
  * the `strong_scaling` object (config 5, BASELINE.json configs[4], the north star's ~10M-DOF
    system): test/pore_without_dna/pore_without_dna.geo meshed natively (scale 0.85), refined
    k=6 (8.87 M DOF), ONE mesh RCB-split over the N ranks (src/pnp_solver_main.cc:106-108
    loadBalance), run at every N (N=1 included: its single-GPU, past-the-Infinity-Cache rates).
    `--scaling strong` makes it the primary line.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md); the measured stream ceilings
#                       are in the line (`measured_stream_gbs`, tools/micro/stream.hip)
PMC_SUMMARY = os.path.join(ROOT, "profiles", "r06", "pmc_summary.json")
SCRUB_BYTES = 1 << 30  # > 4x the 256 MiB Infinity Cache


def pmc_summary():
    """The newest committed rocprofv3 PMC summary (tools/pmc_summary.py), or None."""
    for path in (PMC_SUMMARY, PMC_SUMMARY.replace("r06", "r05")):
        try:
            with open(path) as f:
                d = json.load(f)
            d["path"] = os.path.relpath(path, ROOT)
            return d
        except (OSError, ValueError):
            continue
    return None


def pmc_traffic(kernel_prefix):
    """Per-launch HBM-side bytes of a kernel from the committed rocprofv3 PMC summary, or None."""
    d = pmc_summary()
    if not d:
        return None
    for name, v in d["kernels"].items():
        if kernel_prefix in name:
            return v["traffic_bytes"]
    return None


ASM_REGIMES = os.path.join(ROOT, "profiles", "r06", "asm_regimes_config3.json")
BICG_SPLIT = os.path.join(ROOT, "profiles", "r06", "bicg_split.json")


def profile_bicg(config):
    """The committed per-config BiCGSTAB kernel split (tools/prof_bicg.py under rocprofv3
    --kernel-trace, split by tools/bicg_split.py): per kernel class the trace's device time per unit,
    the event timers' time of the same pass and the fraction of 8 TB/s on the stored-format bytes;
    None when absent."""
    for path in (BICG_SPLIT,):
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        for ph in d["phases"]:
            if ph["config"] == config:
                return dict(ph["classes"], source=os.path.relpath(path, ROOT))
    return None


ILU_MODEL = os.path.join(ROOT, "profiles", "r06", "ilu_launch_model.json")


def ilu_launch_model():
    """The committed per-launch model of the ILU(0) application (tools/ilu_launch_model.py: each
    colour launch's PMC bytes against its trace time, fitted as fixed + bytes / marginal rate,
    beside the measured floor of a launch of the same shape), or None."""
    try:
        with open(ILU_MODEL) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return {"fixed_us_per_launch": d["fixed_us_per_launch"], "marginal_gbs": d["marginal_gbs"],
            "launches_per_apply": len(d["launches"]),
            "launch_floor_us_800wg": d["launch_floor_us_800wg"],
            "note": "time = fixed + bytes / marginal over the colour launches (PMC bytes against "
                    "trace times); launch_floor: an 800-workgroup kernel of the same shape, empty "
                    "/ with its own load and store / plus one dependent gather",
            "source": os.path.relpath(ILU_MODEL, ROOT)}


def profile_regime(name):
    """The committed rocprofv3 trace's average for one assembly regime (tools/asm_regimes.py:
    warm / in_situ / cold launches of the config-3 assembly), or None."""
    try:
        with open(ASM_REGIMES) as f:
            d = json.load(f)
        r = d["regimes"][name]
        return {"avg_launch_us": r["avg_us"], "frac": r["frac"], "launches": r["launches"],
                "source": os.path.relpath(ASM_REGIMES, ROOT)}
    except (OSError, ValueError, KeyError):
        return None


BLAS_KERNELS = ("k_update_fwd0", "k_update_xr", "k_update_p", "k_reduce")


PMC_DOFS = 2214099  # the committed PMC summaries profile config 3 (tools/prof_target.py 4)


def pmc_blas_bytes(dofs=PMC_DOFS):
    """HBM-side bytes per BiCGSTAB iteration of the vector-update and reduction kernels (the
    device timers' `blas` class), from the committed PMC summary: per kernel its mean bytes per
    launch x its launches per iteration (the summary records the iterations its run made), FETCH_SIZE
    x 2 as calibrated in profiles/r04/calib (every access width the hot path uses), scaled from the
    profiled system's DOFs to `dofs` (the update kernels stream whole vectors: bytes per DOF are
    size-independent).  None when no summary records its iteration count."""
    d = pmc_summary()
    if not d or not d.get("bicgstab_iterations"):
        return None
    it = d["bicgstab_iterations"]
    scale = dofs / float(d.get("dofs", PMC_DOFS))
    tot, parts = 0.0, {}
    for name, v in d["kernels"].items():
        if any(k in name for k in BLAS_KERNELS):
            b = v["traffic_bytes"] * v["launches_fetch"] / it * scale
            parts[name.split("(")[0].replace("void pnp::(anonymous namespace)::", "")] = b
            tot += b
    return {"bytes": tot, "per_kernel": parts, "source": d["path"],
            "scaled_from_dofs": float(d.get("dofs", PMC_DOFS))}


def tile_mesh(mesh, n):
    """n mirrored copies along x, glued at the x-max plane of each copy (weak scaling)."""
    if n == 1:
        return mesh
    xy, tri, bseg, bg = [mesh.xy], [mesh.tri], [], []
    x0, x1 = mesh.xy[:, 0].min(), mesh.xy[:, 0].max()
    L = x1 - x0
    nv = mesh.nv
    cur_xy = mesh.xy
    offset = 0
    glue_prev = None  # map: vertex index in copy k-1 on its x-max plane -> global id
    all_b = [(mesh.bseg, mesh.bgroup, 0)]
    gmap_prev = np.arange(nv)
    total = nv
    xy_out = [mesh.xy]
    tri_out = [mesh.tri]
    seg_out = []
    for k in range(1, n):
        right = x0 + k * L  # plane shared with the previous copy
        new_xy = cur_xy.copy()
        new_xy[:, 0] = 2 * right - cur_xy[:, 0]
        on_plane = np.isclose(cur_xy[:, 0], right, rtol=0, atol=1e-12 * max(1.0, abs(right)))
        gmap = np.empty(nv, dtype=np.int64)
        gmap[on_plane] = gmap_prev[on_plane]
        fresh = ~on_plane
        gmap[fresh] = total + np.arange(fresh.sum())
        total += int(fresh.sum())
        xy_out.append(new_xy[fresh])
        tri_out.append(gmap[mesh.tri])
        all_b.append((mesh.bseg, mesh.bgroup, k, gmap))
        cur_xy, gmap_prev = new_xy, gmap
    # boundary segments: drop those on glued planes
    xy_all = np.concatenate(xy_out)
    bs, bgs = [], []
    gmaps = [np.arange(nv)] + [a[3] for a in all_b[1:]]
    for k in range(n):
        g = gmaps[k]
        s = g[mesh.bseg]
        xs = xy_all[s][:, :, 0]
        glued = np.zeros(len(s), dtype=bool)
        for p in range(1, n):
            plane = x0 + p * L
            glued |= np.all(np.isclose(xs, plane, rtol=0, atol=1e-9), axis=1)
        bs.append(s[~glued])
        bgs.append(mesh.bgroup[~glued])
    return P.Mesh(xy_all, np.concatenate(tri_out), np.concatenate(bs), np.concatenate(bgs))


_T0 = time.perf_counter()


def progress(rank, msg):
    """One line per leg on rank 0's stderr (the JSON line stays alone on stdout), so a long run
    shows where it is."""
    if rank == 0:
        print(f"[bench {time.perf_counter() - _T0:7.1f} s] {msg}", file=sys.stderr, flush=True)


def guarded(rank, name, fn):
    """A secondary leg (time to solution, SSORk, per-config, config 5): an error it raises on
    every rank costs the line that leg only, recorded as {"error": ...}; the primary metric has
    been measured before any of them runs."""
    try:
        return fn()
    except (P.PnpError, RuntimeError, ValueError, KeyError, OSError) as exc:
        progress(rank, f"{name} failed: {type(exc).__name__}: {exc}")
        return {"error": f"{type(exc).__name__}: {exc}"}


def barrier_sync(dist, world):
    import torch
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()


def max_over_ranks(dist, world, v):
    """The job's time: the slowest rank's (gloo all-reduce MAX on the host)."""
    if world == 1:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(cfg, refine, seconds):
    """The oracle (C restatement of the reference algorithm: FD Jacobian with PDELab eps,
    BCRS-style CSR scatter, ISTL BiCGSTAB) single-threaded on the host, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import meshio
    import oracle_py as O
    pmesh = P.Mesh.read_gmsh(cfg.meshfile).refine(refine)
    mesh = meshio.Mesh(pmesh.xy, pmesh.tri, pmesh.bseg, pmesh.bgroup)
    s = cfg.system
    surfs = [meshio.Surface(q.cb, q.cflux, q.cpot, q.pb, q.pflux, q.pconc, q.mb, q.mflux, q.mconc)
             for q in cfg.surfaces]
    orc = O.Problem(mesh, surfs, l_b=s["l_b"], c0=s["c0"], tau=s["tau"],
                    cylindrical=s["cylindrical"])
    rng = np.random.default_rng(20261015)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    t_asm, J = orc.time_fd_assembly(op, x, 0.5 * seconds)
    b = orc.residual(op, x)
    # ISTL BiCGSTAB on the assembled system, a fixed number of iterations (reduction 1e-30 never
    # stops it), timed by the oracle itself (preconditioner setup and iteration loop apart):
    # NOPREC (the reference's stationary backend), ILU(0) (the GPU run's preconditioner, fp64
    # factors) and SSOR (SeqSSOR(A,1,1) in the natural order: the reference's default BCGS_SSORk,
    # src/instationary_pnp_from_pb_md.hh:188-191) on one thread, then on all the job's host
    # threads: OpenMP row-parallel SpMV / dots / updates, and the preconditioners block-Jacobi on
    # `threads` vertex ranges swept in parallel (orc_set_block_jacobi: what the NOVLP backend
    # applies with that many MPI ranks)
    bthreads = int(O.lib().orc_num_threads())
    rates = {}
    for label, par, its in (("1t", 0, 4), ("mt", 1, 8)):
        O.lib().orc_set_parallel(par)
        O.lib().orc_set_block_jacobi(bthreads if par else 0, 3)
        try:
            for pname, pc, k in (("nonprec", O.PREC_NONE, 2 * its), ("ilu0", O.PREC_ILU0, its),
                                 ("ssor", O.PREC_SSOR, its)):
                _, res = O.bicgstab(J, b, prec=pc, reduction=1e-30, maxit=k)
                rates[f"{pname}_{label}"] = {
                    "iters": res.iterations, "s_per_it": res.iter_seconds / max(res.iterations, 1),
                    "setup_s": res.setup_seconds}
        finally:
            O.lib().orc_set_parallel(0)
            O.lib().orc_set_block_jacobi(0, 3)
    t_it, t_it_mt = rates["nonprec_1t"]["s_per_it"], rates["nonprec_mt"]["s_per_it"]
    # (ii) all host cores: the same algorithm, element colours + OpenMP (orc_assemble_mt)
    t_mt, threads, _, _ = orc.time_fd_assembly_mt(op, x, 0.2 * seconds)
    # residual / Jacobian match of the GPU path against the CPU restatement on this sample (the
    # oracle as checker): analytic vs analytic, and vs the reference's FD Jacobian just timed
    ctx = P.Context(pmesh, P.Params.from_config(cfg), device=0)
    ctx.set_operator(P.OP_PNP)
    r_gpu, J_gpu = ctx.residual(x), ctx.jacobian(x)
    ctx.close()
    J_an = orc.jacobian(op, x)
    jscale = abs(J_an).max()
    parity = {"sample_dofs": 3 * nv,
              "residual_rel_err": float(np.max(np.abs(r_gpu - b)) / np.max(np.abs(b))),
              "jacobian_rel_err_vs_analytic": float(abs(J_gpu - J_an).max() / jscale),
              "jacobian_rel_err_vs_reference_fd": float(abs(J_gpu - J).max() / jscale),
              "tolerance": "residual and analytic Jacobian <= 1e-12 of max|.|; FD Jacobian "
                           "<= 1e-5 (forward-difference truncation, SURVEY.md §8(c))"}
    return {"parity": parity, "dofs": 3 * nv, "assembly_s": t_asm, "dofs_per_s": 3 * nv / t_asm,
            "bicgstab_nonprec_s_per_it": t_it, "iterations": rates["nonprec_1t"]["iters"],
            "bicgstab_nonprec_s_per_it_mt": t_it_mt, "bicgstab_rates": rates,
            "bicgstab_threads": bthreads,
            "nnz_full": int(J.nnz), "mt_assembly_s": t_mt, "mt_threads": threads,
            "mt_dofs_per_s": 3 * nv / t_mt}


def cpu_bicg_rates(cb):
    """The CPU leg's preconditioned BiCGSTAB rates (the GPU run's preconditioner
    and the reference's default BCGS_SSORk), one thread and all the job's threads, fp64 factors."""
    r, t = cb["bicgstab_rates"], cb["bicgstab_threads"]
    out = {}
    for pname, key in (("ilu0", "bicgstab_ilu0_iters_per_s"),
                       ("ssor", "bicgstab_ssork_iters_per_s"),
                       ("nonprec", "bicgstab_nonprec_iters_per_s")):
        out[key] = 1.0 / r[f"{pname}_1t"]["s_per_it"]
        out[key + f"_{t}t"] = 1.0 / r[f"{pname}_mt"]["s_per_it"]
    out["bicgstab_ilu0_factorisation_s"] = r["ilu0_1t"]["setup_s"]
    out["bicgstab_cpu_note"] = (
        f"oracle ISTL-semantics BiCGSTAB on the sample's assembled Jacobian, a fixed iteration count "
        f"each, timed inside the oracle (iteration loop only; ILU(0) factorisation apart). 1 thread: "
        f"SeqILU0 (fp64 factors) and SeqSSOR(A,1,1) in the reference's natural DOF order (BCGS_SSORk). "
        f"{t} threads: OpenMP row-parallel SpMV / dots / updates, the ILU(0) and SSOR block-Jacobi on "
        f"{t} vertex ranges swept in parallel (the NOVLP backend's per-rank SeqILU0 / SeqSSOR with {t} "
        f"ranks, orc_set_block_jacobi)")
    return out


def host_cpu_info():
    """The GPU box's host CPU as the CPU baseline ran on it: model name from /proc/cpuinfo, the
    machine's logical CPUs (nproc --all) and the ones this process may run on (nproc)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"cpu_model": model or platform.processor() or platform.machine(),
            "host_logical_cpus": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def measured_stream_gbs(device, reps=10):
    """HBM ceilings measured on this box with hand-written dwordx4 streaming kernels
    (tools/micro/stream.hip, 2 GiB buffers, 8x the Infinity Cache): read-only, write-only, copy
    and the assembly's 26:74 read:write mix, each bytes moved / average launch time (GB/s).  The
    guide's float4 copy reads 6.29 TB/s (MI355X_MICROARCH.md); torch's copy_ is not a ceiling."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "micro", "libstream.so"))
    out = (ctypes.c_double * 4)()
    shapes = (ctypes.c_double * 20)()
    rc = lib.stream_measure(ctypes.c_int(device), ctypes.c_int(reps), out, shapes)
    if rc != 0:
        raise RuntimeError(f"stream_measure: HIP error {rc}")
    names = ("read", "write", "copy", "asm_mix")
    return {"read": out[0], "write": out[1], "copy": out[2], "asm_mix": out[3],
            "shapes": {sh: {names[k]: shapes[4 * i + k] for k in range(4)}
                       for i, sh in enumerate(("u1", "u2", "u4", "u8", "resident_u4"))},
            "source": "tools/micro/stream.hip: dwordx4 kernels on 2 GiB buffers, the fastest of "
                      f"5 shapes, mean of {reps} event-timed launches; asm_mix = 26:74 read:write "
                      "(the assembly's PMC split)"}


# which measured ceiling bounds each BiCGSTAB kernel class: the SpMV and the ILU(0) sweeps are
# read streams (PMC: 266 MB read / 18 MB written per SpMV), the vector updates read and write
STREAM_CEILING = {"spmv": "read", "ilu0_apply": "read", "blas_per_iter": "copy"}


def with_stream_fracs(kernels, stream_gbs):
    """Each kernel's achieved rate also as a fraction of its measured stream ceiling."""
    out = {}
    for k, v in kernels.items():
        if v is None:
            out[k] = None
            continue
        c = STREAM_CEILING[k]
        out[k] = dict(v, measured_ceiling=c,
                      frac_of_measured=v["achieved"] / stream_gbs[c] if stream_gbs else None)
    return out


def byte_models(info, nf, N_local, T_local, prec):
    """Per-launch bytes: SURVEY.md §8(d) contract (reduced CSR) and the stored formats."""
    V = info["nv_owned"]
    nnz_red = info["nvb"] * info["nblocks"]
    n_loc = nf * (info["nv_owned"] + info["nv_ghost"])
    B_asm = 8 * nnz_red + 16 * N_local + 12 * T_local + 16 * V
    pre = prec != P.PREC_NONE
    B_it = (48 if pre else 24) * nnz_red + (304 if pre else 232) * N_local
    # stored formats: SpMV = k-form values + a 4-B column index per slot, x gathered once, y
    # written, the fused dot's operand read
    spmv = info["nslots"] * (8 * info["nks"] + 4) + 8 * n_loc + 16 * N_local
    # ILU(0) apply: split factors (NV expanded values + index per slot), d read, forward result
    # written, re-read by the backward sweep (gathers counted once), v written
    # bytes per block of the stored factors: float (quads + the remainder), bfloat16 (the 7-value
    # PNP block in 14 B, linalg.hip ILU_BF16_B7; other NV rounded up to 8 shorts), or double;
    # mode 3: bfloat16 factors and a 4-B forward intermediate (scalar systems run 2 and 3 as 1)
    nvb = info["nvb"]
    mode = info["ilu_f32"] if nvb > 1 or info["ilu_f32"] < 2 else 1
    vb = {1: 4 * nvb, 2: 2 * (nvb if nvb in (1, 7) else (nvb + 7) // 8 * 8)}.get(min(mode, 2), 8 * nvb)
    yb = 4 if mode == 3 else 8
    ilu = (info["lslots"] + info["uslots"]) * (vb + 4) + 8 * N_local + (2 * yb + 8) * n_loc
    if mode == 1 and nvb == 7:
        ilu -= 16 * V  # the forward steps read only the 12-B lower tail of each diagonal block
    pb = pmc_blas_bytes(N_local)
    # the update kernels' counted bytes (PMC); ~24 vector passes (the contract's 192 N) only when
    # no committed summary has them
    blas = pb["bytes"] if pb else 192 * N_local
    return {"asm": B_asm, "it_contract": B_it, "spmv_stored": spmv, "ilu_stored": ilu,
            "blas": blas, "blas_source": (f"PMC: {pb['source']}" if pb else "model: 192 N"),
            "blas_per_kernel": pb["per_kernel"] if pb else None,
            "it_stored": 2 * spmv + (2 * ilu if pre else 0) + blas}


TRANSPORT = "rccl"  # --transport: rccl (one GPU per rank) or host (pnp_comm.host over gloo)


def new_context(mesh, par, rank, world, local, dist):
    """This rank's context: RCCL at N > 1 (the unique id broadcast from rank 0), or with
    --transport host the host-staged transport over the gloo group (ranks may share a GPU:
    rehearses the N > 1 bench on a one-GPU box)."""
    if world > 1 and TRANSPORT == "host":
        return P.Context(mesh, par, device=local, rank=rank, size=world,
                         host_transport=P.TorchDistTransport(dist))
    uid = None
    if world > 1:
        obj = [P.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    return P.Context(mesh, par, device=local, rank=rank, size=world, unique_id=uid)


def make_context(mesh, cfg, rank, world, local, dist):
    ctx = new_context(mesh, P.Params.from_config(cfg), rank, world, local, dist)
    # Boltzmann initial state: PB Newton, then the BCExtension interpolation
    t_setup = time.perf_counter()
    ctx.set_operator(P.OP_PB)
    pb_prec = P.PREC_ILU0 if "without_dna" in cfg.meshfile else P.PREC_SSOR
    phi_pb, pb_res = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=pb_prec,
                                linear_maxit=20000)
    phi_pb = ctx.sync_vector(phi_pb, 1)  # each rank returns its owned entries; combine
    x0 = ctx.initial_state(phi_pb)
    ctx.set_operator(P.OP_PNP)
    ctx.state_set(x0)
    return ctx, x0, pb_res, time.perf_counter() - t_setup


def measure(ctx, mesh, args, prec, dist, world):
    """Timed regions on one context: warm assembly (the metric), BiCGSTAB, then the event-timed
    passes (warm, cache-cold) the rooflines are computed from."""
    info = ctx.info()
    ctx.assemble_state(1)  # the solve needs an assembled Jacobian
    ctx.bicgstab_iterations(max(1, args.warmup), prec)
    # the W warmup assemblies right before the timed ones: after a solve the matrix lines are out
    # of the Infinity Cache and it takes two launches to bring the write stream back (rocprofv3
    # trace r2bg: 87, 77, then 48 us)
    ctx.assemble_state(max(2, args.warmup))
    # ---- timed region 1: assembly --------------------------------------------------------------
    barrier_sync(dist, world)
    t0 = time.perf_counter()
    ctx.assemble_state(args.steps)
    barrier_sync(dist, world)
    t_asm = time.perf_counter() - t0
    # ---- timed region 2: BiCGSTAB --------------------------------------------------------------
    barrier_sync(dist, world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.bicgstab_iterations(args.bicg_iters, prec)
    barrier_sync(dist, world)
    t_bicg = time.perf_counter() - t0
    # ---- event-timed passes (library stream) ---------------------------------------------------
    ctx.assemble_state(2)  # untimed, as before region 1: the warm pass follows two assemblies
    ctx.timers(enable=True, reset=True)
    ctx.assemble_state(args.steps)
    ctx.bicgstab_iterations(args.bicg_iters, prec)
    tm = ctx.timers(enable=False)
    ctx.timers(reset=True)
    for _ in range(args.steps):  # cache-cold: 1 GiB read between launches (untimed)
        ctx.cache_scrub(SCRUB_BYTES)
        ctx.timers(enable=True)
        ctx.assemble_state(1)
        ctx.timers(enable=False)
    tm_cold = ctx.timers()
    # in situ: each assembly right after a BiCGSTAB block, as pnp_newton runs it (the solve's
    # vector and matrix streams have replaced the assembly's data in the caches)
    ctx.timers(reset=True)
    for _ in range(args.steps):
        ctx.bicgstab_iterations(args.bicg_iters, prec)
        ctx.timers(enable=True)
        ctx.assemble_state(1)
        ctx.timers(enable=False)
    tm_situ = ctx.timers()
    # the warm roofline's launch time: one event pair around K back-to-back launches (the per-launch
    # event pairs above add ~3 us each, r2bj: 50.2 us against rocprofv3's 47.4 us)
    ctx.assemble_state(2)
    asm_batch_s = ctx.assemble_state_timed(args.steps) / args.steps
    # BiCGSTAB with fp64 ILU(0) factors (the default stores them in single precision)
    t_bicg64 = None
    f_default = ctx.get_option(P.OPT_ILU_F32)
    if prec == P.PREC_ILU0:
        ctx.set_option(P.OPT_ILU_F32, 0)
        ctx.bicgstab_iterations(2, prec)
        barrier_sync(dist, world)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            ctx.bicgstab_iterations(args.bicg_iters, prec)
        barrier_sync(dist, world)
        t_bicg64 = max_over_ranks(dist, world, time.perf_counter() - t0)
        ctx.set_option(P.OPT_ILU_F32, f_default)
    t_asm, t_bicg = max_over_ranks(dist, world, t_asm), max_over_ranks(dist, world, t_bicg)

    nf = 3
    N_global = 3 * mesh.nv
    N_local = 3 * info["nv_owned"]
    T_local = int(round(mesh.nt * info["nv_owned"] / mesh.nv))
    B = byte_models(info, nf, N_local, T_local, prec)
    asm_ev_s = tm["assemble_ms"] / max(1, tm["assemble_launches"]) / 1e3
    asm_s = asm_batch_s
    asm_cold_s = tm_cold["assemble_ms"] / max(1, tm_cold["assemble_launches"]) / 1e3
    asm_situ_s = tm_situ["assemble_ms"] / max(1, tm_situ["assemble_launches"]) / 1e3
    it_ev = (tm["spmv_ms"] + tm["prec_ms"] + tm["blas_ms"] + tm["halo_ms"] +
             tm["allreduce_ms"]) / 1e3 / args.bicg_iters
    spmv_s = tm["spmv_ms"] / max(1, tm["spmv_launches"]) / 1e3
    prec_s = tm["prec_ms"] / max(1, tm["prec_launches"]) / 1e3
    blas_s = tm["blas_ms"] / 1e3 / args.bicg_iters
    rl = lambda b, t: {"bytes": b, "seconds": t, "achieved": b / t / 1e9,  # noqa: E731
                       "frac": b / t / 1e9 / HBM_PEAK_GBS}
    return {
        "info": info, "N_global": N_global, "N_local": N_local, "t_asm": t_asm,
        "t_bicg": t_bicg, "timers": tm, "timers_cold": tm_cold, "bytes": B,
        "dofs_per_s": N_global * args.steps / t_asm,
        "iters_per_s": args.steps * args.bicg_iters / t_bicg,
        "asm_warm": rl(B["asm"], asm_s), "asm_cold": rl(B["asm"], asm_cold_s),
        "asm_situ": rl(B["asm"], asm_situ_s),
        "iters_per_s_f64_factors": (args.steps * args.bicg_iters / t_bicg64) if t_bicg64 else None,
        "asm_warm_per_launch_events_s": asm_ev_s,
        "it_contract": rl(B["it_contract"], it_ev), "it_stored": rl(B["it_stored"], it_ev),
        "spmv_stored": rl(B["spmv_stored"], spmv_s),
        "ilu_stored": rl(B["ilu_stored"], prec_s) if prec != P.PREC_NONE else None,
        "blas": dict(rl(B["blas"], blas_s), source=B["blas_source"],
                     per_kernel_bytes=B["blas_per_kernel"]),
    }


def rccl_parity(sctx, smesh, scfg, x0, rank, world, local, dist):
    """Self-check of the multi-GPU path on the config-5 (strong) system: the global residual R(x0)
    and the converged PNP Newton solution (reduction 1e-10, linear solves to 1e-8; BiCGSTAB with the
    aggregation AMG, ILU(0) smoother, block-Jacobi across ranks -- with ILU(0) alone the tight solve
    takes ~30 s on one GPU) of the partitioned context, against a one-rank context on rank 0's GPU.
    At N = 1 the "partitioned" side is a context with a 1-rank RCCL communicator of its own (every reduction an ncclAllReduce, the
    halo-split SpMV path).  Bounds: residual 1e-13 relative, solution 1e-6."""
    s = scfg.system
    # the linear solves to 1e-8 (pore.cfg's newtonMinLinearReduction is 1e-5): with 1e-5 the two
    # solutions differed by 2.0e-6 at N = 2 (gpurun_out/r5l), the loose last linear solve's error
    # under two different block-Jacobi AMG preconditioners, not the partitioned numerics
    kw = dict(reduction=1e-10, min_linear_reduction=min(1e-8, s["newtonMinLinearReduction"]),
              prec=P.PREC_AMG, linear_maxit=int(s["linearSolverIterations"]), maxit=20)
    t0 = time.perf_counter()
    par = P.Params.from_config(scfg)
    dctx = sctx if world > 1 else P.Context(smesh, par, device=local, rank=0, size=1,
                                             unique_id=P.rccl_unique_id())
    dctx.set_operator(P.OP_PNP)
    dctx.amg_configure(smoother=P.PREC_ILU0)
    dctx.timers(enable=True, reset=True)
    r_d = dctx.sync_vector(dctx.residual(x0))
    u_d, res_d = dctx.newton(x0, **kw)
    u_d = dctx.sync_vector(u_d)
    tm = dctx.timers(enable=False)
    # the same at the config's own newtonMinLinearReduction (reported, not gated)
    kw_cfg = dict(kw, min_linear_reduction=s["newtonMinLinearReduction"])
    u_dc, res_dc = dctx.newton(x0, **kw_cfg)
    u_dc = dctx.sync_vector(u_dc)
    dinfo = dctx.info()
    mine = {"rank": rank, "transport": dinfo["transport"], "nranks": dinfo["nranks"],
            "nv_owned": dinfo["nv_owned"], "nv_ghost": dinfo["nv_ghost"],
            "halo_ms": tm["halo_ms"], "allreduce_ms": tm["allreduce_ms"],
            "spmv_launches": tm["spmv_launches"]}
    if world > 1:
        allr = [None] * world
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
        dctx.close()
    out = None
    if rank == 0:
        c1 = P.Context(smesh, par, device=local)
        c1.set_operator(P.OP_PNP)
        c1.amg_configure(smoother=P.PREC_ILU0)
        r1 = c1.residual(x0)
        u1, res1 = c1.newton(x0, **kw)
        u1c, res1c = c1.newton(x0, **kw_cfg)
        c1.close()
        er = float(np.max(np.abs(r_d - r1)) / np.max(np.abs(r1)))
        eu = float(np.max(np.abs(u_d - u1)) / np.max(np.abs(u1)))
        euc = float(np.max(np.abs(u_dc - u1c)) / np.max(np.abs(u1c)))
        out = {"system": f"config 5 ({3 * smesh.nv} DOFs), x0 = Boltzmann initial state",
               "ranks": world, "transport": ["plain", "local", "rccl", "host"][allr[0]["transport"]],
               "rccl_ranks_seen": allr[0]["nranks"],
               "residual_rel_err": er, "solution_rel_err": eu,
               "newton_converged": [res_d["converged"], res1["converged"]],
               "newton_steps": [res_d["iterations"], res1["iterations"]],
               "bicgstab_iterations": [res_d["linear_iterations"], res1["linear_iterations"]],
               "halo_ms_max_over_ranks": max(a["halo_ms"] for a in allr),
               "allreduce_ms_max_over_ranks": max(a["allreduce_ms"] for a in allr),
               "ghost_vertices_per_rank": [a["nv_ghost"] for a in allr],
               "pass": bool(er <= 1e-13 and eu <= 1e-6 and res_d["converged"] == 1 and
                            res1["converged"] == 1),
               "bounds": "residual <= 1e-13, solution <= 1e-6 (relative, max norm); linear "
                         "solves to 1e-8",
               "at_config_linear_reduction": {
                   "min_linear_reduction": s["newtonMinLinearReduction"],
                   "solution_rel_err": euc,
                   "newton_converged": [res_dc["converged"], res1c["converged"]],
                   "bicgstab_iterations": [res_dc["linear_iterations"],
                                           res1c["linear_iterations"]],
                   "gated": False,
                   "note": "pore.cfg's own linear tolerance: the two block-Jacobi AMG "
                           "preconditioners leave different last-solve errors (not gated)"},
               "seconds": None}
    barrier_sync(dist, world)
    if out is not None:
        out["seconds"] = time.perf_counter() - t0
    return out


def ssork_natural_leg(ctx, mesh, x0, nit, dist=None, world=1):
    """The reference's default linear solver, BCGS_SSORk (BiCGSTAB + ISTL SeqSSOR in the
    reference's DOF order, PNP_PREC_SSOR_NATURAL: bitwise the oracle's SeqSSOR on one rank; each
    rank sweeps its owned rows at N > 1, the NOVLP backend's block SeqSSOR), on the PNP system at x0
    and on the PB system at its potential: one preconditioner application (device timers) and one
    BiCGSTAB iteration (two applications, two SpMVs, the reductions), after two untimed
    iterations.  Every rank that owns its GPU runs the one-launch dataflow schedule (its rank's
    `schedule` field counts the applications per schedule); at N > 1 the per-rank ms per
    application and the slowest rank's iteration time."""
    out = {}
    nv = mesh.nv
    for name, op, x in (("pnp", P.OP_PNP, x0), ("pb", P.OP_PB, x0[:nv])):
        ctx.set_operator(op)
        ctx.state_set(x)
        ctx.assemble_state(1)
        ctx.bicgstab_iterations(2, P.PREC_SSOR_NATURAL)
        barrier_sync(dist, world)
        t0 = time.perf_counter()
        ctx.bicgstab_iterations(nit, P.PREC_SSOR_NATURAL)
        barrier_sync(dist, world)
        wall = max_over_ranks(dist, world, (time.perf_counter() - t0) / nit)
        info0 = ctx.info()
        ctx.timers(enable=True, reset=True)
        ctx.bicgstab_iterations(nit, P.PREC_SSOR_NATURAL)
        tm = ctx.timers(enable=False)
        ctx.timers(reset=True)
        info1 = ctx.info()
        mine = {"ms_per_apply": tm["prec_ms"] / max(1, tm["prec_launches"]),
                "dataflow_applies": info1["nat_flow_applies"] - info0["nat_flow_applies"],
                "level_applies": info1["nat_level_applies"] - info0["nat_level_applies"]}
        if world > 1:
            allr = [None] * world
            dist.all_gather_object(allr, mine)
        else:
            allr = [mine]
        out[name] = {"dofs": int(len(x)), "ms_per_apply": max(a["ms_per_apply"] for a in allr),
                     "ms_per_apply_per_rank": [a["ms_per_apply"] for a in allr],
                     "dataflow_applies_per_rank": [a["dataflow_applies"] for a in allr],
                     "ms_per_iter": 1e3 * wall, "iters_per_s": 1.0 / wall}
    ctx.set_operator(P.OP_PNP)
    out["schedule"] = ("forward and backward sweep each: the wide levels as dataflow units, the "
                       "narrow ones (at most the resident chain groups' count of rows) as chains, "
                       "one wave per chain group (ssor_natural.hip)")
    return out


def asm_bicg_rates(ctx, n, prec, nasm=10, nit=20):
    """Warm assembly (one event pair around nasm back-to-back launches after two untimed ones) and
    BiCGSTAB (nit fixed iterations after two untimed ones, wall clock) on the context's state."""
    ctx.assemble_state(2)
    t_asm = ctx.assemble_state_timed(nasm) / nasm
    ctx.bicgstab_iterations(2, prec)
    t0 = time.perf_counter()
    ctx.bicgstab_iterations(nit, prec)
    t_it = (time.perf_counter() - t0) / nit
    return {"assemble_us": t_asm * 1e6, "assembled_dofs_per_s": n / t_asm,
            "bicgstab_ms_per_iter": t_it * 1e3, "bicgstab_iters_per_s": 1.0 / t_it}


def newton_summary(res, seconds):
    return {"seconds": seconds, "converged": res["converged"], "iterations": res["iterations"],
            "linear_iterations": res["linear_iterations"],
            "assemble_s": res["assemble_seconds"], "solve_s": res["solve_seconds"]}


def per_config_legs(prec, ie_steps=10):
    """SURVEY.md §8(d)'s other configurations, bounded (N = 1 only, ~20 s):
      config 1: PB on test/sphere_pb refined k=6 (733 K DOF; BASELINE configs[0]): PB Newton from
                0, assembled DOFs/s, BiCGSTAB ms/it with the bench's preconditioner and with the
                reference's default BCGS_SSORk (natural-order SSOR);
      config 2: 2-ion PNP on test/cylinder.msh refined k=6 (3.3 M DOF): PB -> BCExtension -> PNP
                Newton (time to solution), assembled DOFs/s, BiCGSTAB it/s;
      config 4: instationary PNP (PnpOperator + PnpTOperator, implicit Euler, dt = tau,
                src/instationary_pnp_from_pb.hh:409-431): the 100 steps on test/pore.msh that
                BASELINE names, and ie_steps steps on pore_pnp k=3 (556 K DOF) with per-step
                assembly and BiCGSTAB rates and the Newton / BiCGSTAB counts, and the same
                steps again with the aggregation AMG preconditioning BiCGSTAB."""
    out = {}
    # ---- config 1 -------------------------------------------------------------------------------
    t0 = time.perf_counter()
    cfg = P.read_config(os.path.join(ROOT, "data", "sphere_pb", "sphere.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(6)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PB)
    t1 = time.perf_counter()
    phi, res = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=prec)
    pbn = newton_summary(res, time.perf_counter() - t1)
    ctx.state_set(phi)
    r = asm_bicg_rates(ctx, mesh.nv, prec)
    r_nat = asm_bicg_rates(ctx, mesh.nv, P.PREC_SSOR_NATURAL, nasm=1)
    ctx.close()
    out["1"] = {"workload": "PB, test/sphere_pb/sphere.msh refined k=6", "dofs": mesh.nv,
                "pb_newton": pbn, **r,
                "bicgstab_ssork_natural_ms_per_iter": r_nat["bicgstab_ms_per_iter"],
                "leg_seconds": time.perf_counter() - t0}
    # ---- config 2 -------------------------------------------------------------------------------
    t0 = time.perf_counter()
    cfg = P.read_config(os.path.join(ROOT, "data", "cylinder_config.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(6)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PB)
    t1 = time.perf_counter()
    phi, pres = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=prec)
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    s = cfg.system
    t2 = time.perf_counter()
    u, res = ctx.newton(x0, reduction=s["newtonReduction"],
                        min_linear_reduction=s["newtonMinLinearReduction"], prec=prec,
                        linear_maxit=int(s["linearSolverIterations"]))
    t3 = time.perf_counter()
    ctx.state_set(x0)
    r = asm_bicg_rates(ctx, 3 * mesh.nv, prec)
    ctx.close()
    out["2"] = {"workload": "2-ion PNP, test/cylinder.msh refined k=6", "dofs": 3 * mesh.nv,
                "pb_newton_s": t2 - t1, "pnp_newton": newton_summary(res, t3 - t2),
                "time_to_solution_s": t3 - t1, **r, "leg_seconds": time.perf_counter() - t0}
    # ---- config 4 -------------------------------------------------------------------------------
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    s = cfg.system
    # the refined stand-in's tolerances (tools/bench_configs.py config4r): the residual's rounding
    # floor (~2e-10) sits above the reference's relative 1e-9 there
    kw_k3 = dict(reduction=1e-8, abs_limit=1e-9)
    for key, meshfile, refine, nsteps, kw, sprec in (
            ("4", os.path.join(ROOT, "data", "pore.msh"), 0, 100,
             dict(reduction=s["newtonReduction"], min_linear_reduction=s["newtonMinLinearReduction"],
                  abs_limit=1e-12, maxit=int(s["newtonMaxIterations"]),
                  line_search_maxit=int(s["newtonLineSearchMaxIteration"])), prec),
            ("4_pore_pnp_k3", cfg.meshfile, 3, ie_steps, kw_k3, prec),
            # the same steps with the aggregation AMG (ILU(0) smoother) preconditioning BiCGSTAB
            ("4_pore_pnp_k3_amg", cfg.meshfile, 3, ie_steps, kw_k3, P.PREC_AMG)):
        t0 = time.perf_counter()
        mesh = P.Mesh.read_gmsh(meshfile).refine(refine)
        ctx = P.Context(mesh, P.Params.from_config(cfg))
        ctx.set_operator(P.OP_PB)
        phi, _ = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=prec)
        u = ctx.initial_state(phi)
        if sprec == P.PREC_AMG:
            ctx.amg_configure(smoother=P.PREC_ILU0)
        steps = []
        t1 = time.perf_counter()
        for i in range(nsteps):
            ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=s["tau"], x_old=u)
            u, res = ctx.newton(u, prec=sprec, **kw)
            steps.append(res)
            if not res["converged"]:
                break
        t2 = time.perf_counter()
        n = 3 * mesh.nv
        lin = sum(r_["linear_iterations"] for r_ in steps)
        newt = sum(r_["iterations"] for r_ in steps)
        t_as = sum(r_["assemble_seconds"] for r_ in steps)
        t_so = sum(r_["solve_seconds"] for r_ in steps)
        o = {"workload": f"implicit Euler PNP, {os.path.relpath(meshfile, ROOT)} refined k={refine}",
             "dofs": n, "steps": len(steps), "all_converged": all(r_["converged"] for r_ in steps),
             "seconds": t2 - t1, "ms_per_step": 1e3 * (t2 - t1) / max(1, len(steps)),
             "newton_iterations": newt, "bicgstab_iterations": lin,
             "newton_tolerances": {k: v for k, v in kw.items()},
             "per_step": {"newton_iterations": newt / max(1, len(steps)),
                          "bicgstab_iterations": lin / max(1, len(steps)),
                          "assemble_s": t_as / max(1, len(steps)),
                          "solve_s": t_so / max(1, len(steps)),
                          "bicgstab_iters_per_s_in_solve": lin / t_so if t_so > 0 else None}}
        if sprec == P.PREC_AMG:
            o["preconditioner"] = "amg (ILU0 smoother)"
        elif refine > 0:  # event-timed rates on the last step's system (the small mesh is
            ctx.state_set(u)  # launch-bound: its rates say nothing about the kernels)
            o.update(asm_bicg_rates(ctx, n, prec))
        ctx.close()
        o["leg_seconds"] = time.perf_counter() - t0
        out[key] = o
    return out


def strong_mesh(refine):
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_without_dna", "pore.cfg"))
    return cfg, P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(refine)


def primary_mesh(args, world):
    if args.scaling == "strong":
        return strong_mesh(args.strong_refine)
    cfg = P.read_config(args.cfg)
    return cfg, tile_mesh(P.Mesh.read_gmsh(cfg.meshfile).refine(args.refine), world)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--refine", type=int, default=4)
    ap.add_argument("--bicg-iters", type=int, default=20)
    ap.add_argument("--prec", default="ilu0", choices=["none", "jacobi", "ssor", "ilu0", "amg"])
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="primary line: weak (config 3 per GPU, default) or strong (config 5 "
                         "split over the ranks)")
    ap.add_argument("--strong-refine", type=int, default=6,
                    help="refinement of the config-5 mesh (6: 8.87 M DOF)")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the config-5 strong-scaling leg")
    ap.add_argument("--no-solve", action="store_true",
                    help="skip the time-to-solution PNP Newton after the timed regions")
    ap.add_argument("--no-amg", action="store_true",
                    help="skip the AMG-preconditioned time-to-solution leg")
    ap.add_argument("--amg-multi", action="store_true",
                    help="run the AMG time-to-solution leg at N>1 too (default: N=1 only)")
    ap.add_argument("--no-ssork", action="store_true",
                    help="skip the BCGS_SSORk (natural-order SSOR) leg")
    ap.add_argument("--no-per-config", action="store_true",
                    help="skip the configs 1 / 2 / 4 legs (per_config, N=1 only)")
    ap.add_argument("--no-parity", action="store_true",
                    help="skip the multi-GPU self-check (rccl_parity) on the config-5 system")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--cpu-refine", type=int, default=4,
                    help="refinement of the CPU sample (4: the config-3 mesh itself)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cfg", default=os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    ap.add_argument("--transport", default="rccl", choices=["rccl", "host"],
                    help="N > 1: RCCL (default, one GPU per rank) or the host-staged transport over "
                         "gloo (pnp_comm.host; ranks may share a GPU: a one-box rehearsal)")
    ap.add_argument("--newton-reduction", type=float, default=None,
                    help="time-to-solution leg: Newton reduction (default: the config's)")
    ap.add_argument("--min-linear-reduction", type=float, default=None,
                    help="time-to-solution leg: min linear reduction (default: the config's)")
    args = ap.parse_args()

    global TRANSPORT
    TRANSPORT = args.transport
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(1)))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # torch only syncs around the timed regions: bind it to this rank's GPU (its default is device
    # 0, whatever LOCAL_RANK the library runs on); the host transport may put several ranks on one
    import torch
    if args.transport == "host":
        local = local % max(1, torch.cuda.device_count())
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    prec = P.PREC_BY_NAME[args.prec]

    progress(rank, f"N = {world}: stream ceilings")
    try:  # a measurement helper: its failure costs the line the measured ceilings, nothing else
        stream_gbs = measured_stream_gbs(local)
    except (OSError, RuntimeError) as exc:
        progress(rank, f"measured_stream_gbs unavailable: {exc}")
        stream_gbs = None
    progress(rank, "primary system: mesh, PB Newton, timed assembly and BiCGSTAB")
    cfg, mesh = primary_mesh(args, world)
    ctx, x0, pb_res, t_setup = make_context(mesh, cfg, rank, world, local, dist)
    M = measure(ctx, mesh, args, prec, dist, world)
    info = M["info"]

    # ---- time to solution (reported beside the metric): PNP Newton from the Boltzmann state ----
    newton = None
    progress(rank, "time to solution: PNP Newton (ILU(0) f32 / f64, AMG)")
    nt_red = args.newton_reduction or cfg.system["newtonReduction"]
    nt_linred = args.min_linear_reduction or cfg.system["newtonMinLinearReduction"]

    def tts_leg():
        barrier_sync(dist, world)
        t0 = time.perf_counter()
        # bounded (10 Newton steps) so a block-Jacobi preconditioner that converges slowly at N>1
        # cannot stall the scaling runs; the metric does not include this leg
        _, nres = ctx.newton(x0, reduction=nt_red, min_linear_reduction=nt_linred, prec=prec,
                             linear_maxit=int(cfg.system["linearSolverIterations"]), maxit=10)
        barrier_sync(dist, world)
        return {"seconds": time.perf_counter() - t0, "converged": nres["converged"],
                "status": nres["status"], "iterations": nres["iterations"],
                "linear_iterations": nres["linear_iterations"],
                "first_defect": nres["first_defect"], "defect": nres["defect"],
                "assemble_s": nres["assemble_seconds"], "solve_s": nres["solve_seconds"],
                "precision_retries": nres.get("precision_retries"),
                "reduction": nt_red, "min_linear_reduction": nt_linred,
                "preconditioner": args.prec + (
                    ", " + {1: "f32 factors", 2: "bf16 factors",
                            3: "bf16 factors, f32 intermediate"}.get(
                        ctx.get_option(P.OPT_ILU_F32), "f64 factors")
                    if prec == P.PREC_ILU0 else "")}
    if not args.no_solve:
        newton = guarded(rank, "time to solution", tts_leg)
    # the same with fp64 ILU(0) factors (the default stores them in single precision): the f32
    # choice's effect on time to solution, linear iterations and seconds side by side
    newton_f64 = None

    def tts_f64_leg():
        f_default = ctx.get_option(P.OPT_ILU_F32)
        ctx.set_option(P.OPT_ILU_F32, 0)
        try:
            barrier_sync(dist, world)
            t0 = time.perf_counter()
            _, nres = ctx.newton(x0, reduction=nt_red, min_linear_reduction=nt_linred, prec=prec,
                                 linear_maxit=int(cfg.system["linearSolverIterations"]), maxit=10)
            barrier_sync(dist, world)
        finally:
            ctx.set_option(P.OPT_ILU_F32, f_default)
        return {"seconds": time.perf_counter() - t0, "converged": nres["converged"],
                "iterations": nres["iterations"],
                "linear_iterations": nres["linear_iterations"], "defect": nres["defect"],
                "assemble_s": nres["assemble_seconds"], "solve_s": nres["solve_seconds"],
                "preconditioner": "ilu0, fp64 factors"}
    if not args.no_solve and prec == P.PREC_ILU0:
        newton_f64 = guarded(rank, "time to solution (fp64 factors)", tts_f64_leg)
    # the same with the aggregation AMG (PNP_PREC_AMG, ILU(0) smoother) preconditioning BiCGSTAB
    newton_amg = None

    def tts_amg_leg():
        ctx.amg_configure(smoother=P.PREC_ILU0)  # defaults: omega 0.8, 2 coarse sweeps
        # warm-up (untimed): first AMG setup loads rocSOLVER's getrf/getri kernels
        ctx.newton(x0, reduction=nt_red, min_linear_reduction=nt_linred, prec=P.PREC_AMG,
                   linear_maxit=20, maxit=1)
        barrier_sync(dist, world)
        t0 = time.perf_counter()
        _, nres = ctx.newton(x0, reduction=nt_red, min_linear_reduction=nt_linred,
                             prec=P.PREC_AMG,
                             linear_maxit=int(cfg.system["linearSolverIterations"]), maxit=10)
        barrier_sync(dist, world)
        return {"seconds": time.perf_counter() - t0, "converged": nres["converged"],
                "status": nres["status"], "iterations": nres["iterations"],
                "linear_iterations": nres["linear_iterations"], "defect": nres["defect"],
                "linear_fallbacks": nres["linear_fallbacks"],
                "preconditioner": "amg (ILU0 smoother, 2 block-Jacobi sweeps omega=0.8 "
                                  "on the coarse levels)",
                "amg_rows": ctx.amg_info()["rows"]}
    if not args.no_solve and not args.no_amg and (world == 1 or args.amg_multi):
        newton_amg = guarded(rank, "time to solution (AMG)", tts_amg_leg)
    ssork = None
    if not args.no_ssork:
        progress(rank, "BCGS_SSORk (natural-order SSOR)")
        ssork = guarded(rank, "BCGS_SSORk",
                        lambda: ssork_natural_leg(ctx, mesh, x0, args.bicg_iters, dist, world))
    ctx.close()
    per_config = None
    if world == 1 and not args.no_per_config:
        progress(rank, "per-config legs (configs 1, 2, 4)")
        per_config = guarded(rank, "per-config legs", lambda: per_config_legs(prec))

    # ---- config 5, one mesh split over the ranks (strong scaling of the north-star system) -----
    strong = parity = None

    def strong_leg():
        progress(rank, "config 5 (strong scaling)")
        scfg, smesh = strong_mesh(args.strong_refine)
        sctx, sx0, spb, s_setup = make_context(smesh, scfg, rank, world, local, dist)
        try:
            S = measure(sctx, smesh, args, prec, dist, world)
            par = None
            if not args.no_parity:
                progress(rank, "rccl_parity (partitioned vs one-rank Newton on config 5)")
                par = guarded(rank, "rccl_parity",
                              lambda: rccl_parity(sctx, smesh, scfg, sx0, rank, world, local, dist))
        finally:
            sctx.close()
        st = {"workload": f"config 5: stationary 3-ion PNP, test/pore_without_dna .geo meshed "
                          f"natively (scale 0.85), refined k={args.strong_refine}, one mesh "
                          f"RCB-split over {world} GPU(s)",
              "scaling": "strong", "dofs": S["N_global"], "dofs_per_gpu": S["N_local"],
              "assembled_dofs_per_s": S["dofs_per_s"],
              "ms_per_step": 1e3 * S["t_asm"] / args.steps,
              "bicgstab_iters_per_s": S["iters_per_s"],
              "bicgstab_ms_per_iter": 1e3 * S["t_bicg"] / (args.steps * args.bicg_iters),
              "roofline_assembly_warm": S["asm_warm"], "roofline_assembly_cold": S["asm_cold"],
              "roofline_bicgstab_stored": S["it_stored"], "spmv_stored": S["spmv_stored"],
              "roofline_assembly_in_situ": S["asm_situ"],
              "ilu0_apply_stored": S["ilu_stored"], "blas_per_iter": S["blas"],
              "kernels_profile": profile_bicg(5) if world == 1 else None,
              "colors": S["info"]["ncolors"],
              "ghost_vertices": S["info"]["nv_ghost"], "setup_s": s_setup,
              "halo_ms_per_iter": S["timers"]["halo_ms"] / args.bicg_iters,
              "allreduce_ms_per_iter": S["timers"]["allreduce_ms"] / args.bicg_iters}
        return st, par
    if args.scaling == "weak" and not args.no_strong:
        res = guarded(rank, "config 5 (strong scaling)", strong_leg)
        strong, parity = (res, None) if isinstance(res, dict) else res

    cpu = cpu_all = None
    if rank == 0 and world == 1 and not args.no_cpu:  # the contract: rank 0 at N=1 only
        progress(rank, "CPU baseline (oracle, 1 and 16 threads)")
        hostcpu = host_cpu_info()
        cb = cpu_baseline(cfg if args.scaling == "weak" else P.read_config(args.cfg),
                          args.cpu_refine, args.cpu_seconds)
        cpu = {"value": cb["dofs_per_s"], "unit": "assembled DOFs/s", "cores": 1, "kind": "port",
               "sample": (f"oracle/pnp_oracle.c (C restatement of the reference: PnpOperator "
                          f"residual + PDELab forward-difference Jacobian + BCRS-style scatter) on "
                          f"pore_pnp refined k={args.cpu_refine} ({cb['dofs']} DOFs), "
                          f"{cb['assembly_s']:.3f} s per assembly, single thread on "
                          f"{hostcpu['cpu_model']}; ISTL BiCGSTAB NOPREC "
                          f"on the same system {cb['bicgstab_nonprec_s_per_it'] * 1e3:.2f} ms/it"),
               "bicgstab_nonprec_iters_per_s_at_sample": 1.0 / cb["bicgstab_nonprec_s_per_it"],
               **cpu_bicg_rates(cb),
               "host": hostcpu,
               "gpu_vs_cpu_parity": cb["parity"]}
        cpu_all = {"value": cb["mt_dofs_per_s"], "unit": "assembled DOFs/s",
                   "cores": cb["mt_threads"], "kind": "port",
                   "label": f"{cb['mt_threads']} threads (not all {hostcpu['host_logical_cpus']} "
                            f"host CPUs: the GPU box gives one GPU's job a 16-CPU share and sets "
                            f"OMP_NUM_THREADS={hostcpu['omp_num_threads']})",
                   "sample": (f"the same assembly on the same sample with OpenMP over element "
                              f"colours (orc_assemble_mt), {cb['mt_threads']} threads "
                              f"(OMP_NUM_THREADS), {cb['mt_assembly_s']:.4f} s per "
                              f"assembly; ISTL BiCGSTAB NOPREC row-parallel "
                              f"{cb['bicgstab_nonprec_s_per_it_mt'] * 1e3:.2f} ms/it"),
                   "bicgstab_nonprec_iters_per_s": 1.0 / cb["bicgstab_nonprec_s_per_it_mt"],
                   "host": hostcpu}

    if rank == 0:
        tm = M["timers"]
        aw, ac, asit = M["asm_warm"], M["asm_cold"], M["asm_situ"]
        traffic = pmc_traffic("k_assemble_ga<0, 1, 3, 9, 6")
        if args.scaling == "weak":
            workload = (f"config 3: stationary 3-ion PNP, test/pore_pnp/pore.msh refined "
                        f"k={args.refine} x {world} mirrored copies")
        else:
            workload = (f"config 5: stationary 3-ion PNP, test/pore_without_dna .geo meshed "
                        f"natively (scale 0.85), refined k={args.strong_refine}, one mesh "
                        f"RCB-split over {world} GPU(s)")
        line = {
            "metric": "assembled DOFs/s + BiCGStab iters/s, 3-species PNP on pore.msh-refined",
            "value": M["dofs_per_s"],
            "unit": "assembled DOFs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * M["t_asm"] / args.steps,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "reference inputs: test/pore_pnp mesh (refined) + pore.cfg; state = Boltzmann "
                    "initial state from a GPU PB Newton solve (no synthetic vectors)",
            "config": {"workload": workload,
                       "dofs": M["N_global"], "dofs_per_gpu": M["N_local"],
                       "mesh_vertices": mesh.nv, "triangles": mesh.nt,
                       "parallelism": f"mesh partition (RCB) x{world}",
                       "preconditioner": args.prec, "colors": info["ncolors"],
                       "sell_slots": info["nslots"], "blocks": info["nblocks"]},
            "bicgstab_iters_per_s": M["iters_per_s"],
            "bicgstab_ms_per_iter": 1e3 * M["t_bicg"] / (args.steps * args.bicg_iters),
            "bicgstab_iters_per_s_f64_factors": M["iters_per_s_f64_factors"],
            # the headline roofline: the assembly launch as Newton runs it (right after a
            # BiCGSTAB block, the solve's streams have replaced the assembly's data in the caches);
            # the back-to-back (warm) launch behind `value` is roofline_warm
            "roofline": {"bound": "hbm", "achieved": asit["achieved"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": asit["frac"], "traffic": traffic,
                         "kernel": "k_assemble_ga<OP_PNP,1> (gather-all fan walk), in situ: each "
                                   f"launch right after {args.bicg_iters} BiCGSTAB iterations",
                         "regime": "in_situ",
                         "achieved_is": "algorithmic (contract) bytes, SURVEY.md §8(d) B_asm, per "
                                        "launch / launch time (HIP event pair per launch on the "
                                        "library stream)",
                         "bytes_per_launch": asit["bytes"], "avg_launch_us": asit["seconds"] * 1e6,
                         "profile": (profile_regime("in_situ") if args.scaling == "weak"
                                     else None),
                         "hbm_gbs_from_traffic": (traffic / asit["seconds"] / 1e9) if traffic
                                                 else None,
                         "frac_of_measured_asm_mix": (asit["achieved"] / stream_gbs["asm_mix"]
                                                      if stream_gbs else None),
                         "hbm_frac_of_measured_asm_mix":
                             (traffic / asit["seconds"] / 1e9 / stream_gbs["asm_mix"])
                             if traffic and stream_gbs else None,
                         "traffic_source": ((pmc_summary() or {}).get("path", "none") +
                                            " (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch, "
                                            "separate passes; x2 calibrated in profiles/r04/calib)")},
            "roofline_warm": {"bound": "hbm", "achieved": aw["achieved"], "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": aw["frac"], "traffic": traffic,
                              "regime": "warm",
                              "hbm_gbs_from_traffic": (traffic / aw["seconds"] / 1e9) if traffic
                                                      else None,
                              "hbm_frac_of_measured_asm_mix":
                                  (traffic / aw["seconds"] / 1e9 / stream_gbs["asm_mix"])
                                  if traffic and stream_gbs else None,
                              "bytes_per_launch": aw["bytes"], "avg_launch_us": aw["seconds"] * 1e6,
                              "timing": "one HIP event pair on the library stream around K back-"
                                        "to-back launches (the timed region behind `value`)",
                              "avg_launch_us_per_launch_events":
                                  M["asm_warm_per_launch_events_s"] * 1e6,
                              "profile": profile_regime("warm") if args.scaling == "weak" else None,
                              "note": "back-to-back launches: at config 3 the matrix write stream "
                                      "partly stays in the 256 MiB Infinity Cache, so counted bytes "
                                      "move faster than the measured HBM mix ceiling; not an HBM "
                                      "fraction"},
            "roofline_cold": {"bound": "hbm", "achieved": ac["achieved"], "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": ac["frac"], "bytes_per_launch": ac["bytes"],
                              "avg_launch_us": ac["seconds"] * 1e6,
                              "frac_of_measured_asm_mix": (ac["achieved"] / stream_gbs["asm_mix"]
                                                           if stream_gbs else None),
                              "hbm_frac_of_measured_asm_mix":
                                  (traffic / ac["seconds"] / 1e9 / stream_gbs["asm_mix"])
                                  if traffic and stream_gbs else None,
                              "profile": profile_regime("cold") if args.scaling == "weak" else None,
                              "scrub": f"{SCRUB_BYTES >> 20} MiB read between launches"},
            "measured_stream_gbs": stream_gbs,
            "roofline_bicgstab": {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "event_ms_per_iter": M["it_stored"]["seconds"] * 1e3,
                                  "bytes_per_iter": M["it_stored"]["bytes"],
                                  "achieved": M["it_stored"]["achieved"],
                                  "frac": M["it_stored"]["frac"],
                                  "byte_model": "stored formats (k-form SELL + 4-B index per "
                                                "slot, split ILU(0) factors, vectors)",
                                  "ilu_factor_precision": {0: "f64", 1: "f32", 2: "bf16",
                                                           3: "bf16"}.get(info["ilu_f32"], "f32"),
                                  "ilu_intermediate_precision": "f32" if info["ilu_f32"] == 3
                                                                else "f64",
                                  "contract_bytes_per_iter": M["it_contract"]["bytes"],
                                  "contract_model_gbs": M["it_contract"]["achieved"],
                                  "contract_model_ratio": M["it_contract"]["frac"],
                                  "contract_model_note": "SURVEY.md §8(d)'s fp64-CSR byte count "
                                                         "/ iteration time / 8 TB/s: a ratio of "
                                                         "the contract model, NOT a bandwidth "
                                                         "(the k-form SELL values and the f32 "
                                                         "factors move fewer bytes than the "
                                                         "fp64 CSR the contract counts)",
                                  "kernels": with_stream_fracs(
                                      {"spmv": M["spmv_stored"], "ilu0_apply": M["ilu_stored"],
                                       "blas_per_iter": M["blas"]}, stream_gbs),
                                  "kernels_profile": (profile_bicg(3) if args.scaling == "weak"
                                                      and world == 1 else None),
                                  "ilu0_launch_model": (ilu_launch_model() if world == 1
                                                        else None),
                                  "kernels_timing": "event pairs around each unit's launches "
                                                    "(launch gaps included); kernels_profile: "
                                                    "the same pass's device time per unit from "
                                                    "the committed kernel trace"},
            "cpu_baseline": cpu,
            "cpu_baseline_multithread": cpu_all,
            "setup_s": t_setup,
            "pb_newton": {"iterations": pb_res["iterations"],
                          "linear_iterations": pb_res["linear_iterations"],
                          "converged": pb_res["converged"]},
            "event_timers_ms": tm,
            "pnp_newton_time_to_solution": newton,
            "pnp_newton_time_to_solution_f64_factors": newton_f64,
            "pnp_newton_time_to_solution_amg": newton_amg,
            "bicgstab_ssork_natural": ssork,
            "per_config": per_config,
            "strong_scaling": strong,
            "rccl_parity": parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
