"""Multi-rank parity on ONE GPU (-m gpu): P contexts in one process, one host thread per rank,
joined through the in-process test transport (pnp_comm.local_group).  This runs the same
partition (RCB), ghost/halo exchange, owned-row reductions and block-Jacobi preconditioner code
as the RCCL path; only the byte movement differs (device-to-device copies + host barriers
instead of ncclSend/ncclRecv/ncclAllReduce).  Results must equal the single-rank ones."""
import itertools
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import scipy.sparse as sp

import pnp_amd as P
from conftest import DATA
from test_gpu import golden

pytestmark = pytest.mark.gpu
_grp = itertools.count()


def run_ranks(nranks, mesh, par, fn):
    name = f"t{next(_grp)}"

    def work(r):
        ctx = P.Context(mesh, par, device=0, rank=r, size=nranks, local_group=name)
        try:
            return fn(ctx, r)
        finally:
            ctx.close()
    with ThreadPoolExecutor(nranks) as ex:
        return list(ex.map(work, range(nranks)))


@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_residual_and_jacobian_partitioned(nranks):
    z, mesh, par, orc = golden("pore_small_k0")
    x = z["pnp_x"]

    def fn(ctx, r):
        ctx.set_operator(P.OP_PNP)
        res = ctx.residual(x)
        J = ctx.jacobian(x)
        return res, J, ctx.info()
    outs = run_ranks(nranks, mesh, par, fn)
    r = sum(o[0] for o in outs)
    J = sum(o[1] for o in outs)
    assert sum(o[2]["nv_owned"] for o in outs) == mesh.nv
    assert all(o[2]["nv_ghost"] > 0 for o in outs)
    ctx1 = P.Context(mesh, par)
    ctx1.set_operator(P.OP_PNP)
    r1, J1 = ctx1.residual(x), ctx1.jacobian(x)
    assert np.max(np.abs(r - r1)) <= 1e-13 * np.max(np.abs(r1))
    assert abs(J - J1).max() <= 1e-13 * abs(J1).max()


@pytest.mark.parametrize("nranks,prec", [(2, P.PREC_NONE), (2, P.PREC_SSOR), (4, P.PREC_SSOR),
                                         (2, P.PREC_ILU0), (4, P.PREC_ILU0)])
def test_linear_solve_partitioned(nranks, prec):
    z, mesh, par, orc = golden("pore_small_k0")
    x = z["newton_pnp_x0"]  # the first Newton system (see test_gpu.test_linear_solve_...)

    def fn(ctx, r):
        ctx.set_operator(P.OP_PNP)
        J = ctx.jacobian(x)
        rhs = ctx.sync_vector(ctx.residual(x))
        sol, res = ctx.linear_solve(rhs, prec=prec, reduction=1e-8, maxit=20000)
        return ctx.sync_vector(sol), res, J, rhs
    outs = run_ranks(nranks, mesh, par, fn)
    J = sum(o[2] for o in outs)
    rhs = outs[0][3]
    for sol, res, _, _ in outs:
        assert res["converged"] == 1, res
        assert np.linalg.norm(J @ sol - rhs) <= 1.001e-8 * np.linalg.norm(rhs)
    # every rank sees the same global scalars
    assert len({o[1]["iterations"] for o in outs}) == 1
    np.testing.assert_array_equal(outs[0][0], outs[-1][0])


@pytest.mark.parametrize("nranks,prec", [(2, P.PREC_SSOR), (4, P.PREC_SSOR), (4, P.PREC_ILU0)])
def test_newton_partitioned_matches_single_rank(nranks, prec):
    """(Jacobi is covered on the scalar PB system in test_pb_jacobi_partitioned.)"""
    z, mesh, par, orc = golden("pore_small_k0")

    def fn(ctx, r):
        ctx.set_operator(P.OP_PNP)
        u, res = ctx.newton(z["newton_pnp_x0"], prec=prec)
        return ctx.sync_vector(u), res
    outs = run_ranks(nranks, mesh, par, fn)
    ref = z["newton_pnp_u"]
    for u, res in outs:
        assert res["converged"] == 1 and res["status"] == 0, res
        assert np.max(np.abs(u - ref)) <= 1e-6 * np.max(np.abs(ref))


def test_pb_then_pnp_partitioned_on_refined_mesh():
    """The driver sequence (PB Newton -> BCExtension -> PNP Newton) on test/cylinder.msh refined
    once, 4 ranks vs 1 rank."""
    cfg = P.read_config(os.path.join(DATA, "cylinder_config.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(1)
    par = P.Params.from_config(cfg)

    def seq(ctx, r):
        ctx.set_operator(P.OP_PB)
        phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_SSOR)
        phi = ctx.sync_vector(phi, 1)
        x0 = ctx.initial_state(phi)
        ctx.set_operator(P.OP_PNP)
        u, res = ctx.newton(x0, prec=P.PREC_SSOR)
        return ctx.sync_vector(u), res, rpb
    outs = run_ranks(4, mesh, par, seq)
    ctx1 = P.Context(mesh, par)
    u1, res1, _ = seq(ctx1, 0)
    assert res1["converged"] == 1, res1
    for u, res, rpb in outs:
        assert rpb["converged"] == 1 and res["converged"] == 1, (rpb, res)
        assert np.max(np.abs(u - u1)) <= 1e-6 * np.max(np.abs(u1))


def test_pb_then_pnp_partitioned_on_refined_pore_ilu0():
    """The hard pore case (24.1 V, refined once) on 4 ranks with block-Jacobi ILU(0)."""
    cfg = P.read_config(os.path.join(DATA, "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(1)
    par = P.Params.from_config(cfg)

    def seq(ctx, r):
        ctx.set_operator(P.OP_PB)
        phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0)
        phi = ctx.sync_vector(phi, 1)
        x0 = ctx.initial_state(phi)
        ctx.set_operator(P.OP_PNP)
        u, res = ctx.newton(x0, prec=P.PREC_ILU0, reduction=1e-8)
        return ctx.sync_vector(u), res, rpb
    outs = run_ranks(4, mesh, par, seq)
    ctx1 = P.Context(mesh, par)
    u1, res1, _ = seq(ctx1, 0)
    assert res1["converged"] == 1, res1
    for u, res, rpb in outs:
        assert rpb["converged"] == 1 and res["converged"] == 1, (rpb, res)
        assert np.max(np.abs(u - u1)) <= 1e-5 * np.max(np.abs(u1))


def test_tiled_mesh_parity_single_and_partitioned():
    """bench.py's weak-scaling mesh (mirrored copies, so half the triangles are clockwise):
    residual and Jacobian vs the oracle on one rank, and the same on 2 ranks."""
    import importlib.util
    import meshio
    import oracle_py as O
    spec = importlib.util.spec_from_file_location(
        "bench", os.path.join(os.path.dirname(DATA), "bench.py"))
    B = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(B)
    cfg = P.read_config(os.path.join(DATA, "pore_pnp", "pore.cfg"))
    mesh = B.tile_mesh(P.Mesh.read_gmsh(cfg.meshfile), 2)
    par = P.Params.from_config(cfg)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    rng = np.random.default_rng(11)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ro = orc.residual(op, x)
    Jo = orc.jacobian(op, x)  # analytic
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    r1, J1 = ctx.residual(x), ctx.jacobian(x)
    assert np.max(np.abs(r1 - ro)) <= 1e-12 * np.max(np.abs(ro))
    assert abs(J1 - Jo).max() <= 1e-12 * abs(Jo).max()

    def fn(c, r):
        c.set_operator(P.OP_PNP)
        return c.residual(x), c.jacobian(x)
    outs = run_ranks(2, mesh, par, fn)
    assert np.max(np.abs(sum(o[0] for o in outs) - r1)) <= 1e-13 * np.max(np.abs(r1))
    assert abs(sum(o[1] for o in outs) - J1).max() <= 1e-13 * abs(J1).max()


@pytest.mark.parametrize("nranks", [2, 4])
def test_pb_jacobi_partitioned(nranks):
    """Jacobi BiCGSTAB on the PB system (first Newton step) on 2 and 4 ranks."""
    z, mesh, par, orc = golden("pore_small_k0")
    x = np.zeros(mesh.nv)

    def fn(ctx, r):
        ctx.set_operator(P.OP_PB)
        J = ctx.jacobian(x)
        rhs = ctx.sync_vector(ctx.residual(x), 1)
        sol, res = ctx.linear_solve(rhs, prec=P.PREC_JACOBI, reduction=1e-8, maxit=20000)
        return ctx.sync_vector(sol, 1), res, J, rhs
    outs = run_ranks(nranks, mesh, par, fn)
    J = sum(o[2] for o in outs)
    rhs = outs[0][3]
    for sol, res, _, _ in outs:
        assert res["converged"] == 1, res
        assert np.linalg.norm(J @ sol - rhs) <= 1.001e-8 * np.linalg.norm(rhs)


@pytest.mark.parametrize("nranks", [2, 4])
def test_ion_flux_partitioned(nranks):
    z, mesh, par, orc = golden("pore_small_k0")
    x = z["newton_pnp_u"]
    ipo, imo = orc.ion_flux(x)
    outs = run_ranks(nranks, mesh, par, lambda ctx, r: ctx.ion_flux(x))
    scale = max(np.max(np.abs(ipo)), np.max(np.abs(imo)))
    for ip, im in outs:
        assert np.max(np.abs(ip - ipo)) <= 1e-12 * scale
        assert np.max(np.abs(im - imo)) <= 1e-12 * scale


@pytest.mark.parametrize("nranks,kind", [(2, "pnp"), (3, "pb")])
def test_amg_solve_partitioned(nranks, kind):
    """PNP_PREC_AMG across ranks: each rank's hierarchy covers its owned rows (block-Jacobi of
    AMGs, like the sweeps); the outer Krylov solve is global and reaches the reduction."""
    z, mesh, par, orc = golden("pore_small_k0")
    x = z["newton_pnp_x0"] if kind == "pnp" else np.zeros(mesh.nv)
    op = P.OP_PNP if kind == "pnp" else P.OP_PB
    method = P.METHOD_BICGSTAB if kind == "pnp" else P.METHOD_CG

    def fn(ctx, r):
        ctx.set_operator(op)
        if kind == "pnp":
            ctx.amg_configure(smoother=P.PREC_ILU0, coarse_target=8)
        else:
            ctx.amg_configure(smoother=P.PREC_SSOR, coarse_target=8)
        J = ctx.jacobian(x)
        rhs = ctx.sync_vector(ctx.residual(x))
        sol, res = ctx.linear_solve(rhs, prec=P.PREC_AMG, reduction=1e-8, maxit=5000,
                                    method=method)
        return ctx.sync_vector(sol), res, J, rhs, ctx.amg_info()
    outs = run_ranks(nranks, mesh, par, fn)
    J = sum(o[2] for o in outs)
    rhs = outs[0][3]
    for sol, res, _, _, info in outs:
        assert res["converged"] == 1, res
        assert np.linalg.norm(J @ sol - rhs) <= 1.001e-8 * np.linalg.norm(rhs)
        assert info["levels"] >= 2
    assert len({o[1]["iterations"] for o in outs}) == 1
    assert sum(o[4]["rows"][0] for o in outs) == mesh.nv


def _config5_mesh(k=1):
    """BASELINE configs[4]'s geometry: test/pore_without_dna/pore_without_dna.geo meshed natively
    (scale 0.85, as bench.py's strong-scaling leg), refined k times."""
    cfg = P.read_config(os.path.join(DATA, "pore_without_dna", "pore.cfg"))
    return cfg, P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(k)


def test_config5_geometry_8_ranks_residual_jacobian():
    """8 in-process ranks (the north star's GPU count) on the config-5 geometry: residual and
    Jacobian (analytic and FD) = one rank's."""
    cfg, mesh = _config5_mesh(1)
    par = P.Params.from_config(cfg)
    rng = np.random.default_rng(8)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])

    def fn(ctx, r):
        ctx.set_operator(P.OP_PNP)
        return ctx.residual(x), ctx.jacobian(x), ctx.jacobian(x, fd=True), ctx.info()
    outs = run_ranks(8, mesh, par, fn)
    assert sum(o[3]["nv_owned"] for o in outs) == nv
    ctx1 = P.Context(mesh, par)
    ctx1.set_operator(P.OP_PNP)
    r1, J1, F1 = ctx1.residual(x), ctx1.jacobian(x), ctx1.jacobian(x, fd=True)
    assert np.max(np.abs(sum(o[0] for o in outs) - r1)) <= 1e-13 * np.max(np.abs(r1))
    assert abs(sum(o[1] for o in outs) - J1).max() <= 1e-13 * abs(J1).max()
    assert abs(sum(o[2] for o in outs) - F1).max() <= 1e-13 * abs(F1).max()


def test_config5_geometry_8_ranks_driver_sequence():
    """PB Newton -> BCExtension -> PNP Newton (the config's reductions, block-Jacobi ILU(0)) on 8
    in-process ranks vs one rank, config-5 geometry refined once."""
    cfg, mesh = _config5_mesh(1)
    par = P.Params.from_config(cfg)
    s = cfg.system

    def seq(ctx, r):
        ctx.set_operator(P.OP_PB)
        phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0, reduction=1e-10)
        phi = ctx.sync_vector(phi, 1)
        x0 = ctx.initial_state(phi)
        ctx.set_operator(P.OP_PNP)
        u, res = ctx.newton(x0, prec=P.PREC_ILU0, reduction=1e-10,
                            min_linear_reduction=s["newtonMinLinearReduction"])
        return ctx.sync_vector(u), res, rpb
    outs = run_ranks(8, mesh, par, seq)
    u1, res1, rpb1 = seq(P.Context(mesh, par), 0)
    assert res1["converged"] == 1 and rpb1["converged"] == 1
    for u, res, rpb in outs:
        assert rpb["converged"] == 1 and res["converged"] == 1, (rpb, res)
        assert np.max(np.abs(u - u1)) <= 1e-6 * np.max(np.abs(u1))


def test_implicit_euler_8_ranks():
    """Config 4's operator (PnpOperator + PnpTOperator, implicit Euler, dt = tau) for 3 steps on 8
    in-process ranks vs one rank, config-5 geometry refined once."""
    cfg, mesh = _config5_mesh(1)
    par = P.Params.from_config(cfg)
    dt = cfg.system["tau"]

    def steps(ctx, r):
        ctx.set_operator(P.OP_PB)
        phi, _ = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0, reduction=1e-10)
        x = ctx.initial_state(ctx.sync_vector(phi, 1))
        out = []
        for n in range(3):
            ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=x)
            # abs_limit above the residual's rounding floor (~1e-12 on this mesh)
            u, res = ctx.newton(x, prec=P.PREC_ILU0, reduction=1e-8, abs_limit=1e-10)
            assert res["converged"] == 1, res
            x = ctx.sync_vector(u)
            out.append(x)
        return out
    outs = run_ranks(8, mesh, par, steps)
    ref = steps(P.Context(mesh, par), 0)
    for traj in outs:
        for a, b in zip(traj, ref):
            assert np.max(np.abs(a - b)) <= 1e-6 * np.max(np.abs(b))


@pytest.mark.parametrize("nranks", [2, 4])
def test_parallel_dot_and_norm_equal_single_rank(nranks):
    """pnp_dot / pnp_norm (the NOVLP backend's norm behind Newton's defect, src/stationary_pnp_from_pb.hh:
    355-358): every rank reads only its owned entries and gets the global value, whatever its other
    entries hold -- here each rank's copy is garbage outside its owned rows."""
    z, mesh, par, orc = golden("pore_small_k0")
    nv = mesh.nv
    rng = np.random.default_rng(21)
    a, b = rng.standard_normal(3 * nv), rng.standard_normal(3 * nv)
    c1 = P.Context(mesh, par)
    d1, n1, s1 = c1.dot(a, b), c1.norm(a), c1.norm(a[:nv], nfields=1)
    assert abs(n1 - np.linalg.norm(a)) <= 1e-14 * n1 and abs(d1 - a @ b) <= 1e-13 * abs(a @ b)

    def fn(ctx, r):
        lay = P.Layout(mesh, r, nranks)
        own = np.zeros(nv, dtype=bool)
        own[lay.l2g[:lay.n_owned]] = True
        own3 = np.tile(own, 3)
        ga = np.where(own3, a, 1e30 * (r + 1))
        gb = np.where(own3, b, -7.0)
        return ctx.dot(ga, gb), ctx.norm(ga), ctx.norm(ga[:nv], nfields=1)
    for d, n, s in run_ranks(nranks, mesh, par, fn):
        assert abs(d - d1) <= 1e-14 * abs(d1) * 10 and abs(n - n1) <= 1e-14 * n1
        assert abs(s - s1) <= 1e-14 * s1


def _square():
    """4 vertices, 2 triangles: the smallest mesh a partition can split to one vertex per rank"""
    xy = np.array([[0.0, 1.0], [1.0, 1.0], [1.0, 2.0], [0.0, 2.0]])
    tri = np.array([[0, 1, 2], [0, 2, 3]], dtype=np.int32)
    bseg = np.array([[0, 1], [1, 2], [2, 3], [3, 0]], dtype=np.int32)
    bgroup = np.array([0, 1, 0, 1], dtype=np.int32)
    surf = [P.Surface(cb=1, cflux=0.3, cpot=0.0, pb=1, pflux=-0.2, pconc=0.0, mb=1, mflux=0.1,
                      mconc=0.0),
            P.Surface(cb=0, cflux=0.0, cpot=1.0, pb=0, pflux=0.0, pconc=0.05, mb=0, mflux=0.0,
                      mconc=0.07)]
    return P.Mesh(xy, tri, bseg, bgroup), P.Params(surf, l_b=0.7, c0=0.06, tau=1.0)


def test_one_vertex_per_rank_matches_single_rank():
    """the ragged extreme: as many ranks as vertices, every rank one owned row and the rest ghosts"""
    mesh, par = _square()
    rng = np.random.default_rng(4)
    x = np.concatenate([rng.uniform(-1, 1, 4), 0.06 * rng.uniform(0.5, 1.5, 8)])

    x0 = np.concatenate([np.zeros(4), np.full(8, 0.06)])

    def fn(ctx, r):
        ctx.set_operator(P.OP_PNP)
        out = ctx.residual(x), ctx.jacobian(x), ctx.info()["nv_owned"]
        u, res = ctx.newton(x0, prec=P.PREC_ILU0)
        return out + (ctx.sync_vector(u), res)
    outs = run_ranks(4, mesh, par, fn)
    assert [o[2] for o in outs] == [1, 1, 1, 1]
    ctx1 = P.Context(mesh, par)
    ctx1.set_operator(P.OP_PNP)
    r1, J1 = ctx1.residual(x), ctx1.jacobian(x)
    u1, res1 = ctx1.newton(x0, prec=P.PREC_ILU0)
    ctx1.close()
    assert np.max(np.abs(sum(o[0] for o in outs) - r1)) <= 1e-13 * np.max(np.abs(r1))
    assert abs(sum(o[1] for o in outs) - J1).max() <= 1e-13 * abs(J1).max()
    assert res1["converged"] == 1, res1
    for o in outs:  # block-Jacobi ILU(0) of one row per rank: the same Newton solution
        assert o[4]["converged"] == 1 and o[4]["status"] == 0, o[4]
        assert np.max(np.abs(o[3] - u1)) <= 1e-6 * np.max(np.abs(u1))


def test_more_ranks_than_vertices_fails_on_every_rank():
    """an empty part is refused by every rank before the group joins (no rank left waiting)"""
    mesh, par = _square()
    name = f"t{next(_grp)}"

    def work(r):
        try:
            P.Context(mesh, par, device=0, rank=r, size=6, local_group=name).close()
        except P.PnpError as e:
            return str(e)
        return None
    with ThreadPoolExecutor(6) as ex:
        errs = list(ex.map(work, range(6)))
    assert all(e and "owns no vertices" in e for e in errs), errs
