"""CPU tests: pin the C oracle (oracle/pnp_oracle.c) against the committed golden fixtures
(independent numpy restatement, tests/golden/make_golden.py) and against the reference's only
known-answer data (Gouy-Chapman, test/one_wall_dh/one_wall.gp:4-12)."""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import meshio
import oracle_py as O
from conftest import DATA

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KINDS = {"pnp": O.OP_PNP, "pnp_ie": O.OP_PNP_IE, "pb": O.OP_PB, "diff": O.OP_DIFF,
         "poisson": O.OP_POISSON}


def load(name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    m = meshio.Mesh(z["xy"], z["tri"].astype(np.int32), z["bseg"].astype(np.int32),
                    z["bgroup"].astype(np.int32))
    surfs = [meshio.Surface(int(s[0]), s[1], s[2], int(s[3]), s[4], s[5], int(s[6]), s[7], s[8])
             for s in z["surfaces"]]
    l_b, c0, tau, cyl, pi = z["params"]
    P = O.Problem(m, surfs, l_b=l_b, c0=c0, tau=tau, cylindrical=int(cyl), pi=pi)
    return z, m, P


def build_op(z, P, kind):
    flux = P.flux()
    mask = np.ascontiguousarray(z[kind + "_mask"])
    kw = {}
    if kind == "pnp_ie":
        kw = dict(dt=float(z["params"][2]), x_old=np.ascontiguousarray(z["pnp_ie_x_old"]))
    if kind == "diff":
        kw = dict(z=-1.0, phi=np.ascontiguousarray(z["diff_phi"]))
    if kind == "poisson":
        kw = dict(cp=np.ascontiguousarray(z["poisson_cp"]),
                  cm=np.ascontiguousarray(z["poisson_cm"]))
    return P.operator(KINDS[kind], flux=flux, mask=mask, **kw)


def csr(z, key):
    n = z[key + "_indptr"].shape[0] - 1
    return sp.csr_matrix((z[key + "_data"], z[key + "_indices"], z[key + "_indptr"]),
                         shape=(n, n))


CASES = [("cylinder_k0", "pnp"), ("cylinder_k0", "pb"), ("pore_small_k0", "pnp"),
         ("pore_small_k0", "pnp_ie"), ("pore_small_k0", "pb"), ("pore_small_k0", "diff"),
         ("pore_small_k0", "poisson"), ("pore_pnp_k0", "pnp"), ("pore_pnp_k0", "pb"),
         ("sphere_k0", "pb"), ("one_wall_k1", "pnp"), ("one_wall_k1", "pb")]


@pytest.mark.parametrize("name,kind", CASES)
def test_residual_matches_golden(name, kind):
    z, m, P = load(name)
    op = build_op(z, P, kind)
    r = P.residual(op, z[kind + "_x"])
    ref = z[kind + "_r"]
    # residual tolerance: ||dr||_inf / ||r||_inf <= 1e-12
    assert np.max(np.abs(r - ref)) <= 1e-12 * np.max(np.abs(ref))


@pytest.mark.parametrize("name,kind", [c for c in CASES if c[0] != "pore_pnp_k0"])
def test_jacobian_matches_golden(name, kind):
    z, m, P = load(name)
    op = build_op(z, P, kind)
    x = z[kind + "_x"]
    J = P.jacobian(op, x, fd=False)
    Jref = csr(z, kind + "_J")
    scale = abs(Jref).max()
    assert abs(J - Jref).max() <= 1e-12 * scale          # analytic vs analytic
    Jfd = P.jacobian(op, x, fd=True)
    Jfd_ref = csr(z, kind + "_Jfd")
    # two FD evaluations differ by rounding/eps: (eps_mach*|r|/delta)
    assert abs(Jfd - Jfd_ref).max() <= 1e-6 * scale
    # analytic vs reference-faithful FD: entrywise relative <= 1e-5 where |A_ij| > 1e-12 ||A||
    D = (J - Jfd).tocoo()
    Jd = J.tocsr()
    big = np.abs(np.asarray(Jd[D.row, D.col]).ravel()) > 1e-12 * scale
    rel = np.abs(D.data) / np.maximum(np.abs(np.asarray(Jd[D.row, D.col]).ravel()), 1e-300)
    assert np.all(rel[big] <= 1e-5) or np.max(np.abs(D.data)) <= 1e-5 * scale


def test_csr_pattern_is_full_volume_pattern():
    z, m, P = load("cylinder_k0")
    op = build_op(z, P, "pnp")
    J = P.jacobian(op, z["pnp_x"])
    # 9 * (V + 2E) entries: V + 2E = sum of (degree+1)
    edges = set()
    for t in m.tri:
        for a, b in ((0, 1), (1, 2), (0, 2)):
            edges.add(tuple(sorted((int(t[a]), int(t[b])))))
    assert J.nnz == 9 * (m.nv + 2 * len(edges))


@pytest.mark.parametrize("name", ["cylinder_k0", "pore_small_k0"])
def test_newton_pnp_matches_golden(name):
    z, m, P = load(name)
    mask = P.mask(3)
    np.testing.assert_array_equal(mask, z["pnp_mask"])
    op = P.operator(O.OP_PNP, flux=P.flux(), mask=mask)
    u, res = P.newton(op, z["newton_pnp_x0"], prec=O.PREC_ILU0)
    assert res.converged == 1 and res.status == 0
    ref = z["newton_pnp_u"]
    assert np.max(np.abs(u - ref)) <= 1e-6 * np.max(np.abs(ref))
    assert res.defect <= 1e-9 * res.first_defect or res.defect < 1e-12


@pytest.mark.parametrize("name", ["pore_small_k0", "sphere_k0", "one_wall_k1"])
def test_newton_pb_matches_golden(name):
    z, m, P = load(name)
    op = P.operator(O.OP_PB, flux=P.flux(), mask=P.mask(1))
    u, res = P.newton(op, np.zeros(m.nv), prec=O.PREC_ILU0)
    assert res.converged == 1
    ref = z["newton_pb_u"]
    assert np.max(np.abs(u - ref)) <= 1e-6 * max(np.max(np.abs(ref)), 1e-12)


def test_bicgstab_preconditioners_agree():
    z, m, P = load("pore_small_k0")
    op = build_op(z, P, "pnp")
    J = P.jacobian(op, z["pnp_x"])
    b = np.ones(J.shape[0])
    sols = {}
    for prec in (O.PREC_ILU0, O.PREC_SSOR, O.PREC_JACOBI):
        x, res = O.bicgstab(J, b, prec=prec, reduction=1e-12)
        assert res.converged
        assert np.linalg.norm(J @ x - b) <= 1e-10 * np.linalg.norm(b)
        sols[prec] = x
    # ISTL counts half steps: iterations = ceil(it)
    x, res = O.bicgstab(J, b, prec=O.PREC_ILU0, reduction=1e-12)
    assert res.iterations == int(np.ceil(res.it_half))


@pytest.mark.parametrize("prec", [O.PREC_ILU0, O.PREC_SSOR])
def test_block_jacobi_preconditioner_is_the_block_diagonal_one(prec):
    """orc_set_block_jacobi (the CPU baseline's all-core SSOR / ILU(0): the NOVLP backend's
    per-rank SeqSSOR / SeqILU0 on nblocks vertex ranges) equals the sequential preconditioner of
    the block-diagonal matrix bit for bit, and BiCGSTAB with it converges to the same solution."""
    z, m, P = load("pore_small_k0")
    op = build_op(z, P, "pnp")
    J = P.jacobian(op, z["pnp_x"]).tocsr()
    nv, nb = m.nv, 5
    blk = (np.arange(J.shape[0]) % nv) * nb // nv
    C = J.tocoo()
    keep = blk[C.row] == blk[C.col]
    Jbd = sp.csr_matrix((C.data[keep], (C.row[keep], C.col[keep])), shape=J.shape)
    d = np.random.default_rng(3).uniform(-1, 1, J.shape[0])
    ref = O.prec_apply(Jbd, d, prec)
    O.lib().orc_set_block_jacobi(nb, 3)
    try:
        got = O.prec_apply(J, d, prec)
        b = np.ones(J.shape[0])
        x, res = O.bicgstab(J, b, prec=prec, reduction=1e-12)
    finally:
        O.lib().orc_set_block_jacobi(0, 1)
    np.testing.assert_array_equal(got, ref)
    assert not np.array_equal(got, O.prec_apply(J, d, prec))  # the couplings were dropped
    assert res.converged and np.linalg.norm(J @ x - b) <= 1e-10 * np.linalg.norm(b)
    assert res.setup_seconds >= 0 and res.iter_seconds > 0


def test_bicgstab_trivial_rhs_returns_immediately():
    A = sp.identity(10, format="csr")
    x, res = O.bicgstab(A, np.zeros(10))
    assert res.converged and res.iterations == 0


def test_pnp_nonprec_hits_maxit_like_reference():
    """Stationary PNP with NOPREC (src/stationary_pnp_from_pb.hh:329-331) on the cylindrical
    pore mesh does not converge within a small iteration cap; Newton reports the linear-solver
    failure (PDELab NewtonLinearSolverError), exactly the status the product must report."""
    z, m, P = load("pore_pnp_k0")
    op = P.operator(O.OP_PNP, flux=P.flux(), mask=P.mask(3))
    _, res = P.newton(op, z["pnp_x"], prec=O.PREC_NONE, linear_maxit=50)
    assert res.status == -3


def test_gouy_chapman_known_answer():
    """Planar PB against the reference's analytic curve family (test/one_wall_dh/one_wall.gp:
    4-12, Gouy-Chapman): -phi'' + kappa^2 sinh(phi) = 0, phi'(0) = j, phi(L) = 0.  The 1-D
    solution is computed to high accuracy with scipy.solve_bvp on the same finite slab; the
    semi-infinite Gouy-Chapman closed form is checked against it as well."""
    from scipy.integrate import solve_bvp
    cfg = meshio.read_config(os.path.join(DATA, "one_wall_dh", "one_wall.cfg"))
    m = meshio.refine(meshio.read_gmsh(cfg.meshfile), 3)
    s = cfg.system
    P = O.Problem(m, cfg.surfaces, l_b=s["l_b"], c0=s["c0"], tau=s["tau"],
                  cylindrical=int(s["cylindrical"]))
    op = P.operator(O.OP_PB, flux=P.flux(), mask=P.mask(1))
    u, res = P.newton(op, np.zeros(m.nv), prec=O.PREC_ILU0, reduction=1e-12)
    assert res.converged
    k2 = 8 * 3.1415 * s["l_b"] * s["c0"]
    j = cfg.surfaces[0].cflux
    L = m.xy[:, 0].max()
    sol = solve_bvp(lambda x, y: np.vstack([y[1], k2 * np.sinh(y[0])]),
                    lambda ya, yb: np.array([ya[1] - j, yb[0]]),
                    np.linspace(0, L, 200), np.zeros((2, 200)), tol=1e-10, max_nodes=100000)
    assert sol.success
    exact = sol.sol(m.xy[:, 0])[0]
    err = np.max(np.abs(u - exact))
    assert err <= 2e-3 * np.max(np.abs(exact))
    # semi-infinite Gouy-Chapman closed form (one_wall.gp:9-10) near the wall
    kappa = np.sqrt(k2)
    phi0 = -2 * np.arcsinh(j / (2 * kappa))
    g = np.tanh(phi0 / 4)
    xs = np.linspace(0, 2, 5)
    gc = 2 * np.log((1 + g * np.exp(-kappa * xs)) / (1 - g * np.exp(-kappa * xs)))
    assert np.max(np.abs(gc - sol.sol(xs)[0])) <= 0.02 * abs(phi0)


def test_initial_state_dirichlet_values():
    """BCExtension (src/dirichlet_bc.hh:54-123) puts the configured Dirichlet values on the
    constrained vertices it finds, and the Boltzmann extension elsewhere."""
    cfg = meshio.read_config(os.path.join(DATA, "pore_pnp", "pore.cfg"))
    m = meshio.read_gmsh(cfg.meshfile)
    s = cfg.system
    P = O.Problem(m, cfg.surfaces, l_b=s["l_b"], c0=s["c0"], tau=s["tau"],
                  cylindrical=int(s["cylindrical"]))
    rng = np.random.default_rng(1)
    phi = rng.uniform(-0.5, 0.5, m.nv)
    x0 = P.initial_state(phi)
    mask = P.mask(3)
    outflow = m.bseg[m.bgroup == 4].ravel()
    assert np.all(x0[outflow] == 24.1)
    free = mask[:m.nv] == 0
    np.testing.assert_allclose(x0[m.nv:2 * m.nv][free], 0.06 * np.exp(-phi[free]), rtol=1e-15)
    np.testing.assert_allclose(x0[2 * m.nv:][free], 0.06 * np.exp(phi[free]), rtol=1e-15)


def _ion_flux_numpy(mesh, surfaces, x, cylindrical, pi=3.1415):
    """Independent restatement of calcIonFlux (src/ionFlux.hh:8-96), per boundary segment:
    the segment's element, fields at the segment midpoint, outward unit normal."""
    nv = mesh.xy.shape[0]
    tri = mesh.tri
    owner = {}
    for e, t in enumerate(tri):
        for a, b in ((t[0], t[1]), (t[0], t[2]), (t[1], t[2])):
            owner.setdefault((min(a, b), max(a, b)), []).append(e)
    ip = np.zeros(len(surfaces))
    im = np.zeros(len(surfaces))
    for b, (a, c) in enumerate(mesh.bseg):
        e = owner[(min(a, c), max(a, c))][0]
        t = tri[e]
        P = mesh.xy[t]
        J = np.array([P[1] - P[0], P[2] - P[0]]).T
        G = np.linalg.solve(J.T, np.array([[-1.0, 1.0, 0.0], [-1.0, 0.0, 1.0]]))  # 2 x 3
        gphi, gcp, gcm = (G @ x[k * nv + t] for k in range(3))
        o = [v for v in t if v != a and v != c][0]
        pa, pc, po = mesh.xy[a], mesh.xy[c], mesh.xy[o]
        mid = 0.5 * (pa + pc)
        cp = 0.5 * (x[nv + a] + x[nv + c])
        cm = 0.5 * (x[2 * nv + a] + x[2 * nv + c])
        tvec = pc - pa
        ln = np.hypot(*tvec)
        fac = ln * (2 * pi * mid[1] if cylindrical else 1.0)
        n = np.array([tvec[1], -tvec[0]]) / ln
        if n @ (po - pa) > 0:
            n = -n
        g = mesh.bgroup[b]
        ip[g] += fac * (-gcp + cp * gphi) @ n
        im[g] += fac * (-gcm - cm * gphi) @ n
    return ip, im


@pytest.mark.parametrize("name", ["cylinder_k0", "pore_small_k0", "one_wall_k1"])
def test_ion_flux_matches_numpy_restatement(name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    mesh = meshio.Mesh(z["xy"], z["tri"], z["bseg"], z["bgroup"])
    surfs = [meshio.Surface(int(s[0]), s[1], s[2], int(s[3]), s[4], s[5], int(s[6]), s[7], s[8])
             for s in z["surfaces"]]
    l_b, c0, tau, cyl, pi = z["params"]
    orc = O.Problem(mesh, surfs, l_b=l_b, c0=c0, tau=tau, cylindrical=int(cyl), pi=pi)
    x = z["newton_pnp_u"] if "newton_pnp_u" in z.files else z["pnp_x"]
    ip, im = orc.ion_flux(x)
    ipn, imn = _ion_flux_numpy(mesh, surfs, x, int(cyl), pi)
    scale = max(np.max(np.abs(ipn)), np.max(np.abs(imn)))
    assert scale > 0
    np.testing.assert_allclose(ip, ipn, rtol=0, atol=1e-12 * scale)
    np.testing.assert_allclose(im, imn, rtol=0, atol=1e-12 * scale)


def test_cg_oracle_solves_pb_system_and_counts_matvecs():
    """orc_cg (ISTL CGSolver semantics) on the PB Jacobian at phi = 0: converges, the solution
    satisfies the system, and CG_NOPREC / CG_Jacobi agree with a numpy CG restatement on the
    iteration count (matrix-vector products)."""
    z = np.load(os.path.join(GOLD, "pore_small_k0.npz"))
    mesh = meshio.Mesh(z["xy"], z["tri"], z["bseg"], z["bgroup"])
    surfs = [meshio.Surface(int(s[0]), s[1], s[2], int(s[3]), s[4], s[5], int(s[6]), s[7], s[8])
             for s in z["surfaces"]]
    l_b, c0, tau, cyl, pi = z["params"]
    orc = O.Problem(mesh, surfs, l_b=l_b, c0=c0, tau=tau, cylindrical=int(cyl), pi=pi)
    op = orc.operator(O.OP_PB, flux=orc.flux(), mask=orc.mask(1))
    x = np.zeros(mesh.xy.shape[0])
    J = orc.jacobian(op, x).tocsr()
    b = orc.residual(op, x)
    for prec in (O.PREC_NONE, O.PREC_JACOBI):
        sol, res = O.cg(J, b, prec=prec, reduction=1e-10, maxit=5000)
        assert res.converged
        assert np.linalg.norm(J @ sol - b) <= 1.001e-10 * np.linalg.norm(b)
        Dinv = 1 / J.diagonal() if prec == O.PREC_JACOBI else np.ones_like(b)
        r = b.copy()
        p = Dinv * r
        rho = p @ r
        d0 = np.linalg.norm(r)
        for it in range(1, 5001):
            q = J @ p
            lam = rho / (p @ q)
            r -= lam * q
            if np.linalg.norm(r) < 1e-10 * d0:
                break
            q = Dinv * r
            rho_new = q @ r
            p = q + rho_new / rho * p
            rho = rho_new
        assert res.iterations == it


def test_multicolour_ssor_diverges_where_natural_order_converges():
    """Why the GPU test on config 5's geometry uses ILU(0): on the first PNP Newton system of
    test/pore_without_dna (meshed natively, refined once) ISTL SSOR(k=1, w=1) in the file's
    vertex order converges, but the same SSOR in the multicolour vertex-blocked order the GPU
    sweeps use (pnp_layout: colour-major, fields inside a vertex) does not converge in 2000
    iterations (it diverges or stalls, depending on the colouring) -- Gauss-Seidel on a
    drift-dominated non-symmetric system depends on the order.  ILU(0) in that order converges
    with ~25 % more iterations than in the natural order.  All on the oracle (CPU)."""
    import pnp_amd as P
    cfg = P.read_config(os.path.join(DATA, "pore_without_dna", "pore.cfg"))
    mesh = P.Mesh.load(cfg.meshfile).refine(1)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    x0 = orc.initial_state(np.zeros(mesh.nv))
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    r = orc.residual(op, x0)
    J = orc.jacobian(op, x0).tocsr()
    lay = P.Layout(mesh)
    nv = mesh.nv
    perm = np.array([f * nv + lay.l2g[q] for q in range(nv) for f in range(3)])
    Jp = J[perm][:, perm]
    _, nat = O.bicgstab(J, r, prec=O.PREC_SSOR, reduction=1e-8)
    _, mc = O.bicgstab(Jp, r[perm], prec=O.PREC_SSOR, reduction=1e-8, maxit=2000)
    _, ilu_nat = O.bicgstab(J, r, prec=O.PREC_ILU0, reduction=1e-8)
    _, ilu_mc = O.bicgstab(Jp, r[perm], prec=O.PREC_ILU0, reduction=1e-8)
    assert nat.converged == 1
    assert mc.converged == 0 and mc.reduction > 1e-3
    assert ilu_nat.converged == 1 and ilu_mc.converged == 1
    assert ilu_mc.iterations < 1.5 * ilu_nat.iterations


@pytest.mark.parametrize("kind", ["pnp", "pb"])
def test_all_core_assembly_matches_serial(kind):
    """The all-core CPU baseline (orc_assemble_mt, element colours + OpenMP) assembles the same
    residual and forward-difference Jacobian as the serial reference-faithful path."""
    z, m, P = load("pore_small_k0")
    op = build_op(z, P, kind)
    x = z[kind + "_x"]
    _, threads, A, r = P.time_fd_assembly_mt(op, x, 0.0)
    assert threads >= 1
    r1 = P.residual(op, x)
    J1 = P.jacobian(op, x, fd=True)
    np.testing.assert_allclose(r, r1, rtol=0, atol=1e-12 * np.max(np.abs(r1)))
    assert abs(A - J1).max() <= 1e-12 * abs(J1).max()


@pytest.mark.parametrize("order,npts", [(2, 3), (3, 4), (5, 7)])
def test_quadrature_rules_are_exact_to_their_order(order, npts):
    """The simplex rules the oracle (and, through the 1e-12 parity tests, the kernels) use for the
    reference's intorders: each integrates every monomial xi^a eta^b with a + b <= order exactly
    over the reference triangle (a! b! / (a + b + 2)!) and some monomial of degree order + 1 not
    (the rule is of that order, no more).  Which order-2 / order-3 point set dune-geometry's
    SimplexQuadraturePoints<2> picks is not pinned by any reference fixture: PNP
    and Poisson integrands are polynomials the rule integrates exactly, so they do not depend on
    it; PB's sinh and the cylindrical PnpT mass do, at the rule's truncation error."""
    from math import factorial
    xi, eta, w = O.quadrature_rule(order)
    assert len(w) == npts
    assert abs(w.sum() - 0.5) <= 1e-15
    assert np.all((xi > 0) & (eta > 0) & (xi + eta < 1))  # interior points
    for deg in range(order + 2):
        errs = [abs(np.sum(w * xi ** a * eta ** (deg - a)) -
                    factorial(a) * factorial(deg - a) / factorial(deg + 2)) for a in range(deg + 1)]
        if deg <= order:
            assert max(errs) <= 1e-15, (deg, errs)
        else:
            assert max(errs) > 1e-6, (deg, errs)
