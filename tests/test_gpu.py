"""GPU parity tests (-m gpu): the HIP path through the C ABI against the CPU oracle and the
committed golden fixtures.  Tolerances:
  residual                      ||dr||_inf <= 1e-12 ||r||_inf
  Jacobian vs analytic oracle   |dJ|       <= 1e-12 max|J|
  Jacobian vs FD oracle         rel        <= 1e-5 (reference-faithful forward differences)
  converged Newton solution     ||du||_inf <= 1e-6 ||u||_inf, and both reach the reduction
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

import meshio
import oracle_py as O
import pnp_amd as P
from conftest import DATA

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

KIND_P = {"pnp": P.OP_PNP, "pnp_ie": P.OP_PNP_IMPLICIT_EULER, "pb": P.OP_PB,
          "diff": P.OP_DIFF, "poisson": P.OP_POISSON}
KIND_O = {"pnp": O.OP_PNP, "pnp_ie": O.OP_PNP_IE, "pb": O.OP_PB, "diff": O.OP_DIFF,
          "poisson": O.OP_POISSON}


def golden(name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    mesh = P.Mesh(z["xy"], z["tri"], z["bseg"], z["bgroup"])
    surfs = [P.Surface(int(s[0]), s[1], s[2], int(s[3]), s[4], s[5], int(s[6]), s[7], s[8])
             for s in z["surfaces"]]
    l_b, c0, tau, cyl, pi = z["params"]
    par = P.Params(surfs, l_b=l_b, c0=c0, tau=tau, cylindrical=int(cyl), pi=pi)
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup),
                    [meshio.Surface(*[getattr(s, f) for f in ("cb", "cflux", "cpot", "pb",
                                                               "pflux", "pconc", "mb", "mflux",
                                                               "mconc")]) for s in surfs],
                    l_b=l_b, c0=c0, tau=tau, cylindrical=int(cyl), pi=pi)
    return z, mesh, par, orc


def set_ops(z, ctx, orc, kind):
    kw_p, kw_o = {}, {}
    if kind == "pnp_ie":
        kw_p = dict(dt=float(z["params"][2]), x_old=z["pnp_ie_x_old"])
        kw_o = dict(dt=float(z["params"][2]), x_old=np.ascontiguousarray(z["pnp_ie_x_old"]))
    if kind == "diff":
        kw_p = dict(z=-1.0, field=2, phi=z["diff_phi"])
        kw_o = dict(z=-1.0, phi=np.ascontiguousarray(z["diff_phi"]))
    if kind == "poisson":
        kw_p = dict(cp=z["poisson_cp"], cm=z["poisson_cm"])
        kw_o = dict(cp=np.ascontiguousarray(z["poisson_cp"]),
                    cm=np.ascontiguousarray(z["poisson_cm"]))
    ctx.set_operator(KIND_P[kind], **kw_p)
    nf = 3 if kind.startswith("pnp") else 1
    if kind == "diff":
        mask = orc.mask(3)[2 * z["xy"].shape[0]:].copy()
    else:
        mask = orc.mask(nf)
    op = orc.operator(KIND_O[kind], flux=orc.flux(), mask=np.ascontiguousarray(mask), **kw_o)
    return op


CASES = [("cylinder_k0", "pnp"), ("cylinder_k0", "pb"), ("pore_small_k0", "pnp"),
         ("pore_small_k0", "pnp_ie"), ("pore_small_k0", "pb"), ("pore_small_k0", "diff"),
         ("pore_small_k0", "poisson"), ("pore_pnp_k0", "pnp"), ("pore_pnp_k0", "pb"),
         ("sphere_k0", "pb"), ("one_wall_k1", "pnp"), ("one_wall_k1", "pb")]


@pytest.mark.parametrize("name,kind", CASES)
def test_residual_parity(name, kind):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    op = set_ops(z, ctx, orc, kind)
    x = z[kind + "_x"]
    r = ctx.residual(x)
    ro = orc.residual(op, x)
    scale = np.max(np.abs(ro))
    assert np.max(np.abs(r - ro)) <= 1e-12 * scale
    assert np.max(np.abs(r - z[kind + "_r"])) <= 1e-12 * scale


@pytest.mark.parametrize("name,kind", [c for c in CASES if c[0] != "pore_pnp_k0"])
def test_jacobian_parity(name, kind):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    op = set_ops(z, ctx, orc, kind)
    x = z[kind + "_x"]
    J = ctx.jacobian(x)
    Jo = orc.jacobian(op, x, fd=False)
    scale = abs(Jo).max()
    assert abs(J - Jo).max() <= 1e-12 * scale
    Jfd = orc.jacobian(op, x, fd=True)
    D = (J - Jfd).tocoo()
    assert np.max(np.abs(D.data)) <= 1e-5 * scale
    # constrained rows are identity rows
    mask = op._keep[1] if len(op._keep) > 1 else None
    Jc = J.tocsr()
    nf = 3 if kind.startswith("pnp") else 1
    m = (orc.mask(nf) if kind != "diff" else orc.mask(3)[2 * mesh.nv:])
    for i in np.nonzero(m)[0][:50]:
        row = Jc.getrow(i)
        assert row.nnz >= 1 and np.isclose(row[0, i], 1.0)
        assert np.allclose(np.delete(row.toarray()[0], i), 0.0)


def test_residual_parity_full_size():
    """Config-3 mesh (test/pore_pnp/pore.msh refined k=4, 2.2 M DOF): residual vs the oracle."""
    cfg = P.read_config(os.path.join(DATA, "pore_pnp/pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    par = P.Params.from_config(cfg)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup),
                    [meshio.Surface(*[getattr(q, f) for f in ("cb", "cflux", "cpot", "pb",
                                                               "pflux", "pconc", "mb", "mflux",
                                                               "mconc")]) for q in cfg.surfaces],
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    rng = np.random.default_rng(20261015)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    r = ctx.residual(x)
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    ro = orc.residual(op, x)
    assert np.max(np.abs(r - ro)) <= 1e-12 * np.max(np.abs(ro))
    # size-independent property: the Jacobian applied to a direction equals the directional
    # derivative of the (bilinear) residual: R(x + d) - R(x) = J d + O(d^2) (exact for R
    # quadratic: R(x+d) + R(x-d) - 2R(x) = 2 Q(d))
    J = ctx.jacobian(x)
    d = 1e-3 * rng.standard_normal(3 * nv)
    d[op._keep[1] == 1] = 0.0
    rp, rm = ctx.residual(x + d), ctx.residual(x - d)
    lhs = 0.5 * (rp - rm)
    assert np.max(np.abs(lhs - J @ d)) <= 1e-9 * np.max(np.abs(J @ d))


def test_jacobian_parity_full_size():
    """Config-3 mesh (2.2 M DOF, 36 M stored nonzeros): the GPU's analytic Jacobian entry by entry
    against the oracle's analytic Jacobian, 1e-12 of max|J|."""
    cfg = P.read_config(os.path.join(DATA, "pore_pnp/pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    par = P.Params.from_config(cfg)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    rng = np.random.default_rng(20261015)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    J = ctx.jacobian(x)
    ctx.close()
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    Jo = orc.jacobian(op, x)
    assert abs(J - Jo).max() <= 1e-12 * abs(Jo).max()


def test_residual_and_jacobian_parity_config5():
    """Config 5 (test/pore_without_dna's .geo meshed natively, scale 0.85, refined k=6: 8.87 M DOF,
    the north star's system): residual and analytic Jacobian entry by entry vs the oracle, 1e-12
    of max|r| and of max|J|."""
    cfg = P.read_config(os.path.join(DATA, "pore_without_dna", "pore.cfg"))
    mesh = P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(6)
    par = P.Params.from_config(cfg)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    rng = np.random.default_rng(5)
    nv = mesh.nv
    assert 3 * nv > 8_000_000
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    r = ctx.residual(x)
    J = ctx.jacobian(x)
    ctx.close()
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    ro = orc.residual(op, x)
    assert np.max(np.abs(r - ro)) <= 1e-12 * np.max(np.abs(ro))
    Jo = orc.jacobian(op, x)
    assert J.shape == Jo.shape == (3 * nv, 3 * nv)
    assert abs(J - Jo).max() <= 1e-12 * abs(Jo).max()


@pytest.mark.parametrize("kind,prec", [("pnp", P.PREC_NONE), ("pnp", P.PREC_SSOR),
                                       ("pnp", P.PREC_ILU0), ("pb", P.PREC_JACOBI),
                                       ("pb", P.PREC_SSOR), ("pb", P.PREC_ILU0)])
def test_linear_solve_reduces_residual(kind, prec):
    """The first Newton system of the golden run (PNP: Jacobian and residual at the Boltzmann
    initial state; PB: at phi = 0).  BiCGSTAB's iterates depend on summation order, so a case
    is used only where the ISTL recurrence converges robustly: PNP with NONE converged 8/8
    under 1e-14 perturbations of the right-hand side (numpy restatement of the recurrence), the
    preconditioned cases converge in tens of iterations.  Jacobi is tested on the scalar PB
    system: on the PNP system it converged 8/8 in one summation order and broke down (exact-zero
    rho, ISTL's 1e-80 test) after a row reordering - a property of the method on that system."""
    z, mesh, par, orc = golden("pore_small_k0")
    ctx = P.Context(mesh, par)
    op = set_ops(z, ctx, orc, kind)
    x = z["newton_pnp_x0"] if kind == "pnp" else np.zeros(mesh.nv)
    J = ctx.jacobian(x)
    rhs = ctx.residual(x)
    sol, res = ctx.linear_solve(rhs, prec=prec, reduction=1e-8, maxit=20000)
    assert res["converged"] == 1, res
    assert np.linalg.norm(J @ sol - rhs) <= 1.001e-8 * np.linalg.norm(rhs)
    assert res["iterations"] == int(np.ceil(res["it_half"]))
    # same system through the oracle's ISTL BiCGSTAB
    xo, ro = O.bicgstab(orc.jacobian(op, x), rhs, prec=O.PREC_ILU0, reduction=1e-12, maxit=20000)
    assert ro.converged
    assert np.max(np.abs(sol - xo)) <= 1e-5 * np.max(np.abs(xo))


def test_bicgstab_nonprec_matches_oracle_on_long_run():
    """NOPREC over ~200 iterations: the Krylov iterates depend on summation order (the product
    sums dots in a different order and DOF layout than the oracle), so iteration counts agree
    only statistically; the converged solutions agree."""
    z, mesh, par, orc = golden("cylinder_k0")
    ctx = P.Context(mesh, par)
    op = set_ops(z, ctx, orc, "pnp")
    x = z["pnp_x"]
    J = ctx.jacobian(x)
    rhs = ctx.residual(x)
    sol, res = ctx.linear_solve(rhs, prec=P.PREC_NONE, reduction=1e-8, maxit=20000,
                                check_every=1)
    xo, ro = O.bicgstab(orc.jacobian(op, x), rhs, prec=O.PREC_NONE, reduction=1e-8, maxit=20000)
    assert ro.converged and res["converged"]
    # the oracle itself needs 697..1282 iterations on this system under 1e-14 perturbations of
    # the right-hand side: only convergence and the solution are comparable
    assert np.linalg.norm(J @ sol - rhs) <= 1.001e-8 * np.linalg.norm(rhs)
    assert np.max(np.abs(sol - xo)) <= 1e-5 * np.max(np.abs(xo))


@pytest.mark.parametrize("reduction", [1e-3, 1e-6, 1e-9])
def test_bicgstab_half_step_counting_matches_istl(reduction):
    """Well-conditioned system (implicit-Euler diffusion with a small step: mass dominated), few
    iterations, so rounding cannot move the stopping point: the ISTL half-step counter, the
    iteration count and the convergence flag match the oracle exactly."""
    z, mesh, par, orc = golden("pore_small_k0")
    nv = mesh.nv
    phi = np.ascontiguousarray(z["diff_phi"])
    xo_ = np.ascontiguousarray(z["pnp_ie_x_old"][nv:2 * nv])
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_DIFF_IMPLICIT_EULER, dt=1e-3, z=1.0, field=1, phi=phi, x_old=xo_)
    op = orc.operator(O.OP_DIFF_IE, flux=orc.flux(), mask=np.ascontiguousarray(orc.mask(3)[nv:2 * nv]),
                      dt=1e-3, z=1.0, phi=phi, x_old=xo_)
    x = xo_.copy()
    J = ctx.jacobian(x)
    rhs = ctx.residual(x) + 0.01
    rhs[op._keep[1] == 1] = 0.0
    sol, res = ctx.linear_solve(rhs, prec=P.PREC_NONE, reduction=reduction, maxit=1000,
                                check_every=1)
    xo, ro = O.bicgstab(orc.jacobian(op, x), rhs, prec=O.PREC_NONE, reduction=reduction,
                        maxit=1000)
    assert res["converged"] == ro.converged == 1
    assert res["it_half"] == ro.it_half
    assert res["iterations"] == ro.iterations
    assert np.max(np.abs(sol - xo)) <= 1e-9 * np.max(np.abs(xo))


# NOPREC inside Newton (the reference's stationary setting) is not asserted to converge: past
# the first step its BiCGSTAB runs hit rounding-noise breakdowns in some realisations (the GPU
# and the oracle differ only in summation order); the first-step NOPREC solve is tested above,
# and failure reporting in test_nonprec_stationary_pnp_reports_linear_failure.
@pytest.mark.parametrize("name,prec", [("cylinder_k0", P.PREC_SSOR), ("pore_small_k0", P.PREC_SSOR),
                                       ("cylinder_k0", P.PREC_ILU0), ("pore_small_k0", P.PREC_ILU0)])
def test_newton_pnp_matches_golden(name, prec):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    u, res = ctx.newton(z["newton_pnp_x0"], prec=prec, linear_maxit=20000)
    assert res["status"] == 0 and res["converged"] == 1, res
    ref = z["newton_pnp_u"]
    assert np.max(np.abs(u - ref)) <= 1e-6 * np.max(np.abs(ref))
    assert res["defect"] <= 1e-9 * res["first_defect"]


@pytest.mark.parametrize("name", ["pore_small_k0", "sphere_k0", "one_wall_k1"])
def test_newton_pb_matches_golden(name):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PB)
    u, res = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_SSOR)
    assert res["converged"] == 1, res
    ref = z["newton_pb_u"]
    assert np.max(np.abs(u - ref)) <= 1e-6 * max(np.max(np.abs(ref)), 1e-12)


def test_implicit_euler_step_matches_oracle():
    """One implicit-Euler step of PnpOperator + PnpTOperator (config 4 semantics)."""
    z, mesh, par, orc = golden("pore_small_k0")
    x_old = z["newton_pnp_x0"]
    dt = 1.0
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=dt, x_old=x_old)
    u, res = ctx.newton(x_old, prec=P.PREC_SSOR, reduction=1e-10)
    assert res["converged"] == 1, res
    op = orc.operator(O.OP_PNP_IE, flux=orc.flux(), mask=orc.mask(3), dt=dt,
                      x_old=np.ascontiguousarray(x_old))
    uo, ro = orc.newton(op, x_old, prec=O.PREC_ILU0, reduction=1e-10)
    assert ro.converged
    assert np.max(np.abs(u - uo)) <= 1e-6 * np.max(np.abs(uo))


def test_nonprec_stationary_pnp_reports_linear_failure():
    """Like the reference (NOPREC BiCGSTAB inside Newton, src/stationary_pnp_from_pb.hh:329-369)
    the product reports the linear solver's failure instead of returning garbage."""
    z, mesh, par, orc = golden("pore_pnp_k0")
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    u, res = ctx.newton(z["pnp_x"], prec=P.PREC_NONE, linear_maxit=50)
    assert res["status"] == P.E_NOT_CONVERGED and res["converged"] == 0


def test_bench_path_fixed_iterations():
    z, mesh, par, orc = golden("pore_pnp_k0")
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    ctx.state_set(z["pnp_x"])
    ctx.timers(enable=True, reset=True)
    ctx.assemble_state(3)
    res = ctx.bicgstab_iterations(10, P.PREC_SSOR)
    t = ctx.timers()
    assert res["iterations"] == 10
    assert t["assemble_launches"] == 3 and t["assemble_ms"] > 0
    assert np.isfinite(res["defect"]) and res["defect"] < res["defect0"]
    info = ctx.info()
    assert info["nblocks"] == info["nv_owned"] + 2 * len(
        set(map(tuple, np.sort(np.concatenate([mesh.tri[:, [0, 1]], mesh.tri[:, [1, 2]],
                                               mesh.tri[:, [0, 2]]]), axis=1).tolist())))


def test_cpp_driver_matches_python_api(tmp_path):
    """The C++ driver (PB Newton -> BCExtension -> PNP Newton, like src/stationary_pnp_from_pb.hh)
    reproduces the same solve through the Python mirror of the C ABI."""
    import subprocess
    exe = os.path.join(os.path.dirname(P.LIB_PATH), "pnp_main")
    cfgp = os.path.join(DATA, "cylinder_config.cfg")
    out = subprocess.run([exe, cfgp, "--prec", "ssor", "--out", str(tmp_path / "cyl")],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    u_drv = np.loadtxt(tmp_path / "cyl_pnp.dat").T.ravel()
    cfg = P.read_config(cfgp)
    mesh = P.Mesh.read_gmsh(cfg.meshfile)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    s = cfg.system
    ctx.set_operator(P.OP_PB)
    phi, _ = ctx.newton(np.zeros(mesh.nv), reduction=s["newtonReduction"],
                        min_linear_reduction=s["newtonMinLinearReduction"], prec=P.PREC_SSOR)
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    u, res = ctx.newton(x0, reduction=s["newtonReduction"],
                        min_linear_reduction=s["newtonMinLinearReduction"], prec=P.PREC_SSOR)
    assert res["converged"] == 1
    assert np.max(np.abs(u_drv - u)) <= 1e-8 * np.max(np.abs(u))


def test_cpp_driver_reference_solvers(tmp_path):
    """pnp_main --reference-solvers: the stationary driver with the reference's own linear solvers
    (src/stationary_pnp_from_pb.hh:168-169 PB with BCGS_SSORk, :329-331 PNP with BCGS_NOPREC) --
    PNP_PREC_SSOR_NATURAL for PB and no preconditioner for PNP -- equals the same sequence through
    the Python mirror of the C ABI."""
    import subprocess
    exe = os.path.join(os.path.dirname(P.LIB_PATH), "pnp_main")
    cfgp = os.path.join(DATA, "cylinder_config.cfg")
    out = subprocess.run([exe, cfgp, "--reference-solvers", "--out", str(tmp_path / "cyl")],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    u_drv = np.loadtxt(tmp_path / "cyl_pnp.dat").T.ravel()
    cfg = P.read_config(cfgp)
    mesh = P.Mesh.read_gmsh(cfg.meshfile)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    s = cfg.system
    ctx.set_operator(P.OP_PB)
    phi, rpb = ctx.newton(np.zeros(mesh.nv), reduction=s["newtonReduction"],
                          min_linear_reduction=s["newtonMinLinearReduction"],
                          prec=P.PREC_SSOR_NATURAL)
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    u, res = ctx.newton(x0, reduction=s["newtonReduction"],
                        min_linear_reduction=s["newtonMinLinearReduction"], prec=P.PREC_NONE)
    assert res["converged"] == 1
    assert np.max(np.abs(u_drv - u)) <= 1e-8 * np.max(np.abs(u))


# ---- multicolour ILU(0) --------------------------------------------------------------------------
# stored block patterns (dune-pnp_amd/csrc/kernels.h kPatPnp / kPatPnpIE): PnpOperator has no
# c+/c- coupling; PnpTOperator's c- mass term lands in the c+ rows (quirk Q2) -> (1,2) present
PATS = {"pnp": [(f, g) for f in range(3) for g in range(3) if (f, g) not in ((1, 2), (2, 1))],
        "pnp_ie": [(f, g) for f in range(3) for g in range(3) if (f, g) != (2, 1)],
        "pb": [(0, 0)]}


def _ilu0_dense(A, M):
    """Textbook IKJ ILU(0) restricted to the pattern M (Saad, Alg. 10.4); pivots not inverted."""
    A = A.copy()
    n = A.shape[0]
    for i in range(n):
        for k in np.nonzero(M[i, :i])[0]:
            A[i, k] /= A[k, k]
            q = np.nonzero(M[i, k + 1:] & M[k, k + 1:])[0] + k + 1
            A[i, q] -= A[i, k] * A[k, q]
    return A


@pytest.mark.parametrize("f32", [0, 1, 2, 3])
@pytest.mark.parametrize("name,kind", [("pore_small_k0", "pnp"), ("pore_small_k0", "pnp_ie"),
                                       ("pore_small_k0", "pb"), ("cylinder_k0", "pnp")])
def test_ilu0_application_matches_textbook_ilu0(name, kind, f32):
    """pnp_prec_apply(ILU0) = (LU)^{-1} d with L, U the ILU(0) factors of the Jacobian on the
    stored block pattern, ordered colour-major by vertex with fields ascending.
    f32 = 0: fp64 factors, to rounding (1e-10); f32 = 1: the factors stored in single precision,
    fp64 sweeps -- the same operator to float rounding of the factors (2e-5 of max|v| on these
    well-conditioned small systems); f32 = 2 (PNP_OPT_ILU_F32's default): bfloat16 factors for
    block systems (8 significant bits: 2e-2 of max|v|), single precision for scalar ones; f32 = 3:
    2 with the forward intermediate in single precision (the same bound)."""
    import scipy.linalg as sla
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    ctx.set_option(P.OPT_ILU_F32, f32)
    assert ctx.get_option(P.OPT_ILU_F32) == f32
    set_ops(z, ctx, orc, kind)
    nf = 3 if kind.startswith("pnp") else 1
    A = ctx.jacobian(z[kind + "_x"]).toarray()
    lay = P.Layout(mesh)
    nv = mesh.nv
    perm = np.array([f * nv + lay.l2g[r] for r in range(nv) for f in range(nf)])
    Ap = A[np.ix_(perm, perm)]
    M = np.zeros_like(Ap, dtype=bool)
    pat = PATS[kind]
    for r in range(nv):
        for c in lay.row_cols(r):
            for f, g in pat:
                M[r * nf + f, c * nf + g] = True
    assert not np.any(Ap[~M]), "Jacobian has entries outside the stored pattern"
    # couplings of two rows of one colour (mesh.cc absorb_top) are outside the sweeps' pattern
    col = np.repeat(np.arange(len(lay.color_ptr) - 1), np.diff(lay.color_ptr))
    for r in range(nv):
        for c in lay.row_cols(r):
            if c != r and c < nv and col[c] == col[r]:
                M[r * nf:(r + 1) * nf, c * nf:(c + 1) * nf] = False
    F = _ilu0_dense(Ap, M)
    d = np.random.default_rng(5).standard_normal(nf * nv)
    y = sla.solve_triangular(np.tril(F, -1) + np.eye(len(F)), d[perm], lower=True)
    v_ref = sla.solve_triangular(np.triu(F), y, lower=False)
    v = ctx.prec_apply(d, P.PREC_ILU0)[perm]
    tol = 1e-10 if f32 == 0 else (2e-2 if f32 >= 2 and nf > 1 else 2e-5)
    assert np.max(np.abs(v - v_ref)) <= tol * np.max(np.abs(v_ref))


def test_pb_then_pnp_on_refined_pore_converges_with_ilu0():
    """The hard stationary case (test/pore_pnp, 24.1 V Dirichlet, refined once): BiCGSTAB with
    SSOR/Jacobi breaks down on the first Newton step; ILU(0) converges.  The converged state is
    checked with the oracle's residual."""
    cfg = P.read_config(os.path.join(DATA, "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(1)
    par = P.Params.from_config(cfg)
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PB)
    phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0)
    assert rpb["converged"] == 1, rpb
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    u, res = ctx.newton(x0, prec=P.PREC_ILU0, reduction=1e-8)
    assert res["converged"] == 1 and res["status"] == 0, res
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    r0 = np.linalg.norm(orc.residual(op, x0))
    r1 = np.linalg.norm(orc.residual(op, u))
    assert r1 <= 1e-8 * r0 * 1.01


@pytest.mark.parametrize("prec", ["ILU0"])
def test_pb_then_pnp_on_the_meshed_pore_without_dna(prec):
    """Config 5's geometry: test/pore_without_dna's .geo meshed natively (tests/test_mesher.py),
    refined once, PB Newton then PNP Newton (the reference's stationary driver sequence).  The
    converged state is checked with the oracle's residual.  (SSOR in the multicolour order
    diverges on this system -- in the oracle as well, see
    test_oracle.py::test_multicolour_ssor_diverges_where_natural_order_converges.)"""
    cfg = P.read_config(os.path.join(DATA, "pore_without_dna", "pore.cfg"))
    mesh = P.Mesh.load(cfg.meshfile).refine(1)
    par = P.Params.from_config(cfg)
    ctx = P.Context(mesh, par)
    pr = getattr(P, "PREC_" + prec)
    ctx.set_operator(P.OP_PB)
    phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=pr)
    assert rpb["converged"] == 1, rpb
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    u, res = ctx.newton(x0, prec=pr, reduction=1e-8)
    assert res["converged"] == 1 and res["status"] == 0, res
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    r0 = np.linalg.norm(orc.residual(op, x0))
    r1 = np.linalg.norm(orc.residual(op, u))
    assert r1 <= 1e-8 * r0 * 1.01


def test_operator_switch_leaves_no_stale_matrix_entries():
    """PB Newton then PNP in one context (the driver sequence): the PNP solve must behave exactly
    as in a fresh context (SELL padding slots hold zeros for the new block layout)."""
    cfg = P.read_config(os.path.join(DATA, "cylinder_config.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(1)
    par = P.Params.from_config(cfg)
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PB)
    phi, _ = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_SSOR)
    x0 = ctx.initial_state(phi)
    out = []
    for c in (ctx, P.Context(mesh, par)):
        c.set_operator(P.OP_PNP)
        c.jacobian(x0, export=False)
        r = c.residual(x0)
        out.append(c.linear_solve(r, prec=P.PREC_SSOR, reduction=1e-8, maxit=2000))
    (za, ra), (zb, rb) = out
    assert ra["converged"] == rb["converged"] == 1
    assert ra["it_half"] == rb["it_half"]
    np.testing.assert_array_equal(za, zb)


# ---- f3: ion-current observable ----------------------------------------------------------------
@pytest.mark.parametrize("name", ["cylinder_k0", "pore_small_k0", "one_wall_k1"])
def test_ion_flux_matches_oracle(name):
    """pnp_ion_flux (GPU, one thread per boundary segment) vs the oracle's calcIonFlux
    (src/ionFlux.hh:8-96) on the golden converged state; host vector and context state."""
    z, mesh, par, orc = golden(name)
    x = z["newton_pnp_u"] if "newton_pnp_u" in z.files else z["pnp_x"]
    ipo, imo = orc.ion_flux(x)
    ctx = P.Context(mesh, par)
    ip, im = ctx.ion_flux(x)
    scale = max(np.max(np.abs(ipo)), np.max(np.abs(imo)))
    assert np.max(np.abs(ip - ipo)) <= 1e-12 * scale
    assert np.max(np.abs(im - imo)) <= 1e-12 * scale
    ctx.set_operator(P.OP_PNP)
    ctx.state_set(x)
    ip2, im2 = ctx.ion_flux()
    np.testing.assert_array_equal(ip2, ip)
    np.testing.assert_array_equal(im2, im)


# ---- f1: operator-split driver (src/instationary_pnp_from_pb_md.hh) -----------------------------
def _md_oracle(orc, cfg, x0, nsteps):
    """The _md time loop on the oracle's operators with exact sparse solves: Alexander2 for c+
    and c- (DiffusionOperator + DiffusionTOperator), PoissonOperator problem every
    potentialUpdateFreq steps, calcIonFlux every outputFreq steps, a final Poisson solve."""
    import scipy.sparse.linalg as spla
    s = cfg.system
    nv = orc.nv
    phi, cp, cm = x0[:nv].copy(), x0[nv:2 * nv].copy(), x0[2 * nv:].copy()
    a, dt = 1.0 - 0.5 * np.sqrt(2.0), s["tau"]
    upd, outf = max(1, int(s["potentialUpdateFreq"])), max(1, int(s["outputFreq"]))
    m3 = orc.mask(3)

    def solve(op, x, extra=None):
        r = orc.residual(op, x) + (0 if extra is None else extra)
        return x - spla.spsolve(orc.jacobian(op, x).tocsc(), r)

    def poisson(phi, cp, cm):
        op = orc.operator(O.OP_POISSON, flux=orc.flux(), mask=orc.mask(1),
                          cp=np.ascontiguousarray(cp), cm=np.ascontiguousarray(cm))
        return solve(op, phi)

    def alexander2(c, z, field, phi):
        mask = np.ascontiguousarray(m3[field * nv:(field + 1) * nv])
        u0 = np.ascontiguousarray(c)
        op1 = orc.operator(O.OP_DIFF_IE, mask=mask, dt=a * dt, z=z, phi=np.ascontiguousarray(phi),
                           x_old=u0)
        u1 = solve(op1, u0.copy())
        opr = orc.operator(O.OP_DIFF, mask=mask, z=z, phi=np.ascontiguousarray(phi))
        r1 = (1.0 - a) * dt * orc.residual(opr, u1)
        return solve(op1, u1, r1)

    t, fluxes = 0.0, []
    for i in range(nsteps):
        cp = alexander2(cp, +1.0, 1, phi)
        cm = alexander2(cm, -1.0, 2, phi)
        t += dt
        if i % upd == 0:
            phi = poisson(phi, cp, cm)
        if i % outf == 0:
            fluxes.append((t, orc.ion_flux(np.concatenate([phi, cp, cm]))))
    phi = poisson(phi, cp, cm)
    return np.concatenate([phi, cp, cm]), fluxes


def test_md_driver_matches_oracle_loop(tmp_path):
    """The C++ driver's operator-split mode (pnp_main --mode md, 11 steps, linear reductions
    1e-12) against the same loop on the oracle with exact solves, from the driver's own
    Boltzmann initial state: final phi/c+/c- and the current.dat lines."""
    import subprocess
    exe = os.path.join(os.path.dirname(P.LIB_PATH), "pnp_main")
    cfgp = os.path.join(DATA, "cylinder_config.cfg")
    pre = str(tmp_path / "md")
    out = subprocess.run([exe, cfgp, "--mode", "md", "--steps", "11", "--md-reduction", "1e-12",
                          "--out", pre], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    x0 = np.loadtxt(pre + "_x0.dat").T.ravel()
    u_drv = np.loadtxt(pre + "_pnp.dat").T.ravel()
    cur = np.atleast_2d(np.loadtxt(pre + "_current.dat"))
    cfg = P.read_config(cfgp)
    mesh = P.Mesh.read_gmsh(cfg.meshfile)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    u_orc, fluxes = _md_oracle(orc, cfg, x0, 11)
    nv = mesh.nv
    for f in range(3):
        ref = u_orc[f * nv:(f + 1) * nv]
        assert np.max(np.abs(u_drv[f * nv:(f + 1) * nv] - ref)) <= 1e-8 * max(np.max(np.abs(ref)), 1e-30)
    assert cur.shape[0] == len(fluxes)
    for row, (t, (ip, im)) in zip(cur, fluxes):
        assert row[0] == pytest.approx(t)
        got = row[1:].reshape(-1, 4)
        scale = max(np.max(np.abs(ip)), np.max(np.abs(im)), 1e-30)
        assert np.max(np.abs(got[:, 0] - ip)) <= 1e-8 * scale
        assert np.max(np.abs(got[:, 2] - im)) <= 1e-8 * scale
        assert np.all(got[:, 1] == 0) and np.all(got[:, 3] == 0)


# ---- f4: ISTL CGSolver (LINEARSOLVER CG_NOPREC / CG_Jacobi) ---------------------------------------
@pytest.mark.parametrize("prec", [P.PREC_NONE, P.PREC_JACOBI])
def test_cg_matches_oracle_cg(prec):
    """Device-resident CG vs the oracle's ISTL CGSolver on the PB system (phi = 0): same solution,
    iteration counts equal up to one (the stop test compares a norm with summation-order
    rounding)."""
    z, mesh, par, orc = golden("pore_small_k0")
    ctx = P.Context(mesh, par)
    op = set_ops(z, ctx, orc, "pb")
    x = np.zeros(mesh.nv)
    J = ctx.jacobian(x)
    rhs = ctx.residual(x)
    sol, res = ctx.linear_solve(rhs, prec=prec, reduction=1e-10, maxit=5000, method=P.METHOD_CG)
    assert res["converged"] == 1, res
    assert np.linalg.norm(J @ sol - rhs) <= 1.001e-10 * np.linalg.norm(rhs)
    xo, ro = O.cg(orc.jacobian(op, x), rhs, prec=O.PREC_JACOBI if prec == P.PREC_JACOBI
                  else O.PREC_NONE, reduction=1e-10, maxit=5000)
    assert ro.converged
    assert abs(res["iterations"] - ro.iterations) <= 1
    assert np.max(np.abs(sol - xo)) <= 1e-8 * np.max(np.abs(xo))


@pytest.mark.parametrize("name,kind", [("pore_small_k0", "pnp"), ("pore_small_k0", "pnp_ie"),
                                       ("pore_small_k0", "pb"), ("cylinder_k0", "pnp")])
def test_ilu0_single_precision_intermediate(name, kind):
    """PNP_OPT_ILU_F32 = 3 (opt-in) against 2: the same bfloat16 factors, the forward sweep's
    intermediate L^-1 d rounded to single precision between the colour launches.  Block systems:
    the application differs from 2's (so the single-precision path ran) by float rounding only
    (1e-6 of max|v|), and BiCGSTAB converges with either; scalar systems keep f32 factors and fp64
    intermediates under both, bit for bit."""
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    set_ops(z, ctx, orc, kind)
    nf = 3 if kind.startswith("pnp") else 1
    x = z[kind + "_x"]
    ctx.jacobian(x, export=False)
    d = np.random.default_rng(11).standard_normal(nf * mesh.nv)
    rhs = ctx.residual(x)
    out = {}
    for f32 in (2, 3):
        ctx.set_option(P.OPT_ILU_F32, f32)
        v = ctx.prec_apply(d, P.PREC_ILU0)
        sol, res = ctx.linear_solve(rhs, prec=P.PREC_ILU0, reduction=1e-12, maxit=20000)
        assert res["converged"]
        out[f32] = (v, sol)
    (v2, s2), (v3, s3) = out[2], out[3]
    if nf == 1:
        assert np.array_equal(v2, v3) and np.array_equal(s2, s3)
        return
    assert not np.array_equal(v2, v3)
    assert np.max(np.abs(v3 - v2)) <= 1e-6 * np.max(np.abs(v2))


@pytest.mark.parametrize("f32", [0, 1])
@pytest.mark.parametrize("name,kind", [("pore_small_k0", "pnp"), ("pore_small_k0", "pnp_ie"),
                                       ("pore_small_k0", "pb")])
def test_fused_ilu0_factorisation_is_bitwise_the_three_pass_one(name, kind, f32):
    """PNP_OPT_ILU_FUSED_FACTOR (expand + factor + split in one launch per colour, the default)
    gives the factors of the three-pass path bit for bit: same preconditioner output."""
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    set_ops(z, ctx, orc, kind)
    ctx.set_option(P.OPT_ILU_F32, f32)
    nf = 3 if kind.startswith("pnp") else 1
    ctx.jacobian(z[kind + "_x"], export=False)
    d = np.random.default_rng(7).standard_normal(nf * mesh.nv)
    out = {}
    for fused in (0, 1):
        ctx.set_option(P.OPT_ILU_FUSED_FACTOR, fused)
        out[fused] = ctx.prec_apply(d, P.PREC_ILU0)
    assert np.array_equal(out[0], out[1])
    # and a re-split after a switch to SSOR (the split storage reused) still gives the factors
    ctx.prec_apply(d, P.PREC_SSOR)
    assert np.array_equal(ctx.prec_apply(d, P.PREC_ILU0), out[1])


@pytest.mark.parametrize("prec", [P.PREC_NONE, P.PREC_ILU0, P.PREC_SSOR])
def test_two_reduction_bicgstab_keeps_istl_counts(prec):
    """PNP_OPT_BICG_TWORED (the multi-rank default): rho_new from omega's reduction and the second
    half step's test lagged into the next <rt,v> reduction -- the same solution to the solve's
    tolerance as the three-reduction iteration.  rho_new = <rt,s> - omega <rt,t> differs from
    <rt,r> by rounding, and on this first Newton system (hundreds of iterations) the Krylov
    iterates drift apart by rounding, so the half-step counts agree to 10 % (measured: 47 / 45.5
    with ILU(0), 92 / 87 with SSOR, 933.5 / 939 without preconditioner); exact ISTL counting
    with the lagged test: test_bicgstab_half_step_counting_matches_istl (run with
    PNP_BICG_TWORED=1, profiles/r02)."""
    z, mesh, par, orc = golden("pore_small_k0")
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    x = z["newton_pnp_x0"]
    J = ctx.jacobian(x)
    b = ctx.residual(x)
    out = {}
    for tr in (0, 1):
        ctx.set_option(P.OPT_BICG_TWORED, tr)
        out[tr] = ctx.linear_solve(b, prec=prec, reduction=1e-8, maxit=20000)
    assert out[0][1]["converged"] == 1 and out[1][1]["converged"] == 1
    # without a preconditioner the ~1,000-iteration run is chaotic in the last bits (the oracle
    # spans 697 .. 1,282 iterations on a like system under 1e-14 perturbations, see
    # test_bicgstab_nonprec_matches_oracle_on_long_run): 30 % there, 20 % with a preconditioner
    # (ILU(0) on the round-6 fixture, whose x0 moved in its last bits with the per-element boundary
    # order of make_golden.py: 52 / 44.5 half steps, gpurun_out r6c; 47 / 45.5 before -- the same
    # +-15 % spread as the config-3 solves under one-ulp perturbations)
    tol = 0.3 if prec == P.PREC_NONE else 0.2
    assert abs(out[0][1]["it_half"] - out[1][1]["it_half"]) <= tol * out[0][1]["it_half"] + 0.5
    for tr in (0, 1):
        assert np.linalg.norm(J @ out[tr][0] - b) <= 1.001e-8 * np.linalg.norm(b)
