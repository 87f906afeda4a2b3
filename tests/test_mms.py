"""Independent pin of the discrete operators: convergence-rate studies against exact solutions of
the PDEs the reference discretises ("Next" item 2).

* Cylindrical PNP, manufactured solution (tests/mms.py): non-trivial r-dependence, mixed
  Dirichlet/Neumann faces (per field), the reference's PI = 3.1415 in both the 2 PI r weight and
  4 PI l_b.  The observed L2 order must be 2.0 +- 0.15 in every field -- on the oracle (CPU,
  k = 1..4) and on the GPU path through the C ABI (k = 1..5, PnpOperator residual + the load as
  pnp_op_args.c_extra, Newton with ILU(0) BiCGStab).  Negative controls show the study's power:
  the same loads built with the drift signs swapped, or with the radial weight's derivative
  dropped, do not converge.
* Gouy-Chapman (the reference's own known answer, test/one_wall_dh/one_wall.gp:4-12): PB on the
  one_wall strip against a tight solve_bvp solution, L2 order 2.0 +- 0.15 (oracle k = 1..4,
  GPU k = 1..5).
"""
import numpy as np
import pytest
import scipy.sparse.linalg as spl

import meshio
import mms
import oracle_py as O
import test_equilibrium as TE

ORDER, ORDER_TOL = 2.0, 0.15


def _mesh(k, product=False):
    base = mms.strip_mesh(4)
    if not product:
        return meshio.refine(base, k)
    import pnp_amd as P
    m = P.Mesh(base.xy, base.tri, base.bseg, base.bgroup).refine(k)
    return m


def _oracle_problem(m):
    return O.Problem(meshio.Mesh(m.xy, m.tri, m.bseg, m.bgroup), mms.surfaces(), l_b=mms.L_B,
                     c0=mms.C0, tau=1.0, cylindrical=1, pi=mms.PI)


def _oracle_mms_solve(m, variant=None):
    """Newton on R(u) - L = 0 with the oracle's residual and analytic Jacobian, direct solves."""
    orc = _oracle_problem(m)
    mask = orc.mask(3)
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=mask)
    L = mms.load(m, mms.surfaces(), variant) * (mask == 0)
    u = mms.start(m, mask)
    r0 = None
    for _ in range(20):
        r = orc.residual(op, u) - L
        nr = np.linalg.norm(r)
        r0 = nr if r0 is None else r0
        if nr <= 1e-11 * r0:
            break
        u = u - spl.spsolve(orc.jacobian(op, u).tocsc(), r)
    assert nr <= 1e-11 * r0
    return u


def test_manufactured_fields_derivatives():
    mms.check_derivatives()


def test_mms_cylindrical_pnp_oracle_order2():
    errs = np.array([mms.l2_errors(m, _oracle_mms_solve(m)) for m in (_mesh(k) for k in range(1, 5))])
    for f in range(3):
        r = mms.rates(errs[:, f])
        assert np.all(np.abs(r - ORDER) <= ORDER_TOL), (f, r, errs[:, f])


@pytest.mark.parametrize("variant", ["flip_drift", "planar_div"])
def test_mms_negative_controls_do_not_converge(variant):
    """A wrong operator (here: loads manufactured from a different PDE) leaves an O(1) error: the
    rate study would catch a drift-sign or radial-weight mistake in the operator."""
    errs = np.array([mms.l2_errors(m, _oracle_mms_solve(m, variant)) for m in (_mesh(k) for k in (3, 4))])
    ok = np.array([mms.l2_errors(m, _oracle_mms_solve(m)) for m in (_mesh(k) for k in (3, 4))])
    assert np.any(errs[-1] > 20 * ok[-1]), (errs, ok)
    # and the error no longer falls like h^2 once it is dominated by the model error
    assert min(mms.rates(errs[:, f])[0] for f in range(3)) < 1.0, errs


@pytest.mark.gpu
def test_mms_cylindrical_pnp_gpu_order2():
    import pnp_amd as P
    errs = []
    for k in range(1, 6):
        m = _mesh(k, product=True)
        surfs = [P.Surface(**vars(s)) for s in mms.surfaces()]
        par = P.Params(surfs, l_b=mms.L_B, c0=mms.C0, tau=1.0, cylindrical=1, pi=mms.PI)
        mask, _ = P.setup_boundary(m, par, 3)
        L = mms.load(m, mms.surfaces()) * (mask == 0)
        ctx = P.Context(m, par)
        ctx.set_operator(P.OP_PNP, c_extra=-L)
        u, res = ctx.newton(mms.start(m, mask), prec=P.PREC_ILU0, reduction=1e-11,
                            abs_limit=1e-15, min_linear_reduction=1e-6)
        assert res["converged"] == 1, (k, res)
        errs.append(mms.l2_errors(m, u))
        if k == 3:  # the GPU's discrete solution is the oracle's (same mesh, same loads)
            uo = _oracle_mms_solve(m)
            for f in range(3):
                sl = slice(f * m.nv, (f + 1) * m.nv)
                assert np.max(np.abs(u[sl] - uo[sl])) <= 1e-8 * np.max(np.abs(uo[sl]))
        ctx.close()
    errs = np.array(errs)
    for f in range(3):
        r = mms.rates(errs[:, f])
        assert np.all(np.abs(r - ORDER) <= ORDER_TOL), (f, r, errs[:, f])


# ---- Gouy-Chapman (PB, the reference's one_wall known answer) ------------------------------------
def _gc_reference(cfg, L):
    from scipy.integrate import solve_bvp
    s = cfg.system
    k2 = 8 * 3.1415 * s["l_b"] * s["c0"]
    j = cfg.surfaces[0].cflux
    sol = solve_bvp(lambda x, y: np.vstack([y[1], k2 * np.sinh(y[0])]),
                    lambda ya, yb: np.array([ya[1] - j, yb[0]]),
                    np.linspace(0, L, 400), np.zeros((2, 400)), tol=1e-10, max_nodes=200000)
    assert sol.success
    return lambda x: sol.sol(x)[0]


def _gc_l2(m, phi, exact):
    xi, eta, wq = mms.tri_rule()
    t = m.tri
    p0, p1, p2 = m.xy[t[:, 0]], m.xy[t[:, 1]], m.xy[t[:, 2]]
    adet = np.abs((p1[:, 0] - p0[:, 0]) * (p2[:, 1] - p0[:, 1]) -
                  (p2[:, 0] - p0[:, 0]) * (p1[:, 1] - p0[:, 1]))
    e2 = 0.0
    for q in range(len(wq)):
        x = p0[:, 0] + xi[q] * (p1[:, 0] - p0[:, 0]) + eta[q] * (p2[:, 0] - p0[:, 0])
        uh = (1 - xi[q] - eta[q]) * phi[t[:, 0]] + xi[q] * phi[t[:, 1]] + eta[q] * phi[t[:, 2]]
        e2 += np.sum((uh - exact(x)) ** 2 * wq[q] * adet)
    return np.sqrt(e2)


def test_gouy_chapman_pb_oracle_order2():
    cfg = meshio.read_config(TE.CFG)
    s = cfg.system
    base = meshio.read_gmsh(cfg.meshfile)
    exact = _gc_reference(cfg, base.xy[:, 0].max())
    errs = []
    for k in range(1, 5):
        m = meshio.refine(base, k)
        orc = O.Problem(m, cfg.surfaces, l_b=s["l_b"], c0=s["c0"], tau=s["tau"],
                        cylindrical=int(s["cylindrical"]))
        pb = orc.operator(O.OP_PB, flux=orc.flux(), mask=orc.mask(1))
        phi, r = orc.newton(pb, np.zeros(m.nv), prec=O.PREC_ILU0, reduction=1e-12)
        assert r.converged
        errs.append(_gc_l2(m, phi, exact))
    r = mms.rates(errs)
    assert np.all(np.abs(r - ORDER) <= ORDER_TOL), (r, errs)


@pytest.mark.gpu
def test_gouy_chapman_pb_gpu_order2():
    import pnp_amd as P
    cfg = P.read_config(TE.CFG)
    base = P.Mesh.load(cfg.meshfile)
    exact = _gc_reference(meshio.read_config(TE.CFG), base.xy[:, 0].max())
    errs = []
    for k in range(1, 6):
        m = base.refine(k)
        ctx = P.Context(m, P.Params.from_config(cfg))
        ctx.set_operator(P.OP_PB)
        phi, res = ctx.newton(np.zeros(m.nv), prec=P.PREC_ILU0, reduction=1e-12)
        assert res["converged"] == 1
        errs.append(_gc_l2(m, phi, exact))
        ctx.close()
    r = mms.rates(errs)
    assert np.all(np.abs(r - ORDER) <= ORDER_TOL), (r, errs)
