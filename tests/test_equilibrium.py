"""Known answer for the stationary PNP path: the reference's one_wall case
(test/one_wall_dh/one_wall.cfg) has zero ion flux on every wall but the far one, where
phi = 0 and c+- = c0.  Its exact stationary state is therefore thermodynamic equilibrium, with
phi the Poisson-Boltzmann (Gouy-Chapman) profile of the one_wall.gp:4-12 curve family.

Signs follow the reference's PNP operator: the c+ flux is grad c+ - c+ grad phi
(src/pnp_operator.hh:179-181) and the Poisson source 4 pi l_b (c+ - c-) (:169-171), so the
equilibrium is c+ = c0 exp(+phi), c- = c0 exp(-phi), consistent with the PB operator's
+8 pi l_b c0 sinh(phi) (src/pb_operator.hh:116-118).  The reference's "Boltzmann" initial state
(src/dirichlet_bc.hh:107,115) uses the opposite signs, c+ = c0 exp(-phi); that quirk is kept
(parity), and is why the PNP Newton from it takes several steps.  Here the Newton is started
from phi = 0, c = c0, far from equilibrium, so the Newton/line-search/BiCGStab path has to
find it.

The oracle leg runs on the CPU; the GPU leg runs the same solve through the C ABI."""
import os

import numpy as np
import pytest

import meshio
import oracle_py as O
from conftest import DATA

CFG = os.path.join(DATA, "one_wall_dh", "one_wall.cfg")
REFINE = 3


def bvp_profile(cfg, xs, L):
    """-phi'' + kappa^2 sinh(phi) = 0, phi'(0) = j, phi(L) = 0 (one_wall.gp:4-12)."""
    from scipy.integrate import solve_bvp
    s = cfg.system
    k2 = 8 * 3.1415 * s["l_b"] * s["c0"]
    j = cfg.surfaces[0].cflux
    sol = solve_bvp(lambda x, y: np.vstack([y[1], k2 * np.sinh(y[0])]),
                    lambda ya, yb: np.array([ya[1] - j, yb[0]]),
                    np.linspace(0, L, 200), np.zeros((2, 200)), tol=1e-10, max_nodes=100000)
    assert sol.success
    return sol.sol(xs)[0]


def check_equilibrium(xy, u, cfg, pb_phi):
    nv = xy.shape[0]
    c0 = cfg.system["c0"]
    phi, cp, cm = u[:nv], u[nv:2 * nv], u[2 * nv:]
    exact = bvp_profile(cfg, xy[:, 0], xy[:, 0].max())
    scale = np.max(np.abs(exact))
    # the same discretisation-error bound as the PB known-answer test (test_oracle.py)
    assert np.max(np.abs(phi - exact)) <= 2e-3 * scale
    # PNP's potential is the PB potential of the same mesh up to the discretisation of the drift
    # (measured 4.4e-7 on the oracle)
    assert np.max(np.abs(phi - pb_phi)) <= 1e-5 * scale
    # Boltzmann distribution of both species, relative to the size of the double layer
    # (measured 3.3e-5 / 3.9e-5 on the oracle: P1 drift-diffusion is not exact for exponentials)
    dev = c0 * np.max(np.abs(np.expm1(phi)))
    assert np.max(np.abs(cp - c0 * np.exp(phi))) <= 1e-3 * dev
    assert np.max(np.abs(cm - c0 * np.exp(-phi))) <= 1e-3 * dev
    # the double layer is there: phi < 0 at the charged wall, c- enriched, c+ depleted
    wall = xy[:, 0] == xy[:, 0].min()
    assert np.all(phi[wall] < 0)
    assert np.all(cm[wall] > c0) and np.all(cp[wall] < c0)


def test_pnp_equilibrium_oracle():
    cfg = meshio.read_config(CFG)
    m = meshio.refine(meshio.read_gmsh(cfg.meshfile), REFINE)
    s = cfg.system
    P = O.Problem(m, cfg.surfaces, l_b=s["l_b"], c0=s["c0"], tau=s["tau"],
                  cylindrical=int(s["cylindrical"]))
    pb = P.operator(O.OP_PB, flux=P.flux(), mask=P.mask(1))
    phi_pb, rpb = P.newton(pb, np.zeros(m.nv), prec=O.PREC_ILU0, reduction=1e-12)
    assert rpb.converged
    op = P.operator(O.OP_PNP, flux=P.flux(), mask=P.mask(3))
    u, res = P.newton(op, P.initial_state(np.zeros(m.nv)), prec=O.PREC_ILU0, reduction=1e-10)
    assert res.converged == 1 and res.status == 0
    check_equilibrium(m.xy, u, cfg, phi_pb)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["ilu0", "amg"])
def test_pnp_equilibrium_gpu(prec):
    import pnp_amd as P
    cfg = P.read_config(CFG)
    mesh = P.Mesh.load(cfg.meshfile).refine(REFINE)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PB)
    phi_pb, rpb = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0, reduction=1e-12)
    assert rpb["converged"] == 1
    x0 = ctx.initial_state(np.zeros(mesh.nv))
    ctx.set_operator(P.OP_PNP)
    pc = P.PREC_ILU0 if prec == "ilu0" else P.PREC_AMG
    u, res = ctx.newton(x0, prec=pc, reduction=1e-10)
    assert res["converged"] == 1
    check_equilibrium(mesh.xy, u, meshio.read_config(CFG), phi_pb)


def _ie_steps(step, x0, nmax=80, tol=1e-11):
    """Implicit-Euler steps (PnpOperator + PnpTOperator, config 4's operator) until the state
    stops moving; returns the final state and the number of steps."""
    x = x0
    for n in range(1, nmax + 1):
        u = step(x)
        if np.max(np.abs(u - x)) <= tol * np.max(np.abs(u)):
            return u, n
        x = u
    return x, nmax


DT = 20.0


def test_pnp_implicit_euler_relaxes_to_equilibrium_oracle():
    """The instationary path (rows a4/a13) on the same known answer: implicit-Euler steps from
    phi = 0, c = c0 relax to the stationary equilibrium (the time term vanishes there, so the
    PnpTOperator quirk Q2 does not move it)."""
    cfg = meshio.read_config(CFG)
    m = meshio.refine(meshio.read_gmsh(cfg.meshfile), REFINE)
    s = cfg.system
    P = O.Problem(m, cfg.surfaces, l_b=s["l_b"], c0=s["c0"], tau=s["tau"],
                  cylindrical=int(s["cylindrical"]))
    pb = P.operator(O.OP_PB, flux=P.flux(), mask=P.mask(1))
    phi_pb, _ = P.newton(pb, np.zeros(m.nv), prec=O.PREC_ILU0, reduction=1e-12)
    flux, mask = P.flux(), P.mask(3)

    def step(x_old):
        op = P.operator(O.OP_PNP_IE, flux=flux, mask=mask, dt=DT, x_old=np.ascontiguousarray(x_old))
        u, res = P.newton(op, x_old, prec=O.PREC_ILU0, reduction=1e-12)
        assert res.converged
        return u
    u, n = _ie_steps(step, P.initial_state(np.zeros(m.nv)))
    assert n < 80
    check_equilibrium(m.xy, u, cfg, phi_pb)


@pytest.mark.gpu
def test_pnp_implicit_euler_relaxes_to_equilibrium_gpu():
    import pnp_amd as P
    cfg = P.read_config(CFG)
    mesh = P.Mesh.load(cfg.meshfile).refine(REFINE)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PB)
    phi_pb, _ = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0, reduction=1e-12)
    x0 = ctx.initial_state(np.zeros(mesh.nv))

    def step(x_old):
        ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=DT, x_old=x_old)
        u, res = ctx.newton(x_old, prec=P.PREC_ILU0, reduction=1e-12)
        assert res["converged"] == 1
        return u
    u, n = _ie_steps(step, x0)
    assert n < 80
    check_equilibrium(mesh.xy, u, meshio.read_config(CFG), phi_pb)
