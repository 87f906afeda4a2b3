"""Config 4 (BASELINE.json configs[3]): instationary PNP on test/pore.msh,
100 implicit-Euler steps of PnpOperator + PnpTOperator with dt = tau = 1, 1 -> 4 GPUs.

The reference's time loop is src/instationary_pnp_from_pb.hh:320-431 (its explicit Euler is
singular for PNP -- M has zero phi rows, SURVEY.md §3.5 -- so config 4 runs implicit Euler,
M(u1) - M(u0) + dt R(u1) = 0, each step a PDELab Newton).  Newton settings are the reference's:
newtonReduction 1e-9 and newtonMinLinearReduction 1e-8 from test/pore_pnp/pore.cfg:9-10, and
PDELab's default absolute limit 1e-12 (the config sets none).  No extra abs_limit is needed on
this mesh: test_newton_target_is_above_the_rounding_floor measures where Newton stagnates.

Legs:
  * oracle (CPU): the same 100-step loop on oracle/pnp_oracle.c (natural-order ILU(0) BiCGStab);
  * GPU, 1 rank: the C++ driver, pnp_main --mode instationary (the reference's binary shape),
    state dumped after steps 1, 10 and 100;
  * GPU, 4 ranks: the same loop through the Python mirror on 4 local_group ranks (RCB partition,
    halo exchange, global reductions, block-Jacobi ILU(0)) vs 1 rank.
Trajectories must agree within 1e-6 of each field's magnitude at steps 1, 10 and 100: both
sides stop Newton at 1e-9 of the first defect, with different (equally valid) Krylov iterates.
"""
import os
import subprocess

import numpy as np
import pytest

import meshio
import oracle_py as O
from conftest import DATA

CFG = os.path.join(DATA, "pore_pnp", "pore.cfg")
MESH = os.path.join(DATA, "pore.msh")  # test/pore.msh (BASELINE.json configs[3])
STEPS = 100
CHECK = (1, 10, 100)
ABS_LIMIT = 1e-12  # PDELab Newton default (the reference's configs do not set one)
TOL = 1e-6


def _oracle_problem():
    cfg = meshio.read_config(CFG)
    m = meshio.read_gmsh(MESH)
    s = cfg.system
    orc = O.Problem(m, cfg.surfaces, l_b=s["l_b"], c0=s["c0"], tau=s["tau"],
                    cylindrical=int(s["cylindrical"]))
    return cfg, m, orc


def _newton_kw(cfg):
    s = cfg.system
    return dict(reduction=s["newtonReduction"], min_linear_reduction=s["newtonMinLinearReduction"],
                abs_limit=ABS_LIMIT, maxit=int(s["newtonMaxIterations"]),
                line_search_maxit=int(s["newtonLineSearchMaxIteration"]))


def oracle_trajectory(x0, steps=STEPS, check=CHECK):
    """The config-4 loop on the oracle: {step: state} at the check steps, plus Newton stats."""
    cfg, m, orc = _oracle_problem()
    flux, mask = orc.flux(), orc.mask(3)
    kw = _newton_kw(cfg)
    x, out, stats = np.array(x0, dtype=np.float64), {}, []
    for n in range(1, steps + 1):
        op = orc.operator(O.OP_PNP_IE, flux=flux, mask=mask, dt=cfg.system["tau"],
                          x_old=np.ascontiguousarray(x))
        x, res = orc.newton(op, x, prec=O.PREC_ILU0, **kw)
        assert res.converged == 1 and res.status == 0, (n, res.first_defect, res.defect)
        stats.append((res.first_defect, res.defect, res.iterations))
        if n in check:
            out[n] = x.copy()
    return out, stats


def oracle_x0():
    """The reference driver's initial state: PB Newton (SSOR BiCGStab) from 0, then the
    BCExtension interpolation (src/stationary_pnp_from_pb.hh:105-282)."""
    cfg, m, orc = _oracle_problem()
    pb = orc.operator(O.OP_PB, flux=orc.flux(), mask=orc.mask(1))
    phi, r = orc.newton(pb, np.zeros(m.nv), prec=O.PREC_SSOR, **_newton_kw(cfg))
    assert r.converged == 1
    return orc.initial_state(phi)


def assert_same_state(u, ref, nv, what):
    for f, name in enumerate(("phi", "c+", "c-")):
        a, b = u[f * nv:(f + 1) * nv], ref[f * nv:(f + 1) * nv]
        scale = np.max(np.abs(b))
        err = np.max(np.abs(a - b))
        assert err <= TOL * scale, f"{what}: {name} differs by {err:.3e} (scale {scale:.3e})"


def test_newton_target_is_above_the_rounding_floor():
    """Evidence for the Newton limits of config 4 (oracle, CPU): at the check steps, after the
    step converged, Newton is continued with no limit at all; the defect it stagnates at is the
    residual's rounding floor.  The reference's target max(1e-9 d0, 1e-12) must sit above it,
    else the relative test alone would stall.  Measured on test/pore.msh: d0 falls from 0.17
    (step 2) to 0.0195 (step 100), the floor stays at 2.5-3e-12, so the target stays >= 6x above
    it and PDELab's own limits suffice.  The floor grows like sqrt(N) (a 2-norm over rows of
    fixed per-row rounding): 1.2e-11 at k=2, which is why the k=3 run of tools/bench_configs.py
    (d0 ~ 1e-2) needs an abs_limit above it."""
    cfg, m, orc = _oracle_problem()
    x = oracle_x0()
    flux, mask = orc.flux(), orc.mask(3)
    kw = _newton_kw(cfg)
    for n in range(1, STEPS + 1):
        op = orc.operator(O.OP_PNP_IE, flux=flux, mask=mask, dt=cfg.system["tau"],
                          x_old=np.ascontiguousarray(x))
        u, res = orc.newton(op, x, prec=O.PREC_ILU0, **kw)
        assert res.converged == 1
        if n in CHECK:
            target = max(kw["reduction"] * res.first_defect, ABS_LIMIT)
            _, stall = orc.newton(op, u, prec=O.PREC_ILU0, reduction=1e-30, abs_limit=0.0,
                                  maxit=6, line_search_maxit=30)
            floor = stall.defect
            assert floor <= target / 4, (n, floor, target)
        x = u


@pytest.mark.gpu
def test_config4_driver_matches_oracle(tmp_path):
    """pnp_main --mode instationary (100 IE steps, ILU(0) BiCGStab, the config's Newton settings)
    against the oracle's loop from the driver's own initial state."""
    import pnp_amd as P
    exe = os.path.join(os.path.dirname(P.LIB_PATH), "pnp_main")
    cfg_txt = open(CFG).read().replace("filename=pore.msh", f"filename={MESH}")
    cfgp = tmp_path / "pore_c4.cfg"
    cfgp.write_text(cfg_txt)
    pre = str(tmp_path / "c4")
    out = subprocess.run([exe, str(cfgp), "--mode", "instationary", "--steps", str(STEPS),
                          "--prec", "ilu0", "--abs-limit", str(ABS_LIMIT), "--dump-steps",
                          ",".join(map(str, CHECK)), "--out", pre],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    x0 = np.loadtxt(pre + "_x0.dat").T.ravel()
    nv = x0.size // 3
    assert_same_state(x0, oracle_x0(), nv, "initial state (PB + BCExtension)")
    ref, _ = oracle_trajectory(x0)
    for n in CHECK:
        u = np.loadtxt(f"{pre}_step{n}.dat").T.ravel()
        assert_same_state(u, ref[n], nv, f"step {n}")
    # the run is not a fixed point: the state moves between the check steps
    assert np.max(np.abs(ref[100] - ref[1])) > 1e3 * TOL * np.max(np.abs(ref[100]))


def _gpu_loop(ctx, x0, steps, check, s):
    import pnp_amd as P
    x, out, stats = np.array(x0), {}, []
    for n in range(1, steps + 1):
        ctx.set_operator(P.OP_PNP_IMPLICIT_EULER, dt=s["tau"], x_old=x)
        u, res = ctx.newton(x, prec=P.PREC_ILU0, reduction=s["newtonReduction"],
                            min_linear_reduction=s["newtonMinLinearReduction"],
                            abs_limit=ABS_LIMIT, maxit=int(s["newtonMaxIterations"]),
                            line_search_maxit=int(s["newtonLineSearchMaxIteration"]))
        assert res["converged"] == 1 and res["status"] == 0, (n, res)
        x = ctx.sync_vector(u, 3)
        stats.append(res["iterations"])
        if n in check:
            out[n] = x.copy()
    return out, stats


@pytest.mark.gpu
def test_config4_four_ranks_match_one_rank_and_oracle():
    """The same 100 steps on 4 in-process ranks (local_group transport: the RCCL path's
    partition, halo and reduction code) vs 1 rank, and both vs the oracle."""
    import pnp_amd as P
    from test_gpu_multirank import run_ranks
    cfg = P.read_config(CFG)
    mesh = P.Mesh.read_gmsh(MESH)
    par = P.Params.from_config(cfg)
    x0 = oracle_x0()
    s = cfg.system
    ctx1 = P.Context(mesh, par)
    one, _ = _gpu_loop(ctx1, x0, STEPS, CHECK, s)
    ctx1.close()
    four = run_ranks(4, mesh, par, lambda c, r: _gpu_loop(c, x0, STEPS, CHECK, s)[0])
    ref, _ = oracle_trajectory(x0)
    nv = mesh.nv
    for n in CHECK:
        assert_same_state(one[n], ref[n], nv, f"1 rank, step {n}")
        for r, o in enumerate(four):
            assert_same_state(o[n], one[n], nv, f"4 ranks (rank {r}) vs 1 rank, step {n}")
