"""Iteration counts per rank count P (-m gpu), SURVEY.md §8(e)'s parity row: the config-5 system
(test/pore_without_dna's .geo meshed natively, scale 0.85 as bench.py's strong leg, refined k=4:
555,627 DOFs) split over P = 1, 2, 4, 8 ranks by RCB (the reference's loadBalance,
/root/reference/src/pnp_solver_main.cc:106-108) -- P in-process ranks on one GPU through the
local_group transport, which runs the partition, halo and reduction code of the RCCL path.

For each P and preconditioner (block-Jacobi ILU(0), and the aggregation AMG with an ILU(0) smoother,
both rank-local like the reference's NOVLP SSOR) the driver sequence runs: PB Newton, BCExtension,
PNP Newton with the config's settings tightened to reduction 1e-10.  Asserted: convergence at every
P, and the converged PNP state within 1e-6 of P = 1's.  Recorded (printed as one JSON line per case,
collected in DESIGN.md): PB / PNP Newton steps, BiCGSTAB iterations per Newton step."""
import json
import os
from concurrent.futures import ThreadPoolExecutor
import itertools

import numpy as np
import pytest

import pnp_amd as P
from conftest import DATA

pytestmark = pytest.mark.gpu
_grp = itertools.count()
_REF = {}


def _mesh(k=4):
    cfg = P.read_config(os.path.join(DATA, "pore_without_dna", "pore.cfg"))
    return cfg, P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(k)


def _run(nranks, mesh, par, fn):
    name = f"it{next(_grp)}"

    def work(r):
        ctx = P.Context(mesh, par, device=0, rank=r, size=nranks,
                        local_group=name if nranks > 1 else None)
        try:
            return fn(ctx, r)
        finally:
            ctx.close()
    with ThreadPoolExecutor(nranks) as ex:
        return list(ex.map(work, range(nranks)))


def _case(nranks, prec):
    cfg, mesh = _mesh(4)
    par = P.Params.from_config(cfg)
    s = cfg.system
    pr = P.PREC_BY_NAME[prec]

    def seq(ctx, r):
        if pr == P.PREC_AMG:
            ctx.amg_configure(smoother=P.PREC_ILU0)
        ctx.set_operator(P.OP_PB)
        phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=pr, reduction=1e-10)
        pb_its = ctx.newton_history()[0].tolist()
        phi = ctx.sync_vector(phi, 1)
        x0 = ctx.initial_state(phi)
        ctx.set_operator(P.OP_PNP)
        u, res = ctx.newton(x0, prec=pr, reduction=1e-10,
                            min_linear_reduction=s["newtonMinLinearReduction"],
                            linear_maxit=int(s["linearSolverIterations"]))
        pnp_its = ctx.newton_history()[0].tolist()
        return ctx.sync_vector(u), res, rpb, pb_its, pnp_its, ctx.info()["nv_ghost"]
    outs = _run(nranks, mesh, par, seq)
    u, res, rpb, pb_its, pnp_its, _ = outs[0]
    for o in outs:
        assert o[2]["converged"] == 1 and o[1]["converged"] == 1, (o[2], o[1])
        assert o[4] == pnp_its  # the same global iteration on every rank
    rec = {"P": nranks, "prec": prec, "dofs": 3 * mesh.nv,
           "ghost_vertices": [o[5] for o in outs],
           "pb_newton_steps": rpb["iterations"], "pb_linear_per_step": pb_its,
           "pnp_newton_steps": res["iterations"], "pnp_linear_per_step": pnp_its,
           "pnp_linear_total": res["linear_iterations"]}
    print("ITERS_PER_P " + json.dumps(rec))
    return u


@pytest.mark.parametrize("nranks,prec", [(p, q) for q in ("ilu0", "amg") for p in (1, 2, 4, 8)])
def test_iterations_per_rank_count(nranks, prec):
    if prec not in _REF:
        _REF[prec] = _case(1, prec)
    u = _REF[prec] if nranks == 1 else _case(nranks, prec)
    ref = _REF[prec]
    assert np.max(np.abs(u - ref)) <= 1e-6 * np.max(np.abs(ref))
