"""One-launch ILU(0) application (PNP_OPT_ILU_FLOW, linalg.hip k_ilu0_flow), -m gpu: the dataflow
launch runs the colour launches' arithmetic per row, so every result must be BITWISE the colour
launches' -- single applications (both factor precisions, from colour 0 and, inside BiCGSTAB, from
colour 1), BiCGSTAB solutions and counts (eager and graph-replayed), partitioned ranks, and on the
full config-3 system (2.2 M DOF: ~5,000 units per launch, the size where the hand-offs run under
load, each consumer's L1 warm with lines that other units rewrite during the launch)."""
import hashlib
import os

import numpy as np
import pytest

import pnp_amd as P
from conftest import DATA
from test_gpu import golden
from test_gpu_multirank import run_ranks

pytestmark = pytest.mark.gpu


def h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


def _both(ctx, fn, flow_on=1):
    """fn() with the colour launches, then with the dataflow form `flow_on`; the second run must
    actually launch the dataflow kernel (pnp_info.ilu_flow_applies), and the first must not."""
    out = []
    for flow in (0, flow_on):
        ctx.set_option(P.OPT_ILU_FLOW, flow)
        n0 = ctx.info()["ilu_flow_applies"]
        out.append(fn())
        ran = ctx.info()["ilu_flow_applies"] - n0
        assert (ran > 0) == (flow != 0), f"flow={flow}: {ran} dataflow launches"
    ctx.set_option(P.OPT_ILU_FLOW, 0)
    return out


@pytest.mark.parametrize("name", ["pore_small_k0", "cylinder_k0", "pore_pnp_k0"])
def test_flow_apply_and_solve_bitwise(name):
    z, mesh, par, orc = golden(name)
    x = z["newton_pnp_x0"] if "newton_pnp_x0" in z else z["pnp_x"]
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    ctx.jacobian(x, export=False)
    rhs = ctx.residual(x)
    for f32 in (1, 0):
        ctx.set_option(P.OPT_ILU_F32, f32)
        a, b = _both(ctx, lambda: h(ctx.prec_apply(rhs, P.PREC_ILU0)))
        assert a == b, f"apply f32={f32}"
        for graph in (0, 1):
            ctx.set_option(P.OPT_GRAPH, graph)

            def solve():
                sol, res = ctx.linear_solve(rhs, prec=P.PREC_ILU0, reduction=1e-10, maxit=20000)
                return h(sol), res["iterations"], res["it_half"]
            a, b = _both(ctx, solve)
            assert a == b, f"solve f32={f32} graph={graph}: {a} vs {b}"
    ctx.close()


def test_flow_pb_scalar_newton_bitwise():
    z, mesh, par, orc = golden("pore_small_k0")
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PB)
    a, b = _both(ctx, lambda: (lambda u, r: (h(u), r["linear_iterations"]))(
        *ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0)))
    assert a == b
    ctx.close()


def test_flow_partitioned_ranks_bitwise():
    z, mesh, par, orc = golden("pore_small_k0")
    x = z["newton_pnp_x0"]

    def fn(c, r):
        c.set_operator(P.OP_PNP)
        c.set_option(P.OPT_ILU_F32, 2)  # as in test_flow_config3_bitwise
        c.jacobian(x, export=False)
        b = c.sync_vector(c.residual(x))
        out = []
        # 2: the ticketed form, which needs no residency -- the three in-process ranks share the
        # GPU, where the default resident-grid form falls back to the colour launches
        for flow in (0, 2):
            c.set_option(P.OPT_ILU_FLOW, flow)
            n0 = c.info()["ilu_flow_applies"]
            sol, res = c.linear_solve(b, prec=P.PREC_ILU0, reduction=1e-10, maxit=20000)
            assert (c.info()["ilu_flow_applies"] > n0) == (flow != 0)
            out.append((h(c.sync_vector(sol)), res["iterations"]))
        return out
    outs = run_ranks(3, mesh, par, fn)
    for o in outs:
        assert o[0] == o[1]


def test_flow_config3_bitwise():
    """The bench's system: 2.2 M DOF at the Boltzmann state's neighbourhood (random state of the
    full-size parity test), fixed BiCGSTAB iterations, flow on and off: identical iterates."""
    cfg = P.read_config(os.path.join(DATA, "pore_pnp/pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    par = P.Params.from_config(cfg)
    rng = np.random.default_rng(20261015)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    # bfloat16 factors (2, the default; 3's single-precision forward intermediate lives in the
    # colour launches only: the dataflow form keeps it in fp64 and runs 3 as 2)
    ctx.set_option(P.OPT_ILU_F32, 2)
    ctx.jacobian(x, export=False)
    rhs = ctx.residual(x)

    def run():
        outs = [h(ctx.prec_apply(rhs, P.PREC_ILU0))]
        sol, res = ctx.linear_solve(rhs, prec=P.PREC_ILU0, reduction=1e-12, maxit=60)
        outs += [h(sol), res["it_half"]]
        return outs
    a, b = _both(ctx, run)
    assert a == b
    ctx.close()
