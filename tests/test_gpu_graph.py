"""hipGraph replay of the BiCGSTAB iteration blocks (PNP_OPT_GRAPH, -m gpu): the same kernels with
the same arguments as the eager launches, so every result is bitwise the eager one -- linear solves
with each preconditioner the graphs serve, Newton (operator and state changing between solves, the
captured graphs reused or re-captured), the fixed-iteration bench entry point, and an operator
switch between two solves (the cache must not replay the old operator's launches)."""
import numpy as np
import pytest

import pnp_amd as P
from test_gpu import golden

pytestmark = pytest.mark.gpu


def both(fn, name="pore_small_k0"):
    z, mesh, par, orc = golden(name)
    out = []
    for g in (0, 1):
        ctx = P.Context(mesh, par)
        ctx.set_option(P.OPT_GRAPH, g)
        assert ctx.get_option(P.OPT_GRAPH) == g
        out.append(fn(ctx, z, mesh))
        ctx.close()
    return out


@pytest.mark.parametrize("prec", [P.PREC_NONE, P.PREC_JACOBI, P.PREC_SSOR, P.PREC_ILU0,
                                  P.PREC_SSOR_NATURAL])
def test_graph_linear_solve_bitwise_equals_eager(prec):
    def fn(ctx, z, mesh):
        ctx.set_operator(P.OP_PNP)
        x = z["newton_pnp_x0"]
        ctx.jacobian(x, export=False)
        rhs = ctx.residual(x)
        a = ctx.linear_solve(rhs, prec=prec, reduction=1e-8, maxit=20000)
        b = ctx.linear_solve(rhs, prec=prec, reduction=1e-10, maxit=20000, check_every=5)
        return a, b
    (e, eb), (g, gb) = both(fn)
    for (se, re), (sg, rg) in ((e, g), (eb, gb)):
        assert re["converged"] == 1 and re["iterations"] == rg["iterations"], (re, rg)
        assert re["it_half"] == rg["it_half"]
        np.testing.assert_array_equal(se, sg)


def test_graph_newton_and_operator_switch_bitwise_equal_eager():
    def fn(ctx, z, mesh):
        ctx.set_operator(P.OP_PB)
        phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_SSOR)
        ctx.set_operator(P.OP_PNP)
        u, res = ctx.newton(z["newton_pnp_x0"], prec=P.PREC_ILU0)
        ctx.set_operator(P.OP_PB)  # back: the PB graphs must be re-captured for the new state
        phi2, rpb2 = ctx.newton(phi + 0.01, prec=P.PREC_ILU0)
        return phi, rpb, u, res, phi2, rpb2
    e, g = both(fn)
    for a, b in zip(e, g):
        if isinstance(a, dict):
            assert a["converged"] == 1 and a["linear_iterations"] == b["linear_iterations"], (a, b)
        else:
            np.testing.assert_array_equal(a, b)


def test_graph_fixed_iterations_bitwise_equal_eager():
    """pnp_bicgstab_iterations (the bench's entry point): one eager iteration, then one replay of
    the remaining ones per call."""
    def fn(ctx, z, mesh):
        ctx.set_operator(P.OP_PNP)
        ctx.state_set(z["newton_pnp_x0"])
        ctx.assemble_state(1)
        r = [ctx.bicgstab_iterations(n, P.PREC_ILU0) for n in (1, 2, 9, 9)]
        return [{k: v for k, v in d.items() if k != "elapsed"} for d in r]
    re, rg = both(fn)
    assert re == rg and re[-1]["defect"] > 0
