"""The drop-in boundary items of SURVEY.md §8(b) beyond residual / jacobian / solve (-m gpu):

  * PNP_JAC_FD: the reference's NumericalJacobianVolume (src/pnp_operator.hh:24-27 and the other
    LOPs' mixins) on the GPU, against the oracle's forward-difference Jacobian (oracle/pnp_oracle.c
    orc_op_jacobian(fd=1)): the same element residuals in the same operand order, accumulated in
    element order -- equal to rounding of the final sums for the polynomial operators; PB's sinh
    differs between device and host libm by ulps, amplified by 1/delta ~ 1e7;
  * pnp_jacobian_apply = GridOperator::jacobian_apply (NumericalJacobianApply*, :22-25);
  * PNP_DEVICE_PTRS: residual / Jacobian / jacobian_apply / solve on device vectors;
  * pnp_jacobian_csr_device: the assembled matrix as a device CSR (the BCRSMatrix the ISTL
    solvers take);
  * PNP_OPT_JAC_FD: Newton with the reference's FD Jacobian.
"""
import ctypes as C
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import pnp_amd as P
from test_gpu import golden, set_ops

pytestmark = pytest.mark.gpu

FD_CASES = [("cylinder_k0", "pnp"), ("pore_small_k0", "pnp"), ("pore_small_k0", "pnp_ie"),
            ("pore_small_k0", "pb"), ("pore_small_k0", "diff"), ("pore_small_k0", "poisson"),
            ("one_wall_k1", "pnp"), ("sphere_k0", "pb")]
# FD Jacobian vs the oracle's, relative to max|J|: rounding of the accumulated sums only for the
# polynomial operators; PB: device vs host sinh (ulps) / delta
FD_TOL = {"pb": 1e-8}


@pytest.mark.parametrize("name,kind", FD_CASES)
def test_fd_jacobian_matches_oracle_fd(name, kind):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    op = set_ops(z, ctx, orc, kind)
    x = z[kind + "_x"]
    J = ctx.jacobian(x, fd=True)
    Jo = orc.jacobian(op, x, fd=True)
    scale = abs(Jo).max()
    assert abs(J - Jo).max() <= FD_TOL.get(kind, 1e-13) * scale
    # the analytic Jacobian is the default again afterwards, and differs from FD by truncation
    Ja = ctx.jacobian(x)
    assert abs(Ja - orc.jacobian(op, x)).max() <= 1e-12 * scale
    assert abs(Ja - J).max() <= 1e-5 * scale


@pytest.mark.parametrize("fd", [False, True])
@pytest.mark.parametrize("name,kind", [("pore_small_k0", "pnp"), ("pore_small_k0", "pnp_ie"),
                                       ("pore_small_k0", "pb")])
def test_jacobian_apply(name, kind, fd):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    set_ops(z, ctx, orc, kind)
    x = z[kind + "_x"]
    d = np.random.default_rng(3).standard_normal(x.size)
    y = ctx.jacobian_apply(d, x=x, fd=fd)
    J = ctx.jacobian_export()
    y_ref = J @ d
    assert np.max(np.abs(y - y_ref)) <= 1e-13 * np.max(np.abs(y_ref))
    # x = None: the last assembled Jacobian
    assert np.array_equal(ctx.jacobian_apply(d), y)


class _Hip:
    """Device buffers through the HIP runtime libpnp_amd.so itself links (torch bundles another
    HIP runtime; two runtimes in one process do not share a device)."""

    def __init__(self):
        self.lib = C.CDLL("/opt/rocm/lib/libamdhip64.so")
        self.bufs = []

    def alloc(self, nbytes):
        p = C.c_void_p()
        assert self.lib.hipMalloc(C.byref(p), C.c_size_t(max(8, nbytes))) == 0
        self.bufs.append(p)
        return p.value

    def h2d(self, a):
        a = np.ascontiguousarray(a)
        p = self.alloc(a.nbytes)
        assert self.lib.hipMemcpy(C.c_void_p(p), C.c_void_p(a.ctypes.data), C.c_size_t(a.nbytes),
                                  1) == 0  # hipMemcpyHostToDevice
        return p

    def d2h(self, ptr, n, dtype):
        out = np.empty(n, dtype=dtype)
        assert self.lib.hipMemcpy(C.c_void_p(out.ctypes.data), C.c_void_p(ptr),
                                  C.c_size_t(out.nbytes), 2) == 0  # hipMemcpyDeviceToHost
        return out

    def free(self):
        for p in self.bufs:
            self.lib.hipFree(p)
        self.bufs = []


def test_device_pointers_and_device_csr_view():
    z, mesh, par, orc = golden("pore_small_k0")
    ctx = P.Context(mesh, par)
    set_ops(z, ctx, orc, "pnp")
    hip = _Hip()
    x = z["pnp_x"]
    n = x.size
    xd = hip.h2d(x)
    rd = hip.h2d(np.zeros(n))
    ctx.residual_dev(xd, rd)
    assert np.array_equal(hip.d2h(rd, n, np.float64), ctx.residual(x))
    for fd in (False, True):
        ctx.jacobian_dev(xd, fd=fd)
        J = ctx.jacobian_export()
        v = ctx.jacobian_csr_device()
        rp = hip.d2h(v["rowptr"], v["n"] + 1, np.int32)
        col = hip.d2h(v["col"], v["nnz"], np.int32)
        val = hip.d2h(v["val"], v["nnz"], np.float64)
        assert v["n"] == n and v["nnz"] == J.nnz
        assert np.array_equal(rp, J.indptr) and np.array_equal(col, J.indices)
        assert np.array_equal(val, J.data)
        d = np.random.default_rng(11).standard_normal(n)
        dd, yd = hip.h2d(d), hip.h2d(np.zeros(n))
        ctx.jacobian_apply_dev(0, dd, yd)
        assert np.array_equal(hip.d2h(yd, n, np.float64), ctx.jacobian_apply(d))
    # solve on device vectors = the host-vector solve
    ctx.jacobian(x, export=False)
    b = ctx.residual(x)
    zh, rh = ctx.linear_solve(b, prec=P.PREC_ILU0, reduction=1e-10)
    bd, zd = hip.h2d(b), hip.h2d(np.zeros(n))
    res = ctx.linear_solve_dev(bd, zd, prec=P.PREC_ILU0, reduction=1e-10)
    assert res["converged"] == 1 and res["iterations"] == rh["iterations"]
    assert np.array_equal(hip.d2h(zd, n, np.float64), zh)
    ctx.close()
    hip.free()


@pytest.mark.parametrize("name", ["cylinder_k0", "pore_small_k0"])
def test_newton_with_fd_jacobian_matches_analytic(name):
    """PNP_OPT_JAC_FD: the reference's Newton (every Jacobian by forward differences) converges to
    the analytic-Jacobian Newton's solution."""
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    set_ops(z, ctx, orc, "pnp")
    x0 = z["newton_pnp_x0"]
    ua, ra = ctx.newton(x0, reduction=1e-10, prec=P.PREC_ILU0)
    ctx.set_option(P.OPT_JAC_FD, 1)
    uf, rf = ctx.newton(x0, reduction=1e-10, prec=P.PREC_ILU0)
    ctx.set_option(P.OPT_JAC_FD, 0)
    assert ra["converged"] == 1 and rf["converged"] == 1
    scale = np.max(np.abs(ua))
    assert np.max(np.abs(uf - ua)) <= 1e-6 * scale


def test_fd_jacobian_partitioned():
    """FD Jacobian on 2 and 4 in-process ranks = the single-rank FD Jacobian."""
    z, mesh, par, orc = golden("pore_small_k0")
    x = z["pnp_x"]
    ctx1 = P.Context(mesh, par)
    ctx1.set_operator(P.OP_PNP)
    J1 = ctx1.jacobian(x, fd=True)
    for nranks in (2, 4):
        name = f"fd{nranks}"

        def work(r):
            ctx = P.Context(mesh, par, device=0, rank=r, size=nranks, local_group=name)
            try:
                ctx.set_operator(P.OP_PNP)
                return ctx.jacobian(x, fd=True)
            finally:
                ctx.close()
        with ThreadPoolExecutor(nranks) as ex:
            J = sum(ex.map(work, range(nranks)))
        assert abs(J - J1).max() <= 1e-15 * abs(J1).max()
