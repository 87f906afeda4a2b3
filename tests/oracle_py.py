"""ctypes binding of the CPU oracle (oracle/liboracle.so).  Test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_LIB = None

OP_PNP, OP_PNP_IE, OP_PB, OP_DIFF, OP_DIFF_IE, OP_POISSON = range(6)
PREC_NONE, PREC_SSOR, PREC_ILU0, PREC_JACOBI = range(4)


class OrcMesh(C.Structure):
    _fields_ = [("nv", C.c_int), ("xy", C.c_void_p), ("nt", C.c_int), ("tri", C.c_void_p),
                ("nb", C.c_int), ("bseg", C.c_void_p), ("bgroup", C.c_void_p)]


class OrcSurface(C.Structure):
    _fields_ = [("cb", C.c_int), ("cflux", C.c_double), ("cpot", C.c_double),
                ("pb", C.c_int), ("pflux", C.c_double), ("pconc", C.c_double),
                ("mb", C.c_int), ("mflux", C.c_double), ("mconc", C.c_double)]


class OrcParams(C.Structure):
    _fields_ = [("l_b", C.c_double), ("c0", C.c_double), ("tau", C.c_double), ("pi", C.c_double),
                ("cylindrical", C.c_int), ("nsurf", C.c_int), ("surf", C.c_void_p)]


class OrcCsr(C.Structure):
    _fields_ = [("n", C.c_int), ("nnz", C.c_int), ("rowptr", C.POINTER(C.c_int)),
                ("col", C.POINTER(C.c_int)), ("val", C.POINTER(C.c_double))]


class OrcOperator(C.Structure):
    _fields_ = [("kind", C.c_int), ("flux", C.c_void_p), ("mask", C.c_void_p), ("dt", C.c_double),
                ("z", C.c_double), ("phi", C.c_void_p), ("cp", C.c_void_p), ("cm", C.c_void_p),
                ("x_old", C.c_void_p)]


class OrcPk(C.Structure):
    _fields_ = [("k", C.c_int), ("nl", C.c_int), ("nn", C.c_int), ("nedge", C.c_int),
                ("xy", C.POINTER(C.c_double)), ("enode", C.POINTER(C.c_int))]


class OrcSolveResult(C.Structure):
    _fields_ = [("converged", C.c_int), ("iterations", C.c_int), ("it_half", C.c_double),
                ("reduction", C.c_double), ("defect0", C.c_double), ("defect", C.c_double),
                ("breakdown", C.c_int), ("setup_seconds", C.c_double),
                ("iter_seconds", C.c_double)]


class OrcNewtonOpts(C.Structure):
    _fields_ = [("reduction", C.c_double), ("abs_limit", C.c_double),
                ("min_linear_reduction", C.c_double), ("maxit", C.c_int),
                ("line_search_maxit", C.c_int), ("reassemble_threshold_zero", C.c_int),
                ("linear_maxit", C.c_int), ("prec", C.c_int), ("fd_jacobian", C.c_int)]


class OrcNewtonResult(C.Structure):
    _fields_ = [("converged", C.c_int), ("iterations", C.c_int), ("linear_iterations", C.c_int),
                ("status", C.c_int), ("first_defect", C.c_double), ("defect", C.c_double),
                ("step_linear_iterations", C.c_int * 64)]


def lib():
    global _LIB
    if _LIB is None:
        so = os.path.join(ORACLE_DIR, "liboracle.so")
        srcs = [os.path.join(ORACLE_DIR, f) for f in ("pnp_oracle.c", "pnp_oracle_pk.c",
                                                       "pnp_oracle.h")]
        if not os.path.exists(so) or any(os.path.getmtime(so) < os.path.getmtime(f)
                                         for f in srcs):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        _LIB = C.CDLL(so)
        _LIB.orc_operator_nfields.restype = C.c_int
    return _LIB


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


class Problem:
    """Holds the ctypes views of one mesh + parameter set for the oracle."""

    def __init__(self, mesh, surfaces, l_b=1.0, c0=0.06, tau=1.0, cylindrical=0, pi=3.1415):
        self.mesh = mesh
        self.xy = np.ascontiguousarray(mesh.xy, dtype=np.float64)
        self.tri = np.ascontiguousarray(mesh.tri, dtype=np.int32)
        self.bseg = np.ascontiguousarray(mesh.bseg, dtype=np.int32)
        self.bgroup = np.ascontiguousarray(mesh.bgroup, dtype=np.int32)
        self.m = OrcMesh(mesh.nv, self.xy.ctypes.data, mesh.nt, self.tri.ctypes.data, mesh.nb,
                         self.bseg.ctypes.data, self.bgroup.ctypes.data)
        arr = (OrcSurface * len(surfaces))()
        for i, s in enumerate(surfaces):
            arr[i] = OrcSurface(s.cb, s.cflux, s.cpot, s.pb, s.pflux, s.pconc, s.mb, s.mflux,
                                s.mconc)
        self._surf = arr
        self.p = OrcParams(l_b, c0, tau, pi, cylindrical, len(surfaces),
                           C.cast(arr, C.c_void_p))
        self.nv = mesh.nv

    # setup -----------------------------------------------------------------------------
    def mask(self, nfields):
        out = np.zeros(nfields * self.nv, dtype=np.uint8)
        lib().orc_dirichlet_mask(C.byref(self.m), C.byref(self.p), nfields, _p(out))
        return out

    def flux(self):
        out = np.zeros(3 * self.mesh.nb, dtype=np.float64)
        lib().orc_flux_container(C.byref(self.m), C.byref(self.p), _p(out))
        return out

    def initial_state(self, phi_pb):
        out = np.zeros(3 * self.nv, dtype=np.float64)
        phi = np.ascontiguousarray(phi_pb, dtype=np.float64)
        lib().orc_initial_state(C.byref(self.m), C.byref(self.p), _p(phi), _p(out))
        return out

    def ion_flux(self, x):
        """calcIonFlux (src/ionFlux.hh:8-96): per-surface (ip, im) of the state x."""
        n = self.p.nsurf
        ip = np.zeros(n, dtype=np.float64)
        im = np.zeros(n, dtype=np.float64)
        x = np.ascontiguousarray(x, dtype=np.float64)
        lib().orc_ion_flux(C.byref(self.m), C.byref(self.p), _p(x), _p(ip), _p(im))
        return ip, im

    # operators ---------------------------------------------------------------------------
    def operator(self, kind, flux=None, mask=None, dt=0.0, z=0.0, phi=None, cp=None, cm=None,
                 x_old=None):
        keep = [a for a in (flux, mask, phi, cp, cm, x_old) if a is not None]
        ad = lambda a: None if a is None else a.ctypes.data
        op = OrcOperator(kind, ad(flux), ad(mask), dt, z, ad(phi), ad(cp), ad(cm), ad(x_old))
        op._keep = keep
        return op

    def nfields(self, op):
        return lib().orc_operator_nfields(C.byref(op))

    def residual(self, op, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        r = np.zeros(self.nfields(op) * self.nv, dtype=np.float64)
        lib().orc_op_residual(C.byref(self.m), C.byref(self.p), C.byref(op), _p(x), _p(r))
        return r

    def jacobian(self, op, x, fd=False):
        """Returns a scipy.sparse.csr_matrix (copy) of the operator Jacobian."""
        import scipy.sparse as sp
        x = np.ascontiguousarray(x, dtype=np.float64)
        A = OrcCsr()
        L = lib()
        L.orc_csr_pattern(C.byref(self.m), self.nfields(op), C.byref(A))
        L.orc_op_jacobian(C.byref(self.m), C.byref(self.p), C.byref(op), _p(x), int(fd),
                          C.byref(A))
        n, nnz = A.n, A.nnz
        rp = np.ctypeslib.as_array(A.rowptr, shape=(n + 1,)).copy()
        col = np.ctypeslib.as_array(A.col, shape=(nnz,)).copy()
        val = np.ctypeslib.as_array(A.val, shape=(nnz,)).copy()
        L.orc_csr_free(C.byref(A))
        return sp.csr_matrix((val, col, rp), shape=(n, n))

    def time_fd_assembly(self, op, x, seconds):
        """Reference-faithful assembly timing: PnpOperator residual + NumericalJacobianVolume
        forward-difference Jacobian scattered into a prebuilt CSR (the BCRS pattern is built
        once, like `M m(go)` at src/stationary_pnp_from_pb.hh:318-319). Returns (s/assembly, A)."""
        import time
        x = np.ascontiguousarray(x, dtype=np.float64)
        r = np.zeros(self.nfields(op) * self.nv)
        A = OrcCsr()
        L = lib()
        L.orc_csr_pattern(C.byref(self.m), self.nfields(op), C.byref(A))
        n, t0 = 0, time.perf_counter()
        while True:
            L.orc_op_residual(C.byref(self.m), C.byref(self.p), C.byref(op), _p(x), _p(r))
            L.orc_op_jacobian(C.byref(self.m), C.byref(self.p), C.byref(op), _p(x), 1,
                              C.byref(A))
            n += 1
            if time.perf_counter() - t0 >= seconds:
                break
        dt = (time.perf_counter() - t0) / n
        import scipy.sparse as sp
        rp = np.ctypeslib.as_array(A.rowptr, shape=(A.n + 1,)).copy()
        col = np.ctypeslib.as_array(A.col, shape=(A.nnz,)).copy()
        val = np.ctypeslib.as_array(A.val, shape=(A.nnz,)).copy()
        n = A.n
        L.orc_csr_free(C.byref(A))
        return dt, sp.csr_matrix((val, col, rp), shape=(n, n))

    def time_fd_assembly_mt(self, op, x, seconds):
        """All-core CPU baseline: the same residual + forward-difference Jacobian assembly with
        OpenMP over element colours (orc_assemble_mt).  Returns (s/assembly, threads, A, r)."""
        import time
        import scipy.sparse as sp
        L = lib()
        col = np.zeros(self.mesh.nt, dtype=np.int32)
        ncol = L.orc_element_colors(C.byref(self.m), _p(col))
        assert ncol > 0
        order = np.argsort(col, kind="stable").astype(np.int32)
        cptr = np.zeros(ncol + 1, dtype=np.int32)
        cptr[1:] = np.cumsum(np.bincount(col, minlength=ncol))
        x = np.ascontiguousarray(x, dtype=np.float64)
        r = np.zeros(self.nfields(op) * self.nv)
        A = OrcCsr()
        L.orc_csr_pattern(C.byref(self.m), self.nfields(op), C.byref(A))
        n, t0 = 0, time.perf_counter()
        while True:
            L.orc_assemble_mt(C.byref(self.m), C.byref(self.p), C.byref(op), _p(x), _p(order),
                              _p(cptr), int(ncol), C.byref(A), _p(r))
            n += 1
            if time.perf_counter() - t0 >= seconds:
                break
        dt = (time.perf_counter() - t0) / n
        rp = np.ctypeslib.as_array(A.rowptr, shape=(A.n + 1,)).copy()
        cc = np.ctypeslib.as_array(A.col, shape=(A.nnz,)).copy()
        val = np.ctypeslib.as_array(A.val, shape=(A.nnz,)).copy()
        nn = A.n
        L.orc_csr_free(C.byref(A))
        return dt, int(L.orc_num_threads()), sp.csr_matrix((val, cc, rp), shape=(nn, nn)), r

    def newton(self, op, u, reduction=1e-9, abs_limit=1e-12, min_linear_reduction=1e-8, maxit=50,
               line_search_maxit=500, linear_maxit=20000, prec=PREC_NONE, fd=False):
        u = np.ascontiguousarray(u, dtype=np.float64).copy()
        o = OrcNewtonOpts(reduction, abs_limit, min_linear_reduction, maxit, line_search_maxit, 1,
                          linear_maxit, prec, int(fd))
        res = OrcNewtonResult()
        lib().orc_newton(C.byref(self.m), C.byref(self.p), C.byref(op), _p(u), C.byref(o),
                         C.byref(res))
        return u, res


class PkSpace:
    """The oracle's own Lagrange P_k space on a Problem's mesh (pnp_oracle_pk.c) and the scalar
    operators of the operator-split driver on it.  Vectors are over the space's nn nodes."""

    def __init__(self, prob: Problem, k):
        self.prob, self.k = prob, int(k)
        self.S = OrcPk()
        rc = lib().orc_pk_build(C.byref(prob.m), self.k, C.byref(self.S))
        assert rc == 0, rc
        self.nn, self.nl = self.S.nn, self.S.nl
        self.xy = np.ctypeslib.as_array(self.S.xy, shape=(self.nn, 2)).copy()
        self.enode = np.ctypeslib.as_array(self.S.enode, shape=(prob.mesh.nt, self.nl)).copy()

    def __del__(self):
        try:
            lib().orc_pk_free(C.byref(self.S))
        except Exception:
            pass

    def mask(self, field=0):
        out = np.zeros(self.nn, dtype=np.uint8)
        lib().orc_pk_dirichlet_mask(C.byref(self.prob.m), C.byref(self.S), C.byref(self.prob.p),
                                    int(field), _p(out))
        return out

    def residual(self, op, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        r = np.zeros(self.nn)
        lib().orc_pk_residual(C.byref(self.prob.m), C.byref(self.S), C.byref(self.prob.p),
                              C.byref(op), _p(x), _p(r))
        return r

    def jacobian(self, op, x, fd=False):
        import scipy.sparse as sp
        x = np.ascontiguousarray(x, dtype=np.float64)
        A = OrcCsr()
        L = lib()
        L.orc_pk_csr_pattern(C.byref(self.prob.m), C.byref(self.S), C.byref(A))
        L.orc_pk_jacobian(C.byref(self.prob.m), C.byref(self.S), C.byref(self.prob.p),
                          C.byref(op), _p(x), int(fd), C.byref(A))
        n, nnz = A.n, A.nnz
        rp = np.ctypeslib.as_array(A.rowptr, shape=(n + 1,)).copy()
        col = np.ctypeslib.as_array(A.col, shape=(nnz,)).copy()
        val = np.ctypeslib.as_array(A.val, shape=(nnz,)).copy()
        L.orc_csr_free(C.byref(A))
        return sp.csr_matrix((val, col, rp), shape=(n, n))

    def initial_state(self, phi_pb):
        out = np.zeros(3 * self.nn)
        phi = None if phi_pb is None else np.ascontiguousarray(phi_pb, dtype=np.float64)
        lib().orc_pk_initial_state(C.byref(self.prob.m), C.byref(self.S), C.byref(self.prob.p),
                                   _p(phi), _p(out))
        return out

    def ion_flux(self, x):
        n = self.prob.p.nsurf
        ip, im = np.zeros(n), np.zeros(n)
        x = np.ascontiguousarray(x, dtype=np.float64)
        lib().orc_pk_ion_flux(C.byref(self.prob.m), C.byref(self.S), C.byref(self.prob.p), _p(x),
                              _p(ip), _p(im))
        return ip, im

    def basis(self, xi, eta):
        phi = np.zeros(self.nl)
        dphi = np.zeros((self.nl, 2))
        lib().orc_pk_basis(self.k, C.c_double(xi), C.c_double(eta), _p(phi), _p(dphi))
        return phi, dphi

    def newton(self, op, u, reduction=1e-10, maxit=30):
        """Plain Newton with exact sparse solves on the oracle's residual / analytic Jacobian
        (PB on P_k: PDELab's line search never shortens a step on these problems)."""
        import scipy.sparse.linalg as spla
        u = np.array(u, dtype=np.float64)
        r = self.residual(op, u)
        d0 = np.linalg.norm(r)
        for _ in range(maxit):
            if np.linalg.norm(r) <= reduction * d0 or np.linalg.norm(r) < 1e-14:
                break
            J = self.jacobian(op, u)
            u -= spla.spsolve(J.tocsc(), r)
            r = self.residual(op, u)
        return u


def quadrature_rule(order):
    """(xi, eta, w) of the oracle's simplex rule for an intorder (orc_quadrature_rule)."""
    xi, eta, w = np.zeros(7), np.zeros(7), np.zeros(7)
    n = lib().orc_quadrature_rule(int(order), _p(xi), _p(eta), _p(w))
    return xi[:n], eta[:n], w[:n]


def bicgstab(A, b, prec=PREC_NONE, reduction=1e-8, maxit=20000, x0=None):
    """ISTL-semantics BiCGStab on a scipy CSR matrix (sorted indices)."""
    return _krylov("orc_bicgstab", A, b, prec, reduction, maxit, x0)


def cg(A, b, prec=PREC_NONE, reduction=1e-8, maxit=20000, x0=None):
    """ISTL-semantics CG (CGSolver) on a scipy CSR matrix."""
    return _krylov("orc_cg", A, b, prec, reduction, maxit, x0)


def _csr(A):
    A = A.tocsr()
    A.sort_indices()
    rp = np.ascontiguousarray(A.indptr, dtype=np.int32)
    col = np.ascontiguousarray(A.indices, dtype=np.int32)
    val = np.ascontiguousarray(A.data, dtype=np.float64)
    M = OrcCsr(A.shape[0], A.nnz, rp.ctypes.data_as(C.POINTER(C.c_int)),
               col.ctypes.data_as(C.POINTER(C.c_int)), val.ctypes.data_as(C.POINTER(C.c_double)))
    return M, (rp, col, val)


def prec_apply(A, d, prec):
    """v = W^{-1} d: one application of the oracle's preconditioner (ISTL SeqSSOR / SeqILU0 /
    Jacobi) from v = 0, as inside its BiCGSTAB."""
    M, keep = _csr(A)
    dd = np.ascontiguousarray(d, dtype=np.float64)
    v = np.zeros(A.shape[0])
    lib().orc_prec_apply(C.byref(M), prec, _p(dd), _p(v))
    return v


def _krylov(fn, A, b, prec, reduction, maxit, x0):
    A = A.tocsr()
    A.sort_indices()
    rp = np.ascontiguousarray(A.indptr, dtype=np.int32)
    col = np.ascontiguousarray(A.indices, dtype=np.int32)
    val = np.ascontiguousarray(A.data, dtype=np.float64)
    M = OrcCsr(A.shape[0], A.nnz, rp.ctypes.data_as(C.POINTER(C.c_int)),
               col.ctypes.data_as(C.POINTER(C.c_int)), val.ctypes.data_as(C.POINTER(C.c_double)))
    x = np.zeros(A.shape[0]) if x0 is None else np.array(x0, dtype=np.float64)
    bb = np.array(b, dtype=np.float64)
    res = OrcSolveResult()
    getattr(lib(), fn)(C.byref(M), prec, C.c_double(reduction), maxit, _p(x), _p(bb),
                       C.byref(res))
    return x, res
