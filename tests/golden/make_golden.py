"""Independent numpy restatement of the dune-pnp hot path -> golden fixtures (tests/golden/*.npz).

Run in the dev container only:  python tests/golden/make_golden.py
The committed .npz files are data (inputs + expected outputs); this script is how they were made.

It is written separately from oracle/pnp_oracle.c (vectorised over elements instead of the
reference's per-element loop) so that the two restatements check each other:
  * residuals   : PnpOperator (src/pnp_operator.hh:46-315), PnpTOperator (src/pnp_toperator.hh:
                  31-101), PBOperator (src/pb_operator.hh:46-194), DiffusionOperator
                  (src/diffusion_operator.hh:42-112), PoissonOperator (src/poisson_operator.hh)
  * Jacobians   : analytic, and PDELab NumericalJacobianVolume forward differences (eps 1e-7)
  * constraints : BCType (src/btype.hh:21-53) -> zero residual rows / identity Jacobian rows
  * solvers     : ISTL BiCGSTABSolver + SeqILU0 / SeqSSOR, PDELab Newton (accept-best)
Quadrature: order 3 -> Strang-Fix 4-point (dune-geometry SimplexQuadraturePoints<2> m=4),
order 2 -> 3-point rule, faces -> 2-point Gauss.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import meshio  # noqa: E402

REF = "/root/reference/test"
PI = 3.1415  # Q4, src/pnp_operator.hh:20
SEED = 20261015

Q3 = (np.array([[1 / 3, 1 / 3], [0.6, 0.2], [0.2, 0.6], [0.2, 0.2]]),
      np.array([-27 / 96, 25 / 96, 25 / 96, 25 / 96]))
Q2 = (np.array([[2 / 3, 1 / 6], [1 / 6, 2 / 3], [1 / 6, 1 / 6]]), np.array([1 / 6] * 3))
GL2 = (np.array([0.5 - 0.5 / np.sqrt(3), 0.5 + 0.5 / np.sqrt(3)]), np.array([0.5, 0.5]))


class Geo:
    def __init__(self, m):
        p = m.xy[m.tri]  # [nt,3,2]
        self.p = p
        J = np.stack([p[:, 1] - p[:, 0], p[:, 2] - p[:, 0]], axis=-1)  # [nt,2(x/y),2(xi/eta)]
        self.det = J[:, 0, 0] * J[:, 1, 1] - J[:, 0, 1] * J[:, 1, 0]
        self.adet = np.abs(self.det)
        Jinv = np.linalg.inv(J)                     # [nt,2,2]
        gh = np.array([[-1.0, -1.0], [1.0, 0.0], [0.0, 1.0]])
        self.g = np.einsum("eij,ai->eaj", Jinv, gh)  # (J^{-T} grad_hat)_j = sum_i Jinv_ij gh_i
        self.tri = m.tri
        self.J = J

    def y_at(self, xi):
        return self.p[:, 0, 1] + self.J[:, 1, 0] * xi[0] + self.J[:, 1, 1] * xi[1]


def psi_at(xi):
    return np.array([1 - xi[0] - xi[1], xi[0], xi[1]])


def factors(G, rule, cyl):
    pts, w = rule
    out = []
    for q in range(len(w)):
        f = w[q] * G.adet
        if cyl:
            f = f * G.y_at(pts[q]) * 2 * PI
        out.append(f)
    return out


def scatter(m, nf, loc):
    """loc: [nt, nf, 3] -> global vector (lexicographic fields)."""
    r = np.zeros(nf * m.nv)
    for f in range(nf):
        np.add.at(r, f * m.nv + m.tri, loc[:, f, :])
    return r


def local(m, nf, x):
    return np.stack([x[f * m.nv + m.tri] for f in range(nf)], axis=1)  # [nt,nf,3]


# ----------------------------------------------------------------------------------------------
# element residuals (vectorised); xl: [nt, nf, 3]
# ----------------------------------------------------------------------------------------------
def pnp_vol(G, par, xl):
    out = np.zeros_like(xl)
    pts, w = Q3
    fac = factors(G, Q3, par["cyl"])
    gphi = np.einsum("ea,eaj->ej", xl[:, 0], G.g)
    gcp = np.einsum("ea,eaj->ej", xl[:, 1], G.g)
    gcm = np.einsum("ea,eaj->ej", xl[:, 2], G.g)
    gp_i = np.einsum("ej,eij->ei", gphi, G.g)
    for q in range(len(w)):
        ps = psi_at(pts[q])
        ucp, ucm = xl[:, 1] @ ps, xl[:, 2] @ ps
        f = fac[q][:, None]
        out[:, 0] += (gp_i + 4 * PI * par["l_b"] * (ucp - ucm)[:, None] * ps[None]) * f
        out[:, 1] += (np.einsum("ej,eij->ei", gcp, G.g) - ucp[:, None] * gp_i) * f
        out[:, 2] += (np.einsum("ej,eij->ei", gcm, G.g) + ucm[:, None] * gp_i) * f
    return out


def pnpt_vol(G, par, xl):
    out = np.zeros_like(xl)
    pts, w = Q2
    fac = factors(G, Q2, par["cyl"])
    for q in range(len(w)):
        ps = psi_at(pts[q])
        ucp, ucm = xl[:, 1] @ ps, xl[:, 2] @ ps
        out[:, 1] += par["tau"] * (ucp + ucm)[:, None] * ps[None] * fac[q][:, None]
    return out


def pb_vol(G, par, xl):
    out = np.zeros_like(xl)
    pts, w = Q3
    fac = factors(G, Q3, par["cyl"])
    gu = np.einsum("ea,eaj->ej", xl[:, 0], G.g)
    gg = np.einsum("ej,eij->ei", gu, G.g)
    for q in range(len(w)):
        ps = psi_at(pts[q])
        u = xl[:, 0] @ ps
        out[:, 0] += (gg + 8 * PI * par["l_b"] * par["c0"] * np.sinh(u)[:, None] * ps[None]) * \
            fac[q][:, None]
    return out


def diff_vol(G, z, phil, xl):
    out = np.zeros_like(xl)
    pts, w = Q2
    gu = np.einsum("ea,eaj->ej", xl[:, 0], G.g)
    gP = np.einsum("ea,eaj->ej", phil, G.g)
    gg = np.einsum("ej,eij->ei", gu, G.g)
    gp = np.einsum("ej,eij->ei", gP, G.g)
    for q in range(len(w)):
        ps = psi_at(pts[q])
        u = xl[:, 0] @ ps
        out[:, 0] += (gg + z * u[:, None] * gp) * (w[q] * G.adet)[:, None]
    return out


def poisson_vol(G, par, cpl, cml, xl):
    out = np.zeros_like(xl)
    pts, w = Q3
    fac = factors(G, Q3, par["cyl"])
    gu = np.einsum("ea,eaj->ej", xl[:, 0], G.g)
    gg = np.einsum("ej,eij->ei", gu, G.g)
    for q in range(len(w)):
        ps = psi_at(pts[q])
        cp, cm = cpl @ ps, cml @ ps
        out[:, 0] += (gg + par["l_b"] * 4 * PI * (cm - cp)[:, None] * ps[None]) * fac[q][:, None]
    return out


FACE_V = ((0, 1), (0, 2), (1, 2))  # DUNE reference-triangle faces (local vertex pairs)
CORNER = np.array([[0.0, 0.0], [1.0, 0.0], [0.0, 1.0]])


def boundary(m, par, surfs, nf, scale=1.0):
    """alpha_boundary (src/pnp_operator.hh:198-315) as PDELab assembles it: each boundary segment is
    the face of its element, run from the lower to the higher local vertex; every one of the
    element's three P1 basis functions is evaluated at the face's Gauss points in element
    coordinates (the off-face one is 0 up to rounding) and accumulated with weight `scale`."""
    r = np.zeros(nf * m.nv)
    face_of = {}
    for e, t in enumerate(m.tri):
        for k, (i, j) in enumerate(FACE_V):
            face_of.setdefault((min(t[i], t[j]), max(t[i], t[j])), (e, k))
    ek = np.array([face_of[(min(a, b), max(a, b))] for a, b in m.bseg]).reshape(-1, 2)
    e, k = ek[:, 0], ek[:, 1]
    fv = np.array(FACE_V)[k]
    tv = m.tri[e]
    a = tv[np.arange(len(e)), fv[:, 0]]
    b = tv[np.arange(len(e)), fv[:, 1]]
    d = m.xy[b] - m.xy[a]
    ln = np.hypot(d[:, 0], d[:, 1])
    for q in range(2):
        t = GL2[0][q]
        f = GL2[1][q] * ln
        if par["cyl"]:
            f = f * (m.xy[a, 1] + t * d[:, 1]) * 2 * PI
        loc = CORNER[fv[:, 0]] + (CORNER[fv[:, 1]] - CORNER[fv[:, 0]]) * t
        phi = np.stack([1.0 - loc[:, 0] - loc[:, 1], loc[:, 0], loc[:, 1]], axis=1)
        for fld in range(nf):
            bt = np.array([[s.cb, s.pb, s.mb][fld] for s in surfs])[m.bgroup]
            jf = np.array([[s.cflux, s.pflux, s.mflux][fld] for s in surfs])[m.bgroup]
            on = bt != 0
            for i in range(3):
                np.add.at(r, fld * m.nv + tv[on, i], scale * (jf[on] * phi[on, i] * f[on]))
    return r


def mask_of(m, surfs, nf):
    mk = np.zeros(nf * m.nv, dtype=np.uint8)
    for fld in range(nf):
        bt = np.array([[s.cb, s.pb, s.mb][fld] for s in surfs])[m.bgroup]
        v = m.bseg[bt == 0].ravel()
        mk[fld * m.nv + v] = 1
    return mk


class Op:
    """kind in {pnp, pnp_ie, pb, diff, poisson}"""

    def __init__(self, m, par, surfs, kind, **kw):
        self.m, self.par, self.surfs, self.kind, self.kw = m, par, surfs, kind, kw
        self.G = Geo(m)
        self.nf = 3 if kind.startswith("pnp") else 1
        self.mask = mask_of(m, surfs, self.nf) if kind != "diff" else kw["mask"]
        if kind == "pnp":
            self.bnd = boundary(m, par, surfs, 3)
        elif kind == "pnp_ie":
            self.bnd = boundary(m, par, surfs, 3, scale=kw["dt"])
        elif kind in ("pb", "poisson"):
            self.bnd = boundary(m, par, surfs, 1)
        else:
            self.bnd = np.zeros(m.nv)

    def vol(self, xl):
        k, G, par = self.kind, self.G, self.par
        if k == "pnp":
            return pnp_vol(G, par, xl)
        if k == "pnp_ie":
            return pnpt_vol(G, par, xl) + self.kw["dt"] * pnp_vol(G, par, xl)
        if k == "pb":
            return pb_vol(G, par, xl)
        if k == "diff":
            phil = self.kw["phi"][self.m.tri]
            return diff_vol(G, self.kw["z"], phil, xl)
        if k == "poisson":
            return poisson_vol(G, par, self.kw["cp"][self.m.tri], self.kw["cm"][self.m.tri], xl)
        raise ValueError(k)

    def residual(self, x):
        r = scatter(self.m, self.nf, self.vol(local(self.m, self.nf, x))) + self.bnd
        if self.kind == "pnp_ie":
            r -= scatter(self.m, 3, pnpt_vol(self.G, self.par, local(self.m, 3, self.kw["x_old"])))
        r[self.mask == 1] = 0.0
        return r

    def jacobian(self, x, fd):
        m, nf = self.m, self.nf
        xl = local(m, nf, x)
        nt = m.nt
        nl = 3 * nf
        Jl = np.zeros((nt, nl, nl))
        base = self.vol(xl).reshape(nt, nl)
        if fd:
            for j in range(nl):
                u = xl.reshape(nt, nl).copy()
                delta = 1e-7 * (1.0 + np.abs(u[:, j]))
                u[:, j] += delta
                up = self.vol(u.reshape(nt, nf, 3)).reshape(nt, nl)
                Jl[:, :, j] = (up - base) / delta[:, None]
        else:
            # directional derivative of the (at most quadratic-in-x, or sinh) residual: exact
            # forms per operator
            Jl = self._analytic(xl)
        gidx = np.concatenate([f * m.nv + m.tri for f in range(nf)], axis=1)  # [nt, nl]
        rows = np.repeat(gidx, nl, axis=1).ravel()
        cols = np.tile(gidx, (1, nl)).ravel()
        A = sp.csr_matrix((Jl.reshape(nt, -1).ravel(), (rows, cols)), shape=(nf * m.nv,) * 2)
        A.sum_duplicates()
        A.sort_indices()
        A = A.tolil()
        for i in np.nonzero(self.mask)[0]:
            A.rows[i] = [i]
            A.data[i] = [1.0]
        A = A.tocsr()
        A.sort_indices()
        return A

    def _analytic(self, xl):
        G, par, k = self.G, self.par, self.kind
        nt = xl.shape[0]
        K = np.einsum("eij,ekj->eik", G.g, G.g)  # grad psi_i . grad psi_k
        if k in ("pnp", "pnp_ie"):
            sc = self.kw["dt"] if k == "pnp_ie" else 1.0
            Jl = np.zeros((nt, 9, 9))
            pts, w = Q3
            fac = factors(G, Q3, par["cyl"])
            gphi = np.einsum("ea,eaj->ej", xl[:, 0], G.g)
            gp_i = np.einsum("ej,eij->ei", gphi, G.g)
            for q in range(len(w)):
                ps = psi_at(pts[q])
                f = fac[q][:, None, None]
                ucp, ucm = xl[:, 1] @ ps, xl[:, 2] @ ps
                Kf = K * f
                M = np.outer(ps, ps)[None] * f
                kap = 4 * PI * par["l_b"]
                Jl[:, 0:3, 0:3] += Kf
                Jl[:, 0:3, 3:6] += kap * M
                Jl[:, 0:3, 6:9] -= kap * M
                Jl[:, 3:6, 0:3] -= ucp[:, None, None] * Kf
                Jl[:, 3:6, 3:6] += Kf - gp_i[:, :, None] * ps[None, None, :] * f
                Jl[:, 6:9, 0:3] += ucm[:, None, None] * Kf
                Jl[:, 6:9, 6:9] += Kf + gp_i[:, :, None] * ps[None, None, :] * f
            Jl *= sc
            if k == "pnp_ie":
                pts2, w2 = Q2
                fac2 = factors(G, Q2, par["cyl"])
                for q in range(len(w2)):
                    ps = psi_at(pts2[q])
                    M = par["tau"] * np.outer(ps, ps)[None] * fac2[q][:, None, None]
                    Jl[:, 3:6, 3:6] += M
                    Jl[:, 3:6, 6:9] += M
            return Jl
        Jl = np.zeros((nt, 3, 3))
        if k == "pb":
            pts, w = Q3
            fac = factors(G, Q3, par["cyl"])
            for q in range(len(w)):
                ps = psi_at(pts[q])
                u = xl[:, 0] @ ps
                f = fac[q][:, None, None]
                Jl += K * f + 8 * PI * par["l_b"] * par["c0"] * np.cosh(u)[:, None, None] * \
                    np.outer(ps, ps)[None] * f
            return Jl
        if k == "poisson":
            fac = factors(G, Q3, par["cyl"])
            return K * sum(fac)[:, None, None]
        if k == "diff":
            pts, w = Q2
            gP = np.einsum("ea,eaj->ej", self.kw["phi"][self.m.tri], G.g)
            gp = np.einsum("ej,eij->ei", gP, G.g)
            for q in range(len(w)):
                ps = psi_at(pts[q])
                f = (w[q] * G.adet)[:, None, None]
                Jl += K * f + self.kw["z"] * gp[:, :, None] * ps[None, None, :] * f
            return Jl
        raise ValueError(k)


# ----------------------------------------------------------------------------------------------
# solvers
# ----------------------------------------------------------------------------------------------
def ilu0(A):
    A = A.tocsr().copy()
    A.sort_indices()
    n = A.shape[0]
    ip, ix, v = A.indptr, A.indices, A.data
    diag = np.array([ip[i] + np.searchsorted(ix[ip[i]:ip[i + 1]], i) for i in range(n)])
    for i in range(n):
        for ij in range(ip[i], diag[i]):
            j = ix[ij]
            v[ij] *= v[diag[j]]
            rowj = dict(zip(ix[diag[j] + 1:ip[j + 1]], range(diag[j] + 1, ip[j + 1])))
            for ik in range(ij + 1, ip[i + 1]):
                jk = rowj.get(ix[ik])
                if jk is not None:
                    v[ik] -= v[ij] * v[jk]
        v[diag[i]] = 1.0 / v[diag[i]]
    L = sp.csr_matrix(sp.tril(A, -1))
    U = sp.csr_matrix(sp.triu(A, 1))
    dinv = v[diag]
    import scipy.sparse.linalg as sla
    Lu = (L + sp.eye(n)).tocsr()
    Uu = (U + sp.diags(1.0 / dinv)).tocsr()
    return lambda d: sla.spsolve_triangular(Uu, sla.spsolve_triangular(Lu, d, lower=True),
                                            lower=False)


def bicgstab(A, b, prec, reduction, maxit):
    """ISTL BiCGSTABSolver::apply with x0 = 0; returns x, iterations, converged."""
    Mi = (lambda d: d) if prec == "none" else ilu0(A)
    x = np.zeros_like(b)
    r = b.copy()
    rt = r.copy()
    norm = norm0 = np.linalg.norm(r)
    if norm < reduction * norm0 or norm < 1e-30:
        return x, 0, True
    rho = alpha = omega = 1.0
    p = v = np.zeros_like(b)
    it = 0.5
    conv = False
    while it < maxit:
        rho_new = rt @ r
        if abs(rho) <= 1e-80 or abs(omega) <= 1e-80:
            break
        p = r.copy() if it < 1 else (rho_new / rho) * (alpha / omega) * (p - omega * v) + r
        y = Mi(p)
        v = A @ y
        h = rt @ v
        alpha = rho_new / h
        x = x + alpha * y
        r = r - alpha * v
        if np.linalg.norm(r) < reduction * norm0:
            conv = True
            break
        it += 0.5
        y = Mi(r)
        t = A @ y
        omega = (t @ r) / (t @ t)
        x = x + omega * y
        r = r - omega * t
        rho = rho_new
        nr = np.linalg.norm(r)
        if nr < reduction * norm0 or nr < 1e-30:
            conv = True
            break
        it += 0.5
    return x, int(np.ceil(min(it, maxit))), conv


def newton(op, u, prec, reduction=1e-9, min_lin=1e-8, maxit=50, ls_maxit=500, abs_limit=1e-12,
           lin_maxit=20000):
    u = u.copy()
    r = op.residual(u)
    d = d0 = prev = np.linalg.norm(r)
    its = 0
    lin_total = 0
    while True:
        if d < abs_limit or d < d0 * reduction:
            return u, its, lin_total, True
        if its >= maxit:
            return u, its, lin_total, False
        A = op.jacobian(u, fd=False)
        stop = max(d0 * reduction, abs_limit)
        if stop / (10 * d) > d * d / (prev * prev):
            lr = stop / (10 * d)
        else:
            lr = min(min_lin, d * d / (prev * prev))
        prev = d
        z, li, conv = bicgstab(A, r, prec, lr, lin_maxit)
        lin_total += li
        if not conv:
            return u, its, lin_total, False
        lam, best_lam, best_d = 1.0, 0.0, d
        prevu = u.copy()
        i = 0
        while True:
            u = prevu - lam * z
            r = op.residual(u)
            d = np.linalg.norm(r)
            if d <= (1 - lam / 4) * prev:
                break
            if d < best_d:
                best_d, best_lam = d, lam
            i += 1
            if i >= ls_maxit:
                u = prevu - best_lam * z
                r = op.residual(u)
                d = np.linalg.norm(r)
                break
            lam *= 0.5
        its += 1


# ----------------------------------------------------------------------------------------------
# fixtures
# ----------------------------------------------------------------------------------------------
def cfg_surfaces(path):
    return meshio.read_config(path)


def synthetic_x(nv, nf, seed=SEED):
    rng = np.random.default_rng(seed)
    phi = rng.uniform(-1.0, 1.0, nv)
    if nf == 1:
        return phi
    cp = 0.06 * rng.uniform(0.5, 1.5, nv)
    cm = 0.06 * rng.uniform(0.5, 1.5, nv)
    return np.concatenate([phi, cp, cm])


def csr_pack(prefix, A, out):
    A = A.tocsr()
    A.sort_indices()
    out[prefix + "_indptr"] = A.indptr.astype(np.int32)
    out[prefix + "_indices"] = A.indices.astype(np.int32)
    out[prefix + "_data"] = A.data


def mesh_pack(m, out):
    out["xy"], out["tri"], out["bseg"], out["bgroup"] = m.xy, m.tri, m.bseg, m.bgroup


def make_case(name, cfgpath, refine, kinds, newton_kinds=(), mesh_override=None, jac=True):
    cfg = meshio.read_config(cfgpath)
    m = meshio.refine(meshio.read_gmsh(mesh_override or cfg.meshfile), refine)
    s = cfg.system
    par = {"l_b": s["l_b"], "c0": s["c0"], "tau": s["tau"], "cyl": int(s["cylindrical"])}
    out = {"params": np.array([par["l_b"], par["c0"], par["tau"], par["cyl"], PI])}
    out["surfaces"] = np.array([[sf.cb, sf.cflux, sf.cpot, sf.pb, sf.pflux, sf.pconc, sf.mb,
                                 sf.mflux, sf.mconc] for sf in cfg.surfaces])
    mesh_pack(m, out)
    for kind in kinds:
        nf = 3 if kind.startswith("pnp") else 1
        x = synthetic_x(m.nv, nf)
        kw = {}
        if kind == "pnp_ie":
            kw = {"dt": s["tau"], "x_old": synthetic_x(m.nv, 3, SEED + 1)}
            out["pnp_ie_x_old"] = kw["x_old"]
        if kind == "diff":
            kw = {"z": -1.0, "phi": synthetic_x(m.nv, 1, SEED + 2),
                  "mask": mask_of(m, cfg.surfaces, 3)[2 * m.nv:]}
            out["diff_phi"] = kw["phi"]
        if kind == "poisson":
            xx = synthetic_x(m.nv, 3, SEED + 3)
            kw = {"cp": xx[m.nv:2 * m.nv], "cm": xx[2 * m.nv:]}
            out["poisson_cp"], out["poisson_cm"] = kw["cp"], kw["cm"]
        op = Op(m, par, cfg.surfaces, kind, **kw)
        out[kind + "_x"] = x
        out[kind + "_mask"] = op.mask
        out[kind + "_r"] = op.residual(x)
        if jac:
            csr_pack(kind + "_J", op.jacobian(x, fd=False), out)
            csr_pack(kind + "_Jfd", op.jacobian(x, fd=True), out)
    for kind, prec in newton_kinds:
        if kind == "pb":
            op = Op(m, par, cfg.surfaces, "pb")
            u, its, lin, conv = newton(op, np.zeros(m.nv), prec)
            out["newton_pb_u"] = u
            out["newton_pb_info"] = np.array([its, lin, conv])
        if kind == "pnp":
            # initial state: BCExtension with phi_pb = 0 (the test passes the same phi to both)
            opb = Op(m, par, cfg.surfaces, "pb")
            upb, _, _, _ = newton(opb, np.zeros(m.nv), prec)
            out["newton_pnp_phi_pb"] = upb
            op = Op(m, par, cfg.surfaces, "pnp")
            # restated Dirichlet/Boltzmann extension for the start value (vertex-wise form:
            # Dirichlet value on constrained vertices, Boltzmann elsewhere)
            mk = op.mask
            x0 = np.concatenate([upb, s["c0"] * np.exp(-upb), s["c0"] * np.exp(upb)])
            for fld in range(3):
                for sfi, sf in enumerate(cfg.surfaces):
                    bt = [sf.cb, sf.pb, sf.mb][fld]
                    val = [sf.cpot, sf.pconc, sf.mconc][fld]
                    if bt == 0:
                        v = m.bseg[m.bgroup == sfi].ravel()
                        x0[fld * m.nv + v] = val
            out["newton_pnp_x0"] = x0
            u, its, lin, conv = newton(op, x0, prec)
            out["newton_pnp_u"] = u
            out["newton_pnp_info"] = np.array([its, lin, conv])
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    return path


CASES = [
    # name, cfg, refine, residual/Jacobian kinds, newton runs
    ("cylinder_k0", f"{REF}/cylinder_config.cfg", 0, ["pnp", "pb"], [("pnp", "ilu0")]),
    ("pore_small_k0", f"{REF}/pore_pnp/pore.cfg", 0, ["pnp", "pnp_ie", "pb", "diff", "poisson"],
     [("pb", "ilu0"), ("pnp", "ilu0")], f"{REF}/pore.msh", True),
    ("pore_pnp_k0", f"{REF}/pore_pnp/pore.cfg", 0, ["pnp", "pb"], [], None, False),
    ("sphere_k0", f"{REF}/sphere_pb/sphere.cfg", 0, ["pb"], [("pb", "ilu0")]),
    ("one_wall_k1", f"{REF}/one_wall_dh/one_wall.cfg", 1, ["pnp", "pb"], [("pb", "ilu0")]),
]


def main():
    manifest = {}
    for case in CASES:
        p = make_case(*case)
        manifest[os.path.basename(p)] = hashlib.sha256(open(p, "rb").read()).hexdigest()
        print(p, os.path.getsize(p))
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump({"seed": SEED, "generator": "tests/golden/make_golden.py", "sha256": manifest},
                  f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
