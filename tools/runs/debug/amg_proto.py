"""CPU prototype of the aggregation-AMG preconditioner (design study for PNP_PREC_AMG).

The reference's CG_AMG_SSOR variant (src/instationary_pnp_from_pb_md.hh:24,207-210) uses ISTL's
aggregation AMG (ISTLBackend_NOVLP_CG_AMG_SSOR) for the scalar PB/Poisson/diffusion solves; the
PNP system itself runs BiCGStab + SSORk / NOPREC.  This script measures, on the oracle's matrices,
how many Krylov iterations a vertex-block aggregation AMG V-cycle needs compared with ILU(0), for
PB (CG) and PNP (BiCGStab), so the GPU implementation is sized by evidence.

usage: python tools/amg_proto.py [k]      (pore_pnp refined k times, default 2)
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import meshio  # noqa: E402
import oracle_py as O  # noqa: E402
import pnp_amd as P  # noqa: E402


def vertex_graph(nv, tri):
    i = np.concatenate([tri[:, 0], tri[:, 1], tri[:, 2], tri[:, 1], tri[:, 2], tri[:, 0]])
    j = np.concatenate([tri[:, 1], tri[:, 2], tri[:, 0], tri[:, 0], tri[:, 1], tri[:, 2]])
    G = sp.csr_matrix((np.ones(len(i)), (i, j)), shape=(nv, nv))
    G.data[:] = 1
    return G


def aggregate(S, maxsize=0):
    """Greedy aggregation on a strength graph S (csr, no diagonal): roots with all neighbours
    free take them; leftovers join a neighbouring aggregate; isolated ones form singletons."""
    n = S.shape[0]
    agg = -np.ones(n, dtype=np.int64)
    ip, ix = S.indptr, S.indices
    na = 0
    for i in range(n):
        if agg[i] >= 0:
            continue
        nb = ix[ip[i]:ip[i + 1]]
        if np.all(agg[nb] < 0):
            agg[i] = na
            agg[nb[:maxsize - 1] if maxsize else nb] = na
            na += 1
    for i in range(n):
        if agg[i] >= 0:
            continue
        nb = ix[ip[i]:ip[i + 1]]
        a = agg[nb]
        a = a[a >= 0]
        if len(a):
            agg[i] = -2 - a[0]  # mark, resolve after the pass (do not chain)
    m = agg <= -2
    agg[m] = -2 - agg[m]
    for i in range(n):
        if agg[i] < 0:
            agg[i] = na
            na += 1
    return agg, na


class AMG:
    def __init__(self, A, nf, nv, G, theta=0.0, coarse=2000, smoother="ilu0", cs="jacobi",
                 omega=0.7, damp=1.0, sweeps=1, gamma=1, csweeps=1, maxsize=0):
        """A: vertex-interleaved (row = v*nf + f), G: vertex graph (csr)."""
        self.levels = []
        self.nf = nf
        self.damp = damp
        self.sweeps = sweeps
        self.omega = omega
        self.gamma = gamma
        self.csweeps = csweeps
        Al, Gl, lvl = A.tocsr(), G, 0
        while Al.shape[0] // nf > coarse:
            nvl = Al.shape[0] // nf
            # strength from the field-0 block
            A0 = Al[0::nf, 0::nf].tocsr() if nf > 1 else Al
            S = A0.multiply(Gl).tocsr()
            S.eliminate_zeros()
            if theta > 0:
                d = np.abs(A0.diagonal())
                C = S.tocoo()
                keep = np.abs(C.data) >= theta * np.sqrt(d[C.row] * d[C.col])
                S = sp.csr_matrix((C.data[keep], (C.row[keep], C.col[keep])), shape=S.shape)
            S.setdiag(0)
            S.eliminate_zeros()
            agg, na = aggregate(S, maxsize)
            Pv = sp.csr_matrix((np.ones(nvl), (np.arange(nvl), agg)), shape=(nvl, na))
            Pm = sp.kron(Pv, sp.identity(nf), format="csr")
            lev = {"A": Al, "P": Pm, "n": Al.shape[0]}
            kind = smoother if lvl == 0 else cs
            if kind == "ilu0":
                lev["ilu"] = spla.spilu(Al.tocsc(), drop_tol=0, fill_factor=1, permc_spec="NATURAL",
                                        diag_pivot_thresh=0)
            elif kind == "sgs":
                lev["L"] = sp.tril(Al, format="csr")
                lev["U"] = sp.triu(Al, format="csr")
            else:  # block jacobi
                Db = np.zeros((nvl, nf, nf))
                Ac = Al.tocoo()
                m = (Ac.row // nf) == (Ac.col // nf)
                Db[Ac.row[m] // nf, Ac.row[m] % nf, Ac.col[m] % nf] += Ac.data[m]
                lev["Dinv"] = np.linalg.inv(Db)
            lev["kind"] = kind
            self.levels.append(lev)
            Al = (Pm.T @ Al @ Pm).tocsr()
            Gl = (Pv.T @ Gl @ Pv).tocsr()
            Gl.data[:] = 1
            lvl += 1
        self.coarse = spla.splu(Al.tocsc())
        self.nc = Al.shape[0]

    def smooth(self, lev, b, x, forward=True):
        if lev["kind"] == "ilu0":
            return x + lev["ilu"].solve(b - lev["A"] @ x)
        if lev["kind"] == "sgs":
            if forward:
                x = x + spla.spsolve_triangular(lev["L"], b - lev["A"] @ x, lower=True)
                return x + spla.spsolve_triangular(lev["U"], b - lev["A"] @ x, lower=False)
            x = x + spla.spsolve_triangular(lev["U"], b - lev["A"] @ x, lower=False)
            return x + spla.spsolve_triangular(lev["L"], b - lev["A"] @ x, lower=True)
        nf = self.nf
        r = (b - lev["A"] @ x).reshape(-1, nf)
        return x + self.omega * np.einsum("vij,vj->vi", lev["Dinv"], r).ravel()

    def vcycle(self, l, b):
        if l == len(self.levels):
            return self.coarse.solve(b)
        lev = self.levels[l]
        x = np.zeros_like(b)
        ns = self.sweeps if l == 0 else self.csweeps
        for _ in range(ns):
            x = self.smooth(lev, b, x, True)
        for g in range(self.gamma if l > 0 else 1):
            r = b - lev["A"] @ x
            e = self.vcycle(l + 1, lev["P"].T @ r)
            x = x + self.damp * (lev["P"] @ e)
        for _ in range(ns):
            x = self.smooth(lev, b, x, False)
        return x

    def op(self):
        n = self.levels[0]["n"]
        return spla.LinearOperator((n, n), matvec=lambda b: self.vcycle(0, b))


def count(solver, A, b, M, rtol):
    it = [0]

    def cb(_):
        it[0] += 1
    t = time.perf_counter()
    x, info = solver(A, b, rtol=rtol, atol=0, maxiter=20000, M=M, callback=cb)
    return it[0], info, np.linalg.norm(A @ x - b) / np.linalg.norm(b), time.perf_counter() - t


QUICK = os.environ.get("QUICK") == "1"
SM_PB = ("sgs",) if QUICK else ("sgs", "ilu0")
SM_PNP = ("ilu0",) if QUICK else ("ilu0", "sgs")
CS = ("jacobi",) if QUICK else ("jacobi", "sgs", "ilu0")
DAMP = (1.0,) if QUICK else (1.0, 1.6)


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.load(cfg.meshfile).refine(k)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    nv = mesh.nv
    G = vertex_graph(nv, np.asarray(mesh.tri))
    print(f"pore_pnp k={k}: nv={nv}")
    # PB (scalar, SPD): CG
    pbop = orc.operator(O.OP_PB, flux=orc.flux(), mask=orc.mask(1))
    phi, _ = orc.newton(pbop, np.zeros(nv), prec=O.PREC_ILU0)
    J = orc.jacobian(pbop, phi).tocsr()
    b = np.random.default_rng(1).standard_normal(nv)
    b[orc.mask(1) != 0] = 0
    ilu = spla.spilu(J.tocsc(), drop_tol=0, fill_factor=1, permc_spec="NATURAL", diag_pivot_thresh=0)
    Milu = spla.LinearOperator(J.shape, matvec=ilu.solve)
    print("PB  bicgstab ilu0   its=%d info=%d res=%.1e %.2fs" % count(spla.bicgstab, J, b, Milu, 1e-8))
    for sm in SM_PB:
        for cs in CS:
            for damp in DAMP:
                amg = AMG(J, 1, nv, G, smoother=sm, cs=cs, damp=damp)
                r = count(spla.cg if sm == "sgs" and cs != "ilu0" else spla.bicgstab, J, b,
                          amg.op(), 1e-8)
                print(f"PB  amg sm={sm} cs={cs} damp={damp} levels={len(amg.levels)} nc={amg.nc} "
                      "its=%d info=%d res=%.1e %.2fs" % r)
    # PNP at the Boltzmann initial state: BiCGStab
    x0 = orc.initial_state(phi)
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    r0 = orc.residual(op, x0)
    Jl = orc.jacobian(op, x0).tocsr()
    perm = np.array([f * nv + v for v in range(nv) for f in range(3)])  # vertex-interleaved
    Jp = Jl[perm][:, perm].tocsr()
    bp = r0[perm]
    ilu = spla.spilu(Jp.tocsc(), drop_tol=0, fill_factor=1, permc_spec="NATURAL", diag_pivot_thresh=0)
    Milu = spla.LinearOperator(Jp.shape, matvec=ilu.solve)
    print("PNP bicgstab ilu0   its=%d info=%d res=%.1e %.2fs" % count(spla.bicgstab, Jp, bp, Milu, 1e-8))
    for sm in SM_PNP:
        for cs in CS:
            for damp in DAMP:
                amg = AMG(Jp, 3, nv, G, smoother=sm, cs=cs, damp=damp)
                r = count(spla.bicgstab, Jp, bp, amg.op(), 1e-8)
                print(f"PNP amg sm={sm} cs={cs} damp={damp} levels={len(amg.levels)} nc={amg.nc} "
                      "its=%d info=%d res=%.1e %.2fs" % r)


if __name__ == "__main__":
    main()
