"""Dependency structure of ISTL SeqSSOR in the reference's DOF order (PNP_PREC_SSOR_NATURAL) on
pore_pnp refined k times: per sweep the level count (longest chain of row dependencies), the split
into wide and narrow levels, and the combined forward + backward critical path.  Host-only (numpy /
scipy), the same dependency rule as ctx.cc's schedule.  usage: python tools/nat_dag.py [k] [T]"""
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
nv = mesh.nv
t = mesh.tri
e = np.concatenate([t[:, [0, 1]], t[:, [1, 2]], t[:, [2, 0]]])
e = np.unique(np.sort(e, axis=1), axis=0)
adj = sp.csr_matrix((np.ones(2 * len(e)), (np.r_[e[:, 0], e[:, 1]], np.r_[e[:, 1], e[:, 0]])),
                    shape=(nv, nv))
ip, ix = adj.indptr, adj.indices


def fields_of(f, nf):
    # PNP blocks: the phi row couples phi, c+, c-; a c row couples phi and its own species
    return (0,) if nf == 1 else ((0, 1, 2) if f == 0 else (0, f))


def levels(nf, fwd, lf=None):
    """level of each row; with lf (the forward levels) the backward sweep's combined level"""
    n = nf * nv
    lev = np.zeros(n, dtype=np.int64)
    for R in (range(n) if fwd else range(n - 1, -1, -1)):
        f, i = divmod(R, nv)
        best = -1 if lf is None else lf[R]
        for g in fields_of(f, nf):
            js = np.concatenate([ix[ip[i]:ip[i + 1]], [i]]) + g * nv
            js = js[js < R] if fwd else js[js > R]
            if len(js):
                best = max(best, lev[js].max())
        lev[R] = best + 1
    return lev


def segments(lev):
    w = np.bincount(lev)
    segs = []
    for x in w:
        wide = bool(x > T)
        if segs and segs[-1][0] == wide:
            segs[-1][1] += 1
            segs[-1][2] += int(x)
        else:
            segs.append([wide, 1, int(x)])
    return len(w), int(np.median(w)), segs


print(f"pore_pnp k={k}: {nv} vertices; wide = more than {T} rows")
for name, nf in (("PB", 1), ("PNP", 3)):
    lf = levels(nf, True)
    lb = levels(nf, False)
    comb = levels(nf, False, lf)
    for d, lev in (("forward", lf), ("backward", lb)):
        n, med, segs = segments(lev)
        print(f"{name} {d}: {n} levels, median width {med}, segments (wide?, levels, rows) "
              f"{[tuple(s) for s in segs]}")
    print(f"{name} critical path forward + backward: {comb.max() + 1} hops "
          f"(sum of depths {lf.max() + lb.max() + 2})")
