"""Timing model of the natural-SSOR forward sweep (PB, pore_pnp k=4) under the chain schedule:
head levels as dataflow units (one hop each), tail as heavy-path chains packed into lane groups
(in-register parent: one step; other operands: one hop).  Host-only; hop and step in us."""
import sys, heapq, numpy as np
sys.path.insert(0, 'dune-pnp_amd/python')
import pnp_amd as P
import scipy.sparse as sp
cfg = P.read_config('data/pore_pnp/pore.cfg')
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
nv = mesh.nv; t = mesh.tri
e = np.concatenate([t[:, [0, 1]], t[:, [1, 2]], t[:, [2, 0]]]); e = np.unique(np.sort(e, axis=1), axis=0)
A = sp.csr_matrix((np.ones(len(e)), (e[:, 1], e[:, 0])), shape=(nv, nv))  # lower nbrs (fwd deps)
ip, ix = A.indptr, A.indices
lev = np.zeros(nv, dtype=np.int64)
for i in range(nv):
    if ip[i+1] > ip[i]: lev[i] = lev[ix[ip[i]:ip[i+1]]].max() + 1
nlev = lev.max() + 1
order = np.argsort(lev, kind='stable')
w = np.bincount(lev)
def simulate(T_rows, h=2.5, step=0.35, cap=40000, unit_hop=2.5):
    ltail = nlev
    while T_rows > 0 and ltail > 0 and w[ltail - 1] <= T_rows: ltail -= 1
    tail = order[lev[order] >= ltail]
    parent = np.full(nv, -1); heavy = np.full(nv, -1); hb = np.zeros(nv, dtype=np.int64)
    for R in tail:
        js = ix[ip[R]:ip[R+1]]
        c = js[(lev[js] == lev[R] - 1) & (lev[js] >= ltail)]
        if len(c): parent[R] = c[0]
    for R in tail[::-1]:
        p = parent[R]; hh = 1 + hb[R]
        if p >= 0 and hh > hb[p]: hb[p] = hh; heavy[p] = R
    group = np.full(nv, -1); gprev = {}
    heap = []; ng = 0
    prevrow = np.full(nv, -1); prev2 = np.full(nv, -1)
    grows = []; rr = [0]
    for R in tail:
        if parent[R] >= 0 and heavy[parent[R]] == R: continue
        if heap and heap[0][0] < lev[R]:
            _, g = heapq.heappop(heap)
        elif ng >= cap:
            g = rr[0] % cap; rr[0] += 1
        else:
            g = ng; ng += 1; grows.append([])
        X = R; last = lev[R]
        while X >= 0:
            grows[g].append(X); last = lev[X]; X = heavy[X]
        if ng < cap or True:
            heapq.heappush(heap, (last, g))
    for g, rows in enumerate(grows):
        rows.sort(key=lambda r: lev[r])
        for k, r in enumerate(rows):
            group[r] = g
            if k > 0: prevrow[r] = rows[k-1]
            if k > 1: prev2[r] = rows[k-2]
    T = np.zeros(nv)
    # head: dataflow units: T = max(dep T) + unit_hop
    for l in range(nlev):
        rs = order[ip.size and np.searchsorted(lev[order], l):np.searchsorted(lev[order], l + 1)]
        for R in rs:
            js = ix[ip[R]:ip[R+1]]
            if l < ltail:
                T[R] = (T[js].max() if len(js) else 0.0) + unit_hop
            else:
                tt = 0.0
                for C in js:
                    cost = 0.0 if (C == prevrow[R] or C == prev2[R]) else h
                    tt = max(tt, T[C] + cost)
                if prevrow[R] >= 0: tt = max(tt, T[prevrow[R]])
                T[R] = tt + step
    return T.max(), ltail, ng
for Tr in (4096, 8192, 16384, 32768, 1 << 30):
    tm, lt, ng = simulate(Tr)
    print(f"threshold {Tr}: tail from level {lt}/{nlev}, groups {ng}, modelled fwd sweep {tm:.0f} us")
