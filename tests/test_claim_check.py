"""CPU checks of the dataflow launches' claim protocols (tools/claim_check.py; VERDICT round 4,
next #3): which protocols always drain under a bounded residency, and the counterexamples for the
ones that do not -- including round 4's removed 8-queue ILU(0) form and the steal rule proposed to
fix it, which is not enough on its own."""
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
import claim_check as CC  # noqa: E402
import pnp_amd as P  # noqa: E402
from conftest import DATA  # noqa: E402


def test_protocols_on_a_layered_dag():
    n, deps = CC.layered_dag(12, 16, 3)
    G = 16
    assert CC.check(n, deps, CC.Static(G), G, G) is None
    assert CC.check(n, deps, CC.Static(G), G, G - 1) is not None  # a non-resident worker's unit
    for R in (1, 3, 16):
        assert CC.check(n, deps, CC.Ticket(), G, R) is None
    home = lambda u: (u * 5) % 8  # noqa: E731
    assert CC.check(n, deps, CC.Queues(8, home), 16, 16) is None  # every queue has readers
    w = CC.check(n, deps, CC.Queues(8, home), 16, 5)  # queues 5..7 have no resident reader
    assert w is not None and w["unclaimed_blockers"], w
    assert CC.check(n, deps, CC.Queues(8, home, steal_ready=True), 16, 5) is not None
    for R in (1, 5, 16):
        assert CC.check(n, deps, CC.Queues(8, home, ready_all=True), 16, R) is None


def _nat_units(mesh, rows_per_unit=8):
    """The natural-SSOR forward sweep of the PB operator (scalar P1 pattern) as ssor_natural.hip
    runs it: rows levelled by the dependency rule of ctx.cc's schedule (a row waits for its
    earlier neighbours), units of up to 8 consecutive rows of one level, in level order; a unit
    depends on the units holding its rows' earlier neighbours."""
    nv = mesh.nv
    t = mesh.tri
    e = np.unique(np.sort(np.concatenate([t[:, [0, 1]], t[:, [1, 2]], t[:, [2, 0]]]), axis=1),
                  axis=0)
    A = sp.csr_matrix((np.ones(2 * len(e)), (np.r_[e[:, 0], e[:, 1]], np.r_[e[:, 1], e[:, 0]])),
                      shape=(nv, nv))
    lev = np.zeros(nv, dtype=np.int64)
    for R in range(nv):
        js = A.indices[A.indptr[R]:A.indptr[R + 1]]
        js = js[js < R]
        lev[R] = lev[js].max() + 1 if len(js) else 0
    order = np.lexsort((np.arange(nv), lev))
    unit_of = np.empty(nv, dtype=np.int64)
    units, cur, cur_lev = [], [], -1
    for R in order:
        if lev[R] != cur_lev or len(cur) == rows_per_unit:
            if cur:
                units.append(cur)
            cur, cur_lev = [], lev[R]
        cur.append(R)
    units.append(cur)
    for u, rows in enumerate(units):
        unit_of[rows] = u
    deps = []
    for u, rows in enumerate(units):
        d = set()
        for R in rows:
            js = A.indices[A.indptr[R]:A.indptr[R + 1]]
            d.update(int(unit_of[j]) for j in js[js < R])
        assert all(p < u for p in d)  # every dependency earlier in the unit order
        deps.append(sorted(d))
    return len(units), deps


def test_natural_ssor_units_drain_with_the_resident_grid():
    """k_ssor_nat_flow / _pipe: wave w takes units w, w + G, ... -- it drains when the whole grid
    is resident (the grid is sized from the occupancy query, 4 workgroups per CU), and a grid
    larger than the residency can hang: why the launch never exceeds the resident count."""
    cfg = P.read_config(os.path.join(DATA, "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile)
    n, deps = _nat_units(mesh)
    G = 24
    assert CC.check(n, deps, CC.Static(G), G, G, seeds=4) is None
    assert CC.check(n, deps, CC.Static(G), G, G // 2, seeds=4) is not None
    assert CC.check(n, deps, CC.Ticket(), G, 4, seeds=4) is None


def test_natural_ssor_head_is_probed_before_the_static_schedule():
    """The head's actual protocol since round 6: ssor_natural_flow_resident() first launches the
    head (and chain) kernels in probe mode with their full grid G; only if all G workgroups check
    in at once does the context use the static schedule (wave w: units w, w + G, ...), else the
    level launches (one launch per level, no waits inside a launch: always drains).  So for every
    residency R -- including R < G, where the static schedule alone can hang -- the sweep drains."""
    cfg = P.read_config(os.path.join(DATA, "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile)
    n, deps = _nat_units(mesh)
    G = 24
    for R in (1, 5, G // 2, G - 1, G, 2 * G):
        if CC.probe_arrivals(G, R) >= G:  # probe passed: the static dataflow schedule
            assert R >= G
            assert CC.check(n, deps, CC.Static(G), G, R, seeds=4) is None
        else:  # probe failed: level launches, each a launch without intra-launch waits
            assert R < G
            assert CC.check(n, deps, CC.Static(G), G, R, seeds=2) is not None  # what it avoids
