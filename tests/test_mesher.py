"""The .geo reader + mesher standing in for gmsh (geo_mesh.cc).

The reference's config 5 (test/pore_without_dna/pore.cfg:21) names pore_without_dna.msh, which
only exists as test/pore_without_dna/pore_without_dna.geo: the reference's workflow meshes it
with gmsh first.  No gmsh here and no .msh anywhere, so the mesh itself is not pinned to a
reference output ("parity unpinned" for the vertex positions); what is checked is what the
solver depends on: the geometry (area, boundary lengths per physical group), the validity of
the triangulation, the element quality, and determinism.
"""
import os

import numpy as np
import pytest

import pnp_amd as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEO = os.path.join(ROOT, "data", "pore_without_dna", "pore_without_dna.geo")


def _angles(m):
    xy, t = m.xy, m.tri

    def ang(p, q, r):
        u, v = q - p, r - p
        c = (u * v).sum(1) / np.linalg.norm(u, axis=1) / np.linalg.norm(v, axis=1)
        return np.degrees(np.arccos(np.clip(c, -1, 1)))
    a, b, c = xy[t[:, 0]], xy[t[:, 1]], xy[t[:, 2]]
    return np.stack([ang(a, b, c), ang(b, c, a), ang(c, a, b)], 1)


def _areas(m):
    xy, t = m.xy, m.tri
    a, b = xy[t[:, 1]] - xy[t[:, 0]], xy[t[:, 2]] - xy[t[:, 0]]
    return 0.5 * (a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0])


@pytest.mark.parametrize("scale", [1.0, 0.5])
def test_pore_without_dna_geometry_and_quality(scale):
    m = P.Mesh.from_geo(GEO, scale)
    ar = _areas(m)
    assert np.all(ar > 0), "triangles are counter-clockwise and non-degenerate"
    # box 100 x 55 minus the membrane 20 x 45, whose two pore-side corners are R = 1 fillets;
    # each fillet is a polyline of n chords (n from the size field: lc 2 -> 1 chord at scale 1)
    L = np.linalg.norm(m.xy[m.bseg[:, 0]] - m.xy[m.bseg[:, 1]], axis=1)
    # fillet chords are the group-0 segments that are neither horizontal nor vertical
    d = m.xy[m.bseg[:, 1]] - m.xy[m.bseg[:, 0]]
    arc = (m.bgroup == 0) & (np.abs(d[:, 0]) > 1e-12) & (np.abs(d[:, 1]) > 1e-12)
    n_chords = arc.sum() // 2
    th = np.pi / 2 / n_chords
    seg_area = 0.5 * (th - np.sin(th))  # circle segment cut off by one chord, R = 1
    exact = 100 * 55 - 20 * 45 + 2 * (1 - np.pi / 4) + 2 * n_chords * seg_area
    assert abs(ar.sum() - exact) <= 1e-9 * exact
    # physical groups (pore_without_dna.geo Physical Line 0..5): lengths
    chord = 2 * n_chords * 2 * np.sin(th / 2)
    expect = {0: 2 * 44 + 18 + chord, 1: 100.0, 2: 55.0, 3: 55.0, 4: 40.0, 5: 40.0}
    got = {int(g): L[m.bgroup == g].sum() for g in np.unique(m.bgroup)}
    assert set(got) == set(expect)
    for g in expect:
        assert abs(got[g] - expect[g]) <= 1e-9 * expect[g], (g, got[g], expect[g])
    # every boundary edge of the triangulation is a boundary segment and vice versa
    e = np.sort(np.concatenate([m.tri[:, [0, 1]], m.tri[:, [1, 2]], m.tri[:, [2, 0]]]), axis=1)
    u, cnt = np.unique(e, axis=0, return_counts=True)
    bnd = {tuple(x) for x in u[cnt == 1]}
    assert bnd == {tuple(x) for x in np.sort(m.bseg, axis=1)}
    assert _angles(m).min() >= 25.0
    # the size field: the smallest lc (2) near the pore, the largest (6) at the box corners
    assert 0.7 * scale < L.min() and L.max() <= 6.0 * scale * 1.15  # segment counts are rounded


def test_mesher_is_deterministic_and_msh_round_trips(tmp_path):
    a = P.Mesh.from_geo(GEO, 1.0)
    b = P.Mesh.from_geo(GEO, 1.0)
    for k in ("xy", "tri", "bseg", "bgroup"):
        assert np.array_equal(getattr(a, k), getattr(b, k))
    f = str(tmp_path / "m.msh")
    a.write_gmsh(f)
    c = P.Mesh.read_gmsh(f)
    for k in ("xy", "tri", "bseg", "bgroup"):
        assert np.array_equal(getattr(a, k), getattr(c, k)), k


def test_config_5_mesh_comes_from_the_geo():
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_without_dna", "pore.cfg"))
    assert cfg.meshfile.endswith("pore_without_dna.msh") and not os.path.exists(cfg.meshfile)
    m = P.Mesh.load(cfg.meshfile)
    assert m.nv == P.Mesh.from_geo(GEO).nv
    assert sorted(set(m.bgroup.tolist())) == list(range(len(cfg.surfaces)))  # surface_0..5
    # ~10 M DOF (config 5): size scale 0.85, 6 refinements -> ~3.3 M vertices
    m85 = P.Mesh.from_geo(GEO, 0.85)
    assert 2.8e6 < m85.nv * 4 ** 6 < 3.8e6


def test_square_with_hole(tmp_path):
    geo = tmp_path / "sq.geo"
    geo.write_text("""
    h = 0.1; /* block comment */
    Point(1) = {0, 0, 0, h}; Point(2) = {1, 0, 0, h}; Point(3) = {1, 1, 0, h}; Point(4) = {0, 1, 0, h};
    Point(5) = {0.5, 0.5, 0, h};  // hole centre
    Point(6) = {0.7, 0.5, 0, h/2}; Point(7) = {0.5, 0.7, 0, h/2}; Point(8) = {0.3, 0.5, 0, h/2};
    Point(9) = {0.5, 0.3, 0, h/2};
    Line(1) = {1, 2}; Line(2) = {2, 3}; Line(3) = {3, 4}; Line(4) = {4, 1};
    Circle(5) = {6, 5, 7}; Circle(6) = {7, 5, 8}; Circle(7) = {8, 5, 9}; Circle(8) = {9, 5, 6};
    Line Loop(10) = {1, 2, 3, 4};
    Curve Loop(11) = {5, 6, 7, 8};
    Plane Surface(12) = {10, 11};
    Physical Line(1) = {1, 2, 3, 4};
    Physical Curve(2) = {5, 6, 7, 8};
    Physical Surface(3) = {12};
    """)
    m = P.Mesh.from_geo(str(geo))
    ar = _areas(m)
    assert np.all(ar > 0)
    L = np.linalg.norm(m.xy[m.bseg[:, 0]] - m.xy[m.bseg[:, 1]], axis=1)
    nh = int((m.bgroup == 2).sum())
    hole = 0.5 * nh * 0.04 * np.sin(2 * np.pi / nh)  # inscribed polygon, R = 0.2
    assert abs(ar.sum() - (1 - hole)) <= 1e-9
    assert abs(L[m.bgroup == 1].sum() - 4) <= 1e-12
    assert abs(L[m.bgroup == 2].sum() - nh * 2 * 0.2 * np.sin(np.pi / nh)) <= 1e-12
    assert _angles(m).min() >= 20.0


@pytest.mark.parametrize("text,msg", [
    ("Point(1) = {0, 0, 0, q};", "unknown name"),
    ("Point(1) = {0, 0, 0, 1}; Spline(2) = {1, 1};", "unsupported"),
    ("Point(1) = {0, 0, 0, 1}; Line(2) = {1, 3};", "unknown point"),
    ("a = 1;", "no Plane Surface"),
])
def test_geo_errors(tmp_path, text, msg):
    geo = tmp_path / "bad.geo"
    geo.write_text(text)
    with pytest.raises(P.PnpError, match=msg):
        P.Mesh.from_geo(str(geo))
