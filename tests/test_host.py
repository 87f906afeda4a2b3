"""CPU tests of the product's host side (libpnp_amd.so, no GPU calls): the C ABI loads and
exports every declared symbol, the gmsh reader / refinement / config reader agree with the
independent test-side readers, boundary setup and BCExtension agree with the oracle, and the
fan / colouring / SELL / partition / halo structures are consistent."""
import os

import numpy as np
import pytest

import meshio
import oracle_py as O
import pnp_amd as P
from conftest import DATA

MESHES = ["pore_pnp/pore.msh", "pore.msh", "cylinder.msh", "sphere_pb/sphere.msh",
          "one_wall_dh/one_wall.msh"]
CFGS = ["pore_pnp/pore.cfg", "cylinder_config.cfg", "sphere_pb/sphere.cfg",
        "one_wall_dh/one_wall.cfg", "pore_without_dna/pore.cfg"]


def test_library_exports_every_header_symbol():
    L = P.lib()
    syms = P.header_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(L, s), s


@pytest.mark.parametrize("rel", MESHES)
def test_gmsh_reader_matches_test_reader(rel):
    a = P.Mesh.read_gmsh(os.path.join(DATA, rel))
    b = meshio.read_gmsh(os.path.join(DATA, rel))
    np.testing.assert_array_equal(a.xy, b.xy)
    np.testing.assert_array_equal(a.tri, b.tri)
    np.testing.assert_array_equal(a.bseg, b.bseg)
    np.testing.assert_array_equal(a.bgroup, b.bgroup)


def test_refinement_matches_and_counts():
    a = P.Mesh.read_gmsh(os.path.join(DATA, "pore_pnp/pore.msh"))
    b = meshio.read_gmsh(os.path.join(DATA, "pore_pnp/pore.msh"))
    a2, b2 = a.refine(2), meshio.refine(b, 2)
    np.testing.assert_array_equal(a2.xy, b2.xy)
    np.testing.assert_array_equal(a2.tri, b2.tri)
    np.testing.assert_array_equal(a2.bseg, b2.bseg)
    np.testing.assert_array_equal(a2.bgroup, b2.bgroup)
    # pore_pnp k=3 -> V = 185,209
    assert a.refine(3).nv == 185209


@pytest.mark.parametrize("rel", CFGS)
def test_config_reader_matches(rel):
    a = P.read_config(os.path.join(DATA, rel))
    b = meshio.read_config(os.path.join(DATA, rel))
    assert os.path.normpath(a.meshfile) == os.path.normpath(b.meshfile)
    for k, v in b.system.items():
        assert a.system[k] == pytest.approx(v), k
    assert sorted(P.defaulted_keys(a)) == sorted(b.defaulted)
    assert len(a.surfaces) == len(b.surfaces)
    for sa, sb in zip(a.surfaces, b.surfaces):
        for f in ("cb", "cflux", "cpot", "pb", "pflux", "pconc", "mb", "mflux", "mconc"):
            assert getattr(sa, f) == pytest.approx(getattr(sb, f))


def _problem(rel_cfg, k=0):
    cfg = P.read_config(os.path.join(DATA, rel_cfg))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(k)
    par = P.Params.from_config(cfg)
    s = cfg.system
    orc = O.Problem(meshio.Mesh(mesh.xy, mesh.tri, mesh.bseg, mesh.bgroup), cfg.surfaces,
                    l_b=s["l_b"], c0=s["c0"], tau=s["tau"], cylindrical=s["cylindrical"])
    return cfg, mesh, par, orc


@pytest.mark.parametrize("rel_cfg", ["pore_pnp/pore.cfg", "cylinder_config.cfg",
                                     "one_wall_dh/one_wall.cfg"])
def test_boundary_setup_matches_oracle(rel_cfg):
    cfg, mesh, par, orc = _problem(rel_cfg, 1)
    mask, load = P.setup_boundary(mesh, par, 3, 0)
    np.testing.assert_array_equal(mask, orc.mask(3))
    # oracle: R(0) of PnpOperator = Neumann load (volume terms vanish at x = 0), masked rows 0
    op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
    r0 = orc.residual(op, np.zeros(3 * mesh.nv))
    free = mask == 0
    np.testing.assert_allclose(load[free], r0[free], rtol=1e-13, atol=1e-14)


@pytest.mark.parametrize("rel_cfg,k", [("pore_pnp/pore.cfg", 0), ("pore_pnp/pore.cfg", 1),
                                       ("cylinder_config.cfg", 0), ("sphere_pb/sphere.cfg", 1)])
def test_initial_state_matches_oracle(rel_cfg, k):
    cfg, mesh, par, orc = _problem(rel_cfg, k)
    phi = np.random.default_rng(3).uniform(-1, 1, mesh.nv)
    a = P.setup_initial_state(mesh, par, phi)
    b = orc.initial_state(phi)
    np.testing.assert_array_equal(a, b)


def _mesh_edges(mesh):
    e = np.sort(np.concatenate([mesh.tri[:, [0, 1]], mesh.tri[:, [1, 2]], mesh.tri[:, [0, 2]]]),
                axis=1)
    return set(map(tuple, np.unique(e, axis=0).tolist()))


@pytest.mark.parametrize("rel,k", [("pore_pnp/pore.msh", 0), ("cylinder.msh", 1),
                                   ("one_wall_dh/one_wall.msh", 2)])
def test_fans_sell_and_colouring(rel, k):
    mesh = P.Mesh.read_gmsh(os.path.join(DATA, rel)).refine(k)
    L = P.Layout(mesh)
    assert L.n_owned == mesh.nv and L.n_ghost == 0
    assert sorted(L.l2g.tolist()) == list(range(mesh.nv))
    edges = _mesh_edges(mesh)
    assert L.nblocks == mesh.nv + 2 * len(edges)
    tris = set(tuple(sorted(t)) for t in mesh.tri.tolist())
    seen = {}
    same = 0
    color = L.rowcolor[:L.n_owned].astype(np.int64)
    assert np.all(L.rowcolor[L.n_owned:] == 255)
    for c in range(L.ncolors):
        rows = L.color_idx[L.color_ptr[c]:L.color_ptr[c + 1]]
        assert np.all(color[rows] == c) and np.all(np.diff(rows) > 0)
    assert sorted(L.color_idx.tolist()) == list(range(L.n_owned))
    for i in range(L.n_owned):
        g = L.l2g[i]
        cols = L.row_cols(i)
        assert cols[0] == i
        nb = [L.l2g[j] for j in cols[1:]]
        assert len(set(nb)) == len(nb)
        for u in nb:
            assert (min(g, u), max(g, u)) in edges
        meta = int(L.rowmeta[i])
        ln, closed = meta & 63, (meta >> 6) & 1
        assert ln == len(cols)
        # fan elements: consecutive neighbours (+ wrap if closed) are triangles around g
        elems = []
        for s in range(1, ln):
            t = s + 1 if s + 1 < ln else (1 if closed else -1)
            if t < 0 or (meta >> (8 + s)) & 1:
                continue
            tri = tuple(sorted((g, L.l2g[cols[s]], L.l2g[cols[t]])))
            assert tri in tris
            elems.append(tri)
        assert len(set(elems)) == len(elems)
        for t in elems:
            seen[(g, t)] = 1
        # colouring: no neighbour shares the colour, except the couplings of an absorbed thin
        # top colour (mesh.cc absorb_top), which the layout counts
        same += sum(int(color[j] == color[i]) for j in cols[1:])
    assert same == 2 * L.color_conflicts
    assert L.color_conflicts * 1024 <= L.n_owned * L.max_slots
    # every triangle is visited once from each of its vertices
    assert len(seen) == 3 * mesh.nt
    # padding slots of a chunk point at the row itself
    for c in range(L.nchunks):
        for lane in range(64):
            i = 64 * c + lane
            if i >= L.n_owned:
                continue
            for s in range(L.row_len(i), L.chunk_len[c]):
                assert L.colidx[L.chunk_off[c] + s * 64 + lane] == i


@pytest.mark.parametrize("nranks", [2, 4, 8])
def test_partition_and_halo_consistency(nranks):
    mesh = P.Mesh.read_gmsh(os.path.join(DATA, "pore_pnp/pore.msh")).refine(1)
    lays = [P.Layout(mesh, r, nranks) for r in range(nranks)]
    owned = np.concatenate([L.l2g[:L.n_owned] for L in lays])
    assert sorted(owned.tolist()) == list(range(mesh.nv))
    sizes = [L.n_owned for L in lays]
    assert max(sizes) - min(sizes) <= 1           # RCB splits vertices evenly
    owner = np.empty(mesh.nv, dtype=np.int64)
    for r, L in enumerate(lays):
        owner[L.l2g[:L.n_owned]] = r
    for r, L in enumerate(lays):
        for q_i, q in enumerate(L.nbr_ranks):
            ghosts = L.l2g[L.n_owned + L.recv_ptr[q_i]: L.n_owned + L.recv_ptr[q_i + 1]]
            assert np.all(owner[ghosts] == q)
            Lq = lays[q]
            k = list(Lq.nbr_ranks).index(r)
            sent = Lq.l2g[Lq.send_idx[Lq.send_ptr[k]:Lq.send_ptr[k + 1]]]
            np.testing.assert_array_equal(sent, ghosts)   # same vertices, same order


def test_create_without_gpu_fails_loudly():
    """The product has no CPU fallback: without a GPU pnp_create reports a HIP error."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    mesh = P.Mesh.read_gmsh(os.path.join(DATA, "cylinder.msh"))
    cfg = P.read_config(os.path.join(DATA, "cylinder_config.cfg"))
    with pytest.raises(P.PnpError) as ei:
        P.Context(mesh, P.Params.from_config(cfg))
    assert ei.value.code == P.E_HIP


def test_driver_builds_and_fails_loudly_without_gpu(tmp_path):
    """dune-pnp_amd/driver/pnp_main.cc (the C++ driver over pnp_pdelab_adapter.hh) builds and,
    without a GPU, exits with an error instead of computing anything on the CPU."""
    import subprocess
    import torch
    exe = os.path.join(os.path.dirname(P.LIB_PATH), "pnp_main")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-s", "-C", os.path.dirname(P.LIB_PATH), "pnp_main"])
    out = subprocess.run([exe, "--help"], capture_output=True, text=True)
    assert out.returncode == 0 and "usage" in out.stdout
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    out = subprocess.run([exe, os.path.join(DATA, "cylinder_config.cfg")], capture_output=True,
                         text=True)
    assert out.returncode == 1 and "hip" in out.stderr.lower()


def test_create_option_absorb_thin_color():
    """PNP_CREATE_ABSORB_THIN_COLOR (pnp_set_create_option): on pore_pnp/pore.msh the greedy +
    Kempe colouring leaves a thin fifth colour; absorbed (default) it gives 4 colours and 2
    same-colour couplings outside the sweeps, off it keeps 5 colours and no conflict."""
    m = P.Mesh.read_gmsh(os.path.join(DATA, "pore_pnp", "pore.msh"))
    assert P.get_create_option(P.CREATE_ABSORB_THIN_COLOR) == -1
    try:
        P.set_create_option(P.CREATE_ABSORB_THIN_COLOR, 1)
        on = P.Layout(m)
        P.set_create_option(P.CREATE_ABSORB_THIN_COLOR, 0)
        off = P.Layout(m)
    finally:
        P.set_create_option(P.CREATE_ABSORB_THIN_COLOR, -1)
    assert (len(on.color_ptr) - 1, on.color_conflicts) == (4, 2)
    assert (len(off.color_ptr) - 1, off.color_conflicts) == (5, 0)
    with pytest.raises(P.PnpError):
        P.set_create_option(P.CREATE_ABSORB_THIN_COLOR, 2)
