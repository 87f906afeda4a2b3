"""Test-side gmsh v2 reader, uniform red refinement and INI config reader (numpy).

Independent of the product's C++ mesh code (dune-pnp_amd/csrc/mesh.cc); the CPU tests check
the two against each other.  Semantics follow the reference's inputs:

* GmshReader (dune-grid, third party, called at /root/reference/src/pnp_solver_main.cc:86-91):
  line elements (type 1) become boundary segments in file order (boundarySegmentIndex), with
  their FIRST tag (physical group) recorded in boundaryIndexToEntity; triangles (type 2) become
  elements; vertices are numbered in order of first use by a triangle.  Both the 2-tag
  (test/pore.msh, $MeshFormat 2.2) and 3-tag (test/pore_pnp/pore.msh, 2.1) layouts occur.
* Red refinement: each triangle -> 4, new vertices at edge midpoints, boundary segments split
  in two and keep their group (SURVEY.md §5 "Long-context / sequence parallelism" row).
* Sysparams::readConfigFile (/root/reference/src/sysparams.cc:16-98) with the documented
  defaults of SURVEY.md §5 for keys that some shipped configs omit.
"""
from __future__ import annotations

import configparser
import os
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Mesh:
    xy: np.ndarray       # [nv,2] float64
    tri: np.ndarray      # [nt,3] int32
    bseg: np.ndarray     # [nb,2] int32
    bgroup: np.ndarray   # [nb] int32

    @property
    def nv(self):
        return self.xy.shape[0]

    @property
    def nt(self):
        return self.tri.shape[0]

    @property
    def nb(self):
        return self.bseg.shape[0]


def read_gmsh(path: str) -> Mesh:
    with open(path) as f:
        lines = [ln.strip() for ln in f]
    i = 0
    nodes = {}
    lines_el, tris = [], []
    while i < len(lines):
        ln = lines[i]
        if ln == "$Nodes":
            n = int(lines[i + 1])
            for k in range(n):
                parts = lines[i + 2 + k].split()
                nodes[int(parts[0])] = (float(parts[1]), float(parts[2]))
            i += n + 2
            continue
        if ln == "$Elements":
            n = int(lines[i + 1])
            for k in range(n):
                parts = [int(t) for t in lines[i + 2 + k].split()]
                etype, ntags = parts[1], parts[2]
                tags = parts[3:3 + ntags]
                vs = parts[3 + ntags:]
                if etype == 1:
                    lines_el.append((vs[0], vs[1], tags[0]))
                elif etype == 2:
                    tris.append(vs[:3])
            i += n + 2
            continue
        i += 1
    renum = {}
    xy = []
    tri = np.empty((len(tris), 3), dtype=np.int32)
    for e, t in enumerate(tris):
        for a, v in enumerate(t):
            if v not in renum:
                renum[v] = len(xy)
                xy.append(nodes[v])
            tri[e, a] = renum[v]
    bseg = np.array([[renum[a], renum[b]] for a, b, _ in lines_el], dtype=np.int32).reshape(-1, 2)
    bgroup = np.array([g for _, _, g in lines_el], dtype=np.int32)
    return Mesh(np.array(xy, dtype=np.float64), tri, bseg, bgroup)


def refine(m: Mesh, k: int = 1) -> Mesh:
    for _ in range(k):
        m = _refine_once(m)
    return m


def _refine_once(m: Mesh) -> Mesh:
    nv = m.nv
    edge_id = {}
    newxy = [m.xy]
    extra = []

    def mid(a, b):
        key = (a, b) if a < b else (b, a)
        v = edge_id.get(key)
        if v is None:
            v = nv + len(extra)
            edge_id[key] = v
            extra.append(0.5 * (m.xy[a] + m.xy[b]))
        return v

    tri = np.empty((4 * m.nt, 3), dtype=np.int32)
    for e in range(m.nt):
        a, b, c = (int(t) for t in m.tri[e])
        mab, mbc, mca = mid(a, b), mid(b, c), mid(c, a)
        tri[4 * e + 0] = (a, mab, mca)
        tri[4 * e + 1] = (mab, b, mbc)
        tri[4 * e + 2] = (mca, mbc, c)
        tri[4 * e + 3] = (mab, mbc, mca)
    bseg = np.empty((2 * m.nb, 2), dtype=np.int32)
    bgroup = np.repeat(m.bgroup, 2)
    for s in range(m.nb):
        a, b = int(m.bseg[s, 0]), int(m.bseg[s, 1])
        key = (a, b) if a < b else (b, a)
        mm = edge_id[key]
        bseg[2 * s] = (a, mm)
        bseg[2 * s + 1] = (mm, b)
    if extra:
        newxy.append(np.array(extra))
    return Mesh(np.concatenate(newxy), tri, bseg, bgroup.astype(np.int32))


# ------------------------------------------------------------------------------------------
# config (src/sysparams.cc:16-98)
# ------------------------------------------------------------------------------------------
DEFAULTS = {  # documented defaults (SURVEY.md §5 "Config / flags"), from test/pore_pnp/pore.cfg
    "verbosity": 0, "cylindrical": 0, "l_b": 1.0, "linearSolverIterations": 20000,
    "newtonReassembleThreshold": 0.0, "newtonReduction": 1e-9, "newtonMinLinearReduction": 1e-8,
    "newtonMaxIterations": 50, "newtonLineSearchMaxIteration": 500, "c0": 0.06, "tau": 1.0,
    "outputFreq": 10, "nSteps": 100, "potentialUpdateFreq": 1,
}


@dataclass
class Surface:  # src/sysparams.cc:101-116 defaults
    cb: int = 1
    cflux: float = 0.0
    cpot: float = 0.0
    pb: int = 1
    pflux: float = 0.0
    pconc: float = 0.0
    mb: int = 1
    mflux: float = 0.0
    mconc: float = 0.0


@dataclass
class Config:
    meshfile: str
    n_surfaces: int
    system: dict
    surfaces: list = field(default_factory=list)
    defaulted: list = field(default_factory=list)


def read_config(path: str) -> Config:
    cp = configparser.ConfigParser(inline_comment_prefixes=("#",), comment_prefixes=("#",))
    cp.optionxform = str
    with open(path) as f:
        cp.read_string(f.read())
    sysd = dict(cp["system"]) if cp.has_section("system") else {}
    system, defaulted = {}, []
    for k, dv in DEFAULTS.items():
        if k in sysd:
            system[k] = type(dv)(float(sysd[k])) if isinstance(dv, int) else float(sysd[k])
        else:
            system[k] = dv
            defaulted.append(k)
    n = int(sysd["n_surfaces"])
    surfs = []
    for i in range(n):
        sec = cp[f"surface_{i}"]
        s = Surface()
        s.cb = int(sec["coulombBtype"])
        if s.cb == 0:
            s.cpot = float(sec["coulombPotential"])
        elif s.cb == 1:
            s.cflux = float(sec["coulombFlux"])
        s.pb = int(sec["plusDiffusionBtype"])
        if s.pb == 0:
            s.pconc = float(sec["plusDiffusionConcentration"])
        elif s.pb == 1:
            s.pflux = float(sec["plusDiffusionFlux"])
        s.mb = int(sec["minusDiffusionBtype"])
        if s.mb == 0:
            s.mconc = float(sec["minusDiffusionConcentration"])
        elif s.mb == 1:
            s.mflux = float(sec["minusDiffusionFlux"])
        surfs.append(s)
    meshfile = cp["mesh"]["filename"]
    meshfile = os.path.join(os.path.dirname(path), meshfile)
    return Config(meshfile, n, system, surfs, defaulted)
