"""GPU parity of the assembly's fan-length variants (-m gpu).  Every mesh under data/ has fans of
at most 8 neighbours, which selects the gather-all walk (k_assemble_ga, FANR 9).  A wheel mesh
with one high-degree hub exercises the other two paths: 11 neighbours (register-resident
column indices, FANR 12) and 14 neighbours (index loads in the walk, FANR 0), for the fused
residual + Jacobian and the residual-only (line search) kernels, against the oracle."""
import numpy as np
import pytest

import meshio
import oracle_py as O
import pnp_amd as P

pytestmark = pytest.mark.gpu


def wheel(k, y0=3.0):
    """hub 0, ring 1 (k vertices, radius 1), ring 2 (2k vertices, radius 2), shifted to y > 0"""
    a1 = 2 * np.pi * np.arange(k) / k
    a2 = 2 * np.pi * np.arange(2 * k) / (2 * k)
    xy = np.vstack([[0.0, 0.0], np.c_[np.cos(a1), np.sin(a1)], 2 * np.c_[np.cos(a2), np.sin(a2)]])
    xy[:, 1] += y0
    r1 = 1 + np.arange(k)
    r2 = 1 + k + np.arange(2 * k)
    tri = []
    for i in range(k):
        j = (i + 1) % k
        tri += [(0, r1[i], r1[j]), (r1[i], r2[2 * i], r2[2 * i + 1]),
                (r1[i], r2[2 * i + 1], r1[j]), (r1[j], r2[2 * i + 1], r2[(2 * i + 2) % (2 * k)])]
    bseg = np.array([(r2[j], r2[(j + 1) % (2 * k)]) for j in range(2 * k)], dtype=np.int32)
    bgroup = (np.arange(2 * k) % 2).astype(np.int32)
    return xy, np.array(tri, dtype=np.int32), bseg, bgroup


SURF = [dict(cb=1, cflux=0.3, cpot=0.0, pb=1, pflux=-0.2, pconc=0.0, mb=1, mflux=0.1, mconc=0.0),
        dict(cb=0, cflux=0.0, cpot=1.0, pb=0, pflux=0.0, pconc=0.05, mb=0, mflux=0.0,
             mconc=0.07)]


@pytest.mark.parametrize("k", [11, 14])
@pytest.mark.parametrize("kind", ["pnp", "pb"])
def test_high_degree_fans_match_oracle(k, kind):
    xy, tri, bseg, bgroup = wheel(k)
    mesh = P.Mesh(xy, tri, bseg, bgroup)
    par = P.Params([P.Surface(**s) for s in SURF], l_b=0.7, c0=0.06, tau=1.0, cylindrical=1)
    orc = O.Problem(meshio.Mesh(xy, tri, bseg, bgroup), [meshio.Surface(**s) for s in SURF],
                    l_b=0.7, c0=0.06, tau=1.0, cylindrical=1)
    ctx = P.Context(mesh, par)
    assert ctx.info()["max_slots"] == k + 1
    nv = mesh.nv
    rng = np.random.default_rng(k)
    if kind == "pnp":
        ctx.set_operator(P.OP_PNP)
        op = orc.operator(O.OP_PNP, flux=orc.flux(), mask=orc.mask(3))
        x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                            0.06 * rng.uniform(0.5, 1.5, nv)])
    else:
        ctx.set_operator(P.OP_PB)
        op = orc.operator(O.OP_PB, flux=orc.flux(), mask=orc.mask(1))
        x = rng.uniform(-1, 1, nv)
    r = ctx.residual(x)               # residual-only kernel
    J = ctx.jacobian(x)               # fused residual + Jacobian kernel
    ro = orc.residual(op, x)
    Jo = orc.jacobian(op, x)
    assert np.max(np.abs(r - ro)) <= 1e-12 * np.max(np.abs(ro))
    assert abs(J - Jo).max() <= 1e-12 * abs(Jo).max()
