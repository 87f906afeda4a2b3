"""Helpers of the P_k (PDEGREE 2, 3) tests: node matching between the product's and the oracle's
Lagrange spaces, random operator arguments, and a manufactured cylindrical Poisson problem.

Test infrastructure only.  The manufactured problem is the PDE PoissonOperator discretises
(src/poisson_operator.hh:119-125 with its 2*PI*y weight :85-86):

    -div(w grad u) + 4 PI l_b w (c- - c+) = 0,   w = 2 PI y,

with u the exact field of tests/mms.py (phi) and c- = 0, c+ = g = -(lap u + u_y / y) / (4 PI l_b)
at the nodes; every face Dirichlet (the exact nodal values).  The discrete solution converges to
u at O(h^(k+1)) in L2 when the quadrature is exact enough (P2: the order-3 rule integrates the
degree-2 stiffness exactly); the L2 errors use a 36-point collapsed Gauss rule and the oracle's
own basis, nothing shared with the HIP kernels.
"""
from __future__ import annotations

import numpy as np

import meshio
import mms
import oracle_py as O

KAPPA = 4 * mms.PI * mms.L_B


def match_nodes(xy_prod, xy_orc, tol=1e-9):
    """perm with xy_prod[i] == xy_orc[perm[i]] (to tol, scaled by the domain size)."""
    from scipy.spatial import cKDTree
    scale = max(1.0, float(np.abs(xy_orc).max()))
    d, perm = cKDTree(xy_orc).query(xy_prod)
    assert d.max() <= tol * scale, f"unmatched node, distance {d.max()}"
    assert len(np.unique(perm)) == len(perm), "two product nodes on one oracle node"
    return perm


def poisson_problem(n, cylindrical=1):
    m = mms.strip_mesh(n)
    S = meshio.Surface
    surf = [S(cb=0), S(cb=0), S(cb=0), S(cb=0)]
    orc = O.Problem(m, surf, l_b=mms.L_B, c0=mms.C0, tau=1.0, cylindrical=cylindrical,
                    pi=mms.PI)
    return m, surf, orc


def exact_and_source(xy, cylindrical=1):
    u, gx, gy, lap = mms.phi(xy[:, 0], xy[:, 1])
    g = -(lap + (gy / xy[:, 1] if cylindrical else 0.0)) / KAPPA
    return u, g


def l2_error(space, u_nodes, mesh):
    """||u_h - u||_L2 on the oracle space (its enode / basis), u_nodes over its nodes."""
    xi, eta, w = mms.tri_rule(6)
    B = np.array([space.basis(a, b)[0] for a, b in zip(xi, eta)])  # [nq, nl]
    err = 0.0
    P = mesh.xy[mesh.tri]                                   # [nt, 3, 2]
    J00 = P[:, 1, 0] - P[:, 0, 0]
    J01 = P[:, 2, 0] - P[:, 0, 0]
    J10 = P[:, 1, 1] - P[:, 0, 1]
    J11 = P[:, 2, 1] - P[:, 0, 1]
    adet = np.abs(J00 * J11 - J01 * J10)
    uh = u_nodes[space.enode] @ B.T                          # [nt, nq]
    X = P[:, 0, 0][:, None] + J00[:, None] * xi + J01[:, None] * eta
    Y = P[:, 0, 1][:, None] + J10[:, None] * xi + J11[:, None] * eta
    ue = mms.phi(X, Y)[0]
    err = np.sum(((uh - ue) ** 2) * w[None, :] * adet[:, None])
    return float(np.sqrt(err))


def rates(errs, hs):
    e, h = np.array(errs), np.array(hs)
    return np.log(e[:-1] / e[1:]) / np.log(h[:-1] / h[1:])
