"""Manufactured solutions for the cylindrical (axisymmetric) PNP operator.

Independent of every restatement of the reference's discrete operator: the sources below come
from the PDE the reference's PnpOperator discretises (src/pnp_operator.hh:165-193, with its
2*PI*y weight :110-112 and Neumann term :276-313), written in divergence form in (x, r = y):

    -div(w grad phi)              + 4 PI l_b w (c+ - c-) = S_phi      (w = 2 PI y)
    -div(w (grad c+ - c+ grad phi))                      = S_+
    -div(w (grad c- + c- grad phi))                      = S_-

For exact fields (phi, c+, c-) the load L_i = int S psi_i + int_N w (F . n) psi_i (F the flux of
the equation, N the Neumann faces) makes R_h(u) - L = 0 a consistent Galerkin problem whose
solution converges to the exact fields at O(h^2) in L2 -- if and only if the operator is the PDE
above (a wrong drift sign, a missing or misplaced radial weight, a wrong face term all leave an
O(1) error).  The loads are integrated here with a 36-point collapsed Gauss rule, the L2 errors
likewise; nothing is shared with oracle/pnp_oracle.c or the HIP kernels.  PI is the
reference's 3.1415 (quirk Q4), used consistently in the weight and in 4 PI l_b.
"""
from __future__ import annotations

import numpy as np

import meshio

PI = 3.1415
L_B = 1.0
C0 = 0.06
X0, X1, Y0, Y1 = 0.0, 1.0, 0.5, 1.5  # an annulus in (x, r): away from the axis
# boundary groups of the strip: 0 bottom (r = Y0), 1 right (x = X1), 2 top (r = Y1), 3 left (x = X0)
NORMALS = {0: (0.0, -1.0), 1: (1.0, 0.0), 2: (0.0, 1.0), 3: (-1.0, 0.0)}


def surfaces():
    """Mixed faces: left and top Dirichlet in every field; bottom Neumann in every field; right
    Dirichlet for phi, Neumann for c+ and c- (the Dirichlet values come from the Newton start,
    which holds the exact nodal values; the Neumann flux constants are 0, the manufactured face
    term is part of the load)."""
    S = meshio.Surface
    return [S(cb=1, pb=1, mb=1),       # bottom
            S(cb=0, pb=1, mb=1),       # right
            S(cb=0, pb=0, mb=0),       # top
            S(cb=0, pb=0, mb=0)]       # left


def strip_mesh(n=4):
    """n x n squares on the strip, each split into two counter-clockwise triangles."""
    xs, ys = np.linspace(X0, X1, n + 1), np.linspace(Y0, Y1, n + 1)
    X, Y = np.meshgrid(xs, ys, indexing="ij")
    xy = np.stack([X.ravel(), Y.ravel()], axis=1)
    vid = lambda i, j: i * (n + 1) + j
    tri = []
    for i in range(n):
        for j in range(n):
            a, b, c, d = vid(i, j), vid(i + 1, j), vid(i + 1, j + 1), vid(i, j + 1)
            if (i + j) % 2 == 0:
                tri += [(a, b, c), (a, c, d)]
            else:
                tri += [(a, b, d), (b, c, d)]
    seg, grp = [], []
    for i in range(n):
        seg += [(vid(i, 0), vid(i + 1, 0))]
        grp += [0]
        seg += [(vid(n, i), vid(n, i + 1))]
        grp += [1]
        seg += [(vid(i + 1, n), vid(i, n))]
        grp += [2]
        seg += [(vid(0, i + 1), vid(0, i))]
        grp += [3]
    return meshio.Mesh(xy, np.array(tri, np.int32), np.array(seg, np.int32),
                       np.array(grp, np.int32))


# ---- exact fields: value, gradient, Laplacian -------------------------------------------------
def phi(x, y):
    v = 0.5 * np.sin(2 * x) * np.cos(1.5 * y) + 0.3 * y * y
    gx = np.cos(2 * x) * np.cos(1.5 * y)
    gy = -0.75 * np.sin(2 * x) * np.sin(1.5 * y) + 0.6 * y
    lap = -3.125 * np.sin(2 * x) * np.cos(1.5 * y) + 0.6
    return v, gx, gy, lap


def cplus(x, y):
    v = C0 * (1 + 0.4 * y * np.sin(np.pi * x))
    gx = C0 * 0.4 * np.pi * y * np.cos(np.pi * x)
    gy = C0 * 0.4 * np.sin(np.pi * x)
    lap = -C0 * 0.4 * np.pi ** 2 * y * np.sin(np.pi * x)
    return v, gx, gy, lap


def cminus(x, y):
    v = C0 * (1 + 0.3 * x * x * np.cos(2 * y))
    gx = C0 * 0.6 * x * np.cos(2 * y)
    gy = -C0 * 0.6 * x * x * np.sin(2 * y)
    lap = C0 * 0.6 * np.cos(2 * y) - C0 * 1.2 * x * x * np.cos(2 * y)
    return v, gx, gy, lap


FIELDS = (phi, cplus, cminus)


def fluxes(x, y, sg=1.0):
    """The flux vectors F_f of the three equations (the operator's volume integrands are
    F_f . grad psi_i times the weight); sg = -1 swaps the drift signs (negative control)."""
    p, px, py, _ = phi(x, y)
    cp, cpx, cpy, _ = cplus(x, y)
    cm, cmx, cmy, _ = cminus(x, y)
    return ((px, py), (cpx - sg * cp * px, cpy - sg * cp * py),
            (cmx + sg * cm * px, cmy + sg * cm * py))


def sources(x, y, variant=None):
    """S_f = -div(w F_f) (+ the phi equation's reaction term), w = 2 PI y.  variant (negative
    controls for the test's power): "flip_drift" manufactures c+- with the drift signs swapped,
    "planar_div" drops the radial weight's derivative from the divergence."""
    w, dw = 2 * PI * y, (0.0 if variant == "planar_div" else 2 * PI)
    p, px, py, pl = phi(x, y)
    cp, cpx, cpy, cpl = cplus(x, y)
    cm, cmx, cmy, cml = cminus(x, y)
    div_phi = pl
    sg = -1.0 if variant == "flip_drift" else 1.0
    div_p = cpl - sg * ((cpx * px + cpy * py) + cp * pl)
    div_m = cml + sg * ((cmx * px + cmy * py) + cm * pl)
    (_, fy0), (_, fy1), (_, fy2) = fluxes(x, y, sg)
    s0 = -(w * div_phi + dw * fy0) + 4 * PI * L_B * w * (cp - cm)
    s1 = -(w * div_p + dw * fy1)
    s2 = -(w * div_m + dw * fy2)
    return s0, s1, s2


def _gauss01(n):
    g, w = np.polynomial.legendre.leggauss(n)
    return 0.5 * (g + 1), 0.5 * w


def tri_rule(n=6):
    """Collapsed (Duffy) Gauss rule on the reference triangle: points (xi, eta), weights."""
    u, wu = _gauss01(n)
    U, V = np.meshgrid(u, u, indexing="ij")
    W = np.outer(wu, wu) * (1 - U)
    return U.ravel(), (V * (1 - U)).ravel(), W.ravel()


def _elements(m):
    t = m.tri
    p0, p1, p2 = m.xy[t[:, 0]], m.xy[t[:, 1]], m.xy[t[:, 2]]
    det = (p1[:, 0] - p0[:, 0]) * (p2[:, 1] - p0[:, 1]) - (p2[:, 0] - p0[:, 0]) * (p1[:, 1] - p0[:, 1])
    return t, p0, p1, p2, np.abs(det)


def load(m, surfs, variant=None):
    """L = int S psi_i + int_N w (F . n) psi_i, lexicographic [phi | c+ | c-]."""
    nv = m.nv
    L = np.zeros(3 * nv)
    xi, eta, wq = tri_rule()
    t, p0, p1, p2, adet = _elements(m)
    psi = (1 - xi - eta, xi, eta)
    for q in range(len(wq)):
        x = p0[:, 0] + xi[q] * (p1[:, 0] - p0[:, 0]) + eta[q] * (p2[:, 0] - p0[:, 0])
        y = p0[:, 1] + xi[q] * (p1[:, 1] - p0[:, 1]) + eta[q] * (p2[:, 1] - p0[:, 1])
        S = sources(x, y, variant)
        for f in range(3):
            for a in range(3):
                np.add.at(L, f * nv + t[:, a], S[f] * psi[a][q] * wq[q] * adet)
    g1, w1 = _gauss01(6)
    for s, (v0, v1) in enumerate(m.bseg):
        grp = int(m.bgroup[s])
        nx, ny = NORMALS[grp]
        a, b = m.xy[v0], m.xy[v1]
        ln = np.hypot(*(b - a))
        x, y = a[0] + g1 * (b[0] - a[0]), a[1] + g1 * (b[1] - a[1])
        F = fluxes(x, y, -1.0 if variant == "flip_drift" else 1.0)
        sv = surfs[grp]
        for f, bt in enumerate((sv.cb, sv.pb, sv.mb)):
            if bt == 0:
                continue  # Dirichlet field: its rows are constrained
            fn = (F[f][0] * nx + F[f][1] * ny) * 2 * PI * y * w1 * ln
            L[f * nv + v0] += np.sum(fn * (1 - g1))
            L[f * nv + v1] += np.sum(fn * g1)
    return L


def exact_nodal(m):
    x, y = m.xy[:, 0], m.xy[:, 1]
    return np.concatenate([F(x, y)[0] for F in FIELDS])


def l2_errors(m, u):
    """Per-field L2(Omega) error of the P1 field u against the exact fields."""
    nv = m.nv
    xi, eta, wq = tri_rule()
    t, p0, p1, p2, adet = _elements(m)
    err = np.zeros(3)
    for q in range(len(wq)):
        x = p0[:, 0] + xi[q] * (p1[:, 0] - p0[:, 0]) + eta[q] * (p2[:, 0] - p0[:, 0])
        y = p0[:, 1] + xi[q] * (p1[:, 1] - p0[:, 1]) + eta[q] * (p2[:, 1] - p0[:, 1])
        for f, F in enumerate(FIELDS):
            uf = u[f * nv:(f + 1) * nv]
            uh = (1 - xi[q] - eta[q]) * uf[t[:, 0]] + xi[q] * uf[t[:, 1]] + eta[q] * uf[t[:, 2]]
            err[f] += np.sum((uh - F(x, y)[0]) ** 2 * wq[q] * adet)
    return np.sqrt(err)


def start(m, mask):
    """Newton start: exact values on the constrained DOFs, a smooth perturbation elsewhere."""
    u = exact_nodal(m)
    nv = m.nv
    x, y = m.xy[:, 0], m.xy[:, 1]
    bump = np.sin(np.pi * x) * np.sin(np.pi * (y - Y0))
    pert = np.concatenate([0.2 * bump, 0.01 * bump, -0.01 * bump])
    return np.where(mask.astype(bool), u, u + pert)


def rates(errs):
    """Observed orders between successive refinements (h halves)."""
    e = np.asarray(errs)
    return np.log2(e[:-1] / e[1:])


def check_derivatives():
    """Finite-difference check of the hand-derived gradients/Laplacians above."""
    rng = np.random.default_rng(3)
    x, y = rng.uniform(X0, X1, 20), rng.uniform(Y0, Y1, 20)
    h = 1e-4
    for F in FIELDS:
        v, gx, gy, lap = F(x, y)
        fx = (F(x + h, y)[0] - F(x - h, y)[0]) / (2 * h)
        fy = (F(x, y + h)[0] - F(x, y - h)[0]) / (2 * h)
        fl = (F(x + h, y)[0] + F(x - h, y)[0] + F(x, y + h)[0] + F(x, y - h)[0] - 4 * v) / h ** 2
        assert np.allclose(gx, fx, atol=1e-7) and np.allclose(gy, fy, atol=1e-7)
        assert np.allclose(lap, fl, atol=1e-5)
