/*
 * pnp_oracle.c — CPU restatement of kessel/dune-pnp's assembly + solve hot path.
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h for the parity status and what it pins to).
 *
 * Written to follow the reference's control flow statement by statement where that matters
 * for rounding (quadrature loop, factor = w*|detJ|, factor *= y*2*PI, residual expressions in
 * the reference's operand order), and the PDELab/ISTL semantics the reference calls into.
 */
#include "pnp_oracle.h"

#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdlib.h>
#include <string.h>

/* ----------------------------------------------------------------------------------------
 * Quadrature (dune-geometry SimplexQuadraturePoints<2>, restated; see header)
 * ---------------------------------------------------------------------------------------- */
typedef struct {
  int n;
  double xi[4], eta[4], w[4];
} qrule;

static const qrule Q2 = {3,
                         {4.0 / 6.0, 1.0 / 6.0, 1.0 / 6.0, 0},
                         {1.0 / 6.0, 4.0 / 6.0, 1.0 / 6.0, 0},
                         {0.5 / 3.0, 0.5 / 3.0, 0.5 / 3.0, 0}};
static const qrule Q3 = {4,
                         {10.0 / 30.0, 18.0 / 30.0, 6.0 / 30.0, 6.0 / 30.0},
                         {10.0 / 30.0, 6.0 / 30.0, 18.0 / 30.0, 6.0 / 30.0},
                         {0.5 * -27.0 / 48.0, 0.5 * 25.0 / 48.0, 0.5 * 25.0 / 48.0,
                          0.5 * 25.0 / 48.0}};

static const qrule *rule_for_order(int order) { return order <= 2 ? &Q2 : &Q3; }

/* element geometry: affine map x = p0 + xi*(p1-p0) + eta*(p2-p0) */
typedef struct {
  double x0, y0, J00, J01, J10, J11; /* J = [[x1-x0, x2-x0],[y1-y0, y2-y0]] */
  double det, adet;
  double g[3][2]; /* physical gradients of the P1 basis: jacobianInverseTransposed * grad_hat */
} elgeo;

static void element_geometry(const orc_mesh *m, int e, elgeo *G) {
  const int *t = m->tri + 3 * e;
  const double *p0 = m->xy + 2 * t[0], *p1 = m->xy + 2 * t[1], *p2 = m->xy + 2 * t[2];
  G->x0 = p0[0];
  G->y0 = p0[1];
  G->J00 = p1[0] - p0[0];
  G->J01 = p2[0] - p0[0];
  G->J10 = p1[1] - p0[1];
  G->J11 = p2[1] - p0[1];
  G->det = G->J00 * G->J11 - G->J01 * G->J10;
  G->adet = fabs(G->det);
  /* J^{-T} = 1/det [[J11, -J10], [-J01, J00]] */
  double it00 = G->J11 / G->det, it01 = -G->J10 / G->det;
  double it10 = -G->J01 / G->det, it11 = G->J00 / G->det;
  static const double gh[3][2] = {{-1.0, -1.0}, {1.0, 0.0}, {0.0, 1.0}};
  for (int i = 0; i < 3; i++) {
    G->g[i][0] = it00 * gh[i][0] + it01 * gh[i][1];
    G->g[i][1] = it10 * gh[i][0] + it11 * gh[i][1];
  }
}

static inline double global_y(const elgeo *G, double xi, double eta) {
  return G->y0 + G->J10 * xi + G->J11 * eta;
}

static inline void p1_values(double xi, double eta, double psi[3]) {
  psi[0] = 1.0 - xi - eta;
  psi[1] = xi;
  psi[2] = eta;
}

/* ----------------------------------------------------------------------------------------
 * Local operators (element-local residual on a local DOF vector)
 * ---------------------------------------------------------------------------------------- */

/* PnpOperator::alpha_volume, src/pnp_operator.hh:46-195.  xl/rl: [phi0..2, cp0..2, cm0..2]. */
static void lop_pnp_volume(const elgeo *G, const orc_params *p, const double *xl, double *rl) {
  const double PI = p->pi;
  const qrule *R = rule_for_order(3); /* intorder_ = 3, :40 */
  for (int q = 0; q < R->n; q++) {
    double factor = R->w[q] * G->adet; /* :110 */
    if (p->cylindrical) factor *= global_y(G, R->xi[q], R->eta[q]) * 2 * PI; /* :111-112 */
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double u_phi = 0, u_cp = 0, u_cm = 0; /* :122-131 */
    for (int i = 0; i < 3; i++) u_phi += xl[i] * psi[i];
    for (int i = 0; i < 3; i++) u_cp += xl[3 + i] * psi[i];
    for (int i = 0; i < 3; i++) u_cm += xl[6 + i] * psi[i];
    double gphi[2] = {0, 0}, gcp[2] = {0, 0}, gcm[2] = {0, 0}; /* :154-163 */
    for (int i = 0; i < 3; i++) {
      gphi[0] += xl[i] * G->g[i][0];
      gphi[1] += xl[i] * G->g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      gcp[0] += xl[3 + i] * G->g[i][0];
      gcp[1] += xl[3 + i] * G->g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      gcm[0] += xl[6 + i] * G->g[i][0];
      gcm[1] += xl[6 + i] * G->g[i][1];
    }
    for (int i = 0; i < 3; i++) { /* :167-173 */
      double gg = gphi[0] * G->g[i][0] + gphi[1] * G->g[i][1];
      rl[i] += (gg + 4 * PI * p->l_b * (u_cp - u_cm) * psi[i]) * factor;
    }
    for (int i = 0; i < 3; i++) { /* :177-183 */
      double gc = gcp[0] * G->g[i][0] + gcp[1] * G->g[i][1];
      double gp = gphi[0] * G->g[i][0] + gphi[1] * G->g[i][1];
      rl[3 + i] += (gc - u_cp * gp) * factor;
    }
    for (int i = 0; i < 3; i++) { /* :187-193 */
      double gc = gcm[0] * G->g[i][0] + gcm[1] * G->g[i][1];
      double gp = gphi[0] * G->g[i][0] + gphi[1] * G->g[i][1];
      rl[6 + i] += (gc + u_cm * gp) * factor;
    }
  }
}

/* PnpTOperator::alpha_volume, src/pnp_toperator.hh:31-101 (order 2, tau*u*psi, Q2 quirk:
 * the c- mass is accumulated into the c+ rows, :96-99). */
static void lop_pnpt_volume(const elgeo *G, const orc_params *p, double tau, const double *xl,
                            double *rl) {
  const double PI = p->pi;
  const qrule *R = rule_for_order(2);
  for (int q = 0; q < R->n; q++) {
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double u_cp = 0, u_cm = 0;
    for (int i = 0; i < 3; i++) u_cp += xl[3 + i] * psi[i];
    for (int i = 0; i < 3; i++) u_cm += xl[6 + i] * psi[i];
    double factor = R->w[q] * G->adet; /* :94 */
    if (p->cylindrical) factor *= global_y(G, R->xi[q], R->eta[q]) * 2 * PI;
    for (int i = 0; i < 3; i++) rl[3 + i] += tau * u_cp * psi[i] * factor;
    for (int i = 0; i < 3; i++) rl[3 + i] += tau * u_cm * psi[i] * factor;
  }
}

/* PBOperator::alpha_volume, src/pb_operator.hh:46-122 */
static void lop_pb_volume(const elgeo *G, const orc_params *p, const double *xl, double *rl) {
  const double PI = p->pi;
  const qrule *R = rule_for_order(3);
  for (int q = 0; q < R->n; q++) {
    double factor = R->w[q] * G->adet;
    if (p->cylindrical) factor *= global_y(G, R->xi[q], R->eta[q]) * 2 * PI;
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    double gu[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      gu[0] += xl[i] * G->g[i][0];
      gu[1] += xl[i] * G->g[i][1];
    }
    for (int i = 0; i < 3; i++) { /* :114-120 */
      double gg = gu[0] * G->g[i][0] + gu[1] * G->g[i][1];
      rl[i] += (gg + 8 * PI * p->l_b * p->c0 * sinh(u) * psi[i]) * factor;
    }
  }
}

/* DiffusionOperator::alpha_volume, src/diffusion_operator.hh:42-112 (order 2, no cylindrical
 * weight (Q8), grad Phi of the frozen P1 potential, constant per element). */
static void lop_diff_volume(const elgeo *G, double z, const double *phil, const double *xl,
                            double *rl) {
  const qrule *R = rule_for_order(2);
  for (int q = 0; q < R->n; q++) {
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    double gu[2] = {0, 0}, gP[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      gu[0] += xl[i] * G->g[i][0];
      gu[1] += xl[i] * G->g[i][1];
      gP[0] += phil[i] * G->g[i][0];
      gP[1] += phil[i] * G->g[i][1];
    }
    double factor = R->w[q] * G->adet; /* :100 */
    for (int i = 0; i < 3; i++) {      /* :109-110, a = 0 */
      double gg = gu[0] * G->g[i][0] + gu[1] * G->g[i][1];
      double gp = gP[0] * G->g[i][0] + gP[1] * G->g[i][1];
      rl[i] += (gg + u * z * gp + 0.0 * u * psi[i]) * factor;
    }
  }
}

/* DiffusionTOperator::alpha_volume, src/diffusion_toperator.hh:38-73 (u*psi; order 5 as built
 * at src/instationary_pnp_from_pb_md.hh:363 -- the integrand is quadratic, so the order-2 rule
 * is exact and used here). */
static void lop_difft_volume(const elgeo *G, const double *xl, double *rl) {
  const qrule *R = rule_for_order(2);
  for (int q = 0; q < R->n; q++) {
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    double factor = R->w[q] * G->adet;
    for (int i = 0; i < 3; i++) rl[i] += u * psi[i] * factor;
  }
}

/* PoissonOperator::alpha_volume, src/poisson_operator.hh:46-127 (order 3, (cm-cp) sign) */
static void lop_poisson_volume(const elgeo *G, const orc_params *p, const double *cpl,
                               const double *cml, const double *xl, double *rl) {
  const double PI = p->pi;
  const qrule *R = rule_for_order(3);
  for (int q = 0; q < R->n; q++) {
    double factor = R->w[q] * G->adet;
    if (p->cylindrical) factor *= global_y(G, R->xi[q], R->eta[q]) * 2 * PI;
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double cp = 0, cm = 0;
    for (int i = 0; i < 3; i++) cp += cpl[i] * psi[i];
    for (int i = 0; i < 3; i++) cm += cml[i] * psi[i];
    double gu[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      gu[0] += xl[i] * G->g[i][0];
      gu[1] += xl[i] * G->g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      double gg = gu[0] * G->g[i][0] + gu[1] * G->g[i][1];
      rl[i] += (gg + 1 * p->l_b * 4 * PI * (cm - cp) * psi[i]) * factor;
    }
  }
}

/* alpha_boundary (src/pnp_operator.hh:198-315, src/pb_operator.hh:126-194,
 * src/poisson_operator.hh:131-199): 1-D order-3 Gauss (2 points) on each boundary segment,
 * j*psi_i*factor for each field whose Btype != 0.  Adds into the global vector r. */
static int surface_btype(const orc_params *p, int g, int field) {
  const orc_surface *s = p->surf + g;
  return field == 0 ? s->cb : (field == 1 ? s->pb : s->mb);
}

static void boundary_flux(const orc_mesh *m, const orc_params *p, const double *flux,
                          int nfields, int field0, double scale, double *r) {
  const double PI = p->pi;
  const double gt[2] = {0.5 - 0.5 / sqrt(3.0), 0.5 + 0.5 / sqrt(3.0)};
  for (int b = 0; b < m->nb; b++) {
    int v0 = m->bseg[2 * b], v1 = m->bseg[2 * b + 1];
    int g = m->bgroup[b];
    double dx = m->xy[2 * v1] - m->xy[2 * v0], dy = m->xy[2 * v1 + 1] - m->xy[2 * v0 + 1];
    double len = sqrt(dx * dx + dy * dy);
    for (int q = 0; q < 2; q++) {
      double factor = 0.5 * len;
      double y = m->xy[2 * v0 + 1] + gt[q] * dy;
      if (p->cylindrical) factor *= y * 2 * PI;
      double psi[2] = {1.0 - gt[q], gt[q]};
      for (int f = 0; f < nfields; f++) {
        int field = field0 + f;
        if (surface_btype(p, g, field) == 0) continue; /* isDirichlet */
        double j = flux[3 * b + field];
        r[f * m->nv + v0] += scale * (j * psi[0] * factor);
        r[f * m->nv + v1] += scale * (j * psi[1] * factor);
      }
    }
  }
}

/* ----------------------------------------------------------------------------------------
 * setup: a9 / a10
 * ---------------------------------------------------------------------------------------- */
void orc_dirichlet_mask(const orc_mesh *m, const orc_params *p, int nfields, uint8_t *mask) {
  memset(mask, 0, (size_t)nfields * m->nv);
  for (int b = 0; b < m->nb; b++) {
    int g = m->bgroup[b];
    for (int f = 0; f < nfields; f++) {
      if (surface_btype(p, g, f) == 0) {
        mask[f * m->nv + m->bseg[2 * b]] = 1;
        mask[f * m->nv + m->bseg[2 * b + 1]] = 1;
      }
    }
  }
}

void orc_flux_container(const orc_mesh *m, const orc_params *p, double *flux) {
  for (int b = 0; b < m->nb; b++) {
    const orc_surface *s = p->surf + m->bgroup[b];
    flux[3 * b + 0] = s->cflux;
    flux[3 * b + 1] = s->pflux;
    flux[3 * b + 2] = s->mflux;
  }
}

/* edge -> boundary segment lookup by sorted vertex pair (simple open-addressing hash) */
typedef struct {
  long long *key;
  int *val;
  long long cap;
} ehash;

static long long ekey(int a, int b) {
  if (a > b) {
    int t = a;
    a = b;
    b = t;
  }
  return ((long long)a << 32) | (unsigned)b;
}
static void eh_init(ehash *h, long long n) {
  h->cap = 1;
  while (h->cap < 2 * n + 16) h->cap <<= 1;
  h->key = (long long *)malloc(sizeof(long long) * h->cap);
  h->val = (int *)malloc(sizeof(int) * h->cap);
  for (long long i = 0; i < h->cap; i++) h->key[i] = -1;
}
static void eh_free(ehash *h) {
  free(h->key);
  free(h->val);
}
static long long eh_slot(const ehash *h, long long k) {
  unsigned long long x = (unsigned long long)k * 0x9E3779B97F4A7C15ull;
  long long s = (long long)(x >> 20) & (h->cap - 1);
  while (h->key[s] != -1 && h->key[s] != k) s = (s + 1) & (h->cap - 1);
  return s;
}
static int eh_get(const ehash *h, long long k) {
  long long s = eh_slot(h, k);
  return h->key[s] == k ? h->val[s] : -1;
}
static void eh_put(ehash *h, long long k, int v) {
  long long s = eh_slot(h, k);
  h->key[s] = k;
  h->val[s] = v;
}

/* PDELab's boundary intersections of each element (a8): the faces of the reference triangle in
 * DUNE's numbering, face 0 = local vertices (0,1), face 1 = (0,2), face 2 = (1,2), each a boundary
 * intersection when its edge is a boundary segment.  ebf[3e + k] = that segment, or -1. */
static const int kFaceV[3][2] = {{0, 1}, {0, 2}, {1, 2}};
static int *elem_boundary_faces(const orc_mesh *m) {
  ehash h;
  eh_init(&h, m->nb);
  for (int b = 0; b < m->nb; b++) {
    long long k = ekey(m->bseg[2 * b], m->bseg[2 * b + 1]);
    if (eh_get(&h, k) < 0) eh_put(&h, k, b); /* a segment listed twice: its first record */
  }
  int *ebf = (int *)malloc(sizeof(int) * 3 * (size_t)(m->nt > 0 ? m->nt : 1));
  for (int e = 0; e < m->nt; e++) {
    const int *t = m->tri + 3 * e;
    for (int k = 0; k < 3; k++)
      ebf[3 * e + k] = m->nb ? eh_get(&h, ekey(t[kFaceV[k][0]], t[kFaceV[k][1]])) : -1;
  }
  eh_free(&h);
  return ebf;
}

/* PnpOperator / PBOperator / PoissonOperator::alpha_boundary on face k of element e (segment b)
 * into the element's local residual rl (src/pnp_operator.hh:198-315, src/pb_operator.hh:126-194):
 * the face's geometry runs from its lower to its higher local vertex (ig.geometry(), the
 * reference element's sub-entity order), 2-point Gauss on it, factor = w |face| (* y 2 PI), and
 * for every non-Dirichlet field the loop over ALL of the element's basis functions (lfsv.size())
 * evaluated at the face point in element coordinates (geometryInInside(): P1LocalBasis
 * 1 - x - y, x, y), accumulated with the operator's weight (scale). */
static void boundary_face(const orc_mesh *m, const orc_params *p, const double *flux, int e, int k,
                          int b, int nfields, double scale, double *rl) {
  static const double corner[3][2] = {{0.0, 0.0}, {1.0, 0.0}, {0.0, 1.0}};
  const double PI = p->pi;
  const double gt[2] = {0.5 - 0.5 / sqrt(3.0), 0.5 + 0.5 / sqrt(3.0)};
  const int ia = kFaceV[k][0], ib = kFaceV[k][1];
  const int va = m->tri[3 * e + ia], vb = m->tri[3 * e + ib];
  const int g = m->bgroup[b];
  double dx = m->xy[2 * vb] - m->xy[2 * va], dy = m->xy[2 * vb + 1] - m->xy[2 * va + 1];
  double len = sqrt(dx * dx + dy * dy);
  for (int q = 0; q < 2; q++) {
    double factor = 0.5 * len;
    double y = m->xy[2 * va + 1] + gt[q] * dy;
    if (p->cylindrical) factor *= y * 2 * PI;
    double lx = corner[ia][0] + (corner[ib][0] - corner[ia][0]) * gt[q];
    double ly = corner[ia][1] + (corner[ib][1] - corner[ia][1]) * gt[q];
    double phi[3] = {1.0 - lx - ly, lx, ly};
    for (int f = 0; f < nfields; f++) {
      if (surface_btype(p, g, f) == 0) continue; /* isDirichlet */
      double j = flux[3 * b + f];
      for (int i = 0; i < 3; i++) rl[3 * f + i] += scale * (j * phi[i] * factor);
    }
  }
}

/* Q6: distance of a point to the INFINITE line through a segment, src/dirichlet_bc.hh:21-39 */
static int on_line(const orc_mesh *m, int b, double px, double py) {
  const double *c0 = m->xy + 2 * m->bseg[2 * b], *c1 = m->xy + 2 * m->bseg[2 * b + 1];
  double vx = c1[0] - c0[0], vy = c1[1] - c0[1];
  double n = sqrt(vx * vx + vy * vy);
  vx /= n;
  vy /= n;
  double dx = px - c0[0], dy = py - c0[1];
  double s = dx * vx + dy * vy;
  double ex = vx * s - dx, ey = vy * s - dy;
  return sqrt(ex * ex + ey * ey) < 1e-9;
}

void orc_initial_state(const orc_mesh *m, const orc_params *p, const double *phi_pb, double *x0) {
  orc_initial_state_nodes(m, p, 3, m->tri, m->xy, m->nv, phi_pb, x0);
}

/* the same element loop over nl nodes per element (enode[e*nl+a] at nxy), x0[3 nn] */
void orc_initial_state_nodes(const orc_mesh *m, const orc_params *p, int nl, const int *enode,
                             const double *nxy, int nn, const double *phi_pb, double *x0) {
  int nv = nn, nt = m->nt;
  /* boundary segments by edge, element neighbours by edge */
  ehash bh, eh;
  eh_init(&bh, m->nb);
  for (int b = 0; b < m->nb; b++) eh_put(&bh, ekey(m->bseg[2 * b], m->bseg[2 * b + 1]), b);
  eh_init(&eh, 3LL * nt);
  int *nbr = (int *)malloc(sizeof(int) * 3 * nt); /* neighbour across local edge k */
  int *bsi = (int *)malloc(sizeof(int) * 3 * nt); /* boundary segment on local edge k */
  static const int ed[3][2] = {{0, 1}, {0, 2}, {1, 2}}; /* DUNE reference-triangle faces */
  for (int e = 0; e < nt; e++)
    for (int k = 0; k < 3; k++) {
      nbr[3 * e + k] = -1;
      bsi[3 * e + k] = -1;
    }
  for (int e = 0; e < nt; e++) {
    const int *t = m->tri + 3 * e;
    for (int k = 0; k < 3; k++) {
      long long key = ekey(t[ed[k][0]], t[ed[k][1]]);
      int o = eh_get(&eh, key);
      if (o < 0) {
        eh_put(&eh, key, 3 * e + k);
      } else {
        nbr[3 * e + k] = o / 3;
        nbr[o] = e;
      }
    }
  }
  for (int e = 0; e < nt; e++) {
    const int *t = m->tri + 3 * e;
    for (int k = 0; k < 3; k++)
      if (nbr[3 * e + k] < 0) bsi[3 * e + k] = eh_get(&bh, ekey(t[ed[k][0]], t[ed[k][1]]));
  }
  /* Q5: BCExtension::bctype() falls through every case -> minusDiffusionBtype */
  for (int e = 0; e < nt; e++) {
    for (int a = 0; a < nl; a++) {
      int v = enode[nl * e + a];
      double px = nxy[2 * v], py = nxy[2 * v + 1];
      int pgi = -1;
      for (int k = 0; k < 3; k++) {
        if (bsi[3 * e + k] >= 0) { /* ii->boundary() */
          int b = bsi[3 * e + k];
          if (on_line(m, b, px, py)) {
            if (pgi == -1 || p->surf[pgi].mb != 0) pgi = m->bgroup[b];
          }
        } else if (nbr[3 * e + k] >= 0) { /* ii->neighbor(): scan the neighbour's faces */
          int o = nbr[3 * e + k];
          for (int k2 = 0; k2 < 3; k2++) {
            int b = bsi[3 * o + k2];
            if (b < 0) continue;
            if (on_line(m, b, px, py)) {
              if (pgi == -1 || p->surf[pgi].mb != 0) {
                pgi = m->bgroup[b];
              } else {
                int bct = p->surf[pgi].mb; /* fall-through switch, :149-157 */
                if (bct != 0) pgi = m->bgroup[b];
              }
            }
          }
        }
      }
      double phi = phi_pb ? phi_pb[v] : 0.0;
      /* src/dirichlet_bc.hh:166-190 */
      x0[v] = (pgi > -1 && p->surf[pgi].cb == 0) ? p->surf[pgi].cpot : phi;
      x0[nv + v] = (pgi > -1 && p->surf[pgi].pb == 0) ? p->surf[pgi].pconc : p->c0 * exp(-phi);
      x0[2 * nv + v] = (pgi > -1 && p->surf[pgi].mb == 0) ? p->surf[pgi].mconc : p->c0 * exp(+phi);
    }
  }
  free(nbr);
  free(bsi);
  eh_free(&bh);
  eh_free(&eh);
}

/* ----------------------------------------------------------------------------------------
 * residual drivers (PDELab GridOperator::residual semantics, a8)
 * ---------------------------------------------------------------------------------------- */
int orc_operator_nfields(const orc_operator *op) {
  return (op->kind == ORC_OP_PNP || op->kind == ORC_OP_PNP_IMPLICIT_EULER) ? 3 : 1;
}

static void gather(const orc_mesh *m, int e, int nf, const double *x, double *xl) {
  const int *t = m->tri + 3 * e;
  for (int f = 0; f < nf; f++)
    for (int a = 0; a < 3; a++) xl[3 * f + a] = x[f * m->nv + t[a]];
}
static void scatter_add(const orc_mesh *m, int e, int nf, const double *rl, double *r) {
  const int *t = m->tri + 3 * e;
  for (int f = 0; f < nf; f++)
    for (int a = 0; a < 3; a++) r[f * m->nv + t[a]] += rl[3 * f + a];
}

/* evaluate the element residual of op (volume part only) at local x.  For time-discrete
 * operators the spatial part is scaled by dt and the old-time mass is subtracted outside. */
static void op_volume(const orc_mesh *m, const orc_params *p, const orc_operator *op, int e,
                      const elgeo *G, const double *xl, double *rl) {
  int nf = orc_operator_nfields(op);
  const int *t = m->tri + 3 * e;
  memset(rl, 0, sizeof(double) * 3 * nf);
  switch (op->kind) {
  case ORC_OP_PNP:
    lop_pnp_volume(G, p, xl, rl);
    break;
  case ORC_OP_PNP_IMPLICIT_EULER: {
    double rs[9] = {0};
    lop_pnp_volume(G, p, xl, rs);
    lop_pnpt_volume(G, p, p->tau, xl, rl);
    for (int i = 0; i < 9; i++) rl[i] += op->dt * rs[i];
  } break;
  case ORC_OP_PB:
    lop_pb_volume(G, p, xl, rl);
    break;
  case ORC_OP_DIFF:
  case ORC_OP_DIFF_IMPLICIT_EULER: {
    double phil[3] = {op->phi[t[0]], op->phi[t[1]], op->phi[t[2]]};
    if (op->kind == ORC_OP_DIFF) {
      lop_diff_volume(G, op->z, phil, xl, rl);
    } else {
      double rs[3] = {0};
      lop_diff_volume(G, op->z, phil, xl, rs);
      lop_difft_volume(G, xl, rl);
      for (int i = 0; i < 3; i++) rl[i] += op->dt * rs[i];
    }
  } break;
  case ORC_OP_POISSON: {
    double cpl[3] = {op->cp[t[0]], op->cp[t[1]], op->cp[t[2]]};
    double cml[3] = {op->cm[t[0]], op->cm[t[1]], op->cm[t[2]]};
    lop_poisson_volume(G, p, cpl, cml, xl, rl);
  } break;
  }
}

/* PDELab GridOperator::residual (a8; DefaultLocalAssembler, instantiated at
 * src/stationary_pnp_from_pb.hh:165,315-321), restated: per element in element order, the local
 * residual is alpha_volume, then alpha_boundary of each of the element's boundary intersections in
 * face order (boundary_face), and the local vector is added into r once.  One-step operators
 * (OneStepGridOperator, src/instationary_pnp_from_pb.hh:324; implicit Euler): r starts as the
 * const residual of the old time level, -M(x_old), assembled by its own element pass (preStage);
 * then per element the spatial operator's local vector (volume + boundary, weight dt) is added,
 * then the temporal operator's.  This library writes the implicit-Euler residual as
 * M(u) - M(u_old) + dt R(u); PDELab's implicit scaling R(u) + (M(u) - M(u_old)) / dt is the same
 * equation divided by dt, and every weight is 1 at the reference's tau = dt = 1 (pore.cfg).
 * Constrained rows are zero. */
void orc_op_residual(const orc_mesh *m, const orc_params *p, const orc_operator *op,
                     const double *x, double *r) {
  int nf = orc_operator_nfields(op);
  int n = nf * m->nv;
  memset(r, 0, sizeof(double) * n);
  double xl[9], rl[9];
  const int onestep = op->kind == ORC_OP_PNP_IMPLICIT_EULER || op->kind == ORC_OP_DIFF_IMPLICIT_EULER;
  /* const residual (old time level): -M(x_old), element by element */
  if (onestep) {
    for (int e = 0; e < m->nt; e++) {
      elgeo G;
      element_geometry(m, e, &G);
      gather(m, e, nf, op->x_old, xl);
      memset(rl, 0, sizeof rl);
      if (nf == 3)
        lop_pnpt_volume(&G, p, p->tau, xl, rl);
      else
        lop_difft_volume(&G, xl, rl);
      for (int i = 0; i < 3 * nf; i++) rl[i] = -rl[i];
      scatter_add(m, e, nf, rl, r);
    }
  }
  const int bnd = op->kind == ORC_OP_PNP || op->kind == ORC_OP_PNP_IMPLICIT_EULER ||
                  op->kind == ORC_OP_PB || op->kind == ORC_OP_POISSON;
  int *ebf = bnd ? elem_boundary_faces(m) : NULL;
  const double bscale = op->kind == ORC_OP_PNP_IMPLICIT_EULER ? op->dt : 1.0;
  for (int e = 0; e < m->nt; e++) {
    elgeo G;
    element_geometry(m, e, &G);
    gather(m, e, nf, x, xl);
    if (onestep) {
      /* the spatial operator's local vector, weight dt */
      double rs[9] = {0};
      memset(rl, 0, sizeof rl);
      if (nf == 3) {
        lop_pnp_volume(&G, p, xl, rs);
      } else {
        const int *t = m->tri + 3 * e;
        double phil[3] = {op->phi[t[0]], op->phi[t[1]], op->phi[t[2]]};
        lop_diff_volume(&G, op->z, phil, xl, rs);
      }
      for (int i = 0; i < 3 * nf; i++) rl[i] = op->dt * rs[i];
    } else {
      op_volume(m, p, op, e, &G, xl, rl);
    }
    if (ebf)
      for (int k = 0; k < 3; k++)
        if (ebf[3 * e + k] >= 0) boundary_face(m, p, op->flux, e, k, ebf[3 * e + k], nf, bscale, rl);
    scatter_add(m, e, nf, rl, r);
    if (onestep) { /* the temporal operator's local vector, weight 1 */
      memset(rl, 0, sizeof rl);
      if (nf == 3)
        lop_pnpt_volume(&G, p, p->tau, xl, rl);
      else
        lop_difft_volume(&G, xl, rl);
      scatter_add(m, e, nf, rl, r);
    }
  }
  free(ebf);
  /* constraints: constrained residual rows are zero */
  if (op->mask)
    for (int i = 0; i < n; i++)
      if (op->mask[i]) r[i] = 0.0;
}

void orc_pnp_residual(const orc_mesh *m, const orc_params *p, const double *flux,
                      const uint8_t *mask, const double *x, double *r) {
  orc_operator op;
  memset(&op, 0, sizeof op);
  op.kind = ORC_OP_PNP;
  op.flux = flux;
  op.mask = mask;
  orc_op_residual(m, p, &op, x, r);
}

void orc_pnpt_residual(const orc_mesh *m, const orc_params *p, const double *x, double *r) {
  memset(r, 0, sizeof(double) * 3 * m->nv);
  double xl[9], rl[9];
  for (int e = 0; e < m->nt; e++) {
    elgeo G;
    element_geometry(m, e, &G);
    gather(m, e, 3, x, xl);
    memset(rl, 0, sizeof rl);
    lop_pnpt_volume(&G, p, p->tau, xl, rl);
    scatter_add(m, e, 3, rl, r);
  }
}

void orc_pb_residual(const orc_mesh *m, const orc_params *p, const double *flux,
                     const uint8_t *mask, const double *x, double *r) {
  orc_operator op;
  memset(&op, 0, sizeof op);
  op.kind = ORC_OP_PB;
  op.flux = flux;
  op.mask = mask;
  orc_op_residual(m, p, &op, x, r);
}

void orc_diff_residual(const orc_mesh *m, const orc_params *p, const uint8_t *mask,
                       const double *phi, double z, const double *x, double *r) {
  orc_operator op;
  memset(&op, 0, sizeof op);
  op.kind = ORC_OP_DIFF;
  op.mask = mask;
  op.phi = phi;
  op.z = z;
  orc_op_residual(m, p, &op, x, r);
}

void orc_difft_residual(const orc_mesh *m, const double *x, double *r) {
  memset(r, 0, sizeof(double) * m->nv);
  double xl[3], rl[3];
  for (int e = 0; e < m->nt; e++) {
    elgeo G;
    element_geometry(m, e, &G);
    gather(m, e, 1, x, xl);
    memset(rl, 0, sizeof rl);
    lop_difft_volume(&G, xl, rl);
    scatter_add(m, e, 1, rl, r);
  }
}

void orc_poisson_residual(const orc_mesh *m, const orc_params *p, const double *flux,
                          const uint8_t *mask, const double *cp, const double *cm,
                          const double *x, double *r) {
  orc_operator op;
  memset(&op, 0, sizeof op);
  op.kind = ORC_OP_POISSON;
  op.flux = flux;
  op.mask = mask;
  op.cp = cp;
  op.cm = cm;
  orc_op_residual(m, p, &op, x, r);
}

/* ----------------------------------------------------------------------------------------
 * CSR pattern (FullVolumePattern) and Jacobian (a3, a8)
 * ---------------------------------------------------------------------------------------- */
static int cmp_int(const void *a, const void *b) {
  int x = *(const int *)a, y = *(const int *)b;
  return (x > y) - (x < y);
}

void orc_csr_pattern(const orc_mesh *m, int nf, orc_csr *A) {
  int nv = m->nv;
  /* vertex adjacency (including self) */
  int *deg = (int *)calloc((size_t)(nv > 0 ? nv : 0) + 1, sizeof(int));
  for (int e = 0; e < m->nt; e++)
    for (int a = 0; a < 3; a++) deg[m->tri[3 * e + a] + 1] += 3;
  for (int v = 0; v < nv; v++) deg[v + 1] += deg[v];
  int *adj = (int *)malloc(sizeof(int) * deg[nv]);
  int *fill = (int *)calloc((size_t)(nv > 0 ? nv : 1), sizeof(int));
  for (int e = 0; e < m->nt; e++)
    for (int a = 0; a < 3; a++) {
      int v = m->tri[3 * e + a];
      for (int b = 0; b < 3; b++) adj[deg[v] + fill[v]++] = m->tri[3 * e + b];
    }
  int *vcount = (int *)malloc(sizeof(int) * nv);
  for (int v = 0; v < nv; v++) {
    int *s = adj + deg[v];
    int n = fill[v];
    qsort(s, n, sizeof(int), cmp_int);
    int u = 0;
    for (int i = 0; i < n; i++)
      if (i == 0 || s[i] != s[i - 1]) s[u++] = s[i];
    vcount[v] = u;
  }
  A->n = nf * nv;
  A->rowptr = (int *)malloc(sizeof(int) * (A->n + 1));
  A->rowptr[0] = 0;
  for (int f = 0; f < nf; f++)
    for (int v = 0; v < nv; v++) A->rowptr[f * nv + v + 1] = nf * vcount[v];
  for (int i = 0; i < A->n; i++) A->rowptr[i + 1] += A->rowptr[i];
  A->nnz = A->rowptr[A->n];
  A->col = (int *)malloc(sizeof(int) * A->nnz);
  A->val = (double *)calloc(A->nnz, sizeof(double));
  for (int f = 0; f < nf; f++)
    for (int v = 0; v < nv; v++) {
      int *c = A->col + A->rowptr[f * nv + v];
      int k = 0;
      for (int g = 0; g < nf; g++)
        for (int i = 0; i < vcount[v]; i++) c[k++] = g * nv + adj[deg[v] + i];
    }
  free(deg);
  free(adj);
  free(fill);
  free(vcount);
}

void orc_csr_free(orc_csr *A) {
  free(A->rowptr);
  free(A->col);
  free(A->val);
  memset(A, 0, sizeof *A);
}

static double *csr_find(orc_csr *A, int i, int j) {
  int lo = A->rowptr[i], hi = A->rowptr[i + 1] - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    if (A->col[mid] == j) return A->val + mid;
    if (A->col[mid] < j)
      lo = mid + 1;
    else
      hi = mid - 1;
  }
  return NULL;
}

/* analytic element Jacobians (derivatives of the local residuals above) */
static void jac_pnp_volume(const elgeo *G, const orc_params *p, const double *xl, double *J,
                           double scale) {
  /* J[i*9+j] += scale * dR_i/dx_j */
  const double PI = p->pi;
  const qrule *R = rule_for_order(3);
  for (int q = 0; q < R->n; q++) {
    double factor = R->w[q] * G->adet;
    if (p->cylindrical) factor *= global_y(G, R->xi[q], R->eta[q]) * 2 * PI;
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double u_cp = 0, u_cm = 0, gphi[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      u_cp += xl[3 + i] * psi[i];
      u_cm += xl[6 + i] * psi[i];
      gphi[0] += xl[i] * G->g[i][0];
      gphi[1] += xl[i] * G->g[i][1];
    }
    double kap = 4 * PI * p->l_b;
    for (int i = 0; i < 3; i++) {
      double gp = gphi[0] * G->g[i][0] + gphi[1] * G->g[i][1];
      for (int j = 0; j < 3; j++) {
        double K = (G->g[j][0] * G->g[i][0] + G->g[j][1] * G->g[i][1]) * factor;
        double Mq = psi[j] * psi[i] * factor;
        J[(0 + i) * 9 + 0 + j] += scale * K;
        J[(0 + i) * 9 + 3 + j] += scale * kap * Mq;
        J[(0 + i) * 9 + 6 + j] -= scale * kap * Mq;
        J[(3 + i) * 9 + 0 + j] -= scale * u_cp * K;
        J[(3 + i) * 9 + 3 + j] += scale * (K - psi[j] * gp * factor);
        J[(6 + i) * 9 + 0 + j] += scale * u_cm * K;
        J[(6 + i) * 9 + 6 + j] += scale * (K + psi[j] * gp * factor);
      }
    }
  }
}

static void jac_pnpt_volume(const elgeo *G, const orc_params *p, double tau, double *J) {
  const double PI = p->pi;
  const qrule *R = rule_for_order(2);
  for (int q = 0; q < R->n; q++) {
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double factor = R->w[q] * G->adet;
    if (p->cylindrical) factor *= global_y(G, R->xi[q], R->eta[q]) * 2 * PI;
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        double v = tau * psi[j] * psi[i] * factor;
        J[(3 + i) * 9 + 3 + j] += v;
        J[(3 + i) * 9 + 6 + j] += v; /* Q2 */
      }
  }
}

static void jac_scalar_volume(const orc_params *p, const orc_operator *op, const elgeo *G,
                              const double *xl, const double *phil, double *J, double scale) {
  const double PI = p->pi;
  int kind = op->kind;
  int order = (kind == ORC_OP_PB || kind == ORC_OP_POISSON) ? 3 : 2;
  const qrule *R = rule_for_order(order);
  double gP[2] = {0, 0};
  if (phil)
    for (int i = 0; i < 3; i++) {
      gP[0] += phil[i] * G->g[i][0];
      gP[1] += phil[i] * G->g[i][1];
    }
  for (int q = 0; q < R->n; q++) {
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double factor = R->w[q] * G->adet;
    if (p->cylindrical && (kind == ORC_OP_PB || kind == ORC_OP_POISSON))
      factor *= global_y(G, R->xi[q], R->eta[q]) * 2 * PI;
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    for (int i = 0; i < 3; i++) {
      double gp = gP[0] * G->g[i][0] + gP[1] * G->g[i][1];
      for (int j = 0; j < 3; j++) {
        double K = (G->g[j][0] * G->g[i][0] + G->g[j][1] * G->g[i][1]) * factor;
        double v = K;
        if (kind == ORC_OP_PB) v += 8 * PI * p->l_b * p->c0 * cosh(u) * psi[j] * psi[i] * factor;
        if (kind == ORC_OP_DIFF || kind == ORC_OP_DIFF_IMPLICIT_EULER)
          v += op->z * psi[j] * gp * factor;
        J[i * 3 + j] += scale * v;
      }
    }
  }
}

static void jac_difft_volume(const elgeo *G, double *J) {
  const qrule *R = rule_for_order(2);
  for (int q = 0; q < R->n; q++) {
    double psi[3];
    p1_values(R->xi[q], R->eta[q], psi);
    double factor = R->w[q] * G->adet;
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) J[i * 3 + j] += psi[j] * psi[i] * factor;
  }
}

/* the spatial / temporal element residuals of a one-step operator (the FD Jacobian's evaluations) */
static void onestep_spatial(const orc_mesh *m, const orc_params *p, const orc_operator *op, int e,
                            const elgeo *G, const double *xl, double *rl) {
  int nf = orc_operator_nfields(op);
  memset(rl, 0, sizeof(double) * 3 * nf);
  if (nf == 3) {
    lop_pnp_volume(G, p, xl, rl);
  } else {
    const int *t = m->tri + 3 * e;
    double phil[3] = {op->phi[t[0]], op->phi[t[1]], op->phi[t[2]]};
    lop_diff_volume(G, op->z, phil, xl, rl);
  }
}
static void onestep_temporal(const orc_params *p, int nf, const elgeo *G, const double *xl,
                             double *rl) {
  memset(rl, 0, sizeof(double) * 3 * nf);
  if (nf == 3)
    lop_pnpt_volume(G, p, p->tau, xl, rl);
  else
    lop_difft_volume(G, xl, rl);
}

/* PDELab NumericalJacobianVolume::jacobian_volume, epsilon = 1e-7: J[i nl + j] = w (r_i(u + delta
 * e_j) - r_i(u)) / delta of the element residual `ev`, accumulated with weight w */
typedef void (*elres_fn)(const orc_mesh *, const orc_params *, const orc_operator *, int,
                         const elgeo *, const double *, double *);
static void fd_element(const orc_mesh *m, const orc_params *p, const orc_operator *op, int e,
                       const elgeo *G, const double *xl, int nl, elres_fn ev, double w, double *Jl) {
  double u[9], down[9], up[9];
  memcpy(u, xl, sizeof(double) * nl);
  ev(m, p, op, e, G, u, down);
  for (int j = 0; j < nl; j++) {
    double delta = 1e-7 * (1.0 + fabs(u[j]));
    u[j] += delta;
    ev(m, p, op, e, G, u, up);
    for (int i = 0; i < nl; i++) Jl[i * nl + j] += w * ((up[i] - down[i]) / delta);
    u[j] = xl[j];
  }
}
static void onestep_temporal_ev(const orc_mesh *m, const orc_params *p, const orc_operator *op,
                                int e, const elgeo *G, const double *xl, double *rl) {
  (void)m;
  (void)e;
  onestep_temporal(p, orc_operator_nfields(op), G, xl, rl);
}

/* BCRSMatrix accumulate of an element matrix: row search per entry */
static void scatter_jac(const orc_mesh *m, int e, int nl, const double *Jl, orc_csr *A) {
  const int *t = m->tri + 3 * e;
  const int nv = m->nv;
  for (int i = 0; i < nl; i++) {
    int I = (i / 3) * nv + t[i % 3];
    for (int j = 0; j < nl; j++) {
      int Jc = (j / 3) * nv + t[j % 3];
      *csr_find(A, I, Jc) += Jl[i * nl + j];
    }
  }
}

/* PDELab GridOperator::jacobian (a3, a8), restated like orc_op_residual: per element in element
 * order the local matrix (analytic, or fd = 1: NumericalJacobianVolume's forward differences of
 * the element residual -- the reference's own Jacobian, src/pnp_operator.hh:22-27) is added into
 * A once.  alpha_boundary's terms do not depend on x: NumericalJacobianBoundary adds exact zeros.
 * One-step operators: per element the spatial operator's matrix (weight dt), then the temporal
 * operator's.  Constrained rows -> identity (columns kept, non-symmetric). */
void orc_op_jacobian(const orc_mesh *m, const orc_params *p, const orc_operator *op,
                     const double *x, int fd, orc_csr *A) {
  int nf = orc_operator_nfields(op);
  int nl = 3 * nf;
  memset(A->val, 0, sizeof(double) * A->nnz);
  double xl[9], Jl[81];
  const int onestep = op->kind == ORC_OP_PNP_IMPLICIT_EULER || op->kind == ORC_OP_DIFF_IMPLICIT_EULER;
  for (int e = 0; e < m->nt; e++) {
    elgeo G;
    element_geometry(m, e, &G);
    gather(m, e, nf, x, xl);
    const int *t = m->tri + 3 * e;
    memset(Jl, 0, sizeof Jl);
    if (onestep) {
      if (fd) {
        fd_element(m, p, op, e, &G, xl, nl, onestep_spatial, op->dt, Jl);
      } else if (nf == 3) {
        jac_pnp_volume(&G, p, xl, Jl, op->dt);
      } else {
        double phil[3] = {op->phi[t[0]], op->phi[t[1]], op->phi[t[2]]};
        jac_scalar_volume(p, op, &G, xl, phil, Jl, op->dt);
      }
      scatter_jac(m, e, nl, Jl, A);
      memset(Jl, 0, sizeof Jl);
      if (fd)
        fd_element(m, p, op, e, &G, xl, nl, onestep_temporal_ev, 1.0, Jl);
      else if (nf == 3)
        jac_pnpt_volume(&G, p, p->tau, Jl);
      else
        jac_difft_volume(&G, Jl);
      scatter_jac(m, e, nl, Jl, A);
      continue;
    }
    if (fd) {
      fd_element(m, p, op, e, &G, xl, nl, op_volume, 1.0, Jl);
    } else {
      switch (op->kind) {
      case ORC_OP_PNP:
        jac_pnp_volume(&G, p, xl, Jl, 1.0);
        break;
      case ORC_OP_PB:
      case ORC_OP_POISSON:
        jac_scalar_volume(p, op, &G, xl, NULL, Jl, 1.0);
        break;
      case ORC_OP_DIFF: {
        double phil[3] = {op->phi[t[0]], op->phi[t[1]], op->phi[t[2]]};
        jac_scalar_volume(p, op, &G, xl, phil, Jl, 1.0);
      } break;
      }
    }
    scatter_jac(m, e, nl, Jl, A);
  }
  /* constrained rows -> identity (columns kept, non-symmetric) */
  if (op->mask)
    for (int i = 0; i < A->n; i++)
      if (op->mask[i])
        for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++)
          A->val[k] = (A->col[k] == i) ? 1.0 : 0.0;
}

/* ----------------------------------------------------------------------------------------
 * all-core CPU baseline (SURVEY.md §8(d) "CPU baseline (ii)"): the same reference algorithm
 * (element residual + NumericalJacobianVolume forward differences + BCRS-style scatter) with
 * the elements coloured so that no two elements of a colour share a vertex; each colour is an
 * OpenMP parallel loop with race-free scatters.  Test/bench infrastructure, like the rest.
 * ---------------------------------------------------------------------------------------- */
int orc_element_colors(const orc_mesh *m, int *color) {
  /* greedy: smallest colour not used by an element already coloured around its vertices */
  unsigned long long *used = (unsigned long long *)calloc((size_t)m->nv, sizeof *used);
  int ncol = 0;
  for (int e = 0; e < m->nt; e++) {
    const int *t = m->tri + 3 * e;
    unsigned long long u = used[t[0]] | used[t[1]] | used[t[2]];
    int c = 0;
    while (c < 64 && ((u >> c) & 1ULL)) c++;
    if (c == 64) {
      free(used);
      return -1;
    }
    color[e] = c;
    for (int a = 0; a < 3; a++) used[t[a]] |= 1ULL << c;
    if (c + 1 > ncol) ncol = c + 1;
  }
  free(used);
  return ncol;
}

void orc_assemble_mt(const orc_mesh *m, const orc_params *p, const orc_operator *op,
                     const double *x, const int *eorder, const int *cptr, int ncol, orc_csr *A,
                     double *r) {
  int nf = orc_operator_nfields(op);
  int nl = 3 * nf, nv = m->nv, n = nf * nv;
  memset(A->val, 0, sizeof(double) * A->nnz);
  memset(r, 0, sizeof(double) * n);
  for (int c = 0; c < ncol; c++) {
#pragma omp parallel for schedule(static)
    for (int k = cptr[c]; k < cptr[c + 1]; k++) {
      const int e = eorder[k];
      const int *t = m->tri + 3 * e;
      double xl[9], u[9], down[9], up[9], Jl[81];
      elgeo G;
      element_geometry(m, e, &G);
      gather(m, e, nf, x, xl);
      memcpy(u, xl, sizeof(double) * nl);
      op_volume(m, p, op, e, &G, u, down);
      scatter_add(m, e, nf, down, r);
      for (int j = 0; j < nl; j++) {
        double delta = 1e-7 * (1.0 + fabs(u[j]));
        u[j] += delta;
        op_volume(m, p, op, e, &G, u, up);
        for (int i = 0; i < nl; i++) Jl[i * nl + j] = (up[i] - down[i]) / delta;
        u[j] = xl[j];
      }
      for (int i = 0; i < nl; i++) {
        int I = (i / 3) * nv + t[i % 3];
        for (int j = 0; j < nl; j++) {
          int Jc = (j / 3) * nv + t[j % 3];
          *csr_find(A, I, Jc) += Jl[i * nl + j];
        }
      }
    }
  }
  if (op->kind == ORC_OP_PNP) boundary_flux(m, p, op->flux, 3, 0, 1.0, r);
  if (op->kind == ORC_OP_PB || op->kind == ORC_OP_POISSON)
    boundary_flux(m, p, op->flux, 1, 0, 1.0, r);
  if (op->mask) {
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++)
      if (op->mask[i]) {
        r[i] = 0.0;
        for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++)
          A->val[k] = (A->col[k] == i) ? 1.0 : 0.0;
      }
  }
}

int orc_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ----------------------------------------------------------------------------------------
 * linear algebra: ISTL BiCGSTABSolver + preconditioners (a11)
 * ---------------------------------------------------------------------------------------- */
/* all-core CPU baseline switch (bench cpu_baseline_all_cores): when on, the SpMV, the dots and
 * the vector updates of orc_bicgstab run as OpenMP row-parallel loops (dots then sum in OpenMP's
 * order, not ISTL's; the tests leave it off and keep the serial order) */
static int g_par = 0;
void orc_set_parallel(int on) { g_par = on; }
static int g_bj = 0, g_bj_nf = 1; /* block-Jacobi SSOR / ILU(0): blocks, fields per vertex */
void orc_set_block_jacobi(int nblocks, int nfields) {
  g_bj = nblocks > 1 ? nblocks : 0;
  g_bj_nf = nfields > 0 ? nfields : 1;
}

static double wtime(void) {
#ifdef _OPENMP
  return omp_get_wtime();
#else
  return 0.0;
#endif
}

void orc_spmv(const orc_csr *A, const double *x, double *y) {
#pragma omp parallel for schedule(static) if (g_par)
  for (int i = 0; i < A->n; i++) {
    double s = 0;
    for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++) s += A->val[k] * x[A->col[k]];
    y[i] = s;
  }
}

static double dot(int n, const double *a, const double *b) {
  double s = 0;
  if (g_par) {
#pragma omp parallel for schedule(static) reduction(+ : s)
    for (int i = 0; i < n; i++) s += a[i] * b[i];
    return s;
  }
  for (int i = 0; i < n; i++) s += a[i] * b[i];
  return s;
}

typedef struct {
  int kind;
  const orc_csr *A;
  orc_csr LU; /* ILU0 factors (diag stored inverted) */
  int *diag;
  int nb, nv;  /* block-Jacobi: blocks (0: sequential) and vertices per field */
  orc_csr B;   /* block-Jacobi: A without the couplings between blocks */
} prec_t;

static int bj_block(int nb, int nv, int i) { return (int)((long long)(i % nv) * nb / nv); }

static void prec_init(prec_t *P, const orc_csr *A, int kind) {
  P->kind = kind;
  P->A = A;
  P->nb = 0;
  memset(&P->LU, 0, sizeof P->LU);
  memset(&P->B, 0, sizeof P->B);
  if (g_bj > 1 && (kind == ORC_PREC_SSOR || kind == ORC_PREC_ILU0) && A->n % g_bj_nf == 0 &&
      A->n / g_bj_nf >= g_bj) {
    /* the rank-local matrices of a NOVLP backend: keep only couplings inside a row's block */
    int nb = g_bj, nv = A->n / g_bj_nf;
    orc_csr *B = &P->B;
    B->n = A->n;
    B->rowptr = (int *)malloc(sizeof(int) * (A->n + 1));
    B->col = (int *)malloc(sizeof(int) * A->nnz);
    B->val = (double *)malloc(sizeof(double) * A->nnz);
    int k2 = 0;
    B->rowptr[0] = 0;
    for (int i = 0; i < A->n; i++) {
      int bi = bj_block(nb, nv, i);
      for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++)
        if (bj_block(nb, nv, A->col[k]) == bi) {
          B->col[k2] = A->col[k];
          B->val[k2++] = A->val[k];
        }
      B->rowptr[i + 1] = k2;
    }
    B->nnz = k2;
    P->A = A = B;
    P->nb = nb;
    P->nv = nv;
  }
  P->diag = (int *)malloc(sizeof(int) * A->n);
  for (int i = 0; i < A->n; i++) {
    P->diag[i] = -1;
    for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++)
      if (A->col[k] == i) P->diag[i] = k;
  }
  if (kind == ORC_PREC_ILU0) {
    /* ISTL bilu0_decomposition for 1x1 blocks (IKJ, diagonal stored inverted) */
    orc_csr *L = &P->LU;
    L->n = A->n;
    L->nnz = A->nnz;
    L->rowptr = A->rowptr;
    L->col = A->col;
    L->val = (double *)malloc(sizeof(double) * A->nnz);
    memcpy(L->val, A->val, sizeof(double) * A->nnz);
    for (int i = 0; i < A->n; i++) {
      for (int ij = L->rowptr[i]; ij < L->rowptr[i + 1] && L->col[ij] < i; ij++) {
        int j = L->col[ij];
        L->val[ij] *= L->val[P->diag[j]]; /* A_ij * inv(A_jj) */
        int ik = ij + 1, jk = P->diag[j] + 1;
        while (ik < L->rowptr[i + 1] && jk < L->rowptr[j + 1]) {
          if (L->col[ik] == L->col[jk]) {
            L->val[ik] -= L->val[ij] * L->val[jk];
            ik++;
            jk++;
          } else if (L->col[ik] < L->col[jk])
            ik++;
          else
            jk++;
        }
      }
      L->val[P->diag[i]] = 1.0 / L->val[P->diag[i]];
    }
  }
}

static void prec_free(prec_t *P) {
  free(P->diag);
  if (P->LU.val) free(P->LU.val);
  if (P->B.rowptr) orc_csr_free(&P->B);
}

/* rows of block b in increasing order: field-major, each field's vertex range of the block */
#define BJ_ROWS(P, b, i, BODY)                                                               \
  do {                                                                                       \
    int v0_ = (int)(((long long)(b) * (P)->nv + (P)->nb - 1) / (P)->nb);                    \
    int v1_ = (int)(((long long)((b) + 1) * (P)->nv + (P)->nb - 1) / (P)->nb);              \
    for (int f_ = 0; f_ < (P)->A->n / (P)->nv; f_++)                                         \
      for (int i = f_ * (P)->nv + v0_; i < f_ * (P)->nv + v1_; i++) BODY                    \
  } while (0)
#define BJ_ROWS_REV(P, b, i, BODY)                                                           \
  do {                                                                                       \
    int v0_ = (int)(((long long)(b) * (P)->nv + (P)->nb - 1) / (P)->nb);                    \
    int v1_ = (int)(((long long)((b) + 1) * (P)->nv + (P)->nb - 1) / (P)->nb);              \
    for (int f_ = (P)->A->n / (P)->nv - 1; f_ >= 0; f_--)                                    \
      for (int i = f_ * (P)->nv + v1_ - 1; i >= f_ * (P)->nv + v0_; i--) BODY               \
  } while (0)

/* v = W^{-1} d, v is zero on entry (BiCGSTAB sets y = 0 before _prec.apply) */
static void prec_apply(const prec_t *P, double *v, const double *d) {
  const orc_csr *A = P->A;
  int n = A->n;
  if (P->kind == ORC_PREC_NONE) { /* Richardson, omega = 1 */
    for (int i = 0; i < n; i++) v[i] += 1.0 * d[i];
  } else if (P->kind == ORC_PREC_JACOBI) {
    for (int i = 0; i < n; i++) v[i] = d[i] / A->val[P->diag[i]];
  } else if (P->nb > 1 && P->kind == ORC_PREC_SSOR) { /* each block's SeqSSOR, in parallel */
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < P->nb; b++) {
      BJ_ROWS(P, b, i, {
        double rhs = d[i];
        for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++) rhs -= A->val[k] * v[A->col[k]];
        v[i] += 1.0 * (rhs / A->val[P->diag[i]]);
      });
      BJ_ROWS_REV(P, b, i, {
        double rhs = d[i];
        for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++) rhs -= A->val[k] * v[A->col[k]];
        v[i] += 1.0 * (rhs / A->val[P->diag[i]]);
      });
    }
  } else if (P->nb > 1) { /* each block's ILU(0) solve, in parallel */
    const orc_csr *L = &P->LU;
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < P->nb; b++) {
      BJ_ROWS(P, b, i, {
        double s = d[i];
        for (int k = L->rowptr[i]; k < P->diag[i]; k++) s -= L->val[k] * v[L->col[k]];
        v[i] = s;
      });
      BJ_ROWS_REV(P, b, i, {
        double s = v[i];
        for (int k = P->diag[i] + 1; k < L->rowptr[i + 1]; k++) s -= L->val[k] * v[L->col[k]];
        v[i] = s * L->val[P->diag[i]];
      });
    }
  } else if (P->kind == ORC_PREC_SSOR) { /* SeqSSOR(A, 1, 1.0): bsorf then bsorb */
    for (int i = 0; i < n; i++) {
      double rhs = d[i];
      for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++) rhs -= A->val[k] * v[A->col[k]];
      v[i] += 1.0 * (rhs / A->val[P->diag[i]]);
    }
    for (int i = n - 1; i >= 0; i--) {
      double rhs = d[i];
      for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++) rhs -= A->val[k] * v[A->col[k]];
      v[i] += 1.0 * (rhs / A->val[P->diag[i]]);
    }
  } else { /* ILU0 solve */
    const orc_csr *L = &P->LU;
    for (int i = 0; i < n; i++) {
      double s = d[i];
      for (int k = L->rowptr[i]; k < P->diag[i]; k++) s -= L->val[k] * v[L->col[k]];
      v[i] = s;
    }
    for (int i = n - 1; i >= 0; i--) {
      double s = v[i];
      for (int k = P->diag[i] + 1; k < L->rowptr[i + 1]; k++) s -= L->val[k] * v[L->col[k]];
      v[i] = s * L->val[P->diag[i]];
    }
  }
}

/* one application of the preconditioner from v = 0 (test hook: the GPU's pnp_prec_apply) */
void orc_prec_apply(const orc_csr *A, int prec, const double *d, double *v) {
  prec_t P;
  prec_init(&P, A, prec);
  memset(v, 0, sizeof(double) * A->n);
  prec_apply(&P, v, d);
  prec_free(&P);
}

void orc_bicgstab(const orc_csr *A, int prec, double reduction, int maxit, double *x, double *b,
                  orc_solve_result *res) {
  const double EPSILON = 1e-80;
  int n = A->n;
  double *r = b;
  double *p = (double *)calloc(n, sizeof(double));
  double *v = (double *)calloc(n, sizeof(double));
  double *t = (double *)calloc(n, sizeof(double));
  double *y = (double *)calloc(n, sizeof(double));
  double *rt = (double *)malloc(sizeof(double) * n);
  prec_t P;
  memset(res, 0, sizeof *res);
  double t_setup = wtime();
  prec_init(&P, A, prec);
  res->setup_seconds = wtime() - t_setup;
  double t_iter = wtime();
  /* r = b - A x */
  orc_spmv(A, x, t);
  for (int i = 0; i < n; i++) r[i] -= t[i];
  memcpy(rt, r, sizeof(double) * n);
  double norm = sqrt(dot(n, r, r)), norm_0 = norm;
  double rho = 1, alpha = 1, omega = 1, rho_new, beta, h;
  res->defect0 = norm_0;
  double it = 0;
  if (norm < reduction * norm_0 || norm < 1e-30) {
    res->converged = 1;
    res->defect = norm;
    prec_free(&P);
    free(p); free(v); free(t); free(y); free(rt);
    return;
  }
  for (it = 0.5; it < maxit; it += .5) {
    rho_new = dot(n, rt, r);
    if (fabs(rho) <= EPSILON) { res->breakdown = 1; break; }
    if (fabs(omega) <= EPSILON) { res->breakdown = 2; break; }
    if (it < 1) {
      memcpy(p, r, sizeof(double) * n);
    } else {
      beta = (rho_new / rho) * (alpha / omega);
#pragma omp parallel for schedule(static) if (g_par)
      for (int i = 0; i < n; i++) p[i] = beta * (p[i] - omega * v[i]) + r[i];
    }
    memset(y, 0, sizeof(double) * n);
    prec_apply(&P, y, p);
    orc_spmv(A, y, v);
    h = dot(n, rt, v);
    if (fabs(h) < EPSILON) { res->breakdown = 3; break; }
    alpha = rho_new / h;
#pragma omp parallel for schedule(static) if (g_par)
    for (int i = 0; i < n; i++) {
      x[i] += alpha * y[i];
      r[i] -= alpha * v[i];
    }
    norm = sqrt(dot(n, r, r));
    if (norm < reduction * norm_0) { res->converged = 1; break; }
    it += .5;
    memset(y, 0, sizeof(double) * n);
    prec_apply(&P, y, r);
    orc_spmv(A, y, t);
    omega = dot(n, t, r) / dot(n, t, t);
#pragma omp parallel for schedule(static) if (g_par)
    for (int i = 0; i < n; i++) {
      x[i] += omega * y[i];
      r[i] -= omega * t[i];
    }
    rho = rho_new;
    norm = sqrt(dot(n, r, r));
    if (norm < reduction * norm_0 || norm < 1e-30) { res->converged = 1; break; }
  }
  res->iter_seconds = wtime() - t_iter;
  if (it > maxit) it = maxit;
  res->it_half = it;
  res->iterations = (int)ceil(it);
  res->defect = norm;
  res->reduction = norm / norm_0;
  prec_free(&P);
  free(p); free(v); free(t); free(y); free(rt);
}

/* ISTL CGSolver::apply (dune-istl 2.2 solvers.hh; the ISTLBackend_NOVLP_CG_NOPREC / _CG_Jacobi
 * backends selected by LINEARSOLVER 3 / 4, src/instationary_pnp_from_pb_md.hh:198-206):
 *   r = b - A x; def0 = ||r||; done if def0 < 1e-30;  p = M^{-1} r; rho = <p, r>
 *   for i = 1 .. maxit:  q = A p; lambda = rho / <p, q>; x += lambda p; r -= lambda q;
 *                        def = ||r||; converged if def < reduction def0 or def < 1e-30;
 *                        q = M^{-1} r; rho' = <q, r>; p = q + (rho'/rho) p; rho = rho'
 * iterations = i (matrix-vector products).  b is overwritten with the residual. */
void orc_cg(const orc_csr *A, int prec, double reduction, int maxit, double *x, double *b,
            orc_solve_result *res) {
  int n = A->n;
  double *r = b;
  double *p = (double *)calloc(n, sizeof(double));
  double *q = (double *)calloc(n, sizeof(double));
  prec_t P;
  prec_init(&P, A, prec);
  memset(res, 0, sizeof *res);
  orc_spmv(A, x, q);
  for (int i = 0; i < n; i++) r[i] -= q[i];
  double def0 = sqrt(dot(n, r, r)), def = def0;
  res->defect0 = def0;
  int it = 0;
  if (def0 < 1e-30) {
    res->converged = 1;
  } else {
    prec_apply(&P, p, r);
    double rho = dot(n, p, r);
    for (it = 1; it <= maxit; it++) {
      orc_spmv(A, p, q);
      const double lambda = rho / dot(n, p, q);
      for (int i = 0; i < n; i++) x[i] += lambda * p[i];
      for (int i = 0; i < n; i++) r[i] -= lambda * q[i];
      def = sqrt(dot(n, r, r));
      if (def < reduction * def0 || def < 1e-30) {
        res->converged = 1;
        break;
      }
      memset(q, 0, sizeof(double) * n);
      prec_apply(&P, q, r);
      const double rho_new = dot(n, q, r);
      const double beta = rho_new / rho;
      for (int i = 0; i < n; i++) p[i] = q[i] + beta * p[i];
      rho = rho_new;
    }
    if (it > maxit) it = maxit;
  }
  res->it_half = it;
  res->iterations = it;
  res->defect = def;
  res->reduction = def0 > 0 ? def / def0 : 0.0;
  prec_free(&P);
  free(p);
  free(q);
}

/* ----------------------------------------------------------------------------------------
 * Newton (a12), PDELab newton.hh semantics
 * ---------------------------------------------------------------------------------------- */
void orc_newton(const orc_mesh *m, const orc_params *p, const orc_operator *op, double *u,
                const orc_newton_opts *o, orc_newton_result *res) {
  int nf = orc_operator_nfields(op);
  int n = nf * m->nv;
  double *r = (double *)malloc(sizeof(double) * n);
  double *z = (double *)malloc(sizeof(double) * n);
  double *prevu = (double *)malloc(sizeof(double) * n);
  orc_csr A;
  orc_csr_pattern(m, nf, &A);
  memset(res, 0, sizeof *res);

  orc_op_residual(m, p, op, u, r);
  res->defect = sqrt(dot(n, r, r));
  res->first_defect = res->defect;
  double prev_defect = res->defect;
  for (;;) {
    /* terminate() */
    res->converged = res->defect < o->abs_limit || res->defect < res->first_defect * o->reduction;
    if (res->converged) break;
    if (res->iterations >= o->maxit) { res->status = -1; break; }
    /* prepare_step: reassemble_threshold = 0 -> always */
    orc_op_jacobian(m, p, op, u, o->fd_jacobian, &A);
    double stop_defect = fmax(res->first_defect * o->reduction, o->abs_limit);
    double lin_red;
    if (stop_defect / (10 * res->defect) > res->defect * res->defect / (prev_defect * prev_defect))
      lin_red = stop_defect / (10 * res->defect);
    else
      lin_red = fmin(o->min_linear_reduction,
                     res->defect * res->defect / (prev_defect * prev_defect));
    prev_defect = res->defect;
    /* linearSolve */
    memset(z, 0, sizeof(double) * n);
    orc_solve_result sr;
    orc_bicgstab(&A, o->prec, lin_red, o->linear_maxit, z, r, &sr);
    res->linear_iterations += sr.iterations;
    if (res->iterations < ORC_NEWTON_MAX_RECORD) res->step_linear_iterations[res->iterations] = sr.iterations;
    if (!sr.converged) { res->status = -3; break; }
    /* line_search: hackbuschReuskenAcceptBest */
    double lambda = 1.0, best_lambda = 0.0, best_defect = res->defect;
    memcpy(prevu, u, sizeof(double) * n);
    int i = 0, ls_fail = 0;
    for (;;) {
      for (int k = 0; k < n; k++) u[k] -= lambda * z[k];
      orc_op_residual(m, p, op, u, r);
      res->defect = sqrt(dot(n, r, r));
      if (res->defect <= (1.0 - lambda / 4) * prev_defect) break;
      if (res->defect < best_defect) {
        best_defect = res->defect;
        best_lambda = lambda;
      }
      if (++i >= o->line_search_maxit) {
        if (best_lambda == 0.0) { ls_fail = 1; break; }
        if (best_lambda != lambda) {
          memcpy(u, prevu, sizeof(double) * n);
          for (int k = 0; k < n; k++) u[k] -= best_lambda * z[k];
          orc_op_residual(m, p, op, u, r);
          res->defect = sqrt(dot(n, r, r));
        }
        break;
      }
      lambda *= 0.5;
      memcpy(u, prevu, sizeof(double) * n);
    }
    if (ls_fail) { res->status = -2; break; }
    res->iterations++;
  }
  orc_csr_free(&A);
  free(r);
  free(z);
  free(prevu);
}

/* calcIonFlux, src/ionFlux.hh:8-96.  Elements in tri order, intersections in DUNE's triangle
 * facet order (0: vertices 0-1, 1: 0-2, 2: 1-2).  At the facet centre (local coordinates in the
 * element) the P1 fields are evaluated (:60-66), with the element's constant gradients; factor
 * = facet length (:69), x 2*PI*y(centre) when cylindrical (:70-71, PI = 3.1415 at :4).
 *   gradCp *= -factor; gradCm *= -factor; gradphi *= factor; gradphi *= cp        (:72-76)
 *   ip[g] += (gradCp + gradphi) . n                                               (:80)
 *   gradphi *= cm / cp; im[g] += (gradCm - gradphi) . n                           (:84-85)
 * for boundary intersections only, g = pg[boundarySegmentIndex] (:79), n = unit outer normal. */
void orc_ion_flux(const orc_mesh *m, const orc_params *p, const double *x, double *ip,
                  double *im) {
  static const int fv[3][2] = {{0, 1}, {0, 2}, {1, 2}};
  static const double centre[3][2] = {{0.5, 0.0}, {0.0, 0.5}, {0.5, 0.5}};
  const int nv = m->nv;
  ehash h;
  eh_init(&h, m->nb);
  for (int b = 0; b < m->nb; b++) eh_put(&h, ekey(m->bseg[2 * b], m->bseg[2 * b + 1]), b);
  for (int g = 0; g < p->nsurf; g++) ip[g] = im[g] = 0.0;
  for (int e = 0; e < m->nt; e++) {
    const int *t = m->tri + 3 * e;
    elgeo G;
    element_geometry(m, e, &G);
    double gphi[2] = {0, 0}, gcp[2] = {0, 0}, gcm[2] = {0, 0};
    for (int i = 0; i < 3; i++)
      for (int d = 0; d < 2; d++) {
        gphi[d] += x[t[i]] * G.g[i][d];
        gcp[d] += x[nv + t[i]] * G.g[i][d];
        gcm[d] += x[2 * nv + t[i]] * G.g[i][d];
      }
    for (int k = 0; k < 3; k++) {
      const int ia = fv[k][0], ic = fv[k][1], io = 3 - ia - ic;
      const int b = eh_get(&h, ekey(t[ia], t[ic]));
      if (b < 0) continue;
      double psi[3];
      p1_values(centre[k][0], centre[k][1], psi);
      double cp = 0, cm = 0;
      for (int i = 0; i < 3; i++) {
        cp += psi[i] * x[nv + t[i]];
        cm += psi[i] * x[2 * nv + t[i]];
      }
      const double *pa = m->xy + 2 * t[ia], *pc = m->xy + 2 * t[ic], *po = m->xy + 2 * t[io];
      const double tx = pc[0] - pa[0], ty = pc[1] - pa[1];
      const double len = sqrt(tx * tx + ty * ty);
      double factor = len;
      if (p->cylindrical) factor *= 2 * p->pi * global_y(&G, centre[k][0], centre[k][1]);
      double nx = ty / len, ny = -tx / len;
      if (nx * (po[0] - pa[0]) + ny * (po[1] - pa[1]) > 0) {
        nx = -nx;
        ny = -ny;
      }
      double gCp[2], gCm[2], gPh[2];
      for (int d = 0; d < 2; d++) {
        gCp[d] = -factor * gcp[d];
        gCm[d] = -factor * gcm[d];
        gPh[d] = factor * gphi[d] * cp;
      }
      const int g = m->bgroup[b];
      ip[g] += (gCp[0] + gPh[0]) * nx + (gCp[1] + gPh[1]) * ny;
      for (int d = 0; d < 2; d++) gPh[d] *= cm / cp;
      im[g] += (gCm[0] - gPh[0]) * nx + (gCm[1] - gPh[1]) * ny;
    }
  }
  eh_free(&h);
}
