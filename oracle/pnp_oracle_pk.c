/*
 * pnp_oracle_pk.c — CPU restatement of the reference's P_k (PDEGREE = 2, 3) scalar operators.
 * TEST INFRASTRUCTURE ONLY (see pnp_oracle.h for the parity status): nothing in the product
 * links or calls this code.
 *
 * The reference instantiates its operator-split driver on Pk2DLocalFiniteElementMap<GV, Coord,
 * Real, PDEGREE> (src/instationary_pnp_from_pb_md.hh:26-28, 125, 245-247) and builds one program
 * per (LINEARSOLVER, PDEGREE) pair (src/Makefile.am:43-111).  The local operators loop over the
 * quadrature rule of their intorder and over lfsu.size() basis functions (src/pb_operator.hh:
 * 67-121, src/poisson_operator.hh:67-126, src/diffusion_operator.hh:59-111,
 * src/diffusion_toperator.hh:52-72); nothing in them is P1-specific, so on P_k the same code runs
 * with the degree-k Lagrange basis.  Restated here:
 *   - the P_k Lagrange space (dune-localfunctions Pk2DLocalBasis: equidistant Lagrange points;
 *     the global numbering is this oracle's own: vertices, then the k-1 points of each edge in
 *     order of the edge's first appearance, then the interior points; tests match nodes by
 *     coordinates);
 *   - the basis from the inverse Vandermonde matrix of the monomials xi^p eta^q, p + q <= k (an
 *     independent route to the same functions the product evaluates as products of barycentric
 *     factors);
 *   - quadrature: order 2 the 3-point rule, order 3 the Strang-Fix 4-point rule (as in
 *     pnp_oracle.c), order 5 Radon's 7-point rule (dune-geometry's order-5 simplex rule,
 *     restated: parity with the DUNE tables unpinned), faces the 2-point Gauss rule (order 3);
 *   - alpha_boundary per element face on a boundary segment, with the element's 2-D basis at the
 *     face points (src/pb_operator.hh:126-194, src/poisson_operator.hh:131-199);
 *   - NonoverlappingConformingDirichletConstraints: every node of a Dirichlet face constrained.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "pnp_oracle.h"

/* ---- space -------------------------------------------------------------------------------- */
typedef struct {
  long long key;
  int first; /* 3 * element + face of the first appearance */
} ekey_t;

static int cmp_key(const void *a, const void *b) {
  const ekey_t *x = (const ekey_t *)a, *y = (const ekey_t *)b;
  if (x->key != y->key) return x->key < y->key ? -1 : 1;
  return (x->first > y->first) - (x->first < y->first);
}
static int cmp_first(const void *a, const void *b) {
  const ekey_t *x = (const ekey_t *)a, *y = (const ekey_t *)b;
  return (x->first > y->first) - (x->first < y->first);
}
static long long pair_key(int a, int b) {
  if (a > b) {
    int t = a;
    a = b;
    b = t;
  }
  return ((long long)a << 32) | (unsigned)b;
}
static const int FACE[3][2] = {{0, 1}, {0, 2}, {1, 2}};

/* edge id of a vertex pair: binary search in the sorted (key -> id) table */
typedef struct {
  long long *key;
  int *id;
  int n;
} etab;
static int etab_find(const etab *T, long long k) {
  int lo = 0, hi = T->n - 1;
  while (lo <= hi) {
    int mid = (lo + hi) >> 1;
    if (T->key[mid] == k) return T->id[mid];
    if (T->key[mid] < k)
      lo = mid + 1;
    else
      hi = mid - 1;
  }
  return -1;
}
static void etab_build(const orc_mesh *m, etab *T) {
  ekey_t *all = (ekey_t *)malloc(sizeof(ekey_t) * 3 * (size_t)m->nt);
  for (int e = 0; e < m->nt; e++)
    for (int f = 0; f < 3; f++) {
      all[3 * e + f].key = pair_key(m->tri[3 * e + FACE[f][0]], m->tri[3 * e + FACE[f][1]]);
      all[3 * e + f].first = 3 * e + f;
    }
  qsort(all, 3 * (size_t)m->nt, sizeof(ekey_t), cmp_key);
  int nu = 0;
  for (int i = 0; i < 3 * m->nt; i++)
    if (i == 0 || all[i].key != all[i - 1].key) all[nu++] = all[i];
  ekey_t *byfirst = (ekey_t *)malloc(sizeof(ekey_t) * (nu ? nu : 1));
  memcpy(byfirst, all, sizeof(ekey_t) * nu);
  qsort(byfirst, nu, sizeof(ekey_t), cmp_first);
  /* id = rank by first appearance; table sorted by key */
  T->n = nu;
  T->key = (long long *)malloc(sizeof(long long) * (nu ? nu : 1));
  T->id = (int *)malloc(sizeof(int) * (nu ? nu : 1));
  for (int i = 0; i < nu; i++) T->key[i] = all[i].key;
  for (int r = 0; r < nu; r++) {
    /* position of byfirst[r].key in the sorted table */
    int lo = 0, hi = nu - 1;
    while (lo < hi) {
      int mid = (lo + hi) >> 1;
      if (T->key[mid] < byfirst[r].key)
        lo = mid + 1;
      else
        hi = mid;
    }
    T->id[lo] = r;
  }
  free(all);
  free(byfirst);
}
static void etab_free(etab *T) {
  free(T->key);
  free(T->id);
}

/* lattice (a1, a2) = (k xi, k eta) of local node n in the documented local order */
static void local_lattice(int k, int n, int *a1, int *a2) {
  static const int V[3][2] = {{0, 0}, {1, 0}, {0, 1}};
  if (n < 3) {
    *a1 = k * V[n][0];
    *a2 = k * V[n][1];
    return;
  }
  n -= 3;
  if (n < 3 * (k - 1)) {
    int f = n / (k - 1), s = 1 + n % (k - 1);
    const int *p = V[FACE[f][0]], *q = V[FACE[f][1]];
    *a1 = (k - s) * p[0] + s * q[0];
    *a2 = (k - s) * p[1] + s * q[1];
    return;
  }
  n -= 3 * (k - 1);
  int c = 0;
  for (int i = 1; i < k; i++)
    for (int j = 1; i + j < k; j++, c++)
      if (c == n) {
        *a1 = i;
        *a2 = j;
        return;
      }
}

int orc_pk_build(const orc_mesh *m, int k, orc_pk *S) {
  memset(S, 0, sizeof *S);
  if (k < 1 || k > 3) return -1;
  S->k = k;
  S->nl = (k + 1) * (k + 2) / 2;
  etab T;
  etab_build(m, &T);
  const int ni = (k - 1) * (k - 2) / 2;
  S->nedge = T.n;
  S->nn = m->nv + T.n * (k - 1) + m->nt * ni;
  S->xy = (double *)malloc(sizeof(double) * 2 * (size_t)S->nn);
  S->enode = (int *)malloc(sizeof(int) * (size_t)S->nl * m->nt);
  memcpy(S->xy, m->xy, sizeof(double) * 2 * (size_t)m->nv);
  for (int e = 0; e < m->nt; e++) {
    const int *t = m->tri + 3 * e;
    int *en = S->enode + (size_t)S->nl * e;
    const double *P0 = m->xy + 2 * t[0], *P1 = m->xy + 2 * t[1], *P2 = m->xy + 2 * t[2];
    for (int n = 0; n < S->nl; n++) {
      int a1, a2;
      local_lattice(k, n, &a1, &a2);
      int node;
      if (n < 3) {
        node = t[n];
      } else if (n < 3 + 3 * (k - 1)) {
        int f = (n - 3) / (k - 1), s = 1 + (n - 3) % (k - 1);
        int va = t[FACE[f][0]], vb = t[FACE[f][1]];
        int id = etab_find(&T, pair_key(va, vb));
        int from_lo = va < vb ? s : k - s;
        node = m->nv + id * (k - 1) + from_lo - 1;
        /* edge points: lo + (from_lo / k) (hi - lo) */
        int lo = va < vb ? va : vb, hi = va < vb ? vb : va;
        for (int d = 0; d < 2; d++)
          S->xy[2 * node + d] = m->xy[2 * lo + d] +
                                ((double)from_lo / k) * (m->xy[2 * hi + d] - m->xy[2 * lo + d]);
      } else {
        node = m->nv + T.n * (k - 1) + e * ni + (n - 3 - 3 * (k - 1));
        const int a0 = k - a1 - a2;
        for (int d = 0; d < 2; d++) S->xy[2 * node + d] = (a0 * P0[d] + a1 * P1[d] + a2 * P2[d]) / k;
      }
      en[n] = node;
    }
  }
  etab_free(&T);
  return 0;
}

void orc_pk_free(orc_pk *S) {
  free(S->xy);
  free(S->enode);
  memset(S, 0, sizeof *S);
}

/* ---- basis: inverse Vandermonde of the monomials ------------------------------------------- */
typedef struct {
  int k, nl;
  double C[10][10]; /* phi_n = sum_j C[n][j] mono_j */
  int pw[10][2];
} pkbasis;

static void basis_init(int k, pkbasis *B) {
  B->k = k;
  B->nl = (k + 1) * (k + 2) / 2;
  int nl = B->nl, c = 0;
  for (int d = 0; d <= k; d++)
    for (int q = 0; q <= d; q++, c++) {
      B->pw[c][0] = d - q;
      B->pw[c][1] = q;
    }
  double V[10][20];
  for (int n = 0; n < nl; n++) {
    int a1, a2;
    local_lattice(k, n, &a1, &a2);
    double xi = (double)a1 / k, eta = (double)a2 / k;
    for (int j = 0; j < nl; j++) V[n][j] = pow(xi, B->pw[j][0]) * pow(eta, B->pw[j][1]);
    for (int j = 0; j < nl; j++) V[n][nl + j] = n == j ? 1.0 : 0.0;
  }
  /* Gauss-Jordan with partial pivoting: V -> [I | V^{-1}] ; phi_n(x) = sum_j mono_j(x) Vinv[j][n] */
  for (int col = 0; col < nl; col++) {
    int piv = col;
    for (int r = col + 1; r < nl; r++)
      if (fabs(V[r][col]) > fabs(V[piv][col])) piv = r;
    for (int j = 0; j < 2 * nl; j++) {
      double t = V[col][j];
      V[col][j] = V[piv][j];
      V[piv][j] = t;
    }
    double d = V[col][col];
    for (int j = 0; j < 2 * nl; j++) V[col][j] /= d;
    for (int r = 0; r < nl; r++) {
      if (r == col) continue;
      double f = V[r][col];
      if (f != 0.0)
        for (int j = 0; j < 2 * nl; j++) V[r][j] -= f * V[col][j];
    }
  }
  for (int n = 0; n < nl; n++)
    for (int j = 0; j < nl; j++) B->C[n][j] = V[j][nl + n];
}

static void basis_eval(const pkbasis *B, double xi, double eta, double *phi, double (*dphi)[2]) {
  for (int n = 0; n < B->nl; n++) {
    double v = 0, dx = 0, dy = 0;
    for (int j = 0; j < B->nl; j++) {
      int p = B->pw[j][0], q = B->pw[j][1];
      double c = B->C[n][j];
      v += c * pow(xi, p) * pow(eta, q);
      if (p > 0) dx += c * p * pow(xi, p - 1) * pow(eta, q);
      if (q > 0) dy += c * q * pow(xi, p) * pow(eta, q - 1);
    }
    if (phi) phi[n] = v;
    if (dphi) {
      dphi[n][0] = dx;
      dphi[n][1] = dy;
    }
  }
}

void orc_pk_basis(int k, double xi, double eta, double *phi, double *dphi) {
  pkbasis B;
  basis_init(k, &B);
  basis_eval(&B, xi, eta, phi, (double(*)[2])dphi);
}

/* ---- quadrature ---------------------------------------------------------------------------- */
typedef struct {
  int n;
  double xi[7], eta[7], w[7];
} prule;

static void rule_of(int order, prule *R) {
  if (order <= 2) {
    *R = (prule){3, {4.0 / 6.0, 1.0 / 6.0, 1.0 / 6.0}, {1.0 / 6.0, 4.0 / 6.0, 1.0 / 6.0},
                 {0.5 / 3.0, 0.5 / 3.0, 0.5 / 3.0}};
  } else if (order == 3) {
    *R = (prule){4, {10.0 / 30.0, 18.0 / 30.0, 6.0 / 30.0, 6.0 / 30.0},
                 {10.0 / 30.0, 6.0 / 30.0, 18.0 / 30.0, 6.0 / 30.0},
                 {0.5 * -27.0 / 48.0, 0.5 * 25.0 / 48.0, 0.5 * 25.0 / 48.0, 0.5 * 25.0 / 48.0}};
  } else { /* order 5: Radon's 7-point rule */
    const double s = sqrt(15.0), a1 = (6.0 - s) / 21.0, a2 = (6.0 + s) / 21.0;
    const double w1 = (155.0 - s) / 2400.0, w2 = (155.0 + s) / 2400.0;
    *R = (prule){7,
                 {1.0 / 3.0, a1, 1.0 - 2.0 * a1, a1, a2, 1.0 - 2.0 * a2, a2},
                 {1.0 / 3.0, a1, a1, 1.0 - 2.0 * a1, a2, a2, 1.0 - 2.0 * a2},
                 {9.0 / 80.0, w1, w1, w1, w2, w2, w2}};
  }
}

int orc_quadrature_rule(int order, double *xi, double *eta, double *w) {
  prule R;
  rule_of(order, &R);
  for (int q = 0; q < R.n; q++) {
    xi[q] = R.xi[q];
    eta[q] = R.eta[q];
    w[q] = R.w[q];
  }
  return R.n;
}

/* ---- element geometry ---------------------------------------------------------------------- */
typedef struct {
  double x0, y0, J00, J01, J10, J11, adet;
  double it[2][2]; /* jacobianInverseTransposed */
} pgeo;

static void pgeo_of(const orc_mesh *m, int e, pgeo *G) {
  const int *t = m->tri + 3 * e;
  const double *p0 = m->xy + 2 * t[0], *p1 = m->xy + 2 * t[1], *p2 = m->xy + 2 * t[2];
  G->x0 = p0[0];
  G->y0 = p0[1];
  G->J00 = p1[0] - p0[0];
  G->J01 = p2[0] - p0[0];
  G->J10 = p1[1] - p0[1];
  G->J11 = p2[1] - p0[1];
  double det = G->J00 * G->J11 - G->J01 * G->J10;
  G->adet = fabs(det);
  G->it[0][0] = G->J11 / det;
  G->it[0][1] = -G->J10 / det;
  G->it[1][0] = -G->J01 / det;
  G->it[1][1] = G->J00 / det;
}

/* gradphi = jac.mv(js) (src/pb_operator.hh:103-105) */
static void phys_grads(const pgeo *G, int nl, double (*js)[2], double (*g)[2]) {
  for (int i = 0; i < nl; i++) {
    g[i][0] = G->it[0][0] * js[i][0] + G->it[0][1] * js[i][1];
    g[i][1] = G->it[1][0] * js[i][0] + G->it[1][1] * js[i][1];
  }
}

/* element residual (volume part) of op at local values xl; fl0 / fl1 the frozen fields at the
 * element's nodes; rl zeroed here.  mass_only: DiffusionTOperator alone. */
static void pk_volume(const pkbasis *B, const pgeo *G, const orc_params *p, int kind, double dt,
                      double z, const double *xl, const double *fl0, const double *fl1,
                      int mass_only, double *rl) {
  const int nl = B->nl;
  const double PI = p->pi;
  double phi[10], js[10][2], g[10][2];
  prule R;
  memset(rl, 0, sizeof(double) * nl);
  if (mass_only || kind == ORC_OP_DIFF_IMPLICIT_EULER) {
    /* DiffusionTOperator, intorder 5 (cptop(5), src/instationary_pnp_from_pb_md.hh:363),
     * src/diffusion_toperator.hh:57-72 */
    rule_of(5, &R);
    for (int q = 0; q < R.n; q++) {
      basis_eval(B, R.xi[q], R.eta[q], phi, NULL);
      double u = 0.0;
      for (int i = 0; i < nl; i++) u += xl[i] * phi[i];
      double factor = R.w[q] * G->adet;
      for (int i = 0; i < nl; i++) rl[i] += u * phi[i] * factor;
    }
    if (mass_only) return;
  }
  if (kind == ORC_OP_PB || kind == ORC_OP_POISSON) {
    rule_of(3, &R); /* intorder_ = 3 */
    for (int q = 0; q < R.n; q++) {
      double factor = R.w[q] * G->adet;
      if (p->cylindrical) factor *= (G->y0 + G->J10 * R.xi[q] + G->J11 * R.eta[q]) * 2 * PI;
      basis_eval(B, R.xi[q], R.eta[q], phi, js);
      double u = 0.0;
      for (int i = 0; i < nl; i++) u += xl[i] * phi[i];
      double cp = 0.0, cm = 0.0;
      if (kind == ORC_OP_POISSON) { /* cpDgf / cmDgf.evaluate, src/poisson_operator.hh:97-100 */
        for (int i = 0; i < nl; i++) cp += fl0[i] * phi[i];
        for (int i = 0; i < nl; i++) cm += fl1[i] * phi[i];
      }
      phys_grads(G, nl, js, g);
      double gu[2] = {0.0, 0.0};
      for (int i = 0; i < nl; i++) {
        gu[0] += xl[i] * g[i][0];
        gu[1] += xl[i] * g[i][1];
      }
      for (int i = 0; i < nl; i++) {
        double gg = gu[0] * g[i][0] + gu[1] * g[i][1];
        if (kind == ORC_OP_PB)
          rl[i] += (gg + 8 * PI * p->l_b * p->c0 * sinh(u) * phi[i]) * factor;
        else
          rl[i] += (gg + 1 * p->l_b * 4 * PI * (cm - cp) * phi[i]) * factor;
      }
    }
  } else { /* DiffusionOperator, intorder 2 (constructor default, src/diffusion_operator.hh:36) */
    double rs[10];
    memset(rs, 0, sizeof rs);
    rule_of(2, &R);
    for (int q = 0; q < R.n; q++) {
      basis_eval(B, R.xi[q], R.eta[q], phi, js);
      double u = 0.0;
      for (int i = 0; i < nl; i++) u += xl[i] * phi[i];
      phys_grads(G, nl, js, g);
      double gu[2] = {0.0, 0.0}, gP[2] = {0.0, 0.0};
      for (int i = 0; i < nl; i++) {
        gu[0] += xl[i] * g[i][0];
        gu[1] += xl[i] * g[i][1];
        gP[0] += fl0[i] * g[i][0]; /* DiscreteGridFunctionGradient of phi, :103-105 */
        gP[1] += fl0[i] * g[i][1];
      }
      double factor = R.w[q] * G->adet;
      for (int i = 0; i < nl; i++) {
        double gg = gu[0] * g[i][0] + gu[1] * g[i][1];
        double gp = gP[0] * g[i][0] + gP[1] * g[i][1];
        rs[i] += (gg + u * z * gp + 0.0 * u * phi[i]) * factor; /* :109-110 */
      }
    }
    double sc = kind == ORC_OP_DIFF_IMPLICIT_EULER ? dt : 1.0;
    for (int i = 0; i < nl; i++) rl[i] += sc * rs[i];
  }
}

/* boundary faces: element, local face, segment (sorted pair lookup) */
typedef struct {
  int e, f, b;
} bfacet;

static int boundary_facets(const orc_mesh *m, bfacet **out) {
  ekey_t *seg = (ekey_t *)malloc(sizeof(ekey_t) * (m->nb ? m->nb : 1));
  for (int b = 0; b < m->nb; b++) {
    seg[b].key = pair_key(m->bseg[2 * b], m->bseg[2 * b + 1]);
    seg[b].first = b;
  }
  qsort(seg, m->nb, sizeof(ekey_t), cmp_key);
  bfacet *F = (bfacet *)malloc(sizeof(bfacet) * (m->nb ? m->nb : 1));
  int nf = 0;
  char *used = (char *)calloc(m->nb ? m->nb : 1, 1);
  for (int e = 0; e < m->nt; e++)
    for (int f = 0; f < 3; f++) {
      long long k = pair_key(m->tri[3 * e + FACE[f][0]], m->tri[3 * e + FACE[f][1]]);
      int lo = 0, hi = m->nb - 1, b = -1;
      while (lo <= hi) {
        int mid = (lo + hi) >> 1;
        if (seg[mid].key == k) {
          b = seg[mid].first;
          break;
        }
        if (seg[mid].key < k)
          lo = mid + 1;
        else
          hi = mid - 1;
      }
      if (b >= 0 && !used[b]) {
        used[b] = 1;
        F[nf].e = e;
        F[nf].f = f;
        F[nf].b = b;
        nf++;
      }
    }
  free(seg);
  free(used);
  *out = F;
  return nf;
}

static int sb_type(const orc_params *p, int g, int field) {
  const orc_surface *s = p->surf + g;
  return field == 0 ? s->cb : (field == 1 ? s->pb : s->mb);
}

void orc_pk_dirichlet_mask(const orc_mesh *m, const orc_pk *S, const orc_params *p, int field,
                           uint8_t *mask) {
  memset(mask, 0, (size_t)S->nn);
  bfacet *F;
  int nf = boundary_facets(m, &F);
  for (int i = 0; i < nf; i++) {
    if (sb_type(p, m->bgroup[F[i].b], field) != 0) continue;
    const int *en = S->enode + (size_t)S->nl * F[i].e;
    /* the face's nodes: its two vertices and its k-1 face points */
    mask[en[FACE[F[i].f][0]]] = 1;
    mask[en[FACE[F[i].f][1]]] = 1;
    for (int s = 0; s < S->k - 1; s++) mask[en[3 + F[i].f * (S->k - 1) + s]] = 1;
  }
  free(F);
}

/* alpha_boundary of PBOperator / PoissonOperator (coulomb flux where the coulomb field is not
 * Dirichlet), face intorder 3 = 2-point Gauss, the element's basis at the face point */
static void pk_boundary(const orc_mesh *m, const orc_pk *S, const pkbasis *B, const orc_params *p,
                        const double *flux, double *r) {
  static const double V[3][2] = {{0, 0}, {1, 0}, {0, 1}};
  const double gt[2] = {0.5 - 0.5 / sqrt(3.0), 0.5 + 0.5 / sqrt(3.0)};
  bfacet *F;
  int nf = boundary_facets(m, &F);
  double phi[10];
  for (int i = 0; i < nf; i++) {
    const int e = F[i].e, f = F[i].f, b = F[i].b;
    if (sb_type(p, m->bgroup[b], 0) == 0) continue; /* pbB.isDirichlet */
    const int *t = m->tri + 3 * e;
    const double *pa = m->xy + 2 * t[FACE[f][0]], *pb = m->xy + 2 * t[FACE[f][1]];
    const double len = sqrt((pb[0] - pa[0]) * (pb[0] - pa[0]) + (pb[1] - pa[1]) * (pb[1] - pa[1]));
    const double j = flux ? flux[3 * b + 0] : p->surf[m->bgroup[b]].cflux;
    const int *en = S->enode + (size_t)S->nl * e;
    for (int q = 0; q < 2; q++) {
      double factor = 0.5 * len;
      double gy = pa[1] + gt[q] * (pb[1] - pa[1]);
      if (p->cylindrical) factor *= gy * 2 * p->pi;
      double xi = V[FACE[f][0]][0] + gt[q] * (V[FACE[f][1]][0] - V[FACE[f][0]][0]);
      double eta = V[FACE[f][0]][1] + gt[q] * (V[FACE[f][1]][1] - V[FACE[f][0]][1]);
      basis_eval(B, xi, eta, phi, NULL);
      for (int a = 0; a < S->nl; a++) r[en[a]] += j * phi[a] * factor;
    }
  }
  free(F);
}

static void gather_nodes(const orc_pk *S, int e, const double *x, double *xl) {
  const int *en = S->enode + (size_t)S->nl * e;
  for (int a = 0; a < S->nl; a++) xl[a] = x ? x[en[a]] : 0.0;
}

void orc_pk_residual(const orc_mesh *m, const orc_pk *S, const orc_params *p,
                     const orc_operator *op, const double *x, double *r) {
  pkbasis B;
  basis_init(S->k, &B);
  const int nl = S->nl;
  memset(r, 0, sizeof(double) * S->nn);
  double xl[10], f0[10], f1[10], rl[10];
  const double *a0 = op->kind == ORC_OP_POISSON ? op->cp : op->phi;
  const double *a1 = op->kind == ORC_OP_POISSON ? op->cm : NULL;
  for (int e = 0; e < m->nt; e++) {
    pgeo G;
    pgeo_of(m, e, &G);
    gather_nodes(S, e, x, xl);
    gather_nodes(S, e, a0, f0);
    gather_nodes(S, e, a1, f1);
    pk_volume(&B, &G, p, op->kind, op->dt, op->z, xl, f0, f1, 0, rl);
    const int *en = S->enode + (size_t)nl * e;
    for (int a = 0; a < nl; a++) r[en[a]] += rl[a];
  }
  if (op->kind == ORC_OP_DIFF_IMPLICIT_EULER) { /* r -= M(x_old) */
    for (int e = 0; e < m->nt; e++) {
      pgeo G;
      pgeo_of(m, e, &G);
      gather_nodes(S, e, op->x_old, xl);
      pk_volume(&B, &G, p, op->kind, op->dt, op->z, xl, f0, f1, 1, rl);
      const int *en = S->enode + (size_t)nl * e;
      for (int a = 0; a < nl; a++) r[en[a]] -= rl[a];
    }
  }
  if (op->kind == ORC_OP_PB || op->kind == ORC_OP_POISSON) pk_boundary(m, S, &B, p, op->flux, r);
  if (op->mask)
    for (int i = 0; i < S->nn; i++)
      if (op->mask[i]) r[i] = 0.0;
}

static int cmp_i(const void *a, const void *b) {
  int x = *(const int *)a, y = *(const int *)b;
  return (x > y) - (x < y);
}

void orc_pk_csr_pattern(const orc_mesh *m, const orc_pk *S, orc_csr *A) {
  const int nn = S->nn, nl = S->nl;
  int *cnt = (int *)calloc((size_t)nn + 1, sizeof(int));
  for (int e = 0; e < m->nt; e++)
    for (int a = 0; a < nl; a++) cnt[S->enode[(size_t)nl * e + a] + 1] += nl;
  for (int i = 0; i < nn; i++) cnt[i + 1] += cnt[i];
  int *adj = (int *)malloc(sizeof(int) * (size_t)cnt[nn]);
  int *fill = (int *)calloc((size_t)nn, sizeof(int));
  for (int e = 0; e < m->nt; e++)
    for (int a = 0; a < nl; a++) {
      int v = S->enode[(size_t)nl * e + a];
      for (int b = 0; b < nl; b++) adj[cnt[v] + fill[v]++] = S->enode[(size_t)nl * e + b];
    }
  A->n = nn;
  A->rowptr = (int *)malloc(sizeof(int) * ((size_t)nn + 1));
  A->rowptr[0] = 0;
  for (int v = 0; v < nn; v++) {
    int *s = adj + cnt[v];
    qsort(s, fill[v], sizeof(int), cmp_i);
    int u = 0;
    for (int i = 0; i < fill[v]; i++)
      if (i == 0 || s[i] != s[i - 1]) s[u++] = s[i];
    fill[v] = u;
    A->rowptr[v + 1] = A->rowptr[v] + u;
  }
  A->nnz = A->rowptr[nn];
  A->col = (int *)malloc(sizeof(int) * (size_t)A->nnz);
  A->val = (double *)calloc((size_t)A->nnz, sizeof(double));
  for (int v = 0; v < nn; v++) memcpy(A->col + A->rowptr[v], adj + cnt[v], sizeof(int) * fill[v]);
  free(cnt);
  free(adj);
  free(fill);
}

static double *find_entry(orc_csr *A, int i, int j) {
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

/* Jacobian: fd = 1 PDELab NumericalJacobianVolume (eps 1e-7 (1 + |x_j|)); fd = 0 the analytic
 * derivative of pk_volume; constrained rows -> identity */
void orc_pk_jacobian(const orc_mesh *m, const orc_pk *S, const orc_params *p,
                     const orc_operator *op, const double *x, int fd, orc_csr *A) {
  pkbasis B;
  basis_init(S->k, &B);
  const int nl = S->nl;
  const double PI = p->pi;
  memset(A->val, 0, sizeof(double) * A->nnz);
  const double *a0 = op->kind == ORC_OP_POISSON ? op->cp : op->phi;
  const double *a1 = op->kind == ORC_OP_POISSON ? op->cm : NULL;
  double xl[10], u[10], f0[10], f1[10], down[10], up[10], Jl[100];
  double phi[10], js[10][2], g[10][2];
  for (int e = 0; e < m->nt; e++) {
    pgeo G;
    pgeo_of(m, e, &G);
    gather_nodes(S, e, x, xl);
    gather_nodes(S, e, a0, f0);
    gather_nodes(S, e, a1, f1);
    memset(Jl, 0, sizeof Jl);
    if (fd) {
      memcpy(u, xl, sizeof(double) * nl);
      pk_volume(&B, &G, p, op->kind, op->dt, op->z, u, f0, f1, 0, down);
      for (int j = 0; j < nl; j++) {
        double delta = 1e-7 * (1.0 + fabs(u[j]));
        u[j] += delta;
        pk_volume(&B, &G, p, op->kind, op->dt, op->z, u, f0, f1, 0, up);
        for (int i = 0; i < nl; i++) Jl[i * nl + j] = (up[i] - down[i]) / delta;
        u[j] = xl[j];
      }
    } else {
      prule R;
      if (op->kind == ORC_OP_DIFF_IMPLICIT_EULER) {
        rule_of(5, &R);
        for (int q = 0; q < R.n; q++) {
          basis_eval(&B, R.xi[q], R.eta[q], phi, NULL);
          double factor = R.w[q] * G.adet;
          for (int i = 0; i < nl; i++)
            for (int j = 0; j < nl; j++) Jl[i * nl + j] += phi[j] * phi[i] * factor;
        }
      }
      const int k3 = op->kind == ORC_OP_PB || op->kind == ORC_OP_POISSON;
      rule_of(k3 ? 3 : 2, &R);
      const double sc = op->kind == ORC_OP_DIFF_IMPLICIT_EULER ? op->dt : 1.0;
      for (int q = 0; q < R.n; q++) {
        double factor = R.w[q] * G.adet;
        if (k3 && p->cylindrical) factor *= (G.y0 + G.J10 * R.xi[q] + G.J11 * R.eta[q]) * 2 * PI;
        basis_eval(&B, R.xi[q], R.eta[q], phi, js);
        phys_grads(&G, nl, js, g);
        double uq = 0.0, gP[2] = {0.0, 0.0};
        for (int i = 0; i < nl; i++) {
          uq += xl[i] * phi[i];
          gP[0] += f0[i] * g[i][0];
          gP[1] += f0[i] * g[i][1];
        }
        for (int i = 0; i < nl; i++) {
          double gp = gP[0] * g[i][0] + gP[1] * g[i][1];
          for (int j = 0; j < nl; j++) {
            double v = g[j][0] * g[i][0] + g[j][1] * g[i][1];
            if (op->kind == ORC_OP_PB) v += 8 * PI * p->l_b * p->c0 * cosh(uq) * phi[j] * phi[i];
            if (!k3) v += op->z * phi[j] * gp;
            Jl[i * nl + j] += sc * v * factor;
          }
        }
      }
    }
    const int *en = S->enode + (size_t)nl * e;
    for (int i = 0; i < nl; i++)
      for (int j = 0; j < nl; j++) *find_entry(A, en[i], en[j]) += Jl[i * nl + j];
  }
  if (op->mask)
    for (int i = 0; i < A->n; i++)
      if (op->mask[i])
        for (int k = A->rowptr[i]; k < A->rowptr[i + 1]; k++) A->val[k] = (A->col[k] == i) ? 1.0 : 0.0;
}

void orc_pk_initial_state(const orc_mesh *m, const orc_pk *S, const orc_params *p,
                          const double *phi_pb, double *x0) {
  orc_initial_state_nodes(m, p, S->nl, S->enode, S->xy, S->nn, phi_pb, x0);
}

/* calcIonFlux (src/ionFlux.hh:50-91) on P_k: the fields and their gradients at the centre of
 * each boundary face of its element, x = [phi | c+ | c-] over the nodes */
void orc_pk_ion_flux(const orc_mesh *m, const orc_pk *S, const orc_params *p, const double *x,
                     double *ip, double *im) {
  static const double centre[3][2] = {{0.5, 0.0}, {0.0, 0.5}, {0.5, 0.5}};
  pkbasis B;
  basis_init(S->k, &B);
  const int nl = S->nl, nn = S->nn;
  for (int g = 0; g < p->nsurf; g++) ip[g] = im[g] = 0.0;
  bfacet *F;
  int nf = boundary_facets(m, &F);
  /* element order, then face order (the reference's element / intersection loops) */
  double phi[10], js[10][2], gr[10][2];
  for (int i = 0; i < nf; i++) {
    const int e = F[i].e, f = F[i].f, b = F[i].b;
    const int *t = m->tri + 3 * e, *en = S->enode + (size_t)nl * e;
    pgeo G;
    pgeo_of(m, e, &G);
    basis_eval(&B, centre[f][0], centre[f][1], phi, js);
    phys_grads(&G, nl, js, gr);
    double cp = 0, cm = 0, gphi[2] = {0, 0}, gcp[2] = {0, 0}, gcm[2] = {0, 0};
    for (int a = 0; a < nl; a++) {
      cp += phi[a] * x[nn + en[a]];
      cm += phi[a] * x[2 * nn + en[a]];
      for (int d = 0; d < 2; d++) {
        gphi[d] += x[en[a]] * gr[a][d];
        gcp[d] += x[nn + en[a]] * gr[a][d];
        gcm[d] += x[2 * nn + en[a]] * gr[a][d];
      }
    }
    const int ia = FACE[f][0], ic = FACE[f][1], io = 3 - ia - ic;
    const double *pa = m->xy + 2 * t[ia], *pc = m->xy + 2 * t[ic], *po = m->xy + 2 * t[io];
    const double tx = pc[0] - pa[0], ty = pc[1] - pa[1];
    const double len = sqrt(tx * tx + ty * ty);
    double factor = len;
    if (p->cylindrical)
      factor *= 2 * p->pi * (G.y0 + G.J10 * centre[f][0] + G.J11 * centre[f][1]);
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
  free(F);
}
