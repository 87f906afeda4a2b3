// P_k (k = 2, 3) residual + Jacobian assembly on gfx950: the scalar LocalOperators of the
// reference's operator-split driver with its compile-time PDEGREE (src/instationary_pnp_from_pb_md.hh
// :26-28, 125, 245-247): PBOperator (src/pb_operator.hh:46-122), PoissonOperator
// (src/poisson_operator.hh:46-127), DiffusionOperator (src/diffusion_operator.hh:42-112) and
// DiffusionTOperator (src/diffusion_toperator.hh:38-73), each with its own quadrature order
// (PB / Poisson 3, Diffusion 2 -- the default of its constructor, :36 --, DiffusionT 5, the
// `cptop(5)` of src/instationary_pnp_from_pb_md.hh:363).
//
// One launch, owner-computes, no atomics, deterministic (k_pk_row): one thread per owned node
// row walks the elements that contain its node (ascending element order, the order PDELab's
// element loop accumulates them) and computes only its own row of each element's residual and
// matrix, adding the matrix row into its SELL slots in place.  The row's slots stay in L2 while
// they accumulate, so each is written to HBM once, and no element matrix is ever stored.
// Measured at pore_pnp k=3 (profiles/r02/bench_pk_*.log): a first two-pass form (element matrices
// into SoA scratch, then a per-slot gather of their codes) took 506 us (P2) / 1574 us (P3) per
// Poisson assembly, 80 % of it in the latency-bound gather of 28 / 100 scattered values per
// element.  The row walk's price is the element's quadrature data recomputed for each of its
// nodes; the default launches now split it the other way (k_pk_elem_res / k_pk_elem_jac below):
// each element's rows computed once into per-(element, row) records, then the row walk's own
// accumulation reading them (profiles/r02/ab_pk_res2).  The P1 path keeps its fan-walk kernels
// (assemble.hip).
#include <cmath>
#include <vector>

#include <atomic>

#include "kernels.h"
#include "pk.h"

namespace pnp {

// per-device "done" flags (bit = HIP device id) for function attributes, which are set per device:
// a second context on another device in the same process sets them again
static bool dev_flag_test(const std::atomic<uint64_t> &m) {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= 64) return false;
  return (m.load() >> d) & 1;
}
static void dev_flag_set(std::atomic<uint64_t> &m) {
  int d = 0;
  if (hipGetDevice(&d) == hipSuccess && d >= 0 && d < 64) m.fetch_or(uint64_t(1) << d);
}


namespace {

constexpr int kB = 256;
#ifndef PK_PIPE
#define PK_PIPE 1  // A/B knob (build flag): element nodes one incidence ahead
#endif
#ifndef PK_FUSED
#define PK_FUSED 1  // A/B knob (build flag): residual and Jacobian rows in one pass (pk_row_both)
#endif

template <int NL>
struct PkPoint {
  double xi, eta, w;
  double phi[NL];
  double dphi[NL][2];
};
// the quadrature rules of the reference's intorders on the reference triangle (weights sum to
// 1/2; dune-geometry SimplexQuadraturePoints<2>, restated: order 2 the 3-point rule, order 3 the
// Strang-Fix 4-point rule, order 5 Radon's 7-point rule) and the three face centres (ion flux)
template <int NL>
struct PkTab {
  PkPoint<NL> q2[3], q3[4], q5[7], fc[3];
};
__constant__ PkTab<6> c_tab2;
__constant__ PkTab<10> c_tab3;

template <int K>
struct PkK {
  static constexpr int NL = (K + 1) * (K + 2) / 2;
};

template <int K>
__device__ __forceinline__ const PkTab<PkK<K>::NL> &tab() {
  if constexpr (K == 2)
    return c_tab2;
  else
    return c_tab3;
}

struct PkGeo {
  double y0, J10, J11, adet;
  double it00, it01, it10, it11;  // jacobianInverseTransposed
};

__device__ __forceinline__ PkGeo pk_geometry(double2 p0, double2 p1, double2 p2) {
  PkGeo G;
  const double J00 = p1.x - p0.x, J01 = p2.x - p0.x, J10 = p1.y - p0.y, J11 = p2.y - p0.y;
  const double det = J00 * J11 - J01 * J10;
  G.y0 = p0.y;
  G.J10 = J10;
  G.J11 = J11;
  G.adet = fabs(det);
  G.it00 = J11 / det;
  G.it01 = -J10 / det;
  G.it10 = -J01 / det;
  G.it11 = J00 / det;
  return G;
}

// physical gradient of local basis function b at a table point
template <int NL>
__device__ __forceinline__ void grad(const PkGeo &G, const PkPoint<NL> &P, int b, double &g0,
                                     double &g1) {
  g0 = G.it00 * P.dphi[b][0] + G.it01 * P.dphi[b][1];
  g1 = G.it10 * P.dphi[b][0] + G.it11 * P.dphi[b][1];
}

struct PkArgs {
  int kind, cyl, mass;  // mass: the DiffusionTOperator mass M(x) alone (old time level)
  double l_b, c0, pi, dt, z;
};

// PBOperator's sinh / cosh from one exp and one reciprocal (as assemble.hip's P1 element): where
// a point needs both, the exp and the division are shared; the sinh's error is absolute,
// ~eps * e^|u|, against residual terms of at least that size
__device__ __forceinline__ double pb_sinh(double u) {
  const double e = exp(u);
  return 0.5 * (e - 1.0 / e);
}
__device__ __forceinline__ double pb_cosh(double u) {
  const double e = exp(u);
  return 0.5 * (e + 1.0 / e);
}

// quadrature factor of the reference: weight * integrationElement (* 2 PI y when cylindrical)
template <int NL>
__device__ __forceinline__ double factor(const PkGeo &G, const PkPoint<NL> &P, int cyl, double pi) {
  double f = P.w * G.adet;
  if (cyl) f *= (G.y0 + G.J10 * P.xi + G.J11 * P.eta) * 2 * pi;
  return f;
}

// analytic element matrix row a: J[a][b] = d rl[a] / d xl[b]
template <int K>
__device__ void pk_jac_row(const PkGeo &G, const PkArgs &a, int ra, const double *xl,
                           const double *f0, double *Jr) {
  constexpr int NL = PkK<K>::NL;
  const auto &T = tab<K>();
  const double PI = a.pi;
#pragma unroll
  for (int b = 0; b < NL; b++) Jr[b] = 0.0;
  if (a.kind == OP_DIFF_IE) {
    for (int q = 0; q < 7; q++) {
      const auto &P = T.q5[q];
      const double f = P.w * G.adet;
#pragma unroll
      for (int b = 0; b < NL; b++) Jr[b] += P.phi[ra] * P.phi[b] * f;
    }
  }
  if (a.kind == OP_PB || a.kind == OP_POISSON) {
    for (int q = 0; q < 4; q++) {
      const auto &P = T.q3[q];
      const double f = factor(G, P, a.cyl, PI);
      double c = 0.0;
      if (a.kind == OP_PB) {
        double u = 0.0;
#pragma unroll
        for (int i = 0; i < NL; i++) u += xl[i] * P.phi[i];
        c = 8 * PI * a.l_b * a.c0 * pb_cosh(u) * P.phi[ra];
      }
      double ga0, ga1;
      grad(G, P, ra, ga0, ga1);
#pragma unroll
      for (int b = 0; b < NL; b++) {
        double g0, g1;
        grad(G, P, b, g0, g1);
        Jr[b] += (ga0 * g0 + ga1 * g1 + c * P.phi[b]) * f;
      }
    }
  } else {
    const double sc = a.kind == OP_DIFF_IE ? a.dt : 1.0;
    for (int q = 0; q < 3; q++) {
      const auto &P = T.q2[q];
      double gP0 = 0.0, gP1 = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) {
        double g0, g1;
        grad(G, P, i, g0, g1);
        gP0 += f0[i] * g0;
        gP1 += f0[i] * g1;
      }
      double ga0, ga1;
      grad(G, P, ra, ga0, ga1);
      const double f = P.w * G.adet, drift = a.z * (gP0 * ga0 + gP1 * ga1);
#pragma unroll
      for (int b = 0; b < NL; b++) {
        double g0, g1;
        grad(G, P, b, g0, g1);
        Jr[b] += sc * ((ga0 * g0 + ga1 * g1 + P.phi[b] * drift) * f);
      }
    }
  }
}

// residual of local row ra of the element (the reference's element loop restricted to one test
// function; same statements, so the same value as that row of pk_residual)
template <int K>
__device__ double pk_row_residual(const PkGeo &G, const PkArgs &a, int ra, const double *xl,
                                  const double *f0, const double *f1) {
  constexpr int NL = PkK<K>::NL;
  const auto &T = tab<K>();
  const double PI = a.pi;
  double r = 0.0;
  if (a.mass || a.kind == OP_DIFF_IE) {
    for (int q = 0; q < 7; q++) {
      const auto &P = T.q5[q];
      double u = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) u += xl[i] * P.phi[i];
      const double f = P.w * G.adet;
      r += u * P.phi[ra] * f;
    }
    if (a.mass) return r;
  }
  if (a.kind == OP_PB || a.kind == OP_POISSON) {
    for (int q = 0; q < 4; q++) {
      const auto &P = T.q3[q];
      const double f = factor(G, P, a.cyl, PI);
      double u = 0.0, gu0 = 0.0, gu1 = 0.0, cp = 0.0, cm = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) {
        double g0, g1;
        grad(G, P, i, g0, g1);
        u += xl[i] * P.phi[i];
        gu0 += xl[i] * g0;
        gu1 += xl[i] * g1;
        if (a.kind == OP_POISSON) {
          cp += f0[i] * P.phi[i];
          cm += f1[i] * P.phi[i];
        }
      }
      const double s = a.kind == OP_PB ? 8 * PI * a.l_b * a.c0 * pb_sinh(u) : 1 * a.l_b * 4 * PI * (cm - cp);
      double g0, g1;
      grad(G, P, ra, g0, g1);
      r += (gu0 * g0 + gu1 * g1 + s * P.phi[ra]) * f;
    }
  } else {
    const double sc = a.kind == OP_DIFF_IE ? a.dt : 1.0;
    for (int q = 0; q < 3; q++) {
      const auto &P = T.q2[q];
      double u = 0.0, gu0 = 0.0, gu1 = 0.0, gP0 = 0.0, gP1 = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) {
        double g0, g1;
        grad(G, P, i, g0, g1);
        u += xl[i] * P.phi[i];
        gu0 += xl[i] * g0;
        gu1 += xl[i] * g1;
        gP0 += f0[i] * g0;
        gP1 += f0[i] * g1;
      }
      const double f = P.w * G.adet;
      double g0, g1;
      grad(G, P, ra, g0, g1);
      r += sc * ((gu0 * g0 + gu1 * g1 + u * a.z * (gP0 * g0 + gP1 * g1) + 0.0 * u * P.phi[ra]) * f);
    }
  }
  return r;
}

// pk_row_residual and pk_jac_row in one pass (JAC 1): the same statements, with each quadrature
// point's physical basis gradients computed once and shared by the residual row and the Jacobian
// row (the kernel is VALU-bound: profiles/r02/ab_pk_table_select.log).  Not for the mass-only mode.
template <int K>
__device__ void pk_row_both(const PkGeo &G, const PkArgs &a, int ra, const double *xl,
                            const double *f0, const double *f1, double &r, double *Jr) {
  constexpr int NL = PkK<K>::NL;
  const auto &T = tab<K>();
  const double PI = a.pi;
  r = 0.0;
#pragma unroll
  for (int b = 0; b < NL; b++) Jr[b] = 0.0;
  if (a.kind == OP_DIFF_IE) {
#pragma unroll 1
    for (int q = 0; q < 7; q++) {
      const auto &P = T.q5[q];
      double u = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) u += xl[i] * P.phi[i];
      const double f = P.w * G.adet;
      r += u * P.phi[ra] * f;
#pragma unroll
      for (int b = 0; b < NL; b++) Jr[b] += P.phi[ra] * P.phi[b] * f;
    }
  }
  if (a.kind == OP_PB || a.kind == OP_POISSON) {
#pragma unroll 1
    for (int q = 0; q < 4; q++) {
      const auto &P = T.q3[q];
      const double f = factor(G, P, a.cyl, PI);
      double g[NL][2];
      double u = 0.0, gu0 = 0.0, gu1 = 0.0, cp = 0.0, cm = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) {
        grad(G, P, i, g[i][0], g[i][1]);
        u += xl[i] * P.phi[i];
        gu0 += xl[i] * g[i][0];
        gu1 += xl[i] * g[i][1];
        if (a.kind == OP_POISSON) {
          cp += f0[i] * P.phi[i];
          cm += f1[i] * P.phi[i];
        }
      }
      const double s = a.kind == OP_PB ? 8 * PI * a.l_b * a.c0 * pb_sinh(u) : 1 * a.l_b * 4 * PI * (cm - cp);
      const double c = a.kind == OP_PB ? 8 * PI * a.l_b * a.c0 * pb_cosh(u) * P.phi[ra] : 0.0;
      double ga0, ga1;
      grad(G, P, ra, ga0, ga1);
      r += (gu0 * ga0 + gu1 * ga1 + s * P.phi[ra]) * f;
#pragma unroll
      for (int b = 0; b < NL; b++) Jr[b] += (ga0 * g[b][0] + ga1 * g[b][1] + c * P.phi[b]) * f;
    }
  } else {
    const double sc = a.kind == OP_DIFF_IE ? a.dt : 1.0;
#pragma unroll 1
    for (int q = 0; q < 3; q++) {
      const auto &P = T.q2[q];
      double g[NL][2];
      double u = 0.0, gu0 = 0.0, gu1 = 0.0, gP0 = 0.0, gP1 = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) {
        grad(G, P, i, g[i][0], g[i][1]);
        u += xl[i] * P.phi[i];
        gu0 += xl[i] * g[i][0];
        gu1 += xl[i] * g[i][1];
        gP0 += f0[i] * g[i][0];
        gP1 += f0[i] * g[i][1];
      }
      const double f = P.w * G.adet;
      double ga0, ga1;
      grad(G, P, ra, ga0, ga1);
      r += sc * ((gu0 * ga0 + gu1 * ga1 + u * a.z * (gP0 * ga0 + gP1 * ga1) + 0.0 * u * P.phi[ra]) * f);
      const double drift = a.z * (gP0 * ga0 + gP1 * ga1);
#pragma unroll
      for (int b = 0; b < NL; b++)
        Jr[b] += sc * ((ga0 * g[b][0] + ga1 * g[b][1] + P.phi[b] * drift) * f);
    }
  }
}

// One thread per owned node row (SELL lane order), owner-computes like the P1 fan walk: the row
// walks its incident elements (inc: element << 4 | local index of the row), computes its own row
// of each element's residual and matrix (JAC 0 residual only, 1 analytic, 2 PDELab forward
// differences eps 1e-7 (1 + |x_j|)), and adds the matrix row into its slots (islot: the slot of
// each element node in this row, packed bytes).  The slots accumulate in LDS (acc[s][thread], the
// thread's own column: no atomics, no barrier) and are stored once at the end, slot by slot, i.e.
// one coalesced 512-byte line per slot and wave.  The next incidence's code is fetched before
// the current one is computed.  mode 1 (old-time mass): cvec -= M(x) instead.
template <int K, int JAC>
__global__ __launch_bounds__(kB) void k_pk_row(DevLayout L, PkDev D, const double *__restrict__ x,
                                               const double *__restrict__ aux0,
                                               const double *__restrict__ aux1, PkArgs a, int mode,
                                               const double *__restrict__ cvec_in,
                                               const uint8_t *__restrict__ dmask,
                                               double *__restrict__ r, double *__restrict__ cvec_out,
                                               double *__restrict__ vals) {
  constexpr int NL = PkK<K>::NL, NW = (NL + 3) / 4;
  extern __shared__ double acc[];  // [max_slots][kB]
  const int row = row_block(L, blockIdx.x, gridDim.x) * kB + threadIdx.x;
  if (row >= L.n_owned) return;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = L.chunk_off[chunk], len = int(L.rowmeta[row] & 63);
  double *arow = acc + threadIdx.x;
  if constexpr (JAC != 0)
    for (int s = 0; s < len; s++) arow[s * kB] = 0.0;
  const int ne = D.ne, cnt = D.icnt[row];
  const int ib = D.ioff[chunk] + lane;
  const double2 *xy2 = reinterpret_cast<const double2 *>(L.xy);
  double R = 0.0;
  // software pipeline over the incidences: the element nodes of incidence t+1 and the code of
  // t+2 are in flight while t gathers and computes, so an incidence costs one dependent round
  // trip (its node data), not three (code -> nodes -> data)
  int code = cnt > 0 ? D.inc[ib] : 0;
  int code_next = cnt > 1 ? D.inc[ib + kRows] : 0;
  int nd_next[NL];
  if (PK_PIPE) {
#pragma unroll
    for (int i = 0; i < NL; i++) nd_next[i] = cnt > 0 ? D.enode[size_t(i) * ne + (code >> 4)] : 0;
  }
  for (int t = 0; t < cnt; t++) {
    const int p = ib + t * kRows;
    const int e = code >> 4, ra = code & 15;
    int nd[NL];
    if (PK_PIPE) {
#pragma unroll
      for (int i = 0; i < NL; i++) nd[i] = nd_next[i];
      if (t + 1 < cnt) {
#pragma unroll
        for (int i = 0; i < NL; i++) nd_next[i] = D.enode[size_t(i) * ne + (code_next >> 4)];
      }
      code = code_next;
      if (t + 2 < cnt) code_next = D.inc[p + 2 * kRows];
    } else {
#pragma unroll
      for (int i = 0; i < NL; i++) nd[i] = D.enode[size_t(i) * ne + e];
      code = code_next;
      if (t + 2 < cnt) code_next = D.inc[p + 2 * kRows];
    }
    uint32_t sw[NW];
    if constexpr (JAC != 0) {
#pragma unroll
      for (int w = 0; w < NW; w++) sw[w] = D.islot[size_t(p) * NW + w];
    }
    const PkGeo G = pk_geometry(xy2[nd[0]], xy2[nd[1]], xy2[nd[2]]);
    double xl[NL], f0[NL], f1[NL];
#pragma unroll
    for (int i = 0; i < NL; i++) {
      xl[i] = x[nd[i]];
      f0[i] = aux0 ? aux0[nd[i]] : 0.0;
      f1[i] = aux1 ? aux1[nd[i]] : 0.0;
    }
    double Jr[NL];
    double r0;
    if (JAC == 1 && PK_FUSED && !a.mass)
      pk_row_both<K>(G, a, ra, xl, f0, f1, r0, Jr);
    else
      r0 = pk_row_residual<K>(G, a, ra, xl, f0, f1);
    R += r0;
    if constexpr (JAC != 0) {
      if constexpr (JAC == 1) {
        if (!PK_FUSED || a.mass) pk_jac_row<K>(G, a, ra, xl, f0, Jr);
      } else {
#pragma unroll
        for (int j = 0; j < NL; j++) {
          const double xj = xl[j], delta = 1e-7 * (1.0 + fabs(xj));
          xl[j] = xj + delta;
          Jr[j] = (pk_row_residual<K>(G, a, ra, xl, f0, f1) - r0) / delta;
          xl[j] = xj;
        }
      }
#pragma unroll
      for (int b = 0; b < NL; b++) {
        const int s = (sw[b >> 2] >> (8 * (b & 3))) & 0xff;
        arow[s * kB] += Jr[b];
      }
    }
  }
  if constexpr (JAC != 0) {
    double *vrow = vals + size_t(off) + lane;
    for (int s = 0; s < len; s++) __builtin_nontemporal_store(arow[s * kB], vrow + size_t(s) * kRows);
  }
  if (mode == 1) {
    cvec_out[row] -= R;
  } else {
    const double rv = R + cvec_in[row];
    r[row] = dmask[row] != 0 ? 0.0 : rv;
  }
}

// Residual-only launches in two passes (the Jacobian launches keep k_pk_row).  Pass 1, one thread
// per local element: every row of the element residual, pk_row_residual's statements with each
// quadrature point's u, grad u and source computed once for all NL rows instead of once per row
// (the row walk repeats them for each of the element's NL nodes), into eres[ra * ne + e].
// Pass 2 (k_pk_res_gather): each owned row sums its incidences' entries in the row walk's
// ascending element order, so the residual is the row walk's, bit for bit.
template <int K>
__global__ __launch_bounds__(kB) void k_pk_elem_res(PkDev D, const double *__restrict__ xy,
                                                    const double *__restrict__ x,
                                                    const double *__restrict__ aux0,
                                                    const double *__restrict__ aux1, PkArgs a) {
  constexpr int NL = PkK<K>::NL;
  const int ne = D.ne, e = blockIdx.x * kB + threadIdx.x;
  if (e >= ne) return;
  int nd[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) nd[i] = D.enode[size_t(i) * ne + e];
  const double2 *xy2 = reinterpret_cast<const double2 *>(xy);
  const PkGeo G = pk_geometry(xy2[nd[0]], xy2[nd[1]], xy2[nd[2]]);
  double xl[NL], f0[NL], f1[NL], r[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) {
    xl[i] = x[nd[i]];
    f0[i] = aux0 ? aux0[nd[i]] : 0.0;
    f1[i] = aux1 ? aux1[nd[i]] : 0.0;
    r[i] = 0.0;
  }
  const auto &T = tab<K>();
  const double PI = a.pi;
  if (a.mass || a.kind == OP_DIFF_IE) {
#pragma unroll 1
    for (int q = 0; q < 7; q++) {
      const auto &P = T.q5[q];
      double u = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) u += xl[i] * P.phi[i];
      const double f = P.w * G.adet;
#pragma unroll
      for (int ra = 0; ra < NL; ra++) r[ra] += u * P.phi[ra] * f;
    }
  }
  if (a.mass) {
  } else if (a.kind == OP_PB || a.kind == OP_POISSON) {
#pragma unroll 1
    for (int q = 0; q < 4; q++) {
      const auto &P = T.q3[q];
      const double f = factor(G, P, a.cyl, PI);
      double g[NL][2];
      double u = 0.0, gu0 = 0.0, gu1 = 0.0, cp = 0.0, cm = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) {
        grad(G, P, i, g[i][0], g[i][1]);
        u += xl[i] * P.phi[i];
        gu0 += xl[i] * g[i][0];
        gu1 += xl[i] * g[i][1];
        if (a.kind == OP_POISSON) {
          cp += f0[i] * P.phi[i];
          cm += f1[i] * P.phi[i];
        }
      }
      const double s = a.kind == OP_PB ? 8 * PI * a.l_b * a.c0 * pb_sinh(u) : 1 * a.l_b * 4 * PI * (cm - cp);
#pragma unroll
      for (int ra = 0; ra < NL; ra++)
        r[ra] += (gu0 * g[ra][0] + gu1 * g[ra][1] + s * P.phi[ra]) * f;
    }
  } else {
    const double sc = a.kind == OP_DIFF_IE ? a.dt : 1.0;
#pragma unroll 1
    for (int q = 0; q < 3; q++) {
      const auto &P = T.q2[q];
      double g[NL][2];
      double u = 0.0, gu0 = 0.0, gu1 = 0.0, gP0 = 0.0, gP1 = 0.0;
#pragma unroll
      for (int i = 0; i < NL; i++) {
        grad(G, P, i, g[i][0], g[i][1]);
        u += xl[i] * P.phi[i];
        gu0 += xl[i] * g[i][0];
        gu1 += xl[i] * g[i][1];
        gP0 += f0[i] * g[i][0];
        gP1 += f0[i] * g[i][1];
      }
      const double f = P.w * G.adet;
#pragma unroll
      for (int ra = 0; ra < NL; ra++)
        r[ra] += sc * ((gu0 * g[ra][0] + gu1 * g[ra][1] +
                        u * a.z * (gP0 * g[ra][0] + gP1 * g[ra][1]) + 0.0 * u * P.phi[ra]) * f);
    }
  }
#pragma unroll
  for (int ra = 0; ra < NL; ra++) D.eres[size_t(ra) * ne + e] = r[ra];
}

// pass 2: one thread per owned row (SELL lane order, the spatial block order), the incidence codes
// of up to four elements loaded before their entries, the entries summed in incidence order
__global__ __launch_bounds__(kB) void k_pk_res_gather(DevLayout L, PkDev D, int mode,
                                                      const double *__restrict__ cvec_in,
                                                      const uint8_t *__restrict__ dmask,
                                                      double *__restrict__ r,
                                                      double *__restrict__ cvec_out) {
  const int row = row_block(L, blockIdx.x, gridDim.x) * kB + threadIdx.x;
  if (row >= L.n_owned) return;
  const int chunk = row / kRows, lane = row % kRows;
  const int cnt = D.icnt[row], ib = D.ioff[chunk] + lane;
  const double *__restrict__ er = D.eres;
  double R = 0.0;
  for (int t0 = 0; t0 < cnt; t0 += 4) {
    int code[4];
    double v[4];
#pragma unroll
    for (int j = 0; j < 4; j++) code[j] = t0 + j < cnt ? D.inc[ib + (t0 + j) * kRows] : -1;
#pragma unroll
    for (int j = 0; j < 4; j++)
      v[j] = code[j] >= 0 ? er[size_t(code[j] & 15) * D.ne + (code[j] >> 4)] : 0.0;
#pragma unroll
    for (int j = 0; j < 4; j++)
      if (code[j] >= 0) R += v[j];
  }
  if (mode == 1) {
    cvec_out[row] -= R;
  } else {
    const double rv = R + cvec_in[row];
    r[row] = dmask[row] != 0 ? 0.0 : rv;
  }
}

// Analytic Jacobian launches in two passes as well (PNP_PK_JAC2, default on).  Pass 1, one thread per
// local element: each row ra of the element residual and matrix with pk_row_both's statements,
// the quadrature point's basis gradients, u, grad u and source shared by RG rows at a time (RG
// rows of the matrix in registers: 3 at P2, 5 at P3), into one record of W doubles per
// (element, row): the NL matrix entries, then the residual entry, padded to 16 B.  One thread
// per (element, row group) instead was slower (profiles/r02/ab_pk_elem).
// Pass 2 (k_pk_jac_gather): k_pk_row's slot accumulation with each incidence's record read
// instead of computed -- the same sums in the same order, so residual and matrix are k_pk_row's,
// bit for bit.
#ifndef PK_RG2
#define PK_RG2 3  // A/B knob (build flag): element rows per register group of the P2 element pass
#endif
#ifndef PK_RG3
#define PK_RG3 5  // the same at P3
#endif
template <int K>
struct PkRec {
  static constexpr int NL = PkK<K>::NL, W = (NL + 2) & ~1, RG = K == 2 ? PK_RG2 : PK_RG3;
};

// The element pass consumes the element's node values up front: each quadrature point's scalars
// (factor, u or its source terms, grad u, grad of the frozen field) go to LDS first, so that the
// row groups hold only their matrix rows and the basis gradients and two waves fit per SIMD.
// Holding the node values and the rows in registers together (396 VGPRs at P3, one wave per
// SIMD) left the kernel issue-stalled on fp64 dependencies, P2 134 / P3 390 us against 116 / 350
// (profiles/r02/pmc_sq_pk3_r2bb.txt, ab_pk_elem_pre/).
constexpr int kBE = 128;  // threads per workgroup of k_pk_elem_jac (LDS: 32 doubles each)
template <int K>
__global__ __launch_bounds__(kBE) __attribute__((amdgpu_waves_per_eu(2)))
void k_pk_elem_jac(PkDev D, const double *__restrict__ xy, const double *__restrict__ x,
                       const double *__restrict__ aux0, const double *__restrict__ aux1, PkArgs a) {
  constexpr int NL = PkK<K>::NL, W = PkRec<K>::W, RG = PkRec<K>::RG;
  __shared__ double qv[32][kBE];  // PB / Poisson: 4 x 5 at 0..19; DiffusionT: mass 7 x (u, f) at 0..13,
                                  // then the diffusion's 3 x 6 at 14..31
  const int ne = D.ne, e = blockIdx.x * kBE + threadIdx.x;
  if (e >= ne) return;
  double *my = &qv[0][threadIdx.x];
#define QV(i) my[(i) * kBE]
  const auto &T = tab<K>();
  const double PI = a.pi;
  PkGeo G;
  {
    int nd[NL];
#pragma unroll
    for (int i = 0; i < NL; i++) nd[i] = D.enode[size_t(i) * ne + e];
    const double2 *xy2 = reinterpret_cast<const double2 *>(xy);
    G = pk_geometry(xy2[nd[0]], xy2[nd[1]], xy2[nd[2]]);
    double xl[NL], f0[NL], f1[NL];
#pragma unroll
    for (int i = 0; i < NL; i++) {
      xl[i] = x[nd[i]];
      f0[i] = aux0 ? aux0[nd[i]] : 0.0;
      f1[i] = aux1 ? aux1[nd[i]] : 0.0;
    }
    if (a.kind == OP_DIFF_IE) {
#pragma unroll 1
      for (int q = 0; q < 7; q++) {
        const auto &P = T.q5[q];
        double u = 0.0;
#pragma unroll
        for (int i = 0; i < NL; i++) u += xl[i] * P.phi[i];
        QV(2 * q) = u;
        QV(2 * q + 1) = P.w * G.adet;
      }
    }
    if (a.kind == OP_PB || a.kind == OP_POISSON) {
#pragma unroll 1
      for (int q = 0; q < 4; q++) {
        const auto &P = T.q3[q];
        double u = 0.0, gu0 = 0.0, gu1 = 0.0, cp = 0.0, cm = 0.0;
#pragma unroll
        for (int i = 0; i < NL; i++) {
          double g0, g1;
          grad(G, P, i, g0, g1);
          u += xl[i] * P.phi[i];
          gu0 += xl[i] * g0;
          gu1 += xl[i] * g1;
          if (a.kind == OP_POISSON) {
            cp += f0[i] * P.phi[i];
            cm += f1[i] * P.phi[i];
          }
        }
        QV(5 * q) = factor(G, P, a.cyl, PI);
        QV(1 + 5 * q) = gu0;
        QV(2 + 5 * q) = gu1;
        QV(3 + 5 * q) = a.kind == OP_PB ? 8 * PI * a.l_b * a.c0 * pb_sinh(u) : 1 * a.l_b * 4 * PI * (cm - cp);
        QV(4 + 5 * q) = a.kind == OP_PB ? 8 * PI * a.l_b * a.c0 * pb_cosh(u) : 0.0;
      }
    } else {
#pragma unroll 1
      for (int q = 0; q < 3; q++) {
        const auto &P = T.q2[q];
        double u = 0.0, gu0 = 0.0, gu1 = 0.0, gP0 = 0.0, gP1 = 0.0;
#pragma unroll
        for (int i = 0; i < NL; i++) {
          double g0, g1;
          grad(G, P, i, g0, g1);
          u += xl[i] * P.phi[i];
          gu0 += xl[i] * g0;
          gu1 += xl[i] * g1;
          gP0 += f0[i] * g0;
          gP1 += f0[i] * g1;
        }
        QV(14 + 6 * q) = P.w * G.adet;
        QV(15 + 6 * q) = gu0;
        QV(16 + 6 * q) = gu1;
        QV(17 + 6 * q) = u;
        QV(18 + 6 * q) = gP0;
        QV(19 + 6 * q) = gP1;
      }
    }
  }
  double *rec0 = D.ejac + size_t(e) * NL * W;
#pragma unroll 1
  for (int ra0 = 0; ra0 < NL; ra0 += RG) {
    double r[RG], Jr[RG][NL];
#pragma unroll
    for (int j = 0; j < RG; j++) {
      r[j] = 0.0;
#pragma unroll
      for (int b = 0; b < NL; b++) Jr[j][b] = 0.0;
    }
    if (a.kind == OP_DIFF_IE) {
#pragma unroll 1
      for (int q = 0; q < 7; q++) {
        const auto &P = T.q5[q];
        const double u = QV(2 * q), f = QV(2 * q + 1);
#pragma unroll
        for (int j = 0; j < RG; j++) {
          const int ra = ra0 + j < NL ? ra0 + j : NL - 1;
          r[j] += u * P.phi[ra] * f;
#pragma unroll
          for (int b = 0; b < NL; b++) Jr[j][b] += P.phi[ra] * P.phi[b] * f;
        }
      }
    }
    if (a.kind == OP_PB || a.kind == OP_POISSON) {
#pragma unroll 1
      for (int q = 0; q < 4; q++) {
        const auto &P = T.q3[q];
        const double f = QV(5 * q), gu0 = QV(1 + 5 * q), gu1 = QV(2 + 5 * q);
        const double s = QV(3 + 5 * q), cb = QV(4 + 5 * q);
        double g[NL][2];
#pragma unroll
        for (int i = 0; i < NL; i++) grad(G, P, i, g[i][0], g[i][1]);
#pragma unroll
        for (int j = 0; j < RG; j++) {
          const int ra = ra0 + j < NL ? ra0 + j : NL - 1;
          const double c = a.kind == OP_PB ? cb * P.phi[ra] : 0.0;
          double ga0, ga1;
          grad(G, P, ra, ga0, ga1);
          r[j] += (gu0 * ga0 + gu1 * ga1 + s * P.phi[ra]) * f;
#pragma unroll
          for (int b = 0; b < NL; b++) Jr[j][b] += (ga0 * g[b][0] + ga1 * g[b][1] + c * P.phi[b]) * f;
        }
      }
    } else {
      const double sc = a.kind == OP_DIFF_IE ? a.dt : 1.0;
#pragma unroll 1
      for (int q = 0; q < 3; q++) {
        const auto &P = T.q2[q];
        const double f = QV(14 + 6 * q), gu0 = QV(15 + 6 * q), gu1 = QV(16 + 6 * q);
        const double u = QV(17 + 6 * q), gP0 = QV(18 + 6 * q), gP1 = QV(19 + 6 * q);
        double g[NL][2];
#pragma unroll
        for (int i = 0; i < NL; i++) grad(G, P, i, g[i][0], g[i][1]);
#pragma unroll
        for (int j = 0; j < RG; j++) {
          const int ra = ra0 + j < NL ? ra0 + j : NL - 1;
          double ga0, ga1;
          grad(G, P, ra, ga0, ga1);
          r[j] += sc * ((gu0 * ga0 + gu1 * ga1 + u * a.z * (gP0 * ga0 + gP1 * ga1) + 0.0 * u * P.phi[ra]) * f);
          const double drift = a.z * (gP0 * ga0 + gP1 * ga1);
#pragma unroll
          for (int b = 0; b < NL; b++)
            Jr[j][b] += sc * ((ga0 * g[b][0] + ga1 * g[b][1] + P.phi[b] * drift) * f);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < RG; j++) {
      if (ra0 + j >= NL) break;
      double2 *rec = reinterpret_cast<double2 *>(rec0 + size_t(ra0 + j) * W);
      double v[W];
#pragma unroll
      for (int b = 0; b < NL; b++) v[b] = Jr[j][b];
      v[NL] = r[j];
#pragma unroll
      for (int b = NL + 1; b < W; b++) v[b] = 0.0;
#pragma unroll
      for (int w = 0; w < W / 2; w++) rec[w] = make_double2(v[2 * w], v[2 * w + 1]);
    }
  }
#undef QV
}

// pass 2: one thread per owned row, k_pk_row's slot accumulation in LDS with each incidence's
// record (and slot codes) loaded instead of computed; the code of the next incidence is in flight
// while the current record is added
template <int K>
__global__ __launch_bounds__(kB) void k_pk_jac_gather(DevLayout L, PkDev D,
                                                      const double *__restrict__ cvec_in,
                                                      const uint8_t *__restrict__ dmask,
                                                      double *__restrict__ r,
                                                      double *__restrict__ vals) {
  constexpr int NL = PkK<K>::NL, NW = (NL + 3) / 4, W = PkRec<K>::W;
  extern __shared__ double acc[];  // [max_slots][kB]
  const int row = row_block(L, blockIdx.x, gridDim.x) * kB + threadIdx.x;
  if (row >= L.n_owned) return;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = L.chunk_off[chunk], len = int(L.rowmeta[row] & 63);
  double *arow = acc + threadIdx.x;
  for (int s = 0; s < len; s++) arow[s * kB] = 0.0;
  const int cnt = D.icnt[row], ib = D.ioff[chunk] + lane;
  double R = 0.0;
  int code = cnt > 0 ? D.inc[ib] : 0;
  for (int t = 0; t < cnt; t++) {
    const int p = ib + t * kRows;
    const int e = code >> 4, ra = code & 15;
    if (t + 1 < cnt) code = D.inc[p + kRows];
    uint32_t sw[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) sw[w] = D.islot[size_t(p) * NW + w];
    const double2 *rec = reinterpret_cast<const double2 *>(D.ejac + (size_t(e) * NL + ra) * W);
    double v[W];
#pragma unroll
    for (int w = 0; w < W / 2; w++) {
      const double2 q = rec[w];
      v[2 * w] = q.x;
      v[2 * w + 1] = q.y;
    }
    R += v[NL];
#pragma unroll
    for (int b = 0; b < NL; b++) {
      const int s = (sw[b >> 2] >> (8 * (b & 3))) & 0xff;
      arow[s * kB] += v[b];
    }
  }
  double *vrow = vals + size_t(off) + lane;
  for (int s = 0; s < len; s++) __builtin_nontemporal_store(arow[s * kB], vrow + size_t(s) * kRows);
  const double rv = R + cvec_in[row];
  r[row] = dmask[row] != 0 ? 0.0 : rv;
}

// calcIonFlux (src/ionFlux.hh:50-91) on P_k: one thread per boundary segment of this rank;
// seg = {element (local), local face, group}; the three fields at the face centre from the
// element's nodes.  out[2s] / out[2s+1]: ip / im contributions (summed on the host in segment order)
template <int K>
__global__ __launch_bounds__(kB) void k_pk_ion_flux(int ns, const int4 *__restrict__ seg, int ne,
                                                    const int *__restrict__ enode,
                                                    const double *__restrict__ xy,
                                                    const double *__restrict__ x, int cyl,
                                                    double pi, double *__restrict__ out) {
  constexpr int NL = PkK<K>::NL;
  const int s = blockIdx.x * kB + threadIdx.x;
  if (s >= ns) return;
  const int4 sg = seg[s];
  const int e = sg.x, f = sg.y;
  int nd[NL];
#pragma unroll
  for (int i = 0; i < NL; i++) nd[i] = enode[size_t(i) * ne + e];
  const double2 *xy2 = reinterpret_cast<const double2 *>(xy);
  const double2 p0 = xy2[nd[0]], p1 = xy2[nd[1]], p2 = xy2[nd[2]];
  const PkGeo G = pk_geometry(p0, p1, p2);
  const auto &P = tab<K>().fc[f];
  double phi = 0, cp = 0, cm = 0, gph[2] = {0, 0}, gcp[2] = {0, 0}, gcm[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < NL; i++) {
    double g0, g1;
    grad(G, P, i, g0, g1);
    const double u0 = x[3 * size_t(nd[i])], u1 = x[3 * size_t(nd[i]) + 1], u2 = x[3 * size_t(nd[i]) + 2];
    phi += u0 * P.phi[i];
    cp += u1 * P.phi[i];
    cm += u2 * P.phi[i];
    gph[0] += u0 * g0;
    gph[1] += u0 * g1;
    gcp[0] += u1 * g0;
    gcp[1] += u1 * g1;
    gcm[0] += u2 * g0;
    gcm[1] += u2 * g1;
  }
  (void)phi;
  // face f of the reference triangle: (0,1), (0,2), (1,2); outer normal of the element there
  const int fa[3] = {0, 0, 1}, fb[3] = {1, 2, 2}, fo[3] = {2, 1, 0};
  const double2 V[3] = {p0, p1, p2};
  const double2 A = V[fa[f]], B = V[fb[f]], O = V[fo[f]];
  const double tx = B.x - A.x, ty = B.y - A.y;
  const double len = sqrt(tx * tx + ty * ty);
  double nx = ty / len, ny = -tx / len;
  if (nx * (O.x - A.x) + ny * (O.y - A.y) > 0) {
    nx = -nx;
    ny = -ny;
  }
  double factor = len;
  if (cyl) factor *= 2 * pi * (G.y0 + G.J10 * P.xi + G.J11 * P.eta);
  const double gC0 = -factor * gcp[0], gC1 = -factor * gcp[1];
  const double gM0 = -factor * gcm[0], gM1 = -factor * gcm[1];
  double gp0 = factor * gph[0] * cp, gp1 = factor * gph[1] * cp;
  out[2 * size_t(s)] = (gC0 + gp0) * nx + (gC1 + gp1) * ny;
  gp0 *= cm / cp;
  gp1 *= cm / cp;
  out[2 * size_t(s) + 1] = (gM0 - gp0) * nx + (gM1 - gp1) * ny;
}

template <int NL>
void fill_tab(int k, PkTab<NL> &T) {
  const double s15 = std::sqrt(15.0);
  const double a1 = (6.0 - s15) / 21.0, a2 = (6.0 + s15) / 21.0;
  const double w1 = (155.0 - s15) / 2400.0, w2 = (155.0 + s15) / 2400.0;
  const double q2[3][3] = {{4.0 / 6.0, 1.0 / 6.0, 0.5 / 3.0},
                           {1.0 / 6.0, 4.0 / 6.0, 0.5 / 3.0},
                           {1.0 / 6.0, 1.0 / 6.0, 0.5 / 3.0}};
  const double q3[4][3] = {{10.0 / 30.0, 10.0 / 30.0, 0.5 * -27.0 / 48.0},
                           {18.0 / 30.0, 6.0 / 30.0, 0.5 * 25.0 / 48.0},
                           {6.0 / 30.0, 18.0 / 30.0, 0.5 * 25.0 / 48.0},
                           {6.0 / 30.0, 6.0 / 30.0, 0.5 * 25.0 / 48.0}};
  const double q5[7][3] = {{1.0 / 3.0, 1.0 / 3.0, 9.0 / 80.0},
                           {a1, a1, w1}, {1.0 - 2.0 * a1, a1, w1}, {a1, 1.0 - 2.0 * a1, w1},
                           {a2, a2, w2}, {1.0 - 2.0 * a2, a2, w2}, {a2, 1.0 - 2.0 * a2, w2}};
  const double fc[3][3] = {{0.5, 0.0, 0.0}, {0.0, 0.5, 0.0}, {0.5, 0.5, 0.0}};
  auto set = [&](PkPoint<NL> &P, const double *r) {
    P.xi = r[0];
    P.eta = r[1];
    P.w = r[2];
    double phi[NL], dphi[2 * NL];
    pk_basis(k, P.xi, P.eta, phi, dphi);
    for (int i = 0; i < NL; i++) {
      P.phi[i] = phi[i];
      P.dphi[i][0] = dphi[2 * i];
      P.dphi[i][1] = dphi[2 * i + 1];
    }
  };
  for (int q = 0; q < 3; q++) set(T.q2[q], q2[q]);
  for (int q = 0; q < 4; q++) set(T.q3[q], q3[q]);
  for (int q = 0; q < 7; q++) set(T.q5[q], q5[q]);
  for (int q = 0; q < 3; q++) set(T.fc[q], fc[q]);
}

template <int K>
hipError_t upload_tab(hipStream_t s) {
  static PkTab<PkK<K>::NL> T;  // the same for every context of degree K
  static bool filled = false;
  if (!filled) {
    fill_tab<PkK<K>::NL>(K, T);
    filled = true;
  }
  if constexpr (K == 2)
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_tab2), &T, sizeof T, 0, hipMemcpyHostToDevice, s);
  else
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_tab3), &T, sizeof T, 0, hipMemcpyHostToDevice, s);
}

// PNP_PK_RES2=0 / PNP_PK_JAC2=0 send residual-only / analytic Jacobian launches through the row
// walk (A/B knobs)
bool env_on(const char *name) {
  const char *v = getenv(name);
  return !(v && v[0] == '0');
}
bool res_two_pass() {
  static const bool on = env_on("PNP_PK_RES2");
  return on;
}
bool jac_two_pass() {
  static const bool on = env_on("PNP_PK_JAC2");
  return on;
}

template <int K>
hipError_t jac_launch2(const DevLayout &L, const PkDev &D, const double *x, const double *aux0,
                       const double *aux1, const PkArgs &a, const double *cvec_in,
                       const uint8_t *dmask, double *r, double *vals, hipStream_t s) {
  const size_t lds = size_t(L.max_slots) * kB * sizeof(double);
  static std::atomic<uint64_t> attr{0};  // per device: the attribute is a per-device setting
  if (!dev_flag_test(attr)) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pk_jac_gather<K>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    dev_flag_set(attr);
  }
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_pk_elem_jac<K>, dim3((D.ne + kBE - 1) / kBE), dim3(kBE), 0, s, D, L.xy, x,
                     aux0, aux1, a);
  if (D.n_short > 0) {
    DevLayout Ls = L, Ll = L;
    Ls.blkmap = D.blk_short;
    Ls.blkcount = D.n_short;
    Ll.blkmap = D.blk_long;
    Ll.blkcount = D.n_long;
    const size_t lds_s = size_t(D.short_len) * kB * sizeof(double);
    hipLaunchKernelGGL(k_pk_jac_gather<K>, dim3(D.n_short), dim3(kB), lds_s, s, Ls, D, cvec_in,
                       dmask, r, vals);
    if (D.n_long > 0)
      hipLaunchKernelGGL(k_pk_jac_gather<K>, dim3(D.n_long), dim3(kB), lds, s, Ll, D, cvec_in,
                         dmask, r, vals);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_pk_jac_gather<K>, dim3((L.n_owned + kB - 1) / kB), dim3(kB), lds, s, L, D,
                     cvec_in, dmask, r, vals);
  return hipGetLastError();
}

template <int K, int JAC>
hipError_t row_launch1(const DevLayout &L, const PkDev &D, const double *x, const double *aux0,
                       const double *aux1, const PkArgs &a, int mode, const double *cvec_in,
                       const uint8_t *dmask, double *r, double *cvec_out, double *vals,
                       hipStream_t s) {
  const size_t lds = JAC ? size_t(L.max_slots) * kB * sizeof(double) : 0;
  // up to 160 KB of LDS per workgroup on gfx950 (P3: 55 slots); set once per device
  static std::atomic<uint64_t> attr{0};
  if (JAC && !dev_flag_test(attr)) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void *>(&k_pk_row<K, JAC>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return e;
    dev_flag_set(attr);
  }
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const int nwg = (L.n_owned + kB - 1) / kB;
  hipLaunchKernelGGL((k_pk_row<K, JAC>), dim3(nwg), dim3(kB), lds, s, L, D, x, aux0, aux1, a,
                     mode, cvec_in, dmask, r, cvec_out, vals);
  return hipGetLastError();
}

template <int K>
hipError_t row_launch(const DevLayout &L, const PkDev &D, const double *x, const double *aux0,
                      const double *aux1, const PkArgs &a, int jac, int mode, const double *cvec_in,
                      const uint8_t *dmask, double *r, double *cvec_out, double *vals,
                      hipStream_t s) {
  if (jac == 0 && D.eres && res_two_pass()) {
    hipLaunchKernelGGL(k_pk_elem_res<K>, dim3((D.ne + kB - 1) / kB), dim3(kB), 0, s, D, L.xy, x,
                       aux0, aux1, a);
    hipLaunchKernelGGL(k_pk_res_gather, dim3((L.n_owned + kB - 1) / kB), dim3(kB), 0, s, L, D,
                       mode, cvec_in, dmask, r, cvec_out);
    return hipGetLastError();
  }
  if (jac == 0)
    return row_launch1<K, 0>(L, D, x, aux0, aux1, a, mode, cvec_in, dmask, r, cvec_out, vals, s);
  if (jac == 1 && mode == 0 && !a.mass && D.ejac && jac_two_pass())
    return jac_launch2<K>(L, D, x, aux0, aux1, a, cvec_in, dmask, r, vals, s);
  if (jac == 1)
    return row_launch1<K, 1>(L, D, x, aux0, aux1, a, mode, cvec_in, dmask, r, cvec_out, vals, s);
  return row_launch1<K, 2>(L, D, x, aux0, aux1, a, mode, cvec_in, dmask, r, cvec_out, vals, s);
}

}  // namespace

hipError_t pk_upload_tables(int k, hipStream_t s) {
  if (k == 2) return upload_tab<2>(s);
  if (k == 3) return upload_tab<3>(s);
  return hipErrorInvalidValue;
}

hipError_t launch_pk_assemble(const DevLayout &L, const AsmArgs &aa, const PkDev &P, int jac,
                              hipStream_t s) {
  if (P.k != 2 && P.k != 3) return hipErrorInvalidValue;
  if (L.n_owned == 0) return hipSuccess;
  const bool diff = aa.kind == OP_DIFF || aa.kind == OP_DIFF_IE;
  const double *f0 = (diff || aa.kind == OP_POISSON) ? aa.aux0 : nullptr;
  const double *f1 = aa.kind == OP_POISSON ? aa.aux1 : nullptr;
  PkArgs a{aa.kind, aa.cylindrical, 0, aa.l_b, aa.c0, aa.pi, aa.dt, aa.z};
  return P.k == 2 ? row_launch<2>(L, P, aa.x, f0, f1, a, jac, 0, aa.cvec, aa.dmask, aa.r, nullptr,
                                  aa.vals, s)
                  : row_launch<3>(L, P, aa.x, f0, f1, a, jac, 0, aa.cvec, aa.dmask, aa.r, nullptr,
                                  aa.vals, s);
}

hipError_t launch_pk_mass_apply(const DevLayout &L, const PkDev &P, const double *x_old,
                                double *cvec, hipStream_t s) {
  if (L.n_owned == 0) return hipSuccess;
  PkArgs a{OP_DIFF_IE, 0, 1, 0, 0, 0, 0, 0};
  return P.k == 2 ? row_launch<2>(L, P, x_old, nullptr, nullptr, a, 0, 1, nullptr, nullptr,
                                  nullptr, cvec, nullptr, s)
                  : row_launch<3>(L, P, x_old, nullptr, nullptr, a, 0, 1, nullptr, nullptr,
                                  nullptr, cvec, nullptr, s);
}

hipError_t launch_pk_ion_flux(const DevLayout &L, const PkDev &P, int ns, const int4 *seg,
                              const double *x, int cyl, double pi, double *out, hipStream_t s) {
  if (ns <= 0) return hipSuccess;
  const dim3 g((ns + kB - 1) / kB), b(kB);
  if (P.k == 2)
    hipLaunchKernelGGL(k_pk_ion_flux<2>, g, b, 0, s, ns, seg, P.ne, P.enode, L.xy, x, cyl, pi, out);
  else if (P.k == 3)
    hipLaunchKernelGGL(k_pk_ion_flux<3>, g, b, 0, s, ns, seg, P.ne, P.enode, L.xy, x, cyl, pi, out);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// Store-pattern probe (pnp_probe_slot_stores): thread t writes every SELL slot of row order[t]
// (order null: row t), one 8-B store per slot, as the gather pass stores a finished row.  With the
// rows in SELL order a wave's stores of one slot fill 512 contiguous bytes; in a tile order they
// land wherever the tile's rows sit in the colour-major SELL.
__global__ void __launch_bounds__(256) k_slot_store_probe(int n, const int *order, DevLayout L,
                                                          double *val) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= n) return;
  const int r = order ? order[t] : t;
  const int len = int(L.rowmeta[r] & 63);
  double *p = val + L.chunk_off[r >> 6] + (r & 63);
  for (int sl = 0; sl < len; sl++) p[64 * sl] = double(t) + sl;
}

hipError_t launch_slot_store_probe(const DevLayout &L, const int *order, double *val,
                                   hipStream_t s) {
  if (L.n_owned == 0) return hipSuccess;
  hipLaunchKernelGGL(k_slot_store_probe, dim3((L.n_owned + 255) / 256), dim3(256), 0, s,
                     L.n_owned, order, L, val);
  return hipGetLastError();
}

}  // namespace pnp
