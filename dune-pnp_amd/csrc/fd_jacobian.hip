// Reference-faithful forward-difference Jacobian on the GPU (PNP_JAC_FD).
//
// The reference never differentiates analytically: every LocalOperator inherits PDELab's
// NumericalJacobianVolume (src/pnp_operator.hh:24-27, src/pb_operator.hh:24-27,
// src/diffusion_operator.hh:20-23, src/pnp_toperator.hh:12-13, src/diffusion_toperator.hh:16-17,
// src/poisson_operator.hh:24-27): per element, the local residual at the local DOF vector u and at
// u + delta_j e_j with delta_j = 1e-7 (1 + |u_j|), column j of the local matrix being
// (r(u + delta_j e_j) - r(u)) / delta_j; the local matrices are accumulated into the BCRS matrix
// element by element.  This file restates that on the GPU:
//
//   k_fd_element  one thread per element: the element geometry and the volume residual of the
//                 operator at the quadrature points of the reference's rules, evaluated 1 + 3 NF
//                 times, exactly in the reference's operand order (this file is compiled with
//                 -ffp-contract=off, so no multiply-add is fused), columns written to a per-element
//                 scratch [ne][3NF][3NF];
//   k_fd_gather   one thread per owned row: every block (row, slot) of the SELL matrix sums the
//                 element matrices that touch it in ascending element order (BCRSMatrix
//                 accumulation order), the block pattern's values stored as they are (kPat*FD).
//
// One-step operators (implicit Euler: PnpOperator + PnpTOperator, DiffusionOperator +
// DiffusionTOperator under OneStepGridOperator, src/instationary_pnp_from_pb.hh:324): each local
// operator has its own NumericalJacobianVolume, so per element the spatial operator's matrix
// (weight dt: dt ((r_s(u + delta e_j) - r_s(u)) / delta)) and the temporal operator's are two
// matrices, added into the BCRS matrix one after the other (the oracle's orc_op_jacobian).
//
// The analytic Jacobian (assemble.hip) stays the default; this mode exists for bit-level parity
// with the reference's FD Jacobian.  Polynomial operators (PNP, PnpT, Poisson, Diffusion) give
// the oracle's FD matrix to the last bits; PB goes through sinh, whose device and host libm results
// can differ by an ulp (amplified by 1/delta ~ 1e7).
#include "kernels.h"

namespace pnp {

namespace {

constexpr int kB = 256;

// dune-geometry SimplexQuadraturePoints<2> as restated by the oracle: order 2 -> 3 points,
// order 3 -> Strang-Fix 4 points with centroid weight -27/96
struct QRule {
  int n;
  double xi[4], eta[4], w[4];
};
__device__ __forceinline__ QRule rule2() {
  return {3,
          {4.0 / 6.0, 1.0 / 6.0, 1.0 / 6.0, 0},
          {1.0 / 6.0, 4.0 / 6.0, 1.0 / 6.0, 0},
          {0.5 / 3.0, 0.5 / 3.0, 0.5 / 3.0, 0}};
}
__device__ __forceinline__ QRule rule3() {
  return {4,
          {10.0 / 30.0, 18.0 / 30.0, 6.0 / 30.0, 6.0 / 30.0},
          {10.0 / 30.0, 6.0 / 30.0, 18.0 / 30.0, 6.0 / 30.0},
          {0.5 * -27.0 / 48.0, 0.5 * 25.0 / 48.0, 0.5 * 25.0 / 48.0, 0.5 * 25.0 / 48.0}};
}

// affine element map x = p0 + xi (p1 - p0) + eta (p2 - p0), vertices in the mesh's order
struct ElGeo {
  double y0, J10, J11, adet;
  double g[3][2];  // physical P1 gradients: jacobianInverseTransposed * reference gradient
};
__device__ __forceinline__ ElGeo element_geometry(const double *p0, const double *p1,
                                                  const double *p2) {
  ElGeo G;
  const double J00 = p1[0] - p0[0], J01 = p2[0] - p0[0];
  G.J10 = p1[1] - p0[1];
  G.J11 = p2[1] - p0[1];
  G.y0 = p0[1];
  const double det = J00 * G.J11 - J01 * G.J10;
  G.adet = fabs(det);
  const double it00 = G.J11 / det, it01 = -G.J10 / det;
  const double it10 = -J01 / det, it11 = J00 / det;
  const double gh[3][2] = {{-1.0, -1.0}, {1.0, 0.0}, {0.0, 1.0}};
#pragma unroll
  for (int i = 0; i < 3; i++) {
    G.g[i][0] = it00 * gh[i][0] + it01 * gh[i][1];
    G.g[i][1] = it10 * gh[i][0] + it11 * gh[i][1];
  }
  return G;
}

struct FdArgs {
  int kind, cylindrical;
  double l_b, c0, tau, pi, dt, z;
};

__device__ __forceinline__ double cyl_factor(const ElGeo &G, const QRule &R, int q,
                                             const FdArgs &a, double factor) {
  if (a.cylindrical) factor *= (G.y0 + G.J10 * R.xi[q] + G.J11 * R.eta[q]) * 2 * a.pi;
  return factor;
}

// PnpOperator::alpha_volume (src/pnp_operator.hh:46-195); rl accumulates (+=)
__device__ void lop_pnp(const ElGeo &G, const FdArgs &a, const double *xl, double *rl) {
  const QRule R = rule3();
  for (int q = 0; q < R.n; q++) {
    const double factor = cyl_factor(G, R, q, a, R.w[q] * G.adet);
    const double psi[3] = {1.0 - R.xi[q] - R.eta[q], R.xi[q], R.eta[q]};
    double u_phi = 0, u_cp = 0, u_cm = 0;
    for (int i = 0; i < 3; i++) u_phi += xl[i] * psi[i];
    for (int i = 0; i < 3; i++) u_cp += xl[3 + i] * psi[i];
    for (int i = 0; i < 3; i++) u_cm += xl[6 + i] * psi[i];
    (void)u_phi;
    double gphi[2] = {0, 0}, gcp[2] = {0, 0}, gcm[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      gphi[0] += xl[i] * G.g[i][0];
      gphi[1] += xl[i] * G.g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      gcp[0] += xl[3 + i] * G.g[i][0];
      gcp[1] += xl[3 + i] * G.g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      gcm[0] += xl[6 + i] * G.g[i][0];
      gcm[1] += xl[6 + i] * G.g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      const double gg = gphi[0] * G.g[i][0] + gphi[1] * G.g[i][1];
      rl[i] += (gg + 4 * a.pi * a.l_b * (u_cp - u_cm) * psi[i]) * factor;
    }
    for (int i = 0; i < 3; i++) {
      const double gc = gcp[0] * G.g[i][0] + gcp[1] * G.g[i][1];
      const double gp = gphi[0] * G.g[i][0] + gphi[1] * G.g[i][1];
      rl[3 + i] += (gc - u_cp * gp) * factor;
    }
    for (int i = 0; i < 3; i++) {
      const double gc = gcm[0] * G.g[i][0] + gcm[1] * G.g[i][1];
      const double gp = gphi[0] * G.g[i][0] + gphi[1] * G.g[i][1];
      rl[6 + i] += (gc + u_cm * gp) * factor;
    }
  }
}

// PnpTOperator::alpha_volume (src/pnp_toperator.hh:31-101, order 2, quirk Q2: the c- mass lands
// in the c+ rows)
__device__ void lop_pnpt(const ElGeo &G, const FdArgs &a, const double *xl, double *rl) {
  const QRule R = rule2();
  for (int q = 0; q < R.n; q++) {
    const double psi[3] = {1.0 - R.xi[q] - R.eta[q], R.xi[q], R.eta[q]};
    double u_cp = 0, u_cm = 0;
    for (int i = 0; i < 3; i++) u_cp += xl[3 + i] * psi[i];
    for (int i = 0; i < 3; i++) u_cm += xl[6 + i] * psi[i];
    const double factor = cyl_factor(G, R, q, a, R.w[q] * G.adet);
    for (int i = 0; i < 3; i++) rl[3 + i] += a.tau * u_cp * psi[i] * factor;
    for (int i = 0; i < 3; i++) rl[3 + i] += a.tau * u_cm * psi[i] * factor;
  }
}

// PBOperator::alpha_volume (src/pb_operator.hh:46-122)
__device__ void lop_pb(const ElGeo &G, const FdArgs &a, const double *xl, double *rl) {
  const QRule R = rule3();
  for (int q = 0; q < R.n; q++) {
    const double factor = cyl_factor(G, R, q, a, R.w[q] * G.adet);
    const double psi[3] = {1.0 - R.xi[q] - R.eta[q], R.xi[q], R.eta[q]};
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    double gu[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      gu[0] += xl[i] * G.g[i][0];
      gu[1] += xl[i] * G.g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      const double gg = gu[0] * G.g[i][0] + gu[1] * G.g[i][1];
      rl[i] += (gg + 8 * a.pi * a.l_b * a.c0 * sinh(u) * psi[i]) * factor;
    }
  }
}

// DiffusionOperator::alpha_volume (src/diffusion_operator.hh:42-112; order 2, no cylindrical
// weight: quirk Q8)
__device__ void lop_diff(const ElGeo &G, const FdArgs &a, const double *phil, const double *xl,
                         double *rl) {
  const QRule R = rule2();
  for (int q = 0; q < R.n; q++) {
    const double psi[3] = {1.0 - R.xi[q] - R.eta[q], R.xi[q], R.eta[q]};
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    double gu[2] = {0, 0}, gP[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      gu[0] += xl[i] * G.g[i][0];
      gu[1] += xl[i] * G.g[i][1];
      gP[0] += phil[i] * G.g[i][0];
      gP[1] += phil[i] * G.g[i][1];
    }
    const double factor = R.w[q] * G.adet;
    for (int i = 0; i < 3; i++) {
      const double gg = gu[0] * G.g[i][0] + gu[1] * G.g[i][1];
      const double gp = gP[0] * G.g[i][0] + gP[1] * G.g[i][1];
      rl[i] += (gg + u * a.z * gp + 0.0 * u * psi[i]) * factor;
    }
  }
}

// DiffusionTOperator::alpha_volume (src/diffusion_toperator.hh:38-73; quadratic integrand, the
// order-2 rule is exact)
__device__ void lop_difft(const ElGeo &G, const double *xl, double *rl) {
  const QRule R = rule2();
  for (int q = 0; q < R.n; q++) {
    const double psi[3] = {1.0 - R.xi[q] - R.eta[q], R.xi[q], R.eta[q]};
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    const double factor = R.w[q] * G.adet;
    for (int i = 0; i < 3; i++) rl[i] += u * psi[i] * factor;
  }
}

// PoissonOperator::alpha_volume (src/poisson_operator.hh:46-127; (c- - c+) sign)
__device__ void lop_poisson(const ElGeo &G, const FdArgs &a, const double *cpl, const double *cml,
                            const double *xl, double *rl) {
  const QRule R = rule3();
  for (int q = 0; q < R.n; q++) {
    const double factor = cyl_factor(G, R, q, a, R.w[q] * G.adet);
    const double psi[3] = {1.0 - R.xi[q] - R.eta[q], R.xi[q], R.eta[q]};
    double cp = 0, cm = 0;
    for (int i = 0; i < 3; i++) cp += cpl[i] * psi[i];
    for (int i = 0; i < 3; i++) cm += cml[i] * psi[i];
    double gu[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      gu[0] += xl[i] * G.g[i][0];
      gu[1] += xl[i] * G.g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      const double gg = gu[0] * G.g[i][0] + gu[1] * G.g[i][1];
      rl[i] += (gg + 1 * a.l_b * 4 * a.pi * (cm - cp) * psi[i]) * factor;
    }
  }
}

// the element's volume residual of the operator (time-discrete kinds: temporal part + dt times
// the spatial part; the old-time mass and the boundary loads are x-independent and drop out)
template <int NF>
__device__ void op_volume(const ElGeo &G, const FdArgs &a, const double *f0, const double *f1,
                          const double *xl, double *rl) {
  constexpr int NL = 3 * NF;
  for (int i = 0; i < NL; i++) rl[i] = 0.0;
  if constexpr (NF == 3) {
    if (a.kind == OP_PNP) {
      lop_pnp(G, a, xl, rl);
    } else {  // OP_PNP_IE
      double rs[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      lop_pnp(G, a, xl, rs);
      lop_pnpt(G, a, xl, rl);
      for (int i = 0; i < 9; i++) rl[i] += a.dt * rs[i];
    }
  } else {
    if (a.kind == OP_PB) {
      lop_pb(G, a, xl, rl);
    } else if (a.kind == OP_DIFF) {
      lop_diff(G, a, f0, xl, rl);
    } else if (a.kind == OP_DIFF_IE) {
      double rs[3] = {0, 0, 0};
      lop_diff(G, a, f0, xl, rs);
      lop_difft(G, xl, rl);
      for (int i = 0; i < 3; i++) rl[i] += a.dt * rs[i];
    } else {  // OP_POISSON
      lop_poisson(G, a, f0, f1, xl, rl);
    }
  }
}

// the one-step operators' spatial and temporal element residuals, apart
template <int NF>
__device__ void op_spatial(const ElGeo &G, const FdArgs &a, const double *f0, const double *xl,
                           double *rl) {
  for (int i = 0; i < 3 * NF; i++) rl[i] = 0.0;
  if constexpr (NF == 3)
    lop_pnp(G, a, xl, rl);
  else
    lop_diff(G, a, f0, xl, rl);
}
template <int NF>
__device__ void op_temporal(const ElGeo &G, const FdArgs &a, const double *xl, double *rl) {
  for (int i = 0; i < 3 * NF; i++) rl[i] = 0.0;
  if constexpr (NF == 3)
    lop_pnpt(G, a, xl, rl);
  else
    lop_difft(G, xl, rl);
}

// NumericalJacobianVolume::jacobian_volume, epsilon 1e-7, of the element residual ev, with the
// weight w of the operator's accumulation view: J[i][j] = w ((r(u + delta_j e_j) - r(u))_i / delta_j)
template <int NF, typename F>
__device__ void fd_columns(const double *xl, double w, F &&ev, double *J) {
  constexpr int NL = 3 * NF;
  double u[NL], down[NL], up[NL];
  for (int i = 0; i < NL; i++) u[i] = xl[i];
  ev(u, down);
  for (int j = 0; j < NL; j++) {
    const double delta = 1e-7 * (1.0 + fabs(u[j]));
    u[j] += delta;
    ev(u, up);
    for (int i = 0; i < NL; i++) J[i * NL + j] = w * ((up[i] - down[i]) / delta);
    u[j] = xl[j];
  }
}

// one element per thread: jel[e] (stationary), or jel[2e] (spatial) and jel[2e + 1] (temporal)
template <int NF>
__global__ __launch_bounds__(kB) void k_fd_element(int ne, const int *__restrict__ etri,
                                                   const double *__restrict__ xy,
                                                   const double *__restrict__ x,
                                                   const double *__restrict__ aux0,
                                                   const double *__restrict__ aux1, FdArgs a,
                                                   double *__restrict__ jel) {
  constexpr int NL = 3 * NF;
  const int e = blockIdx.x * kB + threadIdx.x;
  if (e >= ne) return;
  const int t[3] = {etri[3 * e], etri[3 * e + 1], etri[3 * e + 2]};
  const ElGeo G = element_geometry(xy + 2 * size_t(t[0]), xy + 2 * size_t(t[1]),
                                   xy + 2 * size_t(t[2]));
  double xl[NL], f0[3] = {0, 0, 0}, f1[3] = {0, 0, 0};
  for (int f = 0; f < NF; f++)
    for (int k = 0; k < 3; k++) xl[3 * f + k] = x[size_t(t[k]) * NF + f];
  if (aux0)
    for (int k = 0; k < 3; k++) f0[k] = aux0[t[k]];
  if (aux1)
    for (int k = 0; k < 3; k++) f1[k] = aux1[t[k]];
  if (a.kind == OP_PNP_IE || a.kind == OP_DIFF_IE) {
    double *J = jel + size_t(2 * e) * NL * NL;
    fd_columns<NF>(xl, a.dt, [&](const double *u, double *r) { op_spatial<NF>(G, a, f0, u, r); },
                   J);
    fd_columns<NF>(xl, 1.0, [&](const double *u, double *r) { op_temporal<NF>(G, a, u, r); },
                   J + NL * NL);
    return;
  }
  fd_columns<NF>(xl, 1.0, [&](const double *u, double *r) { op_volume<NF>(G, a, f0, f1, u, r); },
                 jel + size_t(e) * NL * NL);
}

// block (row, slot) = sum over its element contributions in ascending element order; cdata per
// row: for each slot, the count then codes e * 9 + a * 3 + b (row = local vertex a of element e,
// column = vertex b)
template <int NF, int PAT, int TWO = 0>
__global__ __launch_bounds__(kB) void k_fd_gather(DevLayout L, const long long *__restrict__ rptr,
                                                  const int *__restrict__ cdata,
                                                  const double *__restrict__ jel,
                                                  double *__restrict__ vals) {
  constexpr int NV = popc9(PAT), NL = 3 * NF;
  const int row = blockIdx.x * kB + threadIdx.x;
  if (row >= L.n_owned) return;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = L.chunk_off[chunk], len = int(L.rowmeta[row] & 63);
  long long p = rptr[row];
  for (int s = 0; s < len; s++) {
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; v++) acc[v] = 0.0;
    const int n = cdata[p++];
    for (int k = 0; k < n; k++) {
      const int code = cdata[p++];
      const int e = code / 9, ab = code % 9, ea = ab / 3, eb = ab % 3;
#pragma unroll
      for (int m = 0; m <= TWO; m++) {  // one-step: the spatial matrix, then the temporal one
        const double *J = jel + size_t((TWO + 1) * e + m) * NL * NL;
#pragma unroll
        for (int f = 0; f < NF; f++)
#pragma unroll
          for (int g = 0; g < NF; g++) {
            const int v = pat_index(PAT, f, g);
            if (v >= 0) acc[v] += J[(3 * f + ea) * NL + 3 * g + eb];
          }
      }
    }
    double *sb = vals + (size_t(off) + size_t(s) * kRows) * NV;
#pragma unroll
    for (int v = 0; v < NV; v++) sb[vin(NV, v, lane)] = acc[v];
  }
}

}  // namespace

hipError_t launch_fd_jacobian(const DevLayout &L, const AsmArgs &aa, int nf, int pat, int ne,
                              const int *etri, const long long *rptr, const int *cdata,
                              double *jel, hipStream_t s) {
  FdArgs a{aa.kind, aa.cylindrical, aa.l_b, aa.c0, aa.tau, aa.pi, aa.dt, aa.z};
  const bool diff = aa.kind == OP_DIFF || aa.kind == OP_DIFF_IE;
  const double *f0 = (diff || aa.kind == OP_POISSON) ? aa.aux0 : nullptr;
  const double *f1 = aa.kind == OP_POISSON ? aa.aux1 : nullptr;
  const dim3 ge((ne + kB - 1) / kB), gr((L.n_owned + kB - 1) / kB);
  if (ne > 0) {
    if (nf == 3)
      hipLaunchKernelGGL((k_fd_element<3>), ge, dim3(kB), 0, s, ne, etri, L.xy, aa.x, f0, f1, a,
                         jel);
    else
      hipLaunchKernelGGL((k_fd_element<1>), ge, dim3(kB), 0, s, ne, etri, L.xy, aa.x, f0, f1, a,
                         jel);
  }
  if (L.n_owned == 0) return hipGetLastError();
  if (nf == 3 && pat == kPatPnpFD)
    hipLaunchKernelGGL((k_fd_gather<3, kPatPnpFD>), gr, dim3(kB), 0, s, L, rptr, cdata, jel,
                       aa.vals);
  else if (nf == 3 && pat == kPatPnpIEFD)
    hipLaunchKernelGGL((k_fd_gather<3, kPatPnpIEFD, 1>), gr, dim3(kB), 0, s, L, rptr, cdata, jel,
                       aa.vals);
  else if (nf == 1 && aa.kind == OP_DIFF_IE)
    hipLaunchKernelGGL((k_fd_gather<1, kPatScalar, 1>), gr, dim3(kB), 0, s, L, rptr, cdata, jel,
                       aa.vals);
  else if (nf == 1)
    hipLaunchKernelGGL((k_fd_gather<1, kPatScalar>), gr, dim3(kB), 0, s, L, rptr, cdata, jel,
                       aa.vals);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace pnp
