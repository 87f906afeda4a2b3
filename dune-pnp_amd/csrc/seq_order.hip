// Reference-order mode (PNP_OPT_SEQ_ORDER): the CPU oracle's sequential restatement of the
// reference's arithmetic, operation for operation and in its order, on the GPU, so that a Newton /
// BiCGSTAB run here takes the same iterates -- and the same iteration counts on chaotic systems --
// as the oracle's single-rank run.  A parity mode, not a speed mode: the fast path (assemble.hip,
// linalg.hip) sums in the GPU's orders and its iteration counts agree with the oracle's only as
// distributions where BiCGSTAB is chaotic.  Since round 6 the oracle, and this file,
// restate PDELab's GridOperator accumulation: alpha_boundary's terms go into the element's local
// vector before its one scatter, and a one-step operator's const residual, spatial and temporal
// local vectors are separate passes / scatters.  Parity with the DUNE program itself stays
// unpinned (its grid's vertex order and dune-geometry's tabulated points are not in the tree).
//
// What "the reference's order" is, per step (this file is compiled with -ffp-contract=off: no
// fused multiply-add anywhere, as on the reference's x86-64 build):
//  * element pass (k_seq_element): per element, in the element's own order, the quadrature loops of
//    PnpOperator / PnpTOperator / PBOperator / DiffusionOperator / DiffusionTOperator /
//    PoissonOperator::alpha_volume (src/pnp_operator.hh:46-195, src/pnp_toperator.hh:31-101,
//    src/pb_operator.hh:46-122, src/diffusion_operator.hh:42-112, src/diffusion_toperator.hh:38-73,
//    src/poisson_operator.hh:46-127) on the local DOFs, with factor = w |det J| (* y 2 PI), the
//    gradients through jacobianInverseTransposed, and PDELab's NumericalJacobianVolume forward
//    differences (delta = 1e-7 (1 + |x_j|), the mixins inherited at src/pnp_operator.hh:22-27) or
//    the analytic element Jacobian;
//  * GridOperator::residual / ::jacobian (PDELab, instantiated at src/stationary_pnp_from_pb.hh:165,
//    315-321): the global vector / BCRS matrix starts at 0 (one-step: at the const residual) and
//    every element adds its local block in element order (k_seq_residual_gather /
//    k_seq_jacobian_gather: one thread per row walks the row's incident elements in ascending
//    element index, so every entry sees its terms in the reference's order); an element's local
//    residual holds alpha_volume and then alpha_boundary of its boundary faces (host values, the
//    oracle's boundary_face statements); constrained rows become 0 / identity rows;
//  * ISTL BiCGSTABSolver / CGSolver (dune-istl, src/stationary_pnp_from_pb.hh:168-169,329-331):
//    BCRSMatrix::mv summed per row in ascending column order (k_seq_spmv), scalar products summed
//    sequentially from entry 0 (k_seq_dot: one lane), the vector updates as their expressions
//    (k_seq_bicg_p, k_seq_axpy2, ...), the scalar recurrences on the host in double.
// The CPU oracle (oracle/pnp_oracle.c, test infrastructure) restates the same statements; the GPU
// tests compare the two bit for bit (tests/test_gpu_seq_order.py).
#include "kernels.h"

namespace pnp {

namespace {
constexpr int kB = 256;

// dune-geometry's triangle rules of order 2 (3 points) and 3 (4 points), as the oracle restates
// them (the same constant expressions, so the same doubles)
struct QRule {
  int n;
  double xi[4], eta[4], w[4];
};
__constant__ QRule kQ2 = {3,
                          {4.0 / 6.0, 1.0 / 6.0, 1.0 / 6.0, 0},
                          {1.0 / 6.0, 4.0 / 6.0, 1.0 / 6.0, 0},
                          {0.5 / 3.0, 0.5 / 3.0, 0.5 / 3.0, 0}};
__constant__ QRule kQ3 = {4,
                          {10.0 / 30.0, 18.0 / 30.0, 6.0 / 30.0, 6.0 / 30.0},
                          {10.0 / 30.0, 6.0 / 30.0, 18.0 / 30.0, 6.0 / 30.0},
                          {0.5 * -27.0 / 48.0, 0.5 * 25.0 / 48.0, 0.5 * 25.0 / 48.0,
                           0.5 * 25.0 / 48.0}};
__device__ __forceinline__ const QRule &rule(int order) { return order <= 2 ? kQ2 : kQ3; }

struct Geo {
  double y0, J10, J11, adet;
  double g[3][2];
};

// affine map p0 + xi (p1 - p0) + eta (p2 - p0); J^{-T} = 1/det [[J11, -J10], [-J01, J00]] times the
// reference gradients {(-1,-1), (1,0), (0,1)}
__device__ void geometry(const double *xy, const int *t, Geo &G) {
  const double x0 = xy[2 * t[0]], y0 = xy[2 * t[0] + 1];
  const double J00 = xy[2 * t[1]] - x0, J01 = xy[2 * t[2]] - x0;
  const double J10 = xy[2 * t[1] + 1] - y0, J11 = xy[2 * t[2] + 1] - y0;
  const double det = J00 * J11 - J01 * J10;
  G.y0 = y0;
  G.J10 = J10;
  G.J11 = J11;
  G.adet = fabs(det);
  const double it00 = J11 / det, it01 = -J10 / det, it10 = -J01 / det, it11 = J00 / det;
  const double gh[3][2] = {{-1.0, -1.0}, {1.0, 0.0}, {0.0, 1.0}};
#pragma unroll
  for (int i = 0; i < 3; i++) {
    G.g[i][0] = it00 * gh[i][0] + it01 * gh[i][1];
    G.g[i][1] = it10 * gh[i][0] + it11 * gh[i][1];
  }
}

__device__ __forceinline__ double global_y(const Geo &G, double xi, double eta) {
  return G.y0 + G.J10 * xi + G.J11 * eta;
}
__device__ __forceinline__ void p1(double xi, double eta, double psi[3]) {
  psi[0] = 1.0 - xi - eta;
  psi[1] = xi;
  psi[2] = eta;
}

// ---- local residuals (rl += ...), the reference's statements in its order ----------------------
__device__ void lop_pnp(const Geo &G, const SeqOp &P, const double *xl, double *rl) {
  const double PI = P.pi;
  const QRule &R = rule(3);  // intorder_ = 3 (src/pnp_operator.hh:40)
  for (int q = 0; q < R.n; q++) {
    double factor = R.w[q] * G.adet;                                           // :110
    if (P.cyl) factor *= global_y(G, R.xi[q], R.eta[q]) * 2 * PI;              // :111-112
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
    double u_phi = 0, u_cp = 0, u_cm = 0;                                      // :122-131
    for (int i = 0; i < 3; i++) u_phi += xl[i] * psi[i];
    for (int i = 0; i < 3; i++) u_cp += xl[3 + i] * psi[i];
    for (int i = 0; i < 3; i++) u_cm += xl[6 + i] * psi[i];
    (void)u_phi;
    double gphi[2] = {0, 0}, gcp[2] = {0, 0}, gcm[2] = {0, 0};                 // :154-163
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
    for (int i = 0; i < 3; i++) {                                              // :167-173
      const double gg = gphi[0] * G.g[i][0] + gphi[1] * G.g[i][1];
      rl[i] += (gg + 4 * PI * P.l_b * (u_cp - u_cm) * psi[i]) * factor;
    }
    for (int i = 0; i < 3; i++) {                                              // :177-183
      const double gc = gcp[0] * G.g[i][0] + gcp[1] * G.g[i][1];
      const double gp = gphi[0] * G.g[i][0] + gphi[1] * G.g[i][1];
      rl[3 + i] += (gc - u_cp * gp) * factor;
    }
    for (int i = 0; i < 3; i++) {                                              // :187-193
      const double gc = gcm[0] * G.g[i][0] + gcm[1] * G.g[i][1];
      const double gp = gphi[0] * G.g[i][0] + gphi[1] * G.g[i][1];
      rl[6 + i] += (gc + u_cm * gp) * factor;
    }
  }
}

// PnpTOperator (order 2, tau u psi; quirk Q2: the c- mass into the c+ rows, src/pnp_toperator.hh:
// 93-99)
__device__ void lop_pnpt(const Geo &G, const SeqOp &P, const double *xl, double *rl) {
  const double PI = P.pi;
  const QRule &R = rule(2);
  for (int q = 0; q < R.n; q++) {
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
    double u_cp = 0, u_cm = 0;
    for (int i = 0; i < 3; i++) u_cp += xl[3 + i] * psi[i];
    for (int i = 0; i < 3; i++) u_cm += xl[6 + i] * psi[i];
    double factor = R.w[q] * G.adet;
    if (P.cyl) factor *= global_y(G, R.xi[q], R.eta[q]) * 2 * PI;
    for (int i = 0; i < 3; i++) rl[3 + i] += P.tau * u_cp * psi[i] * factor;
    for (int i = 0; i < 3; i++) rl[3 + i] += P.tau * u_cm * psi[i] * factor;
  }
}

// PBOperator (src/pb_operator.hh:104-120)
__device__ void lop_pb(const Geo &G, const SeqOp &P, const double *xl, double *rl) {
  const double PI = P.pi;
  const QRule &R = rule(3);
  for (int q = 0; q < R.n; q++) {
    double factor = R.w[q] * G.adet;
    if (P.cyl) factor *= global_y(G, R.xi[q], R.eta[q]) * 2 * PI;
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    double gu[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      gu[0] += xl[i] * G.g[i][0];
      gu[1] += xl[i] * G.g[i][1];
    }
    for (int i = 0; i < 3; i++) {
      const double gg = gu[0] * G.g[i][0] + gu[1] * G.g[i][1];
      rl[i] += (gg + 8 * PI * P.l_b * P.c0 * sinh(u) * psi[i]) * factor;
    }
  }
}

// DiffusionOperator (order 2, no cylindrical weight -- quirk Q8; src/diffusion_operator.hh:97-110)
__device__ void lop_diff(const Geo &G, const SeqOp &P, const double *phil, const double *xl,
                         double *rl) {
  const QRule &R = rule(2);
  for (int q = 0; q < R.n; q++) {
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
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
      rl[i] += (gg + u * P.z * gp + 0.0 * u * psi[i]) * factor;
    }
  }
}

// DiffusionTOperator (u psi, exact at order 2)
__device__ void lop_difft(const Geo &G, const double *xl, double *rl) {
  const QRule &R = rule(2);
  for (int q = 0; q < R.n; q++) {
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    const double factor = R.w[q] * G.adet;
    for (int i = 0; i < 3; i++) rl[i] += u * psi[i] * factor;
  }
}

// PoissonOperator (order 3, the (c- - c+) sign, src/poisson_operator.hh:108-125)
__device__ void lop_poisson(const Geo &G, const SeqOp &P, const double *cpl, const double *cml,
                            const double *xl, double *rl) {
  const double PI = P.pi;
  const QRule &R = rule(3);
  for (int q = 0; q < R.n; q++) {
    double factor = R.w[q] * G.adet;
    if (P.cyl) factor *= global_y(G, R.xi[q], R.eta[q]) * 2 * PI;
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
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
      rl[i] += (gg + 1 * P.l_b * 4 * PI * (cm - cp) * psi[i]) * factor;
    }
  }
}

// the element residual of the operator (volume part), rl zeroed here; implicit Euler: the mass
// of u plus dt times the spatial part
__device__ void volume(const Geo &G, const SeqOp &P, const double *aux, const double *xl,
                       double *rl) {
  const int nl = P.nf * 3;
  for (int i = 0; i < nl; i++) rl[i] = 0.0;
  switch (P.kind) {
    case OP_PNP:
      lop_pnp(G, P, xl, rl);
      break;
    case OP_PNP_IE: {
      double rs[9];
      for (int i = 0; i < 9; i++) rs[i] = 0.0;
      lop_pnp(G, P, xl, rs);
      lop_pnpt(G, P, xl, rl);
      for (int i = 0; i < 9; i++) rl[i] += P.dt * rs[i];
    } break;
    case OP_PB:
      lop_pb(G, P, xl, rl);
      break;
    case OP_DIFF:
      lop_diff(G, P, aux, xl, rl);
      break;
    case OP_DIFF_IE: {
      double rs[3] = {0.0, 0.0, 0.0};
      lop_diff(G, P, aux, xl, rs);
      lop_difft(G, xl, rl);
      for (int i = 0; i < 3; i++) rl[i] += P.dt * rs[i];
    } break;
    case OP_POISSON:
      lop_poisson(G, P, aux, aux + 3, xl, rl);
      break;
  }
}

// ---- analytic element Jacobians (J[i nl + j] += scale dR_i/dx_j), the oracle's statements -------
__device__ void jac_pnp(const Geo &G, const SeqOp &P, const double *xl, double *J, double scale) {
  const double PI = P.pi;
  const QRule &R = rule(3);
  for (int q = 0; q < R.n; q++) {
    double factor = R.w[q] * G.adet;
    if (P.cyl) factor *= global_y(G, R.xi[q], R.eta[q]) * 2 * PI;
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
    double u_cp = 0, u_cm = 0, gphi[2] = {0, 0};
    for (int i = 0; i < 3; i++) {
      u_cp += xl[3 + i] * psi[i];
      u_cm += xl[6 + i] * psi[i];
      gphi[0] += xl[i] * G.g[i][0];
      gphi[1] += xl[i] * G.g[i][1];
    }
    const double kap = 4 * PI * P.l_b;
    for (int i = 0; i < 3; i++) {
      const double gp = gphi[0] * G.g[i][0] + gphi[1] * G.g[i][1];
      for (int j = 0; j < 3; j++) {
        const double K = (G.g[j][0] * G.g[i][0] + G.g[j][1] * G.g[i][1]) * factor;
        const double Mq = psi[j] * psi[i] * factor;
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

__device__ void jac_pnpt(const Geo &G, const SeqOp &P, double *J) {
  const double PI = P.pi;
  const QRule &R = rule(2);
  for (int q = 0; q < R.n; q++) {
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
    double factor = R.w[q] * G.adet;
    if (P.cyl) factor *= global_y(G, R.xi[q], R.eta[q]) * 2 * PI;
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        const double v = P.tau * psi[j] * psi[i] * factor;
        J[(3 + i) * 9 + 3 + j] += v;
        J[(3 + i) * 9 + 6 + j] += v;  // Q2
      }
  }
}

__device__ void jac_scalar(const Geo &G, const SeqOp &P, const double *xl, const double *phil,
                           double *J, double scale) {
  const double PI = P.pi;
  const int kind = P.kind;
  const bool pbp = kind == OP_PB || kind == OP_POISSON;
  const QRule &R = rule(pbp ? 3 : 2);
  double gP[2] = {0, 0};
  if (phil)
    for (int i = 0; i < 3; i++) {
      gP[0] += phil[i] * G.g[i][0];
      gP[1] += phil[i] * G.g[i][1];
    }
  for (int q = 0; q < R.n; q++) {
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
    double factor = R.w[q] * G.adet;
    if (P.cyl && pbp) factor *= global_y(G, R.xi[q], R.eta[q]) * 2 * PI;
    double u = 0;
    for (int i = 0; i < 3; i++) u += xl[i] * psi[i];
    for (int i = 0; i < 3; i++) {
      const double gp = gP[0] * G.g[i][0] + gP[1] * G.g[i][1];
      for (int j = 0; j < 3; j++) {
        const double K = (G.g[j][0] * G.g[i][0] + G.g[j][1] * G.g[i][1]) * factor;
        double v = K;
        if (kind == OP_PB) v += 8 * PI * P.l_b * P.c0 * cosh(u) * psi[j] * psi[i] * factor;
        if (kind == OP_DIFF || kind == OP_DIFF_IE)
          v += P.z * psi[j] * gp * factor;
        J[i * 3 + j] += scale * v;
      }
    }
  }
}

__device__ void jac_difft(const Geo &G, double *J) {
  const QRule &R = rule(2);
  for (int q = 0; q < R.n; q++) {
    double psi[3];
    p1(R.xi[q], R.eta[q], psi);
    const double factor = R.w[q] * G.adet;
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) J[i * 3 + j] += psi[j] * psi[i] * factor;
  }
}

// One thread per element, in the mesh's element order.  mode 0: RL[e] = the element's local
// residual -- alpha_volume, then alpha_boundary's terms of its boundary intersections (bval[bptr[e
// nl + i] .. bptr[e nl + i + 1]), host values in face / quadrature order) added one by one; one-step
// operators: RL[e] = the spatial operator's (weight dt), RLT[e] = the temporal operator's, RLO[e] =
// -(the mass of x_old), the const residual; 1: JL[e] = the analytic element Jacobian; 2: JL[e] =
// NumericalJacobianVolume's forward differences (w ((up - down) / delta)); one-step: JL[e] the
// spatial operator's (w = dt), JLT[e] the temporal operator's (w = 1).
__device__ void spatial(const Geo &G, const SeqOp &P, const double *aux, const double *xl,
                        double *rl) {
  for (int i = 0; i < 3 * P.nf; i++) rl[i] = 0.0;
  if (P.nf == 3)
    lop_pnp(G, P, xl, rl);
  else
    lop_diff(G, P, aux, xl, rl);
}
__device__ void temporal(const Geo &G, const SeqOp &P, const double *xl, double *rl) {
  for (int i = 0; i < 3 * P.nf; i++) rl[i] = 0.0;
  if (P.nf == 3)
    lop_pnpt(G, P, xl, rl);
  else
    lop_difft(G, xl, rl);
}
template <typename F>
__device__ void fd_element(const double *xl, int nl, double w, F &&ev, double *J) {
  double u[9], down[9], up[9];
  for (int i = 0; i < nl; i++) u[i] = xl[i];
  ev(u, down);
  for (int j = 0; j < nl; j++) {
    const double delta = 1e-7 * (1.0 + fabs(u[j]));
    u[j] += delta;
    ev(u, up);
    for (int i = 0; i < nl; i++) J[i * nl + j] += w * ((up[i] - down[i]) / delta);
    u[j] = xl[j];
  }
}

__global__ void __launch_bounds__(kB)
    k_seq_element(SeqMesh M, SeqOp P, const double *__restrict__ x, int mode,
                  double *__restrict__ RL, double *__restrict__ RLT, double *__restrict__ RLO,
                  double *__restrict__ JL, double *__restrict__ JLT, const int *__restrict__ bptr,
                  const double *__restrict__ bval) {
  const int e = blockIdx.x * kB + threadIdx.x;
  if (e >= M.nt) return;
  const int nf = P.nf, nl = 3 * nf, nv = M.nv;
  const bool onestep = P.kind == OP_PNP_IE || P.kind == OP_DIFF_IE;
  const int t[3] = {M.tri[3 * e], M.tri[3 * e + 1], M.tri[3 * e + 2]};
  Geo G;
  geometry(M.xy, t, G);
  double xl[9];
  for (int f = 0; f < nf; f++)
    for (int a = 0; a < 3; a++) xl[3 * f + a] = x[size_t(f) * nv + t[a]];
  double aux[6] = {0, 0, 0, 0, 0, 0};
  if (P.kind == OP_DIFF || P.kind == OP_DIFF_IE)
    for (int a = 0; a < 3; a++) aux[a] = P.phi[t[a]];
  if (P.kind == OP_POISSON)
    for (int a = 0; a < 3; a++) {
      aux[a] = P.cp[t[a]];
      aux[3 + a] = P.cm[t[a]];
    }
  if (mode == 0) {
    double rl[9];
    if (onestep) {
      double rs[9];
      spatial(G, P, aux, xl, rs);
      for (int i = 0; i < nl; i++) rl[i] = P.dt * rs[i];
    } else {
      volume(G, P, aux, xl, rl);
    }
    for (int i = 0; i < nl; i++)
      for (int k = bptr[size_t(e) * nl + i]; k < bptr[size_t(e) * nl + i + 1]; k++) rl[i] += bval[k];
    for (int i = 0; i < nl; i++) RL[size_t(e) * nl + i] = rl[i];
    if (onestep) {
      temporal(G, P, xl, rl);
      for (int i = 0; i < nl; i++) RLT[size_t(e) * nl + i] = rl[i];
      double xo[9];
      for (int f = 0; f < nf; f++)
        for (int a = 0; a < 3; a++) xo[3 * f + a] = P.x_old[size_t(f) * nv + t[a]];
      temporal(G, P, xo, rl);
      for (int i = 0; i < nl; i++) RLO[size_t(e) * nl + i] = -rl[i];
    }
    return;
  }
  double J[81];
  for (int i = 0; i < nl * nl; i++) J[i] = 0.0;
  if (onestep) {
    if (mode == 2)
      fd_element(xl, nl, P.dt, [&](const double *u, double *r) { spatial(G, P, aux, u, r); }, J);
    else if (nf == 3)
      jac_pnp(G, P, xl, J, P.dt);
    else
      jac_scalar(G, P, xl, aux, J, P.dt);
    for (int i = 0; i < nl * nl; i++) JL[size_t(e) * nl * nl + i] = J[i];
    for (int i = 0; i < nl * nl; i++) J[i] = 0.0;
    if (mode == 2)
      fd_element(xl, nl, 1.0, [&](const double *u, double *r) { temporal(G, P, u, r); }, J);
    else if (nf == 3)
      jac_pnpt(G, P, J);
    else
      jac_difft(G, J);
    for (int i = 0; i < nl * nl; i++) JLT[size_t(e) * nl * nl + i] = J[i];
    return;
  }
  if (mode == 2) {
    fd_element(xl, nl, 1.0, [&](const double *u, double *r) { volume(G, P, aux, u, r); }, J);
  } else {
    switch (P.kind) {
      case OP_PNP:
        jac_pnp(G, P, xl, J, 1.0);
        break;
      case OP_PB:
      case OP_POISSON:
        jac_scalar(G, P, xl, nullptr, J, 1.0);
        break;
      case OP_DIFF:
        jac_scalar(G, P, xl, aux, J, 1.0);
        break;
    }
  }
  for (int i = 0; i < nl * nl; i++) JL[size_t(e) * nl * nl + i] = J[i];
}

// r[R] for row R = f nv + v: 0, + (one-step) the const residual's element terms (ascending
// element), + per incident element in ascending order its local residual's term (volume and
// boundary) and (one-step) then its temporal term; then 0 if constrained
__global__ void __launch_bounds__(kB)
    k_seq_residual_gather(SeqMesh M, int nf, int has_old, const double *__restrict__ RL,
                          const double *__restrict__ RLT, const double *__restrict__ RLO,
                          const unsigned char *__restrict__ mask, double *__restrict__ r) {
  const int R = blockIdx.x * kB + threadIdx.x;
  if (R >= nf * M.nv) return;
  const int f = R / M.nv, v = R % M.nv, nl = 3 * nf;
  double s = 0.0;
  if (has_old)
    for (int k = M.vptr[v]; k < M.vptr[v + 1]; k++) {
      const int e = M.vinc[k] >> 2, a = M.vinc[k] & 3;
      s += RLO[size_t(e) * nl + 3 * f + a];
    }
  for (int k = M.vptr[v]; k < M.vptr[v + 1]; k++) {
    const int e = M.vinc[k] >> 2, a = M.vinc[k] & 3;
    s += RL[size_t(e) * nl + 3 * f + a];
    if (has_old) s += RLT[size_t(e) * nl + 3 * f + a];
  }
  if (mask[R]) s = 0.0;
  r[R] = s;
}

// the CSR row R (ascending columns, the GPU's reduced pattern: every entry the operator can make
// non-zero) = 0 + the element blocks' (R, C) terms in ascending element order (one-step: each
// element's spatial block, then its temporal block JLT); constrained rows: identity.  An element
// term whose column is outside the pattern is an exact zero in the reference (never written, or a
// forward difference of an unchanged value): skipped.
__global__ void __launch_bounds__(kB)
    k_seq_jacobian_gather(SeqMesh M, int nf, const double *__restrict__ JL,
                          const double *__restrict__ JLT, const int *__restrict__ rowptr,
                          const int *__restrict__ col, const unsigned char *__restrict__ mask,
                          double *__restrict__ val) {
  const int R = blockIdx.x * kB + threadIdx.x;
  if (R >= nf * M.nv) return;
  const int f = R / M.nv, v = R % M.nv, nl = 3 * nf;
  const int k0 = rowptr[R], k1 = rowptr[R + 1];
  for (int k = k0; k < k1; k++) val[k] = 0.0;
  for (int q = M.vptr[v]; q < M.vptr[v + 1]; q++) {
    const int e = M.vinc[q] >> 2, a = M.vinc[q] & 3;
    const int t[3] = {M.tri[3 * e], M.tri[3 * e + 1], M.tri[3 * e + 2]};
    for (int pass = 0; pass < (JLT ? 2 : 1); pass++) {
      const double *B = pass ? JLT : JL;
      for (int j = 0; j < nl; j++) {
        const int C = (j / 3) * M.nv + t[j % 3];
        int lo = k0, hi = k1 - 1, at = -1;
        while (lo <= hi) {
          const int mid = (lo + hi) >> 1;
          if (col[mid] == C) {
            at = mid;
            break;
          }
          if (col[mid] < C)
            lo = mid + 1;
          else
            hi = mid - 1;
        }
        if (at >= 0) val[at] += B[size_t(e) * nl * nl + size_t(3 * f + a) * nl + j];
      }
    }
  }
  if (mask[R])
    for (int k = k0; k < k1; k++) val[k] = col[k] == R ? 1.0 : 0.0;
}

// ---- ISTL's BLAS in its order -----------------------------------------------------------------
__global__ void __launch_bounds__(kB)
    k_seq_spmv(int n, const int *__restrict__ rowptr, const int *__restrict__ col,
               const double *__restrict__ val, const double *__restrict__ x, double *__restrict__ y) {
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  double s = 0;
  for (int k = rowptr[i]; k < rowptr[i + 1]; k++) s += val[k] * x[col[k]];
  y[i] = s;
}

// s = 0; s += a_i b_i for i = 0 .. n-1: one lane sums, the wave's other lanes fetch ahead
__global__ void __launch_bounds__(64)
    k_seq_dot(int n, const double *__restrict__ a, const double *__restrict__ b,
              double *__restrict__ out) {
  const int lane = threadIdx.x;
  double s = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const double p = i < n ? a[i] * b[i] : 0.0;
    const int m = min(64, n - i0);
    for (int k = 0; k < m; k++) {
      const double pk = __shfl(p, k, 64);
      if (lane == 0) s += pk;
    }
  }
  if (lane == 0) out[0] = s;
}

// p = beta (p - omega v) + r
__global__ void __launch_bounds__(kB)
    k_seq_bicg_p(int n, double beta, double omega, double *__restrict__ p,
                 const double *__restrict__ v, const double *__restrict__ r) {
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i < n) p[i] = beta * (p[i] - omega * v[i]) + r[i];
}

// x += a y; r -= a v
__global__ void __launch_bounds__(kB)
    k_seq_axpy2(int n, double a, double *__restrict__ x, const double *__restrict__ y,
                double *__restrict__ r, const double *__restrict__ v) {
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i < n) {
    x[i] += a * y[i];
    r[i] -= a * v[i];
  }
}

// v (zero on entry) = M^{-1} d: Richardson (v += 1.0 d) or Jacobi (v = d / a_ii)
__global__ void __launch_bounds__(kB)
    k_seq_prec_diag(int n, int jacobi, const double *__restrict__ d, const int *__restrict__ diag,
                    const double *__restrict__ val, double *__restrict__ v) {
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  if (jacobi)
    v[i] = d[i] / val[diag[i]];
  else
    v[i] = 0.0 + 1.0 * d[i];
}

// CG: x += lambda p (own loop), r -= lambda q, p = q + beta p
__global__ void __launch_bounds__(kB)
    k_seq_axpy(int n, double a, double *__restrict__ x, const double *__restrict__ y) {
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i < n) x[i] += a * y[i];
}
__global__ void __launch_bounds__(kB)
    k_seq_aymx(int n, double a, double *__restrict__ x, const double *__restrict__ y) {
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i < n) x[i] -= a * y[i];
}
__global__ void __launch_bounds__(kB)
    k_seq_cg_p(int n, double beta, double *__restrict__ p, const double *__restrict__ q) {
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i < n) p[i] = q[i] + beta * p[i];
}

inline dim3 grid(long long n) { return dim3(unsigned((n + kB - 1) / kB)); }
}  // namespace

hipError_t launch_seq_element(const SeqMesh &M, const SeqOp &P, const double *x, int mode,
                              double *RL, double *RLT, double *RLO, double *JL, double *JLT,
                              const int *bptr, const double *bval, hipStream_t s) {
  if (M.nt <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_seq_element, grid(M.nt), dim3(kB), 0, s, M, P, x, mode, RL, RLT, RLO, JL,
                     JLT, bptr, bval);
  return hipGetLastError();
}
hipError_t launch_seq_residual_gather(const SeqMesh &M, int nf, int has_old, const double *RL,
                                      const double *RLT, const double *RLO,
                                      const unsigned char *mask, double *r, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_residual_gather, grid((long long)nf * M.nv), dim3(kB), 0, s, M, nf,
                     has_old, RL, RLT, RLO, mask, r);
  return hipGetLastError();
}
hipError_t launch_seq_jacobian_gather(const SeqMesh &M, int nf, const double *JL,
                                      const double *JLT, const int *rowptr, const int *col,
                                      const unsigned char *mask, double *val, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_jacobian_gather, grid((long long)nf * M.nv), dim3(kB), 0, s, M, nf, JL,
                     JLT, rowptr, col, mask, val);
  return hipGetLastError();
}
hipError_t launch_seq_spmv(int n, const int *rowptr, const int *col, const double *val,
                           const double *x, double *y, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_spmv, grid(n), dim3(kB), 0, s, n, rowptr, col, val, x, y);
  return hipGetLastError();
}
hipError_t launch_seq_dot(int n, const double *a, const double *b, double *out, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_dot, dim3(1), dim3(64), 0, s, n, a, b, out);
  return hipGetLastError();
}
hipError_t launch_seq_bicg_p(int n, double beta, double omega, double *p, const double *v,
                             const double *r, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_bicg_p, grid(n), dim3(kB), 0, s, n, beta, omega, p, v, r);
  return hipGetLastError();
}
hipError_t launch_seq_axpy2(int n, double a, double *x, const double *y, double *r,
                            const double *v, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_axpy2, grid(n), dim3(kB), 0, s, n, a, x, y, r, v);
  return hipGetLastError();
}
hipError_t launch_seq_prec_diag(int n, int jacobi, const double *d, const int *diag,
                                const double *val, double *v, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_prec_diag, grid(n), dim3(kB), 0, s, n, jacobi, d, diag, val, v);
  return hipGetLastError();
}
hipError_t launch_seq_axpy(int n, double a, double *x, const double *y, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_axpy, grid(n), dim3(kB), 0, s, n, a, x, y);
  return hipGetLastError();
}
hipError_t launch_seq_aymx(int n, double a, double *x, const double *y, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_aymx, grid(n), dim3(kB), 0, s, n, a, x, y);
  return hipGetLastError();
}
hipError_t launch_seq_cg_p(int n, double beta, double *p, const double *q, hipStream_t s) {
  hipLaunchKernelGGL(k_seq_cg_p, grid(n), dim3(kB), 0, s, n, beta, p, q);
  return hipGetLastError();
}

}  // namespace pnp
