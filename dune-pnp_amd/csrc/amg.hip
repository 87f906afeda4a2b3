// Aggregation AMG preconditioner on gfx950 (PNP_PREC_AMG): the reference's CG_AMG_SSOR variant
// (ISTLBackend_NOVLP_CG_AMG_SSOR, src/instationary_pnp_from_pb_md.hh:24,207-210; dune-istl
// Amg::AMG with an SSOR smoother) restated for the GPU.
//
// Hierarchy (amg_setup.cc): level 0 is the assembled SELL matrix itself; level l+1 aggregates the
// vertex rows of level l (greedy, on the matrix graph) with piecewise-constant prolongation, so
// A_{l+1} = P^T A_l P is a plain sum of fine blocks.  Coarse levels are block-CSR with dense
// NF x NF blocks.  The pattern and the per-coarse-block contributor lists are built once on the
// host; the values are summed here after every assembly (deterministic: each coarse block is one
// thread summing its contributors in a fixed order, no atomics).
//
// V-cycle (precond): level 0 pre/post-smoothing with the configured fine smoother (multicolour
// SGS = SSOR(k=1, w=1) by default, or ILU(0) / Jacobi), damped block-Jacobi on the coarse
// levels, an exact dense solve (Gauss-Jordan inverse, one workgroup) on the coarsest.
// Restriction is fused with the residual and the next level's pre-smoothing; prolongation is
// fused into the post-smoothing sweep.  Everything here is HBM/latency bound, fp64.
#include <algorithm>
#include <type_traits>

#include "amg.h"

namespace pnp {

namespace {

constexpr int kB = 256;

// dense NF x NF block position of pattern value v
template <int PAT>
__device__ __forceinline__ int dense_of(int v) {
  int c = 0;
  for (int i = 0; i < 9; i++)
    if ((PAT >> i) & 1) {
      if (c == v) return (i / 3) * (PAT == kPatScalar ? 1 : 3) + (i % 3) * (PAT == kPatScalar ? 0 : 1);
      c++;
    }
  return 0;
}

// ---- Galerkin products ----------------------------------------------------------------------
// level 1 from the SELL k-form matrix: coarse block q = sum of the expanded, row-masked fine
// blocks csrc[cptr[q] .. cptr[q+1]) (code row << 6 | slot)
template <int NF, int PAT>
__global__ __launch_bounds__(kB) void k_galerkin0(DevLayout L, const double *__restrict__ kv,
                                                  long long nq, const long long *__restrict__ cptr,
                                                  const int *__restrict__ csrc,
                                                  double *__restrict__ cv) {
  constexpr int NV = popc9(PAT), NK = nks_of(PAT), NB = NF * NF;
  const long long q = blockIdx.x * (long long)kB + threadIdx.x;
  if (q >= nq) return;
  double acc[NB];
#pragma unroll
  for (int v = 0; v < NB; v++) acc[v] = 0;
  for (long long c = cptr[q]; c < cptr[q + 1]; c++) {
    const int code = csrc[c], row = code >> 6, slot = code & 63;
    const int chunk = row / kRows, lane = row % kRows;
    double K[NK], B[NV];
    load_vals<NK>(kv + (size_t(L.chunk_off[chunk]) + size_t(slot) * kRows) * NK, lane, K);
    expand_k<PAT>(K, B);
    mask_rows<NF, PAT>(B, row_mask<NF>(L, row), slot == 0);
#pragma unroll
    for (int v = 0; v < NV; v++) acc[dense_of<PAT>(v)] += B[v];
  }
#pragma unroll
  for (int v = 0; v < NB; v++) cv[q * NB + v] = acc[v];
}

// level l+1 from level l (block-CSR): coarse block q = sum of fine blocks csrc[..]
template <int NB>
__global__ __launch_bounds__(kB) void k_galerkin(long long nq, const long long *__restrict__ cptr,
                                                 const int *__restrict__ csrc,
                                                 const double *__restrict__ fv,
                                                 double *__restrict__ cv) {
  const long long q = blockIdx.x * (long long)kB + threadIdx.x;
  if (q >= nq) return;
  double acc[NB];
#pragma unroll
  for (int v = 0; v < NB; v++) acc[v] = 0;
  for (long long c = cptr[q]; c < cptr[q + 1]; c++) {
    const double *s = fv + size_t(csrc[c]) * NB;
#pragma unroll
    for (int v = 0; v < NB; v++) acc[v] += s[v];
  }
#pragma unroll
  for (int v = 0; v < NB; v++) cv[q * NB + v] = acc[v];
}

// in-register Gauss-Jordan inverse of an NF x NF block with partial pivoting
template <int NF>
__device__ __forceinline__ void block_inverse(double (&A)[NF * NF], double (&X)[NF * NF]) {
#pragma unroll
  for (int i = 0; i < NF * NF; i++) X[i] = (i % (NF + 1) == 0) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < NF; k++) {
    int p = k;
#pragma unroll
    for (int i = k + 1; i < NF; i++)
      if (fabs(A[i * NF + k]) > fabs(A[p * NF + k])) p = i;
    if (p != k) {
#pragma unroll
      for (int j = 0; j < NF; j++) {
        double t = A[k * NF + j];
        A[k * NF + j] = A[p * NF + j];
        A[p * NF + j] = t;
        t = X[k * NF + j];
        X[k * NF + j] = X[p * NF + j];
        X[p * NF + j] = t;
      }
    }
    const double inv = 1.0 / A[k * NF + k];
#pragma unroll
    for (int j = 0; j < NF; j++) {
      A[k * NF + j] *= inv;
      X[k * NF + j] *= inv;
    }
#pragma unroll
    for (int i = 0; i < NF; i++) {
      if (i == k) continue;
      const double f = A[i * NF + k];
#pragma unroll
      for (int j = 0; j < NF; j++) {
        A[i * NF + j] -= f * A[k * NF + j];
        X[i * NF + j] -= f * X[k * NF + j];
      }
    }
  }
}

// dinv[i] = inverse of the diagonal block of row i (block-CSR, dpos = diagonal block position)
template <int NF>
__global__ __launch_bounds__(kB) void k_dinv(int nb, const int *__restrict__ dpos,
                                             const double *__restrict__ v,
                                             double *__restrict__ dinv) {
  constexpr int NB = NF * NF;
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i >= nb) return;
  double A[NB], X[NB];
#pragma unroll
  for (int k = 0; k < NB; k++) A[k] = v[size_t(dpos[i]) * NB + k];
  block_inverse<NF>(A, X);
#pragma unroll
  for (int k = 0; k < NB; k++) dinv[size_t(i) * NB + k] = X[k];
}

// coarsest level: ROW-major dense copy of the block-CSR matrix A, i.e. A^T column-major.
// rocSOLVER getrf/getri (column-major, in place, ctx.cc amg_setup) then leave (A^T)^-1 =
// (A^-1)^T column-major = A^-1 row-major, the layout k_coarse_apply streams row by row.
__global__ __launch_bounds__(kB) void k_coarse_dense(int nb, int nf, const int *__restrict__ rp,
                                                     const int *__restrict__ col,
                                                     const double *__restrict__ v,
                                                     double *__restrict__ dense) {
  const int r = blockIdx.x * kB + threadIdx.x;
  if (r >= nb) return;
  const int n = nb * nf, nbb = nf * nf;
  for (int q = rp[r]; q < rp[r + 1]; q++)
    for (int e = 0; e < nbb; e++)  // entry (r*nf + e/nf, col*nf + e%nf)
      dense[size_t(r * nf + e / nf) * n + col[q] * nf + e % nf] = v[size_t(q) * nbb + e];
}

// ---- V-cycle kernels ------------------------------------------------------------------------
template <int NF, typename VT = double>
__device__ __forceinline__ void bmv_acc(const VT *__restrict__ B, const double (&x)[NF],
                                        double (&y)[NF]) {
#pragma unroll
  for (int f = 0; f < NF; f++)
#pragma unroll
    for (int g = 0; g < NF; g++) y[f] += double(B[f * NF + g]) * x[g];
}

// The coarse levels are small (68K .. 17 rows at config 3) with ~10-20 blocks per row, so one
// thread per row leaves a chain of dependent gathers per thread and too few waves to hide it
// (the first version took 470 us per V-cycle in these kernels).  Here LPR lanes share a row:
// each takes every LPR-th block / member, and the lanes combine with cross-lane adds.
constexpr int kLpr = 8;

template <int NF, int LPR>
__device__ __forceinline__ void lanes_sum(double (&v)[NF]) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1)
#pragma unroll
    for (int f = 0; f < NF; f++) v[f] += __shfl_xor(v[f], o, LPR);
}

// Row tasks of the grid kernels below: row I, lane q of its LPR lanes; every lane of a row calls
// (live or not: the cross-lane adds need all).

// r = b - A x on a coarse level (block-CSR)
template <int NF, int LPR, typename VT>
__device__ __forceinline__ void resid_task(int I, int q, bool live, const int *__restrict__ rp,
                                           const int *__restrict__ col,
                                           const VT *__restrict__ v,
                                           const double *__restrict__ x,
                                           const double *__restrict__ b, double *__restrict__ r) {
  constexpr int NB = NF * NF;
  double acc[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] = 0;
  if (live)
    for (int k = rp[I] + q; k < rp[I + 1]; k += LPR) {
      double xj[NF];
      load_nf<NF>(x, size_t(col[k]), xj);
      bmv_acc<NF, VT>(v + size_t(k) * NB, xj, acc);
    }
  lanes_sum<NF, LPR>(acc);
  if (!live || q != 0) return;
  double o[NF];
  load_nf<NF>(b, size_t(I), o);
#pragma unroll
  for (int f = 0; f < NF; f++) o[f] -= acc[f];
  store_nf<NF>(r, size_t(I), o);
}

// restriction: bn[J] = sum over the members i of aggregate J of (a - sub)_i (sub may be null);
// pre-smoothing of the coarse level from zero: xn = omega Dinv_J bn[J] (xn null: none)
template <int NF, int LPR>
__device__ __forceinline__ void restrict_task(int J, int q, bool live, const int *__restrict__ mptr,
                                              const int *__restrict__ mem,
                                              const double *__restrict__ a,
                                              const double *__restrict__ sub,
                                              double *__restrict__ bn,
                                              const double *__restrict__ dinvn, double omega,
                                              double *__restrict__ xn) {
  double s[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) s[f] = 0;
  if (live)
    for (int m = mptr[J] + q; m < mptr[J + 1]; m += LPR) {
      const int i = mem[m];
      double ai[NF];
      load_nf<NF>(a, size_t(i), ai);
      if (sub) {
        double si[NF];
        load_nf<NF>(sub, size_t(i), si);
#pragma unroll
        for (int f = 0; f < NF; f++) ai[f] -= si[f];
      }
#pragma unroll
      for (int f = 0; f < NF; f++) s[f] += ai[f];
    }
  lanes_sum<NF, LPR>(s);
  if (!live || q != 0) return;
  store_nf<NF>(bn, size_t(J), s);
  if (xn) {
    double y[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) y[f] = 0;
    bmv_acc<NF>(dinvn + size_t(J) * NF * NF, s, y);
#pragma unroll
    for (int f = 0; f < NF; f++) y[f] *= omega;
    store_nf<NF>(xn, size_t(J), y);
  }
}

// one damped block-Jacobi sweep, with the coarse correction folded in when CORR:
//   xc(j) = x[j] (+ e[agg[j]]),  out[I] = xc(I) + omega Dinv_I (b_I - sum_j A_Ij xc(j))
template <int NF, int LPR, int CORR, typename VT>
__device__ __forceinline__ void jacobi_task(int I, int q, bool live, const int *__restrict__ rp,
                                            const int *__restrict__ col,
                                            const VT *__restrict__ v,
                                            const int *__restrict__ agg,
                                            const double *__restrict__ x,
                                            const double *__restrict__ e,
                                            const double *__restrict__ b,
                                            const double *__restrict__ dinv, double omega,
                                            double *__restrict__ out) {
  constexpr int NB = NF * NF;
  double acc[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] = 0;
  if (live)
    for (int k = rp[I] + q; k < rp[I + 1]; k += LPR) {
      const int j = col[k];
      double xj[NF];
      load_nf<NF>(x, size_t(j), xj);
      if (CORR) {
        double ej[NF];
        load_nf<NF>(e, size_t(agg[j]), ej);
#pragma unroll
        for (int f = 0; f < NF; f++) xj[f] += ej[f];
      }
      bmv_acc<NF, VT>(v + size_t(k) * NB, xj, acc);
    }
  lanes_sum<NF, LPR>(acc);
  if (!live || q != 0) return;
  double r[NF], xi[NF];
  load_nf<NF>(b, size_t(I), r);
#pragma unroll
  for (int f = 0; f < NF; f++) r[f] -= acc[f];
  load_nf<NF>(x, size_t(I), xi);
  if (CORR) {
    double ei[NF];
    load_nf<NF>(e, size_t(agg[I]), ei);
#pragma unroll
    for (int f = 0; f < NF; f++) xi[f] += ei[f];
  }
  double y[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) y[f] = 0;
  bmv_acc<NF>(dinv + size_t(I) * NB, r, y);
#pragma unroll
  for (int f = 0; f < NF; f++) xi[f] += omega * y[f];
  store_nf<NF>(out, size_t(I), xi);
}

template <int NF, int LPR, typename VT>
__global__ __launch_bounds__(kB) void k_resid(int nb, const int *__restrict__ rp,
                                              const int *__restrict__ col,
                                              const VT *__restrict__ v,
                                              const double *__restrict__ x,
                                              const double *__restrict__ b,
                                              double *__restrict__ r) {
  const int gt = blockIdx.x * kB + threadIdx.x, I = gt / LPR;
  resid_task<NF, LPR, VT>(I, gt % LPR, I < nb, rp, col, v, x, b, r);
}

template <int NF, int LPR>
__global__ __launch_bounds__(kB) void k_restrict(int nbn, const int *__restrict__ mptr,
                                                 const int *__restrict__ mem,
                                                 const double *__restrict__ a,
                                                 const double *__restrict__ sub,
                                                 double *__restrict__ bn,
                                                 const double *__restrict__ dinvn, double omega,
                                                 double *__restrict__ xn) {
  const int gt = blockIdx.x * kB + threadIdx.x, J = gt / LPR;
  restrict_task<NF, LPR>(J, gt % LPR, J < nbn, mptr, mem, a, sub, bn, dinvn, omega, xn);
}

// post-smoothing sweep (CORR = 1: with the coarse correction e folded in; 0: plain sweep)
template <int NF, int LPR, int CORR, typename VT>
__global__ __launch_bounds__(kB) void k_post(int nb, const int *__restrict__ rp,
                                             const int *__restrict__ col,
                                             const VT *__restrict__ v,
                                             const int *__restrict__ agg,
                                             const double *__restrict__ x,
                                             const double *__restrict__ e,
                                             const double *__restrict__ b,
                                             const double *__restrict__ dinv, double omega,
                                             double *__restrict__ out) {
  const int gt = blockIdx.x * kB + threadIdx.x, I = gt / LPR;
  jacobi_task<NF, LPR, CORR, VT>(I, gt % LPR, I < nb, rp, col, v, agg, x, e, b, dinv, omega,
                                 out);
}

// coarsest: x = Ainv b, Ainv row-major n x n (n <= kAmgMaxDense; see k_coarse_dense).  One wave
// per row: its 64 lanes stream the row in 1-KB pieces (VEC2, n even: 16-B loads, each row
// 16-B aligned) or 512-B pieces (n odd) against b staged in LDS, four accumulators per lane, then
// a fixed cross-lane tree -- the same sums in the same order every call.  The column-major form
// before it (16 rows per 1,024-thread workgroup: 169 workgroups at n = 2,694, each load four 128-B
// segments) took 25 us per call at config 3, 2.3 TB/s on the 58-MB inverse
// (profiles/r05/amg/split_r5o.txt).
constexpr int kCaWaves = 4;
template <int VEC2>
__global__ __launch_bounds__(64 * kCaWaves) void k_coarse_apply(int n,
                                                               const double *__restrict__ ainv,
                                                               const double *__restrict__ b,
                                                               double *__restrict__ x) {
  __shared__ double bs[kAmgMaxDense];
  for (int j = threadIdx.x; j < n; j += 64 * kCaWaves) bs[j] = b[j];
  __syncthreads();
  const int l = threadIdx.x % 64, i = blockIdx.x * kCaWaves + threadIdx.x / 64;
  if (i >= n) return;
  const double *__restrict__ row = ainv + size_t(i) * n;
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  if constexpr (VEC2) {
    const double2 *__restrict__ r2 = reinterpret_cast<const double2 *>(row);
    const int n2 = n / 2;
    int p = l;
#pragma unroll 4
    for (; p + 64 < n2; p += 128) {
      const double2 u = r2[p], w = r2[p + 64];
      s0 = __builtin_fma(u.x, bs[2 * p], s0);
      s1 = __builtin_fma(u.y, bs[2 * p + 1], s1);
      s2 = __builtin_fma(w.x, bs[2 * p + 128], s2);
      s3 = __builtin_fma(w.y, bs[2 * p + 129], s3);
    }
    if (p < n2) {
      const double2 u = r2[p];
      s0 = __builtin_fma(u.x, bs[2 * p], s0);
      s1 = __builtin_fma(u.y, bs[2 * p + 1], s1);
    }
  } else {
    int j = l;
#pragma unroll 2
    for (; j + 192 < n; j += 256) {
      s0 = __builtin_fma(row[j], bs[j], s0);
      s1 = __builtin_fma(row[j + 64], bs[j + 64], s1);
      s2 = __builtin_fma(row[j + 128], bs[j + 128], s2);
      s3 = __builtin_fma(row[j + 192], bs[j + 192], s3);
    }
    for (; j < n; j += 64) s0 = __builtin_fma(row[j], bs[j], s0);
  }
  double t = (s0 + s1) + (s2 + s3);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  if (l == 0) x[i] = t;
}

// (Running the small levels -- pre-smoothing, residual, restriction, coarsest solve,
// post-smoothing -- inside ONE workgroup with __syncthreads() between the steps was measured and
// lost: 120 us for the levels <= 2048 rows against ~50 us of separate launches, and still +11 us
// per V-cycle for the levels <= 256 rows (profiles/r01/ab_amg_tail_*.log): one CU cannot hide the
// dependent gathers that ~4.5 us launches spread over the whole chip.)

// single-precision copy of a coarse level's block values (the V-cycle's sweeps and residuals read
// it; the Galerkin products, the diagonal inverses and the coarsest solve keep fp64)
__global__ __launch_bounds__(kB) void k_to_f32(long long n, const double *__restrict__ v,
                                               float *__restrict__ vf) {
  for (long long i = blockIdx.x * (long long)kB + threadIdx.x; i < n; i += (long long)gridDim.x * kB)
    vf[i] = float(v[i]);
}

// level 0 prolongation: y = x0 + e1[agg0] (x0 null: the cycle without level-0 pre-smoothing,
// x0 = 0, y = e1[agg0] -- no 17.7-MB memset of x0 per cycle at config 3)
template <int NF>
__global__ __launch_bounds__(kB) void k_prolong0(int n, const int *__restrict__ agg,
                                                 const double *__restrict__ x0,
                                                 const double *__restrict__ e1,
                                                 double *__restrict__ y) {
  const int i = blockIdx.x * kB + threadIdx.x;
  if (i >= n) return;
  double a[NF], c[NF];
  load_nf<NF>(e1, size_t(agg[i]), c);
  if (x0) {
    load_nf<NF>(x0, size_t(i), a);
#pragma unroll
    for (int f = 0; f < NF; f++) c[f] = a[f] + c[f];
  }
  store_nf<NF>(y, size_t(i), c);
}

inline dim3 g1(long long n) { return dim3(unsigned((n + kB - 1) / kB)); }

}  // namespace

#define AMG_NF_DISPATCH(NF_, ...)         \
  do {                                    \
    if ((NF_) == 1) {                     \
      constexpr int NFc = 1;              \
      __VA_ARGS__;                        \
    } else if ((NF_) == 3) {              \
      constexpr int NFc = 3;              \
      __VA_ARGS__;                        \
    } else {                              \
      return hipErrorInvalidValue;        \
    }                                     \
  } while (0)

hipError_t launch_amg_galerkin0(const DevLayout &L, int nf, int pat, const double *kvals,
                                long long nq, const long long *cptr, const int *csrc, double *cv,
                                hipStream_t s) {
  if (nq == 0) return hipSuccess;
  if (nf == 3 && pat == kPatPnp)
    hipLaunchKernelGGL((k_galerkin0<3, kPatPnp>), g1(nq), dim3(kB), 0, s, L, kvals, nq, cptr, csrc, cv);
  else if (nf == 3 && pat == kPatPnpIE)
    hipLaunchKernelGGL((k_galerkin0<3, kPatPnpIE>), g1(nq), dim3(kB), 0, s, L, kvals, nq, cptr, csrc, cv);
  else if (nf == 3 && pat == kPatPnpFD)
    hipLaunchKernelGGL((k_galerkin0<3, kPatPnpFD>), g1(nq), dim3(kB), 0, s, L, kvals, nq, cptr, csrc, cv);
  else if (nf == 3 && pat == kPatPnpIEFD)
    hipLaunchKernelGGL((k_galerkin0<3, kPatPnpIEFD>), g1(nq), dim3(kB), 0, s, L, kvals, nq, cptr, csrc, cv);
  else if (nf == 1)
    hipLaunchKernelGGL((k_galerkin0<1, kPatScalar>), g1(nq), dim3(kB), 0, s, L, kvals, nq, cptr, csrc, cv);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_amg_galerkin(int nf, long long nq, const long long *cptr, const int *csrc,
                               const double *fv, double *cv, hipStream_t s) {
  if (nq == 0) return hipSuccess;
  AMG_NF_DISPATCH(nf, hipLaunchKernelGGL((k_galerkin<NFc * NFc>), g1(nq), dim3(kB), 0, s, nq, cptr,
                                          csrc, fv, cv));
  return hipGetLastError();
}

hipError_t launch_amg_dinv(int nf, int nb, const int *dpos, const double *v, double *dinv,
                           hipStream_t s) {
  if (nb == 0) return hipSuccess;
  AMG_NF_DISPATCH(nf, hipLaunchKernelGGL((k_dinv<NFc>), g1(nb), dim3(kB), 0, s, nb, dpos, v, dinv));
  return hipGetLastError();
}

hipError_t launch_amg_coarse_dense(int nf, int nb, const int *rp, const int *col, const double *v,
                                   double *dense, hipStream_t s) {
  const size_t n = size_t(nb) * nf;
  hipError_t e = hipMemsetAsync(dense, 0, sizeof(double) * n * n, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_coarse_dense, g1(nb), dim3(kB), 0, s, nb, nf, rp, col, v, dense);
  return hipGetLastError();
}

hipError_t launch_amg_restrict(int nf, int nbn, const int *mptr, const int *mem, const double *a,
                               const double *sub, double *bn, const double *dinvn, double omega,
                               double *xn, hipStream_t s) {
  if (nbn == 0) return hipSuccess;
  AMG_NF_DISPATCH(nf, hipLaunchKernelGGL((k_restrict<NFc, kLpr>), g1((long long)nbn * kLpr),
                                         dim3(kB), 0, s, nbn, mptr, mem, a, sub, bn, dinvn, omega,
                                         xn));
  return hipGetLastError();
}

hipError_t launch_amg_resid(int nf, int nb, const int *rp, const int *col, const double *v,
                            const float *vf, const double *x, const double *b, double *r,
                            hipStream_t s) {
  if (nb == 0) return hipSuccess;
  if (vf)
    AMG_NF_DISPATCH(nf, hipLaunchKernelGGL((k_resid<NFc, kLpr, float>), g1((long long)nb * kLpr),
                                           dim3(kB), 0, s, nb, rp, col, vf, x, b, r));
  else
    AMG_NF_DISPATCH(nf, hipLaunchKernelGGL((k_resid<NFc, kLpr, double>), g1((long long)nb * kLpr),
                                           dim3(kB), 0, s, nb, rp, col, v, x, b, r));
  return hipGetLastError();
}

hipError_t launch_amg_to_f32(long long n, const double *v, float *vf, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const long long g = std::min<long long>((n + kB - 1) / kB, 4096);
  hipLaunchKernelGGL(k_to_f32, dim3(unsigned(g)), dim3(kB), 0, s, n, v, vf);
  return hipGetLastError();
}

// the same GEMV on a single-precision copy of the inverse (PNP_AMG_F32), rows padded to ld
// (a multiple of 4) so each lane's 16-B loads carry four columns; fp64 arithmetic, the same
// accumulator and tree shape
__global__ __launch_bounds__(64 * kCaWaves) void k_coarse_apply_f32(int n, int ld,
                                                                   const float *__restrict__ ainv,
                                                                   const double *__restrict__ b,
                                                                   double *__restrict__ x) {
  __shared__ double bs[kAmgMaxDense + 4];
  for (int j = threadIdx.x; j < ld; j += 64 * kCaWaves) bs[j] = j < n ? b[j] : 0.0;
  __syncthreads();
  const int l = threadIdx.x % 64, i = blockIdx.x * kCaWaves + threadIdx.x / 64;
  if (i >= n) return;
  const float4 *__restrict__ r4 = reinterpret_cast<const float4 *>(ainv + size_t(i) * ld);
  const int n4 = ld / 4;
  double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma unroll 4
  for (int p = l; p < n4; p += 64) {
    const float4 u = r4[p];
    s0 = __builtin_fma(double(u.x), bs[4 * p], s0);
    s1 = __builtin_fma(double(u.y), bs[4 * p + 1], s1);
    s2 = __builtin_fma(double(u.z), bs[4 * p + 2], s2);
    s3 = __builtin_fma(double(u.w), bs[4 * p + 3], s3);
  }
  double t = (s0 + s1) + (s2 + s3);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  if (l == 0) x[i] = t;
}

__global__ __launch_bounds__(kB) void k_inverse_to_f32(int n, int ld, const double *__restrict__ a,
                                                       float *__restrict__ af) {
  const long long tot = (long long)n * ld;
  for (long long q = blockIdx.x * (long long)kB + threadIdx.x; q < tot;
       q += (long long)gridDim.x * kB) {
    const int i = int(q / ld), j = int(q % ld);
    af[q] = j < n ? float(a[size_t(i) * n + j]) : 0.0f;
  }
}

hipError_t launch_amg_inverse_to_f32(int n, int ld, const double *a, float *af, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const long long g = std::min<long long>(((long long)n * ld + kB - 1) / kB, 8192);
  hipLaunchKernelGGL(k_inverse_to_f32, dim3(unsigned(g)), dim3(kB), 0, s, n, ld, a, af);
  return hipGetLastError();
}

hipError_t launch_amg_coarse_apply_f32(int n, int ld, const float *ainv, const double *b,
                                       double *x, hipStream_t s) {
  if (n > kAmgMaxDense || ld % 4 || ld < n || ld > kAmgMaxDense + 4) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_coarse_apply_f32, dim3((n + kCaWaves - 1) / kCaWaves), dim3(64 * kCaWaves),
                     0, s, n, ld, ainv, b, x);
  return hipGetLastError();
}

hipError_t launch_amg_coarse_apply(int n, const double *ainv, const double *b, double *x,
                                   hipStream_t s) {
  if (n > kAmgMaxDense) return hipErrorInvalidValue;
  const dim3 g((n + kCaWaves - 1) / kCaWaves), blk(64 * kCaWaves);
  if (n % 2 == 0)
    hipLaunchKernelGGL(k_coarse_apply<1>, g, blk, 0, s, n, ainv, b, x);
  else
    hipLaunchKernelGGL(k_coarse_apply<0>, g, blk, 0, s, n, ainv, b, x);
  return hipGetLastError();
}

hipError_t launch_amg_post(int nf, int nb, const int *rp, const int *col, const double *v,
                           const float *vf, const int *agg, const double *x, const double *e,
                           const double *b, const double *dinv, double omega, double *out,
                           hipStream_t s) {
  if (nb == 0) return hipSuccess;
  auto go = [&](auto corr, auto vt, const auto *vv) -> hipError_t {
    constexpr int CORR = decltype(corr)::value;
    using VT = decltype(vt);
    AMG_NF_DISPATCH(nf, hipLaunchKernelGGL((k_post<NFc, kLpr, CORR, VT>),
                                           g1((long long)nb * kLpr), dim3(kB), 0, s, nb, rp, col,
                                           vv, agg, x, e, b, dinv, omega, out));
    return hipGetLastError();
  };
  if (e && vf) return go(std::integral_constant<int, 1>(), float(), vf);
  if (e) return go(std::integral_constant<int, 1>(), double(), v);
  if (vf) return go(std::integral_constant<int, 0>(), float(), vf);
  return go(std::integral_constant<int, 0>(), double(), v);
}

hipError_t launch_amg_prolong0(int nf, int n, const int *agg, const double *x0, const double *e1,
                               double *y, hipStream_t s) {
  if (n == 0) return hipSuccess;
  AMG_NF_DISPATCH(nf, hipLaunchKernelGGL((k_prolong0<NFc>), g1(n), dim3(kB), 0, s, n, agg, x0, e1,
                                          y));
  return hipGetLastError();
}

}  // namespace pnp
