// Sparse linear algebra of the BiCGSTAB path on gfx950 (replaces ISTL BCRSMatrix::mv,
// BiCGSTABSolver's BLAS-1 and dots, SeqSSOR).
//
// * SpMV: SELL-64, one thread per vertex row, lanes = 64 consecutive rows, so every column-index
//   and value load of a slot is one coalesced 256/512-byte line; x is gathered as NF contiguous
//   doubles per neighbour vertex (L2 / Infinity-Cache resident for Morton-ordered rows).  Dots
//   that BiCGSTAB needs right after a SpMV are fused into its epilogue.
// * Reductions are deterministic: per-block partials in a fixed grid, summed by one block in a
//   fixed order; the BiCGSTAB scalars (rho, alpha, omega, norms, half-step counter, convergence
//   and breakdown flags) never leave the device, so the host only polls for termination.
// * SSOR(k=1, w=1) = one multicolour symmetric Gauss-Seidel sweep: rows of one colour have no
//   coupling among themselves, so each colour is one fully parallel launch (forward: colours
//   ascending, backward: descending); couplings to ghost rows are dropped (block-Jacobi across
//   GPUs, like the reference's non-overlapping SSOR on the local matrix).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include <type_traits>

#include <hip/hip_ext.h>

#include "kernels.h"

// split sweeps: issue a batch's L/U value loads with its column-index loads (1) or after them (0)
#ifndef SPLIT_VALS_EARLY
#define SPLIT_VALS_EARLY 1
#endif

namespace pnp {

namespace {

constexpr int kBlock = 256;
constexpr double kEps = 1e-80;  // ISTL BiCGSTABSolver EPSILON

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum of K values, result written by thread 0 to out[0..K)
template <int K, int NT = kBlock>
__device__ __forceinline__ void block_sum(double (&v)[K], double *out) {
  __shared__ double sh[NT / 64][K > 0 ? K : 1];
  const int w = threadIdx.x / 64, l = threadIdx.x % 64;
#pragma unroll
  for (int k = 0; k < K; k++) {
    double s = wave_sum(v[k]);
    if (l == 0) sh[w][k] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < K; k++) {
      double s = 0;
      for (int i = 0; i < NT / 64; i++) s += sh[i][k];
      out[k] = s;
    }
  }
}

// ------------------------------------------------------------------------------------------
// SpMV (+ fused dots)
// ------------------------------------------------------------------------------------------
template <int NF, int PAT, int MODE, int SB, int LPR, int NT = 0>
__global__ __launch_bounds__(kBlock) void k_spmv(DevLayout L, const double *__restrict__ vals,
                                                 const double *__restrict__ x,
                                                 double *__restrict__ y,
                                                 const double *__restrict__ w,
                                                 double *__restrict__ partials,
                                                 const double *__restrict__ w2) {
  constexpr int NV = popc9(PAT), NK = nks_of(PAT);
  // LPR lanes per row (slots interleaved): block b covers part b % LPR of the 256-row group the
  // spatial block map gives b / LPR
  int row, q;
  if constexpr (LPR == 1) {
    row = row_block(L, blockIdx.x, gridDim.x) * kBlock + threadIdx.x;
    q = 0;
  } else {
    row = row_block(L, blockIdx.x / LPR, gridDim.x / LPR) * kBlock +
          (blockIdx.x % LPR) * (kBlock / LPR) + threadIdx.x / LPR;
    q = threadIdx.x % LPR;
  }
  const bool live = row < L.n_owned;
  double d[3] = {0, 0, 0};
  double acc[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] = 0;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = live ? L.chunk_off[chunk] : 0, len = live ? L.chunk_len[chunk] : 0;
  const int *__restrict__ cix = L.colidx + off + lane;
  const double *__restrict__ vc = vals + size_t(off) * NK;  // chunk base (k-form), see vin()
  // slots in batches of SB: their column indices, then their gathers and values, are issued
  // together (memory-level parallelism inside the thread); lane q takes slots q, q+LPR, ...
  for (int s0 = q; s0 < len; s0 += SB * LPR) {
    int j[SB];
#pragma unroll
    for (int b = 0; b < SB; b++) {
      const int sl = s0 + b * LPR;
      j[b] = sl < len ? cix[sl * kRows] : row;  // (non-temporal here: slower, reused)
    }
    double xj[SB][NF], k[SB][NK];
#pragma unroll
    for (int b = 0; b < SB; b++) {
      const int sl = s0 + b * LPR;
      load_nf<NF>(x, size_t(j[b]), xj[b]);
      if (sl < len) {
        if (NT)
          load_vals_nt<NK>(vc + size_t(sl) * NK * kRows, lane, k[b]);
        else
          load_vals<NK>(vc + size_t(sl) * NK * kRows, lane, k[b]);
      } else {
#pragma unroll
        for (int qq = 0; qq < NK; qq++) k[b][qq] = 0.0;
      }
    }
#pragma unroll
    for (int b = 0; b < SB; b++) {
      double a[NV];
      expand_k<PAT>(k[b], a);
#pragma unroll
      for (int f = 0; f < NF; f++)
#pragma unroll
        for (int g = 0; g < NF; g++) {
          const int v = pat_index(PAT, f, g);
          if (v >= 0) acc[f] += a[v] * xj[b][g];
        }
    }
  }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1)
#pragma unroll
    for (int f = 0; f < NF; f++) acc[f] += __shfl_xor(acc[f], o, 64);
  if (live && q == 0) {
    const unsigned dm = row_mask<NF>(L, row);  // Dirichlet rows are identity rows
    if (dm) {
      double xr[NF];
      load_nf<NF>(x, size_t(row), xr);
#pragma unroll
      for (int f = 0; f < NF; f++)
        if ((dm >> f) & 1) acc[f] = xr[f];
    }
    if constexpr (MODE == 3) {  // residual: y = w - A x
      double wr[NF];
      load_nf<NF>(w, size_t(row), wr);
#pragma unroll
      for (int f = 0; f < NF; f++) acc[f] = wr[f] - acc[f];
    }
    store_nf<NF>(y, size_t(row), acc);
    if constexpr (MODE == 1 || MODE == 2 || MODE == 4) {
      double wr[NF];
      load_nf<NF>(w, size_t(row), wr);
#pragma unroll
      for (int f = 0; f < NF; f++) d[0] += acc[f] * wr[f];
    }
    if constexpr (MODE == 2 || MODE == 4) {
#pragma unroll
      for (int f = 0; f < NF; f++) d[1] += acc[f] * acc[f];
    }
    if constexpr (MODE == 4) {
      double wr[NF];
      load_nf<NF>(w2, size_t(row), wr);
#pragma unroll
      for (int f = 0; f < NF; f++) d[2] += acc[f] * wr[f];
    }
  }
  if constexpr (MODE == 1) {
    double v1[1] = {d[0]};
    block_sum<1>(v1, partials + blockIdx.x);
  } else if constexpr (MODE == 2) {
    double v2[2] = {d[0], d[1]};
    block_sum<2>(v2, partials + 2 * blockIdx.x);
  } else if constexpr (MODE == 4) {
    double v3[3] = {d[0], d[1], d[2]};
    block_sum<3>(v3, partials + 3 * blockIdx.x);
  }
}

// The SpMV with the x gathers staged through LDS (PNP_SPMV_LDS): a workgroup first loads x at the
// distinct columns of its 256 rows (config 3: 1,016 per block against 1,796 slots, so half the
// scattered gathers), then every slot reads its x record from LDS by a 16-bit list position.
// One lane per row, slots in pairs.  The arithmetic order is that of the default k_spmv<.., 2, 2>
// (two lanes per row, even / odd slots, combined at the end; dot partials per 128 rows with the
// same trees), so results and partials are bitwise those of k_spmv: the BiCGSTAB iterates and
// iteration counts do not move (they are sensitive to the last bit on the pore system).
#ifndef SPMV_SU
#define SPMV_SU 4  // staged list entries per thread issued together (build-flag A/B knob)
#endif
#ifndef SPMV_OWN_DIRECT
#define SPMV_OWN_DIRECT 1
#endif
template <int NF, int PAT, int MODE, int SB, int NT>
__global__ __launch_bounds__(kBlock) void k_spmv_lds(DevLayout L, const double *__restrict__ vals,
                                                     const double *__restrict__ x,
                                                     double *__restrict__ y,
                                                     const double *__restrict__ w,
                                                     double *__restrict__ partials,
                                                     const double *__restrict__ w2) {
  constexpr int NV = popc9(PAT), NK = nks_of(PAT);
  extern __shared__ double sx[];  // [cnt][NF]
  const int blk = row_block(L, blockIdx.x, gridDim.x);
  const int row = blk * kBlock + threadIdx.x;
  const bool live = row < L.n_owned;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = live ? L.chunk_off[chunk] : 0, len = live ? L.chunk_len[chunk] : 0;
  // SPMV_OWN_DIRECT (default): the entries past uown[blk] -- columns that are only a row's own
  // slot 0 (and its padding slots) -- are not staged; a slot whose column is the row itself takes
  // x[row] from a direct, coalesced load instead (the same value, so bitwise the staged form)
  const int u0 = L.uptr[blk];
  const int cnt = (SPMV_OWN_DIRECT && L.uown) ? L.uown[blk] : L.uptr[blk + 1] - u0;
  const uint16_t *__restrict__ lix = L.lidx + off + lane;
  const double *__restrict__ vc = vals + size_t(off) * NK;
  double xo[NF];
  int lown = -1;
  if (SPMV_OWN_DIRECT && L.uown && live) {
    load_nf<NF>(x, size_t(row), xo);
    lown = lix[0];
  }
  // one slot pair's list positions and values (issuing the first pair before the staging barrier
  // was measured: config 5 BiCGSTAB +2.5 %, profiles/r03/ab_spmv_staging.log)
  auto fetch = [&](int s0, int (&li)[SB], double (&k)[SB][NK]) {
#pragma unroll
    for (int b = 0; b < SB; b++) {
      const int sl = s0 + b;
      li[b] = sl < len ? lix[sl * kRows] : 0;
      if (sl < len) {
        if (NT)
          load_vals_nt<NK>(vc + size_t(sl) * NK * kRows, lane, k[b]);
        else
          load_vals<NK>(vc + size_t(sl) * NK * kRows, lane, k[b]);
      } else {
#pragma unroll
        for (int qq = 0; qq < NK; qq++) k[b][qq] = 0.0;
      }
    }
  };
  {  // up to SPMV_SU list entries per thread: list loads, then gathers, then LDS stores
    int jj[SPMV_SU];
#pragma unroll
    for (int u = 0; u < SPMV_SU; u++) {
      const int k = int(threadIdx.x) + u * kBlock;
      jj[u] = k < cnt ? L.ulist[u0 + k] : -1;
    }
    double t[SPMV_SU][NF];
#pragma unroll
    for (int u = 0; u < SPMV_SU; u++)
      if (jj[u] >= 0) load_nf<NF>(x, size_t(jj[u]), t[u]);
#pragma unroll
    for (int u = 0; u < SPMV_SU; u++) {
      const int k = int(threadIdx.x) + u * kBlock;
      if (jj[u] >= 0)
#pragma unroll
        for (int f = 0; f < NF; f++) sx[k * NF + f] = t[u][f];
    }
  }
  for (int k = int(threadIdx.x) + SPMV_SU * kBlock; k < cnt; k += kBlock) {  // longer lists
    double t[NF];
    load_nf<NF>(x, size_t(L.ulist[u0 + k]), t);
#pragma unroll
    for (int f = 0; f < NF; f++) sx[k * NF + f] = t[f];
  }
  __syncthreads();
  static_assert(SB == 2, "slot pairs: even slots into acc2[0], odd into acc2[1]");
  double d[3] = {0, 0, 0};
  double acc2[2][NF];
#pragma unroll
  for (int f = 0; f < NF; f++) acc2[0][f] = acc2[1][f] = 0;
  for (int s0 = 0; s0 < len; s0 += SB) {
    int li[SB];
    double k[SB][NK];
    fetch(s0, li, k);
#pragma unroll
    for (int b = 0; b < SB; b++) {
      double a[NV], xj[NF];
      const bool me = SPMV_OWN_DIRECT && li[b] == lown;
      const int lj = me ? 0 : li[b];
#pragma unroll
      for (int g = 0; g < NF; g++) {
        const double t = sx[lj * NF + g];
        xj[g] = me ? xo[g] : t;
      }
      expand_k<PAT>(k[b], a);
#pragma unroll
      for (int f = 0; f < NF; f++)
#pragma unroll
        for (int g = 0; g < NF; g++) {
          const int v = pat_index(PAT, f, g);
          if (v >= 0) acc2[b][f] += a[v] * xj[g];
        }
    }
  }
  double acc[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] = acc2[0][f] + acc2[1][f];
  if (live) {
    const unsigned dm = row_mask<NF>(L, row);  // Dirichlet rows are identity rows
    if (dm) {
      double xr[NF];
      load_nf<NF>(x, size_t(row), xr);
#pragma unroll
      for (int f = 0; f < NF; f++)
        if ((dm >> f) & 1) acc[f] = xr[f];
    }
    if constexpr (MODE == 3) {  // residual: y = w - A x
      double wr[NF];
      load_nf<NF>(w, size_t(row), wr);
#pragma unroll
      for (int f = 0; f < NF; f++) acc[f] = wr[f] - acc[f];
    }
    store_nf<NF>(y, size_t(row), acc);
    if constexpr (MODE == 1 || MODE == 2 || MODE == 4) {
      double wr[NF];
      load_nf<NF>(w, size_t(row), wr);
#pragma unroll
      for (int f = 0; f < NF; f++) d[0] += acc[f] * wr[f];
    }
    if constexpr (MODE == 2 || MODE == 4) {
#pragma unroll
      for (int f = 0; f < NF; f++) d[1] += acc[f] * acc[f];
    }
    if constexpr (MODE == 4) {
      double wr[NF];
      load_nf<NF>(w2, size_t(row), wr);
#pragma unroll
      for (int f = 0; f < NF; f++) d[2] += acc[f] * wr[f];
    }
  }
  if constexpr (MODE == 1 || MODE == 2 || MODE == 4) {
    // the trees of k_spmv<.., 2, 2>'s block_sum: per 32 rows xor 16, 8, 4, 2, 1, then per 128
    // rows the four 32-row sums in order -> two partials per 256-row workgroup
    constexpr int K = MODE == 1 ? 1 : (MODE == 2 ? 2 : 3);
    __shared__ double sh[8][K];
#pragma unroll
    for (int kk = 0; kk < K; kk++) {
      double v = d[kk];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if ((threadIdx.x & 31) == 0) sh[threadIdx.x >> 5][kk] = v;
    }
    __syncthreads();
    if (threadIdx.x < 2) {
      const int h = threadIdx.x;
#pragma unroll
      for (int kk = 0; kk < K; kk++) {
        double t = 0;
        for (int i = 0; i < 4; i++) t += sh[4 * h + i][kk];
        partials[size_t(K) * (2 * blockIdx.x + h) + kk] = t;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// preconditioners
// ------------------------------------------------------------------------------------------
template <int NF, int PAT>
__global__ __launch_bounds__(kBlock) void k_jacobi(DevLayout L, const double *__restrict__ vals,
                                                   const double *__restrict__ d,
                                                   double *__restrict__ v) {
  constexpr int NV = popc9(PAT), NK = nks_of(PAT);
  const int row = blockIdx.x * kBlock + threadIdx.x;
  if (row >= L.n_owned) return;
  const int chunk = row / kRows, lane = row % kRows;
  double K[NK], D[NV];
  load_vals<NK>(vals + size_t(L.chunk_off[chunk]) * NK, lane, K);
  expand_k<PAT>(K, D);
  mask_rows<NF, PAT>(D, row_mask<NF>(L, row), true);
#pragma unroll
  for (int f = 0; f < NF; f++) v[size_t(row) * NF + f] = d[size_t(row) * NF + f] / D[pat_index(PAT, f, f)];
}

// one colour of a Gauss-Seidel sweep: v_i += D_i^{-1} (d_i - sum_j A_ij v_j), rows of the
// colour in parallel (they are never adjacent), the NF fields of a row in sequence (ascending
// forward, descending backward).  The forward sweep starts from v = 0 (ISTL SeqSSOR applies to y = 0): rows of
// later colours are still zero and are skipped, the row's own value is not read.
// Row setup shared by the split sweeps: the row's slots in the L (FWD) or U (!FWD) storage.
// Value type of the split storage: double, or float for the ILU(0) factors when the context
// stores them in single precision (PNP_ILU_F32; the arithmetic stays fp64).  float slots hold NVP
// = NV rounded up to 4 values per row, quad-interleaved (one dwordx4 per lane moves 4 values):
// value q of lane l at (q >> 2) * 4 * kRows + 4 l + (q & 3); NV == 1 is row-contiguous.
// ILU_F32_PACK (default): NV values exactly, the full quads as above and the last NV % 4 values
// as one record of that many floats per lane (NV = 7: a dwordx4 and a dwordx3 per lane, 28 B per
// block instead of 32)
#ifndef ILU_F32_PACK
#define ILU_F32_PACK 1
#endif
template <int NV>
__host__ __device__ constexpr int nvp_f() {
  return NV == 1 ? 1 : ILU_F32_PACK ? NV : ((NV + 3) & ~3);
}
// ILU_F32_LOWTAIL (default, packed NV = 7 only): values 3 and 4 trade places in storage, so that
// the remainder record holds (1,0), (2,0) and (2,2) of the PNP pattern: the strictly lower entries
// of a diagonal block, all a forward step needs of it (one dwordx3 instead of 28 B)
#ifndef ILU_F32_LOWTAIL
#define ILU_F32_LOWTAIL 1
#endif
__host__ __device__ constexpr int fperm(int nv, int q) {
  return (ILU_F32_PACK && ILU_F32_LOWTAIL && nv == 7 && (q == 3 || q == 4)) ? 7 - q : q;
}
__host__ __device__ constexpr int vinf(int nv, int q0, int lane) {
  if (nv == 1) return lane;
  const int q = fperm(nv, q0);
  const int nq = ILU_F32_PACK ? (nv >> 2) : ((nv + 3) >> 2), rem = nv - 4 * nq;
  return q < 4 * nq ? (q >> 2) * 4 * kRows + 4 * lane + (q & 3)
                    : 4 * nq * kRows + rem * lane + (q - 4 * nq);
}
// the values of a float slot-lane (quad-interleaved as vinf) into B[0 .. NV) as doubles
// LOWER: only what a forward step reads of a diagonal block (the remainder record when it holds
// all strictly lower entries, see fperm; the other values are zero then)
template <int NV, int NT, typename T = double, int LOWER = 0>
__device__ __forceinline__ void load_f32_slot(const float *__restrict__ sb, int lane, T *B) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef float f2v __attribute__((ext_vector_type(2)));
  constexpr int NQ = ILU_F32_PACK ? (NV >> 2) : ((NV + 3) >> 2), REM = ILU_F32_PACK ? NV - 4 * NQ : 0;
  constexpr bool TAIL = LOWER && fperm(NV, 3) != 3;  // the remainder holds the lower entries
#pragma unroll
  for (int k = 0; k < NQ; k++) {
    if (TAIL) {
#pragma unroll
      for (int i = 0; i < 4; i++) B[fperm(NV, 4 * k + i)] = T(0);
      continue;
    }
    const f4v *pp = reinterpret_cast<const f4v *>(sb + k * 4 * kRows) + lane;
    const f4v t = NT ? __builtin_nontemporal_load(pp) : *pp;
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (4 * k + i < NV) B[fperm(NV, 4 * k + i)] = T(t[i]);
  }
  const float *pr = sb + NQ * 4 * kRows + REM * lane;
  if constexpr (REM == 2) {
    const f2v t = NT ? __builtin_nontemporal_load(reinterpret_cast<const f2v *>(pr))
                     : *reinterpret_cast<const f2v *>(pr);
    B[fperm(NV, 4 * NQ)] = T(t[0]);
    B[fperm(NV, 4 * NQ + 1)] = T(t[1]);
  } else if constexpr (REM != 0) {
#pragma unroll
    for (int i = 0; i < REM; i++)
      B[fperm(NV, 4 * NQ + i)] = T(NT ? __builtin_nontemporal_load(pr + i) : pr[i]);
  }
}
// bfloat16 factor storage (PNP_OPT_ILU_F32 = 2): the f32 factors rounded to 8 significant bits
// (nearest even), fp64 arithmetic as before.  Slots of NV > 1 values hold NV rounded up to 8
// shorts per lane, so one dwordx4 per lane moves a PNP block (16 B instead of 28): value q of
// lane l at (q >> 3) * 8 * kRows + 8 l + (q & 7); NV == 1 is row-contiguous (2 B per row).
// ILU_BF16_B7 (default): the 7-value stationary PNP block in 14 B instead of 16 -- six shorts per
// lane (one dwordx3) then one short per lane (a 128-B plane) -- with the two strictly lower
// values of the pattern, (1,0) and (2,0), in the dwordx3's last dword: a forward step reads only
// that dword of a diagonal block (4 B instead of 16).  Same values, same arithmetic: bitwise the
// 16-B layout's results.
// Measured first with f32 storage rounded to 8 / 11 bits (ILU_ROUND_BITS): the config-3 PNP
// Newton's BiCGSTAB count stays inside its last-bit spread.
#ifndef ILU_BF16_B7
#define ILU_BF16_B7 1
#endif
typedef unsigned short bf16s;
__host__ __device__ constexpr bool b7(int nv) { return ILU_BF16_B7 && nv == 7; }
__host__ __device__ constexpr int nvp_b(int nv) { return nv == 1 ? 1 : b7(nv) ? 7 : ((nv + 7) & ~7); }
// b7 position of value q: (0,0) (0,1) (0,2) (1,1) | (1,0) (2,0) in the third dword | (2,2) apart
__host__ __device__ constexpr int bperm7(int q) {
  return q == 3 ? 4 : q == 4 ? 3 : q;  // q 5 -> 5, q 6 -> 6
}
__host__ __device__ constexpr int vinb(int nv, int q, int lane) {
  return nv == 1 ? lane
         : b7(nv) ? (bperm7(q) < 6 ? 6 * lane + bperm7(q) : 6 * kRows + lane)
                  : (q >> 3) * 8 * kRows + 8 * lane + (q & 7);
}
__device__ __forceinline__ bf16s to_bf16(float x) {
  unsigned u = __float_as_uint(x);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return bf16s(u >> 16);
}
__device__ __forceinline__ float from_bf16(unsigned h) { return __uint_as_float(h << 16); }
// LOWER (b7 only): just the dword of the two strictly lower values, the others zero
template <int NV, int NT, typename T = double, int LOWER = 0>
__device__ __forceinline__ void load_bf16_slot(const bf16s *__restrict__ sb, int lane, T *B) {
  if constexpr (NV == 1) {
    B[0] = T(from_bf16(NT ? __builtin_nontemporal_load(sb + lane) : sb[lane]));
  } else if constexpr (b7(NV)) {
    const unsigned *pw = reinterpret_cast<const unsigned *>(sb) + 3 * lane;
    auto lo = [](unsigned w) { return from_bf16(w & 0xFFFFu); };
    auto hi = [](unsigned w) { return from_bf16(w >> 16); };
    if constexpr (LOWER) {
      const unsigned w2 = NT ? __builtin_nontemporal_load(pw + 2) : pw[2];
#pragma unroll
      for (int q = 0; q < 7; q++) B[q] = T(0);
      B[3] = T(lo(w2));
      B[5] = T(hi(w2));
    } else {
      typedef unsigned u3v __attribute__((ext_vector_type(3)));
      const u3v t = NT ? __builtin_nontemporal_load(reinterpret_cast<const u3v *>(pw))
                       : *reinterpret_cast<const u3v *>(pw);
      const unsigned short t6 = NT ? __builtin_nontemporal_load(sb + 6 * kRows + lane)
                                   : sb[6 * kRows + lane];
      B[0] = T(lo(t[0]));
      B[1] = T(hi(t[0]));
      B[2] = T(lo(t[1]));
      B[4] = T(hi(t[1]));  // position 3
      B[3] = T(lo(t[2]));  // position 4
      B[5] = T(hi(t[2]));
      B[6] = T(from_bf16(t6));
    }
  } else {
    typedef unsigned u4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int k = 0; k < (NV + 7) / 8; k++) {
      const u4v *pp = reinterpret_cast<const u4v *>(sb + k * 8 * kRows) + lane;
      const u4v t = NT ? __builtin_nontemporal_load(pp) : *pp;
#pragma unroll
      for (int i = 0; i < 8; i++)
        if (8 * k + i < NV) B[8 * k + i] = T(from_bf16((i & 1) ? (t[i >> 1] >> 16) : (t[i >> 1] & 0xFFFFu)));
    }
  }
}

template <int NV, typename VT>
__host__ __device__ constexpr int slot_vals() {
  return std::is_same<VT, float>::value ? nvp_f<NV>()
                                        : (std::is_same<VT, bf16s>::value ? nvp_b(NV) : NV);
}
// the value type a slot's values are kept in between their load and their use
template <typename VT>
using slot_keep_t = typename std::conditional<std::is_same<VT, bf16s>::value, float, VT>::type;

template <int NV, int NT, typename VT, int LOWER = 0>
__device__ __forceinline__ void load_split_vals(const VT *__restrict__ sb, int lane, double *B) {
  if constexpr (std::is_same<VT, double>::value) {
    if (NT)
      load_vals_nt<NV>(sb, lane, B);
    else
      load_vals<NV>(sb, lane, B);
  } else if constexpr (std::is_same<VT, bf16s>::value) {
    load_bf16_slot<NV, NT, double, LOWER>(sb, lane, B);
  } else if constexpr (NV == 1) {
    B[0] = NT ? __builtin_nontemporal_load(sb + lane) : sb[lane];
  } else {
    load_f32_slot<NV, NT, double, LOWER>(sb, lane, B);
  }
}

// Row setup shared by the split sweeps: the slots of split position pos in the L (FWD) or U (!FWD)
// storage, the row stored there (DevLayout lperm / uperm) and the lane of its diagonal block
template <typename VT>
struct SplitRow {
  const int *cix;
  const VT *vc;  // chunk base of the L or U values: slot s at vc + s * slot_vals * kRows
  const VT *dg;  // U chunk base: slot 0 = diagonal block
  int len, lane, dlane, row;
};

template <int NV, int FWD, typename VT = double>
__device__ __forceinline__ SplitRow<VT> split_row(const DevLayout &L, const VT *lv, const VT *uv,
                                                  int pos, bool live) {
  constexpr int NS = slot_vals<NV, VT>();
  const int chunk = pos / kRows, lane = pos % kRows;
  const int uoff = L.uchunk_off[chunk];
  SplitRow<VT> r;
  r.lane = lane;
  r.row = L.lperm ? chunk * kRows + int(FWD ? L.lperm[pos] : L.uperm[pos]) : pos;
  r.dlane = (FWD && L.ldl) ? int(L.ldl[pos]) : lane;
  r.dg = uv + size_t(uoff) * NS;
  if (FWD) {
    const int off = L.lchunk_off[chunk];
    r.cix = L.lcolidx + off + lane;
    r.vc = lv + size_t(off) * NS;
    r.len = live ? (L.llen ? int(L.llen[pos]) : L.lchunk_len[chunk]) : 0;
  } else {
    r.cix = L.ucolidx + uoff + lane;
    r.vc = r.dg;
    r.len = live ? (L.ulen ? int(L.ulen[pos]) : L.uchunk_len[chunk]) : 0;
  }
  return r;
}

// acc[f] -= sum over the row's slots [s0, len) of A_(f,g) v_j[g]; LPR lanes per row (adjacent
// lanes, slots interleaved), partial sums combined across the row's lanes.  A colour holds ~1/6
// of the rows (~2 waves per SIMD at config 3), so latency is hidden inside the thread: the
// column indices of B slots are loaded together, then their gathers and values together.
template <int NF, int PAT, int LPR, int B, int NT = 0, typename VT = double, typename XT = double>
__device__ __forceinline__ void split_row_dot(const SplitRow<VT> &R, int s0, int q, int row,
                                              const XT *__restrict__ v, double (&acc)[NF]) {
  constexpr int NV = popc9(PAT), NS = slot_vals<NV, VT>();
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] = 0.0;
  for (int sb = s0 + q; sb < R.len; sb += B * LPR) {
    int j[B];
#pragma unroll
    for (int b = 0; b < B; b++) {
      const int s = sb + b * LPR;
      j[b] = s < R.len ? R.cix[s * kRows] : row;  // (non-temporal here: slower, reused)
    }
    double vj[B][NF], a[B][NV];
    // values first: they depend on the slot count only, so they are in flight with the column
    // indices instead of waiting for them (padding slots are zeroed after the loads)
#pragma unroll
    for (int b = 0; b < B; b++) {
      const int s = sb + b * LPR;
      if (SPLIT_VALS_EARLY && s < R.len) {
        load_split_vals<NV, NT>(R.vc + size_t(s) * NS * kRows, R.lane, a[b]);
      } else {
#pragma unroll
        for (int qq = 0; qq < NV; qq++) a[b][qq] = 0.0;
      }
    }
#pragma unroll
    for (int b = 0; b < B; b++) {
      const int s = sb + b * LPR;
      const bool use = j[b] != row;  // padding: zero values, v[row] may be stale
      load_nf<NF>(v, size_t(use ? j[b] : row), vj[b]);
      if (!use) {
#pragma unroll
        for (int g = 0; g < NF; g++) vj[b][g] = 0.0;
      }
      if (!SPLIT_VALS_EARLY && use) load_split_vals<NV, NT>(R.vc + size_t(s) * NS * kRows, R.lane, a[b]);
      if (SPLIT_VALS_EARLY && !use) {
#pragma unroll
        for (int qq = 0; qq < NV; qq++) a[b][qq] = 0.0;
      }
    }
#pragma unroll
    for (int b = 0; b < B; b++)
#pragma unroll
      for (int f = 0; f < NF; f++)
#pragma unroll
        for (int g = 0; g < NF; g++) {
          const int qq = pat_index(PAT, f, g);
          if (qq >= 0) acc[f] -= a[b][qq] * vj[b][g];
        }
  }
#pragma unroll
  for (int o = 1; o < LPR; o <<= 1)
#pragma unroll
    for (int f = 0; f < NF; f++) acc[f] += __shfl_xor(acc[f], o, 64);
}

// one colour of a symmetric Gauss-Seidel sweep (ISTL SeqSSOR, w = 1, from v = 0), rows of the
// colour in parallel (never adjacent), the NF fields of a row in sequence (ascending forward,
// descending backward).  Forward: t_i = d_i - sum_{j lower} A_ij v_j, then the block-lower
// solve; backward: v_i += D_i^{-1}(t_i - sum_{j upper} A_ij v_j - D_i v_i), field by field.
// KIND 1 forward, 0 backward, 2 both for the last colour (no upper neighbours: its backward
// step is pointwise, t stays in registers).
template <int NF, int PAT, int KIND, int LPR, int B, int NT>
__global__ __launch_bounds__(kBlock) void k_sgs_color(DevLayout L, int k0, int nk,
                                                      const double *__restrict__ lv,
                                                      const double *__restrict__ uv,
                                                      const double *__restrict__ d,
                                                      double *__restrict__ v,
                                                      double *__restrict__ t) {
  constexpr int NV = popc9(PAT);
  constexpr bool FWD = KIND != 0;
  // XCD remap pays here (+5 % measured): a colour's rows are a contiguous range
  const int gt = xcd_block(blockIdx.x, gridDim.x, 1) * kBlock + threadIdx.x;
  const int k = gt / LPR, q = gt % LPR;
  const bool live = k < nk;
  // colour-major order: the colour's rows are the split positions [k0, k0+nk)
  const SplitRow<double> R = split_row<NV, FWD>(L, lv, uv, k0 + (live ? k : 0), live);
  const int row = R.row;
  // the row's own data and diagonal block do not depend on the neighbours: issued before the
  // neighbour loop so that they share its memory round trips (after the loop they cost one more)
  double rhs[NF], vi[NF], Dg[NV];
  load_nf<NF>(FWD ? d : t, size_t(row), rhs);
  if (!FWD) load_nf<NF>(v, size_t(row), vi);
  load_vals<NV>(R.dg, R.dlane, Dg);
  double acc[NF];
  split_row_dot<NF, PAT, LPR, B, NT>(R, FWD ? 0 : 1, q, row, v, acc);
  if (!live || q != 0) return;
  if (FWD) {
#pragma unroll
    for (int f = 0; f < NF; f++) {
      rhs[f] += acc[f];
      vi[f] = 0.0;
    }
    if (KIND == 1) store_nf<NF>(t, size_t(row), rhs);
  } else {
#pragma unroll
    for (int f = 0; f < NF; f++) rhs[f] += acc[f];
  }
#pragma unroll
  for (int pass = 0; pass < (KIND == 2 ? 2 : 1); pass++)
#pragma unroll
    for (int ff = 0; ff < NF; ff++) {
      const bool up = KIND == 0 || pass == 1;
      const int f = up ? NF - 1 - ff : ff;
      double r = rhs[f];
#pragma unroll
      for (int g = 0; g < NF; g++) {
        const int qq = pat_index(PAT, f, g);
        if (qq >= 0) r -= Dg[qq] * vi[g];
      }
      vi[f] += r / Dg[pat_index(PAT, f, f)];
    }
  store_nf<NF>(v, size_t(row), vi);
}

// ------------------------------------------------------------------------------------------
// multicolour ILU(0)
// ------------------------------------------------------------------------------------------
// Elimination order = colour-major vertex order (the storage order), fields ascending inside a
// vertex; the pattern is the stored block pattern (ISTL bilu0 / SeqILU0 on this ordering).
// Rows of one colour never couple, so each colour is one parallel launch: the rows it needs
// (lower neighbours) were factorised by earlier launches.  Entry (f,g) of slot t of row i is
// lu[(off_c + 64 t) * NV + 64 pat(f,g) + lane].
// Same-colour couplings (mesh.cc absorb_top: a thin top colour merged into the colours below) are
// outside the sweeps' pattern: the split storage has no slot for them and the factorisation
// neither eliminates by them nor updates into them
__device__ __forceinline__ bool same_color(const DevLayout &L, int a, int b) {
  return L.rowcolor[a] == L.rowcolor[b];
}
__device__ __forceinline__ bool dropped(const DevLayout &L, int row, int col) {
  return col != row && col < L.n_owned && same_color(L, row, col);
}

template <int NF, int PAT>
__global__ __launch_bounds__(kBlock) void k_ilu0_factor(DevLayout L, int r0, int r1,
                                                        double *__restrict__ lu) {
  constexpr int NV = popc9(PAT);
  const int row = r0 + xcd_block(blockIdx.x, gridDim.x, 1) * kBlock + threadIdx.x;
  if (row >= r1) return;
  const int ci = row / kRows, li = row % kRows;
  const int offi = L.chunk_off[ci], leni = int(L.rowmeta[row] & 63);
  const int *__restrict__ cixi = L.colidx + offi + li;
  double *__restrict__ vi = lu + size_t(offi) * NV;  // chunk base, see vin()
  auto A = [&](int t, int f, int g) -> double & {
    return vi[size_t(t) * NV * kRows + vin(NV, pat_index(PAT, f, g), li)];
  };
  // 1) eliminate by the lower neighbours j in increasing index order
  int prev = -1;
  for (;;) {
    int j = 0x7fffffff, s = -1;
    for (int t = 1; t < leni; t++) {
      const int c = cixi[t * kRows];
      if (c < row && c > prev && c < j && !same_color(L, c, row)) {
        j = c;
        s = t;
      }
    }
    if (s < 0) break;
    prev = j;
    const int cj = j / kRows, lj = j % kRows;
    const int offj = L.chunk_off[cj], lenj = int(L.rowmeta[j] & 63);
    const int *__restrict__ cixj = L.colidx + offj + lj;
    const double *__restrict__ vj = lu + size_t(offj) * NV;
    auto U = [&](int t, int g, int h) -> double {
      return vj[size_t(t) * NV * kRows + vin(NV, pat_index(PAT, g, h), lj)];
    };
    for (int g = 0; g < NF; g++) {
      const double dinv = U(0, g, g);  // stored inverted
      for (int f = 0; f < NF; f++) {
        if (pat_index(PAT, f, g) < 0) continue;
        const double l = A(s, f, g) * dinv;
        A(s, f, g) = l;
        if (l == 0.0) continue;
        // q = (j, h > g): block (i, j), slot s of row i, diagonal block of row j
        for (int h = g + 1; h < NF; h++)
          if (pat_index(PAT, f, h) >= 0 && pat_index(PAT, g, h) >= 0)
            A(s, f, h) -= l * U(0, g, h);
        // q = (m, h), m > j, m owned, in both rows (m = i included)
        for (int t = 0; t < leni; t++) {
          const int m = cixi[t * kRows];
          if (m <= j || m >= L.n_owned || (t > 0 && m == row)) continue;  // padding -> m == row
          if (dropped(L, row, m) || dropped(L, j, m)) continue;
          for (int u = 1; u < lenj; u++) {
            if (cixj[u * kRows] != m) continue;
            for (int h = 0; h < NF; h++)
              if (pat_index(PAT, f, h) >= 0 && pat_index(PAT, g, h) >= 0) A(t, f, h) -= l * U(u, g, h);
            break;
          }
        }
      }
    }
  }
  // 2) inside the vertex: rows (i,f) eliminated by (i,g<f); invert the pivots
  for (int f = 0; f < NF; f++) {
    for (int g = 0; g < f; g++) {
      if (pat_index(PAT, f, g) < 0) continue;
      const double l = A(0, f, g) * A(0, g, g);  // A(0,g,g) already inverted
      A(0, f, g) = l;
      for (int h = g + 1; h < NF; h++)
        if (pat_index(PAT, f, h) >= 0 && pat_index(PAT, g, h) >= 0) A(0, f, h) -= l * A(0, g, h);
      for (int t = 1; t < leni; t++) {
        const int m = cixi[t * kRows];
        if (m <= row || m >= L.n_owned) continue;
        for (int h = 0; h < NF; h++)
          if (pat_index(PAT, f, h) >= 0 && pat_index(PAT, g, h) >= 0) A(t, f, h) -= l * A(t, g, h);
      }
    }
    A(0, f, f) = 1.0 / A(0, f, f);
  }
}

// The same factorisation with the neighbour-row work hoisted and the expand / split passes folded
// in (one launch per colour, no k_expand / k_split passes), on a row-contiguous scratch copy:
// row i's blocks are aos[(rowoff[i] + t) * NV + q] and its columns rowcol[rowoff[i] + t]
// (t = fan slot), so reading a neighbour row's blocks and columns touches ~4 cache lines instead
// of one line per (slot, value pair) of the SELL layout (the gathers of a factorisation are per
// thread, not per wave, and were 8x over-fetched: profiles/r02/pmc_summary.json).
//   0) the row expands its own k-form blocks (masked) into aos;
//   1) per lower neighbour j (ascending): the L block L_ij = A_ij U_jj^-1 is finished in registers
//      from row j's diagonal block (loaded once), then every block A_im with m > j in both rows is
//      updated from row j's block U_jm, each loaded once per j (the column match of the two rows
//      is computed once per j, not once per field pair);
//   2) inside the vertex, as in k_ilu0_factor;
//   3) the row's blocks are written to the split L / U storage (VT: double or float).
// Per block entry the subtraction order (j ascending, then g ascending) is that of
// k_ilu0_factor, so the factors are bitwise the same.
// KMAX > 0: the row's own blocks live in LDS during the elimination (KMAX >= the fan length +
// 1 of every row) and reach the scratch once, when they are final: the per-row working set of a
// wave does not fit the L2 otherwise, and every update of an own block was a write-back.
// A/B build flag ILU_ROUND_BITS = b: the single-precision factors rounded to b significant bits
// (11: half precision, 8: bfloat16) in f32 storage and range -- what a 16-bit factor format would
// cost in preconditioner quality, measured before building one
__device__ __forceinline__ float ilu_round(float x) {
#ifdef ILU_ROUND_BITS
  constexpr int drop = 24 - ILU_ROUND_BITS;
  unsigned u = __float_as_uint(x);
  u += (1u << (drop - 1)) - 1u + ((u >> drop) & 1u);
  u &= ~((1u << drop) - 1u);
  return __uint_as_float(u);
#else
  return x;
#endif
}

template <int NF, int PAT, typename VT, int KMAX, int TB>
__global__ __launch_bounds__(TB) void k_ilu0_factor_fused(DevLayout L, int r0, int r1,
                                                          const double *__restrict__ kvals,
                                                          const int *__restrict__ rowoff,
                                                          const int *__restrict__ rowcol,
                                                          double *__restrict__ aos,
                                                          VT *__restrict__ lv,
                                                          VT *__restrict__ uv) {
  constexpr int NV = popc9(PAT), NK = nks_of(PAT), NS = slot_vals<NV, VT>();
  __shared__ double own[KMAX > 0 ? KMAX * NV : 1][KMAX > 0 ? TB : 1];
  const int row = r0 + xcd_block(blockIdx.x, gridDim.x, 1) * TB + threadIdx.x;
  if (row >= r1) return;
  const int ci = row / kRows, li = row % kRows;
  const int offi = L.chunk_off[ci], leni = int(L.rowmeta[row] & 63);
  const int *__restrict__ cixi = rowcol + rowoff[row];
  double *__restrict__ vi = aos + size_t(rowoff[row]) * NV;
  const int tl = threadIdx.x;
  auto ld = [&](const double *base, int t, double (&B)[NV]) {
    if (KMAX > 0 && base == vi) {
#pragma unroll
      for (int q = 0; q < NV; q++) B[q] = own[t * NV + q][tl];
      return;
    }
#pragma unroll
    for (int q = 0; q < NV; q++) B[q] = base[size_t(t) * NV + q];
  };
  auto st = [&](double *base, int t, const double (&B)[NV]) {
    if (KMAX > 0 && base == vi) {
#pragma unroll
      for (int q = 0; q < NV; q++) own[t * NV + q][tl] = B[q];
      return;
    }
#pragma unroll
    for (int q = 0; q < NV; q++) base[size_t(t) * NV + q] = B[q];
  };
  // 0) expand + mask the row's blocks into its scratch rows
  {
    const unsigned dm = row_mask<NF>(L, row);
    const double *kb = kvals + size_t(offi) * NK;
    for (int t = 0; t < leni; t++) {
      double K[NK], B[NV];
#pragma unroll
      for (int q = 0; q < NK; q++) K[q] = kb[size_t(t) * NK * kRows + vin(NK, q, li)];
      expand_k<PAT>(K, B);
      mask_rows<NF, PAT>(B, dm, t == 0);
      st(vi, t, B);
    }
  }
  // 1) lower neighbours in increasing index order
  int prev = -1;
  for (;;) {
    int j = 0x7fffffff, s = -1;
    for (int t = 1; t < leni; t++) {
      const int c = cixi[t];
      if (c < row && c > prev && c < j && !same_color(L, c, row)) {
        j = c;
        s = t;
      }
    }
    if (s < 0) break;
    prev = j;
    const int lenj = int(L.rowmeta[j] & 63);
    const int *__restrict__ cixj = rowcol + rowoff[j];
    const double *__restrict__ vj = aos + size_t(rowoff[j]) * NV;
    double Ujj[NV], Lb[NV];
    ld(vj, 0, Ujj);
    ld(vi, s, Lb);
#pragma unroll
    for (int g = 0; g < NF; g++) {
      const double dinv = Ujj[pat_index(PAT, g, g)];  // stored inverted
#pragma unroll
      for (int f = 0; f < NF; f++) {
        if (pat_index(PAT, f, g) < 0) continue;
        const double l = Lb[pat_index(PAT, f, g)] * dinv;
        Lb[pat_index(PAT, f, g)] = l;
        if (l == 0.0) continue;
#pragma unroll
        for (int h = g + 1; h < NF; h++)
          if (pat_index(PAT, f, h) >= 0 && pat_index(PAT, g, h) >= 0)
            Lb[pat_index(PAT, f, h)] -= l * Ujj[pat_index(PAT, g, h)];
      }
    }
    st(vi, s, Lb);
    for (int t = 0; t < leni; t++) {
      const int m = cixi[t];
      if (m <= j || m >= L.n_owned || (t > 0 && m == row)) continue;
      if (dropped(L, row, m) || dropped(L, j, m)) continue;
      int u = 1;
      while (u < lenj && cixj[u] != m) u++;
      if (u == lenj) continue;
      double U[NV], A[NV];
      ld(vj, u, U);
      ld(vi, t, A);
#pragma unroll
      for (int g = 0; g < NF; g++)
#pragma unroll
        for (int f = 0; f < NF; f++) {
          if (pat_index(PAT, f, g) < 0) continue;
          const double l = Lb[pat_index(PAT, f, g)];
          if (l == 0.0) continue;
#pragma unroll
          for (int h = 0; h < NF; h++)
            if (pat_index(PAT, f, h) >= 0 && pat_index(PAT, g, h) >= 0)
              A[pat_index(PAT, f, h)] -= l * U[pat_index(PAT, g, h)];
        }
      st(vi, t, A);
    }
  }
  // 2) inside the vertex: rows (i,f) eliminated by (i,g<f); invert the pivots
  double D[NV];
  ld(vi, 0, D);
  for (int f = 0; f < NF; f++) {
    for (int g = 0; g < f; g++) {
      if (pat_index(PAT, f, g) < 0) continue;
      const double l = D[pat_index(PAT, f, g)] * D[pat_index(PAT, g, g)];
      D[pat_index(PAT, f, g)] = l;
      for (int h = g + 1; h < NF; h++)
        if (pat_index(PAT, f, h) >= 0 && pat_index(PAT, g, h) >= 0)
          D[pat_index(PAT, f, h)] -= l * D[pat_index(PAT, g, h)];
      for (int t = 1; t < leni; t++) {
        const int m = cixi[t];
        if (m <= row || m >= L.n_owned) continue;
        double A[NV];
        ld(vi, t, A);
        for (int h = 0; h < NF; h++)
          if (pat_index(PAT, f, h) >= 0 && pat_index(PAT, g, h) >= 0)
            A[pat_index(PAT, f, h)] -= l * A[pat_index(PAT, g, h)];
        st(vi, t, A);
      }
    }
    D[pat_index(PAT, f, f)] = 1.0 / D[pat_index(PAT, f, f)];
  }
  st(vi, 0, D);
  if constexpr (KMAX > 0) {
    // the finished row, for the rows of later colours: they read only its diagonal block and its
    // blocks of higher owned columns of another colour (step 1), so its lower blocks stay in LDS
    // and the last colour (no later rows) writes nothing (-0.13 GB per factorisation at config 3)
    if (r1 < L.n_owned)
      for (int t = 0; t < leni; t++) {
        const int m = cixi[t];
        if (t > 0 && (m <= row || m >= L.n_owned || same_color(L, m, row))) continue;
#pragma unroll
        for (int q = 0; q < NV; q++) vi[size_t(t) * NV + q] = own[t * NV + q][tl];
      }
  }
  // 3) the split storage: slot 0 and the owned upper columns (slot order) to U, the lower
  // columns (slot order) to L, ghost columns dropped -- the order ctx.cc builds lsrc / usrc in
  const int lla = L.lpinv ? int(L.lpinv[row]) : li, ula = L.upinv ? int(L.upinv[row]) : li;
  auto put = [&](VT *base, int off, int k, const double (&B)[NV]) {
    const int ln = base == lv ? lla : ula;  // the row's lane in the L / U storage
    VT *sb = base + (size_t(off) + size_t(k) * kRows) * NS;
    if constexpr (std::is_same<VT, double>::value) {
#pragma unroll
      for (int q = 0; q < NV; q++) sb[vin(NV, q, ln)] = B[q];
    } else if constexpr (std::is_same<VT, bf16s>::value) {
#pragma unroll
      for (int q = 0; q < NS; q++) sb[vinb(NV, q, ln)] = q < NV ? to_bf16(float(B[q])) : bf16s(0);
    } else {
#pragma unroll
      for (int q = 0; q < NS; q++) sb[vinf(NV, q, ln)] = q < NV ? ilu_round(float(B[q])) : 0.0f;
    }
  };
  const int loff = L.lchunk_off[ci], uoff = L.uchunk_off[ci];
  put(uv, uoff, 0, D);
  int kl = 0, ku = 1;
  for (int t = 1; t < leni; t++) {
    const int c = cixi[t];
    if (c >= L.n_owned || c == row || same_color(L, c, row)) continue;
    double B[NV];
    ld(vi, t, B);
    if (c < row)
      put(lv, loff, kl++, B);
    else
      put(uv, uoff, ku++, B);
  }
}

// y <- Ld^-1 y (unit lower part of the factored diagonal block, fields ascending)
template <int NF, int PAT, int NV>
__device__ __forceinline__ void diag_lower_solve(const double (&Dg)[NV], double (&y)[NF]) {
#pragma unroll
  for (int f = 0; f < NF; f++)
#pragma unroll
    for (int g = 0; g < f; g++) {
      const int qq = pat_index(PAT, f, g);
      if (qq >= 0) y[f] -= Dg[qq] * y[g];
    }
}

// y <- U^-1 y (upper part, pivots stored inverted, fields descending)
template <int NF, int PAT, int NV>
__device__ __forceinline__ void diag_upper_solve(const double (&Dg)[NV], double (&y)[NF]) {
#pragma unroll
  for (int ff = NF - 1; ff >= 0; ff--) {
#pragma unroll
    for (int h = ff + 1; h < NF; h++) {
      const int qq = pat_index(PAT, ff, h);
      if (qq >= 0) y[ff] -= Dg[qq] * y[h];
    }
    y[ff] *= Dg[pat_index(PAT, ff, ff)];
  }
}

// Sweeps over the split factors, one colour per launch, LPR lanes per row as in k_sgs_color.
// KIND kIluFwd / kIluBwd: forward (unit lower, colours ascending) / backward (upper, colours
// descending).  kIluLast: the last colour's forward and backward in one launch -- it has no upper
// neighbours (every row after it in the colour-major order is of its own colour, hence not
// adjacent), so its backward step is pointwise; the arithmetic is that of the two launches.
// (Folding Ld into the coupling blocks, L'_ij = Lo_ij Ld_j^-1, would drop the colour-0 forward
// launch too, but z = Ld y cancels on the strongly coupled drift blocks: +24 % iterations on the
// 24 V pore case, measured -- DESIGN.md §4.)
enum { kIluFwd = 0, kIluBwd = 1, kIluLast = 2 };

// ADD = 1 (backward / last-colour launches): also out_i = add_i + v_i for the finished rows (the
// AMG's post-smoothing update y + M^-1 r without a separate pass).  YT = float (bf16 factors,
// launch_ilu0_apply's yf): the forward colours store y = L^-1 d in yv, rounded to single precision,
// the forward gathers and the backward sweep's own rows read it there; YT = double: y lives in v
template <int NF, int PAT, int KIND, int LPR, int B, int NT, int ADD = 0, typename VT = double,
          typename YT = double>
__global__ __launch_bounds__(kBlock) void k_ilu0_solve(DevLayout L, int r0, int r1,
                                                       const VT *__restrict__ lv,
                                                       const VT *__restrict__ uv,
                                                       const double *__restrict__ d,
                                                       double *__restrict__ v,
                                                       const double *__restrict__ add = nullptr,
                                                       double *__restrict__ out = nullptr,
                                                       YT *__restrict__ yv = nullptr) {
  constexpr int NV = popc9(PAT);
  constexpr bool FWD = KIND != kIluBwd;
  constexpr bool YF = !std::is_same<YT, double>::value;
  const int gt = xcd_block(blockIdx.x, gridDim.x, 1) * kBlock + threadIdx.x;
  const int k = gt / LPR, q = gt % LPR;
  const bool live = r0 + k < r1;
  const SplitRow<VT> R = split_row<NV, FWD, VT>(L, lv, uv, live ? r0 + k : r0, live);
  const int row = R.row;
  // own data and diagonal block first: they share the neighbour loop's round trips
  double own[NF], Dg[NV];
  if constexpr (YF && !FWD)
    load_nf<NF>(yv, size_t(row), own);
  else
    load_nf<NF>(FWD ? d : v, size_t(row), own);
  load_split_vals<NV, 0, VT, KIND == kIluFwd>(R.dg, R.dlane, Dg);
  double acc[NF];
  if constexpr (YF && FWD)
    split_row_dot<NF, PAT, LPR, B, NT, VT>(R, 0, q, row, static_cast<const YT *>(yv), acc);
  else
    split_row_dot<NF, PAT, LPR, B, NT, VT>(R, FWD ? 0 : 1, q, row, v, acc);
  if (!live || q != 0) return;
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] += own[f];
  if (FWD) diag_lower_solve<NF, PAT>(Dg, acc);
  if (KIND != kIluFwd) diag_upper_solve<NF, PAT>(Dg, acc);
  if constexpr (YF && KIND == kIluFwd)
    store_nf<NF>(yv, size_t(row), acc);
  else
    store_nf<NF>(v, size_t(row), acc);
  if constexpr (ADD && KIND != kIluFwd) {
    double ad[NF];
    load_nf<NF>(add, size_t(row), ad);
#pragma unroll
    for (int f = 0; f < NF; f++) ad[f] += acc[f];
    store_nf<NF>(out, size_t(row), ad);
  }
}

// k_ilu0_solve (one lane per row) with the neighbour gathers staged through LDS: the workgroup's
// 256 rows (one block of one colour) first load v at the distinct rows their split slots couple to
// (DevLayout lsx_* / usx_*: config 3 has ~1.8 slots per distinct neighbour), then every slot reads
// its neighbour's record from LDS by a 16-bit list position.  The rows read are of other colours
// -- earlier ones in the forward sweep, later (finished) ones in the backward sweep -- so nothing
// staged is written during the launch.  Each row's sum runs over its slots in the order of
// split_row_dot<.., 1, B>, so v is bitwise k_ilu0_solve's.  The row's own loads, its diagonal
// block and its first slot batch's list positions and factor values are issued before the barrier.
#ifndef ILU_SU
#define ILU_SU 4  // staged list entries per thread issued together (build-flag A/B knob)
#endif
template <int NF, int PAT, int KIND, int B, int NT, int ADD = 0, typename VT = double,
          typename YT = double>
__global__ __launch_bounds__(kBlock) void k_ilu0_solve_lds(DevLayout L, int r0, int r1, int blk0,
                                                           const VT *__restrict__ lv,
                                                           const VT *__restrict__ uv,
                                                           const double *__restrict__ d,
                                                           double *__restrict__ v,
                                                           const double *__restrict__ add = nullptr,
                                                           double *__restrict__ out = nullptr,
                                                           YT *__restrict__ yv = nullptr) {
  constexpr int NV = popc9(PAT), NS = slot_vals<NV, VT>();
  constexpr bool FWD = KIND != kIluBwd;
  constexpr bool YF = !std::is_same<YT, double>::value;  // k_ilu0_solve's YT
  extern __shared__ double sx[];  // [cnt][NF]
  const int bl = xcd_block(blockIdx.x, gridDim.x, 1);
  const bool live = r0 + bl * kBlock + int(threadIdx.x) < r1;
  const int pos = live ? r0 + bl * kBlock + int(threadIdx.x) : r0;
  // the staging list's bounds first: they depend on nothing, so their round trip is the row
  // metadata's (split_row) instead of one more in the chain before the barrier
  const int *__restrict__ ptr = FWD ? L.lsx_ptr : L.usx_ptr;
  const int *__restrict__ lst = FWD ? L.lsx_list : L.usx_list;
  const int u0 = ptr[blk0 + bl], u1 = ptr[blk0 + bl + 1];
  const SplitRow<VT> R = split_row<NV, FWD, VT>(L, lv, uv, pos, live);
  const int row = R.row;
  double own[NF], Dg[NV];
  if constexpr (YF && !FWD)
    load_nf<NF>(yv, size_t(row), own);
  else
    load_nf<NF>(FWD ? d : v, size_t(row), own);
  load_split_vals<NV, 0, VT, KIND == kIluFwd>(R.dg, R.dlane, Dg);
  const int chunk = pos / kRows;
  const uint16_t *__restrict__ lix =
      (FWD ? L.lsx_idx + L.lchunk_off[chunk] : L.usx_idx + L.uchunk_off[chunk]) + R.lane;
  const int s0 = FWD ? 0 : 1;
  // a batch's list positions and factor values (kept as stored, float or double, until used) do
  // not depend on the staging: the first batch is in flight with it
  int li[B];
  using KT = slot_keep_t<VT>;
  KT ar[B][NS];
  auto fetch = [&](int sb) {
#pragma unroll
    for (int b = 0; b < B; b++) {
      const int s = sb + b;
      li[b] = s < R.len ? int(lix[s * kRows]) : 0xFFFF;
      const VT *sbp = R.vc + size_t(s) * NS * kRows;
      if (s >= R.len) {
#pragma unroll
        for (int qq = 0; qq < NS; qq++) ar[b][qq] = KT(0);
      } else if constexpr (std::is_same<VT, double>::value) {
        load_split_vals<NV, NT>(sbp, R.lane, ar[b]);
      } else if constexpr (std::is_same<VT, bf16s>::value) {
        load_bf16_slot<NV, NT, float>(sbp, R.lane, ar[b]);
      } else if constexpr (NV == 1) {
        ar[b][0] = NT ? __builtin_nontemporal_load(sbp + R.lane) : sbp[R.lane];
      } else {
        load_f32_slot<NV, NT, float>(sbp, R.lane, ar[b]);
      }
    }
  };
  fetch(s0);
  // the staging: up to kSU list entries per thread, their list loads, then their gathers, then the
  // LDS stores (two round trips, not two per entry)
  const int cnt = u1 - u0;
  {
    constexpr int kSU = ILU_SU;
    int jj[kSU];
#pragma unroll
    for (int u = 0; u < kSU; u++) {
      const int k = int(threadIdx.x) + u * kBlock;
      jj[u] = k < cnt ? lst[u0 + k] : -1;
    }
    double t[kSU][NF];
#pragma unroll
    for (int u = 0; u < kSU; u++)
      if (jj[u] >= 0) {
        if constexpr (YF && FWD)
          load_nf<NF>(yv, size_t(jj[u]), t[u]);
        else
          load_nf<NF>(v, size_t(jj[u]), t[u]);
      }
#pragma unroll
    for (int u = 0; u < kSU; u++) {
      const int k = int(threadIdx.x) + u * kBlock;
      if (jj[u] >= 0)
#pragma unroll
        for (int f = 0; f < NF; f++) sx[k * NF + f] = t[u][f];
    }
  }
  for (int k = int(threadIdx.x) + ILU_SU * kBlock; k < cnt; k += kBlock) {  // longer lists
    double t[NF];
    if constexpr (YF && FWD)
      load_nf<NF>(yv, size_t(lst[u0 + k]), t);
    else
      load_nf<NF>(v, size_t(lst[u0 + k]), t);
#pragma unroll
    for (int f = 0; f < NF; f++) sx[k * NF + f] = t[f];
  }
  __syncthreads();
  double acc[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] = 0.0;
  for (int sb = s0; sb < R.len; sb += B) {
    if (sb != s0) fetch(sb);
    // explicit fused multiply-adds: the contraction k_ilu0_solve gets from the compiler (with the
    // operand selects the compiler would otherwise split some products into mul + add); each
    // slot's values are converted where they are used (short live ranges: VGPRs, occupancy)
#pragma unroll
    for (int b = 0; b < B; b++) {
      const bool use = li[b] != 0xFFFF;  // padding: zero values, zero operand
      double vj[NF];
#pragma unroll
      for (int g = 0; g < NF; g++) vj[g] = use ? sx[li[b] * NF + g] : 0.0;
#pragma unroll
      for (int f = 0; f < NF; f++)
#pragma unroll
        for (int g = 0; g < NF; g++) {
          const int qq = pat_index(PAT, f, g);
          if (qq >= 0)
            acc[f] = __builtin_fma(-(use ? double(ar[b][qq]) : 0.0), vj[g], acc[f]);
        }
    }
  }
  if (!live) return;
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] += own[f];
  if (FWD) diag_lower_solve<NF, PAT>(Dg, acc);
  if (KIND != kIluFwd) diag_upper_solve<NF, PAT>(Dg, acc);
  if constexpr (YF && KIND == kIluFwd)
    store_nf<NF>(yv, size_t(row), acc);
  else
    store_nf<NF>(v, size_t(row), acc);
  if constexpr (ADD && KIND != kIluFwd) {
    double ad[NF];
    load_nf<NF>(add, size_t(row), ad);
#pragma unroll
    for (int f = 0; f < NF; f++) ad[f] += acc[f];
    store_nf<NF>(out, size_t(row), ad);
  }
}

// ---- the whole application as one dataflow launch (k_ilu0_flow, kernels.h IluFlow) -------------
// A colour launch is a short chain of dependent round trips per block whatever it moves (10-16 us
// at config 3), and the next colour cannot start before the slowest block of this
// one has finished.  Here each 256-row block of each colour launch is a unit: a workgroup takes the
// next unit in the launches' order by an atomic ticket, issues everything that does not depend on
// this application (row metadata, factor values, staging lists, d) at once, waits only for the
// units whose rows it reads, and runs the LDS kernel's arithmetic on its block.  A block of colour
// c + 1 can thus start while other blocks of colour c are still running.
// Progress: a unit waits only on units with smaller tickets, which were claimed by workgroups that
// are running; the smallest unfinished ticket therefore never waits, whatever the residency.  Every
// wait is bounded (kIluFlowTimeout) and sets abort_word, so the grid always drains.
// Visibility (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md § visibility): every store
// of v in the launch is write-through (buffer_store ... sc1), every storing wave drains it
// (s_waitcnt vmcnt(0)) before the workgroup barrier, after which one lane stores the unit's flag
// with an agent-scope atomic; consumers poll flags with relaxed agent-scope loads (sc1) and read
// v only by sc1 loads, which bypass the per-CU L1 that another CU's stores never refresh.  d and
// the factors are not written in the launch and are read plainly.
// Dependencies (host, ctx.cc ilu_flow_build): a forward unit waits for the forward units of the
// rows in its L staging list; a backward unit for the backward units of the rows in its U list,
// the forward units of its own rows (their forward values are its `own`), and every forward unit
// that reads one of its rows (their forward values must be read before it overwrites them).
constexpr unsigned long long kIluFlowTimeout = 100000000ull;  // wall_clock64 ticks (100 MHz): 1 s

__device__ __forceinline__ __amdgpu_buffer_rsrc_t vec_rsrc(const double *p) {
  // range 2^31 - 16 bytes: offsets are 32-bit (vectors of up to 268 M doubles)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(p), 0, 0x7FFFFFF0, 0x00020000);
}
constexpr int kSc1 = 16;  // cache-policy bits of a buffer access: sc1 (write-through / L1 bypass)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <int NF>
__device__ __forceinline__ void load_nf_sc1(__amdgpu_buffer_rsrc_t r, int j, double (&o)[NF]) {
  const int off = j * NF * 8;
  int f = 0;
#pragma unroll
  for (; f + 1 < NF; f += 2) {
    const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(r, off + 8 * f, 0, kSc1);
    o[f] = __hiloint2double(int(a.y), int(a.x));
    o[f + 1] = __hiloint2double(int(a.w), int(a.z));
  }
  if (f < NF) {
    const u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(r, off + 8 * f, 0, kSc1);
    o[f] = __hiloint2double(int(a.y), int(a.x));
  }
}
template <int NF>
__device__ __forceinline__ void store_nf_sc1(__amdgpu_buffer_rsrc_t r, int j, const double (&v)[NF]) {
  const int off = j * NF * 8;
  int f = 0;
#pragma unroll
  for (; f + 1 < NF; f += 2) {
    u32x4 a;
    a.x = unsigned(__double2loint(v[f]));
    a.y = unsigned(__double2hiint(v[f]));
    a.z = unsigned(__double2loint(v[f + 1]));
    a.w = unsigned(__double2hiint(v[f + 1]));
    __builtin_amdgcn_raw_buffer_store_b128(a, r, off + 8 * f, 0, kSc1);
  }
  if (f < NF) {
    u32x2 a;
    a.x = unsigned(__double2loint(v[f]));
    a.y = unsigned(__double2hiint(v[f]));
    __builtin_amdgcn_raw_buffer_store_b64(a, r, off + 8 * f, 0, kSc1);
  }
}

// wave 0 of the workgroup waits until every dependency of unit u has raised its flag
__device__ __forceinline__ void ilu_flow_wait(const IluFlow &F, int u) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  const int p0 = F.dep_ptr[u], p1 = F.dep_ptr[u + 1];
  for (int kb = p0; kb < p1; kb += 64) {
    const int k = kb + lane;
    const int w = k < p1 ? F.dep_list[k] : -1;
    bool ok = w < 0 || __hip_atomic_load(F.flags + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (__all(ok)) continue;
    const unsigned long long t0 = wall_clock64();
    while (true) {
      __builtin_amdgcn_s_sleep(1);
      if (!ok)
        ok = __hip_atomic_load(F.flags + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
      if (__all(ok)) break;
      const bool late = wall_clock64() - t0 > kIluFlowTimeout;
      if (late && lane == 0)
        __hip_atomic_store(F.abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (late || __hip_atomic_load(F.abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        return;  // results are void; the host reports the timeout
    }
  }
}

// one unit = one 256-row block of one colour launch of k_ilu0_solve_lds, the same arithmetic
template <int NF, int PAT, int KIND, int B, typename VT>
__device__ __forceinline__ void ilu_flow_unit(const DevLayout &L, const IluFlow &F, int u, int st,
                                              const VT *__restrict__ lv, const VT *__restrict__ uv,
                                              const double *__restrict__ d, double *v,
                                              double *sx) {
  constexpr int NV = popc9(PAT), NS = slot_vals<NV, VT>();
  constexpr bool FWD = KIND != kIluBwd;
  const __amdgpu_buffer_rsrc_t rv = vec_rsrc(v);
  const int bl = u - F.unit0[st], r0 = F.r0[st], r1 = F.r1[st], blk = F.blk0[st] + bl;
  const bool live = r0 + bl * kBlock + int(threadIdx.x) < r1;
  const int pos = live ? r0 + bl * kBlock + int(threadIdx.x) : r0;
  const int *__restrict__ ptr = FWD ? L.lsx_ptr : L.usx_ptr;
  const int *__restrict__ lst = FWD ? L.lsx_list : L.usx_list;
  const int u0 = ptr[blk], u1 = ptr[blk + 1];
  const SplitRow<VT> R = split_row<NV, FWD, VT>(L, lv, uv, pos, live);
  const int row = R.row;
  double own[NF], Dg[NV];
  if (FWD) load_nf<NF>(d, size_t(row), own);
  load_split_vals<NV, 0, VT, KIND == kIluFwd>(R.dg, R.dlane, Dg);
  const int chunk = pos / kRows;
  const uint16_t *__restrict__ lix =
      (FWD ? L.lsx_idx + L.lchunk_off[chunk] : L.usx_idx + L.uchunk_off[chunk]) + R.lane;
  const int s0 = FWD ? 0 : 1;
  int li[B];
  using KT = slot_keep_t<VT>;
  KT ar[B][NS];
  auto fetch = [&](int sb) {
#pragma unroll
    for (int b = 0; b < B; b++) {
      const int s = sb + b;
      li[b] = s < R.len ? int(lix[s * kRows]) : 0xFFFF;
      const VT *sbp = R.vc + size_t(s) * NS * kRows;
      if (s >= R.len) {
#pragma unroll
        for (int qq = 0; qq < NS; qq++) ar[b][qq] = KT(0);
      } else if constexpr (std::is_same<VT, double>::value) {
        load_split_vals<NV, 0>(sbp, R.lane, ar[b]);
      } else if constexpr (std::is_same<VT, bf16s>::value) {
        load_bf16_slot<NV, 0, float>(sbp, R.lane, ar[b]);
      } else if constexpr (NV == 1) {
        ar[b][0] = sbp[R.lane];
      } else {
        load_f32_slot<NV, 0, float>(sbp, R.lane, ar[b]);
      }
    }
  };
  fetch(s0);
  const int cnt = u1 - u0;
  constexpr int kSU = ILU_SU;
  int jj[kSU];
#pragma unroll
  for (int q = 0; q < kSU; q++) {
    const int k = int(threadIdx.x) + q * kBlock;
    jj[q] = k < cnt ? lst[u0 + k] : -1;
  }
  // the rows this unit reads are final once their units' flags are up
  ilu_flow_wait(F, u);
  __syncthreads();
  if (!FWD) load_nf_sc1<NF>(rv, row, own);
  {
    double t[kSU][NF];
#pragma unroll
    for (int q = 0; q < kSU; q++)
      if (jj[q] >= 0) load_nf_sc1<NF>(rv, jj[q], t[q]);
#pragma unroll
    for (int q = 0; q < kSU; q++) {
      const int k = int(threadIdx.x) + q * kBlock;
      if (jj[q] >= 0)
#pragma unroll
        for (int f = 0; f < NF; f++) sx[k * NF + f] = t[q][f];
    }
  }
  for (int k = int(threadIdx.x) + kSU * kBlock; k < cnt; k += kBlock) {
    double t[NF];
    load_nf_sc1<NF>(rv, lst[u0 + k], t);
#pragma unroll
    for (int f = 0; f < NF; f++) sx[k * NF + f] = t[f];
  }
  __syncthreads();
  double acc[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) acc[f] = 0.0;
  for (int sb = s0; sb < R.len; sb += B) {
    if (sb != s0) fetch(sb);
#pragma unroll
    for (int b = 0; b < B; b++) {
      const bool use = li[b] != 0xFFFF;
      double vj[NF];
#pragma unroll
      for (int g = 0; g < NF; g++) vj[g] = use ? sx[li[b] * NF + g] : 0.0;
#pragma unroll
      for (int f = 0; f < NF; f++)
#pragma unroll
        for (int g = 0; g < NF; g++) {
          const int qq = pat_index(PAT, f, g);
          if (qq >= 0)
            acc[f] = __builtin_fma(-(use ? double(ar[b][qq]) : 0.0), vj[g], acc[f]);
        }
    }
  }
  if (live) {
#pragma unroll
    for (int f = 0; f < NF; f++) acc[f] += own[f];
    if (FWD) diag_lower_solve<NF, PAT>(Dg, acc);
    if (KIND != kIluFwd) diag_upper_solve<NF, PAT>(Dg, acc);
    store_nf_sc1<NF>(rv, row, acc);
  }
  // publish: every storing wave drains its write-through stores, then one lane raises the flag
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(F.flags + u, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NF, int PAT, int B, typename VT>
__global__ __launch_bounds__(kBlock) void k_ilu0_flow(DevLayout L, IluFlow F,
                                                      const VT *__restrict__ lv,
                                                      const VT *__restrict__ uv,
                                                      const double *__restrict__ d, double *v) {
  extern __shared__ double smem[];  // [0, 2): reserved (16-B aligned staging); [2, ..): records
  if (F.persistent) {
    // resident grid (sized from the occupancy query): workgroup b takes units b, b + G, ... in
    // order.  The smallest unfinished unit's workgroup has finished its own earlier units, so it
    // runs that unit, whose dependencies are all finished: progress needs every workgroup of the
    // grid resident, which a single-stream context gives it
    int st = 0;
    for (int u = blockIdx.x; u < F.nunits; u += gridDim.x) {
      while (st + 1 < F.nstages && u >= F.unit0[st + 1]) st++;
      const int kind = F.kind[st];
      if (kind == kIluFwd)
        ilu_flow_unit<NF, PAT, kIluFwd, B, VT>(L, F, u, st, lv, uv, d, v, smem + 2);
      else if (kind == kIluLast)
        ilu_flow_unit<NF, PAT, kIluLast, B, VT>(L, F, u, st, lv, uv, d, v, smem + 2);
      else
        ilu_flow_unit<NF, PAT, kIluBwd, B, VT>(L, F, u, st, lv, uv, d, v, smem + 2);
    }
    return;
  }
  // one workgroup per unit, the unit taken by an atomic ticket (no residency assumption: lower
  // tickets belong to running workgroups); one ticket word serialises ~5,000 dequeues per launch
  int *tk = reinterpret_cast<int *>(smem);
  if (threadIdx.x == 0)
    tk[0] = int(__hip_atomic_fetch_add(F.flags + F.nunits, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT));
  __syncthreads();
  const int u = tk[0];
  if (u >= F.nunits) return;  // uniform (never: the grid is the unit count)
  int st = 0;
  while (st + 1 < F.nstages && u >= F.unit0[st + 1]) st++;
  const int kind = F.kind[st];
  if (kind == kIluFwd)
    ilu_flow_unit<NF, PAT, kIluFwd, B, VT>(L, F, u, st, lv, uv, d, v, smem + 2);
  else if (kind == kIluLast)
    ilu_flow_unit<NF, PAT, kIluLast, B, VT>(L, F, u, st, lv, uv, d, v, smem + 2);
  else
    ilu_flow_unit<NF, PAT, kIluBwd, B, VT>(L, F, u, st, lv, uv, d, v, smem + 2);
}

// split storage position p takes the block (row, slot) = (src >> 6, src & 63) of the full SELL:
// FROMK: expanded and masked from the k-form matrix, else copied from the NV-form ILU factors;
// padding (src < 0) gets zeros
template <int NF, int PAT, int FROMK, typename VT = double>
__global__ __launch_bounds__(kBlock) void k_split(DevLayout L, const double *__restrict__ src,
                                                  const int *__restrict__ lsrc, long long ln,
                                                  const int *__restrict__ usrc, long long un,
                                                  VT *__restrict__ lv, VT *__restrict__ uv) {
  constexpr int NV = popc9(PAT), NK = nks_of(PAT), NS = slot_vals<NV, VT>();
  long long p = blockIdx.x * (long long)kBlock + threadIdx.x;
  const int *ps = lsrc;
  VT *dst = lv;
  if (p >= ln) {
    p -= ln;
    if (p >= un) return;
    ps = usrc;
    dst = uv;
  }
  const int lane = int(p & (kRows - 1));
  VT *sb = dst + (p - lane) * NS;  // slot base (position p - lane is lane 0 of the slot)
  const int code = ps[p];
  double B[NV];
  if (code < 0) {
#pragma unroll
    for (int q = 0; q < NV; q++) B[q] = 0.0;
  } else {
    const int row = code >> 6, slot = code & 63;
    const int chunk = row / kRows, rl = row % kRows;
    if constexpr (FROMK) {
      double K[NK];
      load_vals<NK>(src + (size_t(L.chunk_off[chunk]) + size_t(slot) * kRows) * NK, rl, K);
      expand_k<PAT>(K, B);
      mask_rows<NF, PAT>(B, row_mask<NF>(L, row), slot == 0);
    } else {
      load_vals<NV>(src + (size_t(L.chunk_off[chunk]) + size_t(slot) * kRows) * NV, rl, B);
    }
  }
  // the split position's lane equals the row's lane (same row)
  if constexpr (std::is_same<VT, double>::value) {
#pragma unroll
    for (int q = 0; q < NV; q++) sb[vin(NV, q, lane)] = B[q];
  } else if constexpr (std::is_same<VT, bf16s>::value) {
#pragma unroll
    for (int q = 0; q < NS; q++) sb[vinb(NV, q, lane)] = q < NV ? to_bf16(float(B[q])) : bf16s(0);
  } else {
#pragma unroll
    for (int q = 0; q < NS; q++) sb[vinf(NV, q, lane)] = q < NV ? float(B[q]) : 0.0f;
  }
}

// lu = expand_k + mask_rows of every block of the k-form matrix (NV values per block)
template <int NF, int PAT>
__global__ __launch_bounds__(kBlock) void k_expand(DevLayout L, const double *__restrict__ vals,
                                                   double *__restrict__ lu) {
  constexpr int NV = popc9(PAT), NK = nks_of(PAT);
  const int row = blockIdx.x * kBlock + threadIdx.x;
  if (row >= L.n_owned) return;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = L.chunk_off[chunk], len = L.chunk_len[chunk];
  const unsigned dm = row_mask<NF>(L, row);
  for (int s = 0; s < len; s++) {
    double K[NK], B[NV];
    load_vals<NK>(vals + (size_t(off) + size_t(s) * kRows) * NK, lane, K);
    expand_k<PAT>(K, B);
    mask_rows<NF, PAT>(B, dm, s == 0);
    store_vals<NV>(lu + (size_t(off) + size_t(s) * kRows) * NV, lane, B);
  }
}

// ------------------------------------------------------------------------------------------
// BLAS-1 and reductions
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_update_p(long long n, const Scalars *__restrict__ S,
                                                     const double *__restrict__ r,
                                                     const double *__restrict__ v,
                                                     double *__restrict__ p, int first) {
  if (S->done) return;
  const double beta = first ? 0.0 : (S->rho_new / S->rho) * (S->alpha / S->omega);
  const double om = S->omega;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < n;
       i += (long long)gridDim.x * kBlock)
    p[i] = first ? r[i] : beta * (p[i] - om * v[i]) + r[i];
}

// CG: p = q + beta p (beta kept in S->omega, derive stage 14)
__global__ __launch_bounds__(kBlock) void k_cg_update_p(long long n, const Scalars *__restrict__ S,
                                                        const double *__restrict__ q,
                                                        double *__restrict__ p) {
  if (S->done) return;
  const double beta = S->omega;
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < n;
       i += (long long)gridDim.x * kBlock)
    p[i] = q[i] + beta * p[i];
}

template <int TWO>
__global__ __launch_bounds__(kBlock) void k_update_xr(long long n, const Scalars *__restrict__ S,
                                                      int which, double *__restrict__ x,
                                                      const double *__restrict__ y,
                                                      double *__restrict__ r,
                                                      const double *__restrict__ v,
                                                      const double *__restrict__ rt,
                                                      double *__restrict__ partials,
                                                      const double *__restrict__ y1) {
  const double al = S->alpha;
  if (S->done) {
    if (!(y1 && S->xpend)) return;
    // the first half step converged: its deferred x += alpha y1, as ISTL returns it
    for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < n;
         i += (long long)gridDim.x * kBlock)
      x[i] += al * y1[i];
    return;
  }
  const double a = which ? S->omega : al;
  double acc[2] = {0, 0};
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < n;
       i += (long long)gridDim.x * kBlock) {
    double xi = x[i];
    if (y1) xi += al * y1[i];  // uniform
    xi += a * y[i];
    x[i] = xi;
    const double ri = r[i] - a * v[i];
    r[i] = ri;
    acc[0] += ri * ri;
    if (TWO) acc[1] += rt[i] * ri;
  }
  if (TWO) {
    block_sum<2>(acc, partials + 2 * blockIdx.x);
  } else {
    double a1[1] = {acc[0]};
    block_sum<1>(a1, partials + blockIdx.x);
  }
}

// BiCGSTAB vector updates fused with colour 0 of the ILU(0) forward sweep that consumes them.
// Colour-0 rows come first in the colour-major order, so they have no lower neighbours: their
// forward step is y_i = Ld_i^-1 d_i, pointwise.  The update that produces d (WHICH 0: p = r +
// beta (p - omega v); WHICH 1: x += alpha y, s = r - alpha v with the ||s||^2 partials) applies it
// in the same pass, one row per thread, and the sweep starts at colour 1: one launch and one
// re-read of d fewer per preconditioner application.  yin may alias yout (x += alpha y reads a
// row's y before the row's new y is written, by the same thread).  YT = float: yout is the ILU(0)
// application's single-precision intermediate (launch_ilu0_apply's yf).
template <int NF, int PAT, int WHICH, typename VT = double, typename YT = double>
__global__ __launch_bounds__(kBlock) void k_update_fwd0(DevLayout L, int c0_end,
                                                        Scalars *S, int first,
                                                        double *__restrict__ x, const double *yin,
                                                        double *__restrict__ r,
                                                        const double *__restrict__ v,
                                                        double *__restrict__ p,
                                                        const VT *__restrict__ uv,
                                                        YT *yout,
                                                        double *__restrict__ partials,
                                                        const double *__restrict__ rt) {
  constexpr int NV = popc9(PAT);
  if (S->done) return;  // uniform over the grid
  const int row = blockIdx.x * kBlock + threadIdx.x;
  const bool live = row < L.n_owned;
  double ss = 0, rs = 0;
  if (live) {
    double d[NF], vv[NF];
    load_nf<NF>(r, size_t(row), d);
    load_nf<NF>(v, size_t(row), vv);
    if (WHICH == 0) {
      const double beta = first ? 0.0 : (S->rho_new / S->rho) * (S->alpha / S->omega);
      const double om = S->omega;
      if (!first) {
        double po[NF];
        load_nf<NF>(p, size_t(row), po);
#pragma unroll
        for (int f = 0; f < NF; f++) d[f] = beta * (po[f] - om * vv[f]) + d[f];
      }
      store_nf<NF>(p, size_t(row), d);
    } else {
      const double a = S->alpha;
      double xi[NF], yi[NF];
      if (x) {  // uniform; null: deferred to k_update_xr (S->xpend)
        load_nf<NF>(x, size_t(row), xi);
        load_nf<NF>(yin, size_t(row), yi);
#pragma unroll
        for (int f = 0; f < NF; f++) xi[f] += a * yi[f];
      }
#pragma unroll
      for (int f = 0; f < NF; f++) {
        d[f] -= a * vv[f];
        ss += d[f] * d[f];
      }
      if (rt) {  // <rt, s> for the two-reduction iteration
        double ti[NF];
        load_nf<NF>(rt, size_t(row), ti);
#pragma unroll
        for (int f = 0; f < NF; f++) rs += ti[f] * d[f];
      }
      if (x) store_nf<NF>(x, size_t(row), xi);
      store_nf<NF>(r, size_t(row), d);
    }
    if (row < c0_end) {
      double Dg[NV];
      load_split_vals<NV, 0, VT, 1>(uv + size_t(L.uchunk_off[row / kRows]) * slot_vals<NV, VT>(),
                             L.upinv ? int(L.upinv[row]) : row % kRows, Dg);
      diag_lower_solve<NF, PAT>(Dg, d);
      store_nf<NF>(yout, size_t(row), d);
    }
  }
  if (WHICH == 1) {
    if (!x && blockIdx.x == 0 && threadIdx.x == 0) S->xpend = 1;  // read by k_update_xr only
    if (rt) {  // uniform over the grid
      double a2[2] = {ss, rs};
      block_sum<2>(a2, partials + 2 * blockIdx.x);
    } else {
      double a1[1] = {ss};
      block_sum<1>(a1, partials + blockIdx.x);
    }
  }
}

template <int TWO>
__global__ __launch_bounds__(kBlock) void k_dot(long long n, const double *__restrict__ a,
                                                const double *__restrict__ b,
                                                double *__restrict__ partials) {
  double acc[2] = {0, 0};
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < n;
       i += (long long)gridDim.x * kBlock) {
    acc[0] += a[i] * b[i];
    if (TWO) acc[1] += a[i] * a[i];
  }
  if (TWO) {
    block_sum<2>(acc, partials + 2 * blockIdx.x);
  } else {
    double a1[1] = {acc[0]};
    block_sum<1>(a1, partials + blockIdx.x);
  }
}

__device__ void derive(Scalars *S, int stage);

// Final reduction of per-workgroup partials (deterministic: fixed order for a given np).
// One workgroup of kRedBlock threads; each thread issues its (up to kRedU) partial loads back to
// back before adding, so the ~3K partials of a config-3 SpMV cost one memory round trip instead
// of the ~11 dependent ones of a 256-thread strided loop (13.8 -> see DESIGN.md, reductions).
// 12 partials per thread and pass (6 for 4-5 values per partial): the ~8,600 partials of a
// config-3 SpMV are one pass (4 took three dependent passes); a thread still adds its partials in
// index order (tid, tid + 1024, ...), so every sum is bitwise the 4-per-pass one's.
constexpr int kRedBlock = 1024;
template <int K>
constexpr int red_unroll() { return K <= 3 ? 12 : 6; }  // <= 128 VGPRs at 1024 threads

// the partials of two arrays (KB = 0: one) in the same passes, so the second array's loads are
// in flight with the first's; acc[0 .. KA) sums pa, acc[KA ..) sums pb, each in index order
template <int KA, int KB>
__device__ __forceinline__ void accum_partials(const double *__restrict__ pa, int npa,
                                               const double *__restrict__ pb, int npb,
                                               double *acc) {
  constexpr int kRedU = red_unroll<KA + KB>();
  const int np = npa > npb ? npa : npb;
  for (int i0 = threadIdx.x; i0 < np; i0 += kRedU * kRedBlock) {
    double va[kRedU][KA], vb[kRedU][KB > 0 ? KB : 1];
#pragma unroll
    for (int u = 0; u < kRedU; u++) {
      const int i = i0 + u * kRedBlock;
#pragma unroll
      for (int j = 0; j < KA; j++) va[u][j] = i < npa ? pa[size_t(i) * KA + j] : 0.0;
#pragma unroll
      for (int j = 0; j < KB; j++) vb[u][j] = i < npb ? pb[size_t(i) * KB + j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kRedU; u++) {
#pragma unroll
      for (int j = 0; j < KA; j++) acc[j] += va[u][j];
#pragma unroll
      for (int j = 0; j < KB; j++) acc[KA + j] += vb[u][j];
    }
  }
}

template <int KA, int KB>
__global__ __launch_bounds__(kRedBlock) void k_reduce(const double *__restrict__ pa, int npa,
                                                      const double *__restrict__ pb, int npb,
                                                      Scalars *__restrict__ S, int stage) {
  // the start stages (0 BiCGSTAB, 10 CG) run on a fresh state; everything else stops once done
  if (S->done && stage != 0 && stage != 10) {
    if (stage == 4 && threadIdx.x == 0) S->xpend = 0;  // (derive's stage 4 clears it otherwise)
    return;
  }
  double acc[KA + KB];
#pragma unroll
  for (int j = 0; j < KA + KB; j++) acc[j] = 0;
  accum_partials<KA, KB>(pa, npa, pb, npb, acc);
  double out[KA + KB];
  block_sum<KA + KB, kRedBlock>(acc, out);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < KA + KB; j++) S->red[j] = out[j];
    if (stage >= 0) derive(S, stage);
  }
}

// Multi-workgroup form for long partial arrays (the SpMV's two partials per 256-row workgroup at
// config 5: ~23,000, which one workgroup summed in two dependent passes, 12.3 us for
// k_reduce<2,1>, profiles/r05/final/bicg_split.txt).  G workgroups each sum a contiguous slice
// of the partial indices (every thread its kRedMwPer loads back to back, then the block tree),
// publish the slice sums with agent-scope stores and take a ticket; the workgroup that draws the
// last ticket sums the G slice sums in slice order, derives and re-arms the ticket.  The sums are
// deterministic for a given (np, G): fixed slices, fixed trees, fixed final order.
// mw = [ticket word (8 B) | slice sums, G * (KA + KB) doubles], zeroed once by the context.
constexpr int kRedMwBlock = 256;
constexpr int kRedMwPer = 6;    // partials per thread and slice
constexpr int kRedMwMax = 64;   // workgroups at most (mw holds 1 + 64 * 5 doubles)
constexpr int kRedMwMin = 8192; // below this many partials the one-workgroup k_reduce

template <int KA, int KB>
__global__ __launch_bounds__(kRedMwBlock) void k_reduce_mw(const double *__restrict__ pa, int npa,
                                                           const double *__restrict__ pb, int npb,
                                                           Scalars *__restrict__ S, int stage,
                                                           double *mw) {
  constexpr int K = KA + KB;
  if (S->done && stage != 0 && stage != 10) {  // uniform: S changes only after the last ticket
    if (stage == 4 && blockIdx.x == 0 && threadIdx.x == 0) S->xpend = 0;
    return;
  }
  const int np = npa > npb ? npa : npb;
  const int per = (np + int(gridDim.x) - 1) / int(gridDim.x);
  const int lo = int(blockIdx.x) * per, hi = min(np, lo + per);
  double acc[K];
#pragma unroll
  for (int j = 0; j < K; j++) acc[j] = 0;
  for (int i0 = lo + int(threadIdx.x); i0 < hi; i0 += kRedMwPer * kRedMwBlock) {
    double va[kRedMwPer][K];
#pragma unroll
    for (int u = 0; u < kRedMwPer; u++) {
      const int i = i0 + u * kRedMwBlock;
#pragma unroll
      for (int j = 0; j < KA; j++) va[u][j] = (i < hi && i < npa) ? pa[size_t(i) * KA + j] : 0.0;
#pragma unroll
      for (int j = 0; j < KB; j++)
        va[u][KA + j] = (i < hi && i < npb) ? pb[size_t(i) * KB + j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kRedMwPer; u++)
#pragma unroll
      for (int j = 0; j < K; j++) acc[j] += va[u][j];
  }
  double out[K];
  block_sum<K, kRedMwBlock>(acc, out);
  unsigned *ticket = reinterpret_cast<unsigned *>(mw);
  double *slices = mw + 1;
  __shared__ int last;
  // publish as the dataflow kernels do (cdna_hip_programming.md Guideline 16): agent-scope
  // (write-through) stores drained by s_waitcnt before a relaxed ticket, agent-scope loads by the
  // last workgroup -- no release / acquire fence (the same time, 6.8 / 7.1 us at config 5,
  // gpurun_out r6c / r6d, and no L2 write-back / invalidate for the kernels around it)
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < K; j++)
      __hip_atomic_store(slices + size_t(blockIdx.x) * K + j, out[j], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  double v[K];
#pragma unroll
  for (int j = 0; j < K; j++)
    v[j] = int(threadIdx.x) < int(gridDim.x)
               ? __hip_atomic_load(slices + size_t(threadIdx.x) * K + j, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT)
               : 0.0;
  block_sum<K, kRedMwBlock>(v, out);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int j = 0; j < K; j++) S->red[j] = out[j];
    if (stage >= 0) derive(S, stage);
    __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void k_derive(Scalars *S, int stage) {
  if (threadIdx.x == 0) derive(S, stage);
}

__device__ void derive(Scalars *S, int stage) {
  if (stage == 0) {  // start: red = <r,r> with rt = r
    S->norm0 = S->norm = sqrt(S->red[0]);
    S->rho_new = S->red[0];
    S->rho = S->alpha = S->omega = 1.0;
    S->it_half = 0;
    S->iter = 0;
    S->breakdown = 0;
    S->xpend = 0;  // a solve that ended between k_update_fwd0 and stage 4 must not leak it
    S->done = (S->norm < S->reduction * S->norm0 || S->norm < 1e-30) ? 1 : 0;
    return;
  }
  if (stage == 10) {  // CG start: red = <r, r>
    S->norm0 = S->norm = sqrt(S->red[0]);
    S->it_half = 0;
    S->iter = 0;
    S->breakdown = 0;
    S->xpend = 0;
    S->done = S->norm0 < 1e-30 ? 1 : 0;
    return;
  }
  if (stage == 4) S->xpend = 0;  // the deferred x update (if any) was applied by k_update_xr
  if (S->done) return;
  if (stage == 11) {  // CG: rho = <M^{-1} r, r>
    S->rho = S->red[0];
    return;
  }
  if (stage == 12) {  // CG: lambda = rho / <p, A p>
    S->h = S->red[0];
    S->alpha = S->rho / S->h;
    return;
  }
  if (stage == 13) {  // CG: ||r|| after x += lambda p, r -= lambda A p
    S->norm = sqrt(S->red[0]);
    S->iter += 1;
    S->it_half = S->iter;
    if (S->norm < S->reduction * S->norm0 || S->norm < 1e-30) S->done = 1;
    return;
  }
  if (stage == 14) {  // CG: beta = <q, r> / rho (kept in omega), rho = <q, r>
    S->omega = S->red[0] / S->rho;
    S->rho = S->red[0];
    return;
  }
  if (stage == 31 || stage == 33) {  // the lagged second-half test (stage 4's checks)
    if (S->pending) {
      S->pending = 0;
      const double nr = S->red[stage == 31 ? 1 : 0];
      S->norm = sqrt(nr);
      if (S->norm < S->reduction * S->norm0 || S->norm < 1e-30) {
        S->done = 1;
      } else if (S->divguard && !(S->norm <= 1e10 * S->norm0)) {
        S->done = 2;
        S->breakdown = 4;
      } else if (fabs(S->rho) <= kEps) {
        S->done = 2;
        S->breakdown = 1;
      } else if (fabs(S->omega) <= kEps) {
        S->done = 2;
        S->breakdown = 2;
      }
      if (S->done) return;
    }
    if (stage == 33) return;
    stage = 1;  // then h as in stage 1
  }
  if (stage == 32) {  // red: <t,s>, <t,t>, <t,rt>, ||s||^2, <rt,s>
    S->norm = sqrt(S->red[3]);
    S->it_half += 0.5;
    if (S->norm < S->reduction * S->norm0) {
      S->done = 1;
      return;
    }
    S->omega = S->red[0] / S->red[1];
    S->it_half += 0.5;
    S->iter += 1;
    S->rho = S->rho_new;
    S->rho_new = S->red[4] - S->omega * S->red[2];
    S->pending = 1;
    return;
  }
  if (stage == 1) {  // h = <rt, v>
    S->h = S->red[0];
    if (fabs(S->h) < kEps) {
      S->done = 2;
      S->breakdown = 3;
      return;
    }
    S->alpha = S->rho_new / S->h;
  } else if (stage == 2) {  // first half step norm
    S->norm = sqrt(S->red[0]);
    S->it_half += 0.5;
    if (S->norm < S->reduction * S->norm0) S->done = 1;
  } else if (stage == 3) {  // omega = <t,r>/<t,t>
    S->omega = S->red[0] / S->red[1];
  } else if (stage == 23) {  // the first half step's test (red[2] = ||s||^2), then omega
    S->norm = sqrt(S->red[2]);
    S->it_half += 0.5;
    if (S->norm < S->reduction * S->norm0) {
      S->done = 1;
      return;
    }
    S->omega = S->red[0] / S->red[1];
  } else if (stage == 4) {  // second half step: red = <r,r>, <rt,r>
    S->norm = sqrt(S->red[0]);
    S->it_half += 0.5;
    S->iter += 1;
    S->rho = S->rho_new;
    S->rho_new = S->red[1];
    if (S->norm < S->reduction * S->norm0 || S->norm < 1e-30) {
      S->done = 1;
    } else if (S->divguard && !(S->norm <= 1e10 * S->norm0)) {  // diverged (or not finite)
      S->done = 2;
      S->breakdown = 4;
    } else if (fabs(S->rho) <= kEps) {
      S->done = 2;
      S->breakdown = 1;
    } else if (fabs(S->omega) <= kEps) {
      S->done = 2;
      S->breakdown = 2;
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_axpby(long long n, double a,
                                                  const double *__restrict__ x, double b,
                                                  const double *__restrict__ y,
                                                  double *__restrict__ out) {
  for (long long i = blockIdx.x * (long long)kBlock + threadIdx.x; i < n;
       i += (long long)gridDim.x * kBlock)
    out[i] = a * x[i] + (y ? b * y[i] : 0.0);
}

__global__ __launch_bounds__(kBlock) void k_pack(int n, int nf, const int *__restrict__ idx,
                                                 const double *__restrict__ x,
                                                 double *__restrict__ buf) {
  const int k = blockIdx.x * kBlock + threadIdx.x;
  if (k >= n * nf) return;
  buf[k] = x[size_t(idx[k / nf]) * nf + k % nf];
}

__global__ __launch_bounds__(kBlock) void k_gather_ext(int n, int nf, int nvg,
                                                       const int *__restrict__ l2g,
                                                       const double *__restrict__ ext,
                                                       double *__restrict__ in) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int g = l2g[i];
  for (int f = 0; f < nf; f++) in[size_t(i) * nf + f] = ext[size_t(f) * nvg + g];
}

__global__ __launch_bounds__(kBlock) void k_scatter_ext(int n, int nf, int nvg,
                                                        const int *__restrict__ l2g,
                                                        const double *__restrict__ in,
                                                        double *__restrict__ ext) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int g = l2g[i];
  for (int f = 0; f < nf; f++) ext[size_t(f) * nvg + g] = in[size_t(i) * nf + f];
}

inline dim3 rows_grid(int n) { return dim3((n + kBlock - 1) / kBlock); }

}  // namespace

int blas_nparts(long long n) {
  long long b = (n + 4LL * kBlock - 1) / (4LL * kBlock);
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return int(b);
}

#define PNP_PAT_DISPATCH(NF_, PAT_, CALL)                                 \
  do {                                                                    \
    if ((NF_) == 3 && (PAT_) == kPatPnp) {                                \
      constexpr int NFc = 3, PATc = kPatPnp;                              \
      CALL;                                                               \
    } else if ((NF_) == 3 && (PAT_) == kPatPnpIE) {                       \
      constexpr int NFc = 3, PATc = kPatPnpIE;                            \
      CALL;                                                               \
    } else if ((NF_) == 3 && (PAT_) == kPatPnpFD) {                       \
      constexpr int NFc = 3, PATc = kPatPnpFD;                            \
      CALL;                                                               \
    } else if ((NF_) == 3 && (PAT_) == kPatPnpIEFD) {                     \
      constexpr int NFc = 3, PATc = kPatPnpIEFD;                          \
      CALL;                                                               \
    } else if ((NF_) == 1) {                                              \
      constexpr int NFc = 1, PATc = kPatScalar;                           \
      CALL;                                                               \
    } else {                                                              \
      return hipErrorInvalidValue;                                        \
    }                                                                     \
  } while (0)

// SpMV shape (A/B knobs): PNP_SPMV_BATCH = 1, 2, 4 or 8 slots per batch, PNP_SPMV_LPR = 1 or 2
// lanes per row.  Default 2 lanes x 2-slot batches: ~2 % faster than 1 x 4
// (profiles/r01/ab_spmv_shape.log); 8-slot batches do not help.
static int spmv_batch() {
  static const int v = [] {
    const char *e = std::getenv("PNP_SPMV_BATCH");
    const int b = e ? std::atoi(e) : 2;
    return (b == 1 || b == 2 || b == 4 || b == 8) ? b : 2;
  }();
  return v;
}
// LDS-staged SpMV (k_spmv_lds, one lane per row) when the layout carries its lists (default;
// PNP_SPMV_LDS=0: the direct-gather k_spmv).  Config 3: 57.6 -> 52.4 us per SpMV, BiCGSTAB
// 338.7 -> 327.8 us/it, same result bits (profiles/r02/ab_spmv_lds.log)
static bool spmv_lds() {
  static const bool v = [] {
    const char *e = std::getenv("PNP_SPMV_LDS");
    return !(e && std::atoi(e) == 0);
  }();
  return v;
}
static int spmv_lpr() {
  static const int v = [] {
    const char *e = std::getenv("PNP_SPMV_LPR");
    return (e && std::atoi(e) == 1) ? 1 : 2;
  }();
  return v;
}
static bool spmv_uses_lds(const DevLayout &L) { return spmv_lds() && L.uptr != nullptr; }
// non-temporal loads of the matrix values (streamed once per launch; leaves L2 to the x
// gathers): SpMV -2..3 %, and the following sweeps -1..2 % (profiles/r01/ab_spmv_nt.log);
// PNP_SPMV_NT=0 turns it off (A/B)
static bool spmv_nt() {
  static const bool v = [] {
    const char *e = std::getenv("PNP_SPMV_NT");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <int NF, int PAT, int MODE>
static void spmv_launch(dim3 g, hipStream_t s, const DevLayout &L, const double *vals,
                        const double *x, double *y, const double *w, double *partials,
                        const double *w2, hipEvent_t t0, hipEvent_t t1) {
#define PNP_SPMV_GO(SBc, LPRc)                                                                 \
  hipLaunchKernelGGL((k_spmv<NF, PAT, MODE, SBc, LPRc>), dim3(g.x * LPRc), dim3(kBlock), 0, s, \
                     L, vals, x, y, w, partials, w2)
#define PNP_SPMV_GO2(SBc, LPRc, NTc)                                                        \
  hipLaunchKernelGGL((k_spmv<NF, PAT, MODE, SBc, LPRc, NTc>), dim3(g.x * LPRc), dim3(kBlock), \
                     0, s, L, vals, x, y, w, partials, w2)
  const int b = spmv_batch(), l = spmv_lpr();
  if (spmv_uses_lds(L)) {
    const size_t lds = size_t(SPMV_OWN_DIRECT && L.uown ? L.unmax : L.umax) * NF * sizeof(double);
    hipExtLaunchKernelGGL((k_spmv_lds<NF, PAT, MODE, 2, 1>), g, dim3(kBlock), lds, s, t0, t1, 0, L,
                          vals, x, y, w, partials, w2);
    return;
  }
  // the other forms: the timer events as plain markers around the launch
  if (t0) hipEventRecord(t0, s);
  struct Stop {
    hipEvent_t e;
    hipStream_t s;
    ~Stop() {
      if (e) hipEventRecord(e, s);
    }
  } stop{t1, s};
  if (spmv_nt() && l == 2 && b == 2) {
    PNP_SPMV_GO2(2, 2, 1);
    return;
  }
  if (l == 2) {
    if (b == 8) PNP_SPMV_GO(8, 2);
    else if (b == 2) PNP_SPMV_GO(2, 2);
    else if (b == 1) PNP_SPMV_GO(1, 2);
    else PNP_SPMV_GO(4, 2);
  } else {
    if (b == 8) PNP_SPMV_GO(8, 1);
    else if (b == 2) PNP_SPMV_GO(2, 1);
    else if (b == 1) PNP_SPMV_GO(1, 1);
    else PNP_SPMV_GO(4, 1);
  }
#undef PNP_SPMV_GO
#undef PNP_SPMV_GO2
}

// partials per SpMV launch at most (buffer sizing; launch_spmv returns the actual count)
int spmv_parts(int nrows) { return int(rows_grid(nrows).x) * 2; }

hipError_t launch_spmv(const DevLayout &L, int nf, int pat, const double *vals, const double *x,
                       double *y, int mode, const double *w, double *partials, int *nparts,
                       hipStream_t s, const double *w2, hipEvent_t t0, hipEvent_t t1) {
  if (L.blkcount < 0) {  // an empty block subset (e.g. a rank without interior blocks)
    if (nparts) *nparts = 0;
    return hipSuccess;
  }
  dim3 g = L.blkcount > 0 ? dim3(L.blkcount) : rows_grid(L.n_owned);
  if (nparts) *nparts = int(g.x) * (spmv_uses_lds(L) ? 2 : spmv_lpr());
  if (L.n_owned == 0) return hipSuccess;
  PNP_PAT_DISPATCH(nf, pat, {
    if (mode == 0)
      (spmv_launch<NFc, PATc, 0>)(g, s, L, vals, x, y, w, partials, w2, t0, t1);
    else if (mode == 1)
      (spmv_launch<NFc, PATc, 1>)(g, s, L, vals, x, y, w, partials, w2, t0, t1);
    else if (mode == 2)
      (spmv_launch<NFc, PATc, 2>)(g, s, L, vals, x, y, w, partials, w2, t0, t1);
    else if (mode == 4)
      (spmv_launch<NFc, PATc, 4>)(g, s, L, vals, x, y, w, partials, w2, t0, t1);
    else
      (spmv_launch<NFc, PATc, 3>)(g, s, L, vals, x, y, w, partials, w2, t0, t1);
  });
  return hipGetLastError();
}

hipError_t launch_jacobi(const DevLayout &L, int nf, int pat, const double *vals, const double *d,
                         double *v, hipStream_t s) {
  if (L.n_owned == 0) return hipSuccess;
  PNP_PAT_DISPATCH(nf, pat, {
    hipLaunchKernelGGL((k_jacobi<NFc, PATc>), rows_grid(L.n_owned), dim3(kBlock), 0, s, L, vals,
                       d, v);
  });
  return hipGetLastError();
}

// sweep kernel shape: lanes per row x slot batch (PNP_SWEEP = "LPRxB": 1x2, 2x2, 2x4, default
// 1x4; the other shapes measured in round 1 lost), and non-temporal loads of the
// L/U values in the default shape (PNP_SWEEP_NT=0/1, A/B)
static int sweep_cfg() {
  static const int v = [] {
    const char *e = std::getenv("PNP_SWEEP");
    int l = 1, b = 4;
    if (e && std::sscanf(e, "%dx%d", &l, &b) != 2) l = 1, b = 4;
    const int code = l * 16 + b;
    return (code == 18 || code == 34 || code == 36 || code == 24 || code == 40) ? code : 20;
  }();
  return v;
}
static bool sweep_nt() {  // default on: ILU0 apply -7 %, SGS -7 % (profiles/r01/ab_sweep_nt.log)
  static const bool v = [] {
    const char *e = std::getenv("PNP_SWEEP_NT");
    return !(e && e[0] == '0');
  }();
  return v;
}

#define PNP_LPR_DISPATCH(CALL)                     \
  do {                                             \
    switch (sweep_cfg()) {                         \
      case 18: {                                   \
        constexpr int LPRc = 1, Bc = 2, NTc = 0;   \
        CALL;                                      \
      } break;                                     \
      case 34: {                                   \
        constexpr int LPRc = 2, Bc = 2, NTc = 0;   \
        CALL;                                      \
      } break;                                     \
      case 24: {                                   \
        constexpr int LPRc = 1, Bc = 8, NTc = 1;   \
        CALL;                                      \
      } break;                                     \
      case 40: {                                   \
        constexpr int LPRc = 2, Bc = 8, NTc = 1;   \
        CALL;                                      \
      } break;                                     \
      case 36: {                                   \
        constexpr int LPRc = 2, Bc = 4, NTc = 1;   \
        CALL;                                      \
      } break;                                     \
      default:                                     \
        if (sweep_nt()) {                          \
          constexpr int LPRc = 1, Bc = 4, NTc = 1; \
          CALL;                                    \
        } else {                                   \
          constexpr int LPRc = 1, Bc = 4, NTc = 0; \
          CALL;                                    \
        }                                          \
        break;                                     \
    }                                              \
  } while (0)

hipError_t launch_sgs(const DevLayout &L, const int *cp, int nf, int pat, const double *lv,
                      const double *uv, const double *d, double *v, double *t, hipStream_t s) {
  if (L.n_owned == 0) return hipSuccess;
  const int nc = L.ncolors;
  // the forward sweep writes every owned row exactly once and reads only rows of earlier
  // colours, so v needs no zeroing (ISTL starts the sweep from v = 0)
  PNP_PAT_DISPATCH(nf, pat, PNP_LPR_DISPATCH({
    auto go = [&](auto kind, int c) {
      const int n = cp[c + 1] - cp[c];
      if (n > 0)
        hipLaunchKernelGGL((k_sgs_color<NFc, PATc, decltype(kind)::value, LPRc, Bc, NTc>),
                           rows_grid(n * LPRc), dim3(kBlock), 0, s, L, cp[c], n, lv, uv, d, v, t);
    };
    for (int c = 0; c < nc - 1; c++) go(std::integral_constant<int, 1>(), c);
    go(std::integral_constant<int, 2>(), nc - 1);  // last colour: forward + backward
    for (int c = nc - 2; c >= 0; c--) go(std::integral_constant<int, 0>(), c);
  }));
  return hipGetLastError();
}

hipError_t launch_ilu0_factor(const DevLayout &L, const int *cp, int nf, int pat, double *lu,
                              hipStream_t s) {
  if (L.n_owned == 0) return hipSuccess;
  PNP_PAT_DISPATCH(nf, pat, {
    for (int c = 0; c < L.ncolors; c++) {
      int n = cp[c + 1] - cp[c];
      if (n > 0)
        hipLaunchKernelGGL((k_ilu0_factor<NFc, PATc>), rows_grid(n), dim3(kBlock), 0, s, L, cp[c],
                           cp[c + 1], lu);
    }
  });
  return hipGetLastError();
}

hipError_t launch_ilu0_factor_fused(const DevLayout &L, const int *cp, int nf, int pat,
                                    const double *kvals, const int *rowoff, const int *rowcol,
                                    double *aos, void *lv, void *uv, int f32, hipStream_t s) {
  if (L.n_owned == 0) return hipSuccess;
  // own rows in LDS (64 rows per workgroup) when every fan fits KMAX slots, else in the scratch
  const int ms = L.max_slots;
  auto run = [&](auto vt) -> hipError_t {
    using VT = decltype(vt);
    PNP_PAT_DISPATCH(nf, pat, {
      auto go = [&](auto kmax) {
        constexpr int K = decltype(kmax)::value;
        constexpr int TB = K > 0 ? 64 : kBlock;
        for (int c = 0; c < L.ncolors; c++) {
          int n = cp[c + 1] - cp[c];
          if (n > 0)
            hipLaunchKernelGGL((k_ilu0_factor_fused<NFc, PATc, VT, K, TB>), dim3((n + TB - 1) / TB),
                               dim3(TB), 0, s, L, cp[c], cp[c + 1], kvals, rowoff, rowcol, aos,
                               static_cast<VT *>(lv), static_cast<VT *>(uv));
        }
      };
      if (ms <= 10)
        go(std::integral_constant<int, 10>());
      else if (ms <= 16)
        go(std::integral_constant<int, 16>());
      else
        go(std::integral_constant<int, 0>());
    });
    return hipGetLastError();
  };
  return f32 == 2 ? run(bf16s()) : f32 ? run(float()) : run(double());
}

// LDS-staged sweeps when the layout carries their lists and the sweep shape is the default one
// lane per row (PNP_ILU_LDS=0: the direct gathers, A/B)
static bool ilu_lds() {
  static const bool v = [] {
    const char *e = std::getenv("PNP_ILU_LDS");
    return !(e && e[0] == '0');
  }();
  return v;
}

// PNP_ILU_LDS_B: force the LDS sweeps' slot batch (2, 3, 4 or 8; 0 / unset: by size)
static int ilu_lds_bsel() {
  static const int v = [] {
    const char *e = std::getenv("PNP_ILU_LDS_B");
    const int b = e ? atoi(e) : 0;
    return (b == 2 || b == 3 || b == 4 || b == 8) ? b : 0;
  }();
  return v;
}

hipError_t launch_ilu0_apply(const DevLayout &L, const int *cp, int nf, int pat, const void *lvp,
                             const void *uvp, const double *d, double *v, hipStream_t s,
                             int c_first, const double *add, double *out, int f32, float *yf,
                             hipEvent_t t0, hipEvent_t t1) {
  if (L.n_owned == 0) return hipSuccess;
  if (yf && f32 != 2) return hipErrorInvalidValue;  // the bf16-factor mode only
  const int nc = L.ncolors;
  if (ilu_lds() && L.lsx_ptr && sweep_cfg() == 20) {
    // block numbering of the lists: colour by colour, 256-row blocks
    int blk0[256 + 1];
    if (nc > 256) return hipErrorInvalidValue;
    blk0[0] = 0;
    for (int c = 0; c < nc; c++) blk0[c + 1] = blk0[c] + (cp[c + 1] - cp[c] + kBlock - 1) / kBlock;
    const size_t lds = size_t(L.sx_max) * nf * sizeof(double);
    // the timer events: t0 at the first launch's start, t1 at the last launch's end (launch
    // order: forward colours c_first .. nc-2, the last colour, backward colours nc-2 .. 0)
    int first_c = -1;
    int last_c = -1;
    for (int c = c_first; c < nc; c++)
      if (cp[c + 1] > cp[c]) {
        if (first_c < 0) first_c = c;
        last_c = c;
      }
    for (int c = 0; c < nc - 1; c++)  // the backward launches end with the lowest colour
      if (cp[c + 1] > cp[c]) {
        last_c = -(c + 1);  // encoded: backward launch of colour c
        break;
      }
    auto run = [&](auto vt, auto *yv) -> hipError_t {
      using VT = decltype(vt);
      using YT = std::remove_pointer_t<decltype(yv)>;
      const VT *lv = static_cast<const VT *>(lvp), *uv = static_cast<const VT *>(uvp);
      // slot batch (the sums run over the slots in order whatever the batch, so bitwise alike):
      // 2 -- round 3 chose 3 above 1.5 M rows (config 5 215 -> 207 us, profiles/r03/
      // ab_ilu_lds_batch_r5n.log), but with the bfloat16 factors 2 is faster there too (config 5
      // 181.7 -> 177.6 us per apply, interleaved twice, gpurun_out/r6c5/ab_cfg5.log); 4 and 8
      // lose at both sizes.  PNP_ILU_LDS_B = 2 / 3 / 4 / 8 forces one
      const int kBsel = ilu_lds_bsel() ? ilu_lds_bsel() : 2;
      PNP_PAT_DISPATCH(nf, pat, {
        auto go = [&](auto kind, int c) {
          const int n = cp[c + 1] - cp[c];
          if (n <= 0) return;
          constexpr int K = decltype(kind)::value;
          const hipEvent_t e0 = (K == kIluBwd || c != first_c) ? nullptr : t0;
          const hipEvent_t e1 = (K == kIluBwd ? last_c == -(c + 1) : last_c == c) ? t1 : nullptr;
          auto launch = [&](auto ntc, auto bc) {
            constexpr int NT = decltype(ntc)::value;
            constexpr int BB = decltype(bc)::value;
            if (add && K != kIluFwd)
              hipExtLaunchKernelGGL((k_ilu0_solve_lds<NFc, PATc, K, BB, NT, 1, VT, YT>),
                                    rows_grid(n), dim3(kBlock), lds, s, e0, e1, 0, L, cp[c],
                                    cp[c + 1], blk0[c], lv, uv, d, v, add, out, yv);
            else
              hipExtLaunchKernelGGL((k_ilu0_solve_lds<NFc, PATc, K, BB, NT, 0, VT, YT>),
                                    rows_grid(n), dim3(kBlock), lds, s, e0, e1, 0, L, cp[c],
                                    cp[c + 1], blk0[c], lv, uv, d, v, nullptr, nullptr, yv);
          };
          auto batch = [&](auto ntc) {
            if (kBsel == 8)
              launch(ntc, std::integral_constant<int, 8>());
            else if (kBsel == 4)
              launch(ntc, std::integral_constant<int, 4>());
            else if (kBsel == 3)
              launch(ntc, std::integral_constant<int, 3>());
            else
              launch(ntc, std::integral_constant<int, 2>());
          };
          if (sweep_nt())
            batch(std::integral_constant<int, 1>());
          else
            batch(std::integral_constant<int, 0>());
        };
        for (int c = c_first; c < nc - 1; c++) go(std::integral_constant<int, kIluFwd>(), c);
        go(std::integral_constant<int, kIluLast>(), nc - 1);
        for (int c = nc - 2; c >= 0; c--) go(std::integral_constant<int, kIluBwd>(), c);
      });
      return hipGetLastError();
    };
    if (yf) return run(bf16s(), yf);
    return f32 == 2 ? run(bf16s(), v) : f32 ? run(float(), v) : run(double(), v);
  }
  // the direct-gather form: the timer events as plain markers around its launches
  if (t0) hipEventRecord(t0, s);
  struct Stop {
    hipEvent_t e;
    hipStream_t s;
    ~Stop() {
      if (e) hipEventRecord(e, s);
    }
  } stop{t1, s};
  auto run = [&](auto vt, auto *yv) -> hipError_t {
    using VT = decltype(vt);
    using YT = std::remove_pointer_t<decltype(yv)>;
    const VT *lv = static_cast<const VT *>(lvp), *uv = static_cast<const VT *>(uvp);
    PNP_PAT_DISPATCH(nf, pat, PNP_LPR_DISPATCH({
      auto go = [&](auto kind, int c) {
        const int n = cp[c + 1] - cp[c];
        if (n <= 0) return;
        constexpr int K = decltype(kind)::value;
        if (add && K != kIluFwd)
          hipLaunchKernelGGL((k_ilu0_solve<NFc, PATc, K, LPRc, Bc, NTc, 1, VT, YT>),
                             rows_grid(n * LPRc), dim3(kBlock), 0, s, L, cp[c], cp[c + 1], lv, uv,
                             d, v, add, out, yv);
        else
          hipLaunchKernelGGL((k_ilu0_solve<NFc, PATc, K, LPRc, Bc, NTc, 0, VT, YT>),
                             rows_grid(n * LPRc), dim3(kBlock), 0, s, L, cp[c], cp[c + 1], lv, uv,
                             d, v, nullptr, nullptr, yv);
      };
      // the last colour's backward step runs in its forward launch (kIluLast); c_first = 1:
      // colour 0's forward step was done by launch_update_fwd0
      for (int c = c_first; c < nc - 1; c++) go(std::integral_constant<int, kIluFwd>(), c);
      go(std::integral_constant<int, kIluLast>(), nc - 1);
      for (int c = nc - 2; c >= 0; c--) go(std::integral_constant<int, kIluBwd>(), c);
    }));
    return hipGetLastError();
  };
  if (yf) return run(bf16s(), yf);
  return f32 == 2 ? run(bf16s(), v) : f32 ? run(float(), v) : run(double(), v);
}

// every workgroup of a grid resident at once: CUs x the occupancy at this LDS size (capped by n)
template <typename K>
static int resident_grid(K kern, size_t lds, int n) {
  int dev = 0, cus = 0, per = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, kBlock, lds);
  return std::min(n, std::max(1, cus * std::max(1, per)));
}

hipError_t launch_ilu0_flow(const DevLayout &L, const IluFlow &F, int nf, int pat, const void *lvp,
                            const void *uvp, const double *d, double *v, hipStream_t s, int f32) {
  if (F.nunits <= 0) return hipSuccess;
  if (!L.lsx_ptr || F.nstages > kIluFlowMaxStages) return hipErrorInvalidValue;
  // flags and the ticket, one block from the allocation's start, a multiple of 16 bytes
  hipError_t e = hipMemsetAsync(F.flags, 0, (size_t(F.nunits + 1) * 4 + 15) & ~size_t(15), s);
  if (e != hipSuccess) return e;
  const size_t lds = 16 + size_t(L.sx_max) * nf * sizeof(double);
  const int kBsel = ilu_lds_bsel() ? ilu_lds_bsel() : (L.n_owned > 1500000 ? 3 : 2);
  auto run = [&](auto vt) -> hipError_t {
    using VT = decltype(vt);
    const VT *lv = static_cast<const VT *>(lvp), *uv = static_cast<const VT *>(uvp);
    auto go = [&](auto kern) {
      const int grid = F.persistent ? resident_grid(kern, lds, F.nunits) : F.nunits;
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), lds, s, L, F, lv, uv, d, v);
    };
    PNP_PAT_DISPATCH(nf, pat, {
      if (kBsel == 3)
        go(k_ilu0_flow<NFc, PATc, 3, VT>);
      else
        go(k_ilu0_flow<NFc, PATc, 2, VT>);
    });
    return hipGetLastError();
  };
  return f32 == 2 ? run(bf16s()) : f32 ? run(float()) : run(double());
}

hipError_t launch_update_fwd0(const DevLayout &L, int nf, int pat, int c0_end, const Scalars *S,
                              int which, int first, double *x, const double *yin, double *r,
                              const double *v, double *p, const void *uvp, double *yout,
                              double *partials, int *nparts, hipStream_t s, int f32,
                              const double *rt, float *youtf) {
  const dim3 g = rows_grid(L.n_owned);
  Scalars *Sw = const_cast<Scalars *>(S);  // which 1 with x = null sets S->xpend
  if (nparts) *nparts = int(g.x);
  if (L.n_owned == 0) return hipSuccess;
  if (youtf && f32 != 2) return hipErrorInvalidValue;  // the bf16-factor mode only
  auto run = [&](auto vt, auto *yo) -> hipError_t {
    using VT = decltype(vt);
    using YT = std::remove_pointer_t<decltype(yo)>;
    const VT *uv = static_cast<const VT *>(uvp);
    PNP_PAT_DISPATCH(nf, pat, {
      if (which == 0)
        hipLaunchKernelGGL((k_update_fwd0<NFc, PATc, 0, VT, YT>), g, dim3(kBlock), 0, s, L, c0_end,
                           Sw, first, x, yin, r, v, p, uv, yo, partials, nullptr);
      else
        hipLaunchKernelGGL((k_update_fwd0<NFc, PATc, 1, VT, YT>), g, dim3(kBlock), 0, s, L, c0_end,
                           Sw, first, x, yin, r, v, p, uv, yo, partials, rt);
    });
    return hipGetLastError();
  };
  if (youtf) return run(bf16s(), youtf);
  return f32 == 2 ? run(bf16s(), yout) : f32 ? run(float(), yout) : run(double(), yout);
}

hipError_t launch_split(const DevLayout &L, int nf, int pat, int from_k, const double *src,
                        const int *lsrc, long long ln, const int *usrc, long long un, void *lv,
                        void *uv, hipStream_t s, int f32) {
  const long long n = ln + un;
  if (n == 0) return hipSuccess;
  const dim3 g(unsigned((n + kBlock - 1) / kBlock));
  PNP_PAT_DISPATCH(nf, pat, {
    if (from_k)
      hipLaunchKernelGGL((k_split<NFc, PATc, 1>), g, dim3(kBlock), 0, s, L, src, lsrc, ln, usrc,
                         un, static_cast<double *>(lv), static_cast<double *>(uv));
    else if (f32 == 2)
      hipLaunchKernelGGL((k_split<NFc, PATc, 0, bf16s>), g, dim3(kBlock), 0, s, L, src, lsrc, ln,
                         usrc, un, static_cast<bf16s *>(lv), static_cast<bf16s *>(uv));
    else if (f32)
      hipLaunchKernelGGL((k_split<NFc, PATc, 0, float>), g, dim3(kBlock), 0, s, L, src, lsrc, ln,
                         usrc, un, static_cast<float *>(lv), static_cast<float *>(uv));
    else
      hipLaunchKernelGGL((k_split<NFc, PATc, 0>), g, dim3(kBlock), 0, s, L, src, lsrc, ln, usrc,
                         un, static_cast<double *>(lv), static_cast<double *>(uv));
  });
  return hipGetLastError();
}

hipError_t launch_expand(const DevLayout &L, int nf, int pat, const double *vals, double *lu,
                         hipStream_t s) {
  if (L.n_owned == 0) return hipSuccess;
  PNP_PAT_DISPATCH(nf, pat, {
    hipLaunchKernelGGL((k_expand<NFc, PATc>), rows_grid(L.n_owned), dim3(kBlock), 0, s, L, vals,
                       lu);
  });
  return hipGetLastError();
}

hipError_t launch_update_p(long long n, const Scalars *S, const double *r, const double *v,
                           double *p, int first, hipStream_t s) {
  hipLaunchKernelGGL(k_update_p, dim3(blas_nparts(n)), dim3(kBlock), 0, s, n, S, r, v, p, first);
  return hipGetLastError();
}

hipError_t launch_cg_update_p(long long n, const Scalars *S, const double *q, double *p,
                              hipStream_t s) {
  hipLaunchKernelGGL(k_cg_update_p, dim3(blas_nparts(n)), dim3(kBlock), 0, s, n, S, q, p);
  return hipGetLastError();
}

hipError_t launch_update_xr(long long n, const Scalars *S, int which, double *x, const double *y,
                            double *r, const double *v, const double *rt, double *partials,
                            hipStream_t s, const double *y1) {
  if (rt)
    hipLaunchKernelGGL(k_update_xr<1>, dim3(blas_nparts(n)), dim3(kBlock), 0, s, n, S, which, x, y,
                       r, v, rt, partials, y1);
  else
    hipLaunchKernelGGL(k_update_xr<0>, dim3(blas_nparts(n)), dim3(kBlock), 0, s, n, S, which, x, y,
                       r, v, rt, partials, y1);
  return hipGetLastError();
}

hipError_t launch_dot(long long n, const double *a, const double *b, int two, double *partials,
                      hipStream_t s) {
  if (two)
    hipLaunchKernelGGL(k_dot<1>, dim3(blas_nparts(n)), dim3(kBlock), 0, s, n, a, b, partials);
  else
    hipLaunchKernelGGL(k_dot<0>, dim3(blas_nparts(n)), dim3(kBlock), 0, s, n, a, b, partials);
  return hipGetLastError();
}

// the multi-workgroup grid for np partials, or 0 for the one-workgroup k_reduce.
// PNP_RED_MW_MIN (test hook, read once) lowers the threshold, so that small systems exercise the
// multi-workgroup path (tests/test_gpu_reduce_mw.py)
static int reduce_mw_min() {
  static const int v = [] {
    const char *e = std::getenv("PNP_RED_MW_MIN");
    return e ? std::max(1, std::atoi(e)) : kRedMwMin;
  }();
  return v;
}
static int reduce_mw_grid(int np, const double *mw) {
  if (!mw || np < reduce_mw_min()) return 0;
  const int g = (np + kRedMwPer * kRedMwBlock - 1) / (kRedMwPer * kRedMwBlock);
  return g < 2 ? 0 : (g > kRedMwMax ? kRedMwMax : g);
}

hipError_t launch_reduce(const double *partials, int nparts, int k, Scalars *S, hipStream_t s,
                         int derive_stage, double *mw) {
  if (const int G = reduce_mw_grid(nparts, mw)) {
    const dim3 g(G), b(kRedMwBlock);
    switch (k) {
      case 1: hipLaunchKernelGGL((k_reduce_mw<1, 0>), g, b, 0, s, partials, nparts, nullptr, 0, S, derive_stage, mw); break;
      case 2: hipLaunchKernelGGL((k_reduce_mw<2, 0>), g, b, 0, s, partials, nparts, nullptr, 0, S, derive_stage, mw); break;
      case 3: hipLaunchKernelGGL((k_reduce_mw<3, 0>), g, b, 0, s, partials, nparts, nullptr, 0, S, derive_stage, mw); break;
      case 4: hipLaunchKernelGGL((k_reduce_mw<4, 0>), g, b, 0, s, partials, nparts, nullptr, 0, S, derive_stage, mw); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  const dim3 g(1), b(kRedBlock);
  switch (k) {
    case 1: hipLaunchKernelGGL((k_reduce<1, 0>), g, b, 0, s, partials, nparts, nullptr, 0, S, derive_stage); break;
    case 2: hipLaunchKernelGGL((k_reduce<2, 0>), g, b, 0, s, partials, nparts, nullptr, 0, S, derive_stage); break;
    case 3: hipLaunchKernelGGL((k_reduce<3, 0>), g, b, 0, s, partials, nparts, nullptr, 0, S, derive_stage); break;
    case 4: hipLaunchKernelGGL((k_reduce<4, 0>), g, b, 0, s, partials, nparts, nullptr, 0, S, derive_stage); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_reduce2(const double *pa, int npa, int ka, const double *pb, int npb, int kb,
                          Scalars *S, hipStream_t s, int derive_stage, double *mw) {
  if (const int G = reduce_mw_grid(npa > npb ? npa : npb, mw)) {
    const dim3 g(G), b(kRedMwBlock);
    if (ka == 2 && kb == 1)
      hipLaunchKernelGGL((k_reduce_mw<2, 1>), g, b, 0, s, pa, npa, pb, npb, S, derive_stage, mw);
    else if (ka == 1 && kb == 1)
      hipLaunchKernelGGL((k_reduce_mw<1, 1>), g, b, 0, s, pa, npa, pb, npb, S, derive_stage, mw);
    else if (ka == 2 && kb == 2)
      hipLaunchKernelGGL((k_reduce_mw<2, 2>), g, b, 0, s, pa, npa, pb, npb, S, derive_stage, mw);
    else if (ka == 3 && kb == 2)
      hipLaunchKernelGGL((k_reduce_mw<3, 2>), g, b, 0, s, pa, npa, pb, npb, S, derive_stage, mw);
    else
      return hipErrorInvalidValue;
    return hipGetLastError();
  }
  const dim3 g(1), b(kRedBlock);
  if (ka == 2 && kb == 1)
    hipLaunchKernelGGL((k_reduce<2, 1>), g, b, 0, s, pa, npa, pb, npb, S, derive_stage);
  else if (ka == 1 && kb == 1)
    hipLaunchKernelGGL((k_reduce<1, 1>), g, b, 0, s, pa, npa, pb, npb, S, derive_stage);
  else if (ka == 2 && kb == 2)
    hipLaunchKernelGGL((k_reduce<2, 2>), g, b, 0, s, pa, npa, pb, npb, S, derive_stage);
  else if (ka == 3 && kb == 2)
    hipLaunchKernelGGL((k_reduce<3, 2>), g, b, 0, s, pa, npa, pb, npb, S, derive_stage);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_derive(Scalars *S, int stage, hipStream_t s) {
  hipLaunchKernelGGL(k_derive, dim3(1), dim3(64), 0, s, S, stage);
  return hipGetLastError();
}

hipError_t launch_axpby(long long n, double a, const double *x, double b, const double *y,
                        double *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_axpby, dim3(blas_nparts(n)), dim3(kBlock), 0, s, n, a, x, b, y, out);
  return hipGetLastError();
}

hipError_t launch_pack(int n, int nf, const int *idx, const double *x, double *buf,
                       hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack, rows_grid(n * nf), dim3(kBlock), 0, s, n, nf, idx, x, buf);
  return hipGetLastError();
}

hipError_t launch_gather_ext(int n, int nf, int nvg, const int *l2g, const double *ext,
                             double *in, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_ext, rows_grid(n), dim3(kBlock), 0, s, n, nf, nvg, l2g, ext, in);
  return hipGetLastError();
}

hipError_t launch_scatter_ext(int n, int nf, int nvg, const int *l2g, const double *in,
                              double *ext, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_ext, rows_grid(n), dim3(kBlock), 0, s, n, nf, nvg, l2g, in, ext);
  return hipGetLastError();
}

}  // namespace pnp

namespace pnp {
// Cache scrub for cache-cold timings (bench): every lane streams 16-B loads over n2 double2 and
// folds them; the fold is stored only if it equals a value the zero-filled buffer cannot give,
// so the loads stay live and nothing is written.  Lines brought in are clean, so the matrix lines
// a previous assembly left dirty in the L2 / Infinity Cache are written back during the scrub,
// not inside the next timed launch.
__global__ void __launch_bounds__(256) k_scrub(const double2 *__restrict__ p, long long n2,
                                               double *sink) {
  double a = 0;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n2; i += 256LL * gridDim.x) {
    const double2 t = p[i];
    a += t.x + t.y;
  }
  if (a == 1.2345e300) sink[0] = a;
}

hipError_t launch_scrub(const double *buf, long long n, double *sink, hipStream_t s) {
  if (n < 2) return hipSuccess;
  hipLaunchKernelGGL(k_scrub, dim3(4096), dim3(256), 0, s, reinterpret_cast<const double2 *>(buf),
                     n / 2, sink);
  return hipGetLastError();
}
}  // namespace pnp

namespace pnp {
namespace {
// device CSR view of the assembled Jacobian: entry k takes value v of block (row, slot) =
// (src[k] >> 6, src[k] & 63), expanded from the stored form and row-masked
template <int NF, int PAT>
__global__ __launch_bounds__(kBlock) void k_csr_fill(DevLayout L, const double *__restrict__ vals,
                                                     long long nnz, const int *__restrict__ src,
                                                     const unsigned char *__restrict__ vidx,
                                                     double *__restrict__ out) {
  constexpr int NV = popc9(PAT), NK = nks_of(PAT);
  const long long k = blockIdx.x * (long long)kBlock + threadIdx.x;
  if (k >= nnz) return;
  const int code = src[k], row = code >> 6, slot = code & 63;
  const int chunk = row / kRows, lane = row % kRows;
  double K[NK], B[NV];
  load_vals<NK>(vals + (size_t(L.chunk_off[chunk]) + size_t(slot) * kRows) * NK, lane, K);
  expand_k<PAT>(K, B);
  mask_rows<NF, PAT>(B, row_mask<NF>(L, row), slot == 0);
  out[k] = B[vidx[k]];
}
}  // namespace

hipError_t launch_csr_fill(const DevLayout &L, int nf, int pat, const double *vals, long long nnz,
                           const int *src, const unsigned char *vidx, double *out, hipStream_t s) {
  if (nnz == 0) return hipSuccess;
  const dim3 g(unsigned((nnz + kBlock - 1) / kBlock));
  PNP_PAT_DISPATCH(nf, pat, {
    hipLaunchKernelGGL((k_csr_fill<NFc, PATc>), g, dim3(kBlock), 0, s, L, vals, nnz, src, vidx,
                       out);
  });
  return hipGetLastError();
}
}  // namespace pnp
