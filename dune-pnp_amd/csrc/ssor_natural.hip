// ISTL SeqSSOR (k = 1, omega = 1) in the reference's own DOF order (PNP_PREC_SSOR_NATURAL).
//
// The reference's default linear solver is ISTLBackend_NOVLP_BCGS_SSORk (LINEARSOLVER BCGS_SSORk,
// src/instationary_pnp_from_pb_md.hh:30-31,188-191; the PB phase of src/stationary_pnp_from_pb.hh:
// 168-169): BiCGSTAB preconditioned by one SSOR sweep on the local BCRS matrix, rows visited in the
// lexicographic order of the GridFunctionSpace ([phi | c+ | c-] over the vertex order).  Per row,
// dune-istl's bsorf / bsorb (istl/gsetc.hh) compute
//     rhs = d_i - sum_j A_ij v_j   (all stored columns in ascending order, the diagonal included)
//     v_i += omega * (rhs / A_ii)
// forward over i = 0 .. n-1 from v = 0 (BiCGSTAB zeroes its y before _prec.apply), then backward
// over i = n-1 .. 0.  The multicolour sweeps of linalg.hip (PNP_PREC_SSOR) visit rows in another
// order, so their iterates and iteration counts differ from the reference's; this file restates the
// sequential recurrence exactly.
//
// Schedule: a row depends on the rows it couples to (either direction of the pattern) that come
// before it in the sweep.  Rows are grouped into levels (host, once per block pattern: the longest
// chain of such dependencies ending in the row), and every level is one launch (kL lanes per row,
// below).
// A row therefore reads its earlier neighbours' new values and its later neighbours' values before
// they are touched -- zero in the forward sweep, the forward result in the backward sweep -- i.e.
// exactly the sequential sweep's operands.  Each row's sum runs over its CSR row in ascending column
// order with no fused multiply-add (this file is compiled with -ffp-contract=off), the oracle's
// operand order (oracle/pnp_oracle.c prec_apply): on the same matrix the result is the oracle's bit
// for bit.  Depth at test/pore_pnp/pore.msh k=3: 131 levels per field sweep.
//
// Multi-GPU: each rank sweeps its owned rows; columns of other ranks' DOFs read zero (block-Jacobi
// across ranks, as the reference's NOVLP SSOR acts on the local matrix only).
#include "kernels.h"

namespace pnp {

namespace {
constexpr int kB = 256;

// A level is a short chain of dependent memory round trips per row, whatever its size, so the
// sweep is laid out to keep that chain at two: the level's entries are a column-major ELL of its
// rows (NatSweep: coalesced column / value-index loads that need nothing but the position, padding
// marked by index -1), and each row is served by kL lanes, lane j loading entries j, j + kL, ...
// (kS per pass) and forming their products.  Round trip 1: the row record and the ELL slots; round
// trip 2: d, the diagonal and the gathered values.  The row's first lane then subtracts the
// products in column order, taken from the other lanes by shuffles: the oracle's operations in
// the oracle's order (only loads and products move; a padding slot contributes rhs - (+0.0), which
// is rhs bit for bit).  One thread per row through rowptr, one entry at a time, took 14.1 ms per
// application at config 3 (profiles/r03/ssor_natural_r3t.log).
#ifndef NAT_KL
#define NAT_KL 8  // lanes per row (build-flag A/B knob)
#endif
constexpr int kL = NAT_KL, kS = (24 + kL - 1) / kL, kC = kS * kL;  // PNP rows: <= 21 entries
__global__ void __launch_bounds__(kB)
    k_ssor_nat_level(const int4 *__restrict__ info, const int *__restrict__ ecol,
                     const int *__restrict__ eidx, int n, int width,
                     const double *__restrict__ val, const double *__restrict__ d,
                     double *__restrict__ v) {
  const int g = blockIdx.x * kB + threadIdx.x, t = g / kL, j = g % kL;
  const bool live = t < n;  // whole rows per wavefront: kL divides 64
  const bool head = live && j == 0;
  const int4 I = head ? info[t] : make_int4(0, 0, 0, 0);
  const int base = (threadIdx.x % 64) - j;  // the row's first lane in the wavefront
  double rhs = 0.0;
  for (int kb = 0; kb < width; kb += kC) {  // uniform: width = the level's longest row
    int c[kS], ix[kS];
#pragma unroll
    for (int u = 0; u < kS; u++) {
      const int k = kb + j + u * kL;
      const bool in = live && k < width;
      c[u] = in ? ecol[size_t(k) * n + t] : 0;
      ix[u] = in ? eidx[size_t(k) * n + t] : -1;
    }
    if (kb == 0 && head) rhs = d[I.x];
    double pr[kS];
#pragma unroll
    for (int u = 0; u < kS; u++) pr[u] = ix[u] >= 0 ? val[ix[u]] * v[c[u]] : 0.0;
#pragma unroll
    for (int k = 0; k < kC; k++) {
      const double p = __shfl(pr[k / kL], base + k % kL, 64);
      if (head && kb + k < width) rhs -= p;
    }
  }
  if (head) v[I.x] += 1.0 * (rhs / val[I.z]);
}
}  // namespace

hipError_t launch_ssor_natural(const NatSweep &fwd, const NatSweep &bwd, const double *val,
                               const double *d, double *v, hipStream_t s) {
  for (const NatSweep *W : {&fwd, &bwd})
    for (int l = 0; l < W->nlev; l++) {
      const int n = W->lptr[l + 1] - W->lptr[l];
      const int width = n > 0 ? int((W->eoff[l + 1] - W->eoff[l]) / n) : 0;
      hipLaunchKernelGGL(k_ssor_nat_level, dim3((n * kL + kB - 1) / kB), dim3(kB), 0, s,
                         W->info + W->lptr[l], W->ecol + W->eoff[l], W->eidx + W->eoff[l], n,
                         width, val, d, v);
    }
  return hipGetLastError();
}

}  // namespace pnp
