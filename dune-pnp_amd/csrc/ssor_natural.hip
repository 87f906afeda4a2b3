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
// chain of such dependencies ending in the row), and every level is one launch, one thread per row.
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

__global__ void __launch_bounds__(kB)
    k_ssor_nat_level(const int *__restrict__ rows, int n, const int *__restrict__ rowptr,
                     const int *__restrict__ col, const double *__restrict__ val,
                     const int *__restrict__ diag, const double *__restrict__ d,
                     double *__restrict__ v) {
  const int t = blockIdx.x * kB + threadIdx.x;
  if (t >= n) return;
  const int R = rows[t];
  double rhs = d[R];
  const int k1 = rowptr[R + 1];
  for (int k = rowptr[R]; k < k1; k++) rhs -= val[k] * v[col[k]];
  v[R] += 1.0 * (rhs / val[diag[R]]);
}
}  // namespace

hipError_t launch_ssor_natural(int nlev_f, const int *lptr_f, const int *rows_f, int nlev_b,
                               const int *lptr_b, const int *rows_b, const int *rowptr,
                               const int *col, const double *val, const int *diag, const double *d,
                               double *v, hipStream_t s) {
  for (int l = 0; l < nlev_f; l++) {
    const int n = lptr_f[l + 1] - lptr_f[l];
    hipLaunchKernelGGL(k_ssor_nat_level, dim3((n + kB - 1) / kB), dim3(kB), 0, s,
                       rows_f + lptr_f[l], n, rowptr, col, val, diag, d, v);
  }
  for (int l = 0; l < nlev_b; l++) {
    const int n = lptr_b[l + 1] - lptr_b[l];
    hipLaunchKernelGGL(k_ssor_nat_level, dim3((n + kB - 1) / kB), dim3(kB), 0, s,
                       rows_b + lptr_b[l], n, rowptr, col, val, diag, d, v);
  }
  return hipGetLastError();
}

}  // namespace pnp
