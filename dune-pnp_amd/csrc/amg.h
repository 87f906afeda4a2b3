// Aggregation AMG (PNP_PREC_AMG): host-side hierarchy (amg_setup.cc) and device launchers (amg.hip).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "kernels.h"
#include "mesh.h"

namespace pnp {

// coarsest level: a dense inverse (rocSOLVER getrf + getri, once per assembly) of at most
// kAmgMaxDense unknowns, i.e. at most kAmgMaxCoarse vertex blocks of 3 fields (coarsening stops
// there, so the same hierarchy serves the scalar and the 3-field operators)
constexpr int kAmgMaxDense = 3072;
constexpr int kAmgMaxCoarse = kAmgMaxDense / 3;
constexpr int kAmgMaxLevels = 16;

// One coarse level l >= 1 (block-CSR, dense NF x NF blocks, columns sorted, diagonal present)
// plus the maps to the level below it.
struct AmgLevelHost {
  int nb = 0;                        // rows (aggregates of the level below)
  std::vector<int> rp, col, dpos;    // block-CSR pattern, diagonal block position per row
  std::vector<long long> cptr;       // Galerkin contributors of each block: csrc[cptr[q]..cptr[q+1])
  std::vector<int> csrc;             // level 1: (row << 6 | slot) of the SELL; else block index
  std::vector<int> mptr, mem;        // rows of the level below in each aggregate (restriction)
  std::vector<int> agg;              // rows of the level below -> this level's rows (prolongation)
};

// Greedy aggregation of the owned vertex rows over the matrix graph, recursively, until at most
// coarse_target blocks remain (or max_levels).  Level 0 is the SELL layout of L (owned columns
// only: the AMG is rank-local, i.e. block-Jacobi across ranks like the multicolour sweeps).
bool amg_build(const LocalLayout &L, int coarse_target, int max_levels,
               std::vector<AmgLevelHost> &levels, std::string &err);

// aggregation of one graph (CSR adjacency without the diagonal): returns the number of aggregates
int amg_aggregate(int n, const std::vector<int> &ap, const std::vector<int> &aj,
                  std::vector<int> &agg);

hipError_t launch_amg_galerkin0(const DevLayout &L, int nf, int pat, const double *kvals,
                                long long nq, const long long *cptr, const int *csrc, double *cv,
                                hipStream_t s);
hipError_t launch_amg_galerkin(int nf, long long nq, const long long *cptr, const int *csrc,
                               const double *fv, double *cv, hipStream_t s);
hipError_t launch_amg_dinv(int nf, int nb, const int *dpos, const double *v, double *dinv,
                           hipStream_t s);
// dense (row-major, n = nb*nf, zero-filled here) copy of the coarsest block-CSR matrix, i.e. its
// transpose column-major for rocSOLVER (see k_coarse_dense)
hipError_t launch_amg_coarse_dense(int nf, int nb, const int *rp, const int *col, const double *v,
                                   double *dense, hipStream_t s);
// bn[J] = sum over the members i of aggregate J of (a - sub)_i (sub may be null); xn = omega
// Dinv_J bn[J] (pre-smoothing from zero; xn null: none)
hipError_t launch_amg_restrict(int nf, int nbn, const int *mptr, const int *mem, const double *a,
                               const double *sub, double *bn, const double *dinvn, double omega,
                               double *xn, hipStream_t s);
// r = b - A x on a coarse level (vf non-null: the level's single-precision values instead of v)
hipError_t launch_amg_resid(int nf, int nb, const int *rp, const int *col, const double *v,
                            const float *vf, const double *x, const double *b, double *r,
                            hipStream_t s);
// vf[i] = float(v[i]) (a coarse level's values for the V-cycle, PNP_AMG_F32)
hipError_t launch_amg_to_f32(long long n, const double *v, float *vf, hipStream_t s);
hipError_t launch_amg_coarse_apply(int n, const double *ainv, const double *b, double *x,
                                   hipStream_t s);
// single-precision copy of the row-major inverse, rows padded to ld (a multiple of 4, zeros), and
// the GEMV on it (PNP_AMG_F32)
hipError_t launch_amg_inverse_to_f32(int n, int ld, const double *a, float *af, hipStream_t s);
hipError_t launch_amg_coarse_apply_f32(int n, int ld, const float *ainv, const double *b,
                                       double *x, hipStream_t s);
// e == nullptr: a plain damped block-Jacobi sweep (no correction; agg unused); vf as above
hipError_t launch_amg_post(int nf, int nb, const int *rp, const int *col, const double *v,
                           const float *vf, const int *agg, const double *x, const double *e,
                           const double *b, const double *dinv, double omega, double *out,
                           hipStream_t s);
hipError_t launch_amg_prolong0(int nf, int n, const int *agg, const double *x0, const double *e1,
                               double *y, hipStream_t s);

}  // namespace pnp
