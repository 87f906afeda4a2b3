// Device data structures and kernel launchers of the MI355X PNP hot path.
//
// HBM layout (per GPU / per rank):
//   rows       = owned vertices, coloured, Morton-ordered inside a colour (mesh.cc)
//   vectors    = vertex-interleaved: x[i*NF + f], owned rows first, then ghosts
//   matrix     = SELL-64 of NF x NF vertex-pair blocks. Chunk c holds rows 64c..64c+63 with
//                chunk_len[c] slots; slot 0 is the diagonal block, slot s >= 1 the s-th
//                neighbour of the row's CCW fan.  Column indices: colidx[off_c + 64 s + lane].
//                Only the structurally non-zero entries of a block are stored (BlockPattern):
//                NV doubles per block, value v of slot s at vals[(off_c + 64 s) * NV + 64 v + lane],
//                so every (slot, value) plane of a chunk is one 512-byte coalesced line.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pnp {

constexpr int kRows = 64;  // rows per SELL chunk = one wavefront

// XCD-aware block remap (cdna_hip_programming.md T1): consecutive workgroups are dealt
// round-robin over the 8 XCDs; remap so that each XCD works on one contiguous 1/8 of the rows and
// neighbouring rows' gathered data (x, coordinates) is reused from that XCD's L2.  Bijective for
// any grid size.  Speed only: correctness never depends on placement.
__device__ __forceinline__ int xcd_block(int b, int nwg, int on = 1) {
  if (!on) return b;
  const int q = nwg / 8, r = nwg % 8, xcd = b % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + b / 8;
}

// ---- per-vertex records of NF doubles -------------------------------------------------------
// NF consecutive doubles at x + NF*j in the fewest memory instructions: 16-B loads/stores of
// 8-B-aligned pairs (gfx950 global accesses need 4-B alignment only) plus the odd last value.
// A gather of a 3-field record is 2 instructions instead of 3 (the sweeps and the SpMV are
// VMEM-issue and L1-bound: TA busy ~70 %, TCP pending-stall ~55 % of cycles).
typedef double double2_a8 __attribute__((ext_vector_type(2), aligned(8)));
template <int NF>
__device__ __forceinline__ void load_nf(const double *__restrict__ x, size_t j, double (&o)[NF]) {
  const double *b = x + size_t(NF) * j;
  int f = 0;
#pragma unroll
  for (; f + 1 < NF; f += 2) {
    const double2_a8 a = *reinterpret_cast<const double2_a8 *>(b + f);
    o[f] = a.x;
    o[f + 1] = a.y;
  }
  if (f < NF) o[f] = b[f];
}
template <int NF>
__device__ __forceinline__ void store_nf(double *__restrict__ x, size_t j, const double (&v)[NF]) {
  double *b = x + size_t(NF) * j;
  int f = 0;
#pragma unroll
  for (; f + 1 < NF; f += 2) {
    double2_a8 a;
    a.x = v[f];
    a.y = v[f + 1];
    *reinterpret_cast<double2_a8 *>(b + f) = a;
  }
  if (f < NF) b[f] = v[f];
}
// the ILU(0) forward sweep's single-precision intermediate (PNP_OPT_ILU_F32 = 3): rounded to
// nearest on the store, widened exactly on the load
template <int NF>
__device__ __forceinline__ void load_nf(const float *__restrict__ x, size_t j, double (&o)[NF]) {
  const float *b = x + size_t(NF) * j;
#pragma unroll
  for (int f = 0; f < NF; f++) o[f] = double(b[f]);
}
template <int NF>
__device__ __forceinline__ void store_nf(float *__restrict__ x, size_t j, const double (&v)[NF]) {
  float *b = x + size_t(NF) * j;
#pragma unroll
  for (int f = 0; f < NF; f++) b[f] = float(v[f]);
}

// ---- SELL value layout --------------------------------------------------------------------------
// Slot s of chunk c holds NV values for each of the chunk's 64 rows, at doubles
// [(chunk_off[c] + 64 s) * NV, +64 NV).  Inside a slot, value pairs (q, q+1) (q even, q+1 < NV)
// are interleaved per row as 16-B records, so one dwordx4 per lane moves a pair (dwordx2 stores
// are store-issue bound); an odd last value is row-contiguous.
__host__ __device__ constexpr int vin(int nv, int q, int lane) {
  return q < (nv & ~1) ? (q >> 1) * 2 * kRows + 2 * lane + (q & 1) : (nv - 1) * kRows + lane;
}

// the NV values of one (row, slot): sb = slot base (vals + (chunk_off + 64 s) * NV)
template <int NV>
__device__ __forceinline__ void load_vals(const double *__restrict__ sb, int lane, double *B) {
#pragma unroll
  for (int q = 0; q + 1 < NV; q += 2) {
    const double2 t = reinterpret_cast<const double2 *>(sb + (q >> 1) * 2 * kRows)[lane];
    B[q] = t.x;
    B[q + 1] = t.y;
  }
  if constexpr (NV & 1) B[NV - 1] = sb[(NV - 1) * kRows + lane];
}

// the same with a non-temporal hint (streamed once per launch: leaves L2 to the gathers)
template <int NV>
__device__ __forceinline__ void load_vals_nt(const double *__restrict__ sb, int lane, double *B) {
#pragma unroll
  for (int q = 0; q + 1 < NV; q += 2) {
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v t = __builtin_nontemporal_load(reinterpret_cast<const d2v *>(sb + (q >> 1) * 2 * kRows) + lane);
    B[q] = t.x;
    B[q + 1] = t.y;
  }
  if constexpr (NV & 1) B[NV - 1] = __builtin_nontemporal_load(sb + (NV - 1) * kRows + lane);
}

template <int NV>
__device__ __forceinline__ void store_vals(double *__restrict__ sb, int lane, const double *B) {
#pragma unroll
  for (int q = 0; q + 1 < NV; q += 2)
    reinterpret_cast<double2 *>(sb + (q >> 1) * 2 * kRows)[lane] = make_double2(B[q], B[q + 1]);
  if constexpr (NV & 1) sb[(NV - 1) * kRows + lane] = B[NV - 1];
}

template <int NV>
__device__ __forceinline__ void store_vals_nt(double *__restrict__ sb, int lane, const double *B) {
  typedef double d2v __attribute__((ext_vector_type(2)));
#pragma unroll
  for (int q = 0; q + 1 < NV; q += 2) {
    d2v t;
    t.x = B[q];
    t.y = B[q + 1];
    __builtin_nontemporal_store(t, reinterpret_cast<d2v *>(sb + (q >> 1) * 2 * kRows) + lane);
  }
  if constexpr (NV & 1) __builtin_nontemporal_store(B[NV - 1], sb + (NV - 1) * kRows + lane);
}

// 256-row block processed by workgroup b of a whole-matrix launch of nwg workgroups
template <class DL>
__device__ __forceinline__ int row_block(const DL &L, int b, int nwg) {
  return L.blkmap ? L.blkmap[xcd_block(b, nwg, 1)] : xcd_block(b, nwg, L.xcd_remap);
}

// ---- operator kinds / block patterns ----------------------------------------------------------
enum OpKind : int {
  OP_PNP = 0,
  OP_PNP_IE = 1,
  OP_PB = 2,
  OP_DIFF = 3,
  OP_DIFF_IE = 4,
  OP_POISSON = 5
};

// Block pattern: bit (f*3+g) set if entry (f,g) of a vertex-pair block can be non-zero.
// PNP: c+ and c- never couple (7 of 9).  PNP with the PnpTOperator mass: the c- mass sits in the
// c+ rows (quirk Q2, src/pnp_toperator.hh:99), so (c+, c-) is added (8 of 9).  Scalar: 1x1.
constexpr int kPatPnp = 0x1FF & ~((1 << 5) | (1 << 7));
constexpr int kPatPnpIE = 0x1FF & ~(1 << 7);
constexpr int kPatScalar = 1;
// bit 9: the block's pattern values are stored as they are (no k-form) -- the forward-difference
// Jacobian (PNP_JAC_FD), whose entries do not satisfy the analytic block's identities.  Scalar
// operators need no FD variant (their k-form is the value itself).
constexpr int kPatFD = 1 << 9;
constexpr int kPatPnpFD = kPatPnp | kPatFD;
constexpr int kPatPnpIEFD = kPatPnpIE | kPatFD;

__host__ __device__ constexpr int popc9(int m) {
  int c = 0;
  for (int i = 0; i < 9; i++) c += (m >> i) & 1;
  return c;
}
// position of (f,g) among the stored values (row-major order), -1 if not stored
__host__ __device__ constexpr int pat_index(int mask, int f, int g) {
  if (!((mask >> (f * 3 + g)) & 1)) return -1;
  int c = 0;
  for (int i = 0; i < f * 3 + g; i++) c += (mask >> i) & 1;
  return c;
}

// ---- stored (K-form) block values -----------------------------------------------------------
// The assembled Jacobian stores, per block (row i, column j), only the independent coefficients
// of the operator's block (k-form), unmasked.  PnpOperator (kPatPnp), 5 values:
//   k0 = sum G_ij W, k1 = sum kappa M_ij, k2 = sum G_ij S+, k3 = sum G_ij S-, k4 = sum gp m_j
// PnpOperator + PnpTOperator (kPatPnpIE) add k5 = sum tau M2_ij; scalar operators store the
// value itself.  expand_k gives the block pattern's values exactly (each is one coefficient, its
// negation, or k0 -+ k4 (+ k5)); Dirichlet rows (mask_rows) become identity rows.
__host__ __device__ constexpr int nks_of(int pat) {
  return (pat & kPatFD) ? popc9(pat) : (pat == kPatPnp ? 5 : (pat == kPatPnpIE ? 6 : 1));
}

template <int PAT>
__host__ __device__ __forceinline__ void expand_k(const double *K, double *B) {
  if constexpr ((PAT & kPatFD) != 0) {
#pragma unroll
    for (int q = 0; q < popc9(PAT); q++) B[q] = K[q];
  } else if constexpr (PAT == kPatPnp || PAT == kPatPnpIE) {
    B[pat_index(PAT, 0, 0)] = K[0];
    B[pat_index(PAT, 0, 1)] = K[1];
    B[pat_index(PAT, 0, 2)] = -K[1];
    B[pat_index(PAT, 1, 0)] = -K[2];
    B[pat_index(PAT, 1, 1)] = K[0] - K[4];
    B[pat_index(PAT, 2, 0)] = K[3];
    B[pat_index(PAT, 2, 2)] = K[0] + K[4];
    if constexpr (PAT == kPatPnpIE) {
      B[pat_index(PAT, 1, 1)] += K[5];
      B[pat_index(PAT, 1, 2)] = K[5];
    }
  } else {
    B[0] = K[0];
  }
}

// constrained rows f (bit f of dm): identity row (1 on the diagonal block's (f,f), else 0)
template <int NF, int PAT>
__host__ __device__ __forceinline__ void mask_rows(double *B, unsigned dm, bool diag) {
#pragma unroll
  for (int f = 0; f < NF; f++)
#pragma unroll
    for (int g = 0; g < NF; g++) {
      const int v = pat_index(PAT, f, g);
      if (v >= 0 && ((dm >> f) & 1)) B[v] = (diag && f == g) ? 1.0 : 0.0;
    }
}

// ---- device views ----------------------------------------------------------------------------
struct DevLayout {
  int n_owned = 0, n_local = 0, nchunks = 0, ncolors = 0;
  int max_slots = 0;                // max chunk_len (fan length + 1)
  int xcd_remap = 0;                // A/B knob (PNP_XCD_REMAP): see xcd_block
  const int *chunk_len = nullptr;
  const int *chunk_off = nullptr;   // nchunks + 1
  const int *colidx = nullptr;
  const uint64_t *rowmeta = nullptr;
  const double *xy = nullptr;       // [n_local][2]
  const int *color_idx = nullptr;   // rows of each colour (see mesh.h LocalLayout)
  const uint8_t *rowcolor = nullptr;
  // Spatial block order for the whole-matrix kernels (assembly, SpMV): logical block (XCD-major,
  // see xcd_block) -> 256-row block.  Blocks are sorted by their Morton position inside their
  // colour, so each XCD takes one spatial slice of the domain in every colour and the neighbour
  // gathers of its rows share its L2 (colour-major rows otherwise spread a region over all XCDs).
  const int *blkmap = nullptr;
  // > 0: whole-matrix launches (SpMV) cover only the blkcount 256-row blocks listed in blkmap
  // (the interior / boundary halves of a halo-overlapped SpMV, multi-GPU)
  int blkcount = 0;
  // triangular split of the owned-column pattern, SELL-64 each (same row order and chunks):
  // L = strictly lower slots (columns of earlier colours), U = slot 0 diagonal + upper slots.
  // Padding slots point at the row itself with zero values.  The sweeps read only the half
  // they need (in the full SELL the lanes of a cache line disagree on lower/upper).
  const int *lchunk_len = nullptr, *lchunk_off = nullptr, *lcolidx = nullptr;
  const int *uchunk_len = nullptr, *uchunk_off = nullptr, *ucolidx = nullptr;
  // Dirichlet mask of the current operator, [n_owned * nf] (see mask_rows)
  const uint8_t *dmask = nullptr;
  // LDS-staged SpMV (PNP_SPMV_LDS): per 256-row block the distinct columns its rows touch
  // (ulist[uptr[b] .. uptr[b+1])), and per SELL slot the position of its column in that list
  // (lidx, same indexing as colidx); umax = the longest list
  const int *uptr = nullptr, *ulist = nullptr;
  const uint16_t *lidx = nullptr;
  int umax = 0;
  // per block the number of list entries that are not its own rows (they come first): the
  // assembly walk stages only those; unmax = the largest
  const int *uown = nullptr;
  int unmax = 0;
  // LDS-staged ILU(0) sweeps (k_ilu0_solve_lds): per (colour, 256-row block of the colour) -- blocks
  // numbered colour by colour -- the distinct neighbour rows of its L (forward) / U (backward) split
  // slots (lsx_list[lsx_ptr[b] ..), usx_*), and per split-storage position (the indexing of lcolidx
  // / ucolidx) the neighbour's position in its block's list (0xFFFF: padding or the diagonal slot);
  // sx_max = the longest list
  const int *lsx_ptr = nullptr, *lsx_list = nullptr, *usx_ptr = nullptr, *usx_list = nullptr;
  // lane order of the split storage (ctx.cc, PNP_SPLIT_SORT): position p = 64 chunk + lane holds
  // row 64 chunk + lperm[p] in L, 64 chunk + uperm[p] in U (rows of one colour segment of the
  // chunk, longest first); lpinv / upinv: the lane of a row; llen / ulen: a position's own slot
  // count (U: with the diagonal slot); ldl[p]: the U lane of L position p's row (its diagonal block)
  const uint8_t *lperm = nullptr, *uperm = nullptr, *lpinv = nullptr, *upinv = nullptr;
  const uint8_t *llen = nullptr, *ulen = nullptr, *ldl = nullptr;
  const uint16_t *lsx_idx = nullptr, *usx_idx = nullptr;
  int sx_max = 0;
};

template <int NF>
__device__ __forceinline__ unsigned row_mask(const DevLayout &L, int row) {
  unsigned dm = 0;
#pragma unroll
  for (int f = 0; f < NF; f++) dm |= unsigned(L.dmask[size_t(row) * NF + f] != 0) << f;
  return dm;
}

struct AsmArgs {
  int kind;
  int jac;               // 1: residual + Jacobian, 0: residual only
  double l_b, c0, tau, pi, dt, z;
  int cylindrical;
  const double *x;       // [n_local * NF]
  const double *aux0;    // DIFF: phi [n_local]; POISSON: cp [n_local]
  const double *aux1;    // POISSON: cm [n_local]
  const double *cvec;    // constant part of the residual [n_owned * NF] (Neumann load, old mass)
  const uint8_t *dmask;  // Dirichlet mask [n_owned * NF]
  double *r;             // [n_owned * NF]
  double *vals;          // SELL values
  int cold;              // 1: the launch follows a linear solve (Newton's Jacobian): its inputs are
                         // out of the caches, and the Jacobian takes the LDS-staged walk
};

// BiCGSTAB scalar block, resident on the device (no host round trip per half step)
struct Scalars {
  double rho, rho_new, alpha, omega, h, norm0, norm, reduction;
  double it_half;        // ISTL half-step counter of the last completed half step
  double red[6];         // reduction results (after allreduce)
  int done;              // 0 running, 1 converged, 2 breakdown
  int breakdown;         // 1 rho, 2 omega, 3 h
  int iter;              // full iterations started
  int divguard;          // 1: stop with breakdown 4 once ||r|| > 1e10 ||r0|| (AMG solves)
  int pending;           // two-reduction iteration: the second half step's test is still due
  int xpend;             // x += alpha y of the first half step deferred to the second half's
                         // update (set by launch_update_fwd0 with x = null, cleared by stage 4)
};

// ---- launchers (return hipError_t of the launch) ----------------------------------------------
hipError_t launch_assemble(const DevLayout &L, const AsmArgs &a, hipStream_t s,
                           hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// old-time mass M(x_old) (PnpTOperator / DiffusionTOperator) subtracted into cvec
hipError_t launch_ion_flux(int ns, const int4 *seg, const double *xy, const double *x, int cyl,
                           double pi, double *out, hipStream_t s);
hipError_t launch_mass_apply(const DevLayout &L, int kind, double tau, double pi, int cylindrical,
                             const double *x_old, double *cvec, hipStream_t s);

// y = A x over owned rows; optional fused dots: out partials[block*k + j]
//   mode 0: none; 1: <w, y> (k=1); 2: <y, w>, <y, y> (k=2); 3: y = w - A x (no dots);
//   4: <y, w>, <y, y>, <y, w2> (k=3)
// t0 / t1 (may be null; the LDS-staged form only): events the launch records at the kernel's
// start and end (hipExtLaunchKernelGGL), so the library's timers see the kernel's own duration
hipError_t launch_spmv(const DevLayout &L, int nf, int pat, const double *vals, const double *x,
                       double *y, int mode, const double *w, double *partials, int *nparts,
                       hipStream_t s, const double *w2 = nullptr, hipEvent_t t0 = nullptr,
                       hipEvent_t t1 = nullptr);

// preconditioners: v = M^{-1} d (v over owned rows)
hipError_t launch_jacobi(const DevLayout &L, int nf, int pat, const double *vals, const double *d,
                         double *v, hipStream_t s);
// symmetric multicolour Gauss-Seidel on the split matrix (lv, uv); t = scratch [n_owned * nf]
hipError_t launch_sgs(const DevLayout &L, const int *color_ptr_host, int nf, int pat,  // NOLINT
                      const double *lv, const double *uv, const double *d, double *v, double *t,
                      hipStream_t s);
// fill the L / U split storage (NV values per block) from the k-form matrix (from_k = 1: expand
// and mask) or from the ILU factors (from_k = 0: copy).  lsrc/usrc: (row << 6 | slot) of the
// source block in the full SELL, -1 for padding
// f32 (from_k = 0 only): store the factors in single precision (quad-interleaved, see
// linalg.hip vinf); the sweeps then read float values and compute in fp64
hipError_t launch_split(const DevLayout &L, int nf, int pat, int from_k, const double *src,
                        const int *lsrc, long long ln, const int *usrc, long long un, void *lv,
                        void *uv, hipStream_t s, int f32 = 0);
// lu = the k-form matrix expanded and masked to NV values per block (ILU input)
hipError_t launch_expand(const DevLayout &L, int nf, int pat, const double *vals, double *lu,
                         hipStream_t s);
// ILU(0) of the local (owned x owned) matrix on the stored block pattern, scalar elimination in
// colour-major vertex order (fields ascending inside a vertex); lu = copy of vals on entry,
// factors on exit (unit-lower L strictly below, U on/above the diagonal, diagonal inverted)
hipError_t launch_ilu0_factor(const DevLayout &L, const int *color_ptr_host, int nf, int pat,
                              double *lu, hipStream_t s);
// the same factors from the k-form matrix in one launch per colour, expand and split folded in:
// aos = row-contiguous scratch (row i's blocks at (rowoff[i] + slot) * NV, columns rowcol[rowoff[i]
// + slot]), lv / uv = the split storage (float when f32); bitwise the factors of launch_expand +
// launch_ilu0_factor + launch_split
hipError_t launch_ilu0_factor_fused(const DevLayout &L, const int *color_ptr_host, int nf, int pat,
                                    const double *kvals, const int *rowoff, const int *rowcol,
                                    double *aos, void *lv, void *uv, int f32, hipStream_t s);
// c_first = 1: colour 0's forward step was already applied (launch_update_fwd0); add != null:
// also out = add + v (written row by row as the backward sweep finishes them).  yf != null (bf16
// factors only, f32 = 2): the forward sweep's intermediate y = L^-1 d is stored in single precision
// there (colour 0's by launch_update_fwd0 when c_first = 1) instead of in v, and the forward
// gathers and the backward sweep's own rows read it from there
// t0 / t1 (may be null; the LDS-staged colour launches only): recorded by the first launch's
// start and the last launch's end, so a timer spans the colour launches without marker dispatch
hipError_t launch_ilu0_apply(const DevLayout &L, const int *color_ptr_host, int nf, int pat,
                             const void *lv, const void *uv, const double *d, double *v,
                             hipStream_t s, int c_first = 0, const double *add = nullptr,
                             double *out = nullptr, int f32 = 0, float *yf = nullptr,
                             hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// The same application as ONE dataflow launch (k_ilu0_flow, PNP_ILU_FLOW): the colour launches'
// 256-row blocks become units in the launches' order (forward colours c_first .. nc-2, the last
// colour, backward colours nc-2 .. 0); a workgroup takes the next unit by an atomic ticket, waits
// for the units it reads from (dep_list[dep_ptr[u] .. dep_ptr[u+1]), all earlier in the order) to
// raise their flags, runs the colour launch's arithmetic on its block, stores its rows write-through
// and raises its own flag.  flags[0 .. nunits) and the ticket flags[nunits] are zeroed before every
// launch; abort_word is set when a wait times out (never expected).
constexpr int kIluFlowMaxStages = 32;
struct IluFlow {
  int nstages = 0, nunits = 0;
  // 0: one workgroup per unit, taken by one atomic ticket; 1: a resident grid, workgroup b takes
  // units b, b + G, ...
  int persistent = 1;
  int unit0[kIluFlowMaxStages + 1] = {};  // first unit of each stage
  int kind[kIluFlowMaxStages] = {};       // kIluFwd 0 / kIluBwd 1 / kIluLast 2
  int r0[kIluFlowMaxStages] = {}, r1[kIluFlowMaxStages] = {};  // the stage colour's positions
  int blk0[kIluFlowMaxStages] = {};       // the colour's first block in the staging-list numbering
  const int *dep_ptr = nullptr, *dep_list = nullptr;
  unsigned *flags = nullptr;              // [nunits + 1], padded to 16 B
  unsigned *abort_word = nullptr;
};
hipError_t launch_ilu0_flow(const DevLayout &L, const IluFlow &F, int nf, int pat, const void *lv,
                            const void *uv, const double *d, double *v, hipStream_t s, int f32);
// BiCGSTAB update fused with colour 0 of the ILU(0) forward sweep (rows [0, c0_end)): which 0:
// p = r + beta (p - omega v) (first: p = r), yout = Ld^-1 p on colour 0; which 1: x += alpha yin,
// r -= alpha v, partials ||r||^2 (one per workgroup, *nparts), yout = Ld^-1 r on colour 0.
// which 1 with x = null: x += alpha yin is left to launch_update_xr(.., y1 = yin) (S->xpend).
// youtf != null (bf16 factors, launch_ilu0_apply's yf): colour 0's y goes there, not to yout
hipError_t launch_update_fwd0(const DevLayout &L, int nf, int pat, int c0_end, const Scalars *S,
                              int which, int first, double *x, const double *yin, double *r,
                              const double *v, double *p, const void *uv, double *yout,
                              double *partials, int *nparts, hipStream_t s, int f32 = 0,
                              const double *rt = nullptr, float *youtf = nullptr);

// BLAS-1 over n = n_owned*nf entries
int blas_nparts(long long n);
// p = (it<1) ? r : beta*(p - omega*v) + r, with beta from Scalars
hipError_t launch_update_p(long long n, const Scalars *S, const double *r, const double *v,
                           double *p, int first, hipStream_t s);
// CG: p = q + beta p, beta = S->omega
hipError_t launch_cg_update_p(long long n, const Scalars *S, const double *q, double *p,
                              hipStream_t s);
// x += a*y; r -= a*v; partials <r,r> [, <rt, r>];  a = S->alpha (which=0) or S->omega (which=1)
// y1 != null (which 1): first x += alpha y1, the first half step's update that
// launch_update_fwd0 deferred, then x += omega y -- the same two roundings as two passes, one
// read and write of x fewer; with the first half step converged (S->done, S->xpend) only the
// former
hipError_t launch_update_xr(long long n, const Scalars *S, int which, double *x, const double *y,
                            double *r, const double *v, const double *rt, double *partials,
                            hipStream_t s, const double *y1 = nullptr);
// partials of <a,b> (and <a,a> if two)
hipError_t launch_dot(long long n, const double *a, const double *b, int two, double *partials,
                      hipStream_t s);
// sum partials[nparts][k] -> S->red[0..k) (deterministic order); derive_stage >= 0 also runs
// the derive step in the same launch (single GPU: no allreduce in between).  mw (kRedMwDoubles
// doubles, zeroed once, one per stream): with it, long partial arrays (>= 8,192) are summed by a
// multi-workgroup launch whose last workgroup finishes the sum (linalg.hip k_reduce_mw)
constexpr int kRedMwDoubles = 1 + 64 * 5;
hipError_t launch_reduce(const double *partials, int nparts, int k, Scalars *S, hipStream_t s,
                         int derive_stage = -1, double *mw = nullptr);
// partial-sum count of launch_spmv over nrows rows (allocation bound)
int spmv_parts(int nrows);
// sum partials pa[npa][ka] -> S->red[0..ka) and pb[npb][kb] -> S->red[ka..ka+kb), ka+kb <= 5
hipError_t launch_reduce2(const double *pa, int npa, int ka, const double *pb, int npb, int kb,
                          Scalars *S, hipStream_t s, int derive_stage = -1, double *mw = nullptr);
// derive scalars after a reduction; stage: 0 init (red: <r,r>), 1 after h, 2 after first half
// norm, 3 after <t,r>,<t,t>, 4 after second half (red: <r,r>, <rt,r>); 23 = 2 then 3 from one
// reduction (red: <t,r>, <t,t>, ||s||^2), the first half step's test deferred to the second's;
// two-reduction iteration (multi-GPU: two allreduces per iteration instead of three):
// 31 = h (red[0]) with the previous iteration's second-half test on red[1] = ||r||^2 (lagged),
// 32 = the first half's test and omega from <t,s>, <t,t>, <t,rt>, ||s||^2, <rt,s>, then
// rho_new = <rt,s> - omega <rt,t> and the second half's counters, its test left pending;
// 33 = the pending test alone (red[0] = ||r||^2), after the last iteration
hipError_t launch_derive(Scalars *S, int stage, hipStream_t s);

// y = x - lambda*z (Newton line search), copy/scale helpers
hipError_t launch_axpby(long long n, double a, const double *x, double b, const double *y,
                        double *out, hipStream_t s);
// halo pack: buf[k*nf+f] = x[idx[k]*nf+f]
hipError_t launch_pack(int n, int nf, const int *idx, const double *x, double *buf, hipStream_t s);
// external <-> internal permutation: ext[f*nv_global + l2g[i]] <-> in[i*nf + f], i < n
hipError_t launch_gather_ext(int n, int nf, int nv_global, const int *l2g, const double *ext,
                             double *in, hipStream_t s);
hipError_t launch_scatter_ext(int n, int nf, int nv_global, const int *l2g, const double *in,
                              double *ext, hipStream_t s);
// forward-difference Jacobian (fd_jacobian.hip, PNP_JAC_FD): element matrices of the ne local
// elements (etri: local vertex ids in mesh order, ascending global element id) into jel
// [ne][3nf][3nf], then every SELL block of the owned rows summed from them (rptr / cdata: per row,
// per slot a count and the codes e*9 + a*3 + b) into aa.vals in the FD pattern `pat`
hipError_t launch_fd_jacobian(const DevLayout &L, const AsmArgs &aa, int nf, int pat, int ne,
                              const int *etri, const long long *rptr, const int *cdata,
                              double *jel, hipStream_t s);
// device CSR values of the assembled Jacobian: out[k] = value vidx[k] of block src[k] (row << 6 |
// slot), expanded and row-masked (pnp_jacobian_csr_device)
hipError_t launch_csr_fill(const DevLayout &L, int nf, int pat, const double *vals, long long nnz,
                           const int *src, const unsigned char *vidx, double *out, hipStream_t s);
// ISTL SeqSSOR (k = 1, omega = 1) in the lexicographic DOF order (ssor_natural.hip): v = 0, then
// the forward levels and the backward levels, one launch per level.  Per sweep direction
// (NatSweep): sweep positions t of level l are lptr[l] .. lptr[l+1] (host array); info[t] = {row
// (external index), entry count | the diagonal's offset in the row << 8 (so at most 255 entries
// per row: csr_values() refuses a wider pattern with PNP_E_STATE), index of the row's first
// entry in the external-layout CSR values val (its entries are contiguous there), the row's
// internal position}; the operand codes of the row's entries (ecol, CSR order) as an ELL of the
// level stored unit-major: with tl = t - lptr[l], entry k at eoff[l] + (tl / U * w_l + k) * U +
// tl % U (U = ssor_natural_unit_rows(), w_l the level's width; eoff: host array).  The level
// launches: d / v external-layout vectors.
struct NatSweep {
  int nlev = 0;
  const int *lptr = nullptr;
  const long long *eoff = nullptr;
  const int4 *info = nullptr;
  const int *ecol = nullptr;
};
hipError_t launch_ssor_natural(const NatSweep &fwd, const NatSweep &bwd, const double *val,
                               const double *d, double *v, hipStream_t s);
// The same two sweeps as ONE launch (dataflow): units of up to ssor_natural_unit_rows() rows of one level, int4
// {first sweep position, rows | width << 8 | backward << 16, the ELL stride between a row's
// entries (U), ELL index of the unit's first row}, forward units (nunits_f) then backward ones, each in level order.  An
// operand code in ecol (both forms): c >= 0 the forward value of row c, c == -1 zero, c <= -2 the
// backward value of row -(c + 2).  vf / vb (n each, external layout): forward / backward results;
// d is read in the internal layout, at info.w / rec.w; abort_word[0] is set when an operand wait
// times out.
// rows per unit = rows per wavefront of the flow kernel (64 / its lanes per row)
int ssor_natural_unit_rows();
// the longest row the chain kernel takes (one entry per lane of its wave)
int ssor_natural_chain_width();
// results the chain kernel keeps in registers (operand kind 3 reaches back this many rows)
int ssor_natural_chain_history();
// groups (one wave each) of the chain kernel resident at once on this device
int ssor_natural_chain_capacity();
struct NatFlow {
  const int4 *units = nullptr;
  int nunits = 0, nunits_f = 0;
  // first unit of each sweep's narrow tail (levels of at most PNP_NAT_TAIL / PNP_NAT_CHAIN rows to
  // the sweep's end): forward [tail_f, nunits_f), backward [tail_b, nunits)
  int tail_f = 0, tail_b = 0;
  int max_width = 0;  // the longest row of any unit (the pipelined head takes up to 24 entries)
  // the tails as chains (ssor_natural.hip k_ssor_nat_chain), when ngroups > 0: the wave of group g
  // walks rows gptr[g] .. gptr[g+1] of rec (as NatSweep::info); row q's entries at q * wpad ..
  // + count of ecode (idx << 2 | kind: 0 zero, 1 vf[idx], 2 vb[idx], 3 the group's result idx
  // rows back)
  struct Chains {
    int ngroups = 0, wpad = 0;
    const int *gptr = nullptr, *ecode = nullptr;
    const int4 *rec = nullptr;
  } chain_f, chain_b;
  NatSweep fwd, bwd;
  unsigned *abort_word = nullptr;
};
// 1 if the dataflow launch's head grid and its chain grid are each resident at once on this
// device (each kernel launched once in probe mode with its full grid: workgroups check in and
// wait for the whole grid, bounded), 0 if not, -1 on a HIP error; probe: 2 unsigned of scratch.
// Synchronous (not inside a stream capture)
int ssor_natural_flow_resident(const NatFlow &F, unsigned *probe, hipStream_t s);
hipError_t launch_ssor_natural_flow(const NatFlow &F, int n, const double *val, const double *d,
                                    double *vf, double *vb, hipStream_t s);
// ---- reference-order mode (PNP_OPT_SEQ_ORDER, seq_order.hip) ----------------------------------
// the global mesh in its own element order (external layout): tri [nt][3], xy [nv][2]; per vertex
// v its incident elements in ascending order, vinc[vptr[v] .. vptr[v+1]) = e << 2 | local index
struct SeqMesh {
  int nv = 0, nt = 0;
  const int *tri = nullptr, *vptr = nullptr, *vinc = nullptr;
  const double *xy = nullptr;
};
// the operator: kind (OP_*), nfields, parameters, frozen fields (global vertex order) and x_old
// (external layout)
struct SeqOp {
  int kind = 0, nf = 1, cyl = 0;
  double pi = 3.1415, l_b = 1, c0 = 0, tau = 1, dt = 0, z = 0;
  const double *phi = nullptr, *cp = nullptr, *cm = nullptr, *x_old = nullptr;
};
// element pass (RLT / JLT: the one-step temporal operator's; bptr / bval: alpha_boundary's terms
// per (element, local index), CSR over e * nl + i) and the row gathers of seq_order.hip
hipError_t launch_seq_element(const SeqMesh &M, const SeqOp &P, const double *x, int mode,
                              double *RL, double *RLT, double *RLO, double *JL, double *JLT,
                              const int *bptr, const double *bval, hipStream_t s);
hipError_t launch_seq_residual_gather(const SeqMesh &M, int nf, int has_old, const double *RL,
                                      const double *RLT, const double *RLO,
                                      const unsigned char *mask, double *r, hipStream_t s);
hipError_t launch_seq_jacobian_gather(const SeqMesh &M, int nf, const double *JL,
                                      const double *JLT, const int *rowptr, const int *col,
                                      const unsigned char *mask, double *val, hipStream_t s);
hipError_t launch_seq_spmv(int n, const int *rowptr, const int *col, const double *val,
                           const double *x, double *y, hipStream_t s);
hipError_t launch_seq_dot(int n, const double *a, const double *b, double *out, hipStream_t s);
hipError_t launch_seq_bicg_p(int n, double beta, double omega, double *p, const double *v,
                             const double *r, hipStream_t s);
hipError_t launch_seq_axpy2(int n, double a, double *x, const double *y, double *r,
                            const double *v, hipStream_t s);
hipError_t launch_seq_prec_diag(int n, int jacobi, const double *d, const int *diag,
                                const double *val, double *v, hipStream_t s);
hipError_t launch_seq_axpy(int n, double a, double *x, const double *y, hipStream_t s);
hipError_t launch_seq_aymx(int n, double a, double *x, const double *y, hipStream_t s);
hipError_t launch_seq_cg_p(int n, double beta, double *p, const double *q, hipStream_t s);

// read n doubles of buf (cache scrub before a cache-cold timing; sink is never written)
hipError_t launch_scrub(const double *buf, long long n, double *sink, hipStream_t s);

// ---- P_k (k = 2, 3) scalar operators (pk_assemble.hip, pk.h) ----------------------------------
// ne local elements (every element with an owned node; its nodes are all local), enode[a * ne + e]
// the local node of local node a.  Per owned row i (SELL chunk c, lane l): icnt[i] incident
// elements, the t-th at position p = ioff[c] + 64 t + l: inc[p] = e << 4 | (local index of i in
// e), islot[p * NW + w] the SELL slots (bytes) of the element's nl nodes in row i, NW = ceil(nl/4)
struct PkDev {
  int k = 1, nl = 3, ne = 0;
  const int *enode = nullptr;
  const int *ioff = nullptr, *icnt = nullptr, *inc = nullptr;
  const uint32_t *islot = nullptr;
  double *eres = nullptr;  // [nl][ne] element residual rows of the two-pass residual-only launch
  double *ejac = nullptr;  // [ne][nl][W] element matrix + residual rows of the two-pass Jacobian
  // the two-pass Jacobian's gather split: 256-row blocks whose rows have at most short_len slots
  // (blk_short, in the blkmap order) and the others (blk_long); n_short 0: one launch
  const int *blk_short = nullptr, *blk_long = nullptr;
  int n_short = 0, n_long = 0, short_len = 0;
};
hipError_t pk_upload_tables(int k, hipStream_t s);
// jac 0 residual, 1 analytic Jacobian, 2 forward-difference Jacobian (PNP_JAC_FD)
hipError_t launch_pk_assemble(const DevLayout &L, const AsmArgs &aa, const PkDev &P, int jac,
                              hipStream_t s);
// cvec -= M(x_old): the DiffusionTOperator mass of the old time level
hipError_t launch_pk_mass_apply(const DevLayout &L, const PkDev &P, const double *x_old,
                                double *cvec, hipStream_t s);
// calcIonFlux: seg = {local element, local face, group}; out[2s], out[2s+1]
hipError_t launch_pk_ion_flux(const DevLayout &L, const PkDev &P, int ns, const int4 *seg,
                              const double *x, int cyl, double pi, double *out, hipStream_t s);
// pnp_probe_slot_stores: every SELL slot of every owned row written once, row order[t] by thread t
// (order null: SELL order); val holds chunk_off[nchunks] doubles
hipError_t launch_slot_store_probe(const DevLayout &L, const int *order, double *val,
                                   hipStream_t s);

}  // namespace pnp
