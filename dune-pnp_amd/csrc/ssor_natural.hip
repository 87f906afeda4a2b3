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

#include <climits>
#include <cstdint>
#include <cstdlib>
#include <algorithm>

namespace pnp {

namespace {
constexpr int kB = 256;

// A level is a short chain of dependent memory round trips per row, whatever its size, so the
// sweep is laid out to keep that chain at two: the level's entries are an ELL of its rows, stored
// unit-major (NatSweep: groups of kUR rows, each group's entries k-major -- coalesced column /
// value-index loads that need nothing but the position, padding marked by index -1), and each row
// is served by kL lanes, lane j loading entries j, j + kL, ...
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
constexpr int kUR = 64 / kL;  // rows per dataflow unit (one wavefront): the ELL's group size
__global__ void __launch_bounds__(kB)
    k_ssor_nat_level(const int4 *__restrict__ info, const int *__restrict__ ecol,
                     int n, int width,
                     const double *__restrict__ val, const double *__restrict__ d,
                     double *__restrict__ v) {
  const int g = blockIdx.x * kB + threadIdx.x, t = g / kL, j = g % kL;
  const bool live = t < n;  // whole rows per wavefront: kL divides 64
  const bool head = live && j == 0;
  const int4 I = live ? info[t] : make_int4(0, 0, 0, 0);  // every lane: the row's first entry
  const int len = I.y & 255;
  const int base = (threadIdx.x % 64) - j;  // the row's first lane in the wavefront
  double rhs = 0.0;
  for (int kb = 0; kb < width; kb += kC) {  // uniform: width = the level's longest row
    int c[kS], ix[kS];
#pragma unroll
    for (int u = 0; u < kS; u++) {
      const int k = kb + j + u * kL;
      const bool in = live && k < width;
      const size_t at = (size_t(t / kUR) * width + k) * kUR + size_t(t % kUR);  // unit-major ELL
      c[u] = in ? ecol[at] : -1;
      ix[u] = (in && k < len) ? I.z + k : -1;  // the row's entries are contiguous in val
    }
    if (kb == 0 && head) rhs = d[I.x];
    double pr[kS];
#pragma unroll
    for (int u = 0; u < kS; u++) {
      // in place, every operand code reads v: a zero operand (-1) is a row not yet swept or
      // another rank's, both 0.0 in v
      const double o = c[u] == -1 ? 0.0 : v[c[u] >= 0 ? c[u] : -(c[u] + 2)];
      pr[u] = ix[u] >= 0 ? val[ix[u]] * o : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kC; k++) {
      const double p = __shfl(pr[k / kL], base + k % kL, 64);
      if (head && kb + k < width) rhs -= p;
    }
  }
  if (head) v[I.x] += 1.0 * (rhs / val[I.z + (I.y >> 8)]);
}

// ---- one launch for both sweeps: a dataflow over the level-ordered units ------------------------
// The level launches above cost two round trips plus a dispatch per level (~680 levels at
// config 3).  Here every wave of a resident grid takes units w, w + G, w + 2G, ... (G waves) in
// the level order, loads its rows' entries and operands at once, and waits only for the operands
// that are not there yet: each forward / backward result is written exactly once, as one 8-byte
// agent-scope (write-through) store, into a vector that was set to the all-ones pattern (a NaN no
// arithmetic produces here) before the launch, so a value that is not all-ones is final.  That is
// the data-tagged granule hand-off of cdna_hip_programming.md Guideline 16 (R2) with the value as
// its own tag: relaxed agent-scope atomic loads poll it, no fence is needed.  The critical path is
// the chain of row dependencies (the level count), each hop one store-to-poll latency instead of
// a launch.
// Progress: a unit depends only on units earlier in the order.  The earliest unfinished unit's
// wave has finished all its own earlier units, so it is working on that unit, whose operands are
// all final: some wave always advances, provided every wave of the grid is resident (the grid is
// sized from the occupancy query, and one context runs one stream).  Every wait is bounded: a
// wave that waits longer than kNatTimeout sets abort_word, and every wave that sees it stops
// waiting and takes NaN operands, so the grid always drains.
// The arithmetic is the level kernel's: same products, same shuffle-ordered subtraction, the
// forward result 0.0 + 1.0 * (rhs / a_RR), the backward one v_R + 1.0 * (rhs / a_RR).
#ifndef NAT_POLL_DEPTH
#define NAT_POLL_DEPTH 1  // build-flag A/B knob: polls in flight per pending operand
#endif
constexpr unsigned long long kNatPending = ~0ull;
#ifndef NAT_BACKOFF_MAX
#define NAT_BACKOFF_MAX 1  // build-flag A/B knob: longest pause between polls, in s_sleep 1 units
#endif
// the pause before the next poll of a wait: 1, 2, 4, ... NAT_BACKOFF_MAX s_sleep 1 periods
__device__ __forceinline__ void nat_backoff(int &k) {
  for (int i = 0; i < k; i++) __builtin_amdgcn_s_sleep(1);
  k = k * 2 < NAT_BACKOFF_MAX ? k * 2 : NAT_BACKOFF_MAX;
}
constexpr unsigned long long kNatTimeout = 100000000ull;  // wall_clock64 ticks (100 MHz): 1 s

// The sweeps' tails (PNP_NAT_TAIL, off by default): the natural order's dependency graph is wide
// for its first levels and then narrow for as many again (pore_pnp k=4, PNP: 171 levels holding
// 2.14 M rows, then 177 levels of 78 K rows; PB: 63 levels of 676 K rows, then 206 of 62 K).
// Across CUs each hop costs a write-through store and a poll served from the memory side (~2.5 us
// per level, measured); the tail units can instead run in ONE workgroup of 16 waves on one CU,
// polling each other through that CU's caches (workgroup-scope atomics).  Measured slower: one CU
// works through a tail level's ~55 units 16 at a time, each with its own load latency (PNP
// config 3: 2.36 ms per application without a tail, 3.29 / 4.83 ms with 512 / 1024-row tails;
// profiles/r04/ssor_natural_tail_r4e.log).  Launch order: forward head (the resident grid),
// forward tail (one workgroup), backward head, backward tail.
template <int SCOPE>
__device__ __forceinline__ unsigned long long nat_ld(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, SCOPE);
}

// Co-residency probe (ssor_natural_flow_resident): the head and chain kernels launched with their
// full grid and a negative u0 / bwd only check in -- thread 0 of every workgroup adds one to w[0]
// and waits until the whole grid has arrived.  A grid that is not resident at once cannot arrive
// in full: its waiting workgroups give up after kNatProbeTimeout and set w[1], so the probe always
// drains.  The same kernel, so the same registers and LDS: the probe measures the residency the
// dataflow launch relies on (the occupancy query can over-report by a block per CU, §0.4).
constexpr unsigned long long kNatProbeTimeout = 2000000ull;  // wall_clock64 ticks: 20 ms
__device__ __forceinline__ void nat_probe(unsigned *w) {
  if (threadIdx.x != 0) return;
  __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gridDim.x) {
    if (wall_clock64() - t0 > kNatProbeTimeout) {
      __hip_atomic_store(w + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// PAD > 0: the workgroup reserves PAD bytes of LDS it never uses, so that at most one workgroup
// runs per CU (the sparse tail grid, below).  KS: entries per lane and pass (KS * kL per row and
// pass); rows longer than that take several passes, each a full load -> poll round trip.  KS = 4
// (32 entries) takes PNP's phi rows (3 (degree + 1) entries, 27 at degree 8) in one pass, but was
// slower at config 3 (PNP_NAT_FLOW_KS4, off by default).
template <int BLK, int SCOPE, int PAD = 0, int KS = kS>
__global__ void __launch_bounds__(BLK)
    k_ssor_nat_flow(const int4 *__restrict__ units, int u0, int u1, int nunits_f,
                    const int4 *__restrict__ info_f, const int *__restrict__ ecol_f,
                    const int4 *__restrict__ info_b, const int *__restrict__ ecol_b,
                    const double *__restrict__ val, const double *__restrict__ d,
                    unsigned long long *vf, unsigned long long *vb, unsigned *abort_word,
                    int spec = 0) {
  if constexpr (PAD > 0) {
    __shared__ char pad[PAD];
    if (u0 < -1) reinterpret_cast<volatile char *>(pad)[threadIdx.x] = 1;  // never: u0 >= -1
  }
  if (u0 < 0) {  // co-residency probe
    nat_probe(abort_word);
    return;
  }
  const int lane = threadIdx.x % 64, t = lane / kL, j = lane % kL, base = lane - j;
  const int G = gridDim.x * (BLK / 64);
  for (int u = u0 + blockIdx.x * (BLK / 64) + threadIdx.x / 64; u < u1; u += G) {
    const int4 U = units[u];
    const bool bwd = u >= nunits_f;  // uniform
    const int rows = U.y & 255, width = (U.y >> 8) & 255;
    const int4 *info = bwd ? info_b : info_f;
    const int *ecol = bwd ? ecol_b : ecol_f;
    const bool live = t < rows;
    const bool head = live && j == 0;
    const int4 I = live ? info[U.x + t] : make_int4(0, 0, 0, 0);
    double rhs = 0.0;
    for (int kb = 0; kb < width; kb += KS * kL) {
      int c[KS], ix[KS];
#pragma unroll
      for (int q = 0; q < KS; q++) {
        const int k = kb + j + q * kL;
        const bool in = live && k < width;
        const size_t at = size_t(U.w) + size_t(k) * U.z + t;
        c[q] = in ? ecol[at] : -1;
        ix[q] = (in && k < (I.y & 255)) ? I.z + k : -1;  // the row's entries: contiguous in val
      }
      if (kb == 0 && head) rhs = d[I.w];  // d: internal layout
      unsigned long long b[KS];
      double a[KS];
#pragma unroll
      for (int q = 0; q < KS; q++) {
        a[q] = ix[q] >= 0 ? val[ix[q]] : 0.0;
        // a backward unit's forward-value operands were final when the launch began (the forward
        // sweep is an earlier launch): plain, cacheable loads; only this launch's results are
        // polled (PNP config 3: backward head 464 -> 435 us, profiles/r05/nat_split_r5c.txt).
        // With `spec`, a forward unit also tries a plain load first: a value that is not all-ones
        // is final (each is written once), a pending one is polled as before
        b[q] = c[q] == -1 ? 0ull
               : (c[q] >= 0 && (bwd || spec)) ? vf[c[q]]
                                              : nat_ld<SCOPE>(c[q] >= 0 ? vf + c[q] : vb + (-(c[q] + 2)));
      }
      bool pend = false;
#pragma unroll
      for (int q = 0; q < KS; q++) pend |= b[q] == kNatPending;
      if (__any(pend)) {
        const unsigned long long t0 = wall_clock64();
        // NAT_POLL_DEPTH polls in flight per pending operand: a new poll is issued every pass and
        // the oldest one consumed, so an arriving value is seen about one round trip after it
        // lands instead of up to two (depth 1: issue, wait, check)
        constexpr int PD = NAT_POLL_DEPTH;
        unsigned long long fl[PD > 1 ? PD - 1 : 1][KS];
#pragma unroll
        for (int p = 0; p + 1 < PD; p++) {
#pragma unroll
          for (int q = 0; q < KS; q++)
            fl[p][q] = b[q] == kNatPending
                           ? nat_ld<SCOPE>(c[q] >= 0 ? vf + c[q] : vb + (-(c[q] + 2)))
                           : 0ull;
          __builtin_amdgcn_s_sleep(1);
        }
        while (true) {
          __builtin_amdgcn_s_sleep(1);
          pend = false;
          if constexpr (PD > 1) {
            unsigned long long nw[KS];
#pragma unroll
            for (int q = 0; q < KS; q++)
              nw[q] = b[q] == kNatPending
                          ? nat_ld<SCOPE>(c[q] >= 0 ? vf + c[q] : vb + (-(c[q] + 2)))
                          : 0ull;
#pragma unroll
            for (int q = 0; q < KS; q++)
              if (b[q] == kNatPending) {
                b[q] = fl[0][q];
                pend |= b[q] == kNatPending;
              }
#pragma unroll
            for (int p = 0; p + 2 < PD; p++)
#pragma unroll
              for (int q = 0; q < KS; q++) fl[p][q] = fl[p + 1][q];
#pragma unroll
            for (int q = 0; q < KS; q++) fl[PD - 2][q] = nw[q];
          } else {
#pragma unroll
            for (int q = 0; q < KS; q++)
              if (b[q] == kNatPending) {
                b[q] = nat_ld<SCOPE>(c[q] >= 0 ? vf + c[q] : vb + (-(c[q] + 2)));
                pend |= b[q] == kNatPending;
              }
          }
          if (!__any(pend)) break;
          const bool late = wall_clock64() - t0 > kNatTimeout;
          if (late && lane == 0) __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
          if (late || __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
#pragma unroll
            for (int q = 0; q < KS; q++)
              if (b[q] == kNatPending) b[q] = 0x7FF8000000000000ull;  // NaN: drain the grid
            break;
          }
        }
      }
      double pr[KS];
#pragma unroll
      for (int q = 0; q < KS; q++) pr[q] = ix[q] >= 0 ? a[q] * __longlong_as_double(b[q]) : 0.0;
#pragma unroll
      for (int k = 0; k < KS * kL; k++) {
        const double p = __shfl(pr[k / kL], base + k % kL, 64);
        if (head && kb + k < width) rhs -= p;
      }
    }
    if (head) {
      // the row's own forward value is final: its diagonal entry's operand was waited for above
      double own = 0.0;
      if (bwd) own = __longlong_as_double(vf[I.x]);  // final since the forward launches
      const double out = own + 1.0 * (rhs / val[I.z + (I.y >> 8)]);
      __hip_atomic_store(bwd ? vb + I.x : vf + I.x,
                         (unsigned long long)__double_as_longlong(out), __ATOMIC_RELAXED, SCOPE);
    }
  }
}
// The same dataflow, software-pipelined across a wave's units (the default head; units of at most
// kC entries per row, one pass).  The flow kernel above starts loading a unit's entries only when
// it has finished its previous one: two dependent round trips (ELL slots, then values and
// operands) land on the critical path of every level a wave joins late, ~4.3 us per wide level
// against ~2.4 for a hop (PNP config 3, profiles/r04/chain2/nat_split_d4_8192.txt).  Here the
// wave holds three units at once: it computes unit k while unit k+1's values, d, a_RR and first
// operand loads (stage B, from unit k+1's ELL slots) and unit k+2's record and ELL slots (stage
// A) are in flight.  Each stage has one register set, read before it is reloaded, and every load
// is unconditional (positions clamped into the unit, padding selected afterwards), so the waits
// count loads instead of draining them.  Operands still pending at compute time are polled as in
// the flow kernel; the arithmetic is the flow kernel's, bit for bit.
template <int BLK>
__global__ void __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(4)))
    k_ssor_nat_pipe(const int4 *__restrict__ units, int u0, int u1, int nunits_f,
                    const int4 *__restrict__ info_f, const int *__restrict__ ecol_f,
                    const int4 *__restrict__ info_b, const int *__restrict__ ecol_b,
                    const double *__restrict__ val, const double *__restrict__ d,
                    unsigned long long *vf, unsigned long long *vb, unsigned *abort_word) {
  if (u0 < 0) {  // co-residency probe
    nat_probe(abort_word);
    return;
  }
  const int lane = threadIdx.x % 64, t = lane / kL, j = lane % kL, base = lane - j;
  const int G = gridDim.x * (BLK / 64);
  // wave-uniform (readfirstlane): the unit records become scalar loads, off the vector counter
  const int ufirst =
      __builtin_amdgcn_readfirstlane(u0 + blockIdx.x * (BLK / 64) + int(threadIdx.x) / 64);
  if (ufirst >= u1) return;
  auto opnd = [&](int c) { return c >= 0 ? vf + c : vb + (-(c + 2)); };
  auto ld = [&](const unsigned long long *q) {
    return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  // two register sets per stage, used alternately (the loop below is unrolled by two), so that no
  // stage register is copied while its load is in flight
  int4 aU[2], aI[2];
  int ac[2][kS];
  int bc[2][kS], bx[2][kS], brow[2], bw8[2], bwid[2];
  double ba[2][kS], bd[2], bg[2];
  unsigned long long bb[2][kS], bo[2];
  // stage A: the unit, its rows' records and ELL slots (raw; padding resolved in stage B)
  auto stage_a = [&](int u, int S) {
    const int uu = u < u1 ? u : u1 - 1;
    aU[S] = units[uu];
    const bool bw = uu >= nunits_f;
    const int rows = aU[S].y & 255, width = (aU[S].y >> 8) & 255;
    const int tt = t < rows ? t : rows - 1;
    aI[S] = (bw ? info_b : info_f)[aU[S].x + tt];
    const int *ec = bw ? ecol_b : ecol_f;
#pragma unroll
    for (int q = 0; q < kS; q++) {
      const int k = j + q * kL, kk = k < width ? k : width - 1;
      const size_t at = size_t(aU[S].w) + size_t(kk) * aU[S].z + tt;
      ac[S][q] = ec[at];
    }
  };
  // stage B: what the compute needs, from stage A's registers of the same set
  auto stage_b = [&](int S) {
    const int rows = aU[S].y & 255, width = (aU[S].y >> 8) & 255;
    const bool live = t < rows;
    brow[S] = aI[S].x;
    bw8[S] = t < rows ? 1 : 0;
    bwid[S] = width;  // wave-uniform (the unit record is a scalar load)
#pragma unroll
    for (int q = 0; q < kS; q++) {
      const bool in = live && j + q * kL < width;
      bc[S][q] = in ? ac[S][q] : -1;
      // the row's entries are contiguous in val from aI.z
      bx[S][q] = (in && j + q * kL < (aI[S].y & 255)) ? aI[S].z + j + q * kL : -1;
      // materialised here: the compiler would otherwise sink the selects below the next stage A
      // load into ac / ax, keep both generations live and copy them at the loop latch, waiting
      // for those loads
      asm volatile("" : "+v"(bc[S][q]), "+v"(bx[S][q]));
      ba[S][q] = val[bx[S][q] >= 0 ? bx[S][q] : 0];
      bb[S][q] = ld(ac[S][q] == -1 ? vf : opnd(ac[S][q]));
    }
    asm volatile("" : "+v"(brow[S]), "+v"(bw8[S]));
    bd[S] = d[aI[S].w];  // d: internal layout
    bg[S] = val[aI[S].z + (aI[S].y >> 8)];
    bo[S] = ld(vf + aI[S].x);  // the row's forward value (backward units)
  };
  // Each row of the unit is stored as soon as ITS operands are final (ballot over its kL lanes),
  // not when the whole unit's are: a wide level's unit depends on ~24 producers, and waiting for
  // the last of them put the slowest hand-off of every unit on the critical path.  The products
  // and the ordered subtraction are recomputed for the whole wave whenever a row becomes ready
  // (rows already stored, or not ready, discard theirs).
  auto compute = [&](int u, int S) {
    const bool bwd = u >= nunits_f;  // uniform
    const bool live = bw8[S] & 1, head = live && j == 0;
    const int width = bwid[S];
    unsigned long long b[kS];
#pragma unroll
    for (int q = 0; q < kS; q++) b[q] = bc[S][q] == -1 ? 0ull : bb[S][q];
    unsigned long long own = bo[S];
    bool pend = bwd && head && own == kNatPending;
#pragma unroll
    for (int q = 0; q < kS; q++) pend |= b[q] == kNatPending;
    bool stored = !live;  // per row (all its lanes agree)
    const unsigned long long t0 = wall_clock64();
    int bk = 1;
    while (true) {
      const unsigned long long pm = __ballot(pend);
      const bool ready = !stored && ((pm >> base) & ((1ull << kL) - 1)) == 0;
      if (__any(ready)) {
        double pr[kS];
#pragma unroll
        for (int q = 0; q < kS; q++)
          pr[q] = bx[S][q] >= 0 ? ba[S][q] * __longlong_as_double(b[q]) : 0.0;
        double rhs = bd[S];
        // only the unit's width: a c row of PNP has 14 entries, a PB row at most ~9 of kC = 24
#pragma unroll
        for (int k = 0; k < kC; k++) {
          if (k < width) {  // uniform
            const double p = __shfl(pr[k / kL], base + k % kL, 64);
            if (head) rhs -= p;
          }
        }
        if (head && ready) {
          const double out = (bwd ? __longlong_as_double(own) : 0.0) + 1.0 * (rhs / bg[S]);
          __hip_atomic_store(bwd ? vb + brow[S] : vf + brow[S],
                             (unsigned long long)__double_as_longlong(out), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
        stored |= ready;
      }
      if (__all(stored)) break;
      nat_backoff(bk);
      pend = false;
#pragma unroll
      for (int q = 0; q < kS; q++)
        if (b[q] == kNatPending) {
          b[q] = ld(opnd(bc[S][q]));
          pend |= b[q] == kNatPending;
        }
      if (bwd && head && own == kNatPending) {
        own = ld(vf + brow[S]);
        pend |= own == kNatPending;
      }
      const bool late = wall_clock64() - t0 > kNatTimeout;
      if (late && lane == 0) __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
      if (late || __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
#pragma unroll
        for (int q = 0; q < kS; q++)
          if (b[q] == kNatPending) b[q] = 0x7FF8000000000000ull;  // NaN: drain the grid
        if (own == kNatPending) own = 0x7FF8000000000000ull;
        pend = false;
      }
    }
  };
  stage_a(ufirst, 0);
  stage_b(0);
  stage_a(ufirst + G, 1);
  for (int u = ufirst; u < u1; u += 2 * G) {
    stage_b(1);                // unit u + G
    stage_a(u + 2 * G, 0);
    compute(u, 0);
    stage_b(0);                // unit u + 2G
    stage_a(u + 3 * G, 1);
    if (u + G < u1) compute(u + G, 1);  // uniform
  }
}

// vf[0..n) = vb[0..n) = the all-ones pending pattern, 16-B stores where both are 16-B aligned
__global__ void __launch_bounds__(kB)
    k_nat_pending(int n, double2 *vf2, double2 *vb2, double *vf, double *vb) {
  const int i = blockIdx.x * kB + threadIdx.x;  // one pair of elements per lane
  const double p = __longlong_as_double(~0ll);
  const bool al = ((reinterpret_cast<uintptr_t>(vf) | reinterpret_cast<uintptr_t>(vb)) & 15) == 0;
  if (al && 2 * i + 1 < n) {
    vf2[i] = make_double2(p, p);
    vb2[i] = make_double2(p, p);
  } else {
    for (int k = 2 * i; k < 2 * i + 2 && k < n; k++) {
      vf[k] = p;
      vb[k] = p;
    }
  }
}

constexpr int kTailBlk = 1024;  // the tail workgroup: 16 waves on one CU
// The sparse tail grid (PNP_NAT_TAIL_WPC = 1, 2 or 4 waves per CU): the tail levels on a grid of
// at most one workgroup per CU (96 KB of LDS reserved each), so that a consumer CU's memory queue
// holds only its own few waves' polls -- the hand-off price sits in the consumer CU's queue
// (MI355X_MICROARCH.md handoff-1to1: 0.8-1.1 us between unloaded CUs, 2.3-3.5 us with 8-15 busy
// waves on them), and the head grid's 16 polling waves per CU pay the latter on every tail level.
constexpr int kTailPad = 96 * 1024;

// ---- the narrow tail as chains (NatChains, PNP_NAT_CHAIN) ---------------------------------------
// In the narrow tail almost every row depends on exactly one row of the level just before its own
// (pore_pnp k=4, PB forward: 60,851 of 61,851 tail rows; tools/nat_dag.py): the tail is a forest.
// The host cuts it into heavy paths (each row continues the chain of its child with the longest
// remaining path) and packs the chains into groups by level interval; ONE WAVE walks a group's rows
// in order, lane k holding the row's entry k.  A row's operands that are the results of the group's
// last kChainH rows are taken from the wave's registers (the host marks them), so a step along a
// chain costs the row's arithmetic, not a memory hop.  Other operands are polled as in the flow
// kernel (write-through stores of final values into all-ones vectors).
// Software pipeline, so that a step waits for no memory: the row's record and entry codes are
// loaded 2D steps ahead (stage A), its values, d, a_RR and operands D steps ahead (stage B, from
// stage A's indices); the loop is unrolled by 2D so that every stage lives in fixed registers,
// and every load is unconditional (positions clamped to the group's last row), so the compiler
// can count the loads in flight instead of draining them (round 4's first chain kernel kept its
// stages in rotating structs with predicated loads and waited for every load every step:
// profiles/r04/ssor_natural_chain_r4j.log).
// The arithmetic is the level kernel's: products a_RC * v_C in column order, subtracted from d_R
// one by one, forward 0.0 + 1.0 * (rhs / a_RR), backward v_R + 1.0 * (rhs / a_RR): the oracle's
// SeqSSOR bit for bit.
// Progress: a row depends only on rows of lower levels and a group's rows are in increasing level
// order, so the lowest uncomputed row's group is at that row and its operands are final; every
// group's wave is resident (the host packs at most ssor_natural_chain_capacity() groups).
// Operand codes (host): idx << 2 | kind, kind 0: zero, 1: vf[idx], 2: vb[idx], 3: the group's
// result idx (1..kChainH) rows back.
#ifndef NAT_CHAIN_D
#define NAT_CHAIN_D 2  // build-flag A/B knob: stage-B lead in steps (stage A leads by twice that)
#endif
#ifndef NAT_CHAIN_H
#define NAT_CHAIN_H 4  // build-flag A/B knob: results kept in registers
#endif
constexpr int kChainD = NAT_CHAIN_D, kChainA = 2 * kChainD, kChainH = NAT_CHAIN_H;

__global__ void __launch_bounds__(64)
    k_ssor_nat_chain(const int *__restrict__ gptr, const int4 *__restrict__ rec,
                     const int *__restrict__ ecode, int wpad,
                     const double *__restrict__ val, const double *__restrict__ d,
                     unsigned long long *vf, unsigned long long *vb, int bwd,
                     unsigned *abort_word) {
  constexpr int D = kChainD, A = kChainA;
  if (bwd < 0) {  // co-residency probe
    nat_probe(abort_word);
    return;
  }
  const int lane = threadIdx.x;
  const int p0 = gptr[blockIdx.x], len = gptr[blockIdx.x + 1] - p0;
  if (len <= 0) return;
  const int kl = lane < wpad ? lane : wpad - 1;
  auto ld = [&](const unsigned long long *q) {
    return __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  auto opnd = [&](int c) {  // the operand's address (kind 0 and 3: a harmless dummy)
    const int k = c & 3, i = c >> 2;
    return k == 1 ? vf + i : k == 2 ? vb + i : vf;
  };
  int4 ra[A];
  int ca[A];
  double av[D], dv[D], ov[D], gv[D];
  unsigned long long bv[D];
  auto stage_a = [&](int s, int slot) {
    const int p = p0 + (s < len ? s : len - 1);
    ra[slot] = rec[p];
    ca[slot] = ecode[size_t(p) * wpad + kl];
  };
  auto stage_b = [&](int sa, int sb) {
    // lane k's entry: the row's entries are contiguous in val from rec.z
    av[sb] = val[lane < (ra[sa].y & 255) ? ra[sa].z + lane : 0];
    bv[sb] = ld(opnd(ca[sa]));
    dv[sb] = d[ra[sa].w];  // d: internal layout
    ov[sb] = __longlong_as_double(ld(vf + ra[sa].x));  // the forward value (backward sweep)
    gv[sb] = val[ra[sa].z + (ra[sa].y >> 8)];
  };
#pragma unroll
  for (int i = 0; i < A; i++) stage_a(i, i);
#pragma unroll
  for (int i = 0; i < D; i++) stage_b(i, i);
  double h[kChainH];  // the group's last results, h[0] the latest
#pragma unroll
  for (int q = 0; q < kChainH; q++) h[q] = 0.0;
  for (int s = 0; s < len; s += A) {
#pragma unroll
    for (int i = 0; i < A; i++) {
      const int st = s + i;
      if (st < len) {  // uniform
        const int c = ca[i], kind = c & 3, width = ra[i].y & 255;
        const bool live = lane < width;
        unsigned long long b = bv[i % D];
        bool pend = live && (kind == 1 || kind == 2) && b == kNatPending;
        if (__any(pend)) {
          const unsigned long long t0 = wall_clock64();
          int bk = 1;
          while (true) {
            nat_backoff(bk);
            if (pend) {
              b = ld(opnd(c));
              pend = b == kNatPending;
            }
            if (!__any(pend)) break;
            const bool late = wall_clock64() - t0 > kNatTimeout;
            if (late && lane == 0)
              __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (late || __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
              if (pend) b = 0x7FF8000000000000ull;  // NaN: drain the grid
              break;
            }
          }
        }
        const int hi = c >> 2;
        double hv = h[0];
#pragma unroll
        for (int q = 1; q < kChainH; q++)
          if (hi == q + 1) hv = h[q];
        const double o = kind == 0 ? 0.0 : kind == 3 ? hv : __longlong_as_double(b);
        const double pr = live ? av[i % D] * o : 0.0;  // lane < the row's entry count
        const unsigned long long pb = __double_as_longlong(pr);
        const int plo = int(unsigned(pb)), phi = int(unsigned(pb >> 32));
        double rhs = dv[i % D];
        for (int k = 0; k < width; k++) {
          const unsigned lo = unsigned(__builtin_amdgcn_readlane(plo, k));
          const unsigned hh = unsigned(__builtin_amdgcn_readlane(phi, k));
          rhs -= __longlong_as_double((long long)((unsigned long long)hh << 32 | lo));
        }
        const double own = bwd ? ov[i % D] : 0.0;
        const double out = own + 1.0 * (rhs / gv[i % D]);
        if (lane == 0)
          __hip_atomic_store((bwd ? vb : vf) + ra[i].x, (unsigned long long)__double_as_longlong(out),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int q = kChainH - 1; q > 0; q--) h[q] = h[q - 1];
        h[0] = out;
      }
      stage_b((i + D) % A, i % D);  // step st + D
      stage_a(st + A, i);           // step st + A
    }
  }
}
}  // namespace

int ssor_natural_unit_rows() { return kUR; }
int ssor_natural_chain_width() { return 64; }
int ssor_natural_chain_history() { return kChainH; }
int ssor_natural_chain_capacity() {
  int dev = 0, cus = 0, per = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_ssor_nat_chain, 64, 0);
  return cus * std::max(1, per);
}

// the dataflow launch's configuration (process-wide: grid from the occupancy query, A/B knobs)
struct NatFlowCfg {
  int grid, cus, tail_wpc, spec;
  bool pipe, ks4;
};
static const NatFlowCfg &nat_flow_cfg() {
  static const NatFlowCfg c = [] {
    NatFlowCfg k{};
    int dev = 0, cus = 0, per = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    int per_flow = 0, per_pipe = 0;
    int per_flow4 = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_flow,
                                                 k_ssor_nat_flow<kB, __HIP_MEMORY_SCOPE_AGENT>, kB, 0);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_flow4, k_ssor_nat_flow<kB, __HIP_MEMORY_SCOPE_AGENT, 0, 4>, kB, 0);
    per_flow = std::min(per_flow, per_flow4);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_pipe, k_ssor_nat_pipe<kB>, kB, 0);
    per = std::min(per_flow, per_pipe);  // one grid size for both head kernels: all resident
    // 4 workgroups per CU (16 waves): fewer pollers than the occupancy allows and enough for
    // the wide levels (PNP config 3: 2.25 ms per application against 2.36 at the occupancy, 2.94
    // at 1; profiles/r04/nat_wg*_r4d.log).  PNP_NAT_FLOW_WG_PER_CU overrides (capped at the
    // occupancy).  ssor_natural_flow_resident() checks the result on the device.
    const char *ev = std::getenv("PNP_NAT_FLOW_WG_PER_CU");
    per = std::min(per, (ev && std::atoi(ev) > 0) ? std::atoi(ev) : 4);
    k.grid = std::max(1, cus * std::max(1, per));
    k.cus = std::max(1, cus);
    // PNP_NAT_PIPE=0: the head as the unpipelined flow kernel (A/B)
    ev = std::getenv("PNP_NAT_PIPE");
    k.pipe = !(ev && std::atoi(ev) == 0);
    // PNP_NAT_FLOW_KS4=1: rows of 25-32 entries in one pass of 32 instead of two of 24 (A/B knob,
    // off: PNP config 3 1.584 against 1.553 ms per application, profiles/r05/nat_ks4_r5h.log)
    ev = std::getenv("PNP_NAT_FLOW_KS4");
    k.ks4 = ev && std::atoi(ev) == 1;
    // PNP_NAT_SPEC=1: forward head units try plain loads first (A/B knob, default off)
    ev = std::getenv("PNP_NAT_SPEC");
    k.spec = (ev && std::atoi(ev) != 0) ? 1 : 0;
    ev = std::getenv("PNP_NAT_TAIL_WPC");
    k.tail_wpc = ev ? std::max(0, std::atoi(ev)) : 0;
    return k;
  }();
  return c;
}

int ssor_natural_flow_resident(const NatFlow &F, unsigned *probe, hipStream_t s) {
  const NatFlowCfg &C = nat_flow_cfg();
  unsigned h[2] = {0, 0};
  auto run = [&](auto launch) -> int {
    if (hipMemsetAsync(probe, 0, 2 * sizeof(unsigned), s) != hipSuccess) return -1;
    launch();
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipMemcpyAsync(h, probe, sizeof h, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
      return -1;
    return h[1] == 0 && h[0] >= 1 ? 1 : 0;
  };
  int ok = run([&] {
    if (F.max_width <= kC && C.pipe)
      hipLaunchKernelGGL(k_ssor_nat_pipe<kB>, dim3(C.grid), dim3(kB), 0, s, F.units, -1, 0, 0,
                         F.fwd.info, F.fwd.ecol, F.bwd.info, F.bwd.ecol, nullptr, nullptr, nullptr,
                         nullptr, probe);
    else if (F.max_width <= 4 * kL && C.ks4)
      hipLaunchKernelGGL((k_ssor_nat_flow<kB, __HIP_MEMORY_SCOPE_AGENT, 0, 4>), dim3(C.grid),
                         dim3(kB), 0, s, F.units, -1, 0, 0, F.fwd.info, F.fwd.ecol, F.bwd.info,
                         F.bwd.ecol, nullptr, nullptr, nullptr, nullptr, probe, 0);
    else
      hipLaunchKernelGGL((k_ssor_nat_flow<kB, __HIP_MEMORY_SCOPE_AGENT>), dim3(C.grid), dim3(kB), 0,
                         s, F.units, -1, 0, 0, F.fwd.info, F.fwd.ecol, F.bwd.info, F.bwd.ecol,
                         nullptr, nullptr, nullptr, nullptr, probe, 0);
  });
  const int ng = std::max(F.chain_f.ngroups, F.chain_b.ngroups);
  if (ok == 1 && ng > 0)
    ok = run([&] {
      hipLaunchKernelGGL(k_ssor_nat_chain, dim3(ng), dim3(64), 0, s, F.chain_f.gptr, F.chain_f.rec,
                         F.chain_f.ecode, 0, nullptr, nullptr, nullptr, nullptr, -1, probe);
    });
  return ok;
}

hipError_t launch_ssor_natural_flow(const NatFlow &F, int n, const double *val, const double *d,
                                    double *vf, double *vb, hipStream_t s) {
  const NatFlowCfg &C = nat_flow_cfg();
  const int grid = C.grid, cus = C.cus, tail_wpc = C.tail_wpc, spec = C.spec;
  const bool pipe = C.pipe, ks4 = C.ks4;
  // both result vectors to the pending pattern in one launch (two memsets cost four fill launches,
  // ~23 us at config 3, profiles/r05/nat_split_r5d.txt)
  if (n > 0)
    hipLaunchKernelGGL(k_nat_pending, dim3((n + 2 * kB - 1) / (2 * kB)), dim3(kB), 0, s, n,
                       reinterpret_cast<double2 *>(vf), reinterpret_cast<double2 *>(vb), vf, vb);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  auto vfu = reinterpret_cast<unsigned long long *>(vf);
  auto vbu = reinterpret_cast<unsigned long long *>(vb);
  // [u0, u1) of one sweep: head units on the resident grid, tail units in one workgroup
  auto sweep = [&](int u0, int ut, int u1, const NatFlow::Chains &C, int bwd) {
    if (ut > u0) {
      const int blocks = std::min(grid, (ut - u0 + kB / 64 - 1) / (kB / 64));
      if (F.max_width <= kC && pipe)
        hipLaunchKernelGGL(k_ssor_nat_pipe<kB>, dim3(blocks), dim3(kB), 0, s, F.units, u0, ut,
                           F.nunits_f, F.fwd.info, F.fwd.ecol, F.bwd.info, F.bwd.ecol, val, d,
                           vfu, vbu, F.abort_word);
      else if (F.max_width <= 4 * kL && ks4)
        hipLaunchKernelGGL((k_ssor_nat_flow<kB, __HIP_MEMORY_SCOPE_AGENT, 0, 4>), dim3(blocks),
                           dim3(kB), 0, s, F.units, u0, ut, F.nunits_f, F.fwd.info, F.fwd.ecol,
                           F.bwd.info, F.bwd.ecol, val, d, vfu, vbu, F.abort_word, spec);
      else
        hipLaunchKernelGGL((k_ssor_nat_flow<kB, __HIP_MEMORY_SCOPE_AGENT>), dim3(blocks), dim3(kB),
                           0, s, F.units, u0, ut, F.nunits_f, F.fwd.info, F.fwd.ecol,
                           F.bwd.info, F.bwd.ecol, val, d, vfu, vbu, F.abort_word, spec);
    }
    if (u1 > ut && C.ngroups > 0)
      hipLaunchKernelGGL(k_ssor_nat_chain, dim3(C.ngroups), dim3(64), 0, s, C.gptr, C.rec, C.ecode,
                         C.wpad, val, d, vfu, vbu, bwd, F.abort_word);
    else if (u1 > ut && tail_wpc > 0) {
      const int per = tail_wpc >= 4 ? 4 : tail_wpc >= 2 ? 2 : 1;
      const int blocks = std::min(cus, (u1 - ut + per - 1) / per);
#define NAT_TAIL_GRID(W)                                                                          \
  hipLaunchKernelGGL((k_ssor_nat_flow<64 * W, __HIP_MEMORY_SCOPE_AGENT, kTailPad>), dim3(blocks), \
                     dim3(64 * W), 0, s, F.units, ut, u1, F.nunits_f, F.fwd.info, F.fwd.ecol,     \
                     F.bwd.info, F.bwd.ecol, val, d, vfu, vbu,                                   \
                     F.abort_word)
      if (per == 1) NAT_TAIL_GRID(1);
      else if (per == 2) NAT_TAIL_GRID(2);
      else NAT_TAIL_GRID(4);
#undef NAT_TAIL_GRID
    } else if (u1 > ut)
      hipLaunchKernelGGL((k_ssor_nat_flow<kTailBlk, __HIP_MEMORY_SCOPE_WORKGROUP>), dim3(1),
                         dim3(kTailBlk), 0, s, F.units, ut, u1, F.nunits_f, F.fwd.info, F.fwd.ecol,
                         F.bwd.info, F.bwd.ecol, val, d, vfu, vbu,
                         F.abort_word);
  };
  sweep(0, F.tail_f, F.nunits_f, F.chain_f, 0);
  sweep(F.nunits_f, F.tail_b, F.nunits, F.chain_b, 1);
  return hipGetLastError();
}

hipError_t launch_ssor_natural(const NatSweep &fwd, const NatSweep &bwd, const double *val,
                               const double *d, double *v, hipStream_t s) {
  for (const NatSweep *W : {&fwd, &bwd})
    for (int l = 0; l < W->nlev; l++) {
      const int n = W->lptr[l + 1] - W->lptr[l];
      const int nu = (n + kUR - 1) / kUR;  // the level's unit-major ELL (NatSweep)
      const int width = n > 0 ? int((W->eoff[l + 1] - W->eoff[l]) / ((long long)nu * kUR)) : 0;
      hipLaunchKernelGGL(k_ssor_nat_level, dim3((n * kL + kB - 1) / kB), dim3(kB), 0, s,
                         W->info + W->lptr[l], W->ecol + W->eoff[l], n,
                         width, val, d, v);
    }
  return hipGetLastError();
}

}  // namespace pnp
