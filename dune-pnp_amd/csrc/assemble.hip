// Residual + Jacobian assembly on gfx950: owner-computes, atomic-free, one thread per vertex row.
//
// The reference assembles element by element (PDELab GridOperator over alpha_volume, e.g.
// src/pnp_operator.hh:46-195) and differentiates by forward differences (NumericalJacobianVolume,
// 10 residual evaluations per PNP element), scatter-adding 81 values per element into a BCRS
// matrix.  Here each thread owns one vertex row i and walks the CCW fan of triangles around i
// (mesh.cc build_fans): element (i, v_s, v_{s+1}) contributes to row i's diagonal block, to
// block (i, v_s) and to block (i, v_{s+1}).  Block (i, v_s) only ever receives contributions
// from the two fan elements on either side of edge (i, v_s), which are consecutive in the walk,
// so it is complete after step s: it is kept in registers ("pending"), finished, and stored
// exactly once.  Slot s of the SELL row is the s-th fan neighbour, so at step s every lane of a
// wave stores slot s: all block stores are coalesced 512-byte lines and there are no atomics.
//
// Element integrals are the closed forms of the reference's order-3 quadrature where that rule
// is exact (PnpOperator / PoissonOperator integrands are polynomials of degree <= 3, also with
// the cylindrical 2*PI*y weight); PBOperator (sinh) and the PnpTOperator mass (a cubic under the
// order-2 rule, src/pnp_toperator.hh:26) use the reference's quadrature points explicitly.
#include <cstdlib>

#include <hip/hip_ext.h>

#include "kernels.h"

namespace pnp {

namespace {

struct Geo {
  double gi0, gi1, gb0, gb1, gc0, gc1;  // physical gradients of the P1 basis at i, b, c
  double adet;
};

__device__ __forceinline__ void geometry(double xi, double yi, double xb, double yb, double xc,
                                         double yc, Geo &G) {
  double J00 = xb - xi, J01 = xc - xi, J10 = yb - yi, J11 = yc - yi;
  double det = J00 * J11 - J01 * J10;
  double id = 1.0 / det;
  G.gb0 = J11 * id;
  G.gb1 = -J01 * id;
  G.gc0 = -J10 * id;
  G.gc1 = J00 * id;
  G.gi0 = -G.gb0 - G.gc0;
  G.gi1 = -G.gb1 - G.gc1;
  G.adet = fabs(det);
}

// cylindrical/planar integrals of the P1 basis on the element (i, b, c):
//   W = int w, m_j = int w psi_j, M_ij = int w psi_i psi_j  (w = 2*PI*y or 1)
struct Ints {
  double W, mi, mb, mc, Mii, Mib, Mic;
};
__device__ __forceinline__ void integrals(const Geo &G, int cyl, double pi, double yi, double yb,
                                          double yc, Ints &I) {
  if (cyl) {
    double c = 2 * pi * G.adet;
    double Y = yi + yb + yc;
    I.W = c * Y * (1.0 / 6.0);
    I.mi = c * (Y + yi) * (1.0 / 24.0);
    I.mb = c * (Y + yb) * (1.0 / 24.0);
    I.mc = c * (Y + yc) * (1.0 / 24.0);
    I.Mii = c * (yi * (1.0 / 20.0) + (yb + yc) * (1.0 / 60.0));
    I.Mib = c * ((yi + yb) * (1.0 / 60.0) + yc * (1.0 / 120.0));
    I.Mic = c * ((yi + yc) * (1.0 / 60.0) + yb * (1.0 / 120.0));
  } else {
    I.W = G.adet * 0.5;
    I.mi = I.mb = I.mc = G.adet * (1.0 / 6.0);
    I.Mii = G.adet * (1.0 / 12.0);
    I.Mib = I.Mic = G.adet * (1.0 / 24.0);
  }
}

// order-2 (3-point) rule mass, (PnpTOperator, src/pnp_toperator.hh:26 / dune-geometry order 2);
// barycentric points (1/6, 2/3, 1/6) and permutations, weight 1/6 * |det| * (2 PI y)
__device__ __forceinline__ void mass_q2(const Geo &G, int cyl, double pi, double yi, double yb,
                                        double yc, double &Mii, double &Mib, double &Mic) {
  Mii = Mib = Mic = 0;
  const double a = 1.0 / 6.0, b = 2.0 / 3.0;
  const double P[3][3] = {{a, b, a}, {a, a, b}, {b, a, a}};
#pragma unroll
  for (int q = 0; q < 3; q++) {
    double f = (1.0 / 6.0) * G.adet;
    if (cyl) f *= (P[q][0] * yi + P[q][1] * yb + P[q][2] * yc) * 2 * pi;
    Mii += f * P[q][0] * P[q][0];
    Mib += f * P[q][0] * P[q][1];
    Mic += f * P[q][0] * P[q][2];
  }
}

template <int OP>
struct OpTraits {
  static constexpr int NF = (OP == OP_PNP || OP == OP_PNP_IE) ? 3 : 1;
  static constexpr int PAT = OP == OP_PNP ? kPatPnp : (OP == OP_PNP_IE ? kPatPnpIE : kPatScalar);
  static constexpr int NV = popc9(PAT);
  // independent coefficients of one block (i, j) while it accumulates over the fan:
  //   PNP: k0 = sum G_ij W, k1 = sum kappa M_ij, k2 = sum G_ij S+, k3 = sum G_ij S-,
  //        k4 = sum (grad phi . grad psi_i) m_j, (PNP_IE) k5 = sum tau M2_ij, scaled by dt;
  //   these are what the matrix stores (k-form, kernels.h expand_k)
  static constexpr int NK = nks_of(PAT);
};

// PBOperator: a vertex's e^{u/5} and e^{-u/5}, the factors element() builds the quadrature
// points' e^u from
__device__ __forceinline__ void pb_fifth(double u, double &e, double &ei) {
  e = exp(0.2 * u);
  ei = 1.0 / e;
}

// Contributions of element (i, b, c) to row i: residual res[NF], blocks (i,i), (i,b), (i,c).
template <int OP, int JAC>
__device__ __forceinline__ void element(const AsmArgs &a, const Geo &G, double yi, double yb,
                                        double yc, const double *ui, const double *ub,
                                        const double *uc, double pi_, double pb_, double pc_,
                                        double qi, double qb, double qc, double *res, double *Bd,
                                        double *Bb, double *Bc) {
  const double PI = a.pi;
  double Gii = G.gi0 * G.gi0 + G.gi1 * G.gi1;
  double Gib = G.gb0 * G.gi0 + G.gb1 * G.gi1;
  double Gic = G.gc0 * G.gi0 + G.gc1 * G.gi1;
  if constexpr (OP == OP_PNP || OP == OP_PNP_IE) {
    Ints I;
    integrals(G, a.cylindrical, PI, yi, yb, yc, I);
    double gph0 = ui[0] * G.gi0 + ub[0] * G.gb0 + uc[0] * G.gc0;
    double gph1 = ui[0] * G.gi1 + ub[0] * G.gb1 + uc[0] * G.gc1;
    double gcp0 = ui[1] * G.gi0 + ub[1] * G.gb0 + uc[1] * G.gc0;
    double gcp1 = ui[1] * G.gi1 + ub[1] * G.gb1 + uc[1] * G.gc1;
    double gcm0 = ui[2] * G.gi0 + ub[2] * G.gb0 + uc[2] * G.gc0;
    double gcm1 = ui[2] * G.gi1 + ub[2] * G.gb1 + uc[2] * G.gc1;
    double gp = gph0 * G.gi0 + gph1 * G.gi1;
    double Sp = ui[1] * I.mi + ub[1] * I.mb + uc[1] * I.mc;
    double Sm = ui[2] * I.mi + ub[2] * I.mb + uc[2] * I.mc;
    double kap = 4 * PI * a.l_b;
    double sc = (OP == OP_PNP_IE) ? a.dt : 1.0;
    res[0] += sc * (gp * I.W + kap * ((ui[1] - ui[2]) * I.Mii + (ub[1] - ub[2]) * I.Mib +
                                      (uc[1] - uc[2]) * I.Mic));
    res[1] += sc * ((gcp0 * G.gi0 + gcp1 * G.gi1) * I.W - gp * Sp);
    res[2] += sc * ((gcm0 * G.gi0 + gcm1 * G.gi1) * I.W + gp * Sm);
    double M2ii = 0, M2ib = 0, M2ic = 0;
    if constexpr (OP == OP_PNP_IE) {
      mass_q2(G, a.cylindrical, PI, yi, yb, yc, M2ii, M2ib, M2ic);
      res[1] += a.tau * ((ui[1] + ui[2]) * M2ii + (ub[1] + ub[2]) * M2ib + (uc[1] + uc[2]) * M2ic);
    }
    if constexpr (JAC) {
      auto blk = [&](double *B, double Gij, double Mij, double mj, double M2ij) {
        B[0] += sc * Gij * I.W;
        B[1] += sc * kap * Mij;
        B[2] += sc * Gij * Sp;
        B[3] += sc * Gij * Sm;
        B[4] += sc * gp * mj;
        if constexpr (OP == OP_PNP_IE) B[5] += a.tau * M2ij;
      };
      blk(Bd, Gii, I.Mii, I.mi, M2ii);
      blk(Bb, Gib, I.Mib, I.mb, M2ib);
      blk(Bc, Gic, I.Mic, I.mc, M2ic);
    }
  } else if constexpr (OP == OP_PB) {
    // 4-point order-3 rule, barycentric (psi_i, psi_b, psi_c)
    const double P[4][3] = {{1.0 / 3, 1.0 / 3, 1.0 / 3}, {0.2, 0.6, 0.2}, {0.2, 0.2, 0.6},
                            {0.6, 0.2, 0.2}};
    const double w[4] = {0.5 * -27.0 / 48.0, 0.5 * 25.0 / 48.0, 0.5 * 25.0 / 48.0,
                         0.5 * 25.0 / 48.0};
    double gu0 = ui[0] * G.gi0 + ub[0] * G.gb0 + uc[0] * G.gc0;
    double gu1 = ui[0] * G.gi1 + ub[0] * G.gb1 + uc[0] * G.gc1;
    double gg = gu0 * G.gi0 + gu1 * G.gi1;
    double beta = 8 * PI * a.l_b * a.c0;
    // sinh and cosh at each point from e^u and e^-u (the library's sinh and cosh each cost about
    // two exps; the PB launch is issue-bound on them).  The walk passes each vertex's e^{u/5} and
    // e^{-u/5} (pi_, pb_, pc_ / qi, qb, qc), computed once per vertex of the fan: the three
    // off-centre points are fifths, (0.2, 0.6, 0.2) and its rotations, so there e^u is a product
    // of them; only the centroid takes an exp and a division of its own.  Errors: a few ulps of
    // e^|u|, absolute in the sinh term, against residual terms of at least that size.
    const double Eq = pi_ * pb_ * pc_, Iq = qi * qb * qc;
    const double eu[4] = {exp(P[0][0] * ui[0] + P[0][1] * ub[0] + P[0][2] * uc[0]), Eq * pb_ * pb_,
                          Eq * pc_ * pc_, Eq * pi_ * pi_};
    const double ei[4] = {1.0 / eu[0], Iq * qb * qb, Iq * qc * qc, Iq * qi * qi};
    double W = 0, Ri = 0, Jii = 0, Jib = 0, Jic = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      double f = w[q] * G.adet;
      if (a.cylindrical) f *= (P[q][0] * yi + P[q][1] * yb + P[q][2] * yc) * 2 * PI;
      W += f;
      Ri += f * (0.5 * (eu[q] - ei[q])) * P[q][0];
      if constexpr (JAC) {
        double ch = f * (0.5 * (eu[q] + ei[q])) * P[q][0];
        Jii += ch * P[q][0];
        Jib += ch * P[q][1];
        Jic += ch * P[q][2];
      }
    }
    res[0] += gg * W + beta * Ri;
    if constexpr (JAC) {
      Bd[0] += Gii * W + beta * Jii;
      Bb[0] += Gib * W + beta * Jib;
      Bc[0] += Gic * W + beta * Jic;
    }
  } else if constexpr (OP == OP_DIFF || OP == OP_DIFF_IE) {
    // DiffusionOperator: no cylindrical weight (quirk Q8); grad Phi of the frozen potential
    double W = G.adet * 0.5, m = G.adet * (1.0 / 6.0);
    double gu0 = ui[0] * G.gi0 + ub[0] * G.gb0 + uc[0] * G.gc0;
    double gu1 = ui[0] * G.gi1 + ub[0] * G.gb1 + uc[0] * G.gc1;
    double gP0 = pi_ * G.gi0 + pb_ * G.gb0 + pc_ * G.gc0;
    double gP1 = pi_ * G.gi1 + pb_ * G.gb1 + pc_ * G.gc1;
    double gpP = gP0 * G.gi0 + gP1 * G.gi1;
    double sc = (OP == OP_DIFF_IE) ? a.dt : 1.0;
    res[0] += sc * ((gu0 * G.gi0 + gu1 * G.gi1) * W + a.z * gpP * m * (ui[0] + ub[0] + uc[0]));
    double Mii = G.adet * (1.0 / 12.0), Mij = G.adet * (1.0 / 24.0);
    if constexpr (OP == OP_DIFF_IE) res[0] += ui[0] * Mii + (ub[0] + uc[0]) * Mij;
    if constexpr (JAC) {
      Bd[0] += sc * (Gii * W + a.z * gpP * m);
      Bb[0] += sc * (Gib * W + a.z * gpP * m);
      Bc[0] += sc * (Gic * W + a.z * gpP * m);
      if constexpr (OP == OP_DIFF_IE) {
        Bd[0] += Mii;
        Bb[0] += Mij;
        Bc[0] += Mij;
      }
    }
  } else {  // OP_POISSON: frozen c+ (aux0 -> pi_, ..) and c- (aux1 -> qi, ..)
    Ints I;
    integrals(G, a.cylindrical, PI, yi, yb, yc, I);
    double gu0 = ui[0] * G.gi0 + ub[0] * G.gb0 + uc[0] * G.gc0;
    double gu1 = ui[0] * G.gi1 + ub[0] * G.gb1 + uc[0] * G.gc1;
    double kap = a.l_b * 4 * PI;
    res[0] += (gu0 * G.gi0 + gu1 * G.gi1) * I.W +
              kap * ((qi - pi_) * I.Mii + (qb - pb_) * I.Mib + (qc - pc_) * I.Mic);
    if constexpr (JAC) {
      Bd[0] += Gii * I.W;
      Bb[0] += Gib * I.W;
      Bc[0] += Gic * I.W;
    }
  }
}


// store one block's coefficients (k-form, OpTraits::NK values, unmasked: the Dirichlet rows are
// applied by the consumers, see kernels.h expand_k / mask_rows)
template <int OP>
__device__ __forceinline__ void store_block(double *__restrict__ vc, int lane, int s,
                                            const double *Kc) {
  constexpr int NK = OpTraits<OP>::NK;
  // non-temporal: the blocks are read back only by later kernels (SpMV, split), which stream
  // them non-temporally too; plain stores allocate the 207 MB in the caches and evict the
  // gathered x / xy / column indices.  94 -> 77 us at config 3 (profiles/r01/ab_asm_nt_stores.log)
#ifdef ASM_STORE_PLAIN  // A/B build flag: plain (allocating) block stores
  store_vals<NK>(vc + size_t(s) * NK * kRows, lane, Kc);
#else
  store_vals_nt<NK>(vc + size_t(s) * NK * kRows, lane, Kc);
#endif
}

// One thread per owned vertex row.  JAC = 0: residual only (Newton line search).
// FANR > 0: the row's column indices (fans of at most FANR - 1 neighbours) are loaded once into
// registers, so the fan walk issues no dependent index loads.  On gfx9-family ISAs vmcnt counts
// loads and stores in issue order: an index load issued behind an element's SELL block stores
// could not be consumed before those stores drained (the FANR = 0 path waits vmcnt(0) per
// element).
// (Non-temporal loads of the once-read row streams -- fan metadata, column indices, constant
// load, mask -- and a non-temporal residual store: 77 -> 96 us, profiles/r01/ab_asm_nt_row_streams.log)
template <int OP, int JAC, int MINW, int FANR>
__global__ __launch_bounds__(256, MINW) void k_assemble(DevLayout L, AsmArgs a) {
  using T = OpTraits<OP>;
  constexpr int NF = T::NF, NK = T::NK;
  const int row = xcd_block(blockIdx.x, gridDim.x, L.xcd_remap) * blockDim.x + threadIdx.x;
  if (row >= L.n_owned) return;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = L.chunk_off[chunk];
  const uint64_t meta = L.rowmeta[row];
  const int len = int(meta & 63);
  const bool closed = (meta >> 6) & 1;
  const unsigned brk = unsigned(meta >> 8);  // fan-break bits, bit s: no element after slot s
  const int *__restrict__ cix = L.colidx + off + lane;
  double *__restrict__ vc = a.vals + size_t(off) * NK;  // chunk base (k-form), see vin()

  const double2 pi2 = reinterpret_cast<const double2 *>(L.xy)[row];
  double ui[NF];
#pragma unroll
  for (int f = 0; f < NF; f++) ui[f] = a.x[size_t(row) * NF + f];
  double ai = 0, aq = 0;
  if constexpr (OP == OP_DIFF || OP == OP_DIFF_IE || OP == OP_POISSON) ai = a.aux0[row];
  if constexpr (OP == OP_POISSON) aq = a.aux1[row];
  if constexpr (OP == OP_PB) pb_fifth(ui[0], ai, aq);  // element(): e^{u/5}, e^{-u/5} per vertex

  double R[NF], D[NK], P[NK], F[NK];  // block coefficients, see OpTraits::NK
#pragma unroll
  for (int f = 0; f < NF; f++) R[f] = 0;
#pragma unroll
  for (int v = 0; v < NK; v++) D[v] = P[v] = F[v] = 0;

  // Software-pipelined fan walk.  Element s is (i, v_s, v_t) with t = s+1 (or 1 when a closed
  // fan wraps); consecutive elements share v_{s+1}, so each neighbour's data (coordinates, NF
  // dofs, frozen fields) is gathered once, one element ahead, and its column index two ahead.
  auto next_slot = [&](int s) { return (s + 1 < len) ? s + 1 : (closed ? 1 : -1); };
  auto load_nb = [&](int j, double2 &p, double (&u)[NF], double &a0, double &a1) {
    p = reinterpret_cast<const double2 *>(L.xy)[j];
    load_nf<NF>(a.x, size_t(j), u);
    if constexpr (OP == OP_DIFF || OP == OP_DIFF_IE || OP == OP_POISSON) a0 = a.aux0[j];
    if constexpr (OP == OP_POISSON) a1 = a.aux1[j];
  };
  double2 pc, pn;               // coordinates of v_s (current) and v_t (next)
  double uc[NF], un[NF];        // dofs of v_s, v_t
  double ac0 = 0, ac1 = 0, an0 = 0, an1 = 0;
  constexpr int NC = FANR > 0 ? FANR : 1;
  int cj[NC];
  if constexpr (FANR > 0) {
#pragma unroll
    // branch-free: past the fan, slot 0 (the diagonal, column = row) is read instead, so all
    // index loads issue back to back (guarded loads were serialised by the register allocator)
    for (int k = 1; k < FANR; k++) cj[k] = cix[(k < len ? k : 0) * kRows];
  }
  // column of slot k (FANR path: k is the wave-uniform s + c, or 1 after a wrap)
  auto col = [&](int k) -> int {
    if constexpr (FANR > 0)
      return cj[k];
    else
      return cix[k * kRows];
  };
  load_nb(col(1), pc, uc, ac0, ac1);
  if constexpr (OP == OP_PB) pb_fifth(uc[0], ac0, ac1);
  {
    const int t1 = next_slot(1);
    if (t1 > 0) load_nb(t1 == 1 ? col(1) : col(2), pn, un, an0, an1);
  }
  int jn = -1;  // FANR = 0: column index of the slot needed two elements ahead
  if constexpr (FANR == 0) {
    const int t2 = next_slot(1) > 0 ? next_slot(next_slot(1)) : -1;
    if (t2 > 0 && next_slot(1) != 1) jn = cix[t2 * kRows];
  }
  for (int s = 1; s < len; ++s) {
    const int t = next_slot(s);
    // prefetch the data of the slot the next element needs, and the index after that
    const int tn = (t > 0 && t != 1) ? next_slot(t) : -1;
    double2 pp = pn;
    double up[NF];
    double ap0 = 0, ap1 = 0;
    if (tn > 0) {
      if constexpr (FANR > 0) {
        load_nb(tn == 1 ? col(1) : col(s + 2), pp, up, ap0, ap1);  // tn is s + 2 or a wrap to 1
      } else {
        load_nb(jn, pp, up, ap0, ap1);
        const int tnn = tn != 1 ? next_slot(tn) : -1;
        jn = tnn > 0 ? cix[tnn * kRows] : -1;
      }
    }
    const bool elem = t > 0 && !((brk >> s) & 1);
    // v_t's e^{u/5} for this element and, rotated into v_s, the next one
    if constexpr (OP == OP_PB)
      if (t > 0) pb_fifth(un[0], an0, an1);
    if (elem) {
      Geo G;
      geometry(pi2.x, pi2.y, pc.x, pc.y, pn.x, pn.y, G);
      double Ct[NK];
#pragma unroll
      for (int v = 0; v < NK; v++) Ct[v] = 0;
      // P (pending block of slot s) receives this element's (i, v_s) contribution directly
      element<OP, JAC>(a, G, pi2.y, pc.y, pn.y, ui, uc, un, ai, ac0, an0, aq, ac1, an1, R, D, P,
                       Ct);
      if constexpr (JAC) {
        if (s == 1 && closed) {
#pragma unroll
          for (int v = 0; v < NK; v++) F[v] = P[v];
        } else {
          store_block<OP>(vc, lane, s, P);
        }
#pragma unroll
        for (int v = 0; v < NK; v++) P[v] = Ct[v];
      }
    } else if constexpr (JAC) {
      store_block<OP>(vc, lane, s, P);
#pragma unroll
      for (int v = 0; v < NK; v++) P[v] = 0;
    }
    // rotate: v_t becomes the current neighbour, the prefetched one the next
    pc = pn;
#pragma unroll
    for (int f = 0; f < NF; f++) uc[f] = un[f];
    ac0 = an0;
    ac1 = an1;
    if (tn > 0) {
      pn = pp;
#pragma unroll
      for (int f = 0; f < NF; f++) un[f] = up[f];
      an0 = ap0;
      an1 = ap1;
    }
  }
  if constexpr (JAC) {
    if (closed) {
#pragma unroll
      for (int v = 0; v < NK; v++) F[v] += P[v];
      store_block<OP>(vc, lane, 1, F);
    }
    store_block<OP>(vc, lane, 0, D);
  }
#pragma unroll
  for (int f = 0; f < NF; f++) {
    const size_t q = size_t(row) * NF + f;
    const double rv = R[f] + a.cvec[q];
    a.r[q] = a.dmask[q] != 0 ? 0.0 : rv;
  }
}

// Gather-all variant (GA): every neighbour's data (coordinates, NF dofs, frozen fields) of the
// row's fan is loaded into registers before the walk, so the gathers of the whole fan are in
// flight together (one memory round trip per row instead of one per element; the pipelined walk
// above keeps ~1 element of loads in flight), and the block stores of the walk never sit in front
// of a load the walk still waits for.  Same element() calls with the same operands in the same
// order as k_assemble (the compiler's FMA contraction may still differ in the last bit).  Fans of
// at most FANR - 1 neighbours.  Rows come in the spatial block order (row_block, DevLayout::
// blkmap), so an XCD's rows share the neighbours they gather in its L2.  Config 3: pipelined walk
// 76.5 us; gather-all at 2 waves/SIMD (180 VGPRs) 72.2 us, with the block map 58.5 us; slots 1-5
// first and 6-8 after element 4 (SPLIT 6) fits 3 waves in 160 VGPRs: 54.5 us
// (profiles/r01/ab_asm_gather_all.log, ab_blkmap_gather_all.log, ab_asm_ga_split_blkmap.log).
// SPLIT < FANR: only slots 1 .. SPLIT-1 are gathered up front; the rest are issued after element
// SPLIT-2, when the first elements' neighbour registers are free again (fewer live VGPRs).
// LDSG: the fan neighbours' coordinates, dofs and frozen fields come from LDS, where the
// workgroup first gathered them once per distinct column of its 256 rows (DevLayout::uptr /
// ulist / lidx, as the LDS-staged SpMV): half the scattered gathers of the direct walk.
#ifndef ASM_SU
#define ASM_SU 4  // staged list entries per thread issued together (build-flag A/B knob)
#endif
template <int OP>
__host__ __device__ constexpr int asm_lds_rec() {  // doubles per staged column
  return 2 + OpTraits<OP>::NF + (OP == OP_DIFF || OP == OP_DIFF_IE || OP == OP_POISSON) +
         (OP == OP_POISSON);
}
template <int OP, int JAC, int MINW, int FANR, int SPLIT = FANR, int STAGE = 0, int LDSG = 0>
__global__ __launch_bounds__(256, MINW) void k_assemble_ga(DevLayout L, AsmArgs a) {
  using T = OpTraits<OP>;
  constexpr int NF = T::NF, NK = T::NK, NS = FANR;
  constexpr bool AUX0 = OP == OP_DIFF || OP == OP_DIFF_IE || OP == OP_POISSON;
  constexpr bool AUX1 = OP == OP_POISSON;
  constexpr int RW = asm_lds_rec<OP>();
  extern __shared__ double srec[];  // LDSG: [cnt][RW] = x, y, dofs, aux0, aux1
  const int blk = row_block(L, blockIdx.x, gridDim.x);
  const int row0 = blk * blockDim.x + threadIdx.x;
  const bool live = row0 < L.n_owned;
  if (!LDSG && !live) return;
  // the row's own loads first (LDSG: they are in flight while the workgroup stages the
  // neighbour records, instead of after its barrier)
  const int row = live ? row0 : 0;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = L.chunk_off[chunk];
  const uint64_t meta = L.rowmeta[row];
  const int len = int(meta & 63);
  const bool closed = (meta >> 6) & 1;
  const unsigned brk = unsigned(meta >> 8);  // fan-break bits, bit s: no element after slot s
  double *__restrict__ vc = a.vals + size_t(off) * NK;  // chunk base (k-form), see vin()

  int cj[NS];  // the fan's columns (LDSG: their positions in the staged list)
  if constexpr (LDSG) {
    const uint16_t *__restrict__ lix = L.lidx + off + lane;
#pragma unroll
    for (int k = 1; k < NS; k++) {  // past the fan: entry 0 (slot 0's own row is not staged)
      const int t = lix[(k < len ? k : 0) * kRows];
      cj[k] = k < len ? t : 0;
    }
  } else {
    const int *__restrict__ cix = L.colidx + off + lane;
#pragma unroll
    for (int k = 1; k < NS; k++) cj[k] = cix[(k < len ? k : 0) * kRows];  // past the fan: the row
  }
  const double2 pi2 = reinterpret_cast<const double2 *>(L.xy)[row];
  double ui[NF];
  load_nf<NF>(a.x, size_t(row), ui);
  double ai = 0, aq = 0;
  if constexpr (AUX0) ai = a.aux0[row];
  if constexpr (AUX1) aq = a.aux1[row];
  if constexpr (OP == OP_PB) pb_fifth(ui[0], ai, aq);  // element(): e^{u/5}, e^{-u/5} per vertex
  if constexpr (LDSG) {
    const int u0 = L.uptr[blk], cnt = L.uown[blk];  // the fan neighbours (own rows come after)
    // up to ASM_SU list entries per thread: their list loads, then their gathers, then the LDS
    // stores (two round trips, not two per entry; ~1,000 distinct columns per block at config 3)
    constexpr int kSU = ASM_SU;
    int jj[kSU];
#pragma unroll
    for (int u = 0; u < kSU; u++) {
      const int k = int(threadIdx.x) + u * 256;
      jj[u] = k < cnt ? L.ulist[u0 + k] : -1;
    }
    double t[kSU][RW];
#pragma unroll
    for (int u = 0; u < kSU; u++)
      if (jj[u] >= 0) {
        const double2 p = reinterpret_cast<const double2 *>(L.xy)[jj[u]];
        t[u][0] = p.x;
        t[u][1] = p.y;
        double uu[NF];
        load_nf<NF>(a.x, size_t(jj[u]), uu);
#pragma unroll
        for (int f = 0; f < NF; f++) t[u][2 + f] = uu[f];
        if constexpr (AUX0) t[u][2 + NF] = a.aux0[jj[u]];
        if constexpr (AUX1) t[u][3 + NF] = a.aux1[jj[u]];
      }
#pragma unroll
    for (int u = 0; u < kSU; u++)
      if (jj[u] >= 0)
#pragma unroll
        for (int w = 0; w < RW; w++) srec[size_t(int(threadIdx.x) + u * 256) * RW + w] = t[u][w];
    for (int k = int(threadIdx.x) + kSU * 256; k < cnt; k += blockDim.x) {
      const int j = L.ulist[u0 + k];
      const double2 p = reinterpret_cast<const double2 *>(L.xy)[j];
      double u[NF];
      load_nf<NF>(a.x, size_t(j), u);
      double *r = srec + size_t(k) * RW;
      r[0] = p.x;
      r[1] = p.y;
#pragma unroll
      for (int f = 0; f < NF; f++) r[2 + f] = u[f];
      if constexpr (AUX0) r[2 + NF] = a.aux0[j];
      if constexpr (AUX1) r[3 + NF] = a.aux1[j];
    }
    __syncthreads();
    if (!live) return;
  }
  double2 pn[NS];
  double un[NS][NF], a0[NS], a1[NS];
  auto gather = [&](int k) {
    if constexpr (LDSG) {
      const double *r = srec + size_t(cj[k]) * RW;
      pn[k] = make_double2(r[0], r[1]);
#pragma unroll
      for (int f = 0; f < NF; f++) un[k][f] = r[2 + f];
      a0[k] = AUX0 ? r[2 + NF] : 0.0;
      a1[k] = AUX1 ? r[3 + NF] : 0.0;
    } else {
      pn[k] = reinterpret_cast<const double2 *>(L.xy)[cj[k]];
      load_nf<NF>(a.x, size_t(cj[k]), un[k]);
      a0[k] = AUX0 ? a.aux0[cj[k]] : 0.0;
      a1[k] = AUX1 ? a.aux1[cj[k]] : 0.0;
    }
  };
#pragma unroll
  for (int k = 1; k < SPLIT; k++) gather(k);
  // PB: slot k's e^{u/5} goes to a0[k] / a1[k] when element k - 1 needs it (slot 1: up front)
  if constexpr (OP == OP_PB) pb_fifth(un[1][0], a0[1], a1[1]);

  double R[NF], D[NK], P[NK], F[NK];
#pragma unroll
  for (int f = 0; f < NF; f++) R[f] = 0;
#pragma unroll
  for (int v = 0; v < NK; v++) D[v] = P[v] = F[v] = 0;
  // STAGE: blocks finished before the second-half gathers are issued (slots 1 .. SPLIT-3) wait
  // in LDS and go out right after those gathers: vmcnt retires loads and stores in issue order,
  // so a gather issued behind a store also waits for the store (A/B knob PNP_ASM_GA=6)
  constexpr int NSTG = (STAGE && JAC && SPLIT < NS && SPLIT > 3) ? SPLIT - 3 : 0;
  __shared__ double stg[NSTG > 0 ? NSTG * NK * 256 : 1];
  unsigned staged = 0;
  auto put = [&](int s, const double *Kc) {
    if (NSTG > 0 && s <= NSTG) {
#pragma unroll
      for (int v = 0; v < NK; v++) stg[((s - 1) * NK + v) * 256 + threadIdx.x] = Kc[v];
      staged |= 1u << s;
    } else {
      store_block<OP>(vc, lane, s, Kc);
    }
  };
#pragma unroll
  for (int s = 1; s < NS; s++) {
    if (SPLIT < NS && s == (SPLIT > 2 ? SPLIT - 2 : 1)) {
#pragma unroll
      for (int k = SPLIT; k < NS; k++) gather(k);
      if constexpr (NSTG > 0) {
#pragma unroll
        for (int q = 1; q <= NSTG; q++)
          if ((staged >> q) & 1) {
            double K[NK];
#pragma unroll
            for (int v = 0; v < NK; v++) K[v] = stg[((q - 1) * NK + v) * 256 + threadIdx.x];
            store_block<OP>(vc, lane, q, K);
          }
      }
    }
    if (s < len) {
      const bool has_next = s + 1 < len;
      const int sn = (s + 1 < NS) ? s + 1 : 1;  // static slot of v_{s+1}
      const bool elem = (has_next || closed) && !((brk >> s) & 1);
      if constexpr (OP == OP_PB)
        if (has_next) pb_fifth(un[sn][0], a0[sn], a1[sn]);
      if (elem) {
        // v_t = v_{s+1}, or v_1 when a closed fan wraps
        const double2 pt = has_next ? pn[sn] : pn[1];
        double ut[NF];
#pragma unroll
        for (int f = 0; f < NF; f++) ut[f] = has_next ? un[sn][f] : un[1][f];
        const double at0 = has_next ? a0[sn] : a0[1], at1 = has_next ? a1[sn] : a1[1];
        Geo G;
        geometry(pi2.x, pi2.y, pn[s].x, pn[s].y, pt.x, pt.y, G);
        double Ct[NK];
#pragma unroll
        for (int v = 0; v < NK; v++) Ct[v] = 0;
        element<OP, JAC>(a, G, pi2.y, pn[s].y, pt.y, ui, un[s], ut, ai, a0[s], at0, aq, a1[s],
                         at1, R, D, P, Ct);
        if constexpr (JAC) {
          if (s == 1 && closed) {
#pragma unroll
            for (int v = 0; v < NK; v++) F[v] = P[v];
          } else {
            put(s, P);
          }
#pragma unroll
          for (int v = 0; v < NK; v++) P[v] = Ct[v];
        }
      } else if constexpr (JAC) {
        put(s, P);
#pragma unroll
        for (int v = 0; v < NK; v++) P[v] = 0;
      }
    }
  }
  if constexpr (JAC) {
    if (closed) {
#pragma unroll
      for (int v = 0; v < NK; v++) F[v] += P[v];
      store_block<OP>(vc, lane, 1, F);
    }
    store_block<OP>(vc, lane, 0, D);
  }
#pragma unroll
  for (int f = 0; f < NF; f++) {
    const size_t q = size_t(row) * NF + f;
    const double rv = R[f] + a.cvec[q];
    a.r[q] = a.dmask[q] != 0 ? 0.0 : rv;
  }
}

// cvec[row] -= M(x_old)[row]: PnpTOperator (tau * (c+ + c-) into the c+ row, Q2) or the
// DiffusionTOperator mass, for the implicit Euler residual M(u) - M(u_old) + dt R(u).
template <int OP>
__global__ __launch_bounds__(256) void k_mass_apply(DevLayout L, double tau, double pi, int cyl,
                                                    const double *__restrict__ xo,
                                                    double *__restrict__ cvec) {
  constexpr int NF = OpTraits<OP>::NF;
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= L.n_owned) return;
  const int chunk = row / kRows, lane = row % kRows;
  const int off = L.chunk_off[chunk];
  const uint64_t meta = L.rowmeta[row];
  const int len = int(meta & 63);
  const bool closed = (meta >> 6) & 1;
  const int *cix = L.colidx + off + lane;
  const double2 pi2 = reinterpret_cast<const double2 *>(L.xy)[row];
  double acc = 0;
  for (int s = 1; s < len; ++s) {
    const int t = (s + 1 < len) ? s + 1 : (closed ? 1 : -1);
    if (t < 0 || ((meta >> (8 + s)) & 1)) continue;
    const int b = cix[s * kRows], c = cix[t * kRows];
    const double2 pb2 = reinterpret_cast<const double2 *>(L.xy)[b];
    const double2 pc2 = reinterpret_cast<const double2 *>(L.xy)[c];
    Geo G;
    geometry(pi2.x, pi2.y, pb2.x, pb2.y, pc2.x, pc2.y, G);
    if constexpr (OP == OP_PNP_IE) {
      double Mii, Mib, Mic;
      mass_q2(G, cyl, pi, pi2.y, pb2.y, pc2.y, Mii, Mib, Mic);
      acc += tau * ((xo[size_t(row) * 3 + 1] + xo[size_t(row) * 3 + 2]) * Mii +
                    (xo[size_t(b) * 3 + 1] + xo[size_t(b) * 3 + 2]) * Mib +
                    (xo[size_t(c) * 3 + 1] + xo[size_t(c) * 3 + 2]) * Mic);
    } else {
      acc += xo[row] * G.adet * (1.0 / 12.0) + (xo[b] + xo[c]) * G.adet * (1.0 / 24.0);
    }
  }
  if constexpr (OP == OP_PNP_IE)
    cvec[size_t(row) * NF + 1] -= acc;
  else
    cvec[row] -= acc;
}

// Ion-current observable (calcIonFlux, src/ionFlux.hh:8-96): one thread per boundary segment
// handled by this rank; seg = {a, c, o, group} local vertices (segment a-c, opposite vertex o of
// its element).  out[2k] = ip contribution, out[2k+1] = im contribution (summed on the host in
// segment order, so the result does not depend on the launch).
__global__ __launch_bounds__(256) void k_ion_flux(int ns, const int4 *__restrict__ seg,
                                                  const double *__restrict__ xy,
                                                  const double *__restrict__ x, int cyl,
                                                  double pi, double *__restrict__ out) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ns) return;
  const int4 q = seg[k];
  const double2 pa = reinterpret_cast<const double2 *>(xy)[q.x];
  const double2 pc = reinterpret_cast<const double2 *>(xy)[q.y];
  const double2 po = reinterpret_cast<const double2 *>(xy)[q.z];
  Geo G;  // vertex order (a, c, o): gi = grad psi_a, gb = grad psi_c, gc = grad psi_o
  geometry(pa.x, pa.y, pc.x, pc.y, po.x, po.y, G);
  double gf[3][2];
#pragma unroll
  for (int f = 0; f < 3; f++) {
    const double ua = x[size_t(q.x) * 3 + f], uc = x[size_t(q.y) * 3 + f],
                 uo = x[size_t(q.z) * 3 + f];
    gf[f][0] = ua * G.gi0 + uc * G.gb0 + uo * G.gc0;
    gf[f][1] = ua * G.gi1 + uc * G.gb1 + uo * G.gc1;
  }
  const double cp = 0.5 * (x[size_t(q.x) * 3 + 1] + x[size_t(q.y) * 3 + 1]);
  const double cm = 0.5 * (x[size_t(q.x) * 3 + 2] + x[size_t(q.y) * 3 + 2]);
  const double tx = pc.x - pa.x, ty = pc.y - pa.y;
  const double len = sqrt(tx * tx + ty * ty);
  double factor = len;
  if (cyl) factor *= 2 * pi * (0.5 * (pa.y + pc.y));
  double nx = ty / len, ny = -tx / len;
  if (nx * (po.x - pa.x) + ny * (po.y - pa.y) > 0) {
    nx = -nx;
    ny = -ny;
  }
  const double gp0 = factor * gf[0][0] * cp, gp1 = factor * gf[0][1] * cp;
  out[2 * size_t(k)] = (-factor * gf[1][0] + gp0) * nx + (-factor * gf[1][1] + gp1) * ny;
  const double r = cm / cp;
  out[2 * size_t(k) + 1] =
      (-factor * gf[2][0] - gp0 * r) * nx + (-factor * gf[2][1] - gp1 * r) * ny;
}

}  // namespace

hipError_t launch_ion_flux(int ns, const int4 *seg, const double *xy, const double *x, int cyl,
                           double pi, double *out, hipStream_t s) {
  if (ns == 0) return hipSuccess;
  hipLaunchKernelGGL(k_ion_flux, dim3((ns + 255) / 256), dim3(256), 0, s, ns, seg, xy, x, cyl, pi,
                     out);
  return hipGetLastError();
}

// t0 / t1 (may be null): events the launch itself records at the kernel's start and end
// (hipExtLaunchKernelGGL), so the library's timers see the kernel's own duration -- an event pair
// recorded around the launch adds the dispatch of two markers (~5 us at config 3 in situ, against
// the kernel trace: 75.7 vs 69.6 us, gpurun_out r6final1 / profiles/r06/asm_regimes_config3.json)
hipError_t launch_assemble(const DevLayout &L, const AsmArgs &a, hipStream_t s, hipEvent_t t0,
                           hipEvent_t t1) {
  if (L.n_owned == 0) return hipSuccess;
  dim3 grid((L.n_owned + 255) / 256), block(256);
  // occupancy variant (A/B knob, PNP_ASM_WAVES=3|4): 4 waves/SIMD caps the fused PNP kernel at
  // 128 VGPRs (a few bytes of spill), 3 lets it keep ~134 without spilling
  static const int waves = [] {
    const char *e = getenv("PNP_ASM_WAVES");
    return (e && atoi(e) == 4) ? 4 : 3;
  }();
  // fans up to 11 neighbours keep their column indices in registers (all meshes seen: <= 8)
  static const bool fanr_ok = [] {  // A/B knob: PNP_ASM_FANR=0 forces the index-load path
    const char *e = getenv("PNP_ASM_FANR");
    return !(e && atoi(e) == 0);
  }();
  // A/B knob PNP_ASM_GA: 0 = the pipelined walk (k_assemble), 1 = gather-all at 3 waves/SIMD
  // (spills), 2 = gather-all at 2 waves, 3 / 4 / 5 = gather slots 1-4 / 1-5 / 1-2 first and the
  // rest two elements later at 3 waves; 4 is the default (profiles/r01/ab_asm_ga_*.log)
  static const int ga = [] {
    const char *e = getenv("PNP_ASM_GA");
    return e ? atoi(e) : 4;
  }();
  // column indices in registers: FANR - 1 >= the longest fan (max_slots - 1; 8 on all meshes
  // seen), 12 as the general case, 0 (index loads in the walk) beyond
  const int fanr = !fanr_ok ? 0 : (L.max_slots <= 9 ? 9 : (L.max_slots <= 12 ? 12 : 0));
  // LDS-staged neighbour data (A/B knob PNP_ASM_LDS=1), when the layout has the lists and a
  // workgroup's records fit 53 KiB (3 workgroups per CU at the kernel's 3 waves per SIMD).
  // Measured at config 3, with the row's own loads issued before the staging barrier: warm
  // 53.5 -> 60-63 us, cache-cold 87 -> 77.7 us (profiles/r02/ab_asm_lds2.log): the barrier costs
  // more than the halved gathers save while the inputs sit in the Infinity Cache, and less when
  // they come from HBM.  Off by default (the back-to-back assembly is the benchmark's number).
  // Well past the Infinity Cache every launch is cache-cold, so the Jacobian assembly takes the
  // LDS-staged walk there by default: its k-form write stream (~7 blocks per row on triangle
  // meshes) larger than twice the 256 MiB Infinity Cache.  Config 5 (828 MB): 344.8 -> 319.5 us
  // (profiles/r02/ab_cfg5_lds.log); config 2 (311 MB, still partly cache-resident back to back):
  // 79 -> 84 us, so the direct walk below 512 MiB (ab_cfg2_lds.log).  PNP_ASM_LDS=0 / 1 forces
  // either walk.
  static const int lds_env = [] {
    const char *e = getenv("PNP_ASM_LDS");
    return e ? (atoi(e) == 1 ? 1 : 0) : -1;
  }();
  // The Jacobian assembly inside Newton follows a BiCGSTAB solve, whose matrix and vector streams
  // have replaced the assembly's inputs in the caches: such a launch (a.cold, set by the context
  // after a solve) is cache-cold at any size and takes the LDS-staged walk too (config 3 in situ:
  // profiles/r03/ab_asm_cold_hint.log); PNP_ASM_COLD_HINT=0 ignores the hint (A/B)
  static const bool cold_hint = [] {
    const char *e = getenv("PNP_ASM_COLD_HINT");
    return !(e && e[0] == '0');
  }();
  const auto lds_walk = [&](int nk) {
    return lds_env == 1 ||
           (lds_env < 0 && (size_t(L.n_owned) * 7 * size_t(nk) * 8 > (size_t(512) << 20) ||
                            (cold_hint && a.cold)));
  };
#define PNP_ASM_CASE(OPK)                                                          \
  case OPK:                                                                        \
    if (!fanr && a.jac)                                                            \
      hipExtLaunchKernelGGL((k_assemble<OPK, 1, 3, 0>), grid, block, 0, s, t0, t1, 0, L, a);     \
    else if (!fanr)                                                                \
      hipExtLaunchKernelGGL((k_assemble<OPK, 0, 4, 0>), grid, block, 0, s, t0, t1, 0, L, a);     \
    else if (!a.jac && fanr == 9 && ga && lds_env == 1 && L.uown &&                 \
             size_t(L.unmax) * asm_lds_rec<OPK>() * 8 <= 53 * 1024)                    \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 0, 3, 9, 9, 0, 1>), grid, block,         \
                         size_t(L.unmax) * asm_lds_rec<OPK>() * 8, s, t0, t1, 0, L, a);             \
    else if (!a.jac && fanr == 9 && ga)                                            \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 0, 3, 9>), grid, block, 0, s, t0, t1, 0, L, a);  \
    else if (!a.jac)                                                               \
      hipExtLaunchKernelGGL((k_assemble<OPK, 0, 4, 12>), grid, block, 0, s, t0, t1, 0, L, a);    \
    else if (ga == 1 && fanr == 9)                                                 \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 1, 3, 9>), grid, block, 0, s, t0, t1, 0, L, a);  \
    else if (ga == 2 && fanr == 9)                                                 \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 1, 2, 9>), grid, block, 0, s, t0, t1, 0, L, a);  \
    else if (ga == 3 && fanr == 9)                                                 \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 1, 3, 9, 5>), grid, block, 0, s, t0, t1, 0, L, a); \
    else if (ga == 4 && fanr == 9 && lds_walk(OpTraits<OPK>::NK) && L.uown &&       \
             size_t(L.unmax) * asm_lds_rec<OPK>() * 8 <= 53 * 1024)                    \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 1, 3, 9, 6, 0, 1>), grid, block,         \
                         size_t(L.unmax) * asm_lds_rec<OPK>() * 8, s, t0, t1, 0, L, a);             \
    else if (ga == 4 && fanr == 9)                                                 \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 1, 3, 9, 6>), grid, block, 0, s, t0, t1, 0, L, a); \
    else if (ga == 5 && fanr == 9)                                                 \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 1, 3, 9, 3>), grid, block, 0, s, t0, t1, 0, L, a); \
    else if (ga == 6 && fanr == 9)                                                 \
      hipExtLaunchKernelGGL((k_assemble_ga<OPK, 1, 3, 9, 6, 1>), grid, block, 0, s, t0, t1, 0, L, a); \
    else if (fanr == 12)                                                           \
      hipExtLaunchKernelGGL((k_assemble<OPK, 1, 3, 12>), grid, block, 0, s, t0, t1, 0, L, a);    \
    else if (waves == 3)                                                           \
      hipExtLaunchKernelGGL((k_assemble<OPK, 1, 3, 9>), grid, block, 0, s, t0, t1, 0, L, a);     \
    else                                                                           \
      hipExtLaunchKernelGGL((k_assemble<OPK, 1, 4, 9>), grid, block, 0, s, t0, t1, 0, L, a);     \
    break;
  switch (a.kind) {
    PNP_ASM_CASE(OP_PNP)
    PNP_ASM_CASE(OP_PNP_IE)
    PNP_ASM_CASE(OP_PB)
    PNP_ASM_CASE(OP_DIFF)
    PNP_ASM_CASE(OP_DIFF_IE)
    PNP_ASM_CASE(OP_POISSON)
  default:
    return hipErrorInvalidValue;
  }
#undef PNP_ASM_CASE
  return hipGetLastError();
}

hipError_t launch_mass_apply(const DevLayout &L, int kind, double tau, double pi, int cylindrical,
                             const double *x_old, double *cvec, hipStream_t s) {
  if (L.n_owned == 0) return hipSuccess;
  dim3 grid((L.n_owned + 255) / 256), block(256);
  if (kind == OP_PNP_IE)
    hipLaunchKernelGGL(k_mass_apply<OP_PNP_IE>, grid, block, 0, s, L, tau, pi, cylindrical, x_old,
                       cvec);
  else if (kind == OP_DIFF_IE)
    hipLaunchKernelGGL(k_mass_apply<OP_DIFF_IE>, grid, block, 0, s, L, tau, pi, cylindrical,
                       x_old, cvec);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace pnp
