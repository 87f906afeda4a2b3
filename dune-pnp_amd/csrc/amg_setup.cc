// Host side of the aggregation AMG (PNP_PREC_AMG): the level hierarchy as patterns and
// contributor lists.  Values never pass through the host: amg.hip sums them on the device after
// every assembly.
//
// The reference's CG_AMG_SSOR (src/instationary_pnp_from_pb_md.hh:207-210) builds dune-istl's
// Amg::AMG (aggregation coarsening, piecewise-constant prolongation, SSOR smoother, V-cycle).
// dune-istl is not in the image, so its exact aggregation heuristics are not
// restated; this is the same class of method: greedy aggregation over the matrix graph (a root
// whose neighbours are all free takes them; the rest join a neighbouring aggregate of that
// first pass; isolated leftovers stay singletons), Galerkin coarse operators A_c = P^T A P.
#include <algorithm>
#include <numeric>

#include "amg.h"

namespace pnp {

int amg_aggregate(int n, const std::vector<int> &ap, const std::vector<int> &aj,
                  std::vector<int> &agg) {
  agg.assign(n, -1);
  int na = 0;
  for (int i = 0; i < n; i++) {  // pass 1: roots with all neighbours free
    if (agg[i] >= 0) continue;
    bool free = true;
    for (int q = ap[i]; q < ap[i + 1] && free; q++) free = agg[aj[q]] < 0;
    if (!free) continue;
    agg[i] = na;
    for (int q = ap[i]; q < ap[i + 1]; q++) agg[aj[q]] = na;
    na++;
  }
  std::vector<int> join(n, -1);  // pass 2: join the first pass-1 aggregate among the neighbours
  for (int i = 0; i < n; i++) {
    if (agg[i] >= 0) continue;
    for (int q = ap[i]; q < ap[i + 1]; q++)
      if (agg[aj[q]] >= 0) {
        join[i] = agg[aj[q]];
        break;
      }
  }
  for (int i = 0; i < n; i++)
    if (agg[i] < 0 && join[i] >= 0) agg[i] = join[i];
  for (int i = 0; i < n; i++)  // pass 3: singletons
    if (agg[i] < 0) agg[i] = na++;
  return na;
}

namespace {

// coarse pattern and contributors from the fine blocks (row, col, source code) grouped by coarse
// row: entries (agg[col], code) of all members of aggregate J, sorted, one block per agg[col]
void coarse_level(int na, const std::vector<int> &agg,
                  const std::vector<std::vector<std::pair<int, int>>> &byrow, AmgLevelHost &C) {
  C.nb = na;
  C.agg = agg;
  C.mptr.assign(na + 1, 0);
  for (int a : agg) C.mptr[a + 1]++;
  for (int J = 0; J < na; J++) C.mptr[J + 1] += C.mptr[J];
  C.mem.assign(agg.size(), 0);
  std::vector<int> fill(C.mptr.begin(), C.mptr.end() - 1);
  for (int i = 0; i < int(agg.size()); i++) C.mem[fill[agg[i]]++] = i;
  C.rp.assign(na + 1, 0);
  C.col.clear();
  C.dpos.assign(na, -1);
  C.cptr.assign(1, 0);
  C.csrc.clear();
  std::vector<std::pair<int, int>> ent;
  for (int J = 0; J < na; J++) {
    ent.clear();
    for (int m = C.mptr[J]; m < C.mptr[J + 1]; m++) {
      const int i = C.mem[m];
      for (const auto &e : byrow[i]) ent.push_back({agg[e.first], e.second});
    }
    std::sort(ent.begin(), ent.end());
    for (size_t k = 0; k < ent.size(); k++) {
      if (k == 0 || ent[k].first != ent[k - 1].first) {
        if (k > 0) C.cptr.push_back((long long)C.csrc.size());
        if (ent[k].first == J) C.dpos[J] = int(C.col.size());
        C.col.push_back(ent[k].first);
      }
      C.csrc.push_back(ent[k].second);
    }
    if (!ent.empty()) C.cptr.push_back((long long)C.csrc.size());
    C.rp[J + 1] = int(C.col.size());
  }
}

}  // namespace

bool amg_build(const LocalLayout &L, int coarse_target, int max_levels,
               std::vector<AmgLevelHost> &levels, std::string &err) {
  levels.clear();
  const int n = L.n_owned;
  if (n == 0) return true;
  coarse_target = std::max(1, std::min(coarse_target, kAmgMaxCoarse));
  max_levels = std::max(2, std::min(max_levels, kAmgMaxLevels));
  // level 0: the SELL rows, owned columns only
  std::vector<std::vector<std::pair<int, int>>> byrow(n);  // (col, code)
  std::vector<int> ap(n + 1, 0), aj;
  for (int i = 0; i < n; i++) {
    const int ch = i / kChunk, ln = i % kChunk, len = meta_len(L.rowmeta[i]);
    for (int s = 0; s < len; s++) {
      const int j = L.colidx[size_t(L.chunk_off[ch]) + size_t(kChunk) * s + ln];
      if (j >= n) continue;  // ghost column: the hierarchy is rank-local
      byrow[i].push_back({j, i << 6 | s});
      if (j != i) aj.push_back(j);
    }
    ap[i + 1] = int(aj.size());
  }
  int nrows = n;
  while (int(levels.size()) + 1 < max_levels) {
    std::vector<int> agg;
    const int na = amg_aggregate(nrows, ap, aj, agg);
    if (na >= nrows && !levels.empty()) break;  // no coarsening possible
    AmgLevelHost C;
    coarse_level(na, agg, byrow, C);
    for (int J = 0; J < na; J++)
      if (C.dpos[J] < 0) {
        err = "AMG: coarse row without a diagonal block";
        return false;
      }
    levels.push_back(std::move(C));
    const AmgLevelHost &B = levels.back();
    nrows = B.nb;
    if (nrows <= coarse_target) break;
    // next level's graph and block sources (block index q of this level)
    byrow.assign(nrows, {});
    ap.assign(nrows + 1, 0);
    aj.clear();
    for (int I = 0; I < nrows; I++) {
      for (int q = B.rp[I]; q < B.rp[I + 1]; q++) {
        byrow[I].push_back({B.col[q], q});
        if (B.col[q] != I) aj.push_back(B.col[q]);
      }
      ap[I + 1] = int(aj.size());
    }
  }
  if (levels.back().nb > kAmgMaxDense) {
    err = "AMG: coarsest level has " + std::to_string(levels.back().nb) +
          " blocks (graph does not coarsen; max levels reached?)";
    return false;
  }
  return true;
}

}  // namespace pnp
