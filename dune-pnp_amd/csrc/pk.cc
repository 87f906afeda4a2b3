// Lagrange P_k spaces (k = 1, 2, 3) on the triangle mesh: node numbering, basis, node graph and
// the boundary data on the nodes.  See pk.h.
#include "pk.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <unordered_map>

namespace pnp {

namespace {

inline uint64_t ekey(int a, int b) {
  if (a > b) std::swap(a, b);
  return uint64_t(uint32_t(a)) << 32 | uint32_t(b);
}

// DUNE reference-triangle faces (0,1), (0,2), (1,2)
constexpr int kFace[3][2] = {{0, 1}, {0, 2}, {1, 2}};

// local nodes of degree k: barycentric lattice indices (a0, a1, a2), a0 + a1 + a2 = k, in the
// PkSpace::enode order (vertices, face points, interior points)
void local_lattice(int k, std::vector<std::array<int, 3>> &lat) {
  lat.clear();
  lat.push_back({k, 0, 0});
  lat.push_back({0, k, 0});
  lat.push_back({0, 0, k});
  for (int f = 0; f < 3; f++)
    for (int s = 1; s < k; s++) {  // s steps from the face's first vertex toward its second
      std::array<int, 3> a{0, 0, 0};
      a[kFace[f][0]] = k - s;
      a[kFace[f][1]] = s;
      lat.push_back(a);
    }
  for (int a1 = 1; a1 < k; a1++)
    for (int a2 = 1; a1 + a2 < k; a2++) lat.push_back({k - a1 - a2, a1, a2});
}

}  // namespace

void pk_basis(int k, double xi, double eta, double *phi, double *dphi) {
  std::vector<std::array<int, 3>> lat;
  local_lattice(k, lat);
  const double lam[3] = {1.0 - xi - eta, xi, eta};
  // d lambda_i / d (xi, eta)
  const double dl[3][2] = {{-1.0, -1.0}, {1.0, 0.0}, {0.0, 1.0}};
  for (size_t n = 0; n < lat.size(); n++) {
    // P_a(l) = prod_{m<a} (k l - m) / (m + 1) and its derivative in l
    double P[3], dP[3];
    for (int i = 0; i < 3; i++) {
      const int a = lat[n][i];
      double v = 1.0, d = 0.0;
      for (int m = 0; m < a; m++) {
        const double f = (k * lam[i] - m) / (m + 1);
        d = d * f + v * (double(k) / (m + 1));
        v *= f;
      }
      P[i] = v;
      dP[i] = d;
    }
    if (phi) phi[n] = P[0] * P[1] * P[2];
    if (dphi) {
      const double g0 = dP[0] * P[1] * P[2], g1 = P[0] * dP[1] * P[2], g2 = P[0] * P[1] * dP[2];
      dphi[2 * n] = g0 * dl[0][0] + g1 * dl[1][0] + g2 * dl[2][0];
      dphi[2 * n + 1] = g0 * dl[0][1] + g1 * dl[1][1] + g2 * dl[2][1];
    }
  }
}

bool build_pk_space(const Mesh &m, int k, PkSpace &S, std::string &err) {
  if (k < 1 || k > 3) {
    err = "polynomial degree must be 1, 2 or 3 (PDEGREE, src/instationary_pnp_from_pb_md.hh:26-28)";
    return false;
  }
  S = PkSpace();
  S.k = k;
  S.nl = (k + 1) * (k + 2) / 2;
  S.nv = m.nv;
  std::vector<std::array<int, 3>> lat;
  local_lattice(k, lat);
  S.lref.resize(2 * size_t(S.nl));
  for (int n = 0; n < S.nl; n++) {
    S.lref[2 * n] = double(lat[n][1]) / k;
    S.lref[2 * n + 1] = double(lat[n][2]) / k;
  }
  // edges in order of first appearance (triangle order, faces (0,1), (0,2), (1,2))
  std::unordered_map<uint64_t, int> edge;
  edge.reserve(size_t(m.nt) * 2);
  std::vector<int> elo, ehi;  // global vertices of edge e, elo < ehi
  for (int e = 0; e < m.nt; e++)
    for (int f = 0; f < 3; f++) {
      const int a = m.tri[3 * size_t(e) + kFace[f][0]], b = m.tri[3 * size_t(e) + kFace[f][1]];
      if (edge.emplace(ekey(a, b), int(elo.size())).second) {
        elo.push_back(std::min(a, b));
        ehi.push_back(std::max(a, b));
      }
    }
  S.nedge = int(elo.size());
  const int ni = (k - 1) * (k - 2) / 2;
  const long long nn = (long long)m.nv + (long long)S.nedge * (k - 1) + (long long)m.nt * ni;
  if (nn > (1LL << 30)) {
    err = "P_k space too large";
    return false;
  }
  S.nn = int(nn);
  S.xy.resize(2 * size_t(S.nn));
  std::copy(m.xy.begin(), m.xy.end(), S.xy.begin());
  for (int e = 0; e < S.nedge; e++)
    for (int s = 1; s < k; s++) {
      const size_t n = size_t(m.nv) + size_t(e) * (k - 1) + (s - 1);
      const double t = double(s) / k;
      for (int d = 0; d < 2; d++) {
        const double x0 = m.xy[2 * size_t(elo[e]) + d], x1 = m.xy[2 * size_t(ehi[e]) + d];
        S.xy[2 * n + d] = x0 + t * (x1 - x0);
      }
    }
  S.enode.resize(size_t(m.nt) * S.nl);
  for (int e = 0; e < m.nt; e++) {
    const int *t = &m.tri[3 * size_t(e)];
    int *en = &S.enode[size_t(e) * S.nl];
    int q = 0;
    for (int i = 0; i < 3; i++) en[q++] = t[i];
    for (int f = 0; f < 3; f++) {
      const int a = t[kFace[f][0]], b = t[kFace[f][1]];
      const int id = edge.at(ekey(a, b));
      for (int s = 1; s < k; s++) {  // s steps from a toward b = (k - s) steps from b
        const int from_lo = a < b ? s : k - s;
        en[q++] = m.nv + id * (k - 1) + (from_lo - 1);
      }
    }
    for (int i = 0; i < ni; i++) {
      const size_t n = size_t(m.nv) + size_t(S.nedge) * (k - 1) + size_t(e) * ni + i;
      en[q++] = int(n);
      // interior lattice point (local node q-1): barycentric combination of the vertices
      const auto &L = lat[q - 1];
      for (int d = 0; d < 2; d++)
        S.xy[2 * n + d] = (L[0] * m.xy[2 * size_t(t[0]) + d] + L[1] * m.xy[2 * size_t(t[1]) + d] +
                           L[2] * m.xy[2 * size_t(t[2]) + d]) / k;
    }
  }
  // boundary segments: nodes from bseg[0] to bseg[1], and the element face they lie on
  S.bnode.resize(size_t(m.nb) * (k + 1));
  S.bface.assign(m.nb, -1);
  for (int s = 0; s < m.nb; s++) {
    const int a = m.bseg[2 * size_t(s)], b = m.bseg[2 * size_t(s) + 1];
    auto it = edge.find(ekey(a, b));
    if (it == edge.end()) {
      err = "boundary segment " + std::to_string(s) + " is not an element edge";
      return false;
    }
    int *bn = &S.bnode[size_t(s) * (k + 1)];
    bn[0] = a;
    for (int q = 1; q < k; q++) bn[q] = m.nv + it->second * (k - 1) + ((a < b ? q : k - q) - 1);
    bn[k] = b;
  }
  {
    std::unordered_map<uint64_t, int> seg;
    seg.reserve(size_t(m.nb) * 2);
    for (int s = 0; s < m.nb; s++) seg[ekey(m.bseg[2 * size_t(s)], m.bseg[2 * size_t(s) + 1])] = s;
    for (int e = 0; e < m.nt; e++)
      for (int f = 0; f < 3; f++) {
        auto it = seg.find(ekey(m.tri[3 * size_t(e) + kFace[f][0]], m.tri[3 * size_t(e) + kFace[f][1]]));
        if (it != seg.end() && S.bface[it->second] < 0) S.bface[it->second] = 3 * e + f;
      }
  }
  return true;
}

bool pk_adjacency(const Mesh &m, const PkSpace &S, Fans &f, std::string &err) {
  const int nn = S.nn, nl = S.nl;
  // node -> incident elements (CSR)
  std::vector<int> ip(nn + 1, 0), ie;
  for (size_t q = 0; q < S.enode.size(); q++) ip[S.enode[q] + 1]++;
  for (int n = 0; n < nn; n++) ip[n + 1] += ip[n];
  ie.resize(ip[nn]);
  {
    std::vector<int> at(ip.begin(), ip.end() - 1);
    for (int e = 0; e < m.nt; e++)
      for (int a = 0; a < nl; a++) ie[at[S.enode[size_t(e) * nl + a]]++] = e;
  }
  f = Fans();
  f.ptr.assign(nn + 1, 0);
  f.meta.assign(nn, 0);
  std::vector<int> mark(nn, -1), nb;
  for (int n = 0; n < nn; n++) {
    nb.clear();
    mark[n] = n;
    for (int q = ip[n]; q < ip[n + 1]; q++)
      for (int a = 0; a < nl; a++) {
        const int u = S.enode[size_t(ie[q]) * nl + a];
        if (mark[u] != n) {
          mark[u] = n;
          nb.push_back(u);
        }
      }
    if (ip[n] == ip[n + 1]) {
      err = "node " + std::to_string(n) + " belongs to no element";
      return false;
    }
    std::sort(nb.begin(), nb.end());
    const int len = 1 + int(nb.size());
    if (len > 63) {
      err = "P" + std::to_string(S.k) + " node " + std::to_string(n) + " couples to " +
            std::to_string(len - 1) + " nodes; rows hold at most 62 neighbours";
      return false;
    }
    f.meta[n] = uint64_t(len);
    f.max_slots = std::max(f.max_slots, len);
    f.nbr.insert(f.nbr.end(), nb.begin(), nb.end());
    f.ptr[n + 1] = int(f.nbr.size());
  }
  return true;
}

Mesh pk_node_mesh(const PkSpace &S) {
  Mesh nm;
  nm.nv = S.nn;
  nm.xy = S.xy;
  return nm;
}

void pk_dirichlet_mask(const Mesh &m, const PkSpace &S, const Params &p, int nf, int field0,
                       std::vector<uint8_t> &mask) {
  mask.assign(size_t(S.nn) * nf, 0);
  const int k = S.k;
  for (int s = 0; s < m.nb; s++) {
    const Surface &Sf = p.surf[m.bgroup[s]];
    for (int f = 0; f < nf; f++)
      if (Sf.btype(field0 + f) == 0)
        for (int q = 0; q <= k; q++) mask[size_t(S.bnode[size_t(s) * (k + 1) + q]) * nf + f] = 1;
  }
}

void pk_neumann_load(const Mesh &m, const PkSpace &S, const Params &p, int nf, int field0,
                     std::vector<double> &load) {
  load.assign(size_t(S.nn) * nf, 0.0);
  const int k = S.k;
  const double t[2] = {0.5 - 0.5 / std::sqrt(3.0), 0.5 + 0.5 / std::sqrt(3.0)};
  // 1-D Lagrange basis on the face's k+1 equispaced nodes (the trace of the P_k basis)
  double psi[2][4];
  for (int q = 0; q < 2; q++)
    for (int i = 0; i <= k; i++) {
      double v = 1.0;
      for (int j = 0; j <= k; j++)
        if (j != i) v *= (t[q] - double(j) / k) / (double(i - j) / k);
      psi[q][i] = v;
    }
  for (int s = 0; s < m.nb; s++) {
    const Surface &Sf = p.surf[m.bgroup[s]];
    const int a = m.bseg[2 * size_t(s)], b = m.bseg[2 * size_t(s) + 1];
    const double dx = m.xy[2 * size_t(b)] - m.xy[2 * size_t(a)];
    const double dy = m.xy[2 * size_t(b) + 1] - m.xy[2 * size_t(a) + 1];
    const double len = std::sqrt(dx * dx + dy * dy);
    for (int q = 0; q < 2; q++) {
      double factor = 0.5 * len;
      if (p.cylindrical) factor *= (m.xy[2 * size_t(a) + 1] + t[q] * dy) * 2 * p.pi;
      for (int f = 0; f < nf; f++) {
        if (Sf.btype(field0 + f) == 0) continue;
        const double j = Sf.flux(field0 + f);
        for (int i = 0; i <= k; i++)
          load[size_t(S.bnode[size_t(s) * (k + 1) + i]) * nf + f] += j * psi[q][i] * factor;
      }
    }
  }
}

void pk_initial_state(const Mesh &m, const PkSpace &S, const Params &p, const double *phi_pb,
                      double *x0) {
  initial_state_at(m, p, S.nl, S.enode.data(), S.xy.data(), S.nn, phi_pb, x0);
}

}  // namespace pnp
