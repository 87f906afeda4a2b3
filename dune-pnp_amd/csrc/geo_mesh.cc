// .geo reader and 2-D triangle mesher.
//
// The reference meshes test/pore_without_dna/pore_without_dna.geo with gmsh before the run
// (test/pore_without_dna/pore.cfg:21 names the .msh; none ships, and the image has no gmsh).
// This is the native replacement for that preprocessing step, for the .geo subset the
// reference's geometries use:
//   name = expr;                         (numbers, + - * /, parentheses, earlier names)
//   Point(id) = {x, y, z[, lc]};
//   Line(id) = {p, q};   Circle(id) = {start, centre, end};   (arc < pi, as gmsh)
//   Line Loop(id) = {signed curve ids};  Curve Loop(...) likewise
//   Plane Surface(id) = {outer loop[, holes]};
//   Physical Line(g) = {curve ids};      Physical Curve(...) likewise; other Physical ignored
// Mesher (what gmsh's 1-D + 2-D Delaunay steps do, re-derived):
//   1. every curve is split so that the segment count integrates 1/lc, lc interpolated linearly
//      between the curve's end points (gmsh's size-from-points);
//   2. the size inside comes from the boundary: barycentric interpolation of the boundary node
//      sizes over a triangulation of the boundary nodes (gmsh's "extend from boundary");
//   3. interior nodes: a jittered hexagonal candidate lattice thinned greedily to a minimum
//      spacing of 0.8 h(p) (Poisson-disk), smallest sizes first;
//   4. Bowyer-Watson Delaunay of all nodes, boundary recovery by splitting missing boundary
//      segments (on the curve), removal of triangles whose centroid is outside the domain;
//   5. three rounds of Laplacian smoothing of the interior nodes, each re-triangulated.
// The output numbers vertices in order of first use by a triangle, so writing the mesh as gmsh
// v2 and reading it back (read_gmsh) gives the same mesh.  Boundary segments carry the
// physical group of their curve, in loop order.
#include <algorithm>
#include <array>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <map>
#include <sstream>
#include <unordered_map>
#include <unordered_set>

#include "mesh.h"

namespace pnp {

// ---------------------------------------------------------------------------------------------
// .geo subset
// ---------------------------------------------------------------------------------------------
namespace {

struct Lexer {
  const std::string &s;
  size_t i = 0;
  explicit Lexer(const std::string &str) : s(str) {}
  void ws() {
    while (i < s.size() && std::isspace((unsigned char)s[i])) i++;
  }
  bool eat(char c) {
    ws();
    if (i < s.size() && s[i] == c) {
      i++;
      return true;
    }
    return false;
  }
  bool at_end() {
    ws();
    return i >= s.size();
  }
  std::string ident() {
    ws();
    size_t b = i;
    while (i < s.size() && (std::isalnum((unsigned char)s[i]) || s[i] == '_')) i++;
    return s.substr(b, i - b);
  }
};

struct ExprParser {
  Lexer &L;
  const std::map<std::string, double> &vars;
  std::string &err;
  double primary() {
    if (L.eat('(')) {
      double v = sum();
      if (!L.eat(')')) err = "expected ')'";
      return v;
    }
    if (L.eat('-')) return -primary();
    if (L.eat('+')) return primary();
    L.ws();
    if (L.i < L.s.size() && (std::isdigit((unsigned char)L.s[L.i]) || L.s[L.i] == '.')) {
      const char *b = L.s.c_str() + L.i;
      char *e = nullptr;
      double v = std::strtod(b, &e);
      L.i += size_t(e - b);
      return v;
    }
    std::string id = L.ident();
    if (id.empty()) {
      err = "expected a number or a name";
      return 0;
    }
    if (id == "Pi") return M_PI;
    auto it = vars.find(id);
    if (it == vars.end()) {
      err = "unknown name '" + id + "'";
      return 0;
    }
    return it->second;
  }
  double product() {
    double v = primary();
    for (;;) {
      if (L.eat('*'))
        v *= primary();
      else if (L.eat('/'))
        v /= primary();
      else
        return v;
    }
  }
  double sum() {
    double v = product();
    for (;;) {
      if (L.eat('+'))
        v += product();
      else if (L.eat('-'))
        v -= product();
      else
        return v;
    }
  }
};

std::string strip_comments(const std::string &t) {
  std::string o;
  for (size_t i = 0; i < t.size(); i++) {
    if (t[i] == '/' && i + 1 < t.size() && t[i + 1] == '/') {
      while (i < t.size() && t[i] != '\n') i++;
      o += '\n';
    } else if (t[i] == '/' && i + 1 < t.size() && t[i + 1] == '*') {
      i += 2;
      while (i + 1 < t.size() && !(t[i] == '*' && t[i + 1] == '/')) i++;
      i++;
    } else {
      o += t[i];
    }
  }
  return o;
}

}  // namespace

bool read_geo(const std::string &path, GeoModel &g, std::string &err) {
  std::ifstream in(path);
  if (!in) {
    err = "cannot open geometry file '" + path + "'";
    return false;
  }
  std::stringstream ss;
  ss << in.rdbuf();
  const std::string text = strip_comments(ss.str());
  g = GeoModel();
  std::map<std::string, double> vars;
  size_t p = 0;
  int stmt_no = 0;
  while (p < text.size()) {
    size_t e = text.find(';', p);
    if (e == std::string::npos) e = text.size();
    std::string st = text.substr(p, e - p);
    p = e + 1;
    stmt_no++;
    Lexer L(st);
    if (L.at_end()) continue;
    auto fail = [&](const std::string &m) {
      err = path + ": statement " + std::to_string(stmt_no) + ": " + m;
      return false;
    };
    ExprParser X{L, vars, err};
    std::string w1 = L.ident();
    if (w1.empty()) return fail("expected a keyword or a name");
    std::string kw = w1;
    if (w1 == "Line" || w1 == "Curve" || w1 == "Plane" || w1 == "Physical") {
      size_t save = L.i;
      std::string w2 = L.ident();
      if (w2 == "Loop" || w2 == "Surface" || w2 == "Line" || w2 == "Curve" || w2 == "Point")
        kw = w1 + " " + w2;
      else
        L.i = save;
    }
    if (!L.eat('(')) {  // assignment
      if (!L.eat('=')) return fail("expected '=' after '" + w1 + "'");
      double v = X.sum();
      if (!err.empty()) return fail(err);
      if (!L.at_end()) return fail("trailing characters");
      vars[w1] = v;
      continue;
    }
    double idv = X.sum();
    if (!err.empty()) return fail(err);
    if (!L.eat(')') || !L.eat('=') || !L.eat('{')) return fail("expected ') = {'");
    std::vector<double> list;
    if (!L.eat('}')) {
      for (;;) {
        list.push_back(X.sum());
        if (!err.empty()) return fail(err);
        if (L.eat('}')) break;
        if (!L.eat(',')) return fail("expected ',' or '}'");
      }
    }
    if (!L.at_end()) return fail("trailing characters");
    const int id = int(std::lround(idv));
    auto ids = [&] {
      std::vector<int> v;
      for (double d : list) v.push_back(int(std::lround(d)));
      return v;
    };
    if (kw == "Point") {
      if (list.size() != 3 && list.size() != 4) return fail("Point needs 3 or 4 values");
      g.pts[id] = {list[0], list[1], list.size() == 4 ? list[3] : 0.0};
    } else if (kw == "Line" || kw == "Circle") {
      auto v = ids();
      if (kw == "Line" && v.size() != 2) return fail("Line needs 2 points");
      if (kw == "Circle" && v.size() != 3) return fail("Circle needs start, centre, end");
      for (int q : v)
        if (!g.pts.count(q)) return fail("unknown point " + std::to_string(q));
      GeoModel::Curve c;
      c.circle = kw == "Circle";
      c.a = v[0];
      c.b = v.back();
      c.c = c.circle ? v[1] : -1;
      g.curves[id] = c;
    } else if (kw == "Line Loop" || kw == "Curve Loop") {
      auto v = ids();
      for (int q : v)
        if (!g.curves.count(std::abs(q))) return fail("unknown curve " + std::to_string(q));
      g.loops[id] = v;
    } else if (kw == "Plane Surface") {
      auto v = ids();
      for (int q : v)
        if (!g.loops.count(q)) return fail("unknown loop " + std::to_string(q));
      g.surfaces[id] = v;
    } else if (kw == "Physical Line" || kw == "Physical Curve") {
      for (int q : ids()) {
        if (!g.curves.count(std::abs(q))) return fail("unknown curve " + std::to_string(q));
        g.curve_group[std::abs(q)] = id;
      }
    } else if (kw == "Physical Surface" || kw == "Physical Point") {
      // the reference reads only boundary groups (src/pnp_solver_main.cc:89-90)
    } else {
      return fail("unsupported statement '" + kw + "'");
    }
  }
  if (g.surfaces.empty()) {
    err = path + ": no Plane Surface";
    return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// mesher
// ---------------------------------------------------------------------------------------------
namespace {

struct P2 {
  double x, y;
};

struct BNode {       // boundary node
  P2 p;
  double h;          // target size here
};

struct BSeg {        // boundary segment: nodes (a, b), curve and its parameter interval
  int a, b, curve, group;
  bool rev;          // traversed against the curve's direction
  double t0, t1;     // curve parameters of a and b
};

struct CurveGeom {
  bool circle;
  P2 a, b, c;
  double r = 0, th0 = 0, dth = 0, len = 0;
  double ha, hb;
  P2 at(double t) const {
    if (!circle) return {a.x + (b.x - a.x) * t, a.y + (b.y - a.y) * t};
    double th = th0 + dth * t;
    return {c.x + r * std::cos(th), c.y + r * std::sin(th)};
  }
  double h_at(double t) const { return ha + (hb - ha) * t; }
};

// Delaunay triangulation (Bowyer-Watson) of points q (connectivity only), super-triangle
// removed.  O(n^2) cavity search: the mesher makes coarse base meshes (refine() does the rest).
std::vector<std::array<int, 3>> delaunay(const std::vector<P2> &q) {
  const int n = int(q.size());
  double mnx = 1e300, mny = 1e300, mxx = -1e300, mxy = -1e300;
  for (auto &p : q) {
    mnx = std::min(mnx, p.x);
    mny = std::min(mny, p.y);
    mxx = std::max(mxx, p.x);
    mxy = std::max(mxy, p.y);
  }
  const double D = std::max(mxx - mnx, mxy - mny), cx = 0.5 * (mnx + mxx), cy = 0.5 * (mny + mxy);
  std::vector<P2> pt = q;
  pt.push_back({cx - 40 * D, cy - 30 * D});
  pt.push_back({cx + 40 * D, cy - 30 * D});
  pt.push_back({cx, cy + 40 * D});
  struct T {
    int v[3];
    double ccx, ccy, r2;
    bool alive;
  };
  std::vector<T> tris;
  auto make = [&](int a, int b, int c) {
    const P2 &A = pt[a], &B = pt[b], &C = pt[c];
    double o = (B.x - A.x) * (C.y - A.y) - (B.y - A.y) * (C.x - A.x);
    if (o < 0) std::swap(b, c);
    const P2 &B2 = pt[b], &C2 = pt[c];
    double bx = B2.x - A.x, by = B2.y - A.y, qx = C2.x - A.x, qy = C2.y - A.y;
    double d = 2 * (bx * qy - by * qx);
    double ux = (qy * (bx * bx + by * by) - by * (qx * qx + qy * qy)) / d;
    double uy = (bx * (qx * qx + qy * qy) - qx * (bx * bx + by * by)) / d;
    tris.push_back({{a, b, c}, A.x + ux, A.y + uy, ux * ux + uy * uy, true});
  };
  make(n, n + 1, n + 2);
  std::vector<int> bad;
  std::vector<std::pair<int, int>> edges;
  for (int i = 0; i < n; i++) {
    const P2 &p = pt[i];
    bad.clear();
    for (int t = 0; t < int(tris.size()); t++) {
      if (!tris[t].alive) continue;
      double dx = p.x - tris[t].ccx, dy = p.y - tris[t].ccy;
      if (dx * dx + dy * dy < tris[t].r2) bad.push_back(t);
    }
    edges.clear();
    for (int t : bad) {
      tris[t].alive = false;
      for (int k = 0; k < 3; k++) edges.emplace_back(tris[t].v[k], tris[t].v[(k + 1) % 3]);
    }
    // cavity boundary: edges not shared by two bad triangles
    std::map<std::pair<int, int>, int> cnt;
    for (auto &e : edges) cnt[{std::min(e.first, e.second), std::max(e.first, e.second)}]++;
    for (auto &e : edges)
      if (cnt[{std::min(e.first, e.second), std::max(e.first, e.second)}] == 1)
        make(e.first, e.second, i);
    if (tris.size() > 4 * size_t(n) + 64) {  // compact
      std::vector<T> keep;
      for (auto &t : tris)
        if (t.alive) keep.push_back(t);
      tris.swap(keep);
    }
  }
  std::vector<std::array<int, 3>> out;
  for (auto &t : tris)
    if (t.alive && t.v[0] < n && t.v[1] < n && t.v[2] < n) out.push_back({t.v[0], t.v[1], t.v[2]});
  return out;
}

bool inside(const std::vector<std::vector<P2>> &loops, P2 p) {
  bool in = false;
  for (auto &L : loops)
    for (size_t i = 0, j = L.size() - 1; i < L.size(); j = i++) {
      const P2 &a = L[i], &b = L[j];
      if ((a.y > p.y) != (b.y > p.y) && p.x < (b.x - a.x) * (p.y - a.y) / (b.y - a.y) + a.x) in = !in;
    }
  return in;
}

double seg_dist(P2 p, P2 a, P2 b) {
  double vx = b.x - a.x, vy = b.y - a.y, wx = p.x - a.x, wy = p.y - a.y;
  double l2 = vx * vx + vy * vy, t = l2 > 0 ? (wx * vx + wy * vy) / l2 : 0;
  t = std::min(1.0, std::max(0.0, t));
  double dx = wx - t * vx, dy = wy - t * vy;
  return std::sqrt(dx * dx + dy * dy);
}

double tri_area(P2 a, P2 b, P2 c) { return 0.5 * ((b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x)); }

}  // namespace

bool mesh_geo(const GeoModel &g, double size_scale, Mesh &m, std::string &err) {
  if (!(size_scale > 0)) {
    err = "size scale must be positive";
    return false;
  }
  if (g.surfaces.size() != 1) {
    err = "one Plane Surface expected";
    return false;
  }
  // ---- curves --------------------------------------------------------------------------------
  double lc_max = 0;
  for (auto &kv : g.pts) lc_max = std::max(lc_max, kv.second[2]);
  std::map<int, CurveGeom> cg;
  for (auto &kv : g.curves) {
    const auto &c = kv.second;
    CurveGeom G;
    G.circle = c.circle;
    auto P = [&](int id) { return P2{g.pts.at(id)[0], g.pts.at(id)[1]}; };
    auto H = [&](int id) {
      double h = g.pts.at(id)[2];
      return (h > 0 ? h : lc_max) * size_scale;
    };
    G.a = P(c.a);
    G.b = P(c.b);
    G.ha = H(c.a);
    G.hb = H(c.b);
    if (G.circle) {
      G.c = P(c.c);
      G.r = std::hypot(G.a.x - G.c.x, G.a.y - G.c.y);
      double rb = std::hypot(G.b.x - G.c.x, G.b.y - G.c.y);
      if (std::fabs(rb - G.r) > 1e-9 * std::max(1.0, G.r)) {
        err = "circle " + std::to_string(kv.first) + ": end points at different radii";
        return false;
      }
      G.th0 = std::atan2(G.a.y - G.c.y, G.a.x - G.c.x);
      double th1 = std::atan2(G.b.y - G.c.y, G.b.x - G.c.x);
      G.dth = th1 - G.th0;
      while (G.dth > M_PI) G.dth -= 2 * M_PI;
      while (G.dth < -M_PI) G.dth += 2 * M_PI;
      G.len = G.r * std::fabs(G.dth);
    } else {
      G.len = std::hypot(G.b.x - G.a.x, G.b.y - G.a.y);
    }
    if (!(G.len > 0) || !(G.ha > 0)) {
      err = "curve " + std::to_string(kv.first) + " is degenerate or has no mesh size";
      return false;
    }
    cg[kv.first] = G;
  }
  // parameters of the nodes on a curve: segment count integrates 1/h
  auto split = [&](const CurveGeom &G) {
    const double L = G.len, ha = G.ha, hb = G.hb;
    const bool same = std::fabs(hb - ha) < 1e-12 * ha;
    const double I = same ? L / ha : L / (hb - ha) * std::log(hb / ha);
    const int N = std::max(1, int(std::lround(I)));
    std::vector<double> t(N + 1);
    for (int k = 0; k <= N; k++) {
      const double Ik = I * k / N;
      t[k] = same ? Ik * ha / L : (ha * std::exp((hb - ha) / L * Ik) - ha) / (hb - ha);
    }
    t[0] = 0;
    t[N] = 1;
    return t;
  };
  // ---- boundary nodes and segments, loop by loop ----------------------------------------------
  std::vector<BNode> bn;
  std::vector<BSeg> bs;
  std::vector<int> loop_first;  // first segment of each loop
  const auto &surf = g.surfaces.begin()->second;
  for (int lid : surf) {
    const auto &loop = g.loops.at(lid);
    const int first_node = int(bn.size());
    loop_first.push_back(int(bs.size()));
    P2 start{0, 0}, prev_end{0, 0};
    for (size_t k = 0; k < loop.size(); k++) {
      const int cid = std::abs(loop[k]);
      const bool rev = loop[k] < 0;
      auto git = g.curve_group.find(cid);
      if (git == g.curve_group.end()) {
        err = "curve " + std::to_string(cid) + " of the boundary has no Physical Line";
        return false;
      }
      const CurveGeom &G = cg.at(cid);
      std::vector<double> t = split(G);
      if (rev) std::reverse(t.begin(), t.end());
      const P2 s = G.at(t.front()), e = G.at(t.back());
      if (k == 0) {
        start = s;
        bn.push_back({s, G.h_at(t.front())});
      } else if (std::hypot(s.x - prev_end.x, s.y - prev_end.y) > 1e-9 * (1 + G.len)) {
        err = "line loop " + std::to_string(lid) + " is not closed at curve " + std::to_string(cid);
        return false;
      }
      for (size_t j = 1; j < t.size(); j++) {
        const bool last = k + 1 == loop.size() && j + 1 == t.size();
        const int a = int(bn.size()) - 1;
        int b;
        if (last) {
          if (std::hypot(e.x - start.x, e.y - start.y) > 1e-9 * (1 + G.len)) {
            err = "line loop " + std::to_string(lid) + " does not close";
            return false;
          }
          b = first_node;
        } else {
          bn.push_back({G.at(t[j]), G.h_at(t[j])});
          b = int(bn.size()) - 1;
        }
        bs.push_back({a, b, cid, git->second, rev, t[j - 1], t[j]});
      }
      prev_end = e;
    }
  }
  // ---- domain test and boundary polylines -----------------------------------------------------
  auto loops_poly = [&]() {
    std::vector<std::vector<P2>> L;
    for (size_t li = 0; li < loop_first.size(); li++) {
      const int s0 = loop_first[li], s1 = li + 1 < loop_first.size() ? loop_first[li + 1] : int(bs.size());
      std::vector<P2> poly;
      for (int s = s0; s < s1; s++) poly.push_back(bn[bs[s].a].p);
      L.push_back(poly);
    }
    return L;
  };
  // ---- triangulate with boundary recovery and clipping -----------------------------------------
  // pts = boundary nodes (bn, growing under recovery) then interior nodes
  auto triangulate = [&](std::vector<P2> &interior, std::vector<std::array<int, 3>> &tri) -> bool {
    for (int round = 0; round < 64; round++) {
      const int nb = int(bn.size());
      std::vector<P2> all, jit;
      for (auto &b : bn) all.push_back(b.p);
      for (auto &p : interior) all.push_back(p);
      // connectivity on slightly perturbed coordinates (no exact cocircular / collinear ties);
      // the output keeps the exact ones
      double ext = 0;
      for (auto &p : all) ext = std::max(ext, std::max(std::fabs(p.x), std::fabs(p.y)));
      uint64_t st = 0x9E3779B97F4A7C15ull;
      for (auto &p : all) {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        double u = double(st >> 11) / 9007199254740992.0 - 0.5;
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        double v = double(st >> 11) / 9007199254740992.0 - 0.5;
        jit.push_back({p.x + 1e-9 * ext * u, p.y + 1e-9 * ext * v});
      }
      auto dt = delaunay(jit);
      std::unordered_set<uint64_t> E;
      auto key = [](int a, int b) {
        if (a > b) std::swap(a, b);
        return (uint64_t(uint32_t(a)) << 32) | uint32_t(b);
      };
      for (auto &t : dt)
        for (int k = 0; k < 3; k++) E.insert(key(t[k], t[(k + 1) % 3]));
      std::vector<int> missing;
      for (int s = 0; s < int(bs.size()); s++)
        if (!E.count(key(bs[s].a, bs[s].b))) missing.push_back(s);
      if (missing.empty()) {
        auto L = loops_poly();
        tri.clear();
        for (auto &t : dt) {
          P2 c{(all[t[0]].x + all[t[1]].x + all[t[2]].x) / 3, (all[t[0]].y + all[t[1]].y + all[t[2]].y) / 3};
          if (!inside(L, c)) continue;
          std::array<int, 3> o = t;
          if (tri_area(all[o[0]], all[o[1]], all[o[2]]) < 0) std::swap(o[1], o[2]);
          tri.push_back(o);
        }
        return true;
      }
      // split each missing segment at its curve midpoint (segments after it shift by one)
      std::sort(missing.rbegin(), missing.rend());
      for (int s : missing) {
        BSeg S = bs[s];
        const CurveGeom &G = cg.at(S.curve);
        const double tm = 0.5 * (S.t0 + S.t1);
        bn.push_back({G.at(tm), 0.5 * (bn[S.a].h + bn[S.b].h)});
        const int mnode = int(bn.size()) - 1;
        BSeg S1 = S, S2 = S;
        S1.b = mnode;
        S1.t1 = tm;
        S2.a = mnode;
        S2.t0 = tm;
        bs[s] = S1;
        bs.insert(bs.begin() + s + 1, S2);
        for (auto &f : loop_first)
          if (f > s) f++;
      }
      // interior nodes too close to the new boundary nodes go
      std::vector<P2> keep;
      for (auto &p : interior) {
        bool ok = true;
        for (size_t k = size_t(nb); k < bn.size() && ok; k++)
          ok = std::hypot(p.x - bn[k].p.x, p.y - bn[k].p.y) > 0.5 * bn[k].h;
        if (ok) keep.push_back(p);
      }
      interior.swap(keep);
    }
    err = "boundary recovery did not converge";
    return false;
  };
  // ---- size field: boundary sizes interpolated over the boundary-node triangulation -----------
  std::vector<P2> none;
  std::vector<std::array<int, 3>> bg;
  if (!triangulate(none, bg)) return false;
  double hmin = 1e300, hmax = 0;
  for (auto &b : bn) {
    hmin = std::min(hmin, b.h);
    hmax = std::max(hmax, b.h);
  }
  auto size_at = [&](P2 p) {
    for (auto &t : bg) {
      const P2 &a = bn[t[0]].p, &b = bn[t[1]].p, &c = bn[t[2]].p;
      const double A = tri_area(a, b, c);
      const double l0 = tri_area(p, b, c) / A, l1 = tri_area(a, p, c) / A, l2 = 1 - l0 - l1;
      if (l0 >= -1e-12 && l1 >= -1e-12 && l2 >= -1e-12)
        return l0 * bn[t[0]].h + l1 * bn[t[1]].h + l2 * bn[t[2]].h;
    }
    return hmax;
  };
  // ---- interior candidates, Poisson-disk thinning ---------------------------------------------
  auto L = loops_poly();
  double mnx = 1e300, mny = 1e300, mxx = -1e300, mxy = -1e300;
  for (auto &b : bn) {
    mnx = std::min(mnx, b.p.x);
    mny = std::min(mny, b.p.y);
    mxx = std::max(mxx, b.p.x);
    mxy = std::max(mxy, b.p.y);
  }
  const double s0 = 0.25 * hmin, beta = 0.8;
  const long long ncand = (long long)((mxx - mnx) / s0 + 2) * (long long)((mxy - mny) / (s0 * 0.8660254) + 2);
  if (ncand > 40000000LL) {
    err = "mesh too fine for the base mesher (raise the size scale and refine instead)";
    return false;
  }
  struct Cand {
    P2 p;
    double h;
  };
  std::vector<Cand> cand;
  uint64_t st = 12345;
  int row = 0;
  for (double y = mny; y <= mxy; y += s0 * 0.8660254, row++)
    for (double x = mnx + (row & 1) * 0.5 * s0; x <= mxx; x += s0) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      const double jx = (double(st >> 11) / 9007199254740992.0 - 0.5) * 0.1 * s0;
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      const double jy = (double(st >> 11) / 9007199254740992.0 - 0.5) * 0.1 * s0;
      P2 p{x + jx, y + jy};
      if (!inside(L, p)) continue;
      const double h = size_at(p);
      bool ok = true;
      for (size_t s = 0; s < bs.size() && ok; s++) ok = seg_dist(p, bn[bs[s].a].p, bn[bs[s].b].p) >= 0.6 * h;
      if (ok) cand.push_back({p, h});
    }
  std::stable_sort(cand.begin(), cand.end(), [](const Cand &a, const Cand &b) { return a.h < b.h; });
  // spatial hash of accepted nodes (boundary nodes included)
  const double cell = beta * hmin;
  std::unordered_map<uint64_t, std::vector<P2>> grid;
  auto ck = [&](double x, double y) {
    return (uint64_t(uint32_t(int((x - mnx) / cell) + 1)) << 32) | uint32_t(int((y - mny) / cell) + 1);
  };
  auto add = [&](P2 p) { grid[ck(p.x, p.y)].push_back(p); };
  auto near = [&](P2 p, double r) {
    const int rx = int(r / cell) + 1;
    const int cx = int((p.x - mnx) / cell) + 1, cy = int((p.y - mny) / cell) + 1;
    for (int i = cx - rx; i <= cx + rx; i++)
      for (int j = cy - rx; j <= cy + rx; j++) {
        auto it = grid.find((uint64_t(uint32_t(i)) << 32) | uint32_t(j));
        if (it == grid.end()) continue;
        for (auto &q : it->second)
          if (std::hypot(q.x - p.x, q.y - p.y) < r) return true;
      }
    return false;
  };
  for (auto &b : bn) add(b.p);
  std::vector<P2> interior;
  for (auto &c : cand)
    if (!near(c.p, beta * c.h)) {
      add(c.p);
      interior.push_back(c.p);
    }
  // ---- Delaunay + recovery + clip, then smoothing rounds -------------------------------------
  std::vector<std::array<int, 3>> tri;
  if (!triangulate(interior, tri)) return false;
  for (int it = 0; it < 3; it++) {
    const int nb = int(bn.size()), n = nb + int(interior.size());
    std::vector<double> sx(n, 0), sy(n, 0);
    std::vector<int> deg(n, 0);
    std::vector<P2> all;
    for (auto &b : bn) all.push_back(b.p);
    for (auto &p : interior) all.push_back(p);
    for (auto &t : tri)
      for (int k = 0; k < 3; k++) {
        const int a = t[k], b = t[(k + 1) % 3];
        sx[a] += all[b].x;
        sy[a] += all[b].y;
        deg[a]++;
        sx[b] += all[a].x;
        sy[b] += all[a].y;
        deg[b]++;
      }
    for (int i = nb; i < n; i++)
      if (deg[i] > 0) {
        P2 q{sx[i] / deg[i], sy[i] / deg[i]};
        if (inside(L, q)) interior[i - nb] = q;
      }
    if (!triangulate(interior, tri)) return false;
  }
  // ---- output: vertices in order of first use by a triangle ----------------------------------
  std::vector<P2> all;
  for (auto &b : bn) all.push_back(b.p);
  for (auto &p : interior) all.push_back(p);
  std::vector<int> renum(all.size(), -1);
  m = Mesh();
  m.nt = int(tri.size());
  m.tri.resize(3 * tri.size());
  for (size_t e = 0; e < tri.size(); e++)
    for (int k = 0; k < 3; k++) {
      int v = tri[e][k];
      if (renum[v] < 0) {
        renum[v] = m.nv++;
        m.xy.push_back(all[v].x);
        m.xy.push_back(all[v].y);
      }
      m.tri[3 * e + k] = renum[v];
    }
  m.nb = int(bs.size());
  for (auto &s : bs) {
    if (renum[s.a] < 0 || renum[s.b] < 0) {
      err = "boundary node outside the triangulation";
      return false;
    }
    m.bseg.push_back(renum[s.a]);
    m.bseg.push_back(renum[s.b]);
    m.bgroup.push_back(s.group);
  }
  return validate(m, err);
}

bool write_gmsh(const std::string &path, const Mesh &m, std::string &err) {
  FILE *f = std::fopen(path.c_str(), "w");
  if (!f) {
    err = "cannot write '" + path + "'";
    return false;
  }
  std::fprintf(f, "$MeshFormat\n2.2 0 8\n$EndMeshFormat\n$Nodes\n%d\n", m.nv);
  for (int v = 0; v < m.nv; v++) std::fprintf(f, "%d %.17g %.17g 0\n", v + 1, m.xy[2 * v], m.xy[2 * v + 1]);
  std::fprintf(f, "$EndNodes\n$Elements\n%d\n", m.nb + m.nt);
  int id = 1;
  for (int s = 0; s < m.nb; s++)
    std::fprintf(f, "%d 1 2 %d %d %d %d\n", id++, m.bgroup[s], m.bgroup[s], m.bseg[2 * s] + 1, m.bseg[2 * s + 1] + 1);
  for (int e = 0; e < m.nt; e++)
    std::fprintf(f, "%d 2 2 0 0 %d %d %d\n", id++, m.tri[3 * e] + 1, m.tri[3 * e + 1] + 1, m.tri[3 * e + 2] + 1);
  std::fprintf(f, "$EndElements\n");
  const bool ok = std::fclose(f) == 0;
  if (!ok) err = "write error on '" + path + "'";
  return ok;
}

}  // namespace pnp
