// Host-side mesh pipeline for the MI355X PNP path.
//
//   gmsh v2 reader          (what dune-grid's GmshReader gives the reference at
//                            src/pnp_solver_main.cc:86-91: triangles, boundary segments in file
//                            order = boundarySegmentIndex, physical group = boundaryIndexToEntity)
//   uniform red refinement  (the reference has none; SURVEY.md §5 scaling row)
//   vertex fans             (CCW neighbour sequence around each vertex: the element loop of the
//                            owner-computes assembly kernel is a walk along this fan)
//   RCB partition, colouring, Morton order and the SELL-64 block layout of the local problem.
#pragma once

#include <atomic>

#include <array>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace pnp {

struct Mesh {
  int nv = 0, nt = 0, nb = 0;
  std::vector<double> xy;     // [nv][2]
  std::vector<int> tri;       // [nt][3]
  std::vector<int> bseg;      // [nb][2]
  std::vector<int> bgroup;    // [nb]
};

bool read_gmsh(const std::string &path, Mesh &m, std::string &err);
bool write_gmsh(const std::string &path, const Mesh &m, std::string &err);
Mesh refine(const Mesh &m, int k);
bool validate(const Mesh &m, std::string &err);

// .geo subset and the native mesher standing in for gmsh (geo_mesh.cc)
struct GeoModel {
  std::map<int, std::array<double, 3>> pts;  // id -> x, y, lc (0: none given)
  struct Curve {
    bool circle = false;
    int a = -1, b = -1, c = -1;  // start, end, centre (circle)
  };
  std::map<int, Curve> curves;
  std::map<int, std::vector<int>> loops;     // signed curve ids
  std::map<int, std::vector<int>> surfaces;  // loop ids, outer first
  std::map<int, int> curve_group;            // Physical Line
};
bool read_geo(const std::string &path, GeoModel &g, std::string &err);
// size_scale multiplies every characteristic length (gmsh -clscale)
bool mesh_geo(const GeoModel &g, double size_scale, Mesh &m, std::string &err);

// Vertex fan: for vertex v, neighbours nbr[ptr[v] .. ptr[v+1]) in CCW order around v.
// meta bits: [0,6) L = 1 + #neighbours (slots incl. diagonal), bit 6 closed (an element joins
// the last neighbour back to the first), bits 8+s (s = 1..L-2): NO element between slot s and
// slot s+1 (a break between two fans of a pinched vertex).
struct Fans {
  std::vector<int> ptr, nbr;
  std::vector<uint64_t> meta;
  int max_slots = 0;
};
bool build_fans(const Mesh &m, Fans &f, std::string &err);

static inline int meta_len(uint64_t m) { return int(m & 63); }
static inline bool meta_closed(uint64_t m) { return (m >> 6) & 1; }
static inline bool meta_break(uint64_t m, int s) { return (m >> (8 + s)) & 1; }

// Boundary data of the hot path, computed once per operator.
// field_btype(s, f): surface s, field f (0 coulomb, 1 plus, 2 minus)
struct Surface {
  int cb = 1; double cflux = 0, cpot = 0;
  int pb = 1; double pflux = 0, pconc = 0;
  int mb = 1; double mflux = 0, mconc = 0;
  int btype(int f) const { return f == 0 ? cb : (f == 1 ? pb : mb); }
  double flux(int f) const { return f == 0 ? cflux : (f == 1 ? pflux : mflux); }
};
struct Params {
  double l_b = 1, c0 = 0.06, tau = 1, pi = 3.1415;
  int cylindrical = 0;
  std::vector<Surface> surf;
};

// Dirichlet mask (BCType::isDirichlet, src/btype.hh:21-53), vertex-major [nv][nf]
void dirichlet_mask(const Mesh &m, const Params &p, int nf, int field0, std::vector<uint8_t> &mask);
// Neumann load j*psi*f of alpha_boundary (src/pnp_operator.hh:276-313), vertex-major [nv][nf]
void neumann_load(const Mesh &m, const Params &p, int nf, int field0, std::vector<double> &load);
// BCExtension + interpolate (src/dirichlet_bc.hh:54-123): lexicographic x0[3nv] from phi_pb[nv]
void initial_state(const Mesh &m, const Params &p, const double *phi_pb, double *x0);
// the same over nl nodes per element (enode [nt][nl], node coordinates nxy [nn][2]); x0[3 nn]
void initial_state_at(const Mesh &m, const Params &p, int nl, const int *enode, const double *nxy,
                      int nn, const double *phi_pb, double *x0);

// ---- distribution and local layout -----------------------------------------------------------
// RCB on vertex coordinates into nparts (deterministic); part[v] in [0, nparts)
void rcb_partition(const Mesh &m, int nparts, std::vector<int> &part);

constexpr int kChunk = 64;        // one wavefront of rows per SELL chunk
constexpr int kOrderBlock = 4096;  // window of the slot-count sort

struct LocalLayout {
  int rank = 0, nranks = 1;
  int n_owned = 0, n_ghost = 0;
  std::vector<int> l2g;            // local -> global vertex (owned then ghosts)
  std::vector<int> g2l;            // global -> local, -1 if absent (size nv)
  // Row order: colour-major (rows of colour c are [color_ptr[c], color_ptr[c+1])), Morton order
  // inside a colour.  color_idx lists the rows of each colour in storage order (the identity for
  // this order); rowcolor[i] is the colour of local row/column i (255 for ghosts).
  std::vector<int> color_ptr, color_idx;
  std::vector<uint8_t> rowcolor;
  // SELL-64: chunk c covers rows [64c, 64c+64), has chunk_len[c] slots; slot s of row r is at
  // position chunk_off[c] + s*64 + (r - 64c)
  int nchunks = 0;
  std::vector<int> chunk_len, chunk_off;
  std::vector<int> colidx;         // local column (vertex) per slot; padding: the row itself
  std::vector<uint64_t> rowmeta;   // fan meta per owned row
  std::vector<int> xmap;           // per slot s>=1 of row i (col j owned, j<i... any j owned):
                                   // bits [0,5) slot of i in row j, [5,10) slot of the fan
                                   // predecessor of j (seen from i) in row j, [10,15) successor;
                                   // 31 = absent
  long long nslots = 0;            // total SELL slots incl. padding
  long long nblocks = 0;           // real blocks (V+2E restricted to owned rows)
  long long conflicts = 0;         // owned neighbour pairs of one colour (left out of the sweeps)
  // halo: per neighbour rank q, ghosts [ghost_ptr[q], ghost_ptr[q+1]) (offsets into ghosts) are
  // received from q; send_idx[send_ptr[q] .. send_ptr[q+1]) are local owned rows sent to q
  std::vector<int> nbr_ranks;
  std::vector<int> recv_ptr, send_ptr, send_idx;
};

// PNP_CREATE_ABSORB_THIN_COLOR (pnp_set_create_option): -1 default (on, unless the environment
// variable PNP_COLOR_CONFLICTS=0), 0 off, 1 on -- read by build_local_layout
extern std::atomic<int> g_absorb_thin_color;
bool build_local_layout(const Mesh &m, const Fans &f, const std::vector<int> &part, int rank,
                        int nranks, LocalLayout &L, std::string &err);

}  // namespace pnp
