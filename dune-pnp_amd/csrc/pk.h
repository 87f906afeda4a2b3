// Lagrange P_k spaces on the triangle mesh (k = 1, 2, 3): the reference's compile-time PDEGREE
// (Pk2DLocalFiniteElementMap<GV, Coord, Real, PDEGREE>, src/instationary_pnp_from_pb_md.hh:26-28,
// 125, 245-247; the 15 EXTRA_PROGRAMS dune_pnp_<solver>_<k> of src/Makefile.am:43-111).
//
// DOF nodes ("nodes" below) are the Lagrange points: the mesh vertices first (node v = vertex v),
// then k-1 points per edge, then (k-1)(k-2)/2 interior points per triangle (one for k = 3).  The
// solver side (colouring, SELL-64 layout, SpMV, sweeps, BiCGSTAB, AMG, halo) runs on the node
// graph exactly as it runs on the vertex graph for P1: a node row couples to every node of every
// element that contains it (FullVolumePattern).
#pragma once

#include <string>
#include <vector>

#include "mesh.h"
#include <array>

namespace pnp {

struct PkSpace {
  int k = 1;
  int nl = 3;      // local nodes per element, (k+1)(k+2)/2
  int nn = 0;      // global nodes
  int nv = 0, nedge = 0;
  std::vector<double> xy;    // [nn][2]
  // [nt][nl] global node of each local node.  Local order: vertices 0, 1, 2 (reference (0,0),
  // (1,0), (0,1)), then the k-1 points of the faces (0,1), (0,2), (1,2) (DUNE's reference-
  // triangle face order) from the face's first vertex to its second, then interior points.
  std::vector<int> enode;
  std::vector<double> lref;  // [nl][2] reference coordinates of the local nodes
  std::vector<int> bnode;    // [nb][k+1] nodes of boundary segment s from bseg[2s] to bseg[2s+1]
  std::vector<int> bface;    // [nb] element * 3 + local face of each boundary segment
};

bool build_pk_space(const Mesh &m, int k, PkSpace &S, std::string &err);

// Lagrange basis of degree k on the local nodes of PkSpace::lref, at reference point (xi, eta):
// phi[nl], and the reference gradients dphi[nl][2] (either may be null).  Silvester's product of
// shifted barycentric factors.
void pk_basis(int k, double xi, double eta, double *phi, double *dphi);

// Node graph (the FullVolumePattern of the P_k space) in the Fans shape the layout builder takes:
// sorted neighbour lists, meta = row length only (no fan bits; the P_k assembly is element-based).
bool pk_adjacency(const Mesh &m, const PkSpace &S, Fans &f, std::string &err);

// A Mesh over the nodes (xy of the nodes, no elements): partitioning and Morton order of the
// layout builder read only the coordinates.
Mesh pk_node_mesh(const PkSpace &S);

// Boundary data on the nodes, as mesh.h's dirichlet_mask / neumann_load on the vertices:
// NonoverlappingConformingDirichletConstraints constrain every node of a Dirichlet face; the
// flux of alpha_boundary is integrated with the 2-point Gauss rule (face intorder 3) against the
// trace of the P_k basis on the face.
void pk_dirichlet_mask(const Mesh &m, const PkSpace &S, const Params &p, int nf, int field0,
                       std::vector<uint8_t> &mask);
void pk_neumann_load(const Mesh &m, const PkSpace &S, const Params &p, int nf, int field0,
                     std::vector<double> &load);
// interpolate(BCExtension) at the Lagrange nodes (src/dirichlet_bc.hh:54-123): x0[3 nn] from the
// PB potential at the nodes phi_pb[nn] (null: 0)
void pk_initial_state(const Mesh &m, const PkSpace &S, const Params &p, const double *phi_pb,
                      double *x0);

}  // namespace pnp
