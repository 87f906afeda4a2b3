/*
 * pnp_oracle.h — CPU restatement of kessel/dune-pnp's FEM assembly + BiCGStab path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (dune-pnp_amd/, include/) links, loads
 * or calls this code.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may use it, and only as the checker / the timed CPU baseline ("kind": "port").
 *
 * PARITY STATUS: the reference (DUNE/PDELab/ISTL + UG) cannot be built here or on the GPU box
 * (SURVEY.md §8(c)), and it ships no tests or golden vectors.  This restatement is pinned by:
 *   (1) an independent numpy restatement (tests/golden/make_golden.py) whose outputs are
 *       committed as fixtures under tests/golden/ and checked in the CPU test suite;
 *   (2) the reference's only known-answer data, the Gouy-Chapman / Debye-Hueckel curves in
 *       test/one_wall_dh/one_wall.gp:4-12 (planar PB on a refined strip);
 *   (3) exactness properties (Jacobian vs forward-difference Jacobian, linearity, symmetry).
 * Against the original DUNE binaries the parity is UNPINNED.
 *
 * Third-party semantics restated here (not under /root/reference, no version pin beyond
 * dune.module:10 ">= 0.1" / ">= 2.2"):
 *   - dune-geometry SimplexQuadraturePoints<2>: order<=2 -> 3-point rule (1/6 weights),
 *     order 3 -> Strang-Fix 4-point rule (centroid weight -27/96); 1-D Gauss-Legendre 2-point.
 *   - dune-pdelab NumericalJacobianVolume: eps = 1e-7*(1+|x_j|) forward differences.
 *   - dune-pdelab GridOperator + Dirichlet constraints: constrained residual rows = 0,
 *     constrained Jacobian rows = identity, columns kept.
 *   - dune-pdelab Newton (hackbuschReuskenAcceptBest line search, PDELab 1.x/2.0 newton.hh).
 *   - dune-istl BiCGSTABSolver (half-step iteration counting, EPSILON = 1e-80), SeqSSOR,
 *     SeqILU0.
 *
 * Layouts: vectors are lexicographic [phi | c+ | c-] (GridFunctionSpaceLexicographicMapper,
 * src/stationary_pnp_from_pb.hh:228-231) for the 3-field system, or length nv for scalar
 * operators.  Vertex order = order of the mesh arrays passed in.
 */
#ifndef PNP_ORACLE_H
#define PNP_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int nv;
  const double *xy; /* [nv][2] */
  int nt;
  const int *tri; /* [nt][3] */
  int nb;
  const int *bseg;   /* [nb][2]  boundary segment i = boundarySegmentIndex i */
  const int *bgroup; /* [nb]     physical group of segment i (boundaryIndexToEntity) */
} orc_mesh;

/* src/sysparams.hh:34-48 (class Surface) */
typedef struct {
  int cb;
  double cflux, cpot;
  int pb;
  double pflux, pconc;
  int mb;
  double mflux, mconc;
} orc_surface;

/* src/sysparams.hh:9-31 (the fields the hot path reads) */
typedef struct {
  double l_b, c0, tau, pi;
  int cylindrical;
  int nsurf;
  const orc_surface *surf;
} orc_params;

/* ---- setup: a9 / a10 ---------------------------------------------------------------- */
/* BCType::isDirichlet (src/btype.hh:21-53) + PDELab constraints(): mask[f*nv+v] = 1 if vertex v
 * lies on a boundary segment whose group has Btype_f == 0.  nfields = 3 (PNP) or 1 (PB/Poisson:
 * coulomb component only, src/stationary_pnp_from_pb.hh:116-124). */
void orc_dirichlet_mask(const orc_mesh *m, const orc_params *p, int nfields, uint8_t *mask);
/* flux container, src/stationary_pnp_from_pb.hh:131-156: flux[b*3+k] */
void orc_flux_container(const orc_mesh *m, const orc_params *p, double *flux);
/* BCExtension::evaluate via PDELab interpolate (src/dirichlet_bc.hh:54-123): x0[3nv] from the PB
 * potential phi_pb[nv]; element loop in tri[] order, last write wins. */
void orc_initial_state(const orc_mesh *m, const orc_params *p, const double *phi_pb, double *x0);
/* the same element loop over nl nodes per element (enode[e*nl+a] at node coordinates nxy[nn][2]):
 * x0[3 nn] (P_k: the Lagrange nodes) */
void orc_initial_state_nodes(const orc_mesh *m, const orc_params *p, int nl, const int *enode,
                             const double *nxy, int nn, const double *phi_pb, double *x0);

/* ---- residuals (a1,a2,a4,a5,a6,a7,f1) -------------------------------------------------- */
/* PnpOperator alpha_volume + alpha_boundary (src/pnp_operator.hh:46-315) + constraints. */
void orc_pnp_residual(const orc_mesh *m, const orc_params *p, const double *flux,
                      const uint8_t *mask, const double *x, double *r);
/* PnpTOperator alpha_volume (src/pnp_toperator.hh:31-101), no constraints applied. */
void orc_pnpt_residual(const orc_mesh *m, const orc_params *p, const double *x, double *r);
/* PBOperator (src/pb_operator.hh:46-194) + constraints. */
void orc_pb_residual(const orc_mesh *m, const orc_params *p, const double *flux,
                     const uint8_t *mask, const double *x, double *r);
/* DiffusionOperator (src/diffusion_operator.hh:42-112) + constraints; phi frozen, z valency. */
void orc_diff_residual(const orc_mesh *m, const orc_params *p, const uint8_t *mask,
                       const double *phi, double z, const double *x, double *r);
/* DiffusionTOperator (src/diffusion_toperator.hh:38-73), no constraints applied. */
void orc_difft_residual(const orc_mesh *m, const double *x, double *r);
/* PoissonOperator (src/poisson_operator.hh:46-199) + constraints; cp, cm frozen. */
void orc_poisson_residual(const orc_mesh *m, const orc_params *p, const double *flux,
                          const uint8_t *mask, const double *cp, const double *cm,
                          const double *x, double *r);

/* ---- matrices (a3, a8) ---------------------------------------------------------------- */
typedef struct {
  int n;
  int nnz;
  int *rowptr; /* n+1 */
  int *col;    /* nnz, sorted per row */
  double *val; /* nnz */
} orc_csr;

/* FullVolumePattern (PDELab) for nfields fields per vertex: all local pairs. */
void orc_csr_pattern(const orc_mesh *m, int nfields, orc_csr *A);
void orc_csr_free(orc_csr *A);

enum { ORC_OP_PNP = 0, ORC_OP_PNP_IMPLICIT_EULER = 1, ORC_OP_PB = 2, ORC_OP_DIFF = 3,
       ORC_OP_DIFF_IMPLICIT_EULER = 4, ORC_OP_POISSON = 5 };

typedef struct {
  int kind;            /* ORC_OP_* */
  const double *flux;  /* [nb][3] */
  const uint8_t *mask; /* constraint mask, nfields*nv */
  double dt;           /* implicit Euler dt (stepped operators) */
  double z;            /* valency (DIFF) */
  const double *phi;   /* frozen potential (DIFF) */
  const double *cp, *cm; /* frozen concentrations (POISSON) */
  const double *x_old; /* previous time level (implicit Euler) */
} orc_operator;

int orc_operator_nfields(const orc_operator *op);
/* residual of the (possibly time-discrete) operator, constraints applied */
void orc_op_residual(const orc_mesh *m, const orc_params *p, const orc_operator *op,
                     const double *x, double *r);
/* All-core CPU baseline (bench only): element colouring (no two elements of a colour share a
 * vertex; returns the colour count or -1) and the residual + forward-difference Jacobian
 * assembly of the ops's PnpOperator / PB / Poisson path with OpenMP over the elements of each
 * colour (eorder lists the elements colour by colour, cptr[ncol+1] the colour offsets). */
int orc_element_colors(const orc_mesh *m, int *color);
void orc_assemble_mt(const orc_mesh *m, const orc_params *p, const orc_operator *op,
                     const double *x, const int *eorder, const int *cptr, int ncol, orc_csr *A,
                     double *r);
int orc_num_threads(void);
/* Jacobian into A (pattern from orc_csr_pattern).  fd=1: PDELab NumericalJacobianVolume
 * forward differences (reference-faithful); fd=0: analytic. Constrained rows -> identity. */
void orc_op_jacobian(const orc_mesh *m, const orc_params *p, const orc_operator *op,
                     const double *x, int fd, orc_csr *A);

/* ---- linear algebra (a11) -------------------------------------------------------------- */
enum { ORC_PREC_NONE = 0, ORC_PREC_SSOR = 1, ORC_PREC_ILU0 = 2, ORC_PREC_JACOBI = 3 };
typedef struct {
  int converged;
  int iterations; /* ceil(it), ISTL InverseOperatorResult */
  double it_half; /* the raw half-step counter */
  double reduction;
  double defect0, defect;
  int breakdown; /* 1 rho, 2 omega, 3 h */
  double setup_seconds; /* preconditioner construction (ILU(0) factorisation, block split) */
  double iter_seconds;  /* the iteration loop (wall clock, omp_get_wtime) */
} orc_solve_result;

void orc_spmv(const orc_csr *A, const double *x, double *y);
/* ISTL BiCGSTABSolver::apply(x, b, res): x overwritten (start value = x), b overwritten. */
/* 1: OpenMP row-parallel SpMV / dots / updates in orc_bicgstab (all-core CPU baseline) */
void orc_set_parallel(int on);
/* nblocks > 1: SSOR and ILU(0) act block-Jacobi on nblocks vertex ranges (row f*nv + v is in
 * block v*nblocks/nv; couplings between blocks dropped), the blocks swept in parallel -- what the
 * reference's ISTLBackend_NOVLP_* applies with nblocks MPI ranks, each rank's SeqSSOR / SeqILU0
 * on its own rows (src/stationary_pnp_from_pb.hh:168-169), here with contiguous vertex ranges
 * instead of the reference's load-balanced partition.  0 or 1: the sequential preconditioner. */
void orc_set_block_jacobi(int nblocks, int nfields);
void orc_bicgstab(const orc_csr *A, int prec, double reduction, int maxit, double *x, double *b,
                  orc_solve_result *res);
/* v = W^{-1} d, one application of preconditioner prec from v = 0 (ISTL SeqSSOR / SeqILU0 /
 * Jacobi / Richardson as inside orc_bicgstab) */
void orc_prec_apply(const orc_csr *A, int prec, const double *d, double *v);
/* ISTL CGSolver (LINEARSOLVER CG_NOPREC / CG_Jacobi), see pnp_oracle.c */
void orc_cg(const orc_csr *A, int prec, double reduction, int maxit, double *x, double *b,
            orc_solve_result *res);

/* ---- nonlinear / time (a12, a13) ------------------------------------------------------ */
typedef struct {
  double reduction, abs_limit, min_linear_reduction;
  int maxit, line_search_maxit, reassemble_threshold_zero;
  int linear_maxit, prec, fd_jacobian;
} orc_newton_opts;
#define ORC_NEWTON_MAX_RECORD 64
typedef struct {
  int converged, iterations, linear_iterations, status;
  double first_defect, defect;
  int step_linear_iterations[ORC_NEWTON_MAX_RECORD]; /* BiCGSTAB iterations of each Newton step */
} orc_newton_result;
/* PDELab Newton::apply on op, u in/out. status: 0 ok, -1 not converged, -2 line search,
 * -3 linear solver did not converge (NewtonLinearSolverError). */
void orc_newton(const orc_mesh *m, const orc_params *p, const orc_operator *op, double *u,
                const orc_newton_opts *o, orc_newton_result *res);

/* ---- f3: ion-current observable ---------------------------------------------------------
 * calcIonFlux, src/ionFlux.hh:8-96 (called from src/instationary_pnp_from_pb_md.hh:443):
 * x = [phi | c+ | c-] (lexicographic, 3*nv).  ip, im: [nsurf], indexed by bgroup. */
void orc_ion_flux(const orc_mesh *m, const orc_params *p, const double *x, double *ip,
                  double *im);

/* ---- f4: P_k elements (PDEGREE 2, 3), pnp_oracle_pk.c --------------------------------------
 * The scalar operators of the operator-split driver on the Lagrange space of degree k
 * (src/instationary_pnp_from_pb_md.hh:26-28, 125, 245-247).  Vectors are over the space's nodes
 * (S->nn); op->phi / cp / cm / x_old too.  PB and Poisson add their coulomb Neumann flux
 * (op->flux [nb][3], or the surfaces' coulomb flux when NULL). */
typedef struct {
  int k, nl, nn, nedge;
  double *xy; /* [nn][2] */
  int *enode; /* [nt][nl]: vertices, face points (faces (0,1),(0,2),(1,2)), interior points */
} orc_pk;
int orc_pk_build(const orc_mesh *m, int k, orc_pk *S);
void orc_pk_free(orc_pk *S);
/* Lagrange basis of degree k on the local nodes at (xi, eta): phi[nl], dphi[nl][2] */
void orc_pk_basis(int k, double xi, double eta, double *phi, double *dphi);
/* the simplex rule of an intorder on the reference triangle (order <= 2: 3 points, 3: 4, else the
 * 7-point order-5 rule): n points into xi / eta / w (room for 7), returns n */
int orc_quadrature_rule(int order, double *xi, double *eta, double *w);
void orc_pk_dirichlet_mask(const orc_mesh *m, const orc_pk *S, const orc_params *p, int field,
                           uint8_t *mask);
void orc_pk_residual(const orc_mesh *m, const orc_pk *S, const orc_params *p,
                     const orc_operator *op, const double *x, double *r);
void orc_pk_csr_pattern(const orc_mesh *m, const orc_pk *S, orc_csr *A);
void orc_pk_jacobian(const orc_mesh *m, const orc_pk *S, const orc_params *p,
                     const orc_operator *op, const double *x, int fd, orc_csr *A);
void orc_pk_initial_state(const orc_mesh *m, const orc_pk *S, const orc_params *p,
                          const double *phi_pb, double *x0);
void orc_pk_ion_flux(const orc_mesh *m, const orc_pk *S, const orc_params *p, const double *x,
                     double *ip, double *im);

#ifdef __cplusplus
}
#endif
#endif
