/*
 * pnp_capi.h — C ABI of the MI355X-native dune-pnp hot path (libpnp_amd.so).
 *
 * Replaces, for one GPU per context, what the reference gets from PDELab/ISTL on its hot path
 * (SURVEY.md §8(b)):
 *   - the LocalOperators PnpOperator / PnpTOperator / PBOperator / DiffusionOperator /
 *     DiffusionTOperator / PoissonOperator   (src/pnp_operator.hh:22-325, src/pnp_toperator.hh:
 *     10-106, src/pb_operator.hh:22-202, src/diffusion_operator.hh:18-178,
 *     src/diffusion_toperator.hh:15-77, src/poisson_operator.hh:22-209)
 *     and the GridOperator that loops them: GridOperator::residual / ::jacobian
 *     (instantiated at src/stationary_pnp_from_pb.hh:165,315-321)            -> pnp_set_operator,
 *                                                                  pnp_residual, pnp_jacobian
 *   - the linear solver backends ISTLBackend_NOVLP_BCGS_NOPREC / _SSORk
 *     (src/stationary_pnp_from_pb.hh:168-169,329-331)                     -> pnp_linear_solve
 *   - PDELab Newton (src/stationary_pnp_from_pb.hh:355-369)                -> pnp_newton
 *   - BCType / BCExtension / flux container setup (src/btype.hh:21-53, src/dirichlet_bc.hh:54-123,
 *     src/stationary_pnp_from_pb.hh:131-156)                              -> pnp_create,
 *                                                                          pnp_initial_state
 * and the process-level pieces the driver needs: gmsh input (src/pnp_solver_main.cc:86-91) and
 * the INI config (src/sysparams.cc:16-98).
 *
 * Conventions
 *   - Every function returns PNP_OK (0) or a negative PNP_E_* code; pnp_last_error() gives the
 *     message.  No C++ exception crosses this boundary.  "Not converged" is reported in the
 *     result structs (like ISTL's InverseOperatorResult), not as an error.
 *   - Vectors at this boundary use the reference's layout: lexicographic [phi | c+ | c-] over the
 *     mesh's vertex order (GridFunctionSpaceLexicographicMapper, src/stationary_pnp_from_pb.hh:
 *     228-231), length nfields*nv.  Internally the context keeps a vertex-interleaved, coloured,
 *     Morton-ordered copy in HBM.
 *   - Host pointers are borrowed for the duration of the call.  A context is single-thread-affine
 *     and owns one HIP stream; every call is synchronous on return.
 *   - Multi-GPU: one process (and one context) per GPU.  pnp_comm carries the RCCL unique id;
 *     every rank passes the same global mesh and the library partitions it (RCB).
 */
#ifndef PNP_CAPI_H
#define PNP_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNP_CAPI_VERSION 1

enum {
  PNP_OK = 0,
  PNP_E_ARG = -1,
  PNP_E_HIP = -2,
  PNP_E_RCCL = -3,
  PNP_E_BREAKDOWN = -4,  /* BiCGSTAB breakdown (ISTLError in the reference) */
  PNP_E_NOT_CONVERGED = -5,
  PNP_E_IO = -6,
  PNP_E_MESH = -7,
  PNP_E_STATE = -8       /* call order (e.g. no operator set) */
};

typedef struct pnp_ctx pnp_ctx;

/* ---- mesh ---------------------------------------------------------------------------------- */
typedef struct {
  int32_t nv;
  const double *coords;      /* [nv][2] */
  int32_t nt;
  const int32_t *tri;        /* [nt][3], 0-based */
  int32_t nbseg;
  const int32_t *bseg;       /* [nbseg][2]; index = boundarySegmentIndex */
  const int32_t *bseg_group; /* [nbseg]; physical group = boundaryIndexToEntity */
} pnp_mesh;

typedef struct pnp_mesh_buf pnp_mesh_buf; /* library-owned mesh */

/* GmshReader equivalent (src/pnp_solver_main.cc:86-91): ASCII gmsh 2.x, P1 triangles. */
int pnp_mesh_read_gmsh(const char *path, pnp_mesh_buf **out);
/* k levels of uniform red refinement (midpoints; boundary segments split, groups kept) */
int pnp_mesh_refine(const pnp_mesh *in, int32_t k, pnp_mesh_buf **out);
/* gmsh's preprocessing step for a .geo geometry (the reference runs gmsh on
 * test/pore_without_dna/pore_without_dna.geo to get the .msh its pore.cfg:21 names): the .geo
 * subset of the reference's geometries (variables, Point, Line, Circle, Line/Curve Loop, Plane
 * Surface, Physical Line) meshed natively; size_scale multiplies every characteristic length
 * (gmsh -clscale).  Deterministic. */
int pnp_mesh_from_geo(const char *path, double size_scale, pnp_mesh_buf **out);
/* write ASCII gmsh 2.2 (boundary segments with their physical group, then triangles);
 * pnp_mesh_read_gmsh of the file gives the same mesh back when the vertices are numbered in
 * order of first use by a triangle (as every mesh this library makes is) */
int pnp_mesh_write_gmsh(const pnp_mesh *m, const char *path);
/* view into a library-owned mesh (valid until pnp_mesh_free) */
int pnp_mesh_view(const pnp_mesh_buf *m, pnp_mesh *view);
void pnp_mesh_free(pnp_mesh_buf *m);

/* ---- configuration (class Sysparams / Surface, src/sysparams.hh:9-48) ------------------------ */
typedef struct {
  int32_t coulomb_btype;  /* 0 Dirichlet, 1 Neumann (flux), 2 iPBS (treated as Neumann) */
  double coulomb_flux, coulomb_potential;
  int32_t plus_btype;
  double plus_flux, plus_concentration;
  int32_t minus_btype;
  double minus_flux, minus_concentration;
} pnp_surface;

typedef struct {
  double l_b, c0, tau;
  double pi;           /* 3.1415 in the reference (quirk Q4); pass 3.141592653589793 to fix */
  int32_t cylindrical; /* axisymmetric: r = y, integrands * 2*pi*y */
  int32_t n_surfaces;
  const pnp_surface *surfaces;
} pnp_params;

#define PNP_MAX_SURFACES 64
typedef struct {
  char meshfile[1024];   /* resolved relative to the .cfg directory */
  int32_t n_surfaces, verbosity, cylindrical, linear_solver_iterations;
  double l_b, newton_reassemble_threshold, newton_reduction, newton_min_linear_reduction;
  int32_t newton_max_iterations, newton_line_search_max_iteration;
  double c0, tau;
  int32_t output_freq, n_steps, potential_update_freq;
  pnp_surface surfaces[PNP_MAX_SURFACES];
  uint32_t defaulted;    /* bitmask of [system] keys that were absent and defaulted */
} pnp_config;

/* Sysparams::readConfigFile (src/sysparams.cc:16-98); absent [system] keys get the documented
 * defaults of test/pore_pnp/pore.cfg (the reference would abort: SURVEY.md §4). */
int pnp_config_read(const char *path, pnp_config *out);

/* ---- context ------------------------------------------------------------------------------- */
/* Host-staged transport (pnp_comm.host): the halo exchange and the reductions go through the
 * caller's own communicator (an MPI, gloo or socket layer of the host program -- the reference's
 * MPI under UG's loadBalance, src/pnp_solver_main.cc:93-108), with the bytes staged through
 * pinned host memory.  For processes that cannot use RCCL (several ranks on one GPU, a host
 * without xGMI peers, a debugging run); the partition, halo layout, owner masks and solver are the
 * RCCL path's.  Both callbacks are collective and blocking and return 0 on success. */
typedef struct {
  void *user;
  /* for q < nnbr: send scount[q] doubles at sbuf + soff[q] to rank nbr[q] and receive rcount[q]
     doubles from it into rbuf + roff[q] (the same neighbour list on both sides of every pair) */
  int32_t (*exchange)(void *user, int32_t nnbr, const int32_t *nbr, const double *sbuf,
                      const int64_t *soff, const int64_t *scount, double *rbuf,
                      const int64_t *roff, const int64_t *rcount);
  /* buf[0..k) = its sum over all ranks, in place (every rank calls with the same k) */
  int32_t (*allreduce_sum)(void *user, double *buf, int32_t k);
} pnp_host_transport;

typedef struct {
  int32_t rank, size;          /* this process' rank / number of GPUs (size 1: no RCCL) */
  const void *rccl_unique_id;  /* 128-byte ncclUniqueId from rank 0 (ignored when size == 1) */
  const char *local_group;     /* test transport: if non-NULL (and no RCCL id), the `size`
                                  contexts created in THIS process with the same group name form
                                  the communicator (one host thread per rank; device-to-device
                                  copies + host barriers instead of RCCL).  Same partition, halo
                                  and reduction code paths as RCCL. */
  const pnp_host_transport *host; /* if non-NULL (and no RCCL id / local group): the host-staged
                                  transport above, borrowed for the context's lifetime */
} pnp_comm;

int pnp_create(const pnp_mesh *mesh, const pnp_params *params, int32_t device,
               const pnp_comm *comm, pnp_ctx **out);
/* The same on the Lagrange P_k space of degree 1, 2 or 3: the reference's compile-time PDEGREE
 * (Pk2DLocalFiniteElementMap<GV, Coord, Real, PDEGREE>, src/instationary_pnp_from_pb_md.hh:26-28,
 * 125, 245-247; the dune_pnp_<solver>_<k> programs of src/Makefile.am:43-111).  pnp_create is
 * degree 1.  For degree > 1 the DOFs are the Lagrange nodes (pnp_space): the mesh vertices first,
 * then k-1 points per edge, then the interior points (k = 3: one per triangle); every vector at
 * this boundary has nfields x nnodes entries, and the operators are the scalar ones of the
 * operator-split driver (PB, Poisson, diffusion, diffusion + mass) -- PnpOperator is P1 in the
 * reference (src/stationary_pnp_from_pb.hh:206-208) and is refused. */
int pnp_create_pk(const pnp_mesh *mesh, const pnp_params *params, int32_t degree, int32_t device,
                  const pnp_comm *comm, pnp_ctx **out);
void pnp_destroy(pnp_ctx *ctx);
/* message of the last failure on ctx (or of the last failed pnp_create / mesh call if ctx NULL) */
const char *pnp_last_error(const pnp_ctx *ctx);
/* fills a 128-byte buffer with a fresh RCCL unique id (rank 0 calls this, then broadcasts); a
   1-rank pnp_comm given one gets an RCCL communicator of its own (pnp_info.transport) */
int pnp_rccl_unique_id(void *out128);

typedef struct {
  int32_t nv_global, nv_owned, nv_ghost, nfields;
  int32_t ncolors, nchunks, max_slots, nranks;
  int64_t nblocks;       /* vertex-pair blocks of the owned rows (V + 2E on one GPU) */
  int64_t nnz_reduced;   /* scalar nonzeros of the stored block pattern */
  int64_t nslots;        /* SELL slots incl. padding */
  int64_t device_bytes;
  int32_t nks;           /* stored values per block of the current operator (k-form) */
  int32_t nvb;           /* block-pattern values per block (expanded, e.g. 7 for PNP) */
  int64_t lslots, uslots;/* slots of the strictly-lower / diagonal+upper split storage */
  int32_t ilu_f32;       /* PNP_OPT_ILU_F32 */
  int32_t degree;        /* polynomial degree of the space (pnp_create_pk); nv_global = its nodes */
  int64_t color_conflicts; /* owned neighbour pairs sharing a colour: couplings the multicolour
                              sweeps (SSOR, ILU(0)) leave out, see DESIGN.md §3 */
  int32_t transport;     /* 0 one rank, 1 in-process local group, 2 RCCL (also a 1-rank RCCL
                            communicator: a pnp_comm of size 1 with an RCCL id runs the
                            multi-rank code path, every reduction an ncclAllReduce), 3 the
                            host-staged transport (pnp_comm.host) */
  int64_t nat_flow_applies;  /* PNP_PREC_SSOR_NATURAL applications run as one dataflow launch
                                (any context that owns its GPU: one rank, or one RCCL rank) */
  int64_t nat_level_applies; /* ... and as level launches (the in-process local group, whose
                                ranks share one device; or PNP_NAT_FLOW=0) */
  int64_t ilu_flow_applies;  /* PNP_PREC_ILU0 applications launched as one dataflow launch
                                (PNP_OPT_ILU_FLOW; a graph capture counts once) */
  int64_t lslots_live, uslots_live; /* split slots that hold a coupling (lslots / uslots without
                                       the lane padding; U with the diagonal slot) */
  int64_t lsx_entries, usx_entries; /* the LDS sweeps' staged neighbour rows, summed over the
                                       256-row blocks: the gathers of one ILU(0) application */
} pnp_info;
int pnp_get_info(pnp_ctx *ctx, pnp_info *info);

/* The DOF space of the context (GridFunctionSpace): nnodes Lagrange nodes (= nv_global), their
 * coordinates xy[nnodes][2] and the nodes of each triangle enode[nt][nlocal] (local order:
 * vertices 0, 1, 2; the k-1 points of the faces (0,1), (0,2), (1,2) from the face's first vertex to
 * its second; interior points).  xy / enode may be NULL (query the sizes first). */
typedef struct {
  int32_t degree, nnodes, nt, nlocal;
} pnp_space_info;
int pnp_space(pnp_ctx *ctx, pnp_space_info *info, double *xy, int32_t *enode);

/* ---- operators (LocalOperator + GridOperator) ---------------------------------------------- */
enum {
  PNP_OP_PNP = 0,            /* PnpOperator (stationary 3-field)                              */
  PNP_OP_PNP_IMPLICIT_EULER, /* M(u)-M(u_old) + dt*R_pnp(u), M = PnpTOperator (Q2 kept)        */
  PNP_OP_PB,                 /* PBOperator                                                     */
  PNP_OP_DIFF,               /* DiffusionOperator, frozen phi, valency z                       */
  PNP_OP_DIFF_IMPLICIT_EULER,/* DiffusionTOperator mass + dt * DiffusionOperator              */
  PNP_OP_POISSON             /* PoissonOperator, frozen c+, c-                                 */
};

typedef struct {
  int32_t kind;
  double dt;          /* implicit Euler step (PNP_IMPLICIT_EULER, DIFF_IMPLICIT_EULER) */
  double z;           /* valency (DIFF*) */
  int32_t field;      /* DIFF*: which BCType component constrains the ion (1 plus, 2 minus) */
  const double *phi;  /* DIFF*: frozen potential [nv] */
  const double *cp, *cm; /* POISSON: frozen concentrations [nv] */
  const double *x_old;   /* *_IMPLICIT_EULER: previous time level, external layout */
  /* optional constant added to the residual (external layout, nfields x nv; constrained rows
   * stay 0): the explicit part of a multi-stage step, e.g. (1-a) dt R(u_1) in the second
   * stage of Alexander2 (PDELab OneStepMethod, src/instationary_pnp_from_pb_md.hh:387-391) */
  const double *c_extra;
} pnp_op_args;

int pnp_set_operator(pnp_ctx *ctx, const pnp_op_args *args);
/* number of fields of the current operator (3 or 1) */
int pnp_nfields(pnp_ctx *ctx);

/* r = residual(x) with constrained rows zero (GridOperator::residual + constraints);
 * x, r: host, external layout */
int pnp_residual(pnp_ctx *ctx, const double *x, double *r);
/* assemble the Jacobian at x into the context (GridOperator::jacobian + constrained rows ->
 * identity).  Analytic derivative of the reference's residual (the reference differentiates
 * numerically: NumericalJacobianVolume, eps 1e-7). */
int pnp_jacobian(pnp_ctx *ctx, const double *x);
/* copy the assembled Jacobian out as a CSR matrix in the external layout (sorted columns;
 * only the stored block pattern, i.e. structurally-zero c+/c- couplings are omitted).
 * Pass NULL arrays to query nnz first. */
int pnp_jacobian_export(pnp_ctx *ctx, int64_t *nnz, int32_t *rowptr, int32_t *col, double *val);

/* ---- call flags, device pointers, FD Jacobian, jacobian_apply, device CSR view ---------------- */
enum {
  /* vectors passed to the call are DEVICE pointers (same device as the context), external
   * layout; results are written to device memory (this rank's owned entries) and the call is
   * synchronous on return */
  PNP_DEVICE_PTRS = 1,
  /* the Jacobian is PDELab's NumericalJacobianVolume (src/pnp_operator.hh:24-27 and the other
   * LOPs' mixins): per element the local residual at u and at u + delta_j e_j, delta_j =
   * 1e-7 (1 + |u_j|), columns (r(u + delta_j e_j) - r(u)) / delta_j, accumulated element by element
   * in mesh order.  Computed on the GPU in the reference's operand order (no FMA contraction):
   * for the polynomial operators it is the oracle's FD matrix to the last bits. */
  PNP_JAC_FD = 2
};
/* pnp_residual with flags (PNP_DEVICE_PTRS) */
int pnp_residual_ex(pnp_ctx *ctx, const double *x, double *r, int32_t flags);
/* pnp_jacobian with flags (PNP_DEVICE_PTRS, PNP_JAC_FD) */
int pnp_jacobian_ex(pnp_ctx *ctx, const double *x, int32_t flags);
/* GridOperator::jacobian_apply (the LOPs' NumericalJacobianApplyVolume, src/pnp_operator.hh:22-25):
 * y = J(x) z with J the matrix pnp_jacobian assembles (constrained rows identity).  x != NULL
 * assembles J(x) first (PNP_JAC_FD: by forward differences); x == NULL applies the last
 * assembled Jacobian.  z, y: external layout, nfields*nv; PNP_DEVICE_PTRS for device vectors. */
int pnp_jacobian_apply(pnp_ctx *ctx, const double *x, const double *z, double *y, int32_t flags);
/* device CSR view of the last assembled Jacobian (the ISTL BCRSMatrix<1x1> the reference's
 * solvers take): external layout, sorted columns, the stored block pattern (structurally zero
 * c+/c- couplings omitted), constrained rows identity.  The arrays are DEVICE memory owned by the
 * context, valid until the next Jacobian assembly, pnp_set_operator or pnp_destroy. */
typedef struct {
  int32_t n;            /* rows = nfields * nv (rows owned by other ranks are empty) */
  int64_t nnz;
  const int32_t *rowptr;/* n + 1 */
  const int32_t *col;
  const double *val;
} pnp_csr_view;
int pnp_jacobian_csr_device(pnp_ctx *ctx, pnp_csr_view *view);

/* ---- linear solve (ISTL BiCGSTABSolver semantics) ----------------------------------------- */
enum { PNP_PREC_NONE = 0, PNP_PREC_SSOR = 1, PNP_PREC_ILU0 = 2, PNP_PREC_JACOBI = 3,
       PNP_PREC_AMG = 4, /* aggregation AMG V-cycle (ISTL Amg::AMG of LINEARSOLVER CG_AMG_SSOR,
                            src/instationary_pnp_from_pb_md.hh:207-210); see pnp_amg_configure */
       /* ISTL SeqSSOR(A, 1, 1.0) exactly: one forward and one backward Gauss-Seidel sweep in the
        * reference's lexicographic DOF order ([phi | c+ | c-] over the vertex order), each row's
        * sum over its columns in ascending order -- the preconditioner of the reference's default
        * ISTLBackend_NOVLP_BCGS_SSORk (src/instationary_pnp_from_pb_md.hh:30-31,188-191,
        * src/stationary_pnp_from_pb.hh:168-169), so iteration counts compare with the reference's.
        * Level-scheduled on the GPU (one launch per dependency level, ~100-300 levels): a parity
        * mode, slower than the multicolour PNP_PREC_SSOR.  Block-Jacobi across ranks. */
       PNP_PREC_SSOR_NATURAL = 5 };
enum { PNP_METHOD_BICGSTAB = 0, PNP_METHOD_CG = 1 };
typedef struct {
  int32_t prec;       /* SSOR = one multicolour symmetric Gauss-Seidel sweep (k=1, w=1) */
  double reduction;   /* stop when ||r|| < reduction * ||r0|| (checked every half step) */
  int32_t maxit;
  int32_t check_every; /* host convergence poll period in iterations (0: default 8) */
  int32_t method;     /* PNP_METHOD_BICGSTAB (ISTL BiCGSTABSolver, the default) or
                         PNP_METHOD_CG (ISTL CGSolver: LINEARSOLVER CG_NOPREC / CG_Jacobi,
                         src/instationary_pnp_from_pb_md.hh:198-206) */
} pnp_solve_opts;
typedef struct {
  int32_t converged, iterations, breakdown; /* iterations = ceil(half-step counter); breakdown:
      1 rho, 2 omega, 3 h (ISTL's 1e-80 tests), 4 diverged (PNP_PREC_AMG only) */
  double it_half, defect0, defect, reduction, elapsed;
} pnp_solve_result;

/* v = M^{-1} d for one preconditioner application on the last assembled Jacobian (the
 * Dune::Preconditioner::apply step inside ISTL's BiCGSTABSolver, istl/solvers.hh); d, v host,
 * external layout, owned rows.  PNP_PREC_ILU0 factorises on first use after an assembly.
 * Multicolour semantics: SSOR = one forward + one backward multicolour
 * Gauss-Seidel sweep, ILU0 = ILU(0) of the stored block pattern in colour-major vertex order. */
int pnp_prec_apply(pnp_ctx *ctx, int32_t prec, const double *d, double *v);

/* ---- aggregation AMG (PNP_PREC_AMG) ---------------------------------------------------------
 * Replaces the preconditioner of ISTLBackend_NOVLP_CG_AMG_SSOR (the reference's LINEARSOLVER
 * CG_AMG_SSOR, src/instationary_pnp_from_pb_md.hh:24,207-210, constructed with maxiter from the
 * config).  Greedy aggregation over the matrix graph, piecewise-constant prolongation, Galerkin
 * coarse operators (nf x nf blocks), one V-cycle per application: the level-0 smoother below
 * before and after the coarse correction, damped block-Jacobi (omega) on the coarse levels, a
 * dense direct solve on the coarsest.  Rank-local (block-Jacobi across ranks, like the sweeps).
 * With PNP_METHOD_CG and smoother SSOR this is CG_AMG_SSOR; it also preconditions BiCGSTAB. */
typedef struct {
  int32_t smoother;       /* level-0 smoother: PNP_PREC_SSOR (default), PNP_PREC_ILU0, PNP_PREC_JACOBI */
  int32_t coarse_target;  /* coarsen until at most this many vertex blocks (1..1024, default 1024:
                             the coarsest level is inverted densely, rocSOLVER getrf/getri,
                             <= 3072 unknowns) */
  int32_t max_levels;     /* levels including the fine one (2..16, default 12) */
  double omega;           /* damped block-Jacobi weight on the coarse levels (default 0.8) */
  int32_t coarse_sweeps;  /* block-Jacobi sweeps per coarse pre-/post-smoothing (1..8, default 2) */
  int32_t level0_presmooth; /* level-0 pre-smoothing: 1 yes, 0 no (post-smoothing only), -1 auto
                             (default): yes for CG and pnp_prec_apply (the V-cycle must be
                             symmetric), no for BiCGSTAB (same iterations at 2/3 of the cycle's
                             cost on config 3) */
} pnp_amg_opts;
int pnp_amg_configure(pnp_ctx *ctx, const pnp_amg_opts *opts);
typedef struct {
  int32_t levels;         /* including level 0 */
  int32_t smoother;
  int32_t rows[16];       /* vertex-block rows per level */
  int64_t blocks[16];     /* stored blocks per level */
  double omega;
} pnp_amg_stats;
/* valid after the first AMG application on this context */
int pnp_amg_info(pnp_ctx *ctx, pnp_amg_stats *stats);
/* aggregate map of level -> level+1 (test hook): level 0 indexed by global vertex (-1: not owned
 * by this rank, agg sized nv), coarser levels by row */
int pnp_amg_aggregates(pnp_ctx *ctx, int32_t level, int32_t *agg);

/* ---- context options ------------------------------------------------------------------------ */
enum {
  /* Storage precision of the ILU(0) factors (PNP_PREC_ILU0 and the AMG's ILU(0) smoother); the
   * sweeps compute in fp64 whatever it is.  The matrix, the SpMV, SSOR/Jacobi and every vector stay
   * fp64, so the operator and the converged solutions are those of the fp64 path; only the
   * preconditioner is a rounded ILU(0).  2 (default): bfloat16 factors for block systems (8
   * significant bits, 14 B per PNP block instead of 28; config 3: apply 66 -> 57 us, Newton counts
   * within their last-bit spread).  3 (opt-in): the factors of 2, and the forward sweep's
   * intermediate L^-1 d kept in single precision between the colour launches (12 B per PNP row
   * instead of 24; apply -1.8 us at config 3); the rounding makes the preconditioner nonlinear,
   * and BiCGSTAB then needs up to 2.6x the iterations on config 5; with
   * PNP_OPT_ILU_FLOW on, 3 runs as 2.  2 and 3 keep
   * single-precision factors for scalar systems (PB, Poisson, diffusion); 1: single precision
   * (apply 119 -> 95 us against fp64 in round 2, Newton 9,295 -> 9,177 iterations); 0: fp64.
   * The environment variable PNP_ILU_F32 = 0 .. 3 sets the default. */
  PNP_OPT_ILU_F32 = 1,
  /* 1 (default): ILU(0) factorisation in one launch per colour with the k-form expansion and the
   * split into L / U storage folded in; 0: the three-pass path (expand, factor, split).  Both
   * give the same factors bit for bit. */
  PNP_OPT_ILU_FUSED_FACTOR = 2,
  /* 1: every Jacobian assembly of the context (pnp_jacobian, Newton, pnp_assemble_state) is the
   * reference's forward-difference Jacobian (as PNP_JAC_FD); 0 (default): analytic */
  PNP_OPT_JAC_FD = 3,
  /* BiCGSTAB with two global reductions per iteration instead of three: rho_new = <rt,s> -
   * omega <rt,t> comes from omega's reduction, and the second half step's convergence test is
   * folded into the next iteration's <rt,v> reduction (a converged solve runs the first kernels
   * of one more iteration, whose updates are skipped).  ISTL half-step counting is unchanged.
   * -1 (default): on when the context has more than one rank (each reduction is an allreduce
   * round trip over xGMI); 0 off; 1 on. */
  PNP_OPT_BICG_TWORED = 4,
  /* 1: pnp_newton re-solves a step whose AMG-preconditioned BiCGSTAB failed with the AMG's
   * level-0 smoother alone (pnp_newton_result.linear_fallbacks).  0 (default).  The round-1
   * divergence this guarded against came from a too-small coarsest level (<= 64 blocks): with
   * the default (<= 1024 blocks, exact dense solve) config 4 runs 100 steps without a failed
   * AMG solve (profiles/r02/amg_c4_*.log). */
  PNP_OPT_AMG_FALLBACK = 5,
  /* BiCGSTAB (pnp_linear_solve, pnp_newton, pnp_bicgstab_iterations) runs the iterations between
   * two polls of its device-resident scalars as one hipGraph replay, captured on first use and
   * kept until the operator or an option changes.  Same kernels, same arguments, same results;
   * it saves the host's per-kernel launch cost where the kernels are shorter than it.  -1
   * (default): on for contexts of up to 131,072 owned rows; 0 off; 1 on (the environment
   * variable PNP_GRAPH=0/1 sets the default).  Not used with AMG, timers or more than one rank. */
  PNP_OPT_GRAPH = 6,
  /* 1: reference-order mode.  pnp_residual / pnp_jacobian / pnp_jacobian_apply / pnp_linear_solve /
   * pnp_prec_apply / pnp_newton then perform the CPU oracle's single-rank arithmetic in its order,
   * which restates PDELab's GridOperator (oracle/pnp_oracle.c): per element in element order one
   * local vector -- alpha_volume, then alpha_boundary of the element's boundary faces in DUNE's
   * face order -- added into the CSR view / residual once; implicit Euler as OneStepGridOperator:
   * the const residual -M(x_old) first, then per element the spatial and the temporal local
   * vectors; ISTL's sequential mv / dot / vector updates; PDELab Newton's defect as a sequential
   * sum.  So iterates and iteration counts are the oracle's even where BiCGSTAB is chaotic in the
   * last bits.  What the restatement cannot see -- the DUNE grid's own vertex order and
   * dune-geometry's tabulated quadrature points -- leaves parity with the DUNE program's rounding
   * unpinned (the reference ships no vectors and DUNE cannot be built here).  A parity mode, far
   * slower than the default.  Preconditioners NONE, JACOBI, SSOR_NATURAL; P1 contexts of one rank;
   * pnp_op_args.c_extra unsupported.  0 (default): the GPU's own summation orders. */
  PNP_OPT_SEQ_ORDER = 7,
  /* 1: each ILU(0) application (PNP_PREC_ILU0) is ONE dataflow launch instead of one launch per
   * colour and sweep direction: every 256-row block of every colour launch is a unit taken in the
   * launches' order by an atomic ticket, and a unit waits only for the units whose rows it reads
   * (linalg.hip k_ilu0_flow).  The same arithmetic per row, so the same results bit for bit.
   * 0: the colour launches (the environment variable PNP_ILU_FLOW=0/1 sets the default).  1: the
   * resident-grid form where the context owns its GPU (one rank), else the colour launches.
   * 2: the ticketed form, which needs no residency (also ranks sharing one GPU).
   * pnp_info.ilu_flow_applies counts the dataflow launches. */
  PNP_OPT_ILU_FLOW = 8,
  /* PNP_PREC_SSOR_NATURAL's schedule.  -1 (default): one dataflow launch per application
   * (ssor_natural.hip) whenever the context owns its GPU -- one rank, or one rank of an RCCL
   * communicator (one process per GPU) -- and the level launches for the in-process local group,
   * whose ranks share one device.  0: always the level launches.  1: always the dataflow launch;
   * with local-group ranks the caller must keep their preconditioner applications from running
   * concurrently (the dataflow needs every workgroup of its grid resident).  Both schedules give
   * the same results bit for bit; pnp_info.nat_flow_applies / nat_level_applies count them.  The
   * environment variable PNP_NAT_FLOW=0 turns the automatic choice off. */
  PNP_OPT_NAT_FLOW = 9,
  /* 1 (default): pnp_newton re-solves a Newton step whose BiCGSTAB with reduced-precision ILU(0)
   * factors (PNP_OPT_ILU_F32 = 1, 2 or 3; PNP_PREC_ILU0, or the AMG's ILU(0) smoother) broke down
   * or stopped unconverged, with the factors in fp64 -- ISTL's own SeqILU0 precision -- and keeps
   * fp64 for the rest of that call (pnp_newton_result.precision_retries).  A rounded
   * preconditioner is a different M; the retry makes the fp64 preconditioner the fallback
   * whenever the cheaper one stalls.  0: a failed solve ends Newton as in ISTL. */
  PNP_OPT_ILU_RETRY = 10
};
int pnp_set_option(pnp_ctx *ctx, int32_t option, int64_t value);

/* ---- creation options (process-wide; read by every later pnp_create / pnp_create_pk /
 * pnp_layout_build, since the row colouring and the layout are built at creation) ------------ */
enum {
  /* the thin top colour of the greedy colouring (at most 1/1024 of the rows, each coupled to all
   * colours below) is absorbed into the colours below, and its few same-colour couplings
   * (pnp_info.color_conflicts) are left out of the multicolour SSOR / ILU(0) sweeps: one colour
   * -- two sweep launches per preconditioner application -- fewer.  1 on (default), 0 off (the
   * sweeps act on the whole matrix, one colour more), -1 the default (the environment variable
   * PNP_COLOR_CONFLICTS=0 turns it off).  DESIGN.md §4.1. */
  PNP_CREATE_ABSORB_THIN_COLOR = 1
};
int pnp_set_create_option(int32_t option, int64_t value);
int pnp_get_create_option(int32_t option, int64_t *value);
int pnp_get_option(pnp_ctx *ctx, int32_t option, int64_t *value);

/* solve J z = rhs with the last assembled Jacobian; rhs, z host, external layout */
int pnp_linear_solve(pnp_ctx *ctx, const double *rhs, double *z, const pnp_solve_opts *opts,
                     pnp_solve_result *res);
/* pnp_linear_solve with flags (PNP_DEVICE_PTRS) */
int pnp_linear_solve_ex(pnp_ctx *ctx, const double *rhs, double *z, const pnp_solve_opts *opts,
                        pnp_solve_result *res, int32_t flags);

/* ---- Newton (PDELab Newton with hackbuschReuskenAcceptBest) -------------------------------- */
typedef struct {
  double reduction, abs_limit, min_linear_reduction;
  int32_t maxit, line_search_maxit;
  pnp_solve_opts linear;   /* reduction field ignored (set per step by Newton) */
} pnp_newton_opts;
typedef struct {
  int32_t converged, iterations, linear_iterations, status; /* status: PNP_OK, or
      PNP_E_NOT_CONVERGED (NewtonNotConverged / NewtonLinearSolverError / line search),
      PNP_E_BREAKDOWN */
  double first_defect, defect, elapsed, assemble_seconds, solve_seconds;
  int32_t linear_fallbacks; /* PNP_PREC_AMG with PNP_OPT_AMG_FALLBACK = 1 only: Newton steps
      whose AMG-preconditioned solve failed (diverged: ||r|| > 1e10 ||r0||, breakdown or maxit)
      and were re-solved with the AMG's level-0 smoother alone; linear_iterations counts both
      solves.  Off by default: a failed AMG solve ends Newton like any linear-solver failure. */
  int32_t precision_retries; /* PNP_OPT_ILU_RETRY: Newton steps whose linear solve with
      reduced-precision ILU(0) factors (PNP_OPT_ILU_F32 1..3; PNP_PREC_ILU0, or PNP_PREC_AMG with
      the ILU(0) smoother) broke down or did not converge and were re-solved with fp64 factors;
      the rest of that pnp_newton call then keeps fp64 factors.  linear_iterations counts both. */
} pnp_newton_result;
int pnp_newton(pnp_ctx *ctx, double *u, const pnp_newton_opts *opts, pnp_newton_result *res);
/* per-step record of the last pnp_newton on ctx (PDELab Newton's verbose per-step output,
 * src/stationary_pnp_from_pb.hh:355-369): for step k < min(cap, *nsteps) the linear solver's
 * iterations and the defect after the line search; *nsteps = the number of steps (either array
 * may be NULL) */
int pnp_newton_history(pnp_ctx *ctx, int32_t *linear_iterations, double *defects, int32_t cap,
                       int32_t *nsteps);

/* Multi-GPU: v (host, external layout, nfields*nv) holds this rank's owned entries (as returned
 * by pnp_newton / pnp_linear_solve / pnp_residual); on return it holds the global vector on every
 * rank (collective; a no-op on one GPU). */
int pnp_sync_vector(pnp_ctx *ctx, double *v, int32_t nfields);

/* The NOVLP backends' parallel scalar product (ISTL's OwnerOverlapCopy-style "owner-masked local
 * dot + allreduce", behind LS::norm at src/stationary_pnp_from_pb.hh:355-358 and the Newton
 * defect): *out = sum over the DOFs each rank owns of a_i b_i, summed over all ranks, so every rank
 * gets the global value whatever the other entries of its vectors hold.  a, b: external layout,
 * nfields x nv (host, or device memory with PNP_DEVICE_PTRS); only this rank's owned entries are
 * read.  Collective on multi-GPU.  pnp_norm = sqrt(pnp_dot(a, a)). */
int pnp_dot(pnp_ctx *ctx, const double *a, const double *b, int32_t nfields, int32_t flags,
            double *out);
int pnp_norm(pnp_ctx *ctx, const double *a, int32_t nfields, int32_t flags, double *out);

/* BCExtension interpolation: x0 (3*nv, external layout) from the PB potential phi_pb (nv). */
int pnp_initial_state(pnp_ctx *ctx, const double *phi_pb, double *x0);

/* Ion-current observable, calcIonFlux (src/ionFlux.hh:8-96, written to current.dat by
 * src/instationary_pnp_from_pb_md.hh:443-450): per boundary group g < nsurf,
 *   ip[g] = sum over its segments of len (x 2 PI y) (-grad c+ + c+ grad phi) . n,
 *   im[g] = ... (-grad c- - c- grad phi) . n,
 * fields at the segment midpoint, n the unit outer normal.  x: [phi | c+ | c-] (host, external
 * layout) or NULL for the context's current 3-field state.  Collective on multi-GPU. */
int pnp_ion_flux(pnp_ctx *ctx, const double *x, int32_t nsurf, double *ip, double *im);

/* ---- device-resident hot path (benchmarks: inputs already in HBM) --------------------------- */
/* upload x (external layout) into the context's state vector */
int pnp_state_set(pnp_ctx *ctx, const double *x);
int pnp_state_get(pnp_ctx *ctx, double *x);
/* n fused residual+Jacobian assemblies of the state vector, on the device */
int pnp_assemble_state(pnp_ctx *ctx, int32_t n);  /* n < 0: |n| residual-only assemblies */
/* the same, with the device time of the whole batch from one HIP event pair around it (ms) */
int pnp_assemble_state_timed(pnp_ctx *ctx, int32_t n, double *ms);
/* n BiCGSTAB iterations (no convergence stop) on J z = r of the last assembly */
int pnp_bicgstab_iterations(pnp_ctx *ctx, int32_t n, int32_t prec, pnp_solve_result *res);

/* Store-pattern probe of a P_k context (measurement hook, no reference counterpart): the time of
 * writing every SELL slot of every owned row once, one thread per row, with the rows taken in
 * (a) SELL order -- what the Jacobian's gather pass does -- (b) a spatial tile order: tiles of
 * `tile_elems` consecutive local elements (ascending element id), each row in the tile of its
 * first incident element, in the order the tile's elements reach them, as an element-tiled
 * assembly that kept whole rows in LDS would store them, (c) the same tiles with each tile's rows
 * sorted into SELL order (the best such a tile can do), and (d) a seeded random order.  Averages
 * over `reps` launches after two untimed ones, one HIP event pair each; rows_whole counts the rows
 * whose incident elements all lie in one tile (the rows such a tile could finish without
 * spilling). */
typedef struct {
  double us_sell, us_tile, us_tile_sorted, us_random;
  int64_t slot_bytes;  /* 8 B x (sum of row lengths): the bytes each launch stores */
  int64_t rows, rows_whole, tiles, elements;
} pnp_store_probe;
int pnp_probe_slot_stores(pnp_ctx *ctx, int32_t tile_elems, int32_t reps, pnp_store_probe *out);

/* read `bytes` of a context-owned scratch buffer on the context's stream, then synchronise:
 * evicts the matrix and vectors from the L2s and the Infinity Cache before a cache-cold timing
 * (dirty lines are written back here, outside the timed launch) */
int pnp_cache_scrub(pnp_ctx *ctx, int64_t bytes);

/* per-phase device time from HIP events recorded on the context's stream (enable first) */
typedef struct {
  double assemble_ms, spmv_ms, prec_ms, blas_ms, halo_ms, allreduce_ms;
  int64_t assemble_launches, spmv_launches, prec_launches, blas_launches;
  double factor_ms;          /* ILU(0) factorisations (once per assembly), not in prec_ms */
  int64_t factor_launches;
} pnp_timers;
int pnp_timers_enable(pnp_ctx *ctx, int32_t on);
int pnp_timers_get(pnp_ctx *ctx, pnp_timers *t);
int pnp_timers_reset(pnp_ctx *ctx);


/* ---- host-only setup / layout inspection (no GPU needed) ----------------------------------- */
/* BCType mask (src/btype.hh:21-53) and alpha_boundary Neumann load (e.g. src/pnp_operator.hh:
 * 276-313) for fields field0 .. field0+nfields-1, lexicographic [f*nv + v] */
int pnp_setup_boundary(const pnp_mesh *mesh, const pnp_params *params, int32_t nfields,
                       int32_t field0, uint8_t *mask, double *load);
/* BCExtension + interpolate (src/dirichlet_bc.hh:54-123), element loop in tri[] order */
int pnp_setup_initial_state(const pnp_mesh *mesh, const pnp_params *params, const double *phi_pb,
                            double *x0);

typedef struct pnp_layout_buf pnp_layout_buf;
typedef struct {
  int32_t n_owned, n_ghost, ncolors, nchunks, nnbr, max_slots;
  int64_t nslots, nblocks;
  const int32_t *l2g;          /* n_owned + n_ghost: local row/column -> global vertex */
  const int32_t *color_ptr;    /* ncolors + 1 */
  const int32_t *color_idx;    /* n_owned: rows of colour c at [color_ptr[c], color_ptr[c+1]) */
  const uint8_t *rowcolor;     /* n_owned + n_ghost (255 = ghost) */
  const int32_t *chunk_len;    /* nchunks */
  const int32_t *chunk_off;    /* nchunks + 1 */
  const int32_t *colidx;       /* nslots (SELL-64, see dune-pnp_amd/csrc/kernels.h) */
  const uint64_t *rowmeta;     /* n_owned: fan length / closed / break bits */
  const int32_t *nbr_ranks;    /* nnbr */
  const int32_t *recv_ptr;     /* nnbr + 1: ghost ranges received from each neighbour */
  const int32_t *send_ptr;     /* nnbr + 1 */
  const int32_t *send_idx;     /* local owned rows sent to each neighbour */
  int64_t color_conflicts;     /* owned neighbour pairs sharing a colour (absorbed thin top colour,
                                  mesh.cc absorb_top); left out of the multicolour sweeps */
} pnp_layout;
/* the partition + local layout pnp_create would build for (rank, nranks) */
int pnp_layout_build(const pnp_mesh *mesh, int32_t rank, int32_t nranks, pnp_layout_buf **out);
int pnp_layout_view(const pnp_layout_buf *b, pnp_layout *view);
void pnp_layout_free(pnp_layout_buf *b);

#ifdef __cplusplus
}
#endif
#endif
