// pnp_pdelab_adapter.hh — header-only C++ adapter that gives the C ABI (pnp_capi.h) the shape
// of the PDELab / ISTL objects the reference's drivers use, so a driver like
// src/stationary_pnp_from_pb.hh:293-369 keeps its structure:
//
//   reference (PDELab 1.x / ISTL 2.2)                  adapter
//   ------------------------------------------------   ----------------------------------------
//   LOP lop(phiB_t, cpB_t, cmB_t, f, s, flux)  :293    pnp_gpu::Operator lop(PNP_OP_PNP)
//   GO go(gfs,cc,gfs,cc,lop)                   :315    pnp_gpu::GridOperator<V> go(ctx, lop)
//   M m(go); m = 0.0; go.jacobian(u, m)        :318    pnp_gpu::Matrix m; go.jacobian(u, m)
//   go.residual(u, r)  (r accumulates)                 go.residual(u, r)  (r accumulates)
//   ISTLBackend_NOVLP_BCGS_NOPREC<GFS> ls(gfs,
//       maxit, verbose)                        :329    pnp_gpu::BiCGStabBackend<V> ls(ctx, maxit,
//                                                          PNP_PREC_NONE, verbose)
//   ls.apply(m, z, r, reduction); ls.result()          same
//   Newton<GO,LS,U> newton(go, u, ls)          :355    pnp_gpu::Newton<V> newton(go, u, ls)
//   newton.setReduction(...); newton.apply()   :357-366 same setters, apply()
//
// V is any vector type with contiguous double storage in the lexicographic [phi|c+|c-] order of
// GridFunctionSpaceLexicographicMapper: std::vector<double>, or Dune::BlockVector<FieldVector<
// double,1>> through the pnp_gpu::data() overloads below.  Errors become pnp_gpu::Error (a
// std::runtime_error), matching the reference's DUNE exceptions caught at src/dune_pnp.cc:33-38.
#ifndef PNP_PDELAB_ADAPTER_HH
#define PNP_PDELAB_ADAPTER_HH

#include <cmath>
#include <cstdio>
#include <fstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "pnp_capi.h"

namespace pnp_gpu {

class Error : public std::runtime_error {
 public:
  Error(int code, const std::string &msg) : std::runtime_error(msg), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

inline void check(int rc, const pnp_ctx *ctx = nullptr) {
  if (rc != PNP_OK) throw Error(rc, std::string("pnp: ") + pnp_last_error(ctx));
}

// contiguous storage access (overload for other vector types as needed)
inline double *data(std::vector<double> &v) { return v.data(); }
inline const double *data(const std::vector<double> &v) { return v.data(); }
inline size_t size(const std::vector<double> &v) { return v.size(); }

// ---- mesh / config (GmshReader, Sysparams) ---------------------------------------------------
class Mesh {
 public:
  // the .msh a config names; when it does not exist but the .geo of the same name does, the
  // geometry is meshed here (the reference's workflow runs gmsh on the .geo first)
  explicit Mesh(const std::string &gmsh_file, int refine = 0, double size_scale = 1.0) {
    pnp_mesh_buf *b = nullptr;
    const std::string geo = gmsh_file.substr(0, gmsh_file.rfind('.')) + ".geo";
    if (!std::ifstream(gmsh_file) && std::ifstream(geo))
      check(pnp_mesh_from_geo(geo.c_str(), size_scale, &b));
    else
      check(pnp_mesh_read_gmsh(gmsh_file.c_str(), &b));
    if (refine > 0) {
      pnp_mesh v;
      pnp_mesh_view(b, &v);
      pnp_mesh_buf *r = nullptr;
      int rc = pnp_mesh_refine(&v, refine, &r);
      pnp_mesh_free(b);
      check(rc);
      b = r;
    }
    buf_ = b;
    pnp_mesh_view(buf_, &view_);
  }
  ~Mesh() { pnp_mesh_free(buf_); }
  Mesh(const Mesh &) = delete;
  Mesh &operator=(const Mesh &) = delete;
  const pnp_mesh &view() const { return view_; }
  int nv() const { return view_.nv; }

 private:
  pnp_mesh_buf *buf_ = nullptr;
  pnp_mesh view_{};
};

struct Sysparams {
  pnp_config cfg{};
  explicit Sysparams(const std::string &file) { check(pnp_config_read(file.c_str(), &cfg)); }
  pnp_params params(double pi = 3.1415) const {  // PI = 3.1415 in the reference (quirk Q4)
    pnp_params p{};
    p.l_b = cfg.l_b;
    p.c0 = cfg.c0;
    p.tau = cfg.tau;
    p.pi = pi;
    p.cylindrical = cfg.cylindrical;
    p.n_surfaces = cfg.n_surfaces;
    p.surfaces = cfg.surfaces;
    return p;
  }
};

// ---- one GPU (one rank) ------------------------------------------------------------------------
class Context {
 public:
  // degree: the GridFunctionSpace's Pk2DLocalFiniteElementMap degree (PDEGREE); vectors are over
  // its nv() Lagrange nodes (the mesh vertices for degree 1)
  Context(const Mesh &mesh, const pnp_params &params, int device = 0,
          const pnp_comm *comm = nullptr, int degree = 1) {
    int rc = pnp_create_pk(&mesh.view(), &params, degree, device, comm, &ctx_);
    check(rc);
    pnp_info info{};
    check(pnp_get_info(ctx_, &info), ctx_);
    nv_ = info.nv_global;
  }
  ~Context() { pnp_destroy(ctx_); }
  Context(const Context &) = delete;
  Context &operator=(const Context &) = delete;
  pnp_ctx *get() const { return ctx_; }
  int nv() const { return nv_; }
  // multi-GPU: turn this rank's owned entries into the global vector (collective)
  template <class V>
  void sync(V &v, int nfields) const {
    check(pnp_sync_vector(ctx_, data(v), nfields), ctx_);
  }
  // PNP_PREC_AMG options (ISTLBackend_NOVLP_CG_AMG_SSOR's AMG; defaults: SSOR smoother)
  void amg_configure(int smoother = PNP_PREC_SSOR, int coarse_target = 1024, int max_levels = 12,
                     double omega = 0.8, int coarse_sweeps = 2, int level0_presmooth = -1) {
    pnp_amg_opts o{smoother, coarse_target, max_levels, omega, coarse_sweeps, level0_presmooth};
    check(pnp_amg_configure(ctx_, &o), ctx_);
  }

 private:
  pnp_ctx *ctx_ = nullptr;
  int nv_ = 0;
};

// LocalOperator selection (PnpOperator, PnpTOperator+PnpOperator, PBOperator, ...)
struct Operator {
  pnp_op_args args{};
  explicit Operator(int kind) { args.kind = kind; }
  int nfields() const {
    return (args.kind == PNP_OP_PNP || args.kind == PNP_OP_PNP_IMPLICIT_EULER) ? 3 : 1;
  }
};

// The assembled Jacobian lives on the GPU; this handle marks "assembled for this operator".
struct Matrix {
  bool assembled = false;
  Matrix &operator=(double) {  // `m = 0.0` in the reference
    assembled = false;
    return *this;
  }
};

template <class V>
class GridOperator {
 public:
  GridOperator(Context &ctx, const Operator &lop) : ctx_(ctx), lop_(lop) { bind(); }
  void bind() const { check(pnp_set_operator(ctx_.get(), &lop_.args), ctx_.get()); }
  size_t size() const { return size_t(lop_.nfields()) * ctx_.nv(); }
  // PDELab semantics: r += R(x)
  void residual(const V &x, V &r) const {
    std::vector<double> tmp(size());
    check(pnp_residual(ctx_.get(), data(x), tmp.data()), ctx_.get());
    double *rp = data(r);
    for (size_t i = 0; i < tmp.size(); i++) rp[i] += tmp[i];
  }
  void jacobian(const V &x, Matrix &m) const {
    check(pnp_jacobian_ex(ctx_.get(), data(x), numerical_ ? PNP_JAC_FD : 0), ctx_.get());
    m.assembled = true;
  }
  // PDELab semantics: y += J(x) z (the LOPs' NumericalJacobianApplyVolume/Boundary mixins)
  void jacobian_apply(const V &x, const V &z, V &y) const {
    std::vector<double> tmp(size());
    check(pnp_jacobian_apply(ctx_.get(), data(x), data(z), tmp.data(), numerical_ ? PNP_JAC_FD : 0),
          ctx_.get());
    double *yp = data(y);
    for (size_t i = 0; i < tmp.size(); i++) yp[i] += tmp[i];
  }
  // the reference's NumericalJacobianVolume (forward differences, eps 1e-7) instead of the analytic
  // Jacobian, for this operator's jacobian / jacobian_apply and for Newton on this context
  void setNumericalJacobian(bool on) {
    numerical_ = on;
    check(pnp_set_option(ctx_.get(), PNP_OPT_JAC_FD, on ? 1 : 0), ctx_.get());
  }
  Context &context() const { return ctx_; }

 private:
  Context &ctx_;
  Operator lop_;
  bool numerical_ = false;
};

struct InverseOperatorResult {  // Dune::InverseOperatorResult
  int iterations = 0;
  double reduction = 0, conv_rate = 0, elapsed = 0;
  bool converged = false;
};

template <class V>
class BiCGStabBackend {
 public:
  // method PNP_METHOD_CG gives the ISTLBackend_NOVLP_CG_* backends (ISTL CGSolver)
  BiCGStabBackend(Context &ctx, int maxit, int prec = PNP_PREC_NONE, int verbose = 0,
                  int method = PNP_METHOD_BICGSTAB)
      : ctx_(ctx), maxit_(maxit), prec_(prec), verbose_(verbose), method_(method) {}
  // z = A^{-1} r (A = last assembled Jacobian), ISTL BiCGSTABSolver semantics
  void apply(Matrix &A, V &z, V &r, double reduction) {
    if (!A.assembled) throw Error(PNP_E_STATE, "pnp: matrix not assembled");
    pnp_solve_opts o{prec_, reduction, maxit_, 8, method_};
    pnp_solve_result res{};
    int rc = pnp_linear_solve(ctx_.get(), data(r), data(z), &o, &res);
    if (rc != PNP_OK && rc != PNP_E_BREAKDOWN) check(rc, ctx_.get());
    if (rc == PNP_E_BREAKDOWN) throw Error(rc, "breakdown in BiCGSTAB");  // ISTLError
    res_.iterations = res.iterations;
    res_.reduction = res.reduction;
    res_.converged = res.converged != 0;
    res_.elapsed = res.elapsed;
    res_.conv_rate = res.it_half > 0 ? std::pow(res.reduction, 1.0 / res.it_half) : 0.0;
    if (verbose_ > 0)
      std::printf("=== BiCGSTABSolver: rate=%g, T=%g, IT=%d\n", res_.conv_rate, res_.elapsed,
                  res_.iterations);
  }
  // the NOVLP backend's parallel norm / scalar product: owned entries of every rank, allreduced
  // (pnp_norm / pnp_dot); v holds nfields x nv entries in the lexicographic order
  double norm(const V &v) const {
    double out = 0;
    check(pnp_norm(ctx_.get(), data(v), nfields(v), 0, &out), ctx_.get());
    return out;
  }
  double dot(const V &a, const V &b) const {
    double out = 0;
    check(pnp_dot(ctx_.get(), data(a), data(b), nfields(a), 0, &out), ctx_.get());
    return out;
  }
  const InverseOperatorResult &result() const { return res_; }
  int nfields(const V &v) const {
    const size_t n = size(v), nv = size_t(ctx_.nv());
    if (nv == 0 || n % nv != 0 || n / nv < 1 || n / nv > 3)
      throw Error(PNP_E_ARG, "pnp: vector length is not nfields x nv");
    return int(n / nv);
  }
  int prec() const { return prec_; }
  int maxit() const { return maxit_; }
  int method() const { return method_; }

 private:
  Context &ctx_;
  int maxit_, prec_, verbose_, method_;
  InverseOperatorResult res_;
};

// PDELab Newton with hackbuschReuskenAcceptBest; runs entirely through pnp_newton (the
// residual, Jacobian and BiCGSTAB stay in HBM between steps)
template <class V>
class Newton {
 public:
  struct Result {
    int iterations = 0, linear_iterations = 0;
    double first_defect = 0, defect = 0, elapsed = 0;
    bool converged = false;
  };
  Newton(GridOperator<V> &go, V &u, BiCGStabBackend<V> &ls) : go_(go), u_(u), ls_(ls) {}
  void setReduction(double r) { o_.reduction = r; }
  void setMinLinearReduction(double r) { o_.min_linear_reduction = r; }
  void setMaxIterations(int n) { o_.maxit = n; }
  void setLineSearchMaxIterations(int n) { o_.line_search_maxit = n; }
  void setAbsoluteLimit(double a) { o_.abs_limit = a; }
  void setReassembleThreshold(double) {}  // the GPU path reassembles every step (threshold 0)
  void setVerbosityLevel(int v) { verbose_ = v; }
  void apply() {
    go_.bind();
    o_.linear.prec = ls_.prec();
    o_.linear.maxit = ls_.maxit();
    o_.linear.method = ls_.method();
    o_.linear.check_every = 8;
    pnp_newton_result r{};
    check(pnp_newton(go_.context().get(), data(u_), &o_, &r), go_.context().get());
    res_.iterations = r.iterations;
    res_.linear_iterations = r.linear_iterations;
    res_.first_defect = r.first_defect;
    res_.defect = r.defect;
    res_.elapsed = r.elapsed;
    res_.converged = r.converged != 0;
    if (verbose_ > 1) {  // PDELab Newton's per-step lines (verbosity 2)
      int32_t n = 0;
      check(pnp_newton_history(go_.context().get(), nullptr, nullptr, 0, &n), go_.context().get());
      std::vector<int32_t> its(n);
      std::vector<double> dfs(n);
      check(pnp_newton_history(go_.context().get(), its.data(), dfs.data(), n, &n),
            go_.context().get());
      for (int k = 0; k < n; k++)
        std::printf("  Newton iteration %3d.  New defect: %12.4e  (linear iterations %d)\n", k + 1,
                    dfs[k], its[k]);
    }
    if (verbose_ > 0)
      std::printf("  Newton converged=%d after %d iterations (%d linear), defect %.6e -> %.6e\n",
                  r.converged, r.iterations, r.linear_iterations, r.first_defect, r.defect);
    if (r.status != PNP_OK)  // NewtonNotConverged / NewtonLinearSolverError / line search
      throw Error(r.status, "Newton did not converge");
  }
  const Result &result() const { return res_; }

 private:
  GridOperator<V> &go_;
  V &u_;
  BiCGStabBackend<V> &ls_;
  pnp_newton_opts o_{1e-8, 1e-12, 1e-3, 40, 10, {PNP_PREC_NONE, 0.0, 20000, 8, PNP_METHOD_BICGSTAB}};
  Result res_;
  int verbose_ = 0;
};

}  // namespace pnp_gpu

#endif
