// pnp_main — process driver over the C ABI, mirroring the reference's compiled binary:
//   src/dune_pnp.cc:9-39  (main, exception handling)
//   src/pnp_solver_main.cc:70-116  (config, gmsh read, grid, scenario)
//   src/stationary_pnp_from_pb.hh:93-369  (PB Newton -> BCExtension -> PNP Newton)
//   src/instationary_pnp_from_pb.hh:320-431  (time loop; implicit Euler here)
//   src/instationary_pnp_from_pb_md.hh:295-454  (operator split: Poisson + Alexander2 diffusion,
//                                                 ion current to current.dat)
//
// usage: pnp_main <config.cfg> [--refine k] [--mode stationary|instationary|md|pb] [--steps n]
//                 [--prec none|ssor|ssor_natural|jacobi|ilu0|amg] [--pb-prec ...] [--amg-smoother s]
//                 [--device d] [--out prefix]
//                 [--md-reduction r]
//                 [--linear-solver bcgs_ssork|bcgs_ssork_mc|bcgs_noprec|cg_noprec|cg_jacobi|cg_amg_ssor]
//                 (bcgs_ssork, the reference's default: ISTL SeqSSOR in the lexicographic order,
//                  PNP_PREC_SSOR_NATURAL; bcgs_ssork_mc: the multicolour sweep, same method, other order)
//                 [--degree k]   (md / pb modes: PDEGREE, src/instationary_pnp_from_pb_md.hh:26-28;
//                                 the dune_pnp_<solver>_<k> programs of src/Makefile.am:43-111)
//                 [--reference-order]  (--reference-solvers with PNP_OPT_SEQ_ORDER: the CPU oracle's
//                                 sequential arithmetic, so every Newton step's BiCGSTAB count is the
//                                 oracle's; parity with the DUNE program itself unpinned)
//                 [--reference-solvers]  (stationary / pb / instationary: the reference's own
//                                 choices, src/stationary_pnp_from_pb.hh:168-169,329-331 -- PB with
//                                 ISTLBackend_NOVLP_BCGS_SSORk = --pb-prec ssor_natural, PNP with
//                                 ISTLBackend_NOVLP_BCGS_NOPREC = --prec none; the defaults are the
//                                 multicolour SSOR for both, same methods' faster relatives)
// Multi-GPU: run one process per GPU with RANK / WORLD_SIZE / LOCAL_RANK in the environment and
// PNP_RCCL_ID_FILE pointing to a shared path (rank 0 writes the RCCL unique id there).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pnp_pdelab_adapter.hh"

using V = std::vector<double>;

static int prec_of(const std::string &s) {
  if (s == "none" || s == "nonprec") return PNP_PREC_NONE;
  if (s == "ssor") return PNP_PREC_SSOR;
  if (s == "ssor_natural") return PNP_PREC_SSOR_NATURAL;  // ISTL SeqSSOR in the reference's order
  if (s == "jacobi") return PNP_PREC_JACOBI;
  if (s == "ilu0") return PNP_PREC_ILU0;
  if (s == "amg") return PNP_PREC_AMG;  // level-0 smoother: --amg-smoother (PB: ssor, PNP: ilu0)
  throw pnp_gpu::Error(PNP_E_ARG, "unknown preconditioner " + s);
}

static void usage() {
  std::printf(
      "usage: pnp_main <config.cfg> [--refine k] [--mesh-scale s] [--mode stationary|instationary|md|pb]\n"
      "                [--steps n] [--prec none|ssor|ssor_natural|jacobi|ilu0|amg] [--pb-prec p]\n"
      "                [--device d]\n"
      "                [--amg-smoother ssor|ilu0|jacobi]\n"
      "                [--out prefix] [--md-reduction r]\n"
      "                [--linear-solver bcgs_ssork|bcgs_ssork_mc|bcgs_noprec|cg_noprec|cg_jacobi|cg_amg_ssor]\n"
      "                [--abs-limit a] [--dump-steps n1,n2,...] [--degree 1|2|3]\n"
      "                [--reference-solvers]  (PB: ISTL SeqSSOR in DOF order, PNP: no preconditioner)\n"
      "                [--reference-order]    (the same solvers in the CPU oracle's summation orders,\n"
      "                                        PNP_OPT_SEQ_ORDER: per-step iteration counts as the oracle's)\n");
}

static void write_vector(const std::string &path, const V &v, int nv) {
  std::ofstream f(path);
  f.precision(17);
  int nf = int(v.size()) / nv;
  for (int i = 0; i < nv; i++) {
    for (int k = 0; k < nf; k++) f << (k ? " " : "") << v[size_t(k) * nv + i];
    f << "\n";
  }
}

// StationaryLinearProblemSolver::apply (PDELab; used at src/instationary_pnp_from_pb_md.hh:
// 349-350, 383-386): r = R(x), A = J(x), solve A z = r to `reduction`, x -= z.
static void linear_problem(pnp_gpu::Context &ctx, pnp_gpu::GridOperator<V> &go,
                           pnp_gpu::BiCGStabBackend<V> &ls, V &x, int nfields, double reduction) {
  V r(x.size(), 0.0), z(x.size(), 0.0);
  pnp_gpu::Matrix m;
  go.residual(x, r);
  go.jacobian(x, m);
  ctx.sync(r, nfields);
  ls.apply(m, z, r, reduction);
  ctx.sync(z, nfields);
  for (size_t i = 0; i < x.size(); i++) x[i] -= z[i];
}

// Operator-split time loop of src/instationary_pnp_from_pb_md.hh:411-454.
//   c+ and c- each take one OneStepMethod<Alexander2> step (a = 1 - sqrt(2)/2):
//     stage 1: M(u1) - M(u0) + a dt R(u1) = 0                      (DIFF_IMPLICIT_EULER, a dt)
//     stage 2: M(u2) - M(u0) + (1-a) dt R(u1) + a dt R(u2) = 0      (same + c_extra)
//   with R = DiffusionOperator (frozen phi, z = +-1) and M = DiffusionTOperator, each stage one
//   linear solve (StationaryLinearProblemSolver, reduction 1e-5, :380-384); every
//   potentialUpdateFreq steps the PoissonOperator problem with the new c+- (reduction 1e-10,
//   :349-350, :421-423); every outputFreq steps the ion current (calcIonFlux) to current.dat
//   (:424-451) as "time ip_0 im_0 ip_1 im_1 ..." with each ip/im a 2-vector (component 1 = 0).
static void md_loop(pnp_gpu::Context &ctx, const pnp_gpu::Sysparams &s, V &u, int nv, int rank,
                    int steps, double md_reduction, int prec, int method,
                    const std::string &out) {
  V phi(u.begin(), u.begin() + nv), cp(u.begin() + nv, u.begin() + 2 * size_t(nv)),
      cm(u.begin() + 2 * size_t(nv), u.end());
  const double a = 1.0 - 0.5 * std::sqrt(2.0), dt = s.cfg.tau;
  const double red_diff = md_reduction > 0 ? md_reduction : 1e-5;
  const double red_pois = md_reduction > 0 ? md_reduction : 1e-10;
  const int nsteps = steps > 0 ? steps : s.cfg.n_steps;
  const int upd = std::max(1, s.cfg.potential_update_freq), outf = std::max(1, s.cfg.output_freq);
  const int nsurf = s.cfg.n_surfaces;
  pnp_gpu::BiCGStabBackend<V> ls(ctx, s.cfg.linear_solver_iterations, prec, 0, method);
  std::ofstream current;
  if (rank == 0) current.open(out.empty() ? std::string("current.dat") : out + "_current.dat");
  current.precision(17);
  auto poisson = [&]() {
    pnp_gpu::Operator op(PNP_OP_POISSON);
    op.args.cp = cp.data();
    op.args.cm = cm.data();
    pnp_gpu::GridOperator<V> go(ctx, op);
    linear_problem(ctx, go, ls, phi, 1, red_pois);
  };
  auto alexander2 = [&](V &c, double z, int field) {
    const V u0 = c;
    pnp_gpu::Operator s1(PNP_OP_DIFF_IMPLICIT_EULER);
    s1.args.dt = a * dt;
    s1.args.z = z;
    s1.args.field = field;
    s1.args.phi = phi.data();
    s1.args.x_old = u0.data();
    V u1 = u0;
    {
      pnp_gpu::GridOperator<V> go(ctx, s1);
      linear_problem(ctx, go, ls, u1, 1, red_diff);
    }
    pnp_gpu::Operator sp(PNP_OP_DIFF);
    sp.args.z = z;
    sp.args.field = field;
    sp.args.phi = phi.data();
    V r1(nv, 0.0);
    {
      pnp_gpu::GridOperator<V> go(ctx, sp);
      go.residual(u1, r1);
      ctx.sync(r1, 1);
    }
    for (auto &v : r1) v *= (1.0 - a) * dt;
    pnp_gpu::Operator s2 = s1;
    s2.args.c_extra = r1.data();
    V u2 = u1;
    {
      pnp_gpu::GridOperator<V> go(ctx, s2);
      linear_problem(ctx, go, ls, u2, 1, red_diff);
    }
    c = u2;
  };
  double time = 0;
  std::vector<double> ip(nsurf), im(nsurf);
  V x(3 * size_t(nv));
  for (int i = 0; i < nsteps; i++) {
    alexander2(cp, +1.0, 1);
    alexander2(cm, -1.0, 2);
    time += dt;
    if (i % upd == 0) poisson();
    if (i % outf == 0) {
      std::copy(phi.begin(), phi.end(), x.begin());
      std::copy(cp.begin(), cp.end(), x.begin() + nv);
      std::copy(cm.begin(), cm.end(), x.begin() + 2 * size_t(nv));
      pnp_gpu::check(pnp_ion_flux(ctx.get(), x.data(), nsurf, ip.data(), im.data()), ctx.get());
      if (rank == 0) {
        current << time;
        for (int g = 0; g < nsurf; g++) current << " " << ip[g] << " 0 " << im[g] << " 0";
        current << std::endl;
      }
    }
  }
  poisson();
  std::copy(phi.begin(), phi.end(), u.begin());
  std::copy(cp.begin(), cp.end(), u.begin() + nv);
  std::copy(cm.begin(), cm.end(), u.begin() + 2 * size_t(nv));
}

int main(int argc, char **argv) {
  if (argc < 2 || !std::strcmp(argv[1], "--help") || !std::strcmp(argv[1], "-h")) {
    usage();
    return argc < 2 ? 1 : 0;
  }
  std::string cfgfile = argv[1], mode = "stationary", prec = "ssor", pb_prec = "ssor", out;
  std::string amg_smoother;  // empty: SSOR for the PB phase, ILU(0) for the PNP phases
  int refine = 0, steps = -1, device = -1, degree = 1;
  bool ref_order = false;
  double mesh_scale = 1.0;  // size scale when the mesh comes from a .geo (gmsh -clscale)
  double md_reduction = -1;  // md mode: override the linear reductions (1e-5 diffusion, 1e-10 Poisson)
  // Newton absolute limit (PDELab NewtonTerminate abs_limit, default 1e-12 as in PDELab); the
  // instationary run needs it above the residual's rounding floor
  double abs_limit = 1e-12;
  std::vector<int> dump_steps;  // instationary: write the state after these steps (1-based)
  // md mode: PbLS, the compile-time LINEARSOLVER of src/instationary_pnp_from_pb_md.hh:20-32,188-211
  std::string linsolver = "bcgs_ssork";
  for (int i = 2; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) throw pnp_gpu::Error(PNP_E_ARG, "missing value for " + a);
      return argv[++i];
    };
    if (a == "--refine") refine = std::atoi(next().c_str());
    else if (a == "--mesh-scale") mesh_scale = std::atof(next().c_str());
    else if (a == "--mode") mode = next();
    else if (a == "--steps") steps = std::atoi(next().c_str());
    else if (a == "--prec") prec = next();
    else if (a == "--pb-prec") pb_prec = next();
    else if (a == "--amg-smoother") amg_smoother = next();
    else if (a == "--device") device = std::atoi(next().c_str());
    else if (a == "--out") out = next();
    else if (a == "--md-reduction") md_reduction = std::atof(next().c_str());
    else if (a == "--linear-solver") linsolver = next();
    else if (a == "--abs-limit") abs_limit = std::atof(next().c_str());
    else if (a == "--degree") degree = std::atoi(next().c_str());
    else if (a == "--reference-solvers") {
      pb_prec = "ssor_natural";
      prec = "none";
    } else if (a == "--reference-order") {  // the reference's solvers in its summation orders
      pb_prec = "ssor_natural";
      prec = "none";
      ref_order = true;
    }
    else if (a == "--dump-steps") {
      std::string l = next();
      for (size_t p = 0; p < l.size();) {
        size_t q = l.find(',', p);
        if (q == std::string::npos) q = l.size();
        dump_steps.push_back(std::atoi(l.substr(p, q - p).c_str()));
        p = q + 1;
      }
    } else {
      usage();
      return 1;
    }
  }
  try {
    int rank = std::getenv("RANK") ? std::atoi(std::getenv("RANK")) : 0;
    int world = std::getenv("WORLD_SIZE") ? std::atoi(std::getenv("WORLD_SIZE")) : 1;
    if (device < 0) device = std::getenv("LOCAL_RANK") ? std::atoi(std::getenv("LOCAL_RANK")) : 0;
    pnp_gpu::Sysparams s(cfgfile);
    pnp_gpu::Mesh mesh(s.cfg.meshfile, refine, mesh_scale);
    pnp_params params = s.params();
    std::vector<char> uid(128, 0);
    pnp_comm comm{rank, world, nullptr, nullptr};
    if (world > 1) {  // RCCL unique-id bootstrap through a shared file
      const char *idf = std::getenv("PNP_RCCL_ID_FILE");
      if (!idf) throw pnp_gpu::Error(PNP_E_ARG, "WORLD_SIZE > 1 needs PNP_RCCL_ID_FILE");
      if (rank == 0) {
        pnp_gpu::check(pnp_rccl_unique_id(uid.data()));
        std::string tmp = std::string(idf) + ".tmp";
        std::ofstream(tmp, std::ios::binary).write(uid.data(), 128);
        std::rename(tmp.c_str(), idf);
      } else {
        for (int t = 0; t < 6000; t++) {
          std::ifstream f(idf, std::ios::binary);
          if (f && f.read(uid.data(), 128)) break;
          std::this_thread::sleep_for(std::chrono::milliseconds(10));
        }
      }
      comm.rccl_unique_id = uid.data();
    }
    if (degree != 1 && mode != "md" && mode != "pb")  // PnpOperator is P1 in the reference
      throw pnp_gpu::Error(PNP_E_ARG, "--degree applies to the md and pb modes (the stationary "
                                      "and instationary drivers are P1: src/stationary_pnp_from_pb.hh:206-208)");
    pnp_gpu::Context ctx(mesh, params, device, world > 1 ? &comm : nullptr, degree);
    // PNP_OPT_SEQ_ORDER: element-order assembly, ISTL's sequential mv / dot / updates, so every
    // Newton step takes the CPU oracle's BiCGSTAB iteration count (one rank, P1; the DUNE
    // program's own rounding order is unpinned)
    if (ref_order) pnp_gpu::check(pnp_set_option(ctx.get(), PNP_OPT_SEQ_ORDER, 1), ctx.get());
    const int newton_verbosity = rank == 0 ? (ref_order ? 2 : 1) : 0;
    int nv = ctx.nv();  // DOF nodes of the P_degree space
    if (rank == 0)
      std::printf("mesh %s refined %d: %d vertices, P%d: %d nodes, config %s (%s)\n",
                  s.cfg.meshfile, refine, mesh.nv(), degree, nv, cfgfile.c_str(),
                  s.cfg.cylindrical ? "cylindrical" : "planar");

    // ---- PB (src/stationary_pnp_from_pb.hh:105-185): pbu = 0, Newton, BCGS_SSORk ----------
    pnp_gpu::Operator pblop(PNP_OP_PB);
    pnp_gpu::GridOperator<V> pbgo(ctx, pblop);
    pnp_gpu::BiCGStabBackend<V> pbls(ctx, s.cfg.linear_solver_iterations, prec_of(pb_prec),
                                     rank == 0 ? s.cfg.verbosity : 0);
    auto amg_for = [&](const char *dflt) {  // PNP_PREC_AMG's level-0 smoother for a phase
      ctx.amg_configure(prec_of(amg_smoother.empty() ? std::string(dflt) : amg_smoother));
    };
    if (pb_prec == "amg") amg_for("ssor");
    V pbu(nv, 0.0);
    pnp_gpu::Newton<V> pbnewton(pbgo, pbu, pbls);
    pbnewton.setReduction(s.cfg.newton_reduction);
    pbnewton.setMinLinearReduction(s.cfg.newton_min_linear_reduction);
    pbnewton.setMaxIterations(s.cfg.newton_max_iterations);
    pbnewton.setLineSearchMaxIterations(s.cfg.newton_line_search_max_iteration);
    pbnewton.setVerbosityLevel(newton_verbosity);
    try {
      pbnewton.apply();
    } catch (pnp_gpu::Error &e) {
      std::printf("Something has happened (%s)\n", e.what());  // :181-185
    }
    ctx.sync(pbu, 1);  // owned entries of every rank -> global PB potential
    if (!out.empty() && rank == 0) write_vector(out + "_pb.dat", pbu, nv);
    if (mode == "pb") return 0;
    // ---- PNP initial state (interpolate(BCExtension), :282) --------------------------------
    V u(3 * size_t(nv));
    pnp_gpu::check(pnp_initial_state(ctx.get(), pbu.data(), u.data()), ctx.get());
    pnp_gpu::BiCGStabBackend<V> ls(ctx, s.cfg.linear_solver_iterations, prec_of(prec),
                                   rank == 0 ? s.cfg.verbosity : 0);
    if (prec == "amg") amg_for("ilu0");
    auto configure = [&](pnp_gpu::Newton<V> &nw) {
      nw.setReduction(s.cfg.newton_reduction);
      nw.setMinLinearReduction(s.cfg.newton_min_linear_reduction);
      nw.setMaxIterations(s.cfg.newton_max_iterations);
      nw.setLineSearchMaxIterations(s.cfg.newton_line_search_max_iteration);
      nw.setAbsoluteLimit(abs_limit);
      nw.setVerbosityLevel(newton_verbosity);
    };
    int status = 0;
    if (mode == "stationary") {  // :293-369
      pnp_gpu::Operator lop(PNP_OP_PNP);
      pnp_gpu::GridOperator<V> go(ctx, lop);
      pnp_gpu::Newton<V> newton(go, u, ls);
      configure(newton);
      try {
        newton.apply();
      } catch (pnp_gpu::Error &e) {
        std::printf("Something has happened (%s)\n", e.what());  // :365-369
        status = 2;
      }
    } else if (mode == "instationary") {  // :409-431, implicit Euler, dt = tau
      int n = steps > 0 ? steps : 100;
      if (!out.empty() && rank == 0) write_vector(out + "_x0.dat", u, nv);
      for (int i = 0; i < n; i++) {
        if (i > 0) ctx.sync(u, 3);
        V uold = u;
        pnp_gpu::Operator lop(PNP_OP_PNP_IMPLICIT_EULER);
        lop.args.dt = s.cfg.tau;
        lop.args.x_old = uold.data();
        pnp_gpu::GridOperator<V> go(ctx, lop);
        pnp_gpu::Newton<V> newton(go, u, ls);
        configure(newton);
        newton.setVerbosityLevel(0);
        try {
          newton.apply();
        } catch (pnp_gpu::Error &e) {
          std::printf("step %d: Something has happened (%s)\n", i, e.what());
          status = 2;
          break;
        }
        if (rank == 0 && (i % std::max(1, s.cfg.output_freq) == 0 || i + 1 == n))
          std::printf("step %d t=%g newton it %d (linear %d) defect %.3e\n", i, (i + 1) * s.cfg.tau,
                      newton.result().iterations, newton.result().linear_iterations,
                      newton.result().defect);
        if (std::find(dump_steps.begin(), dump_steps.end(), i + 1) != dump_steps.end()) {
          V g = u;
          ctx.sync(g, 3);
          if (!out.empty() && rank == 0)
            write_vector(out + "_step" + std::to_string(i + 1) + ".dat", g, nv);
        }
      }
    } else if (mode == "md") {  // src/instationary_pnp_from_pb_md.hh:295-454
      if (!out.empty() && rank == 0) write_vector(out + "_x0.dat", u, nv);
      // BCGS_SSORk (the default of src/instationary_pnp_from_pb_md.hh:30-31, ISTLBackend_NOVLP_
      // BCGS_SSORk(gfs, maxit, 1, verbose) at :188-191): SeqSSOR in the GFS's lexicographic order
      int lmethod = PNP_METHOD_BICGSTAB, lprec = PNP_PREC_SSOR_NATURAL;
      if (linsolver == "bcgs_ssork_mc") lprec = PNP_PREC_SSOR;
      else if (linsolver == "bcgs_noprec") lprec = PNP_PREC_NONE;
      else if (linsolver == "cg_noprec") lmethod = PNP_METHOD_CG, lprec = PNP_PREC_NONE;
      else if (linsolver == "cg_jacobi") lmethod = PNP_METHOD_CG, lprec = PNP_PREC_JACOBI;
      else if (linsolver == "cg_amg_ssor") lmethod = PNP_METHOD_CG, lprec = PNP_PREC_AMG;
      else if (linsolver != "bcgs_ssork")
        throw pnp_gpu::Error(PNP_E_ARG, "unknown --linear-solver " + linsolver);
      md_loop(ctx, s, u, nv, rank, steps, md_reduction, lprec, lmethod, out);
    } else {
      usage();
      return 1;
    }
    ctx.sync(u, 3);
    if (!out.empty() && rank == 0) write_vector(out + "_pnp.dat", u, nv);
    return status;
  } catch (pnp_gpu::Error &e) {  // src/dune_pnp.cc:33-38
    std::fprintf(stderr, "Dune reported error: %s\n", e.what());
    return 1;
  } catch (std::exception &e) {
    std::fprintf(stderr, "Unknown exception thrown: %s\n", e.what());
    return 1;
  }
}
