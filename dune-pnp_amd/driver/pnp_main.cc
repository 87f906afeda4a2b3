// pnp_main — process driver over the C ABI, mirroring the reference's compiled binary:
//   src/dune_pnp.cc:9-39  (main, exception handling)
//   src/pnp_solver_main.cc:70-116  (config, gmsh read, grid, scenario)
//   src/stationary_pnp_from_pb.hh:93-369  (PB Newton -> BCExtension -> PNP Newton)
//   src/instationary_pnp_from_pb.hh:320-431  (time loop; implicit Euler here)
//
// usage: pnp_main <config.cfg> [--refine k] [--mode stationary|instationary|pb] [--steps n]
//                 [--prec none|ssor|jacobi] [--pb-prec ...] [--device d] [--out prefix]
// Multi-GPU: run one process per GPU with RANK / WORLD_SIZE / LOCAL_RANK in the environment and
// PNP_RCCL_ID_FILE pointing to a shared path (rank 0 writes the RCCL unique id there).
#include <chrono>
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
  if (s == "jacobi") return PNP_PREC_JACOBI;
  if (s == "ilu0") return PNP_PREC_ILU0;
  throw pnp_gpu::Error(PNP_E_ARG, "unknown preconditioner " + s);
}

static void usage() {
  std::printf(
      "usage: pnp_main <config.cfg> [--refine k] [--mode stationary|instationary|pb]\n"
      "                [--steps n] [--prec none|ssor|jacobi] [--pb-prec p] [--device d]\n"
      "                [--out prefix]\n");
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

int main(int argc, char **argv) {
  if (argc < 2 || !std::strcmp(argv[1], "--help") || !std::strcmp(argv[1], "-h")) {
    usage();
    return argc < 2 ? 1 : 0;
  }
  std::string cfgfile = argv[1], mode = "stationary", prec = "ssor", pb_prec = "ssor", out;
  int refine = 0, steps = -1, device = -1;
  for (int i = 2; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) throw pnp_gpu::Error(PNP_E_ARG, "missing value for " + a);
      return argv[++i];
    };
    if (a == "--refine") refine = std::atoi(next().c_str());
    else if (a == "--mode") mode = next();
    else if (a == "--steps") steps = std::atoi(next().c_str());
    else if (a == "--prec") prec = next();
    else if (a == "--pb-prec") pb_prec = next();
    else if (a == "--device") device = std::atoi(next().c_str());
    else if (a == "--out") out = next();
    else {
      usage();
      return 1;
    }
  }
  try {
    int rank = std::getenv("RANK") ? std::atoi(std::getenv("RANK")) : 0;
    int world = std::getenv("WORLD_SIZE") ? std::atoi(std::getenv("WORLD_SIZE")) : 1;
    if (device < 0) device = std::getenv("LOCAL_RANK") ? std::atoi(std::getenv("LOCAL_RANK")) : 0;
    pnp_gpu::Sysparams s(cfgfile);
    pnp_gpu::Mesh mesh(s.cfg.meshfile, refine);
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
    pnp_gpu::Context ctx(mesh, params, device, world > 1 ? &comm : nullptr);
    int nv = mesh.nv();
    if (rank == 0)
      std::printf("mesh %s refined %d: %d vertices, config %s (%s)\n", s.cfg.meshfile, refine, nv,
                  cfgfile.c_str(), s.cfg.cylindrical ? "cylindrical" : "planar");

    // ---- PB (src/stationary_pnp_from_pb.hh:105-185): pbu = 0, Newton, BCGS_SSORk ----------
    pnp_gpu::Operator pblop(PNP_OP_PB);
    pnp_gpu::GridOperator<V> pbgo(ctx, pblop);
    pnp_gpu::BiCGStabBackend<V> pbls(ctx, s.cfg.linear_solver_iterations, prec_of(pb_prec),
                                     rank == 0 ? s.cfg.verbosity : 0);
    V pbu(nv, 0.0);
    pnp_gpu::Newton<V> pbnewton(pbgo, pbu, pbls);
    pbnewton.setReduction(s.cfg.newton_reduction);
    pbnewton.setMinLinearReduction(s.cfg.newton_min_linear_reduction);
    pbnewton.setMaxIterations(s.cfg.newton_max_iterations);
    pbnewton.setLineSearchMaxIterations(s.cfg.newton_line_search_max_iteration);
    pbnewton.setVerbosityLevel(rank == 0 ? 1 : 0);
    try {
      pbnewton.apply();
    } catch (pnp_gpu::Error &e) {
      std::printf("Something has happened (%s)\n", e.what());  // :181-185
    }
    ctx.sync(pbu, 1);  // owned entries of every rank -> global PB potential
    if (mode == "pb") {
      if (!out.empty() && rank == 0) write_vector(out + "_pb.dat", pbu, nv);
      return 0;
    }
    // ---- PNP initial state (interpolate(BCExtension), :282) --------------------------------
    V u(3 * size_t(nv));
    pnp_gpu::check(pnp_initial_state(ctx.get(), pbu.data(), u.data()), ctx.get());
    pnp_gpu::BiCGStabBackend<V> ls(ctx, s.cfg.linear_solver_iterations, prec_of(prec),
                                   rank == 0 ? s.cfg.verbosity : 0);
    auto configure = [&](pnp_gpu::Newton<V> &nw) {
      nw.setReduction(s.cfg.newton_reduction);
      nw.setMinLinearReduction(s.cfg.newton_min_linear_reduction);
      nw.setMaxIterations(s.cfg.newton_max_iterations);
      nw.setLineSearchMaxIterations(s.cfg.newton_line_search_max_iteration);
      nw.setVerbosityLevel(rank == 0 ? 1 : 0);
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
      }
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
