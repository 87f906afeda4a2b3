// INI config reader: Sysparams::readConfigFile (src/sysparams.cc:16-98) semantics, with the
// documented defaults (test/pore_pnp/pore.cfg values, cylindrical = 0) for [system] keys that
// some shipped configs omit (test/cylinder_config.cfg, test/sphere_pb/sphere.cfg): the reference
// would throw Dune::RangeError there.  Each defaulted key sets a bit in pnp_config::defaulted.
#include <cctype>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <string>

#include "../../include/pnp_capi.h"

namespace {

std::string trim(const std::string &s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) a++;
  while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
  return s.substr(a, b - a);
}

}  // namespace

extern "C" int pnp_config_read(const char *path, pnp_config *out) {
  if (!path || !out) return PNP_E_ARG;
  std::ifstream in(path);
  if (!in) return PNP_E_IO;
  std::map<std::string, std::string> kv;  // "section.key" -> value
  std::string line, section;
  while (std::getline(in, line)) {
    size_t h = line.find('#');
    if (h != std::string::npos) line = line.substr(0, h);
    line = trim(line);
    if (line.empty()) continue;
    if (line.front() == '[' && line.back() == ']') {
      section = trim(line.substr(1, line.size() - 2));
      continue;
    }
    size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    kv[section + "." + trim(line.substr(0, eq))] = trim(line.substr(eq + 1));
  }
  std::memset(out, 0, sizeof *out);
  auto has = [&](const std::string &k) { return kv.count(k) > 0; };
  auto getd = [&](const std::string &k, double d) { return has(k) ? std::stod(kv[k]) : d; };
  auto geti = [&](const std::string &k, int d) { return has(k) ? int(std::stod(kv[k])) : d; };
  if (!has("mesh.filename") || !has("system.n_surfaces")) return PNP_E_IO;
  std::string dir = path;
  size_t sl = dir.find_last_of('/');
  dir = (sl == std::string::npos) ? std::string() : dir.substr(0, sl + 1);
  std::string mf = kv["mesh.filename"];
  if (!mf.empty() && mf[0] != '/') mf = dir + mf;
  std::snprintf(out->meshfile, sizeof out->meshfile, "%s", mf.c_str());
  out->n_surfaces = geti("system.n_surfaces", 0);
  if (out->n_surfaces < 0 || out->n_surfaces > PNP_MAX_SURFACES) return PNP_E_ARG;
  struct Def {
    const char *key;
    double val;
  };
  static const Def defs[] = {{"verbosity", 0},
                             {"cylindrical", 0},
                             {"l_b", 1.0},
                             {"linearSolverIterations", 20000},
                             {"newtonReassembleThreshold", 0.0},
                             {"newtonReduction", 1e-9},
                             {"newtonMinLinearReduction", 1e-8},
                             {"newtonMaxIterations", 50},
                             {"newtonLineSearchMaxIteration", 500},
                             {"c0", 0.06},
                             {"tau", 1.0},
                             {"outputFreq", 10},
                             {"nSteps", 100},
                             {"potentialUpdateFreq", 1}};
  double v[sizeof defs / sizeof defs[0]];
  for (size_t i = 0; i < sizeof defs / sizeof defs[0]; i++) {
    std::string k = std::string("system.") + defs[i].key;
    if (has(k)) {
      v[i] = std::stod(kv[k]);
    } else {
      v[i] = defs[i].val;
      out->defaulted |= 1u << i;
    }
  }
  out->verbosity = int(v[0]);
  out->cylindrical = int(v[1]);
  out->l_b = v[2];
  out->linear_solver_iterations = int(v[3]);
  out->newton_reassemble_threshold = v[4];
  out->newton_reduction = v[5];
  out->newton_min_linear_reduction = v[6];
  out->newton_max_iterations = int(v[7]);
  out->newton_line_search_max_iteration = int(v[8]);
  out->c0 = v[9];
  out->tau = v[10];
  out->output_freq = int(v[11]);
  out->n_steps = int(v[12]);
  out->potential_update_freq = int(v[13]);
  for (int i = 0; i < out->n_surfaces; i++) {
    std::string p = "surface_" + std::to_string(i) + ".";
    pnp_surface &s = out->surfaces[i];
    // class Surface defaults, src/sysparams.cc:101-116
    s.coulomb_btype = s.plus_btype = s.minus_btype = 1;
    if (!has(p + "coulombBtype") || !has(p + "plusDiffusionBtype") ||
        !has(p + "minusDiffusionBtype"))
      return PNP_E_IO;
    s.coulomb_btype = geti(p + "coulombBtype", 1);
    if (s.coulomb_btype == 0) s.coulomb_potential = getd(p + "coulombPotential", 0);
    if (s.coulomb_btype == 1) s.coulomb_flux = getd(p + "coulombFlux", 0);
    s.plus_btype = geti(p + "plusDiffusionBtype", 1);
    if (s.plus_btype == 0) s.plus_concentration = getd(p + "plusDiffusionConcentration", 0);
    if (s.plus_btype == 1) s.plus_flux = getd(p + "plusDiffusionFlux", 0);
    s.minus_btype = geti(p + "minusDiffusionBtype", 1);
    if (s.minus_btype == 0) s.minus_concentration = getd(p + "minusDiffusionConcentration", 0);
    if (s.minus_btype == 1) s.minus_flux = getd(p + "minusDiffusionFlux", 0);
  }
  return PNP_OK;
}
