// C-ABI implementation (include/pnp_capi.h): context, device buffers, halo exchange over RCCL,
// device-resident BiCGSTAB (ISTL semantics) and PDELab-semantics Newton, host-orchestrated.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <queue>
#include <random>
#include <chrono>
#include <condition_variable>
#include <map>
#include <unordered_map>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/pnp_capi.h"
#include "amg.h"
#include "kernels.h"
#include "mesh.h"
#include "pk.h"

namespace {

thread_local std::string g_err;  // errors without a context (create / mesh calls)

template <typename T>
struct DBuf {
  T *p = nullptr;
  size_t n = 0;
  hipError_t alloc(size_t count) {
    release();
    n = count;
    if (count == 0) return hipSuccess;
    hipError_t e = hipMalloc(&p, sizeof(T) * count);
    if (e == hipSuccess) e = hipMemset(p, 0, sizeof(T) * count);  // no reliance on fresh pages
    // the memset runs on the null stream, which does not order against the context's
    // non-blocking streams: finish it before a kernel there writes the buffer (seen as zeroed
    // FD element matrices with 8 in-process ranks competing for the GPU)
    if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
  ~DBuf() { release(); }
};

enum TimerCat { T_ASM = 0, T_SPMV, T_PREC, T_BLAS, T_HALO, T_ALLRED, T_FACT, T_NCAT };

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

}  // namespace

struct pnp_mesh_buf {
  pnp::Mesh m;
};

// In-process communicator for tests on one GPU (pnp_comm::local_group): ranks are contexts in
// one process, each driven by its own host thread.  Collectives are host barriers plus
// device-to-device copies; every call synchronises, which is fine for correctness tests.
struct LocalGroup {
  int size = 0;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long generation = 0;
  std::vector<pnp_ctx *> members;
  std::vector<std::vector<double>> host;  // per-rank published host values (allreduce)
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    long gen = generation;
    if (++arrived == size) {
      arrived = 0;
      generation++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
};
static std::mutex g_groups_m;
static std::map<std::string, std::shared_ptr<LocalGroup>> g_groups;

struct pnp_ctx {
  std::string err;
  int device = 0;
  hipStream_t stream = nullptr;
  int rank = 0, nranks = 1;
  // the multi-rank code path (reduce -> allreduce -> derive, halo-split SpMV, two-reduction
  // BiCGSTAB): more than one rank, or one rank with an RCCL communicator of its own (a pnp_comm of
  // size 1 with an RCCL id -- the N > 1 path on one GPU, every allreduce a real ncclAllReduce)
  bool dist = false;
  ncclComm_t comm = nullptr;
  std::shared_ptr<LocalGroup> lg;  // test transport instead of RCCL
  pnp_host_transport ht{};         // host-staged transport (pnp_comm.host), if ht.exchange
  double *h_send = nullptr, *h_recv = nullptr, *h_red = nullptr;  // its pinned staging buffers
  size_t h_red_n = 0;
  bool host_tr() const { return ht.exchange != nullptr; }

  // P_k, k > 1 (pnp_create_pk): `mesh` is the node mesh (nv = Lagrange nodes, no elements) the
  // partition, layout and external vectors are built on; tmesh the triangle mesh, pks the space
  int degree = 1;
  pnp::Mesh mesh, tmesh;
  pnp::PkSpace pks;
  pnp::PkDev pkd;
  DBuf<int> pk_enode, pk_ioff, pk_icnt, pk_inc;
  DBuf<uint32_t> pk_islot;
  DBuf<double> pk_eres, pk_ejac;
  DBuf<int> pk_blk_short, pk_blk_long;
  pnp::Params params;
  pnp::Fans fans;
  pnp::LocalLayout L;
  pnp::DevLayout dl;

  DBuf<int> d_chunk_len, d_chunk_off, d_colidx, d_l2g, d_send_idx, d_color_idx;
  DBuf<uint8_t> d_rowcolor;
  DBuf<uint64_t> d_rowmeta;
  DBuf<int> d_uptr, d_ulist;   // LDS-staged SpMV lists (PNP_SPMV_LDS, DevLayout::uptr)
  DBuf<int> d_uown;            // per block: list entries before its own rows (DevLayout::uown)
  DBuf<int> d_lsx_ptr, d_lsx_list, d_usx_ptr, d_usx_list;  // LDS-staged sweeps (DevLayout lsx_*)
  DBuf<uint16_t> d_lsx_idx, d_usx_idx;
  DBuf<uint8_t> d_lperm, d_uperm, d_lpinv, d_upinv, d_llen, d_ulen, d_ldl;  // split lane order
  DBuf<uint16_t> d_lidx;
  DBuf<double> d_xy;

  // operator
  int kind = -1, nf = 0, pat = 0, nvb = 0, nks = 0;  // nvb: block pattern size, nks: stored
  std::vector<uint8_t> hmask;  // Dirichlet mask of the current operator, owned rows x nf
  pnp::AsmArgs aa{};
  DBuf<double> vals, lu;  // matrix and its ILU(0) factors
  bool lu_valid = false;
  // triangular split storage (DevLayout l*/u*): lvals/uvals hold either the matrix (SSOR) or the
  // ILU(0) factors; split_of says which is current (0 none, 1 matrix, 2 factors)
  DBuf<int> d_lchunk_len, d_lchunk_off, d_lcolidx, d_lsrc, d_uchunk_len, d_uchunk_off, d_ucolidx,
      d_usrc;
  DBuf<double> lvals, uvals, tsgs;
  int split_of = 0;
  // ILU(0) factors in the split storage in single precision (PNP_OPT_ILU_F32, default 1; the
  // sweeps compute in fp64, the matrix, SpMV, SSOR and every vector stay fp64).  Measured at
  // config 3: ILU(0) apply 119 -> 95 us, BiCGSTAB 428 -> 389 us/it, Newton 9,295 -> 9,177
  // iterations (profiles/r02/ab_ilu_f32.log)
  // 2 (the default since round 5): bfloat16 factors for block systems (linalg.hip bf16s: 14 B per
  // PNP block instead of 28 -- 16 B until ILU_BF16_B7; ILU(0) apply 66.3 -> 58.6 us, BiCGSTAB 0.285 -> 0.270 ms per
  // iteration at config 3, Newton counts inside their last-bit spread); scalar
  // systems (PB, Poisson, diffusion: one value per block, 2 B saved per slot) keep f32, where the
  // PB Newton at config 1 took 13 % more iterations with bf16
  // 3 (opt-in): the bf16 factors of 2, and the forward sweep's intermediate y = L^-1 d kept in
  // single precision (ilu_y32: 12 B per PNP row written, re-read by the backward sweep and gathered
  // by the forward one, instead of 24): apply 56.3 -> 54.5 us at config 3, but the rounding makes
  // the preconditioner nonlinear (2-5e-8 relative per application), which BiCGSTAB's short
  // recurrences do not tolerate: 408 -> 710 iterations on a config-5 solve, the config-5 Newton
  // and the config-4 AMG steps stall, so not the default.  The dataflow form (PNP_OPT_ILU_FLOW) keeps y in fp64 and runs
  // 3 as 2
  int ilu_f32 = [] {
    const char *e = std::getenv("PNP_ILU_F32");
    const int v = e ? std::atoi(e) : 2;
    return (v >= 0 && v <= 3) ? v : 2;
  }();
  int ilu_eff() const { return (ilu_f32 >= 2 && nf == 1) ? 1 : ilu_f32; }
  // the factors' storage: 0 fp64, 1 f32, 2 bf16 (the kernels' f32 argument)
  int ilu_fac() const { return ilu_eff() == 3 ? 2 : ilu_eff(); }
  int f32_now() const { return split_of == 2 ? ilu_fac() : 0; }
  // the single-precision forward intermediate of the colour launches, or null
  DBuf<float> ilu_y32buf;
  float *ilu_y32() const {
    return (split_of == 2 && ilu_eff() == 3 && !ilu_flow_opt) ? ilu_y32buf.p : nullptr;
  }
  int ilu_fused = 1;  // PNP_OPT_ILU_FUSED_FACTOR
  int amg_fallback = 0;  // PNP_OPT_AMG_FALLBACK
  int ilu_retry = 1;     // PNP_OPT_ILU_RETRY
  int twored_opt = [] {  // PNP_OPT_BICG_TWORED: -1 auto (on with more than one rank), 0, 1
    const char *ev = std::getenv("PNP_BICG_TWORED");
    return ev ? (std::atoi(ev) != 0 ? 1 : 0) : -1;
  }();
  DBuf<int> d_blkmap;
  DBuf<int> d_rowoff, d_rowcol;  // row-contiguous block offsets / columns (fused ILU(0) factor)
  // halo-overlapped SpMV (multi-GPU): 256-row blocks without / with ghost columns, each in the
  // spatial order of blkmap; the halo runs on cstream while the interior blocks compute
  DBuf<int> d_blk_int, d_blk_bnd;
  int n_blk_int = 0, n_blk_bnd = 0;
  bool split_spmv = false;
  pnp::DevLayout sub_layout(bool interior) const {
    pnp::DevLayout d = dl;
    d.blkmap = interior ? d_blk_int.p : d_blk_bnd.p;
    const int n = interior ? n_blk_int : n_blk_bnd;
    d.blkcount = n > 0 ? n : -1;  // -1: no block (launch nothing)
    return d;
  }
  hipStream_t cstream = nullptr;
  hipEvent_t ev_ready = nullptr, ev_halo = nullptr;
  DBuf<double> scrub;  // pnp_cache_scrub (cache-cold benchmark timings)
  // forward-difference Jacobian (PNP_JAC_FD, fd_jacobian.hip): local elements, per-row block
  // contribution lists, element matrices; built on first use
  bool fd_built = false, fd_mode = false;
  int fd_opt = 0;  // PNP_OPT_JAC_FD: every Jacobian assembly (Newton's too) by forward differences
  int fd_ne = 0;
  DBuf<int> fd_etri, fd_cdata;
  DBuf<long long> fd_rptr;
  DBuf<double> fd_jel;
  // device CSR view (pnp_jacobian_csr_device): structure per block pattern, values per request
  int csr_pat = -1, csr_nf = 0;
  long long csr_nnz = 0;
  DBuf<int> csr_rowptr, csr_col, csr_src;
  DBuf<unsigned char> csr_vidx;
  DBuf<double> csr_val;
  bool csr_vals_valid = false;  // csr_val holds the current Jacobian
  // natural-order SSOR (PNP_PREC_SSOR_NATURAL, ssor_natural.hip): level schedules of the forward
  // and backward sweeps over the external-layout rows with each level's rows as an ELL over the
  // CSR (pnp::NatSweep; built with the CSR structure), and external-layout work vectors
  struct NatDir {
    std::vector<int> lptr;
    std::vector<long long> eoff;
    DBuf<int4> info;
    DBuf<int> ecol;
    // the tail as chains (PNP_NAT_CHAIN): lane-group row lists, rows, padded entries
    bool chain_ok = false;
    int chain_groups = 0, chain_wpad = 0;
    DBuf<int> cgptr, cecode;
    DBuf<int4> crec;
    pnp::NatFlow::Chains chains() const {
      pnp::NatFlow::Chains c;
      if (!chain_ok) return c;
      c.ngroups = chain_groups;
      c.wpad = chain_wpad;
      c.gptr = cgptr.p;
      c.rec = crec.p;
      c.ecode = cecode.p;
      return c;
    }
    pnp::NatSweep view() const {
      pnp::NatSweep w;
      w.nlev = int(lptr.size()) - 1;
      w.lptr = lptr.data();
      w.eoff = eoff.data();
      w.info = info.p;
      w.ecol = ecol.p;
      return w;
    }
  };
  NatDir nat_f, nat_b;
  DBuf<double> nat_d, nat_v, nat_vf;  // external layout: d (level launches), vb, vf
  DBuf<double> nat_di, nat_vi;        // internal layout temporaries (reference-order mode)
  // the one-launch dataflow sweep (launch_ssor_natural_flow): units, forward units first
  std::vector<int4> nat_units;
  DBuf<int4> d_nat_units;
  int nat_units_f = 0, nat_tail_f = 0, nat_tail_b = 0, nat_max_width = 0;
  bool nat_units_ok = false;
  DBuf<unsigned> nat_abort;  // [0]: set by a sweep whose operand wait timed out (sticky)
  DBuf<int> csr_diag;        // index of each CSR-view row's diagonal entry
  // ILU(0) application as one dataflow launch (PNP_OPT_ILU_FLOW, linalg.hip k_ilu0_flow): per
  // c_first (0: every colour in the launch, 1: colour 0's forward step done by the update kernel)
  // the unit table and dependency lists, built on first use from the staging lists (host copies
  // kept from the layout build: rows at each L / U split position, lsx / usx lists)
  int ilu_flow_opt = [] {
    const char *e = std::getenv("PNP_ILU_FLOW");
    return (e && std::atoi(e) != 0) ? 1 : 0;
  }();
  std::vector<int> h_posrowL, h_posrowU, h_lsx_ptr, h_lsx_list, h_usx_ptr, h_usx_list;
  int64_t lslots_live = 0, uslots_live = 0;  // pnp_info
  struct IluFlowDev {
    bool built = false, ok = false;
    pnp::IluFlow F;
    DBuf<int> dep_ptr, dep_list;
    DBuf<unsigned> flags;
  };
  IluFlowDev ilu_flow[2];
  DBuf<unsigned> ilu_flow_abort;
  bool ilu_flow_used = false;  // a flow launch ran since the last check
  long long ilu_flow_n = 0;    // flow launches issued (pnp_info; a graph capture counts once)
  // ---- reference-order mode (PNP_OPT_SEQ_ORDER, seq_order.hip) -----------------------------
  int seq_opt = 0;
  bool seq_built = false, seq_op_valid = false;
  DBuf<int> seq_tri, seq_vptr, seq_vinc;
  DBuf<double> seq_xy;
  // the operator's data as the reference holds it: constrained rows (external layout), frozen
  // fields, x_old, implicit-Euler dt / valency (host copies taken by pnp_set_operator)
  std::vector<uint8_t> seq_mask_h;
  std::vector<double> seq_phi_h, seq_cp_h, seq_cm_h, seq_xold_h;
  double seq_dt = 0, seq_z = 0;
  bool seq_cextra = false;
  DBuf<unsigned char> seq_mask;
  DBuf<int> seq_bptr;
  DBuf<double> seq_bval, seq_phi, seq_cp, seq_cm, seq_xold;
  DBuf<double> seq_rl, seq_rlt, seq_rlo, seq_jl, seq_jlt, seq_vec, seq_dotv;
  int nat_pat = -1, nat_nf = 0;
  // ion-current observable (pnp_ion_flux): boundary segments handled by this rank (the owner of
  // the segment's lower global vertex), {a, c, opposite vertex, group} in local indices, in
  // global segment order
  DBuf<int4> d_fseg;
  std::vector<int> fseg_group;
  DBuf<double> fluxout, fluxx, fluxred;
  DBuf<uint8_t> dmask;
  DBuf<double> cvec, aux0, aux1;
  bool assembled = false;
  bool after_solve = false;  // a linear solve ran since the last Jacobian assembly (AsmArgs::cold)

  // aggregation AMG (PNP_PREC_AMG, amg.h): the pattern hierarchy is built once per context (it
  // depends on the layout only), the coarse values after every assembly
  pnp_amg_opts amg_opts{PNP_PREC_SSOR, pnp::kAmgMaxCoarse, 12, 0.8, 2, -1};
  bool amg_symmetric = true;  // set per solve: CG needs the symmetric V-cycle
  std::vector<pnp::AmgLevelHost> amg_h;
  struct AmgDev {
    int nb = 0;
    DBuf<int> rp, col, dpos, mptr, mem, agg, csrc;
    DBuf<long long> cptr;
    DBuf<double> v, dinv, b, x, x2;
    DBuf<float> vf;  // single-precision values for the V-cycle's sweeps (amg_f32; null: fp64)
  };
  // PNP_AMG_F32 (default 1): the coarse levels' sweeps and residuals read single-precision block
  // values, and the coarsest solve a single-precision copy of its inverse (the arithmetic, the
  // Galerkin products, the diagonal inverses and the LU / inverse themselves stay fp64), as the
  // ILU(0) factors do; 0 keeps fp64 (A/B)
  static bool amg_f32() {
    static const bool v = [] {
      const char *e = std::getenv("PNP_AMG_F32");
      return !(e && e[0] == '0');
    }();
    return v;
  }
  std::vector<std::unique_ptr<AmgDev>> amg_d;  // amg_d[k] = level k + 1
  bool amg_built = false, amg_valid = false;
  int amg_nf = 0;
  double amg_setup_ms = 0;
  DBuf<double> amg_ainv, amg_x0, amg_t, amg_y, amg_r, amg_z;
  DBuf<float> amg_ainv_f;  // amg_f32(): the inverse in single precision, rows padded to amg_ld
  int amg_ld = 0;
  DBuf<int> amg_ipiv, amg_info;
  rocblas_handle blas = nullptr;  // rocSOLVER getrf/getri of the AMG's coarsest level


  // vectors (sized n_local * 3)
  DBuf<double> x, r, rs, z, rt, p, v, t, y, y2, b, prevu, ext, sendbuf, partials, partials2;
  DBuf<double> redmw;  // the multi-workgroup reduction's ticket and slice sums (main stream only)
  std::vector<int> newton_its;        // pnp_newton_history: linear iterations per Newton step
  std::vector<double> newton_defects; // and the defect after each step
  DBuf<pnp::Scalars> S;
  pnp::Scalars *hS = nullptr;  // pinned host mirror

  // timers / debugging
  bool timing = false;
  bool debug_trace = [] {
    const char *e = std::getenv("PNP_DEBUG_BICGSTAB");
    return e && std::atoi(e) != 0;
  }();
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending[T_NCAT];
  std::vector<hipEvent_t> ev_pool;
  double t_ms[T_NCAT] = {0};
  long long t_n[T_NCAT] = {0};

  ~pnp_ctx() {
    graphs_clear();
    for (auto &v : ev_pending)
      for (auto &pr : v) {
        hipEventDestroy(pr.first);
        hipEventDestroy(pr.second);
      }
    for (auto e : ev_pool) hipEventDestroy(e);
    if (hS) hipHostFree(hS);
    if (h_send) hipHostFree(h_send);
    if (h_recv) hipHostFree(h_recv);
    if (h_red) hipHostFree(h_red);
    if (comm) ncclCommDestroy(comm);
    if (blas) rocblas_destroy_handle(blas);
    if (ev_ready) hipEventDestroy(ev_ready);
    if (ev_halo) hipEventDestroy(ev_halo);
    if (cstream) hipStreamDestroy(cstream);
    if (stream) hipStreamDestroy(stream);
  }

  // ---- hipGraph replay of BiCGSTAB iteration blocks (PNP_OPT_GRAPH) ------------------------------
  // -1 auto: on for up to 131,072 owned rows (launch-bound sizes), 0 off, 1 on
  int graph_opt = [] {
    const char *e = std::getenv("PNP_GRAPH");
    return e ? (std::atoi(e) != 0 ? 1 : 0) : -1;
  }();
  bool use_graphs() const {
    return graph_opt == 1 || (graph_opt < 0 && L.n_owned <= (1 << 17) && !profiled());
  }
  // rocprofv3 (ROCm 7.2) --kernel-trace dies with SIGSEGV once it has traced some 12,000-15,000
  // graph-launched kernels, whatever the graph (tools/micro/graph_capture_prof.hip):
  // under the profiler (its launcher exports ROCPROF_* variables) graph replay stays off unless
  // PNP_OPT_GRAPH forces it; the eager launches give the same results bit for bit
  static bool profiled() {
    static const bool p = [] {
      extern char **environ;
      for (char **e = environ; e && *e; e++)
        if (std::strncmp(*e, "ROCPROF_", 8) == 0) return true;
      return false;
    }();
    return p;
  }
  struct GraphKey {
    int count, prec, fuse, nf, pat, f32, flow;
    const void *zout, *dmask;
    long long epoch;
    bool operator==(const GraphKey &o) const {
      return count == o.count && prec == o.prec && fuse == o.fuse && nf == o.nf && pat == o.pat &&
             f32 == o.f32 && flow == o.flow && zout == o.zout && dmask == o.dmask &&
             epoch == o.epoch;
    }
  };
  // kernel arguments captured in a graph stay valid while the buffers and the layout do: anything
  // that changes an operator, an option or a buffer bumps the epoch
  long long graph_epoch = 0;
  bool graphs_failed = false;  // a capture / instantiation failed: eager launches from then on
  struct GraphSlot {
    GraphKey key;
    hipGraphExec_t exec = nullptr;
  };
  std::vector<GraphSlot> graph_cache;
  // the natural-order SSOR's level launches (ssor_natural.hip: ~2 x 131 levels per field sweep
  // at pore_pnp k=3) replayed as one graph: their arguments are context buffers only
  hipGraphExec_t nat_exec = nullptr;
  bool nat_graph_failed = false;
  void nat_graph_clear() {
    if (nat_exec) hipGraphExecDestroy(nat_exec);
    nat_exec = nullptr;
    nat_graph_failed = false;
  }
  void graphs_clear() {
    nat_graph_clear();
    for (auto &g : graph_cache)
      if (g.exec) hipGraphExecDestroy(g.exec);
    graph_cache.clear();
    graph_epoch++;
    graphs_failed = false;
  }
  // replay the launches `issue` makes on the stream as a graph (captured on first use of `key`)
  // *captured = false when the failure happened before any launch ran (capture / instantiate):
  // the caller can then run the same iterations eagerly
  template <typename F>
  int graph_run(const GraphKey &key, F &&issue, bool *captured = nullptr) {
    if (captured) *captured = true;
    for (auto &g : graph_cache)
      if (g.key == key) {
        hipError_t e = hipGraphLaunch(g.exec, stream);
        return e == hipSuccess ? PNP_OK : hipfail(e, "graph launch");
      }
    if (captured) *captured = false;
    hipError_t e = hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) return hipfail(e, "graph capture");
    const int rc = issue();
    hipGraph_t graph = nullptr;
    hipError_t e2 = hipStreamEndCapture(stream, &graph);
    if (rc) {
      if (graph) hipGraphDestroy(graph);
      return rc;
    }
    if (e2 != hipSuccess) return hipfail(e2, "graph capture");
    hipGraphExec_t exec = nullptr;
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    hipGraphDestroy(graph);
    if (e != hipSuccess) return hipfail(e, "graph instantiate");
    if (captured) *captured = true;
    if (graph_cache.size() >= 8) {
      hipGraphExecDestroy(graph_cache.front().exec);
      graph_cache.erase(graph_cache.begin());
    }
    graph_cache.push_back({key, exec});
    e = hipGraphLaunch(exec, stream);
    return e == hipSuccess ? PNP_OK : hipfail(e, "graph launch");
  }

  int fail(int code, const std::string &msg) {
    err = msg;
    return code;
  }
  int hipfail(hipError_t e, const char *what) {
    err = std::string(what) + ": " + hipGetErrorString(e);
    return PNP_E_HIP;
  }

  // ---- timers -------------------------------------------------------------------------------
  hipEvent_t ev_get() {
    if (!ev_pool.empty()) {
      hipEvent_t e = ev_pool.back();
      ev_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
  }
  hipEvent_t tb(int cat) {
    if (!timing) return nullptr;
    hipEvent_t e = ev_get();
    hipEventRecord(e, stream);
    (void)cat;
    return e;
  }
  void te(int cat, hipEvent_t start) {
    if (!timing || !start) return;
    hipEvent_t e = ev_get();
    hipEventRecord(e, stream);
    ev_pending[cat].push_back({start, e});
    t_n[cat]++;
  }
  void timers_flush() {
    hipStreamSynchronize(stream);
    for (int c = 0; c < T_NCAT; c++) {
      for (auto &pr : ev_pending[c]) {
        float ms = 0;
        hipEventElapsedTime(&ms, pr.first, pr.second);
        t_ms[c] += ms;
        ev_pool.push_back(pr.first);
        ev_pool.push_back(pr.second);
      }
      ev_pending[c].clear();
    }
  }

  // ---- helpers ------------------------------------------------------------------------------
  long long nown() const { return (long long)L.n_owned * nf; }

  int halo(double *vec, int nfv) { return halo_on(vec, nfv, stream); }

  int halo_on(double *vec, int nfv, hipStream_t hs) {
    if (nranks == 1) return PNP_OK;
    if (lg) return halo_local(vec, nfv);
    if (host_tr()) return halo_host(vec, nfv);
    if (L.nbr_ranks.empty()) return PNP_OK;
    hipEvent_t t0 = hs == stream ? tb(T_HALO) : nullptr;
    int ns = int(L.send_idx.size());
    hipError_t e = pnp::launch_pack(ns, nfv, d_send_idx.p, vec, sendbuf.p, hs);
    if (e != hipSuccess) return hipfail(e, "halo pack");
    if (ncclGroupStart() != ncclSuccess) return fail(PNP_E_RCCL, "ncclGroupStart");
    for (size_t q = 0; q < L.nbr_ranks.size(); q++) {
      int peer = L.nbr_ranks[q];
      size_t sc = size_t(L.send_ptr[q + 1] - L.send_ptr[q]) * nfv;
      size_t rc = size_t(L.recv_ptr[q + 1] - L.recv_ptr[q]) * nfv;
      if (ncclSend(sendbuf.p + size_t(L.send_ptr[q]) * nfv, sc, ncclDouble, peer, comm, hs) !=
          ncclSuccess)
        return fail(PNP_E_RCCL, "ncclSend");
      if (ncclRecv(vec + (size_t(L.n_owned) + L.recv_ptr[q]) * nfv, rc, ncclDouble, peer, comm,
                   hs) != ncclSuccess)
        return fail(PNP_E_RCCL, "ncclRecv");
    }
    if (ncclGroupEnd() != ncclSuccess) return fail(PNP_E_RCCL, "ncclGroupEnd");
    if (t0) te(T_HALO, t0);
    return PNP_OK;
  }

  // halo exchange of vin's ghosts + y = A vin (mode / dots as launch_spmv).  Multi-GPU with the
  // split layout: the interior blocks (no ghost columns) run while the halo is in flight on
  // cstream, then the boundary blocks; their partials follow each other, *nsp counts both.
  int halo_spmv(double *vin, double *yout, int mode, const double *w, const double *w2, int *nsp) {
    hipError_t e;
    if (!split_spmv) {
      int rc = halo(vin, nf);
      if (rc) return rc;
      // the launch records the timer events itself (the kernel's own duration)
      hipEvent_t t0 = nullptr, t1 = nullptr;
      if (timing && L.n_owned > 0) {
        t0 = ev_get();
        t1 = ev_get();
      }
      e = pnp::launch_spmv(dl, nf, pat, vals.p, vin, yout, mode, w, partials.p, nsp, stream, w2,
                           t0, t1);
      if (e != hipSuccess) return hipfail(e, "spmv");
      if (t1) {
        ev_pending[T_SPMV].push_back({t0, t1});
        t_n[T_SPMV]++;
      }
      return PNP_OK;
    }
    const int kd = mode == 4 ? 3 : (mode == 2 ? 2 : 1);
    const pnp::DevLayout dl_int = sub_layout(true), dl_bnd = sub_layout(false);
    int n1 = 0, n2 = 0, rc;
    if (lg || host_tr()) {  // in-process / host-staged transport: synchronous halo between the halves
      hipEvent_t t0 = tb(T_SPMV);
      e = pnp::launch_spmv(dl_int, nf, pat, vals.p, vin, yout, mode, w, partials.p, &n1, stream, w2);
      if (e != hipSuccess) return hipfail(e, "spmv interior");
      te(T_SPMV, t0);
      if ((rc = halo(vin, nf))) return rc;
    } else {
      if ((e = hipEventRecord(ev_ready, stream)) != hipSuccess ||
          (e = hipStreamWaitEvent(cstream, ev_ready, 0)) != hipSuccess)
        return hipfail(e, "halo stream order");
      if ((rc = halo_on(vin, nf, cstream))) return rc;
      if ((e = hipEventRecord(ev_halo, cstream)) != hipSuccess) return hipfail(e, "halo event");
      hipEvent_t t0 = tb(T_SPMV);
      e = pnp::launch_spmv(dl_int, nf, pat, vals.p, vin, yout, mode, w, partials.p, &n1, stream, w2);
      if (e != hipSuccess) return hipfail(e, "spmv interior");
      te(T_SPMV, t0);
      if ((e = hipStreamWaitEvent(stream, ev_halo, 0)) != hipSuccess)
        return hipfail(e, "halo wait");
    }
    hipEvent_t t1 = tb(T_SPMV);
    e = pnp::launch_spmv(dl_bnd, nf, pat, vals.p, vin, yout, mode, w, partials.p + size_t(n1) * kd,
                         &n2, stream, w2);
    if (e != hipSuccess) return hipfail(e, "spmv boundary");
    te(T_SPMV, t1);
    *nsp = n1 + n2;
    return PNP_OK;
  }

  // host-staged halo: pack on the device, copy to pinned host memory, the caller's exchange, copy
  // the received ghosts back (synchronous, on the context's stream)
  int halo_host(double *vec, int nfv) {
    hipEvent_t t0 = tb(T_HALO);
    const int ns = int(L.send_idx.size()), nq = int(L.nbr_ranks.size());
    const size_t nsend = size_t(ns) * nfv, nrecv = size_t(L.n_ghost) * nfv;
    hipError_t e = pnp::launch_pack(ns, nfv, d_send_idx.p, vec, sendbuf.p, stream);
    if (e == hipSuccess && nsend)
      e = hipMemcpyAsync(h_send, sendbuf.p, sizeof(double) * nsend, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "halo pack");
    std::vector<int64_t> soff(nq), scnt(nq), roff(nq), rcnt(nq);
    for (int q = 0; q < nq; q++) {
      soff[q] = int64_t(L.send_ptr[q]) * nfv;
      scnt[q] = int64_t(L.send_ptr[q + 1] - L.send_ptr[q]) * nfv;
      roff[q] = int64_t(L.recv_ptr[q]) * nfv;
      rcnt[q] = int64_t(L.recv_ptr[q + 1] - L.recv_ptr[q]) * nfv;
    }
    if (ht.exchange(ht.user, nq, L.nbr_ranks.data(), h_send, soff.data(), scnt.data(), h_recv,
                    roff.data(), rcnt.data()) != 0)
      return fail(PNP_E_RCCL, "host transport: exchange failed");
    if (nrecv)
      e = hipMemcpyAsync(vec + size_t(L.n_owned) * nfv, h_recv, sizeof(double) * nrecv,
                         hipMemcpyHostToDevice, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);  // h_recv is reused by the next call
    if (e != hipSuccess) return hipfail(e, "halo copy");
    if (t0) te(T_HALO, t0);
    return PNP_OK;
  }

  int halo_local(double *vec, int nfv) {
    int ns = int(L.send_idx.size());
    hipError_t e = pnp::launch_pack(ns, nfv, d_send_idx.p, vec, sendbuf.p, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "halo pack");
    lg->barrier();  // every rank has packed
    for (size_t q = 0; q < L.nbr_ranks.size(); q++) {
      pnp_ctx *peer = lg->members[L.nbr_ranks[q]];
      const pnp::LocalLayout &PL = peer->L;
      size_t k = 0;
      while (k < PL.nbr_ranks.size() && PL.nbr_ranks[k] != rank) k++;
      if (k == PL.nbr_ranks.size()) return fail(PNP_E_STATE, "asymmetric halo");
      size_t cnt = size_t(L.recv_ptr[q + 1] - L.recv_ptr[q]) * nfv;
      if (cnt != size_t(PL.send_ptr[k + 1] - PL.send_ptr[k]) * nfv)
        return fail(PNP_E_STATE, "halo size mismatch");
      e = hipMemcpyAsync(vec + (size_t(L.n_owned) + L.recv_ptr[q]) * nfv,
                         peer->sendbuf.p + size_t(PL.send_ptr[k]) * nfv, sizeof(double) * cnt,
                         hipMemcpyDeviceToDevice, stream);
      if (e != hipSuccess) return hipfail(e, "halo copy");
    }
    e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "halo copy");
    lg->barrier();  // nobody repacks before every copy out of the send buffers is done
    return PNP_OK;
  }

  // in-place sum over ranks of k doubles in device memory
  int allreduce_dev(double *d, int k) {
    if (!dist) return PNP_OK;
    if (lg) {
      std::vector<double> h(k);
      hipError_t e = hipMemcpyAsync(h.data(), d, sizeof(double) * k, hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      if (e != hipSuccess) return hipfail(e, "allreduce");
      lg->host[rank] = h;
      lg->barrier();
      std::vector<double> sum(k, 0.0);
      for (int r = 0; r < nranks; r++)  // fixed rank order: deterministic
        for (int j = 0; j < k; j++) sum[j] += lg->host[r][j];
      lg->barrier();
      e = hipMemcpyAsync(d, sum.data(), sizeof(double) * k, hipMemcpyHostToDevice, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      return e == hipSuccess ? PNP_OK : hipfail(e, "allreduce");
    }
    if (host_tr()) {
      if (size_t(k) > h_red_n) {
        if (h_red) hipHostFree(h_red);
        h_red = nullptr;
        h_red_n = 0;
        hipError_t e = hipHostMalloc(&h_red, sizeof(double) * size_t(k));
        if (e != hipSuccess) return hipfail(e, "allreduce staging");
        h_red_n = size_t(k);
      }
      hipError_t e = hipMemcpyAsync(h_red, d, sizeof(double) * k, hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      if (e != hipSuccess) return hipfail(e, "allreduce");
      if (ht.allreduce_sum(ht.user, h_red, k) != 0)
        return fail(PNP_E_RCCL, "host transport: allreduce failed");
      e = hipMemcpyAsync(d, h_red, sizeof(double) * k, hipMemcpyHostToDevice, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      return e == hipSuccess ? PNP_OK : hipfail(e, "allreduce");
    }
    ncclResult_t nr = ncclAllReduce(d, d, k, ncclDouble, ncclSum, comm, stream);
    if (nr != ncclSuccess)
      return fail(PNP_E_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(nr));
    return PNP_OK;
  }

  int allreduce_red(int k) {
    if (!dist) return PNP_OK;
    hipEvent_t t0 = tb(T_ALLRED);
    double *red = reinterpret_cast<double *>(reinterpret_cast<char *>(S.p) +
                                             offsetof(pnp::Scalars, red));
    int rc = allreduce_dev(red, k);
    if (rc) return rc;
    te(T_ALLRED, t0);
    return PNP_OK;
  }

  // S->red = sum of partials (all ranks), then the derive step of BiCGSTAB stage `stage`
  int reduce_derive(int np, int k, int stage, bool from2 = false) {
    hipError_t e;
    const double *src = from2 ? partials2.p : partials.p;
    if (!dist) {
      e = pnp::launch_reduce(src, np, k, S.p, stream, stage, redmw.p);
      return e == hipSuccess ? PNP_OK : hipfail(e, "reduce");
    }
    e = pnp::launch_reduce(src, np, k, S.p, stream, -1, redmw.p);
    if (e != hipSuccess) return hipfail(e, "reduce");
    int rc = allreduce_red(k);
    if (rc) return rc;
    e = pnp::launch_derive(S.p, stage, stream);
    return e == hipSuccess ? PNP_OK : hipfail(e, "derive");
  }

  // S->red[0..ka) = sum of partials (spmv), S->red[ka..) = sum of partials2, all ranks; derive
  int reduce_derive2(int npa, int ka, int npb, int kb, int stage) {
    hipError_t e;
    if (!dist) {
      e = pnp::launch_reduce2(partials.p, npa, ka, partials2.p, npb, kb, S.p, stream, stage,
                              redmw.p);
      return e == hipSuccess ? PNP_OK : hipfail(e, "reduce");
    }
    e = pnp::launch_reduce2(partials.p, npa, ka, partials2.p, npb, kb, S.p, stream, -1, redmw.p);
    if (e != hipSuccess) return hipfail(e, "reduce");
    int rc = allreduce_red(ka + kb);
    if (rc) return rc;
    e = pnp::launch_derive(S.p, stage, stream);
    return e == hipSuccess ? PNP_OK : hipfail(e, "derive");
  }

  // norm over owned rows of a vector, synchronous
  int norm(const double *vec, double &out) {
    hipEvent_t t0 = tb(T_BLAS);
    hipError_t e = pnp::launch_dot(nown(), vec, vec, 0, partials.p, stream);
    if (e == hipSuccess) {
      // reduce through the scalar block without touching the BiCGSTAB state: use a scratch
      // Scalars at S.p + 1
      e = pnp::launch_reduce(partials.p, pnp::blas_nparts(nown()), 1, S.p + 1, stream);
    }
    if (e != hipSuccess) return hipfail(e, "norm");
    te(T_BLAS, t0);
    if (dist) {
      double *red = reinterpret_cast<double *>(reinterpret_cast<char *>(S.p + 1) +
                                               offsetof(pnp::Scalars, red));
      int rc = allreduce_dev(red, 1);
      if (rc) return rc;
    }
    e = hipMemcpyAsync(hS + 1, S.p + 1, sizeof(pnp::Scalars), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "norm readback");
    out = std::sqrt(hS[1].red[0]);
    return PNP_OK;
  }

  // external (lexicographic, global) vector -> the internal layout; devptr: `host` is a device
  // pointer (PNP_DEVICE_PTRS), gathered from directly
  int upload_ext(const double *host, int nfv, double *dev, bool with_ghosts, bool devptr = false) {
    size_t ne = size_t(mesh.nv) * nfv;
    hipError_t e = hipSuccess;
    if (!devptr)
      e = hipMemcpyAsync(ext.p, host, sizeof(double) * ne, hipMemcpyHostToDevice, stream);
    if (e == hipSuccess)
      e = pnp::launch_gather_ext(with_ghosts ? L.n_owned + L.n_ghost : L.n_owned, nfv, mesh.nv,
                                 d_l2g.p, devptr ? host : ext.p, dev, stream);
    if (e != hipSuccess) return hipfail(e, "upload");
    return PNP_OK;
  }

  // internal -> external; this rank's owned entries are written (devptr: into device memory,
  // synchronised before return)
  int download_ext(const double *dev, int nfv, double *host, bool devptr = false) {
    if (devptr) {
      hipError_t e = pnp::launch_scatter_ext(L.n_owned, nfv, mesh.nv, d_l2g.p, dev, host, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      return e == hipSuccess ? PNP_OK : hipfail(e, "download");
    }
    size_t ne = size_t(mesh.nv) * nfv;
    hipError_t e = pnp::launch_scatter_ext(L.n_owned, nfv, mesh.nv, d_l2g.p, dev, ext.p, stream);
    std::vector<double> tmp(ne);
    if (e == hipSuccess)
      e = hipMemcpyAsync(tmp.data(), ext.p, sizeof(double) * ne, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "download");
    for (int i = 0; i < L.n_owned; i++) {
      int g = L.l2g[i];
      for (int f = 0; f < nfv; f++) host[size_t(f) * mesh.nv + g] = tmp[size_t(f) * mesh.nv + g];
    }
    return PNP_OK;
  }

  int assemble(const double *xdev, int jac) {
    if (kind < 0) return fail(PNP_E_STATE, "no operator set (pnp_set_operator)");
    int rc;
    if (jac && (rc = set_fd(fd_opt != 0))) return rc;
    aa.x = xdev;
    aa.jac = fd_mode ? 0 : jac;
    aa.r = r.p;
    aa.cold = after_solve ? 1 : 0;
    // the P1 analytic assembly is one launch: it records its own start / end events (the
    // kernel's duration, as the kernel trace reports it); the other forms take an event pair
    const bool one = degree == 1 && !(jac && fd_mode);
    hipEvent_t t0 = nullptr, t1 = nullptr;
    if (timing && one) {
      t0 = ev_get();
      t1 = ev_get();
    } else {
      t0 = tb(T_ASM);
    }
    hipError_t e;
    if (degree > 1)
      e = pnp::launch_pk_assemble(dl, aa, pkd, jac ? (fd_mode ? 2 : 1) : 0, stream);
    else
      e = pnp::launch_assemble(dl, aa, stream, t1 ? t0 : nullptr, t1);
    if (e == hipSuccess && jac && fd_mode && degree == 1)
      e = pnp::launch_fd_jacobian(dl, aa, nf, pat, fd_ne, fd_etri.p, fd_rptr.p, fd_cdata.p,
                                  fd_jel.p, stream);
    if (e != hipSuccess) return hipfail(e, "assemble");
    if (t1) {
      ev_pending[T_ASM].push_back({t0, t1});
      t_n[T_ASM]++;
    } else {
      te(T_ASM, t0);
    }
    if (jac) {
      assembled = true;
      lu_valid = false;
      split_of = 0;
      amg_valid = false;
      csr_vals_valid = false;
      after_solve = false;
    }
    return PNP_OK;
  }

  // structure of the external-layout CSR view of the current block pattern (host, once per
  // pattern): rows f*nv + g of the owned vertices, columns sorted; per entry the source block
  // (row << 6 | slot) and the value's index in the block pattern.  Also the natural-order SSOR
  // level schedule over these rows.
  int csr_structure() {
    const int nv = mesh.nv, mask = pat & 0x1FF;
    if (csr_pat == mask && csr_nf == nf) return PNP_OK;
    // the BiCGSTAB block graphs captured with SSOR_NATURAL hold csr_val, nat_d / nat_v and the level
    // buffers, all rebuilt below: drop every graph (bumps graph_epoch, part of GraphKey)
    graphs_clear();
    const int n = nf * nv;
    std::vector<int> cnt(n + 1, 0);
    for (int i = 0; i < L.n_owned; i++) {
      const int len = pnp::meta_len(L.rowmeta[i]);
      for (int f = 0; f < nf; f++) {
        int k = 0;
        for (int g = 0; g < nf; g++) k += pnp::pat_index(mask, f, g) >= 0;
        cnt[f * nv + L.l2g[i] + 1] += k * len;
      }
    }
    for (int i = 0; i < n; i++) cnt[i + 1] += cnt[i];
    const long long nnz = cnt[n];
    std::vector<int> col(nnz), src(nnz);
    std::vector<unsigned char> vid(nnz);
    struct E {
      int col, src;
      unsigned char v;
    };
    std::vector<E> tmp;
    for (int i = 0; i < L.n_owned; i++) {
      const int chunk = i / pnp::kRows, lane = i % pnp::kRows, len = pnp::meta_len(L.rowmeta[i]);
      for (int f = 0; f < nf; f++) {
        tmp.clear();
        for (int sl = 0; sl < len; sl++) {
          const int j = L.colidx[size_t(L.chunk_off[chunk]) + size_t(sl) * pnp::kRows + lane];
          for (int g = 0; g < nf; g++) {
            const int v = pnp::pat_index(mask, f, g);
            if (v >= 0) tmp.push_back({g * nv + L.l2g[j], i << 6 | sl, (unsigned char)v});
          }
        }
        std::sort(tmp.begin(), tmp.end(), [](const E &a, const E &b) { return a.col < b.col; });
        long long q = cnt[f * nv + L.l2g[i]];
        for (const E &e : tmp) {
          col[q] = e.col;
          src[q] = e.src;
          vid[q] = e.v;
          q++;
        }
      }
    }
    int rc;
    if ((rc = upv(csr_rowptr, cnt, "csr rowptr")) || (rc = upv(csr_col, col, "csr col")) ||
        (rc = upv(csr_src, src, "csr src")) || (rc = upv(csr_vidx, vid, "csr vidx")))
      return rc;
    hipError_t e = csr_val.alloc(std::max<long long>(1, nnz));
    if (e != hipSuccess) return hipfail(e, "csr values");
    // natural-order SSOR schedule.  A row R must run after every row it shares a matrix entry with
    // (A_RC or A_CR stored) that comes before it in the sweep, and before every such later row:
    // level(R) = 1 + max level of its earlier partners, computed in sweep order with the partners
    // of the transposed entries pushed forward.  Rows of other ranks' vertices are empty and stay
    // out (their columns read zero).
    auto empty = [&](int R) { return cnt[R] == cnt[R + 1]; };
    std::vector<int> diag(n, -1);
    for (int R = 0; R < n; R++)
      for (int k = cnt[R]; k < cnt[R + 1]; k++)
        if (col[k] == R) diag[R] = k;
    for (int R = 0; R < n; R++)
      if (!empty(R) && diag[R] < 0) return fail(PNP_E_STATE, "natural SSOR: row without diagonal");
    if ((rc = upv(csr_diag, diag, "csr diagonal"))) return rc;
    // the dataflow sweeps keep their results and operands in the external (lexicographic) layout
    // R = f * nv + g, which is local in the sweep order (indexing them by internal position
    // instead made the PNP heads 10-16 % slower, profiles/r05/nat_split_r5e.txt), but read d at
    // the row's INTERNAL position g2l[g] * nf + f (info.w / rec.w), so that the preconditioner's
    // input needs no scatter into an external copy (PNP config 3: 20 us per application,
    // profiles/r05/nat_split_r5d.txt); the result is gathered out of vb afterwards
    auto P = [&](int R) { return L.g2l[R % nv] * nf + R / nv; };
    // NatSweep::info packs a row's entry count and its diagonal's offset into one int as
    // len | offset << 8 (the kernels decode len & 255): at most 255 entries per row (P1 PNP rows
    // have <= 3 * 21); a wider pattern would corrupt both, so refuse it here
    for (int R = 0; R < n; R++)
      if (cnt[R + 1] - cnt[R] > 255)
        return fail(PNP_E_STATE, "natural SSOR: a row has more than 255 CSR entries (row " +
                                     std::to_string(R) + ")");
    auto schedule = [&](bool fwd, NatDir &W) -> int {
      std::vector<int> &lptr = W.lptr;
      std::vector<int> lev(n, -1), push(n, 0);
      int nlev = 0;
      for (int s = 0; s < n; s++) {
        const int R = fwd ? s : n - 1 - s;
        if (empty(R)) continue;
        int l = push[R];
        for (int k = cnt[R]; k < cnt[R + 1]; k++) {
          const int C = col[k];
          if (C != R && (fwd ? C < R : C > R) && !empty(C)) l = std::max(l, lev[C] + 1);
        }
        lev[R] = l;
        nlev = std::max(nlev, l + 1);
        for (int k = cnt[R]; k < cnt[R + 1]; k++) {
          const int C = col[k];
          if (C != R && (fwd ? C > R : C < R) && !empty(C)) push[C] = std::max(push[C], l + 1);
        }
      }
      lptr.assign(nlev + 1, 0);
      for (int R = 0; R < n; R++)
        if (lev[R] >= 0) lptr[lev[R] + 1]++;
      for (int l = 0; l < nlev; l++) lptr[l + 1] += lptr[l];
      std::vector<int> fill(lptr.begin(), lptr.end() - 1), rl(std::max(1, lptr[nlev]));
      for (int R = 0; R < n; R++)
        if (lev[R] >= 0) rl[fill[lev[R]]++] = R;
      // per level an ELL of its rows' entries (CSR order), width = its longest row, padding
      // slots with value index -1, stored unit by unit: the level's rows in groups of UR (the
      // dataflow units), each group's entries k-major, entry k of the group's row r at
      // (group * width + k) * UR + r.  A unit's slots are then one contiguous run of lines that no
      // other unit touches (column-major over the whole level, 4 units shared every line of a
      // slot, fetched once per XCD that ran one of them: the PNP head missed L2 ~16.7 M times per
      // launch, profiles/r05/nat_pmc_mem_r5a.json)
      const int UR = pnp::ssor_natural_unit_rows();
      std::vector<int4> info(std::max(1, lptr[nlev]));
      std::vector<int> lwidth(nlev, 0);
      W.eoff.assign(nlev + 1, 0);
      for (int l = 0; l < nlev; l++) {
        int w = 0;
        for (int t = lptr[l]; t < lptr[l + 1]; t++) w = std::max(w, cnt[rl[t] + 1] - cnt[rl[t]]);
        lwidth[l] = w;
        W.eoff[l + 1] = W.eoff[l] + (long long)w * UR * ((lptr[l + 1] - lptr[l] + UR - 1) / UR);
      }
      // operand codes (NatSweep): the forward sweep reads the new value of an earlier row (C < R)
      // and zero for the row itself and later rows; the backward sweep reads the forward value of
      // rows C <= R and the new backward value of later rows; rows of other ranks read zero
      std::vector<int> ecol(std::max<long long>(1, W.eoff[nlev]), -1);
      for (int l = 0; l < nlev; l++) {
        for (int t = lptr[l]; t < lptr[l + 1]; t++) {
          const int R = rl[t], len = cnt[R + 1] - cnt[R], tl = t - lptr[l];
          info[t] = make_int4(R, len | (diag[R] - cnt[R]) << 8, cnt[R], P(R));
          for (int k = 0; k < len; k++) {
            const size_t q =
                size_t(W.eoff[l]) + (size_t(tl / UR) * lwidth[l] + k) * UR + size_t(tl % UR);
            const int C = col[cnt[R] + k];
            ecol[q] = empty(C) ? -1 : fwd ? (C < R ? C : -1) : (C <= R ? C : -(C + 2));
          }
        }
      }
      // dataflow units for the one-launch sweep: up to ssor_natural_unit_rows() consecutive rows of one level,
      // {first sweep position, rows | width << 8, the ELL stride between a row's entries (UR), ELL
      // index of the unit's first row}; forward units in level order, then backward units in level
      // order.  The
      // sweep's tail -- the levels from the last one wider than PNP_NAT_TAIL rows to its end --
      // can run in one workgroup (ssor_natural.hip); default 0 (no tail): one CU is slower
      // (PNP config 3: 2.36 ms per application without, 3.29 / 4.83 ms with 512 / 1024-row tails,
      // profiles/r04/ssor_natural_tail_r4e.log)
      static const int tail_rows = [] {
        const char *ev = std::getenv("PNP_NAT_TAIL");
        return ev ? std::max(0, std::atoi(ev)) : 0;
      }();
      // PNP_NAT_CHAIN (rows): the tail as chains (k_ssor_nat_chain; takes precedence over
      // PNP_NAT_TAIL).  Default: the levels of at most as many rows as the chain kernel keeps
      // groups resident (8,192 on MI355X), so that no two chains share a group at one level
      // (pore_pnp k=4 per application, PB 1.31 -> 0.57 ms, PNP config 3 2.22 -> 1.57 ms;
      // threshold sweep profiles/r04/chain2/).  PNP_NAT_CHAIN=0: dataflow units only
      static const int chain_rows = [] {
        const char *ev = std::getenv("PNP_NAT_CHAIN");
        return ev ? std::max(0, std::atoi(ev)) : std::max(0, pnp::ssor_natural_chain_capacity());
      }();
      const int trows = chain_rows > 0 ? chain_rows : tail_rows;
      int ltail = nlev;
      while (trows > 0 && ltail > 0 && lptr[ltail] - lptr[ltail - 1] <= trows) ltail--;
      W.chain_ok = false;
      if (chain_rows > 0 && ltail < nlev) {
        // heavy-path chains of the tail: parent = the first dependency on the level just before
        // (inside the tail); each row continues the chain of its child with the longest path
        // below it; chains packed into lane groups by level interval (greedy, by start level)
        const int t0 = lptr[ltail], t1 = lptr[nlev];
        auto isdep = [&](int R, int C) {
          return C != R && !empty(C) && (fwd ? C < R : C > R);
        };
        std::vector<int> parent(n, -1), heavy(n, -1), hbest(n, 0);
        int wmax = 0;
        for (int t = t0; t < t1; t++) {
          const int R = rl[t];
          wmax = std::max(wmax, cnt[R + 1] - cnt[R]);
          for (int k = cnt[R]; k < cnt[R + 1]; k++) {
            const int C = col[k];
            if (isdep(R, C) && lev[C] == lev[R] - 1 && lev[C] >= ltail) {
              parent[R] = C;
              break;
            }
          }
        }
        for (int t = t1 - 1; t >= t0; t--) {  // decreasing level
          const int R = rl[t], P = parent[R], h = 1 + hbest[R];
          if (P >= 0 && h > hbest[P]) {
            hbest[P] = h;
            heavy[P] = R;
          }
        }
        // at most the grid's resident lane groups (the kernel's progress needs them all
        // resident): past that, a chain shares the group that frees first, its rows interleaved
        // by level (a row whose parent is not the group's previous row reads it from memory)
        const int gcap = std::max(1, pnp::ssor_natural_chain_capacity());
        std::vector<std::vector<int>> grows;
        std::priority_queue<std::pair<int, int>, std::vector<std::pair<int, int>>,
                            std::greater<std::pair<int, int>>> freeq;  // (end level, group)
        bool shared = false;
        long long rr = 0;  // over the cap: chains dealt round-robin (a balanced share per group)
        std::vector<int> gend;  // each group's last level; heap entries that disagree are stale
        for (int t = t0; t < t1; t++) {
          const int R = rl[t];
          if (parent[R] >= 0 && heavy[parent[R]] == R) continue;  // inside a chain
          while (!freeq.empty() && freeq.top().first != gend[freeq.top().second]) freeq.pop();
          int g;
          if (!freeq.empty() && freeq.top().first < lev[R]) {
            g = freeq.top().second;
            freeq.pop();
          } else if (int(grows.size()) >= gcap) {
            g = int(rr++ % gcap);
            shared = true;
          } else {
            g = int(grows.size());
            grows.emplace_back();
            gend.push_back(-1);
          }
          int X = R, last = lev[R];
          for (; X >= 0; X = heavy[X]) {
            grows[g].push_back(X);
            last = lev[X];
          }
          gend[g] = std::max(gend[g], last);
          freeq.push({gend[g], g});
        }
        if (shared)  // every group's rows in level order (stable: a chain's rows stay in order)
          for (auto &G : grows)
            std::stable_sort(G.begin(), G.end(), [&](int a, int b) { return lev[a] < lev[b]; });
        const int wpad = wmax;
        if (wpad <= pnp::ssor_natural_chain_width()) {
          std::vector<int> gptr(1, 0), ecode;
          std::vector<int4> rec;
          for (const auto &G : grows) {
            const int H = pnp::ssor_natural_chain_history();
            for (size_t t = 0; t < G.size(); t++) {
              const int R = G[t];
              const int len = cnt[R + 1] - cnt[R];
              rec.push_back(make_int4(R, len | (diag[R] - cnt[R]) << 8, cnt[R], P(R)));
              for (int k = 0; k < wpad; k++) {
                if (k < len) {
                  const int C = col[cnt[R] + k];
                  const int fc = empty(C) ? -1 : fwd ? (C < R ? C : -1) : (C <= R ? C : -(C + 2));
                  // kind: 0 zero, 1 forward value, 2 backward value, 3 in the wave's registers
                  int code = fc == -1 ? 0 : fc >= 0 ? (fc << 2 | 1) : ((-(fc + 2)) << 2 | 2);
                  const bool fresh = fwd ? (code & 3) == 1 : (code & 3) == 2;  // this sweep's value
                  for (int h = 1; fresh && h <= H && size_t(h) <= t; h++)
                    if (G[t - h] == C) {
                      code = h << 2 | 3;
                      break;
                    }
                  ecode.push_back(code);
                } else {
                  ecode.push_back(0);
                }
              }
            }
            gptr.push_back(int(rec.size()));
          }
          int rc2;
          if ((rc2 = upv(W.cgptr, gptr, "natural SSOR chains")) ||
              (rc2 = upv(W.crec, rec, "natural SSOR chains")) ||
              (rc2 = upv(W.cecode, ecode, "natural SSOR chains")))
            return rc2;
          W.chain_groups = int(grows.size());
          W.chain_wpad = wpad;
          W.chain_ok = true;
        }
      }
      if (chain_rows > 0 && !W.chain_ok) {
        // no chains (rows wider than the chain kernel takes): the tail is PNP_NAT_TAIL's again
        // (default none), not the chain threshold's -- a one-workgroup tail of ~8K rows would run
        // every narrow level on one CU
        ltail = nlev;
        while (tail_rows > 0 && ltail > 0 && lptr[ltail] - lptr[ltail - 1] <= tail_rows) ltail--;
      }
      for (int l = 0; l < nlev && nat_units_ok; l++) {
        if (l == ltail) (fwd ? nat_tail_f : nat_tail_b) = int(nat_units.size());
        const long long w = lwidth[l];
        for (int t0 = lptr[l]; t0 < lptr[l + 1]; t0 += UR) {
          const long long e0 = W.eoff[l] + (t0 - lptr[l]) / UR * w * UR;
          if (w > 255 || W.eoff[l + 1] > INT32_MAX) {
            nat_units_ok = false;
            break;
          }
          const int rows = std::min(UR, lptr[l + 1] - t0);
          nat_units.push_back(make_int4(t0, rows | int(w) << 8 | (fwd ? 0 : 1 << 16), UR, int(e0)));
          nat_max_width = std::max(nat_max_width, int(w));
        }
      }
      if (ltail >= nlev) (fwd ? nat_tail_f : nat_tail_b) = int(nat_units.size());
      if (fwd) nat_units_f = int(nat_units.size());
      int rc2;
      if ((rc2 = upv(W.info, info, "natural SSOR rows"))) return rc2;
      return upv(W.ecol, ecol, "natural SSOR columns");
    };
    nat_units.clear();
    nat_units_ok = true;
    nat_resident = -1;
    nat_max_width = 0;
    if ((rc = schedule(true, nat_f)) || (rc = schedule(false, nat_b))) return rc;
    if (nat_units_ok && (rc = upv(d_nat_units, nat_units, "natural SSOR units"))) return rc;
    const int ni = std::max(1, nf * (L.n_owned + L.n_ghost));  // internal layout
    if ((e = nat_d.alloc(std::max(1, n))) != hipSuccess || (e = nat_v.alloc(std::max(1, n))) != hipSuccess ||
        (e = nat_vf.alloc(std::max(1, n))) != hipSuccess || (e = nat_di.alloc(ni)) != hipSuccess ||
        (e = nat_vi.alloc(ni)) != hipSuccess || (e = nat_abort.alloc(4)) != hipSuccess ||
        (e = hipMemset(nat_abort.p, 0, 16)) != hipSuccess)
      return hipfail(e, "natural SSOR vectors");
    csr_nnz = nnz;
    csr_pat = mask;
    csr_nf = nf;
    csr_vals_valid = false;
    return PNP_OK;
  }

  // the CSR view's values from the current k-form matrix (once per assembly)
  int csr_values() {
    int rc;
    if ((rc = csr_structure())) return rc;
    if (csr_vals_valid) return nat_probe_run();
    hipError_t e = pnp::launch_csr_fill(dl, nf, pat, vals.p, csr_nnz, csr_src.p, csr_vidx.p,
                                        csr_val.p, stream);
    if (e != hipSuccess) return hipfail(e, "csr fill");
    csr_vals_valid = true;
    return nat_probe_run();
  }

  // v = SSOR_natural^{-1} d on internal-layout owned rows (ssor_natural.hip); csr_values() first
  // (internal layout, owned rows; d == vout allowed: the result is gathered into vout after both
  // sweeps)
  hipError_t ssor_natural(const double *d, double *vout) { return nat_sweep(d, vout); }
  // one launch for both sweeps (ssor_natural.hip, launch_ssor_natural_flow) whenever this context
  // owns its GPU: one rank, or one rank of an RCCL communicator (one process per GPU, each rank
  // sweeping its owned rows -- block Jacobi across ranks, as ISTL's NOVLP SeqSSOR on the local
  // matrix).  The in-process local group keeps the level launches: its ranks share one device, and
  // the dataflow needs every workgroup of its grid resident.  PNP_NAT_FLOW=0 keeps the level
  // launches everywhere
  bool use_nat_flow() const {
    static const bool env_on = [] {
      const char *ev = std::getenv("PNP_NAT_FLOW");
      return !(ev && std::atoi(ev) == 0);
    }();
    return nat_resident != 0 &&
           (nat_flow_opt == 0   ? false
            : nat_flow_opt == 1 ? nat_units_ok
                                : env_on && !lg && !host_tr() && nat_units_ok);
  }
  int nat_flow_opt = -1;  // PNP_OPT_NAT_FLOW: -1 auto (above), 0 level launches, 1 dataflow
  // the dataflow's progress needs its whole grid resident: checked once per schedule on the device
  // (pnp::ssor_natural_flow_resident) before the first dataflow application; 0 keeps the level
  // launches (the same results bit for bit).  -1 not yet checked
  int nat_resident = -1;
  DBuf<unsigned> nat_probe;
  int nat_probe_run() {
    if (nat_resident >= 0 || !use_nat_flow()) return PNP_OK;
    // test hook: PNP_NAT_PROBE_FAIL=1 takes the probe's "not resident" answer without running it
    // (tests/test_gpu_ssor_natural.py: the level launches are then used, bitwise the same)
    if (const char *ev = std::getenv("PNP_NAT_PROBE_FAIL"); ev && std::atoi(ev) == 1) {
      nat_resident = 0;
      return PNP_OK;
    }
    hipError_t e = nat_probe.p ? hipSuccess : nat_probe.alloc(2);
    if (e != hipSuccess) return hipfail(e, "natural SSOR probe");
    const int r = pnp::ssor_natural_flow_resident(nat_flow_view(), nat_probe.p, stream);
    if (r < 0) return fail(PNP_E_HIP, "natural SSOR: co-residency probe failed");
    nat_resident = r;
    return PNP_OK;
  }
  long long nat_flow_n = 0, nat_level_n = 0;  // applications per schedule (pnp_info)
  hipError_t nat_sweep(const double *d, double *vout) {
    if (use_nat_flow()) {
      nat_flow_n++;
      return ssor_natural_flow(d, vout);
    }
    nat_level_n++;
    return ssor_natural_levels(d, vout);
  }
  pnp::NatFlow nat_flow_view() const {
    pnp::NatFlow F;
    F.units = d_nat_units.p;
    F.nunits = int(nat_units.size());
    F.nunits_f = nat_units_f;
    F.tail_f = nat_tail_f;
    F.tail_b = nat_tail_b;
    F.max_width = nat_max_width;
    F.chain_f = nat_f.chains();
    F.chain_b = nat_b.chains();
    F.fwd = nat_f.view();
    F.bwd = nat_b.view();
    F.abort_word = nat_abort.p;
    return F;
  }
  hipError_t ssor_natural_flow(const double *d, double *vout) {
    const pnp::NatFlow F = nat_flow_view();
    hipError_t e = pnp::launch_ssor_natural_flow(F, nf * mesh.nv, csr_val.p, d, nat_vf.p, nat_v.p,
                                                 stream);
    // the result out of the external-layout vb (storing it at internal positions from the
    // backward kernels as well cost more than this gather: +40 against 22 us, r5f)
    if (e == hipSuccess)
      e = pnp::launch_gather_ext(L.n_owned, nf, mesh.nv, d_l2g.p, nat_v.p, vout, stream);
    return e;
  }
  // a dataflow sweep that timed out (never expected: every unit waits only on earlier units, all
  // resident) leaves NaN results and a sticky word; the solve reports it as an error
  int nat_check() {
    if (!use_nat_flow() || !nat_abort.p) return PNP_OK;
    unsigned w = 0;
    hipError_t e = hipMemcpyAsync(&w, nat_abort.p, 4, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "natural SSOR status");
    if (w) {
      hipMemsetAsync(nat_abort.p, 0, 16, stream);
      return fail(PNP_E_HIP, "natural SSOR: dataflow sweep timed out waiting for an operand");
    }
    return PNP_OK;
  }
  // ---- ILU(0) application as one dataflow launch (PNP_OPT_ILU_FLOW) -----------------------------
  // Units in the colour launches' order (forward colours c_first .. nc-2, the last colour, backward
  // colours nc-2 .. 0), one per 256-position block of the colour.  A unit's dependencies (all
  // earlier in the order): forward / last -- the forward units of the rows in its L staging list;
  // backward -- the backward (or last-colour) units of the rows in its U list, the forward units of
  // its own rows (their forward values are its input) and every forward unit whose L list holds one
  // of its rows (which must have read that row's forward value before it is overwritten).
  int ilu_flow_build(int c_first, IluFlowDev &D) {
    D.built = true;
    D.ok = false;
    const int nc = int(L.color_ptr.size()) - 1;
    const std::vector<int> &cp = L.color_ptr;
    if (!dl.lsx_ptr || nc < 2 || h_posrowL.empty()) return PNP_OK;
    std::vector<int> nb(nc), blk0(nc + 1, 0);
    for (int c = 0; c < nc; c++) {
      nb[c] = (cp[c + 1] - cp[c] + 255) / 256;
      blk0[c + 1] = blk0[c] + nb[c];
    }
    std::vector<std::pair<int, int>> stages;  // {kind, colour}
    for (int c = c_first; c < nc - 1; c++) stages.push_back({0, c});
    stages.push_back({2, nc - 1});
    for (int c = nc - 2; c >= 0; c--) stages.push_back({1, c});
    if (int(stages.size()) > pnp::kIluFlowMaxStages) return PNP_OK;
    pnp::IluFlow F;
    F.nstages = int(stages.size());
    int nu = 0;
    for (int s = 0; s < F.nstages; s++) {
      const int c = stages[s].second;
      F.unit0[s] = nu;
      F.kind[s] = stages[s].first;
      F.r0[s] = cp[c];
      F.r1[s] = cp[c + 1];
      F.blk0[s] = blk0[c];
      nu += nb[c];
    }
    F.unit0[F.nstages] = nu;
    F.nunits = nu;
    const int no = L.n_owned;
    std::vector<int> fwdu(no, -1), bwdu(no, -1);
    for (int s = 0; s < F.nstages; s++) {
      const int c = stages[s].second, kind = stages[s].first;
      for (int p = cp[c]; p < cp[c + 1]; p++) {
        const int u = F.unit0[s] + (p - cp[c]) / 256;
        if (kind != 1) fwdu[h_posrowL[p]] = u;
        if (kind != 0) bwdu[h_posrowU[p]] = u;
      }
    }
    // readers[r]: forward / last units whose L list holds row r (CSR)
    std::vector<int> rptr(no + 1, 0), rdr;
    auto lblock = [&](int s, int u) { return F.blk0[s] + (u - F.unit0[s]); };
    for (int pass = 0; pass < 2; pass++) {
      for (int s = 0; s < F.nstages; s++) {
        if (F.kind[s] == 1) continue;
        for (int u = F.unit0[s]; u < F.unit0[s + 1]; u++) {
          const int b = lblock(s, u);
          for (int k = h_lsx_ptr[b]; k < h_lsx_ptr[b + 1]; k++) {
            const int j = h_lsx_list[k];
            if (pass == 0)
              rptr[j + 1]++;
            else
              rdr[rptr[j]++] = u;
          }
        }
      }
      if (pass == 0) {
        for (int r = 0; r < no; r++) rptr[r + 1] += rptr[r];
        rdr.assign(rptr[no], 0);
      } else {
        for (int r = no; r > 0; r--) rptr[r] = rptr[r - 1];
        rptr[0] = 0;
      }
    }
    std::vector<int> dptr(nu + 1, 0), dlist, dep;
    for (int s = 0; s < F.nstages; s++) {
      const int c = stages[s].second;
      for (int u = F.unit0[s]; u < F.unit0[s + 1]; u++) {
        const int b = lblock(s, u);
        dep.clear();
        if (F.kind[s] != 1) {
          for (int k = h_lsx_ptr[b]; k < h_lsx_ptr[b + 1]; k++)
            if (fwdu[h_lsx_list[k]] >= 0) dep.push_back(fwdu[h_lsx_list[k]]);
        } else {
          for (int k = h_usx_ptr[b]; k < h_usx_ptr[b + 1]; k++)
            if (bwdu[h_usx_list[k]] >= 0) dep.push_back(bwdu[h_usx_list[k]]);
          const int p0 = cp[c] + 256 * (u - F.unit0[s]), p1 = std::min(cp[c + 1], p0 + 256);
          for (int p = p0; p < p1; p++) {
            const int r = h_posrowU[p];
            if (fwdu[r] >= 0) dep.push_back(fwdu[r]);
            for (int k = rptr[r]; k < rptr[r + 1]; k++) dep.push_back(rdr[k]);
          }
        }
        std::sort(dep.begin(), dep.end());
        dep.erase(std::unique(dep.begin(), dep.end()), dep.end());
        for (int w : dep)
          if (w >= u) return fail(PNP_E_STATE, "ILU(0) dataflow: a unit depends on a later one");
        dlist.insert(dlist.end(), dep.begin(), dep.end());
        dptr[u + 1] = int(dlist.size());
      }
    }
    if (dlist.empty()) dlist.push_back(0);
    auto upv = [&](auto &buf, const auto &vec, const char *what) -> int {
      hipError_t e2 = buf.alloc(vec.size());
      if (e2 == hipSuccess)
        e2 = hipMemcpy(buf.p, vec.data(), sizeof(vec[0]) * vec.size(), hipMemcpyHostToDevice);
      return e2 == hipSuccess ? PNP_OK : hipfail(e2, what);
    };
    int rc;
    if ((rc = upv(D.dep_ptr, dptr, "ILU(0) dataflow deps")) ||
        (rc = upv(D.dep_list, dlist, "ILU(0) dataflow deps")))
      return rc;
    hipError_t e = D.flags.alloc(size_t(nu + 1 + 3) & ~size_t(3));
    if (e == hipSuccess && !ilu_flow_abort.p) {
      e = ilu_flow_abort.alloc(4);
      if (e == hipSuccess) e = hipMemset(ilu_flow_abort.p, 0, 16);
    }
    if (e != hipSuccess) return hipfail(e, "ILU(0) dataflow flags");
    F.dep_ptr = D.dep_ptr.p;
    F.dep_list = D.dep_list.p;
    F.flags = D.flags.p;
    F.abort_word = ilu_flow_abort.p;
    D.F = F;
    D.ok = true;
    return PNP_OK;
  }
  // v = ILU(0)^-1 d over the owned rows, colours from c_first (launch_ilu0_apply's contract): one
  // dataflow launch when PNP_OPT_ILU_FLOW is on and d and v are distinct, else the colour launches
  int ilu_apply(const double *d, double *vout, int c_first, const char *what,
                hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr) {
    // the resident-grid form needs the device to itself: not with in-process ranks sharing it
    // (and one context per GPU at N > 1); PNP_ILU_FLOW_TICKET=1: the ticketed form (any residency)
    // PNP_ILU_FLOW_MODE: IluFlow::persistent (0 ticket, 1 static resident grid, the default).
    // A third form, a resident grid over 8 ticketed queues, hung in the bitwise tests (killed
    // after 180 s of silence, gpurun_out r4i) and was removed
    static const int mode = [] {
      const char *ev = std::getenv("PNP_ILU_FLOW_MODE");
      const int m = ev ? std::atoi(ev) : 1;
      return (m >= 0 && m <= 1) ? m : 1;
    }();
    // PNP_OPT_ILU_FLOW = 2 selects the ticketed form (any residency, so also ranks sharing a GPU)
    const int fmode = ilu_flow_opt == 2 ? 0 : mode;
    if (ilu_flow_opt && d != vout && (c_first == 0 || c_first == 1) && (fmode == 0 || !dist)) {
      IluFlowDev &D = ilu_flow[c_first];
      int rc;
      if (!D.built && (rc = ilu_flow_build(c_first, D))) return rc;
      D.F.persistent = fmode;
      if (D.ok) {
        if (t0) hipEventRecord(t0, stream);
        hipError_t e = pnp::launch_ilu0_flow(dl, D.F, nf, pat, lvals.p, uvals.p, d, vout, stream,
                                             f32_now());
        if (t1) hipEventRecord(t1, stream);
        if (e != hipSuccess) return hipfail(e, what);
        ilu_flow_used = true;
        ilu_flow_n++;
        return PNP_OK;
      }
    }
    hipError_t e = pnp::launch_ilu0_apply(dl, L.color_ptr.data(), nf, pat, lvals.p, uvals.p, d,
                                          vout, stream, c_first, nullptr, nullptr, f32_now(),
                                          ilu_y32(), t0, t1);
    return e == hipSuccess ? PNP_OK : hipfail(e, what);
  }
  // a dataflow application that timed out (never expected) leaves void results and a sticky word
  int ilu_flow_check() {
    if (!ilu_flow_used || !ilu_flow_abort.p) return PNP_OK;
    ilu_flow_used = false;
    unsigned w = 0;
    hipError_t e = hipMemcpyAsync(&w, ilu_flow_abort.p, 4, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "ILU(0) dataflow status");
    if (w) {
      hipMemsetAsync(ilu_flow_abort.p, 0, 16, stream);
      return fail(PNP_E_HIP, "ILU(0) dataflow application timed out waiting for a unit");
    }
    return PNP_OK;
  }
  // the level launches: one graph replay (captured on first use; PNP_NAT_GRAPH=0: eager), or eager
  // when the stream is itself being captured (a BiCGSTAB block graph then holds them), with more
  // than one rank, or after a failed capture
  // (on the context's external-layout nat_d / nat_v, so that the captured level graph's arguments
  // stay valid whatever vectors the caller passes)
  hipError_t ssor_natural_levels(const double *d, double *vout) {
    const int nv = mesh.nv;
    hipError_t e = pnp::launch_scatter_ext(L.n_owned, nf, nv, d_l2g.p, d, nat_d.p, stream);
    if (e == hipSuccess) e = ssor_natural_levels_fixed();
    if (e == hipSuccess) e = pnp::launch_gather_ext(L.n_owned, nf, nv, d_l2g.p, nat_v.p, vout, stream);
    return e;
  }
  hipError_t ssor_natural_levels_fixed() {
    auto issue = [&] {
      hipError_t e0 = hipMemsetAsync(nat_v.p, 0, sizeof(double) * nat_v.n, stream);
      return e0 != hipSuccess ? e0
                              : pnp::launch_ssor_natural(nat_f.view(), nat_b.view(), csr_val.p,
                                                         nat_d.p, nat_v.p, stream);
    };
    static const bool env_on = [] {
      const char *ev = std::getenv("PNP_NAT_GRAPH");
      return !(ev && std::atoi(ev) == 0);
    }();
    // not with more than one rank: in-process ranks share the device, and another rank's thread
    // touching the legacy stream during a capture would invalidate it
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (!env_on || dist || nat_graph_failed || profiled() ||
        hipStreamIsCapturing(stream, &cs) != hipSuccess ||
        cs != hipStreamCaptureStatusNone)
      return issue();
    if (!nat_exec) {
      hipError_t e = hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal);
      if (e == hipSuccess) {
        const hipError_t e1 = issue();
        hipGraph_t g = nullptr;
        const hipError_t e2 = hipStreamEndCapture(stream, &g);
        e = e1 != hipSuccess ? e1 : e2;
        if (e == hipSuccess) e = hipGraphInstantiate(&nat_exec, g, nullptr, nullptr, 0);
        if (g) hipGraphDestroy(g);
      }
      if (e != hipSuccess || !nat_exec) {  // nothing of the capture ran: launch eagerly
        (void)hipGetLastError();
        nat_exec = nullptr;
        nat_graph_failed = true;
        return issue();
      }
    }
    return hipGraphLaunch(nat_exec, stream);
  }

  // analytic (k-form) or forward-difference (expanded, kPat*FD) storage of the next Jacobian
  int set_fd(bool on) {
    if (on == fd_mode) return PNP_OK;
    graphs_clear();
    int rc;
    // P_k: the element kernel differentiates by itself; scalar blocks need no FD value layout
    if (on && !fd_built && degree == 1 && (rc = fd_build())) return rc;
    const int base = kind == PNP_OP_PNP ? pnp::kPatPnp
                                        : (kind == PNP_OP_PNP_IMPLICIT_EULER ? pnp::kPatPnpIE
                                                                            : pnp::kPatScalar);
    pat = (on && nf == 3) ? (base | pnp::kPatFD) : base;
    nks = pnp::nks_of(pat);
    fd_mode = on;
    assembled = false;
    lu_valid = false;
    split_of = 0;
    amg_valid = false;
    if (on && degree == 1) {
      // one-step operators keep two matrices per element (spatial, temporal: fd_jacobian.hip)
      const size_t need = size_t(fd_ne) * 9 * nf * nf * 2;
      if (fd_jel.n < need) {
        hipError_t e = fd_jel.alloc(need);
        if (e != hipSuccess) return hipfail(e, "fd element matrices");
      }
    }
    // padding slots must read as zeros in the new value layout (the SpMV multiplies them)
    hipError_t e = hipMemsetAsync(vals.p, 0, sizeof(double) * size_t(L.nslots) * nks, stream);
    return e == hipSuccess ? PNP_OK : hipfail(e, "clear matrix");
  }

  // P_k element lists (once per context): the local elements (every element with an owned node,
  // ascending global id) and their local nodes (SoA); per owned row its incident elements in
  // ascending order, in SELL-chunk layout (PkDev), with the row's slot of every element node
  int pk_build() {
    const pnp::Mesh &m = tmesh;
    const int nl = pks.nl, nw = (nl + 3) / 4;
    std::vector<int> en;
    std::vector<int> elist;
    for (int e = 0; e < m.nt; e++) {
      const int *g = &pks.enode[size_t(e) * nl];
      bool mine = false, local = true;
      for (int a = 0; a < nl; a++) {
        const int l = L.g2l[g[a]];
        mine = mine || (l >= 0 && l < L.n_owned);
        local = local && l >= 0;
      }
      if (!mine) continue;
      if (!local) return fail(PNP_E_MESH, "P_k: element not local");
      elist.push_back(e);
    }
    const int ne = int(elist.size());
    if (ne >= (1 << 27)) return fail(PNP_E_MESH, "P_k: too many local elements");
    en.resize(size_t(ne) * nl);
    for (int e = 0; e < ne; e++)
      for (int a = 0; a < nl; a++) en[size_t(a) * ne + e] = L.g2l[pks.enode[size_t(elist[e]) * nl + a]];
    auto slot_of = [&](int row, int col) -> int {
      const int ch = row / pnp::kRows, ln = row % pnp::kRows, len = pnp::meta_len(L.rowmeta[row]);
      if (col == row) return 0;
      for (int sl = 1; sl < len; sl++)
        if (L.colidx[L.chunk_off[ch] + 64LL * sl + ln] == col) return sl;
      return -1;
    };
    // incidences per owned row, ascending element order
    std::vector<int> icnt(L.n_owned, 0);
    for (int e = 0; e < ne; e++)
      for (int a = 0; a < nl; a++) {
        const int ra = en[size_t(a) * ne + e];
        if (ra < L.n_owned) icnt[ra]++;
      }
    std::vector<int> ioff(L.nchunks + 1, 0);
    for (int c = 0; c < L.nchunks; c++) {
      int mx = 0;
      for (int ln = 0; ln < pnp::kRows && c * pnp::kRows + ln < L.n_owned; ln++)
        mx = std::max(mx, icnt[c * pnp::kRows + ln]);
      ioff[c + 1] = ioff[c] + pnp::kRows * mx;
    }
    std::vector<int> inc(std::max(1, ioff[L.nchunks]), 0), fill(L.n_owned, 0);
    std::vector<uint32_t> islot(size_t(std::max(1, ioff[L.nchunks])) * nw, 0);
    for (int e = 0; e < ne; e++)
      for (int a = 0; a < nl; a++) {
        const int ra = en[size_t(a) * ne + e];
        if (ra >= L.n_owned) continue;
        const int c = ra / pnp::kRows, ln = ra % pnp::kRows;
        const size_t p = size_t(ioff[c]) + size_t(pnp::kRows) * fill[ra]++ + ln;
        inc[p] = e << 4 | a;
        for (int b = 0; b < nl; b++) {
          const int sl = slot_of(ra, en[size_t(b) * ne + e]);
          if (sl < 0) return fail(PNP_E_MESH, "P_k: element pair outside the pattern");
          islot[p * nw + (b >> 2)] |= uint32_t(sl) << (8 * (b & 3));
        }
      }
    int rc;
    if ((rc = upv(pk_enode, en, "P_k elements")) || (rc = upv(pk_ioff, ioff, "P_k ioff")) ||
        (rc = upv(pk_icnt, icnt, "P_k icnt")) || (rc = upv(pk_inc, inc, "P_k incidences")) ||
        (rc = upv(pk_islot, islot, "P_k slots")))
      return rc;
    hipError_t e = pk_eres.alloc(std::max<size_t>(1, size_t(ne) * nl));
    if (e != hipSuccess) return hipfail(e, "P_k element residual scratch");
    e = pk_ejac.alloc(std::max<size_t>(1, size_t(ne) * nl * ((nl + 2) & ~1)));
    if (e != hipSuccess) return hipfail(e, "P_k element matrix scratch");
    e = pnp::pk_upload_tables(pks.k, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "P_k tables");
    pkd.k = pks.k;
    pkd.nl = nl;
    pkd.ne = ne;
    pkd.enode = pk_enode.p;
    pkd.ioff = pk_ioff.p;
    pkd.icnt = pk_icnt.p;
    pkd.inc = pk_inc.p;
    pkd.islot = pk_islot.p;
    pkd.eres = pk_eres.p;
    pkd.ejac = pk_ejac.p;
    // the Jacobian gather pass accumulates a row's slots in LDS, sized for the longest row: the
    // vertex rows (up to 55 slots at P3) would hold every workgroup to one per CU.  When the
    // longest row needs more than 64 KB per workgroup, blocks whose rows are all at most the
    // median block length (the edge and interior node rows) run in a launch of their own with an
    // LDS accumulator of that length: P3 438 -> 395 us; at P2 (one launch at 3 workgroups per CU)
    // the second launch costs more than it gains, 135 -> 145 us (profiles/r02/ab_pk_split).
    // PNP_PK_SPLIT=0: always one launch, 1: split whenever the median is at most half the longest
    {
      const char *ev = getenv("PNP_PK_SPLIT");
      const int nblk = (L.n_owned + 255) / 256;
      std::vector<int> order(nblk), blen(nblk, 0);
      for (int b = 0; b < nblk; b++) order[b] = b;
      if (dl.blkmap && nblk > 0) {
        e = hipMemcpy(order.data(), dl.blkmap, sizeof(int) * nblk, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hipfail(e, "blkmap");
      }
      for (int r = 0; r < L.n_owned; r++)
        blen[r / 256] = std::max(blen[r / 256], pnp::meta_len(L.rowmeta[r]));
      std::vector<int> srt(blen);
      std::nth_element(srt.begin(), srt.begin() + nblk / 2, srt.end());
      const int T = nblk > 0 ? srt[nblk / 2] : 0;
      const int mx = nblk > 0 ? *std::max_element(blen.begin(), blen.end()) : 0;
      const bool want = ev ? ev[0] == '1' : size_t(mx) * 256 * sizeof(double) > 64 * 1024;
      if (want && nblk > 0 && 2 * T <= mx) {
        std::vector<int> sh, lo;
        for (int b : order) (blen[b] <= T ? sh : lo).push_back(b);
        if ((rc = upv(pk_blk_short, sh, "P_k short blocks")) ||
            (rc = upv(pk_blk_long, lo, "P_k long blocks")))
          return rc;
        pkd.blk_short = pk_blk_short.p;
        pkd.blk_long = pk_blk_long.p;
        pkd.n_short = int(sh.size());
        pkd.n_long = int(lo.size());
        pkd.short_len = T;
      }
    }
    // ion-flux segments handled by this rank: those whose element is local and whose lower
    // global vertex is owned here, {local element, face, group}, in global segment order
    std::vector<int> eloc(m.nt, -1);
    for (int e2 = 0; e2 < ne; e2++) eloc[elist[e2]] = e2;
    std::vector<int4> segs;
    fseg_group.clear();
    for (int sg = 0; sg < m.nb; sg++) {
      const int a = m.bseg[2 * size_t(sg)], b = m.bseg[2 * size_t(sg) + 1];
      const int lo = L.g2l[std::min(a, b)];
      if (lo < 0 || lo >= L.n_owned) continue;
      const int bf = pks.bface[sg];
      if (bf < 0 || eloc[bf / 3] < 0) return fail(PNP_E_MESH, "ion flux: the element of a boundary segment is not local");
      segs.push_back(make_int4(eloc[bf / 3], bf % 3, m.bgroup[sg], 0));
      fseg_group.push_back(m.bgroup[sg]);
    }
    if ((rc = upv(d_fseg, segs, "P_k flux segments"))) return rc;
    e = fluxout.alloc(2 * segs.size() + 2);
    if (e != hipSuccess) return hipfail(e, "flux out");
    return PNP_OK;
  }

  // local elements (ascending global id, vertices in mesh order) and, per owned row and slot, the
  // element entries summed into that block, in ascending element order
  int fd_build() {
    const pnp::Mesh &m = mesh;
    std::vector<int> et;
    for (int e = 0; e < m.nt; e++) {
      const int *t = &m.tri[3 * size_t(e)];
      const int l0 = L.g2l[t[0]], l1 = L.g2l[t[1]], l2 = L.g2l[t[2]];
      const bool mine = (l0 >= 0 && l0 < L.n_owned) || (l1 >= 0 && l1 < L.n_owned) ||
                        (l2 >= 0 && l2 < L.n_owned);
      if (!mine) continue;
      if (l0 < 0 || l1 < 0 || l2 < 0) return fail(PNP_E_MESH, "FD Jacobian: element not local");
      et.push_back(l0);
      et.push_back(l1);
      et.push_back(l2);
    }
    const int ne = int(et.size() / 3);
    auto pos_of = [&](int row, int col) -> long long {
      const int ch = row / pnp::kRows, ln = row % pnp::kRows, len = pnp::meta_len(L.rowmeta[row]);
      if (col == row) return L.chunk_off[ch] + ln;
      for (int sl = 1; sl < len; sl++) {
        const long long p = L.chunk_off[ch] + 64LL * sl + ln;
        if (L.colidx[p] == col) return p;
      }
      return -1;
    };
    std::vector<int> cnt(size_t(L.nslots) + 1, 0);
    for (int e = 0; e < ne; e++)
      for (int a = 0; a < 3; a++) {
        const int va = et[3 * size_t(e) + a];
        if (va >= L.n_owned) continue;
        for (int b = 0; b < 3; b++) {
          const long long p = pos_of(va, et[3 * size_t(e) + b]);
          if (p < 0) return fail(PNP_E_MESH, "FD Jacobian: element pair outside the pattern");
          cnt[p]++;
        }
      }
    // per row: for each slot, the count then its codes
    std::vector<long long> rptr(L.n_owned + 1, 0);
    for (int i = 0; i < L.n_owned; i++) {
      const int ch = i / pnp::kRows, ln = i % pnp::kRows, len = pnp::meta_len(L.rowmeta[i]);
      long long n = 0;
      for (int sl = 0; sl < len; sl++) n += 1 + cnt[L.chunk_off[ch] + 64LL * sl + ln];
      rptr[i + 1] = rptr[i] + n;
    }
    std::vector<long long> at((size_t)L.nslots, -1LL);  // next free code position of each block
    std::vector<int> data((size_t)rptr[L.n_owned]);
    for (int i = 0; i < L.n_owned; i++) {
      const int ch = i / pnp::kRows, ln = i % pnp::kRows, len = pnp::meta_len(L.rowmeta[i]);
      long long q = rptr[i];
      for (int sl = 0; sl < len; sl++) {
        const long long p = L.chunk_off[ch] + 64LL * sl + ln;
        data[q] = cnt[p];
        at[p] = q + 1;
        q += 1 + cnt[p];
      }
    }
    for (int e = 0; e < ne; e++)
      for (int a = 0; a < 3; a++) {
        const int va = et[3 * size_t(e) + a];
        if (va >= L.n_owned) continue;
        for (int b = 0; b < 3; b++) {
          const long long p = pos_of(va, et[3 * size_t(e) + b]);
          data[at[p]++] = e * 9 + a * 3 + b;
        }
      }
    int rc;
    if ((rc = upv(fd_etri, et, "fd elements")) || (rc = upv(fd_rptr, rptr, "fd rptr")) ||
        (rc = upv(fd_cdata, data, "fd contributions")))
      return rc;
    fd_ne = ne;
    fd_built = true;
    return PNP_OK;
  }

  // ILU(0) factors of the current matrix (once per assembly).  Default: the fused factorisation
  // (expand and split folded in, neighbour-row work hoisted; PNP_OPT_ILU_FUSED_FACTOR = 0 runs the
  // three-pass path, the same bits)
  int ilu_factor() {
    if (lu_valid) return PNP_OK;
    hipEvent_t t0 = tb(T_FACT);
    hipError_t e;
    if (ilu_fused) {
      e = pnp::launch_ilu0_factor_fused(dl, L.color_ptr.data(), nf, pat, vals.p, d_rowoff.p,
                                        d_rowcol.p, lu.p, lvals.p, uvals.p, ilu_fac(), stream);
    } else {
      e = pnp::launch_expand(dl, nf, pat, vals.p, lu.p, stream);
      if (e == hipSuccess)
        e = pnp::launch_ilu0_factor(dl, L.color_ptr.data(), nf, pat, lu.p, stream);
    }
    if (e != hipSuccess) return hipfail(e, "ilu0 factorisation");
    te(T_FACT, t0);
    lu_valid = true;
    split_of = ilu_fused ? 2 : 0;
    return PNP_OK;
  }

  // bring the split storage up to date with the matrix (which = 1) or the factors (which = 2)
  int split(int which) {
    if (split_of == which) return PNP_OK;
    if (which == 2 && ilu_fused) {  // the fused factorisation keeps no SELL copy: redo it
      lu_valid = false;
      return ilu_factor();
    }
    hipEvent_t t0 = tb(T_FACT);
    hipError_t e = pnp::launch_split(dl, nf, pat, which == 1 ? 1 : 0, which == 2 ? lu.p : vals.p,
                                     d_lsrc.p, (long long)d_lsrc.n, d_usrc.p, (long long)d_usrc.n,
                                     lvals.p, uvals.p, stream, which == 2 ? ilu_fac() : 0);
    if (e != hipSuccess) return hipfail(e, "split");
    te(T_FACT, t0);
    split_of = which;
    return PNP_OK;
  }

  // ---- aggregation AMG ------------------------------------------------------------------------
  template <typename T>
  int upv(DBuf<T> &d, const std::vector<T> &h, const char *what) {
    hipError_t e = d.alloc(std::max<size_t>(1, h.size()));
    if (e == hipSuccess && !h.empty())
      e = hipMemcpy(d.p, h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice);
    return e == hipSuccess ? PNP_OK : hipfail(e, what);
  }

  // hierarchy patterns (once), value/vector buffers (per field count), coarse values (per
  // assembly): Galerkin sums, block-diagonal inverses, the coarsest dense inverse
  int amg_setup() {
    int rc;
    if (!assembled) return fail(PNP_E_STATE, "no Jacobian assembled");
    if (!amg_built) {
      amg_d.clear();
      if (!pnp::amg_build(L, amg_opts.coarse_target, amg_opts.max_levels, amg_h, err))
        return PNP_E_STATE;
      for (const auto &H : amg_h) {
        auto D = std::make_unique<AmgDev>();
        D->nb = H.nb;
        if ((rc = upv(D->rp, H.rp, "amg rp")) || (rc = upv(D->col, H.col, "amg col")) ||
            (rc = upv(D->dpos, H.dpos, "amg dpos")) || (rc = upv(D->mptr, H.mptr, "amg mptr")) ||
            (rc = upv(D->mem, H.mem, "amg mem")) || (rc = upv(D->agg, H.agg, "amg agg")) ||
            (rc = upv(D->csrc, H.csrc, "amg csrc")) || (rc = upv(D->cptr, H.cptr, "amg cptr")))
          return rc;
        amg_d.push_back(std::move(D));
      }
      amg_built = true;
      amg_nf = 0;
    }
    if (amg_d.empty()) return fail(PNP_E_STATE, "AMG: no owned rows");
    const int K = int(amg_d.size());
    if (amg_d[K - 1]->nb * nf > pnp::kAmgMaxDense)
      return fail(PNP_E_STATE, "AMG: coarsest level too large for the dense solve");
    if (amg_nf != nf) {
      const size_t nb2 = size_t(nf) * nf;
      for (auto &D : amg_d) {
        hipError_t e;
        if ((amg_f32() && D.get() != amg_d.back().get() &&
             (e = D->vf.alloc(std::max<size_t>(1, D->col.n) * nb2)) != hipSuccess) ||
            (e = D->v.alloc(std::max<size_t>(1, D->col.n) * nb2)) != hipSuccess ||
            (e = D->dinv.alloc(size_t(D->nb) * nb2)) != hipSuccess ||
            (e = D->b.alloc(size_t(D->nb) * nf)) != hipSuccess ||
            (e = D->x.alloc(size_t(D->nb) * nf)) != hipSuccess ||
            (e = D->x2.alloc(size_t(D->nb) * nf)) != hipSuccess)
          return hipfail(e, "amg level buffers");
      }
      const size_t nc = size_t(amg_d[K - 1]->nb) * nf, nl = size_t(L.n_owned + L.n_ghost) * nf;
      hipError_t e;
      amg_ld = int((nc + 3) & ~size_t(3));
      if ((amg_f32() && (e = amg_ainv_f.alloc(nc * size_t(amg_ld))) != hipSuccess) ||
          (e = amg_ainv.alloc(nc * nc)) != hipSuccess || (e = amg_ipiv.alloc(nc)) != hipSuccess ||
          (e = amg_info.alloc(1)) != hipSuccess ||
          (e = amg_x0.alloc(nl)) != hipSuccess || (e = amg_t.alloc(nl)) != hipSuccess ||
          (e = amg_y.alloc(nl)) != hipSuccess || (e = amg_r.alloc(nl)) != hipSuccess ||
          (e = amg_z.alloc(nl)) != hipSuccess)
        return hipfail(e, "amg vectors");
      amg_nf = nf;
      amg_valid = false;
    }
    const int sm = amg_opts.smoother;
    if (sm == PNP_PREC_SSOR && (rc = split(1))) return rc;
    if (sm == PNP_PREC_SSOR_NATURAL && (rc = csr_values())) return rc;
    if (sm == PNP_PREC_ILU0 && ((rc = ilu_factor()) || (rc = split(2)))) return rc;
    if (amg_valid) return PNP_OK;
    hipEvent_t t0 = tb(T_FACT);
    double ts = now_s();
    hipError_t e = pnp::launch_amg_galerkin0(dl, nf, pat, vals.p, (long long)amg_h[0].col.size(),
                                             amg_d[0]->cptr.p, amg_d[0]->csrc.p, amg_d[0]->v.p,
                                             stream);
    for (int k = 1; k < K && e == hipSuccess; k++)
      e = pnp::launch_amg_galerkin(nf, (long long)amg_h[k].col.size(), amg_d[k]->cptr.p,
                                   amg_d[k]->csrc.p, amg_d[k - 1]->v.p, amg_d[k]->v.p, stream);
    for (int k = 0; k + 1 < K && e == hipSuccess; k++)
      e = pnp::launch_amg_dinv(nf, amg_d[k]->nb, amg_d[k]->dpos.p, amg_d[k]->v.p,
                               amg_d[k]->dinv.p, stream);
    for (int k = 0; k + 1 < K && e == hipSuccess; k++)
      if (amg_d[k]->vf.p)
        e = pnp::launch_amg_to_f32((long long)amg_d[k]->col.n * nf * nf, amg_d[k]->v.p,
                                   amg_d[k]->vf.p, stream);
    if (e == hipSuccess)
      e = pnp::launch_amg_coarse_dense(nf, amg_d[K - 1]->nb, amg_d[K - 1]->rp.p,
                                       amg_d[K - 1]->col.p, amg_d[K - 1]->v.p, amg_ainv.p, stream);
    if (e != hipSuccess) return hipfail(e, "amg setup");
    {  // coarsest inverse in place: LU with partial pivoting, then the inverse -- of A^T column-
       // major, which leaves A^-1 row-major for k_coarse_apply
      if (!blas) {
        if (rocblas_create_handle(&blas) != rocblas_status_success)
          return fail(PNP_E_HIP, "rocblas_create_handle failed");
      }
      if (rocblas_set_stream(blas, stream) != rocblas_status_success)
        return fail(PNP_E_HIP, "rocblas_set_stream failed");
      const int nc = amg_d[K - 1]->nb * nf;
      if (rocsolver_dgetrf(blas, nc, nc, amg_ainv.p, nc, amg_ipiv.p, amg_info.p) !=
              rocblas_status_success ||
          rocsolver_dgetri(blas, nc, amg_ainv.p, nc, amg_ipiv.p, amg_info.p) !=
              rocblas_status_success)
        return fail(PNP_E_HIP, "rocsolver getrf/getri of the AMG coarsest level failed");
      int info = 0;
      e = hipMemcpyAsync(&info, amg_info.p, sizeof info, hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      if (e != hipSuccess) return hipfail(e, "amg setup");
      if (info != 0)
        return fail(PNP_E_STATE, "AMG: coarsest matrix singular (getrf info " +
                                     std::to_string(info) + ")");
      if (amg_ainv_f.p &&
          (e = pnp::launch_amg_inverse_to_f32(nc, amg_ld, amg_ainv.p, amg_ainv_f.p, stream)) !=
              hipSuccess)
        return hipfail(e, "amg setup");
    }
    te(T_FACT, t0);
    amg_setup_ms = (now_s() - ts) * 1e3;  // host-side issue time (device time: T_FACT timers)
    amg_valid = true;
    return PNP_OK;
  }

  // block-Jacobi sweeps on coarse level k + 1 (amg_d[k]): the configured count; PNP_AMG_DEEP_SWEEPS
  // (A/B, environment) overrides it below level 1, where the kernels sit at the launch floor
  int amg_sweeps(int k) const {
    static const int deep = [] {
      const char *e = std::getenv("PNP_AMG_DEEP_SWEEPS");
      return e ? std::atoi(e) : 0;
    }();
    return (k >= 1 && deep >= 1) ? deep : amg_opts.coarse_sweeps;
  }

  // one V-cycle: vout = B d (owned rows); see amg.hip for the kernels
  int amg_apply(const double *d, double *vout) {
    const int K = int(amg_d.size()), sm = amg_opts.smoother, n = L.n_owned;
    const double om = amg_opts.omega;
    const long long nn = nown();
    int rc, nsp = 0;
    hipError_t e;
    // level 0 pre-smoothing from zero, residual (SpMV residual mode), restriction (+ level-1
    // pre-smoothing); without level-0 pre-smoothing x0 = 0 and the restriction takes d itself
    // amg_opts.level0_presmooth: 1 always, 0 never, -1 (auto) only when the V-cycle must stay
    // symmetric (CG, or a bare pnp_prec_apply); BiCGSTAB takes the post-smoothing-only cycle
    const bool pre0 = amg_opts.level0_presmooth > 0 ||
                      (amg_opts.level0_presmooth < 0 && amg_symmetric);
    if (pre0) {
      if ((rc = smoother(sm, d, amg_x0.p))) return rc;
      e = pnp::launch_spmv(dl, nf, pat, vals.p, amg_x0.p, amg_t.p, 3, d, partials.p, &nsp,
                           stream);
    } else {
      e = hipSuccess;  // x0 = 0: the restriction takes d, the prolongation no x0
    }
    if (e == hipSuccess)
      e = pnp::launch_amg_restrict(nf, amg_d[0]->nb, amg_d[0]->mptr.p, amg_d[0]->mem.p,
                                   pre0 ? amg_t.p : d, nullptr, amg_d[0]->b.p, amg_d[0]->dinv.p,
                                   om, K > 1 ? amg_d[0]->x.p : nullptr, stream);
    for (int k = 0; k + 1 < K && e == hipSuccess; k++) {
      AmgDev &C = *amg_d[k], &N = *amg_d[k + 1];
      for (int sw = 1; sw < amg_sweeps(k) && e == hipSuccess; sw++) {  // more pre-smoothing
        e = pnp::launch_amg_post(nf, C.nb, C.rp.p, C.col.p, C.v.p, C.vf.p, nullptr, C.x.p,
                                 nullptr, C.b.p, C.dinv.p, om, C.x2.p, stream);
        std::swap(C.x.p, C.x2.p);
      }
      // residual of level k+1 into its x2 (free until its post-smoothing), then restriction
      if (e == hipSuccess)
        e = pnp::launch_amg_resid(nf, C.nb, C.rp.p, C.col.p, C.v.p, C.vf.p, C.x.p, C.b.p,
                                  C.x2.p, stream);
      if (e == hipSuccess)
        e = pnp::launch_amg_restrict(nf, N.nb, N.mptr.p, N.mem.p, C.x2.p, nullptr, N.b.p,
                                     N.dinv.p, om, k + 2 < K ? N.x.p : nullptr, stream);
    }
    if (e == hipSuccess)
      e = amg_ainv_f.p
              ? pnp::launch_amg_coarse_apply_f32(amg_d[K - 1]->nb * nf, amg_ld, amg_ainv_f.p,
                                                 amg_d[K - 1]->b.p, amg_d[K - 1]->x.p, stream)
              : pnp::launch_amg_coarse_apply(amg_d[K - 1]->nb * nf, amg_ainv.p, amg_d[K - 1]->b.p,
                                       amg_d[K - 1]->x.p, stream);
    const double *res = amg_d[K - 1]->x.p;  // the solution of the level just finished
    for (int k = K - 2; k >= 0 && e == hipSuccess; k--) {
      AmgDev &C = *amg_d[k];
      e = pnp::launch_amg_post(nf, C.nb, C.rp.p, C.col.p, C.v.p, C.vf.p, amg_d[k + 1]->agg.p,
                               C.x.p, res, C.b.p, C.dinv.p, om, C.x2.p, stream);
      res = C.x2.p;
      for (int sw = 1; sw < amg_sweeps(k) && e == hipSuccess; sw++) {  // more post-smoothing
        double *out = res == C.x2.p ? C.x.p : C.x2.p;
        e = pnp::launch_amg_post(nf, C.nb, C.rp.p, C.col.p, C.v.p, C.vf.p, nullptr, res,
                                 nullptr, C.b.p, C.dinv.p, om, out, stream);
        res = out;
      }
    }
    // level 0: prolongation, post-smoothing x += M^{-1} (d - A x)
    if (e == hipSuccess)
      e = pnp::launch_amg_prolong0(nf, n, amg_d[0]->agg.p, pre0 ? amg_x0.p : nullptr, res,
                                   amg_y.p, stream);
    if (e == hipSuccess)
      e = pnp::launch_spmv(dl, nf, pat, vals.p, amg_y.p, amg_r.p, 3, d, partials.p, &nsp, stream);
    if (e != hipSuccess) return hipfail(e, "amg v-cycle");
    if (sm == PNP_PREC_ILU0) {  // vout = y + M^-1 r, written by the backward sweep
      e = pnp::launch_ilu0_apply(dl, L.color_ptr.data(), nf, pat, lvals.p, uvals.p, amg_r.p,
                                 amg_z.p, stream, 0, amg_y.p, vout, f32_now(), ilu_y32());
      return e == hipSuccess ? PNP_OK : hipfail(e, "amg v-cycle");
    }
    if ((rc = smoother(sm, amg_r.p, amg_z.p))) return rc;
    e = pnp::launch_axpby(nn, 1.0, amg_y.p, 1.0, amg_z.p, vout, stream);
    return e == hipSuccess ? PNP_OK : hipfail(e, "amg v-cycle");
  }

  // the single-level preconditioners, untimed, prerequisites (split / factors) in place
  int smoother(int prec, const double *d, double *vout) {
    hipError_t e = hipSuccess;
    if (prec == PNP_PREC_JACOBI) {
      e = pnp::launch_jacobi(dl, nf, pat, vals.p, d, vout, stream);
    } else if (prec == PNP_PREC_SSOR) {
      e = pnp::launch_sgs(dl, L.color_ptr.data(), nf, pat, lvals.p, uvals.p, d, vout, tsgs.p,
                          stream);
    } else if (prec == PNP_PREC_ILU0) {
      return ilu_apply(d, vout, 0, "preconditioner");
    } else if (prec == PNP_PREC_SSOR_NATURAL) {
      e = ssor_natural(d, vout);
    } else {
      e = hipMemcpyAsync(vout, d, sizeof(double) * nown(), hipMemcpyDeviceToDevice, stream);
    }
    return e == hipSuccess ? PNP_OK : hipfail(e, "preconditioner");
  }

  // v = M^{-1} d over owned rows (v sized n_local)
  int precond(int prec, const double *d, double *vout) {
    int rc;
    if (prec == PNP_PREC_SSOR && (rc = split(1))) return rc;
    if (prec == PNP_PREC_SSOR_NATURAL && (rc = csr_values())) return rc;
    if (prec == PNP_PREC_ILU0 && ((rc = ilu_factor()) || (rc = split(2)))) return rc;
    if (prec == PNP_PREC_AMG && (rc = amg_setup())) return rc;
    hipEvent_t t0 = tb(T_PREC);
    if (prec == PNP_PREC_AMG) {
      if ((rc = amg_apply(d, vout))) return rc;
      te(T_PREC, t0);
      return PNP_OK;
    }
    if ((rc = smoother(prec, d, vout))) return rc;
    te(T_PREC, t0);
    return PNP_OK;
  }

  // BiCGSTAB on J zout = bdev (owned rows), zout zero start.  fixed > 0: exactly that many
  // iterations, no convergence stop (reduction 0), used by the benchmarks.
  int bicgstab(const double *bdev, double *zout, const pnp_solve_opts &o, pnp_solve_result &res,
               int fixed) {
    if (!assembled) return fail(PNP_E_STATE, "no Jacobian assembled");
    double t_start = now_s();
    long long n = nown();
    int np = pnp::blas_nparts(n);
    int rows_np = (L.n_owned + 255) / 256;
    (void)rows_np;
    hipError_t e;
    e = hipMemsetAsync(zout, 0, sizeof(double) * n, stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(rs.p + 0, bdev, sizeof(double) * n, hipMemcpyDeviceToDevice, stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(rt.p, bdev, sizeof(double) * n, hipMemcpyDeviceToDevice, stream);
    if (e == hipSuccess) e = hipMemsetAsync(v.p, 0, sizeof(double) * n, stream);
    if (e == hipSuccess) e = hipMemsetAsync(p.p, 0, sizeof(double) * n, stream);
    if (e != hipSuccess) return hipfail(e, "bicgstab init");
    // set reduction, reset flags
    pnp::Scalars &init = hS[2];  // pinned staging slot
    std::memset(&init, 0, sizeof init);
    init.reduction = fixed > 0 ? 0.0 : o.reduction;
    // divergence guard for the AMG preconditioner only (a non-symmetric V-cycle can make
    // BiCGSTAB diverge; ISTL semantics otherwise: run to maxit)
    init.divguard = (o.prec == PNP_PREC_AMG && fixed <= 0) ? 1 : 0;
    e = hipMemcpyAsync(S.p, &init, sizeof init, hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return hipfail(e, "bicgstab scalars");
    hipEvent_t t0 = tb(T_BLAS);
    e = pnp::launch_dot(n, rs.p, rs.p, 0, partials.p, stream);
    if (e != hipSuccess) return hipfail(e, "bicgstab norm0");
    int rc = reduce_derive(np, 1, 0);
    if (rc) return rc;
    te(T_BLAS, t0);
    int maxit = fixed > 0 ? fixed : o.maxit;
    int check = o.check_every > 0 ? o.check_every : 8;
    if (fixed > 0) check = fixed;
    int prec = o.prec;
    if (prec == PNP_PREC_ILU0 && ((rc = ilu_factor()) || (rc = split(2)))) return rc;
    if (prec == PNP_PREC_SSOR && (rc = split(1))) return rc;
    if (prec == PNP_PREC_SSOR_NATURAL && (rc = csr_values())) return rc;
    if (prec == PNP_PREC_AMG && (rc = amg_setup())) return rc;
    int nsp = 0, npu = 0;
    // ILU(0): the two vector updates that feed the preconditioner also do colour 0 of its
    // forward sweep (launch_update_fwd0); PNP_FUSE=0 keeps them apart (A/B)
    static const bool fuse_env = [] {
      const char *ev = std::getenv("PNP_FUSE");
      return !(ev && std::atoi(ev) == 0);
    }();
    const bool fuse = fuse_env && prec == PNP_PREC_ILU0 && L.color_ptr.size() > 2;
    const int c0_end = L.color_ptr.size() > 1 ? L.color_ptr[1] : 0;
    // the colour launches record the timer events themselves: the first launch's start and the
    // last launch's end (no marker dispatch in the measured span)
    auto ilu_from1 = [&](const double *d, double *out) -> int {
      hipEvent_t t0 = nullptr, t1 = nullptr;
      if (timing && L.n_owned > 0) {
        t0 = ev_get();
        t1 = ev_get();
      }
      const int rc1 = ilu_apply(d, out, 1, "preconditioner", t0, t1);
      if (rc1) return rc1;
      if (t1) {
        ev_pending[T_PREC].push_back({t0, t1});
        t_n[T_PREC]++;
      }
      return PNP_OK;
    };
    // two-reduction iteration (two allreduces per iteration instead of three: rho_new from the
    // same reduction as omega, the second half step's test lagged into the next h reduction):
    // on by default with more than one rank, where each reduction is an allreduce round trip;
    // PNP_OPT_BICG_TWORED (or PNP_BICG_TWORED) 0/1 forces it off/on.  Half-step counts keep
    // ISTL's semantics.
    const bool twored = twored_opt >= 0 ? twored_opt == 1 : dist;
    // fused ILU(0), one reduction per half step: the first half step's x += alpha y is applied by
    // the second half's update (one read and write of x per iteration fewer; the second
    // preconditioned vector then goes to y2).  PNP_XDEFER=0 keeps the two passes (A/B).
    static const bool xdefer_env = [] {
      const char *ev = std::getenv("PNP_XDEFER");
      return !(ev && std::atoi(ev) == 0);
    }();
    const bool xdefer = xdefer_env && fuse && !twored;
    double *const y2p = xdefer ? y2.p : y.p;
    int pending_np = 0;
    // one BiCGSTAB iteration; for k >= 1 (and without the two-reduction variant's host state) it
    // launches the same kernels with the same arguments every time, which is what the graph
    // replay below relies on
    auto body = [&](int k) -> int {
      // p = r + beta (p - omega v)
      hipEvent_t t0 = tb(T_BLAS);
      if (fuse)
        e = pnp::launch_update_fwd0(dl, nf, pat, c0_end, S.p, 0, k == 0 ? 1 : 0, nullptr, nullptr,
                                    rs.p, v.p, p.p, uvals.p, y.p, nullptr, nullptr, stream,
                                    f32_now(), nullptr, ilu_y32());
      else
        e = pnp::launch_update_p(n, S.p, rs.p, v.p, p.p, k == 0 ? 1 : 0, stream);
      if (e != hipSuccess) return hipfail(e, "update_p");
      te(T_BLAS, t0);
      // y = M^{-1} p ; v = A y ; h = <rt, v>
      const double *yin = p.p;
      if (fuse) {
        if ((rc = ilu_from1(p.p, y.p))) return rc;
        yin = y.p;
      } else if (prec != PNP_PREC_NONE) {
        if ((rc = precond(prec, p.p, y.p))) return rc;
        yin = y.p;
      }
      if ((rc = halo_spmv(const_cast<double *>(yin), v.p, 1, rt.p, nullptr, &nsp))) return rc;
      if (twored)  // h, with the previous iteration's second-half test (||r||^2 in partials2)
        rc = pending_np > 0 ? reduce_derive2(nsp, 1, pending_np, 1, 31) : reduce_derive(nsp, 1, 31);
      else
        rc = reduce_derive(nsp, 1, 1);
      if (rc) return rc;
      // x += alpha y ; r -= alpha v ; ||r|| (partials2: its half-step test is derived together
      // with omega below -- one reduction and one allreduce fewer per iteration; the second
      // half's kernels ignore a converged first half, update_xr skips on S->done).  Two-reduction
      // iteration (twored): also <rt, s> into partials2, for rho_new without a third reduction.
      t0 = tb(T_BLAS);
      if (fuse)
        e = pnp::launch_update_fwd0(dl, nf, pat, c0_end, S.p, 1, 0, xdefer ? nullptr : zout, yin,
                                    rs.p, v.p, nullptr, uvals.p, y2p, partials2.p, &npu, stream,
                                    f32_now(), twored ? rt.p : nullptr, ilu_y32());
      else
        e = pnp::launch_update_xr(n, S.p, 0, zout, yin, rs.p, v.p, twored ? rt.p : nullptr,
                                  partials2.p, stream);
      if (e != hipSuccess) return hipfail(e, "update x r (1)");
      te(T_BLAS, t0);
      // y = M^{-1} r ; t = A y ; <t,r>, <t,t> (twored: and <t,rt>)
      const double *yin2 = rs.p;
      if (fuse) {
        if ((rc = ilu_from1(rs.p, y2p))) return rc;
        yin2 = y2p;
      } else if (prec != PNP_PREC_NONE) {
        if ((rc = precond(prec, rs.p, y.p))) return rc;
        yin2 = y.p;
      }
      if ((rc = halo_spmv(const_cast<double *>(yin2), t.p, twored ? 4 : 2, rs.p, rt.p, &nsp)))
        return rc;
      if (twored) {
        if ((rc = reduce_derive2(nsp, 3, fuse ? npu : np, 2, 32))) return rc;
        // x += omega y ; r -= omega t ; ||r||^2 into partials2, tested at the next h (stage 31)
        t0 = tb(T_BLAS);
        e = pnp::launch_update_xr(n, S.p, 1, zout, yin2, rs.p, t.p, nullptr, partials2.p, stream);
        if (e != hipSuccess) return hipfail(e, "update x r (2)");
        te(T_BLAS, t0);
        pending_np = np;
      } else {
        if ((rc = reduce_derive2(nsp, 2, fuse ? npu : np, 1, 23))) return rc;
        // x += omega y ; r -= omega t ; ||r||, <rt, r>
        t0 = tb(T_BLAS);
        e = pnp::launch_update_xr(n, S.p, 1, zout, yin2, rs.p, t.p, rt.p, partials.p, stream,
                                  xdefer ? yin : nullptr);
        if (e != hipSuccess) return hipfail(e, "update x r (2)");
        if ((rc = reduce_derive(np, 2, 4))) return rc;
        te(T_BLAS, t0);
      }
      if (debug_trace) {
        e = hipMemcpyAsync(hS, S.p, sizeof(pnp::Scalars), hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        std::fprintf(stderr,
                     "bicgstab it=%d it_half=%.1f rho=%.6e rho_new=%.6e alpha=%.6e omega=%.6e "
                     "h=%.6e norm=%.6e done=%d bd=%d\n",
                     k + 1, hS->it_half, hS->rho, hS->rho_new, hS->alpha, hS->omega, hS->h,
                     hS->norm, hS->done, hS->breakdown);
      }
      return PNP_OK;
    };
    // the iterations between two polls of the device scalars (every `check`): eagerly, or as one
    // hipGraph replay (small systems, where launching ~20 kernels per iteration from the host
    // costs more than running them: PNP_OPT_GRAPH)
    bool graphs = use_graphs() && !dist && !twored && !debug_trace && !timing &&
                  prec != PNP_PREC_AMG && !graphs_failed;
    for (int k = 0; k < maxit;) {
      const int kend = std::min(maxit, (k / check + 1) * check);  // next poll
      if (k == 0) {
        if ((rc = body(0))) return rc;
        k = 1;
      }
      // whole graph blocks of glen iterations (one captured graph per block length, replayed as
      // often as the poll interval holds it), the remainder eagerly; a capture or instantiation
      // failure turns graphs off for the rest of the solve (eager launches, same results)
      const int glen = std::min(check, 16);
      while (graphs && glen > 1 && kend - k >= glen) {
        const GraphKey key{glen, prec, fuse ? 1 : 0, nf, pat, f32_now() + (ilu_y32() ? 4 : 0),
                           ilu_flow_opt * 4 + (nat_flow_opt + 1), zout, dl.dmask, graph_epoch};
        bool captured = true;
        rc = graph_run(key, [&]() -> int {
          for (int i = 0; i < key.count; i++)
            if (int r2 = body(1)) return r2;
          return PNP_OK;
        }, &captured);
        if (rc && !captured) {  // the graph path failed before anything ran: eager from here
          graphs_failed = true;
          graphs = false;
          break;
        }
        if (rc) return rc;
        k += glen;
      }
      for (; k < kend; k++)
        if ((rc = body(k))) return rc;
      e = hipMemcpyAsync(hS, S.p, sizeof(pnp::Scalars), hipMemcpyDeviceToHost, stream);
      if (e == hipSuccess) e = hipStreamSynchronize(stream);
      if (e != hipSuccess) return hipfail(e, "bicgstab poll");
      if (hS->done) break;
    }
    if (twored && pending_np > 0 && (rc = reduce_derive(pending_np, 1, 33, true))) return rc;
    e = hipMemcpyAsync(hS, S.p, sizeof(pnp::Scalars), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "bicgstab result");
    if (prec == PNP_PREC_SSOR_NATURAL && (rc = nat_check())) return rc;
    if (prec == PNP_PREC_ILU0 && (rc = ilu_flow_check())) return rc;
    double it = std::min(double(maxit), hS->it_half);
    res.converged = hS->done == 1 ? 1 : 0;
    res.breakdown = hS->breakdown;
    res.it_half = it;
    res.iterations = int(std::ceil(it));
    res.defect0 = hS->norm0;
    res.defect = hS->norm;
    res.reduction = hS->norm0 > 0 ? hS->norm / hS->norm0 : 0.0;
    res.elapsed = now_s() - t_start;
    return PNP_OK;
  }

  // ISTL CGSolver on J zout = bdev (owned rows), zout zero start; device-resident scalars
  // (derive stages 10-14).  iterations = matrix-vector products.
  int cg(const double *bdev, double *zout, const pnp_solve_opts &o, pnp_solve_result &res) {
    if (!assembled) return fail(PNP_E_STATE, "no Jacobian assembled");
    double t_start = now_s();
    long long n = nown();
    int np = pnp::blas_nparts(n);
    int prec = o.prec, nsp = 0, rc;
    hipError_t e = hipMemsetAsync(zout, 0, sizeof(double) * n, stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(rs.p, bdev, sizeof(double) * n, hipMemcpyDeviceToDevice, stream);
    if (e != hipSuccess) return hipfail(e, "cg init");
    pnp::Scalars &init = hS[2];
    std::memset(&init, 0, sizeof init);
    init.reduction = o.reduction;
    e = hipMemcpyAsync(S.p, &init, sizeof init, hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return hipfail(e, "cg scalars");
    if ((e = pnp::launch_dot(n, rs.p, rs.p, 0, partials.p, stream)) != hipSuccess)
      return hipfail(e, "cg norm0");
    if ((rc = reduce_derive(np, 1, 10))) return rc;
    if ((rc = precond(prec, rs.p, p.p))) return rc;  // p = M^{-1} r
    if ((e = pnp::launch_dot(n, p.p, rs.p, 0, partials.p, stream)) != hipSuccess)
      return hipfail(e, "cg rho");
    if ((rc = reduce_derive(np, 1, 11))) return rc;
    int check = o.check_every > 0 ? o.check_every : 8;
    for (int k = 0; k < o.maxit; k++) {
      if ((rc = halo_spmv(p.p, v.p, 1, p.p, nullptr, &nsp))) return rc;
      hipEvent_t t0 = nullptr;
      if ((rc = reduce_derive(nsp, 1, 12))) return rc;
      t0 = tb(T_BLAS);
      e = pnp::launch_update_xr(n, S.p, 0, zout, p.p, rs.p, v.p, nullptr, partials.p, stream);
      if (e != hipSuccess) return hipfail(e, "cg update");
      if ((rc = reduce_derive(np, 1, 13))) return rc;
      te(T_BLAS, t0);
      if ((k + 1) % check == 0 || k + 1 == o.maxit) {
        e = hipMemcpyAsync(hS, S.p, sizeof(pnp::Scalars), hipMemcpyDeviceToHost, stream);
        if (e == hipSuccess) e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hipfail(e, "cg poll");
        if (hS->done) break;
      }
      if ((rc = precond(prec, rs.p, y.p))) return rc;  // q = M^{-1} r
      t0 = tb(T_BLAS);
      if ((e = pnp::launch_dot(n, y.p, rs.p, 0, partials.p, stream)) != hipSuccess)
        return hipfail(e, "cg rho'");
      if ((rc = reduce_derive(np, 1, 14))) return rc;
      if ((e = pnp::launch_cg_update_p(n, S.p, y.p, p.p, stream)) != hipSuccess)
        return hipfail(e, "cg p");
      te(T_BLAS, t0);
    }
    e = hipMemcpyAsync(hS, S.p, sizeof(pnp::Scalars), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return hipfail(e, "cg result");
    if (o.prec == PNP_PREC_SSOR_NATURAL && (rc = nat_check())) return rc;
    res.converged = hS->done == 1 ? 1 : 0;
    res.breakdown = 0;
    res.iterations = hS->iter;
    res.it_half = hS->iter;
    res.defect0 = hS->norm0;
    res.defect = hS->norm;
    res.reduction = hS->norm0 > 0 ? hS->norm / hS->norm0 : 0.0;
    res.elapsed = now_s() - t_start;
    return PNP_OK;
  }

  // ---- reference-order mode (PNP_OPT_SEQ_ORDER) ------------------------------------------------
  // The reference's single-rank arithmetic in its order (seq_order.hip): element-order assembly
  // into the CSR view, ISTL's sequential mv / dot / updates, the scalar recurrences here in double.
  // External-layout vectors throughout.  P1, one rank.
  bool seq_on() const { return seq_opt && degree == 1 && !dist; }
  int nseq() const { return nf * mesh.nv; }
  enum { SQ_X = 0, SQ_R, SQ_Z, SQ_PREVU, SQ_P, SQ_V, SQ_T, SQ_Y, SQ_RT, SQ_B, SQ_N };
  double *sq(int k) { return seq_vec.p + size_t(k) * size_t(3 * mesh.nv); }

  int seq_build() {
    if (seq_built) return PNP_OK;
    const int nv = mesh.nv, nt = mesh.nt;
    std::vector<int> vptr(nv + 1, 0), vinc(size_t(3) * nt);
    for (int e = 0; e < nt; e++)
      for (int a = 0; a < 3; a++) vptr[mesh.tri[3 * e + a] + 1]++;
    for (int v = 0; v < nv; v++) vptr[v + 1] += vptr[v];
    std::vector<int> fill(vptr.begin(), vptr.end() - 1);
    for (int e = 0; e < nt; e++)  // ascending element index per vertex
      for (int a = 0; a < 3; a++) vinc[fill[mesh.tri[3 * e + a]]++] = e << 2 | a;
    int rc;
    if ((rc = upv(seq_tri, mesh.tri, "seq tri")) || (rc = upv(seq_xy, mesh.xy, "seq xy")) ||
        (rc = upv(seq_vptr, vptr, "seq vptr")) || (rc = upv(seq_vinc, vinc, "seq vinc")))
      return rc;
    hipError_t e;
    if ((e = seq_vec.alloc(size_t(SQ_N) * 3 * nv)) != hipSuccess ||
        (e = seq_dotv.alloc(2)) != hipSuccess || (e = seq_rl.alloc(size_t(9) * nt)) != hipSuccess ||
        (e = seq_rlo.alloc(size_t(9) * nt)) != hipSuccess ||
        (e = seq_rlt.alloc(size_t(9) * nt)) != hipSuccess ||
        (e = seq_jl.alloc(size_t(81) * nt)) != hipSuccess ||
        (e = seq_jlt.alloc(size_t(81) * nt)) != hipSuccess)
      return hipfail(e, "seq buffers");
    seq_built = true;
    return PNP_OK;
  }

  // per operator: constrained rows, alpha_boundary's terms per (element, local index) in the order
  // PDELab adds them into the element's local vector (the oracle's boundary_face statements: the
  // element's faces in DUNE's order (0,1), (0,2), (1,2), each a boundary intersection when its edge
  // is a boundary segment, run from its lower to its higher local vertex; 2-point Gauss; fields in
  // order; every basis function of the element at the face point; rl += scale * (j * phi * factor)),
  // frozen fields
  int seq_prepare() {
    int rc;
    if ((rc = seq_build())) return rc;
    if (seq_op_valid) return PNP_OK;
    if (seq_cextra) return fail(PNP_E_ARG, "PNP_OPT_SEQ_ORDER: pnp_op_args.c_extra is not supported");
    const int nt = mesh.nt, nl = 3 * nf;
    std::vector<std::vector<double>> terms(size_t(nt) * nl);
    const bool bnd = kind == PNP_OP_PNP || kind == PNP_OP_PNP_IMPLICIT_EULER || kind == PNP_OP_PB ||
                     kind == PNP_OP_POISSON;
    if (bnd) {
      std::unordered_map<long long, int> seg;  // edge -> its (first) boundary segment
      auto key = [](int a, int b) { return (long long)std::min(a, b) << 32 | unsigned(std::max(a, b)); };
      for (int b = 0; b < mesh.nb; b++) seg.emplace(key(mesh.bseg[2 * b], mesh.bseg[2 * b + 1]), b);
      static const int kFaceV[3][2] = {{0, 1}, {0, 2}, {1, 2}};
      static const double corner[3][2] = {{0.0, 0.0}, {1.0, 0.0}, {0.0, 1.0}};
      const double PI = params.pi;
      const double scale = kind == PNP_OP_PNP_IMPLICIT_EULER ? seq_dt : 1.0;
      const double gt[2] = {0.5 - 0.5 / std::sqrt(3.0), 0.5 + 0.5 / std::sqrt(3.0)};
      for (int e = 0; e < nt && !seg.empty(); e++)
        for (int k = 0; k < 3; k++) {
          const int ia = kFaceV[k][0], ib = kFaceV[k][1];
          const int va = mesh.tri[3 * e + ia], vb = mesh.tri[3 * e + ib];
          const auto it = seg.find(key(va, vb));
          if (it == seg.end()) continue;
          const pnp::Surface &S = params.surf[mesh.bgroup[it->second]];
          const double dx = mesh.xy[2 * vb] - mesh.xy[2 * va],
                       dy = mesh.xy[2 * vb + 1] - mesh.xy[2 * va + 1];
          const double len = std::sqrt(dx * dx + dy * dy);
          for (int q = 0; q < 2; q++) {
            double factor = 0.5 * len;
            const double y = mesh.xy[2 * va + 1] + gt[q] * dy;
            if (params.cylindrical) factor *= y * 2 * PI;
            const double lx = corner[ia][0] + (corner[ib][0] - corner[ia][0]) * gt[q];
            const double ly = corner[ia][1] + (corner[ib][1] - corner[ia][1]) * gt[q];
            const double phi[3] = {1.0 - lx - ly, lx, ly};
            for (int f = 0; f < nf; f++) {
              if (S.btype(f) == 0) continue;  // isDirichlet
              const double j = S.flux(f);
              for (int i = 0; i < 3; i++)
                terms[size_t(e) * nl + 3 * f + i].push_back(scale * (j * phi[i] * factor));
            }
          }
        }
    }
    std::vector<int> bptr(size_t(nt) * nl + 1, 0);
    std::vector<double> bval;
    for (size_t q = 0; q < terms.size(); q++) {
      bptr[q + 1] = bptr[q] + int(terms[q].size());
      bval.insert(bval.end(), terms[q].begin(), terms[q].end());
    }
    if ((rc = upv(seq_bptr, bptr, "seq boundary")) || (rc = upv(seq_bval, bval, "seq boundary")))
      return rc;
    std::vector<unsigned char> m(seq_mask_h.begin(), seq_mask_h.end());
    if ((rc = upv(seq_mask, m, "seq mask"))) return rc;
    if ((rc = upv(seq_phi, seq_phi_h, "seq phi")) || (rc = upv(seq_cp, seq_cp_h, "seq cp")) ||
        (rc = upv(seq_cm, seq_cm_h, "seq cm")) || (rc = upv(seq_xold, seq_xold_h, "seq x_old")))
      return rc;
    seq_op_valid = true;
    return PNP_OK;
  }
  pnp::SeqMesh seq_mesh() const {
    pnp::SeqMesh M;
    M.nv = mesh.nv;
    M.nt = mesh.nt;
    M.tri = seq_tri.p;
    M.vptr = seq_vptr.p;
    M.vinc = seq_vinc.p;
    M.xy = seq_xy.p;
    return M;
  }
  pnp::SeqOp seq_op() const {
    pnp::SeqOp P;
    P.kind = kind;
    P.nf = nf;
    P.cyl = params.cylindrical;
    P.pi = params.pi;
    P.l_b = params.l_b;
    P.c0 = params.c0;
    P.tau = params.tau;
    P.dt = seq_dt;
    P.z = seq_z;
    P.phi = seq_phi_h.empty() ? nullptr : seq_phi.p;
    P.cp = seq_cp_h.empty() ? nullptr : seq_cp.p;
    P.cm = seq_cm_h.empty() ? nullptr : seq_cm.p;
    P.x_old = seq_xold_h.empty() ? nullptr : seq_xold.p;
    return P;
  }
  // r = R(x), both external layout on the device (GridOperator::residual + constraints)
  int seq_residual(const double *x, double *r) {
    int rc;
    if ((rc = seq_prepare())) return rc;
    const bool old = kind == PNP_OP_PNP_IMPLICIT_EULER || kind == PNP_OP_DIFF_IMPLICIT_EULER;
    hipError_t e = pnp::launch_seq_element(seq_mesh(), seq_op(), x, 0, seq_rl.p, seq_rlt.p,
                                           seq_rlo.p, seq_jl.p, seq_jlt.p, seq_bptr.p, seq_bval.p,
                                           stream);
    if (e == hipSuccess)
      e = pnp::launch_seq_residual_gather(seq_mesh(), nf, old ? 1 : 0, seq_rl.p, seq_rlt.p,
                                          seq_rlo.p, seq_mask.p, r, stream);
    return e == hipSuccess ? PNP_OK : hipfail(e, "seq residual");
  }
  // the CSR view = J(x) (GridOperator::jacobian + constrained rows to identity); fd: PDELab's
  // NumericalJacobianVolume
  int seq_jacobian(const double *x, bool fd) {
    int rc;
    if ((rc = seq_prepare()) || (rc = csr_structure())) return rc;
    const bool onestep = kind == PNP_OP_PNP_IMPLICIT_EULER || kind == PNP_OP_DIFF_IMPLICIT_EULER;
    hipError_t e = pnp::launch_seq_element(seq_mesh(), seq_op(), x, fd ? 2 : 1, seq_rl.p,
                                           seq_rlt.p, seq_rlo.p, seq_jl.p, seq_jlt.p, seq_bptr.p,
                                           seq_bval.p, stream);
    if (e == hipSuccess)
      e = pnp::launch_seq_jacobian_gather(seq_mesh(), nf, seq_jl.p, onestep ? seq_jlt.p : nullptr,
                                          csr_rowptr.p, csr_col.p,
                                          seq_mask.p, csr_val.p, stream);
    if (e != hipSuccess) return hipfail(e, "seq jacobian");
    assembled = true;
    csr_vals_valid = true;  // the CSR view holds this Jacobian; the k-form matrix does not
    lu_valid = false;
    split_of = 0;
    amg_valid = false;
    return PNP_OK;
  }
  double seq_dot(const double *a, const double *b, int &rc) {
    rc = PNP_OK;
    double h = 0;
    hipError_t e = pnp::launch_seq_dot(nseq(), a, b, seq_dotv.p, stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&h, seq_dotv.p, 8, hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) rc = hipfail(e, "seq dot");
    return h;
  }
  // v = M^{-1} d with v zero on entry (ISTL's preconditioners from y = 0)
  int seq_prec(int prec, const double *d, double *v) {
    const int n = nseq();
    hipError_t e;
    if (prec == PNP_PREC_NONE || prec == PNP_PREC_JACOBI) {
      e = pnp::launch_seq_prec_diag(n, prec == PNP_PREC_JACOBI, d, csr_diag.p, csr_val.p, v, stream);
    } else {  // SSOR_NATURAL: the natural-order sweep on the CSR view (internal positions)
      e = pnp::launch_gather_ext(L.n_owned, nf, mesh.nv, d_l2g.p, d, nat_di.p, stream);
      if (e == hipSuccess) e = nat_sweep(nat_di.p, nat_vi.p);
      if (e == hipSuccess) e = pnp::launch_scatter_ext(L.n_owned, nf, mesh.nv, d_l2g.p, nat_vi.p, v, stream);
    }
    return e == hipSuccess ? PNP_OK : hipfail(e, "seq preconditioner");
  }
  // ISTL BiCGSTABSolver::apply in the oracle's statements (oracle/pnp_oracle.c orc_bicgstab):
  // x (zero start) and b (overwritten by the residual), external layout on the device
  int seq_bicgstab(int prec, double reduction, int maxit, double *x, double *b,
                   pnp_solve_result &res) {
    const double EPSILON = 1e-80;
    const int n = nseq();
    double *r = b, *p = sq(SQ_P), *v = sq(SQ_V), *t = sq(SQ_T), *y = sq(SQ_Y), *rt = sq(SQ_RT);
    int rc = PNP_OK;
    hipError_t e = hipSuccess;
    auto ck = [&](hipError_t ee) {
      if (e == hipSuccess) e = ee;
    };
    for (double *q : {p, v, t, y}) ck(hipMemsetAsync(q, 0, sizeof(double) * n, stream));
    std::memset(&res, 0, sizeof res);
    ck(pnp::launch_seq_spmv(n, csr_rowptr.p, csr_col.p, csr_val.p, x, t, stream));  // r = b - A x
    ck(pnp::launch_seq_aymx(n, 1.0, r, t, stream));
    ck(hipMemcpyAsync(rt, r, sizeof(double) * n, hipMemcpyDeviceToDevice, stream));
    if (e != hipSuccess) return hipfail(e, "seq bicgstab");
    double norm = std::sqrt(seq_dot(r, r, rc)), norm_0 = norm;
    if (rc) return rc;
    double rho = 1, alpha = 1, omega = 1, rho_new = 0, beta, h;
    res.defect0 = norm_0;
    double it = 0;
    if (norm < reduction * norm_0 || norm < 1e-30) {
      res.converged = 1;
      res.defect = norm;
      return PNP_OK;
    }
    for (it = 0.5; it < maxit; it += .5) {
      rho_new = seq_dot(rt, r, rc);
      if (rc) return rc;
      if (std::fabs(rho) <= EPSILON) { res.breakdown = 1; break; }
      if (std::fabs(omega) <= EPSILON) { res.breakdown = 2; break; }
      if (it < 1) {
        ck(hipMemcpyAsync(p, r, sizeof(double) * n, hipMemcpyDeviceToDevice, stream));
      } else {
        beta = (rho_new / rho) * (alpha / omega);
        ck(pnp::launch_seq_bicg_p(n, beta, omega, p, v, r, stream));
      }
      ck(hipMemsetAsync(y, 0, sizeof(double) * n, stream));
      if (e != hipSuccess) return hipfail(e, "seq bicgstab");
      if ((rc = seq_prec(prec, p, y))) return rc;
      ck(pnp::launch_seq_spmv(n, csr_rowptr.p, csr_col.p, csr_val.p, y, v, stream));
      if (e != hipSuccess) return hipfail(e, "seq bicgstab");
      h = seq_dot(rt, v, rc);
      if (rc) return rc;
      if (std::fabs(h) < EPSILON) { res.breakdown = 3; break; }
      alpha = rho_new / h;
      ck(pnp::launch_seq_axpy2(n, alpha, x, y, r, v, stream));
      if (e != hipSuccess) return hipfail(e, "seq bicgstab");
      norm = std::sqrt(seq_dot(r, r, rc));
      if (rc) return rc;
      if (norm < reduction * norm_0) { res.converged = 1; break; }
      it += .5;
      ck(hipMemsetAsync(y, 0, sizeof(double) * n, stream));
      if (e != hipSuccess) return hipfail(e, "seq bicgstab");
      if ((rc = seq_prec(prec, r, y))) return rc;
      ck(pnp::launch_seq_spmv(n, csr_rowptr.p, csr_col.p, csr_val.p, y, t, stream));
      if (e != hipSuccess) return hipfail(e, "seq bicgstab");
      const double tr = seq_dot(t, r, rc);
      if (rc) return rc;
      const double tt = seq_dot(t, t, rc);
      if (rc) return rc;
      omega = tr / tt;
      ck(pnp::launch_seq_axpy2(n, omega, x, y, r, t, stream));
      if (e != hipSuccess) return hipfail(e, "seq bicgstab");
      rho = rho_new;
      norm = std::sqrt(seq_dot(r, r, rc));
      if (rc) return rc;
      if (norm < reduction * norm_0 || norm < 1e-30) { res.converged = 1; break; }
    }
    if (it > maxit) it = maxit;
    res.it_half = it;
    res.iterations = int(std::ceil(it));
    res.defect = norm;
    res.reduction = norm / norm_0;
    return PNP_OK;
  }
  // ISTL CGSolver::apply (orc_cg's statements)
  int seq_cg(int prec, double reduction, int maxit, double *x, double *b, pnp_solve_result &res) {
    const int n = nseq();
    double *r = b, *p = sq(SQ_P), *q = sq(SQ_V);
    int rc = PNP_OK;
    hipError_t e = hipSuccess;
    auto ck = [&](hipError_t ee) {
      if (e == hipSuccess) e = ee;
    };
    ck(hipMemsetAsync(p, 0, sizeof(double) * n, stream));
    ck(hipMemsetAsync(q, 0, sizeof(double) * n, stream));
    std::memset(&res, 0, sizeof res);
    ck(pnp::launch_seq_spmv(n, csr_rowptr.p, csr_col.p, csr_val.p, x, q, stream));
    ck(pnp::launch_seq_aymx(n, 1.0, r, q, stream));
    if (e != hipSuccess) return hipfail(e, "seq cg");
    const double def0 = std::sqrt(seq_dot(r, r, rc));
    if (rc) return rc;
    double def = def0;
    res.defect0 = def0;
    int it = 0;
    if (def0 < 1e-30) {
      res.converged = 1;
    } else {
      if ((rc = seq_prec(prec, r, p))) return rc;
      double rho = seq_dot(p, r, rc);
      if (rc) return rc;
      for (it = 1; it <= maxit; it++) {
        ck(pnp::launch_seq_spmv(n, csr_rowptr.p, csr_col.p, csr_val.p, p, q, stream));
        if (e != hipSuccess) return hipfail(e, "seq cg");
        const double pq = seq_dot(p, q, rc);
        if (rc) return rc;
        const double lambda = rho / pq;
        ck(pnp::launch_seq_axpy(n, lambda, x, p, stream));
        ck(pnp::launch_seq_aymx(n, lambda, r, q, stream));
        if (e != hipSuccess) return hipfail(e, "seq cg");
        def = std::sqrt(seq_dot(r, r, rc));
        if (rc) return rc;
        if (def < reduction * def0 || def < 1e-30) {
          res.converged = 1;
          break;
        }
        ck(hipMemsetAsync(q, 0, sizeof(double) * n, stream));
        if (e != hipSuccess) return hipfail(e, "seq cg");
        if ((rc = seq_prec(prec, r, q))) return rc;
        const double rho_new = seq_dot(q, r, rc);
        if (rc) return rc;
        const double beta = rho_new / rho;
        ck(pnp::launch_seq_cg_p(n, beta, p, q, stream));
        if (e != hipSuccess) return hipfail(e, "seq cg");
        rho = rho_new;
      }
      if (it > maxit) it = maxit;
    }
    res.it_half = it;
    res.iterations = it;
    res.defect = def;
    res.reduction = def0 > 0 ? def / def0 : 0.0;
    return PNP_OK;
  }
  int seq_krylov(const pnp_solve_opts &o, double *x, double *b, pnp_solve_result &res) {
    if (!assembled || !csr_vals_valid) return fail(PNP_E_STATE, "no Jacobian assembled");
    if (o.prec != PNP_PREC_NONE && o.prec != PNP_PREC_JACOBI && o.prec != PNP_PREC_SSOR_NATURAL)
      return fail(PNP_E_ARG, "PNP_OPT_SEQ_ORDER: preconditioner must be NONE, JACOBI or SSOR_NATURAL");
    double t0 = now_s();
    int rc;
    if (o.method == PNP_METHOD_CG)
      rc = seq_cg(o.prec, o.reduction, o.maxit, x, b, res);
    else if (o.method == PNP_METHOD_BICGSTAB)
      rc = seq_bicgstab(o.prec, o.reduction, o.maxit, x, b, res);
    else
      return fail(PNP_E_ARG, "unknown solver method");
    if (!rc && o.prec == PNP_PREC_SSOR_NATURAL) rc = nat_check();
    res.elapsed = now_s() - t0;
    return rc;
  }

  // the linear solver selected by o.method
  int krylov(const double *bdev, double *zout, const pnp_solve_opts &o, pnp_solve_result &res) {
    int rc;
    after_solve = true;
    if (o.method == PNP_METHOD_CG) {
      amg_symmetric = true;
      rc = cg(bdev, zout, o, res);
    } else if (o.method == PNP_METHOD_BICGSTAB) {
      amg_symmetric = false;
      rc = bicgstab(bdev, zout, o, res, 0);
    } else {
      return fail(PNP_E_ARG, "unknown solver method");
    }
    amg_symmetric = true;
    return rc;
  }
};

using pnp_ctx_t = pnp_ctx;

// host copy of kernels.h expand_k + mask_rows for the CSR export
static void expand_host(int pat, const double *K, unsigned dm, bool diag, double *B) {
  if (pat == pnp::kPatPnpFD) {
    pnp::expand_k<pnp::kPatPnpFD>(K, B);
    pnp::mask_rows<3, pnp::kPatPnpFD>(B, dm, diag);
  } else if (pat == pnp::kPatPnpIEFD) {
    pnp::expand_k<pnp::kPatPnpIEFD>(K, B);
    pnp::mask_rows<3, pnp::kPatPnpIEFD>(B, dm, diag);
  } else if (pat == pnp::kPatPnp) {
    pnp::expand_k<pnp::kPatPnp>(K, B);
    pnp::mask_rows<3, pnp::kPatPnp>(B, dm, diag);
  } else if (pat == pnp::kPatPnpIE) {
    pnp::expand_k<pnp::kPatPnpIE>(K, B);
    pnp::mask_rows<3, pnp::kPatPnpIE>(B, dm, diag);
  } else {
    pnp::expand_k<pnp::kPatScalar>(K, B);
    pnp::mask_rows<1, pnp::kPatScalar>(B, dm, diag);
  }
}

// ---------------------------------------------------------------------------------------------
// mesh / comm
// ---------------------------------------------------------------------------------------------
extern "C" int pnp_mesh_read_gmsh(const char *path, pnp_mesh_buf **out) {
  if (!path || !out) return PNP_E_ARG;
  auto mb = std::make_unique<pnp_mesh_buf>();
  std::string err;
  if (!pnp::read_gmsh(path, mb->m, err)) {
    g_err = err;
    return err.rfind("cannot open", 0) == 0 ? PNP_E_IO : PNP_E_MESH;
  }
  *out = mb.release();
  return PNP_OK;
}

static bool mesh_from_view(const pnp_mesh *in, pnp::Mesh &m, std::string &err) {
  if (!in || in->nv <= 0 || in->nt <= 0 || !in->coords || !in->tri || in->nbseg < 0 ||
      (in->nbseg > 0 && (!in->bseg || !in->bseg_group))) {
    err = "invalid pnp_mesh";
    return false;
  }
  m.nv = in->nv;
  m.nt = in->nt;
  m.nb = in->nbseg;
  m.xy.assign(in->coords, in->coords + 2 * size_t(in->nv));
  m.tri.assign(in->tri, in->tri + 3 * size_t(in->nt));
  m.bseg.assign(in->bseg, in->bseg + 2 * size_t(in->nbseg));
  m.bgroup.assign(in->bseg_group, in->bseg_group + size_t(in->nbseg));
  return pnp::validate(m, err);
}

extern "C" int pnp_mesh_refine(const pnp_mesh *in, int32_t k, pnp_mesh_buf **out) {
  if (!out || k < 0) return PNP_E_ARG;
  pnp::Mesh m;
  std::string err;
  if (!mesh_from_view(in, m, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  auto mb = std::make_unique<pnp_mesh_buf>();
  mb->m = pnp::refine(m, k);
  *out = mb.release();
  return PNP_OK;
}

extern "C" int pnp_mesh_from_geo(const char *path, double size_scale, pnp_mesh_buf **out) {
  if (!path || !out || !(size_scale > 0)) return PNP_E_ARG;
  pnp::GeoModel g;
  std::string err;
  if (!pnp::read_geo(path, g, err)) {
    g_err = err;
    return err.rfind("cannot open", 0) == 0 ? PNP_E_IO : PNP_E_MESH;
  }
  auto mb = std::make_unique<pnp_mesh_buf>();
  if (!pnp::mesh_geo(g, size_scale, mb->m, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  *out = mb.release();
  return PNP_OK;
}

extern "C" int pnp_mesh_write_gmsh(const pnp_mesh *in, const char *path) {
  if (!path) return PNP_E_ARG;
  pnp::Mesh m;
  std::string err;
  if (!mesh_from_view(in, m, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  if (!pnp::write_gmsh(path, m, err)) {
    g_err = err;
    return PNP_E_IO;
  }
  return PNP_OK;
}

extern "C" int pnp_mesh_view(const pnp_mesh_buf *mb, pnp_mesh *view) {
  if (!mb || !view) return PNP_E_ARG;
  view->nv = mb->m.nv;
  view->coords = mb->m.xy.data();
  view->nt = mb->m.nt;
  view->tri = mb->m.tri.data();
  view->nbseg = mb->m.nb;
  view->bseg = mb->m.bseg.data();
  view->bseg_group = mb->m.bgroup.data();
  return PNP_OK;
}

extern "C" void pnp_mesh_free(pnp_mesh_buf *m) { delete m; }

extern "C" const char *pnp_last_error(const pnp_ctx *ctx) {
  return ctx ? ctx->err.c_str() : g_err.c_str();
}

extern "C" int pnp_rccl_unique_id(void *out128) {
  if (!out128) return PNP_E_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) {
    g_err = "ncclGetUniqueId failed";
    return PNP_E_RCCL;
  }
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  std::memcpy(out128, &id, 128);
  return PNP_OK;
}

// ---------------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------------
static void params_from(const pnp_params *pp, pnp::Params &P) {
  P.l_b = pp->l_b;
  P.c0 = pp->c0;
  P.tau = pp->tau;
  P.pi = pp->pi;
  P.cylindrical = pp->cylindrical;
  P.surf.resize(pp->n_surfaces);
  for (int i = 0; i < pp->n_surfaces; i++) {
    const pnp_surface &s = pp->surfaces[i];
    pnp::Surface &d = P.surf[i];
    d.cb = s.coulomb_btype;
    d.cflux = s.coulomb_flux;
    d.cpot = s.coulomb_potential;
    d.pb = s.plus_btype;
    d.pflux = s.plus_flux;
    d.pconc = s.plus_concentration;
    d.mb = s.minus_btype;
    d.mflux = s.minus_flux;
    d.mconc = s.minus_concentration;
  }
}

#define CK(expr, what)                                 \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return c->hipfail(e_, what); \
  } while (0)

extern "C" int pnp_create(const pnp_mesh *mesh, const pnp_params *params, int32_t device,
                          const pnp_comm *comm, pnp_ctx **out) {
  return pnp_create_pk(mesh, params, 1, device, comm, out);
}

extern "C" int pnp_create_pk(const pnp_mesh *mesh, const pnp_params *params, int32_t degree,
                             int32_t device, const pnp_comm *comm, pnp_ctx **out) {
  if (degree < 1 || degree > 3) {
    g_err = "pnp_create_pk: degree must be 1, 2 or 3 (PDEGREE)";
    return PNP_E_ARG;
  }
  if (!mesh || !params || !out) {
    g_err = "pnp_create: null argument";
    return PNP_E_ARG;
  }
  if (params->n_surfaces < 0 || (params->n_surfaces > 0 && !params->surfaces)) {
    g_err = "pnp_create: invalid surfaces";
    return PNP_E_ARG;
  }
  auto c = std::make_unique<pnp_ctx>();
  std::string err;
  if (!mesh_from_view(mesh, c->mesh, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  for (int s = 0; s < c->mesh.nb; s++)
    if (c->mesh.bgroup[s] < 0 || c->mesh.bgroup[s] >= params->n_surfaces) {
      g_err = "boundary segment " + std::to_string(s) + " has physical group " +
              std::to_string(c->mesh.bgroup[s]) + " but only " +
              std::to_string(params->n_surfaces) + " surfaces are configured";
      return PNP_E_ARG;
    }
  params_from(params, c->params);
  if (comm && comm->size > 1) {
    c->rank = comm->rank;
    c->nranks = comm->size;
    if (comm->rank < 0 || comm->rank >= comm->size ||
        (!comm->rccl_unique_id && !comm->local_group && !comm->host)) {
      g_err = "invalid pnp_comm (need an RCCL unique id, a local group or a host transport)";
      return PNP_E_ARG;
    }
  }
  c->degree = degree;
  if (degree > 1) {  // the layout is built on the node graph of the P_k space
    if (!pnp::validate(c->mesh, err) || !pnp::build_pk_space(c->mesh, degree, c->pks, err)) {
      g_err = err;
      return PNP_E_MESH;
    }
    c->tmesh = std::move(c->mesh);
    c->mesh = pnp::pk_node_mesh(c->pks);
    if (!pnp::pk_adjacency(c->tmesh, c->pks, c->fans, err)) {
      g_err = err;
      return PNP_E_MESH;
    }
  } else if (!pnp::build_fans(c->mesh, c->fans, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  std::vector<int> part;
  pnp::rcb_partition(c->mesh, c->nranks, part);
  {  // every rank computes the same partition: all of them fail here, before any collective or
     // group barrier, when one part is empty (more ranks than vertices)
    std::vector<int> cnt(c->nranks, 0);
    for (int p : part) cnt[p]++;
    for (int r = 0; r < c->nranks; r++)
      if (cnt[r] == 0) {
        g_err = "partition: rank " + std::to_string(r) + " of " + std::to_string(c->nranks) +
                " owns no vertices (the mesh has " + std::to_string(c->mesh.nv) + ")";
        return PNP_E_MESH;
      }
  }
  if (!pnp::build_local_layout(c->mesh, c->fans, part, c->rank, c->nranks, c->L, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    g_err = std::string("hipSetDevice: ") + hipGetErrorString(e);
    return PNP_E_HIP;
  }
  e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    g_err = std::string("hipStreamCreate: ") + hipGetErrorString(e);
    return PNP_E_HIP;
  }
  if (comm && comm->rccl_unique_id && (c->nranks > 1 || comm->size == 1)) {
    ncclUniqueId id;
    std::memcpy(&id, comm->rccl_unique_id, sizeof id);
    ncclResult_t nr = ncclCommInitRank(&c->comm, c->nranks, id, c->rank);
    if (nr != ncclSuccess) {
      g_err = std::string("ncclCommInitRank failed: ") + ncclGetErrorString(nr) + " (" +
              ncclGetLastError(nullptr) + ")";
      return PNP_E_RCCL;
    }
  }
  c->dist = c->nranks > 1 || c->comm != nullptr;
  pnp::LocalLayout &L = c->L;
  int nloc = L.n_owned + L.n_ghost;
  std::vector<double> xy(2 * size_t(nloc));
  for (int i = 0; i < nloc; i++) {
    xy[2 * size_t(i)] = c->mesh.xy[2 * size_t(L.l2g[i])];
    xy[2 * size_t(i) + 1] = c->mesh.xy[2 * size_t(L.l2g[i]) + 1];
  }
  pnp_ctx *cp = c.get();
  auto up = [&](auto &buf, const auto &vec, const char *what) -> int {
    hipError_t e2 = buf.alloc(vec.size());
    if (e2 == hipSuccess && !vec.empty())
      e2 = hipMemcpy(buf.p, vec.data(), sizeof(vec[0]) * vec.size(), hipMemcpyHostToDevice);
    if (e2 != hipSuccess) return cp->hipfail(e2, what);
    return PNP_OK;
  };
  int rc;
  // triangular split of the owned-column pattern (DevLayout l*/u*).  Lane order (PNP_SPLIT_SORT,
  // default on): inside each 64-row chunk, and inside each colour's segment of it, the rows are
  // stored longest-first in each of L and U, so a slot plane's padding is a tail of lanes that
  // issue no loads (config 3: 17.8 % of the split slots are padding); position p = 64 ch + lane
  // holds row 64 ch + lperm[p] in L and 64 ch + uperm[p] in U.  A row's own arithmetic and slot
  // order are unchanged, so every result is bitwise the identity order's.
  const int no = L.n_owned, npos = 64 * L.nchunks;
  std::vector<int> nlr(npos, 0), nur(npos, 1);
  for (int row = 0; row < no; row++) {
    const int ch = row / 64, ln = row % 64, len = int(L.rowmeta[row] & 63);
    for (int sl = 1; sl < len; sl++) {
      const int j = L.colidx[size_t(L.chunk_off[ch]) + 64 * sl + ln];
      // ghost and same-colour columns are outside the sweeps (mesh.cc absorb_top)
      if (j >= no || j == row || L.rowcolor[j] == L.rowcolor[row]) continue;
      (j < row ? nlr[row] : nur[row])++;
    }
  }
  std::vector<uint8_t> lperm(npos), uperm(npos), lpinv(npos), upinv(npos), llen8(npos, 0),
      ulen8(npos, 0), ldl(npos);
  const bool sort_lanes = [] {
    const char *e = getenv("PNP_SPLIT_SORT");
    return !(e && e[0] == '0');
  }();
  for (int ch = 0; ch < L.nchunks; ch++) {
    for (int ln = 0; ln < 64; ln++) lperm[64 * ch + ln] = uperm[64 * ch + ln] = uint8_t(ln);
    for (int a0 = 64 * ch; a0 < std::min(no, 64 * ch + 64);) {  // colour segments
      int a1 = a0 + 1;
      while (a1 < std::min(no, 64 * ch + 64) && L.rowcolor[a1] == L.rowcolor[a0]) a1++;
      if (sort_lanes) {
        std::vector<int> ord(a1 - a0);
        for (int k = 0; k < a1 - a0; k++) ord[k] = a0 + k;
        std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return nlr[x] > nlr[y]; });
        for (int k = 0; k < a1 - a0; k++) lperm[a0 + k] = uint8_t(ord[k] - 64 * ch);
        for (int k = 0; k < a1 - a0; k++) ord[k] = a0 + k;
        std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return nur[x] > nur[y]; });
        for (int k = 0; k < a1 - a0; k++) uperm[a0 + k] = uint8_t(ord[k] - 64 * ch);
      }
      a0 = a1;
    }
  }
  auto rowL = [&](int pos) { return 64 * (pos / 64) + lperm[pos]; };
  auto rowU = [&](int pos) { return 64 * (pos / 64) + uperm[pos]; };
  for (int pos = 0; pos < npos; pos++) {
    lpinv[rowL(pos)] = uint8_t(pos % 64);
    upinv[rowU(pos)] = uint8_t(pos % 64);
  }
  c->lslots_live = c->uslots_live = 0;
  for (int pos = 0; pos < npos; pos++) {
    llen8[pos] = uint8_t(nlr[rowL(pos)]);
    ulen8[pos] = uint8_t(nur[rowU(pos)]);
    ldl[pos] = upinv[rowL(pos)];
    if (rowL(pos) < no) c->lslots_live += nlr[rowL(pos)];
    if (rowU(pos) < no) c->uslots_live += nur[rowU(pos)];
  }
  std::vector<int> lcl(L.nchunks), lco(L.nchunks + 1, 0), ucl(L.nchunks), uco(L.nchunks + 1, 0);
  for (int ch = 0; ch < L.nchunks; ch++) {
    int ml = 0, mu = 1;
    for (int row = 64 * ch; row < std::min(no, 64 * ch + 64); row++) {
      ml = std::max(ml, nlr[row]);
      mu = std::max(mu, nur[row]);
    }
    lcl[ch] = ml;
    ucl[ch] = mu;
    lco[ch + 1] = lco[ch] + 64 * ml;
    uco[ch + 1] = uco[ch] + 64 * mu;
  }
  std::vector<int> lcol(lco[L.nchunks]), lsrc(lco[L.nchunks], -1), ucol(uco[L.nchunks]),
      usrc(uco[L.nchunks], -1);
  for (int ch = 0; ch < L.nchunks; ch++)
    for (int ln = 0; ln < 64; ln++) {
      const int p = 64 * ch + ln, rl = rowL(p), ru = rowU(p);
      for (int sl = 0; sl < lcl[ch]; sl++) lcol[size_t(lco[ch]) + 64 * sl + ln] = rl;
      for (int sl = 0; sl < ucl[ch]; sl++) ucol[size_t(uco[ch]) + 64 * sl + ln] = ru;
      if (p >= no) continue;
      for (int side = 0; side < 2; side++) {  // 0: L at this position (row rl), 1: U (row ru)
        const int row = side ? ru : rl, rch = row / 64, rln = row % 64;
        const int len = int(L.rowmeta[row] & 63);
        int kl = 0, ku = 1;
        if (side) usrc[size_t(uco[ch]) + ln] = row << 6;  // slot 0: the diagonal block
        for (int sl = 1; sl < len; sl++) {
          const int j = L.colidx[size_t(L.chunk_off[rch]) + 64 * sl + rln];
          if (j >= no || j == row || L.rowcolor[j] == L.rowcolor[row]) continue;
          if (j < row) {
            if (!side) {
              lcol[size_t(lco[ch]) + 64 * kl + ln] = j;
              lsrc[size_t(lco[ch]) + 64 * kl + ln] = row << 6 | sl;
            }
            kl++;
          } else {
            if (side) {
              ucol[size_t(uco[ch]) + 64 * ku + ln] = j;
              usrc[size_t(uco[ch]) + 64 * ku + ln] = row << 6 | sl;
            }
            ku++;
          }
        }
      }
    }
  if ((rc = up(c->d_lperm, lperm, "lperm")) || (rc = up(c->d_uperm, uperm, "uperm")) ||
      (rc = up(c->d_lpinv, lpinv, "lpinv")) || (rc = up(c->d_upinv, upinv, "upinv")) ||
      (rc = up(c->d_llen, llen8, "llen")) || (rc = up(c->d_ulen, ulen8, "ulen")) ||
      (rc = up(c->d_ldl, ldl, "ldl"))) {
    g_err = c->err;
    return rc;
  }
  c->dl.lperm = c->d_lperm.p;
  c->dl.uperm = c->d_uperm.p;
  c->dl.lpinv = c->d_lpinv.p;
  c->dl.upinv = c->d_upinv.p;
  c->dl.llen = c->d_llen.p;
  c->dl.ulen = c->d_ulen.p;
  c->dl.ldl = c->d_ldl.p;
  if ((rc = up(c->d_lchunk_len, lcl, "lchunk_len")) || (rc = up(c->d_lchunk_off, lco, "lchunk_off")) ||
      (rc = up(c->d_lcolidx, lcol, "lcolidx")) || (rc = up(c->d_lsrc, lsrc, "lsrc")) ||
      (rc = up(c->d_uchunk_len, ucl, "uchunk_len")) || (rc = up(c->d_uchunk_off, uco, "uchunk_off")) ||
      (rc = up(c->d_ucolidx, ucol, "ucolidx")) || (rc = up(c->d_usrc, usrc, "usrc"))) {
    g_err = c->err;
    return rc;
  }
  {  // LDS-staged sweep lists (DevLayout lsx_* / usx_*): per colour, per 256-row block of the
     // colour, the distinct rows its L / U split slots couple to; per split position its list
     // position (0xFFFF for padding and the U diagonal slot)
    const int nc = int(L.color_ptr.size()) - 1;
    auto lists = [&](const std::vector<int> &cl, const std::vector<int> &co,
                     const std::vector<int> &cc, int s0, auto rowat, std::vector<int> &ptr,
                     std::vector<int> &lst, std::vector<uint16_t> &idx) -> bool {
      idx.assign(cc.size(), 0xFFFF);
      ptr.assign(1, 0);
      lst.clear();
      std::vector<int> cols;
      for (int c = 0; c < nc; c++) {
        const int a = L.color_ptr[c], b = L.color_ptr[c + 1];
        for (int r0 = a; r0 < b; r0 += 256) {
          const int r1 = std::min(b, r0 + 256);
          cols.clear();
          for (int p = r0; p < r1; p++) {  // positions; the row at p is rowat(p)
            const int ch = p / 64, ln = p % 64, row = rowat(p);
            for (int sl = s0; sl < cl[ch]; sl++) {
              const int j = cc[size_t(co[ch]) + 64 * sl + ln];
              if (j != row) cols.push_back(j);
            }
          }
          std::sort(cols.begin(), cols.end());
          cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
          if (cols.size() >= 0xFFFF) return false;
          for (int p = r0; p < r1; p++) {
            const int ch = p / 64, ln = p % 64, row = rowat(p);
            for (int sl = s0; sl < cl[ch]; sl++) {
              const size_t pos = size_t(co[ch]) + 64 * sl + ln;
              if (cc[pos] != row)
                idx[pos] = uint16_t(std::lower_bound(cols.begin(), cols.end(), cc[pos]) - cols.begin());
            }
          }
          lst.insert(lst.end(), cols.begin(), cols.end());
          ptr.push_back(int(lst.size()));
        }
      }
      return true;
    };
    std::vector<int> lp, ll, up2, ul;
    std::vector<uint16_t> li, ui;
    const bool ok = lists(lcl, lco, lcol, 0, rowL, lp, ll, li) &&
                    lists(ucl, uco, ucol, 1, rowU, up2, ul, ui);
    int mx = 0;
    for (size_t k = 0; ok && k + 1 < lp.size(); k++) mx = std::max(mx, lp[k + 1] - lp[k]);
    for (size_t k = 0; ok && k + 1 < up2.size(); k++) mx = std::max(mx, up2[k + 1] - up2[k]);
    if (ok && nc <= 256 && size_t(mx) * 3 * 8 <= 64 * 1024) {
      if ((rc = up(c->d_lsx_ptr, lp, "lsx ptr")) || (rc = up(c->d_lsx_list, ll, "lsx list")) ||
          (rc = up(c->d_lsx_idx, li, "lsx idx")) || (rc = up(c->d_usx_ptr, up2, "usx ptr")) ||
          (rc = up(c->d_usx_list, ul, "usx list")) || (rc = up(c->d_usx_idx, ui, "usx idx"))) {
        g_err = c->err;
        return rc;
      }
      c->dl.lsx_ptr = c->d_lsx_ptr.p;
      c->dl.lsx_list = c->d_lsx_list.p;
      c->dl.lsx_idx = c->d_lsx_idx.p;
      c->dl.usx_ptr = c->d_usx_ptr.p;
      c->dl.usx_list = c->d_usx_list.p;
      c->dl.usx_idx = c->d_usx_idx.p;
      c->dl.sx_max = mx;
      // host copies for the one-launch ILU(0) application's dependency lists (ilu_flow_build)
      c->h_posrowL.resize(npos);
      c->h_posrowU.resize(npos);
      for (int pos = 0; pos < npos; pos++) {
        c->h_posrowL[pos] = rowL(pos);
        c->h_posrowU[pos] = rowU(pos);
      }
      c->h_lsx_ptr = lp;
      c->h_lsx_list = ll;
      c->h_usx_ptr = up2;
      c->h_usx_list = ul;
      c->ilu_flow[0].built = c->ilu_flow[1].built = false;
    }
  }
  {  // row-contiguous block offsets and columns of the owned rows (fused ILU(0) factorisation)
    std::vector<int> ro(L.n_owned + 1, 0), rcol;
    rcol.reserve(size_t(L.nblocks));
    for (int i = 0; i < L.n_owned; i++) {
      const int ch = i / pnp::kRows, ln = i % pnp::kRows, len = pnp::meta_len(L.rowmeta[i]);
      for (int sl = 0; sl < len; sl++)
        rcol.push_back(L.colidx[size_t(L.chunk_off[ch]) + 64 * size_t(sl) + ln]);
      ro[i + 1] = ro[i] + len;
    }
    if ((rc = up(c->d_rowoff, ro, "rowoff")) || (rc = up(c->d_rowcol, rcol, "rowcol"))) {
      g_err = c->err;
      return rc;
    }
  }
  {  // spatial block order (DevLayout::blkmap) for the whole-matrix kernels (assembly, SpMV):
     // each XCD takes one spatial slice of every colour, so the neighbour gathers of its rows
     // share its L2.  With the gather-all assembly it pays 72.7 -> 58.8 us (the pipelined walk
     // was latency-bound and did not see it; SpMV and sweeps neutral,
     // profiles/r01/ab_blkmap_gather_all.log).  PNP_BLKMAP=0 turns it off (A/B)
    const char *e = getenv("PNP_BLKMAP");
    if (!(e && atoi(e) == 0) && L.n_owned > 0) {
      int nblk = (L.n_owned + 255) / 256;
      std::vector<double> key(nblk);
      for (int b = 0; b < nblk; b++) {
        int r = 256 * b, cc = L.rowcolor[r];
        double lo = L.color_ptr[cc], hi = L.color_ptr[cc + 1];
        key[b] = (r - lo) / std::max(1.0, hi - lo);
      }
      std::vector<int> order(nblk);
      for (int b = 0; b < nblk; b++) order[b] = b;
      std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return key[a] < key[b]; });
      if ((rc = up(c->d_blkmap, order, "blkmap"))) {
        g_err = c->err;
        return rc;
      }
      c->dl.blkmap = c->d_blkmap.p;
    }
  }
  {  // boundary segments for the ion-flux observable
    const pnp::Mesh &mg = c->mesh;
    auto ekey = [](int a, int b) {
      if (a > b) std::swap(a, b);
      return (long long)a << 32 | (unsigned)b;
    };
    std::unordered_map<long long, int> opp;
    opp.reserve(size_t(mg.nb) * 2);
    for (int b = 0; b < mg.nb; b++) opp[ekey(mg.bseg[2 * b], mg.bseg[2 * b + 1])] = -1;
    for (int e = 0; e < mg.nt; e++)
      for (int k = 0; k < 3; k++) {
        auto it = opp.find(ekey(mg.tri[3 * e + k], mg.tri[3 * e + (k + 1) % 3]));
        if (it != opp.end() && it->second < 0) it->second = mg.tri[3 * e + (k + 2) % 3];
      }
    std::vector<int4> segs;
    for (int b = 0; b < mg.nb; b++) {
      const int a = mg.bseg[2 * b], cc = mg.bseg[2 * b + 1], lo = L.g2l[std::min(a, cc)];
      if (lo < 0 || lo >= L.n_owned) continue;  // another rank's segment
      const int o = opp[ekey(a, cc)];
      const int la = L.g2l[a], lc = L.g2l[cc], lop = o >= 0 ? L.g2l[o] : -1;
      if (la < 0 || lc < 0 || lop < 0) {
        g_err = "ion flux: the element of a boundary segment is not local";
        return PNP_E_MESH;
      }
      segs.push_back(make_int4(la, lc, lop, mg.bgroup[b]));
      c->fseg_group.push_back(mg.bgroup[b]);
    }
    if ((rc = up(c->d_fseg, segs, "flux segments"))) {
      g_err = c->err;
      return rc;
    }
  }
  c->dl.lchunk_len = c->d_lchunk_len.p;
  c->dl.lchunk_off = c->d_lchunk_off.p;
  c->dl.lcolidx = c->d_lcolidx.p;
  c->dl.uchunk_len = c->d_uchunk_len.p;
  c->dl.uchunk_off = c->d_uchunk_off.p;
  c->dl.ucolidx = c->d_ucolidx.p;
  if ((rc = up(c->d_chunk_len, L.chunk_len, "chunk_len")) ||
      (rc = up(c->d_chunk_off, L.chunk_off, "chunk_off")) ||
      (rc = up(c->d_colidx, L.colidx, "colidx")) || (rc = up(c->d_rowmeta, L.rowmeta, "rowmeta")) ||
      (rc = up(c->d_xy, xy, "xy")) || (rc = up(c->d_l2g, L.l2g, "l2g")) ||
      (rc = up(c->d_send_idx, L.send_idx, "send_idx")) ||
      (rc = up(c->d_color_idx, L.color_idx, "color_idx")) ||
      (rc = up(c->d_rowcolor, L.rowcolor, "rowcolor"))) {
    g_err = c->err;
    return rc;
  }
  {
    const char *e = getenv("PNP_XCD_REMAP");
    c->dl.xcd_remap = (e && atoi(e) == 1) ? 1 : 0;  // measured: off for assembly / SpMV
  }
  c->dl.n_owned = L.n_owned;
  c->dl.n_local = nloc;
  c->dl.nchunks = L.nchunks;
  c->dl.max_slots = L.chunk_len.empty() ? 0 : *std::max_element(L.chunk_len.begin(), L.chunk_len.end());
  c->dl.ncolors = int(L.color_ptr.size()) - 1;
  c->dl.chunk_len = c->d_chunk_len.p;
  c->dl.chunk_off = c->d_chunk_off.p;
  c->dl.colidx = c->d_colidx.p;
  c->dl.rowmeta = c->d_rowmeta.p;
  if (const char *ev = getenv("PNP_SPMV_LDS"); !(ev && atoi(ev) == 0)) {
    // per 256-row block: its distinct columns, and per slot the column's position among them
    const int nblk = (L.n_owned + 255) / 256;
    std::vector<int> uptr(nblk + 1, 0), ulist;
    std::vector<uint16_t> lidx(size_t(L.nslots), 0);
    std::vector<int> cols, uown(nblk, 0);
    int umax = 0, unmax = 0;
    bool fits = true;
    const bool own_last = [] {
      const char *e = getenv("PNP_LIST_OWN_LAST");
      return !(e && e[0] == '0');
    }();
    for (int b = 0; b < nblk && fits; b++) {
      cols.clear();
      const int r1 = std::min(L.n_owned, 256 * b + 256);
      for (int i = 256 * b; i < r1; i++) {
        const int ch = i / pnp::kRows, ln = i % pnp::kRows;
        for (int sl = 0; sl < L.chunk_len[ch]; sl++)
          cols.push_back(L.colidx[size_t(L.chunk_off[ch]) + 64 * size_t(sl) + ln]);
      }
      std::sort(cols.begin(), cols.end());
      cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
      if (cols.size() > 65535) fits = false;
      umax = std::max(umax, int(cols.size()));
      // columns that are only a row's own slot 0 last (PNP_LIST_OWN_LAST, default): the assembly
      // walk stages only the first uown[b] entries, the columns of slots >= 1 (fan neighbours; a
      // block's rows are mostly of one colour, so its own rows are rarely among them); the SpMV
      // stages all
      std::vector<int> npos(cols.size());
      int nn = 0;
      if (own_last) {
        std::vector<char> nb(cols.size(), 0);
        for (int i = 256 * b; i < r1; i++) {
          const int ch = i / pnp::kRows, ln = i % pnp::kRows;
          for (int sl = 1; sl < L.chunk_len[ch]; sl++) {
            const int j = L.colidx[size_t(L.chunk_off[ch]) + 64 * size_t(sl) + ln];
            if (j != i) nb[std::lower_bound(cols.begin(), cols.end(), j) - cols.begin()] = 1;
          }
        }
        for (size_t k = 0; k < cols.size(); k++)
          if (nb[k]) npos[k] = nn++;
        int no = nn;
        for (size_t k = 0; k < cols.size(); k++)
          if (!nb[k]) npos[k] = no++;
      } else {
        for (size_t k = 0; k < cols.size(); k++) npos[k] = int(k);
        nn = int(cols.size());
      }
      uown[b] = nn;
      unmax = std::max(unmax, nn);
      for (int i = 256 * b; i < r1; i++) {
        const int ch = i / pnp::kRows, ln = i % pnp::kRows;
        for (int sl = 0; sl < L.chunk_len[ch]; sl++) {
          const size_t pos = size_t(L.chunk_off[ch]) + 64 * size_t(sl) + ln;
          lidx[pos] = uint16_t(npos[std::lower_bound(cols.begin(), cols.end(), L.colidx[pos]) - cols.begin()]);
        }
      }
      std::vector<int> reord(cols.size());
      for (size_t k = 0; k < cols.size(); k++) reord[npos[k]] = cols[k];
      ulist.insert(ulist.end(), reord.begin(), reord.end());
      uptr[b + 1] = int(ulist.size());
    }
    if (fits && size_t(umax) * 3 * 8 <= 64 * 1024) {
      if ((rc = up(c->d_uptr, uptr, "uptr")) || (rc = up(c->d_ulist, ulist, "ulist")) ||
          (rc = up(c->d_lidx, lidx, "lidx")) || (rc = up(c->d_uown, uown, "uown"))) {
        g_err = c->err;
        return rc;
      }
      c->dl.uptr = c->d_uptr.p;
      c->dl.ulist = c->d_ulist.p;
      c->dl.lidx = c->d_lidx.p;
      c->dl.umax = umax;
      c->dl.uown = c->d_uown.p;
      c->dl.unmax = unmax;
    }
  }
  c->dl.xy = c->d_xy.p;
  c->dl.color_idx = c->d_color_idx.p;
  c->dl.rowcolor = c->d_rowcolor.p;
  // buffers
  size_t nv3 = 3 * size_t(nloc);
  auto al = [&](auto &buf, size_t n, const char *what) -> int {
    hipError_t e2 = buf.alloc(n);  // zeroed, and the zeroing finished (DBuf::alloc)
    if (e2 != hipSuccess) return cp->hipfail(e2, what);
    return PNP_OK;
  };
  if ((rc = al(c->vals, size_t(L.nslots) * 8, "vals")) ||
      (rc = al(c->lu, size_t(L.nslots) * 8, "lu")) ||
      (rc = al(c->lvals, c->d_lsrc.n * 8, "lvals")) || (rc = al(c->uvals, c->d_usrc.n * 8, "uvals")) ||
      (rc = al(c->tsgs, nv3, "sgs scratch")) || (rc = al(c->fluxx, nv3, "flux state")) ||
      (rc = al(c->fluxout, 2 * c->fseg_group.size() + 2, "flux out")) ||
      (rc = al(c->fluxred, 2 * 256, "flux reduce")) || (rc = al(c->x, nv3, "x")) ||
      (rc = al(c->r, nv3, "r")) || (rc = al(c->rs, nv3, "rs")) || (rc = al(c->z, nv3, "z")) || (rc = al(c->rt, nv3, "rt")) ||
      (rc = al(c->p, nv3, "p")) || (rc = al(c->v, nv3, "v")) || (rc = al(c->t, nv3, "t")) ||
      (rc = al(c->y, nv3, "y")) || (rc = al(c->y2, nv3, "y2")) ||
      (rc = al(c->ilu_y32buf, nv3, "ILU(0) intermediate")) || (rc = al(c->b, nv3, "b")) || (rc = al(c->prevu, nv3, "prevu")) ||
      (rc = al(c->ext, 3 * size_t(c->mesh.nv), "ext")) ||
      (rc = al(c->sendbuf, 3 * std::max<size_t>(1, L.send_idx.size()), "sendbuf")) ||
      // up to 3 partials per workgroup (SpMV mode 4) / 2 (updates with <rt, s>)
      (rc = al(c->partials,
               3 * std::max<size_t>(size_t(pnp::blas_nparts(3LL * nloc)),
                                    size_t(pnp::spmv_parts(L.n_owned))) + 64,
               "partials")) ||
      (rc = al(c->partials2,
               2 * std::max<size_t>(size_t(pnp::blas_nparts(3LL * nloc)),
                                    size_t(pnp::spmv_parts(L.n_owned))) + 64,
               "partials2")) ||
      (rc = al(c->S, 2, "scalars")) || (rc = al(c->redmw, pnp::kRedMwDoubles, "reduce ticket")) ||
      (rc = al(c->dmask, 3 * size_t(L.n_owned), "dmask")) ||
      (rc = al(c->cvec, 3 * size_t(L.n_owned), "cvec")) || (rc = al(c->aux0, nloc, "aux0")) ||
      (rc = al(c->aux1, nloc, "aux1"))) {
    g_err = c->err;
    return rc;
  }
  if ((e = hipHostMalloc(&c->hS, 3 * sizeof(pnp::Scalars))) != hipSuccess) {
    g_err = std::string("hipHostMalloc: ") + hipGetErrorString(e);
    return PNP_E_HIP;
  }
  if (c->dist) {  // halo-overlapped SpMV: interior / boundary 256-row blocks
    const char *ev = getenv("PNP_HALO_OVERLAP");
    if (!(ev && atoi(ev) == 0) && L.n_owned > 0) {
      const int nblk = (L.n_owned + 255) / 256;
      std::vector<int> order(nblk);
      if (c->d_blkmap.p) {
        CK(hipMemcpy(order.data(), c->d_blkmap.p, sizeof(int) * nblk, hipMemcpyDeviceToHost),
           "blkmap");
      } else {
        for (int b = 0; b < nblk; b++) order[b] = b;
      }
      std::vector<int> bi, bb;
      for (int b : order) {
        bool bnd = false;
        for (int i = 256 * b; i < std::min(L.n_owned, 256 * b + 256) && !bnd; i++) {
          const int ch = i / pnp::kRows, ln = i % pnp::kRows, len = pnp::meta_len(L.rowmeta[i]);
          for (int sl = 1; sl < len && !bnd; sl++)
            bnd = L.colidx[size_t(L.chunk_off[ch]) + 64 * size_t(sl) + ln] >= L.n_owned;
        }
        (bnd ? bb : bi).push_back(b);
      }
      if ((rc = up(c->d_blk_int, bi, "interior blocks")) || (rc = up(c->d_blk_bnd, bb, "boundary blocks"))) {
        g_err = c->err;
        return rc;
      }
      c->n_blk_int = int(bi.size());
      c->n_blk_bnd = int(bb.size());
      c->split_spmv = true;
      if (comm->rccl_unique_id) {
        if ((e = hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming)) != hipSuccess) {
          g_err = std::string("halo stream: ") + hipGetErrorString(e);
          return PNP_E_HIP;
        }
      }
    }
  }
  if (degree > 1 && (rc = c->pk_build())) {
    g_err = c->err;
    return rc;
  }
  if (c->nranks > 1 && !comm->rccl_unique_id && !comm->local_group) {  // host-staged transport
    if (!comm->host->exchange || !comm->host->allreduce_sum) {
      g_err = "pnp_host_transport: exchange and allreduce_sum are required";
      return PNP_E_ARG;
    }
    c->ht = *comm->host;
    const size_t ns = 3 * std::max<size_t>(1, L.send_idx.size());
    const size_t nr = 3 * std::max<size_t>(1, size_t(L.n_ghost));
    if ((e = hipHostMalloc(&c->h_send, sizeof(double) * ns)) != hipSuccess ||
        (e = hipHostMalloc(&c->h_recv, sizeof(double) * nr)) != hipSuccess) {
      g_err = std::string("host transport staging: ") + hipGetErrorString(e);
      return PNP_E_HIP;
    }
  }
  if (c->nranks > 1 && !comm->rccl_unique_id && comm->local_group) {  // join the in-process group
    std::shared_ptr<LocalGroup> g;
    {
      std::lock_guard<std::mutex> lk(g_groups_m);
      auto &slot = g_groups[comm->local_group];
      if (!slot || slot->size != c->nranks) {
        slot = std::make_shared<LocalGroup>();
        slot->size = c->nranks;
        slot->members.assign(c->nranks, nullptr);
        slot->host.assign(c->nranks, {});
      }
      g = slot;
      if (g->members[c->rank]) {
        g_err = "rank already present in local group";
        return PNP_E_ARG;
      }
      g->members[c->rank] = c.get();
    }
    c->lg = g;
    g->barrier();  // all ranks created before any collective
  }
  *out = c.release();
  return PNP_OK;
}

extern "C" void pnp_destroy(pnp_ctx *ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  if (ctx->lg) {
    std::lock_guard<std::mutex> lk(g_groups_m);
    ctx->lg->members[ctx->rank] = nullptr;
  }
  delete ctx;
}

extern "C" int pnp_get_info(pnp_ctx *c, pnp_info *info) {
  if (!c || !info) return PNP_E_ARG;
  std::memset(info, 0, sizeof *info);
  info->nv_global = c->mesh.nv;
  info->nv_owned = c->L.n_owned;
  info->nv_ghost = c->L.n_ghost;
  info->nfields = c->nf;
  info->ncolors = int(c->L.color_ptr.size()) - 1;
  info->nchunks = c->L.nchunks;
  info->max_slots = c->fans.max_slots;
  info->nranks = c->nranks;
  info->nblocks = c->L.nblocks;
  info->nnz_reduced = c->L.nblocks * (c->nvb ? c->nvb : 1);
  info->nslots = c->L.nslots;
  info->nks = c->nks;
  info->nvb = c->nvb;
  info->lslots = (int64_t)c->d_lsrc.n;
  info->uslots = (int64_t)c->d_usrc.n;
  info->ilu_f32 = c->ilu_f32;
  info->degree = c->degree;
  info->color_conflicts = c->L.conflicts;
  info->transport = c->comm ? 2 : c->lg ? 1 : c->host_tr() ? 3 : 0;
  info->nat_flow_applies = c->nat_flow_n;
  info->nat_level_applies = c->nat_level_n;
  info->ilu_flow_applies = c->ilu_flow_n;
  info->lslots_live = c->lslots_live;
  info->uslots_live = c->uslots_live;
  info->lsx_entries = (int64_t)c->h_lsx_list.size();
  info->usx_entries = (int64_t)c->h_usx_list.size();
  size_t b = 0;
  b += c->vals.n * 8 + (c->x.n + c->r.n + c->rs.n + c->z.n + c->rt.n + c->p.n + c->v.n + c->t.n + c->y.n +
                        c->y2.n + c->b.n + c->prevu.n + c->ext.n) * 8 + c->ilu_y32buf.n * 4;
  b += c->d_colidx.n * 4 + c->d_rowmeta.n * 8 + c->d_xy.n * 8;
  info->device_bytes = int64_t(b);
  return PNP_OK;
}

// ---------------------------------------------------------------------------------------------
// operators
// ---------------------------------------------------------------------------------------------
extern "C" int pnp_nfields(pnp_ctx *c) { return c ? c->nf : PNP_E_ARG; }

extern "C" int pnp_set_operator(pnp_ctx *c, const pnp_op_args *a) {
  if (!c || !a) return PNP_E_ARG;
  // no graphs_clear() here: the operator's pattern and mask pointer are in the graph key; a change
  // of the CSR view's pattern (SSOR_NATURAL, pnp_jacobian_csr_device) clears the graphs in
  // csr_structure(), which rebuilds the buffers they captured
  if (a->kind < PNP_OP_PNP || a->kind > PNP_OP_POISSON)
    return c->fail(PNP_E_ARG, "unknown operator kind");
  hipSetDevice(c->device);
  int kind = a->kind;
  const bool ie = kind == PNP_OP_PNP_IMPLICIT_EULER || kind == PNP_OP_DIFF_IMPLICIT_EULER;
  if (ie && !(a->dt > 0)) return c->fail(PNP_E_ARG, "implicit Euler needs dt > 0");
  if (ie && !a->x_old) return c->fail(PNP_E_ARG, "implicit Euler needs x_old");
  if ((kind == PNP_OP_DIFF || kind == PNP_OP_DIFF_IMPLICIT_EULER) &&
      (!a->phi || (a->field != 1 && a->field != 2)))
    return c->fail(PNP_E_ARG, "diffusion operator needs phi and field 1 or 2");
  if (kind == PNP_OP_POISSON && (!a->cp || !a->cm))
    return c->fail(PNP_E_ARG, "Poisson operator needs cp and cm");
  if (c->degree > 1 && (kind == PNP_OP_PNP || kind == PNP_OP_PNP_IMPLICIT_EULER))
    return c->fail(PNP_E_ARG,
                   "PnpOperator / PnpTOperator are P1 in the reference (Pk2DLocalFiniteElementMap<..., 1>, "
                   "src/stationary_pnp_from_pb.hh:206-208); P_k contexts take PB, Poisson and diffusion");
  c->kind = kind;
  c->fd_mode = false;  // the next Jacobian picks its form (set_fd)
  c->nf = (kind == PNP_OP_PNP || kind == PNP_OP_PNP_IMPLICIT_EULER) ? 3 : 1;
  c->pat = kind == PNP_OP_PNP ? pnp::kPatPnp
                              : (kind == PNP_OP_PNP_IMPLICIT_EULER ? pnp::kPatPnpIE : pnp::kPatScalar);
  c->nvb = pnp::popc9(c->pat);
  c->nks = pnp::nks_of(c->pat);
  c->assembled = false;
  c->lu_valid = false;
  c->split_of = 0;
  c->amg_valid = false;
  c->csr_vals_valid = false;
  // SELL padding slots point at the row itself and are never written by the assembly, so they
  // must hold zeros in the k-form layout of THIS operator (the SpMV multiplies them)
  CK(hipMemsetAsync(c->vals.p, 0, sizeof(double) * size_t(c->L.nslots) * c->nks, c->stream),
     "clear matrix");
  const pnp::Mesh &m = c->mesh;
  const pnp::LocalLayout &L = c->L;
  int nf = c->nf;
  // Dirichlet mask and constant load (Neumann flux of alpha_boundary), owned rows
  int field0 = (kind == PNP_OP_DIFF || kind == PNP_OP_DIFF_IMPLICIT_EULER) ? a->field : 0;
  std::vector<uint8_t> mask;
  if (c->degree > 1)
    pnp::pk_dirichlet_mask(c->tmesh, c->pks, c->params, nf, field0, mask);
  else
    pnp::dirichlet_mask(m, c->params, nf, field0, mask);
  std::vector<double> load(size_t(m.nv) * nf, 0.0);
  if (kind == PNP_OP_PNP || kind == PNP_OP_PNP_IMPLICIT_EULER || kind == PNP_OP_PB ||
      kind == PNP_OP_POISSON) {
    if (c->degree > 1)
      pnp::pk_neumann_load(c->tmesh, c->pks, c->params, nf, 0, load);
    else
      pnp::neumann_load(m, c->params, nf, 0, load);
    if (kind == PNP_OP_PNP_IMPLICIT_EULER)
      for (auto &v : load) v *= a->dt;
  }
  std::vector<uint8_t> lmask(size_t(L.n_owned) * nf);
  std::vector<double> lload(size_t(L.n_owned) * nf);
  for (int i = 0; i < L.n_owned; i++)
    for (int f = 0; f < nf; f++) {
      lmask[size_t(i) * nf + f] = mask[size_t(L.l2g[i]) * nf + f];
      lload[size_t(i) * nf + f] = load[size_t(L.l2g[i]) * nf + f];
      if (a->c_extra) lload[size_t(i) * nf + f] += a->c_extra[size_t(f) * m.nv + L.l2g[i]];
    }
  CK(hipMemcpy(c->dmask.p, lmask.data(), lmask.size(), hipMemcpyHostToDevice), "dmask");
  // the reference-order mode's copies (external layout, global vertex order)
  c->seq_op_valid = false;
  c->seq_dt = a->dt;
  c->seq_z = a->z;
  c->seq_cextra = a->c_extra != nullptr;
  c->seq_mask_h.assign(size_t(nf) * m.nv, 0);
  if (c->degree == 1)
    for (int g = 0; g < m.nv; g++)
      for (int f = 0; f < nf; f++) c->seq_mask_h[size_t(f) * m.nv + g] = mask[size_t(g) * nf + f];
  auto hcopy = [&](const double *h, size_t cnt, std::vector<double> &out) {
    if (h) out.assign(h, h + cnt); else out.clear();
  };
  const bool dk = kind == PNP_OP_DIFF || kind == PNP_OP_DIFF_IMPLICIT_EULER;
  hcopy(dk ? a->phi : nullptr, m.nv, c->seq_phi_h);
  hcopy(kind == PNP_OP_POISSON ? a->cp : nullptr, m.nv, c->seq_cp_h);
  hcopy(kind == PNP_OP_POISSON ? a->cm : nullptr, m.nv, c->seq_cm_h);
  hcopy(ie ? a->x_old : nullptr, size_t(nf) * m.nv, c->seq_xold_h);
  c->dl.dmask = c->dmask.p;
  c->hmask = lmask;
  CK(hipMemcpy(c->cvec.p, lload.data(), sizeof(double) * lload.size(), hipMemcpyHostToDevice),
     "cvec");
  int nloc = L.n_owned + L.n_ghost;
  auto up_field = [&](const double *h, double *d) -> int {
    std::vector<double> tmp(nloc);
    for (int i = 0; i < nloc; i++) tmp[i] = h[L.l2g[i]];
    hipError_t e = hipMemcpy(d, tmp.data(), sizeof(double) * nloc, hipMemcpyHostToDevice);
    return e == hipSuccess ? PNP_OK : c->hipfail(e, "aux upload");
  };
  int rc;
  if (kind == PNP_OP_DIFF || kind == PNP_OP_DIFF_IMPLICIT_EULER)
    if ((rc = up_field(a->phi, c->aux0.p))) return rc;
  if (kind == PNP_OP_POISSON)
    if ((rc = up_field(a->cp, c->aux0.p)) || (rc = up_field(a->cm, c->aux1.p))) return rc;
  if (ie) {  // cvec -= M(x_old), rows of this rank (x_old with ghosts)
    if ((rc = c->upload_ext(a->x_old, nf, c->prevu.p, true))) return rc;
    int k = kind == PNP_OP_PNP_IMPLICIT_EULER ? pnp::OP_PNP_IE : pnp::OP_DIFF_IE;
    if (c->degree > 1)
      CK(pnp::launch_pk_mass_apply(c->dl, c->pkd, c->prevu.p, c->cvec.p, c->stream), "mass apply");
    else
      CK(pnp::launch_mass_apply(c->dl, k, c->params.tau, c->params.pi, c->params.cylindrical,
                                c->prevu.p, c->cvec.p, c->stream),
         "mass apply");
    CK(hipStreamSynchronize(c->stream), "mass apply");
  }
  pnp::AsmArgs &aa = c->aa;
  aa = pnp::AsmArgs{};
  aa.kind = kind;  // PNP_OP_* == pnp::OP_* by construction
  aa.l_b = c->params.l_b;
  aa.c0 = c->params.c0;
  aa.tau = c->params.tau;
  aa.pi = c->params.pi;
  aa.dt = a->dt;
  aa.z = a->z;
  aa.cylindrical = c->params.cylindrical;
  aa.aux0 = c->aux0.p;
  aa.aux1 = c->aux1.p;
  aa.cvec = c->cvec.p;
  aa.dmask = c->dmask.p;
  aa.vals = c->vals.p;
  return PNP_OK;
}

// reference-order mode: x / r external layout, host or device
static int seq_residual_abi(pnp_ctx *c, const double *x, double *r, bool dev) {
  int rc;
  if ((rc = c->seq_build())) return rc;
  const size_t n = c->nseq();
  double *sx = c->sq(pnp_ctx::SQ_X), *sr = c->sq(pnp_ctx::SQ_R);
  CK(hipMemcpyAsync(sx, x, 8 * n, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream),
     "seq upload");
  if ((rc = c->seq_residual(sx, sr))) return rc;
  CK(hipMemcpyAsync(r, sr, 8 * n, dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream),
     "seq download");
  CK(hipStreamSynchronize(c->stream), "seq residual");
  return PNP_OK;
}
static int seq_jacobian_abi(pnp_ctx *c, const double *x, bool dev, bool fd) {
  int rc;
  if ((rc = c->seq_build())) return rc;
  double *sx = c->sq(pnp_ctx::SQ_X);
  CK(hipMemcpyAsync(sx, x, 8 * size_t(c->nseq()),
                    dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream),
     "seq upload");
  if ((rc = c->seq_jacobian(sx, fd))) return rc;
  CK(hipStreamSynchronize(c->stream), "seq jacobian");
  return PNP_OK;
}

extern "C" int pnp_residual(pnp_ctx *c, const double *x, double *r) {
  if (!c || !x || !r) return PNP_E_ARG;
  if (c->kind < 0) return c->fail(PNP_E_STATE, "no operator set");
  hipSetDevice(c->device);
  if (c->seq_on()) return seq_residual_abi(c, x, r, false);
  int rc;
  if ((rc = c->upload_ext(x, c->nf, c->x.p, true))) return rc;
  if ((rc = c->assemble(c->x.p, 0))) return rc;
  return c->download_ext(c->r.p, c->nf, r);
}

extern "C" int pnp_jacobian(pnp_ctx *c, const double *x) {
  if (!c || !x) return PNP_E_ARG;
  if (c->kind < 0) return c->fail(PNP_E_STATE, "no operator set");
  hipSetDevice(c->device);
  if (c->seq_on()) return seq_jacobian_abi(c, x, false, c->fd_opt != 0);
  int rc;
  if ((rc = c->upload_ext(x, c->nf, c->x.p, true))) return rc;
  if ((rc = c->assemble(c->x.p, 1))) return rc;
  CK(hipStreamSynchronize(c->stream), "jacobian");
  return PNP_OK;
}

extern "C" int pnp_jacobian_export(pnp_ctx *c, int64_t *nnz, int32_t *rowptr, int32_t *col,
                                   double *val) {
  if (!c || !nnz) return PNP_E_ARG;
  if (!c->assembled) return c->fail(PNP_E_STATE, "no Jacobian assembled");
  if (c->seq_on()) {  // the reference-order Jacobian lives in the CSR view
    *nnz = c->csr_nnz;
    if (!rowptr || !col || !val) return PNP_OK;
    const size_t n = c->nseq();
    CK(hipMemcpy(rowptr, c->csr_rowptr.p, 4 * (n + 1), hipMemcpyDeviceToHost), "export");
    CK(hipMemcpy(col, c->csr_col.p, 4 * size_t(c->csr_nnz), hipMemcpyDeviceToHost), "export");
    CK(hipMemcpy(val, c->csr_val.p, 8 * size_t(c->csr_nnz), hipMemcpyDeviceToHost), "export");
    return PNP_OK;
  }
  const pnp::LocalLayout &L = c->L;
  int nf = c->nf, NV = c->nvb, nv = c->mesh.nv;
  long long total = 0;
  for (int i = 0; i < L.n_owned; i++) total += (long long)pnp::meta_len(L.rowmeta[i]);
  total *= NV;
  *nnz = total;
  if (!rowptr || !col || !val) return PNP_OK;
  const int NKS = c->nks;
  std::vector<double> hv(size_t(L.nslots) * NKS);
  CK(hipMemcpy(hv.data(), c->vals.p, sizeof(double) * hv.size(), hipMemcpyDeviceToHost), "export");
  // rows of the external layout: f*nv + g ; count per row
  int n = nf * nv;
  std::vector<int> cnt(n + 1, 0);
  for (int i = 0; i < L.n_owned; i++) {
    int len = pnp::meta_len(L.rowmeta[i]);
    for (int f = 0; f < nf; f++) {
      int k = 0;
      for (int g = 0; g < nf; g++) k += pnp::pat_index(c->pat, f, g) >= 0;
      cnt[f * nv + L.l2g[i] + 1] += k * len;
    }
  }
  for (int i = 0; i < n; i++) cnt[i + 1] += cnt[i];
  std::vector<int> fill(n, 0);
  std::vector<std::pair<int, double>> tmp;
  for (int i = 0; i < L.n_owned; i++) {
    int chunk = i / pnp::kRows, lane = i % pnp::kRows;
    int len = pnp::meta_len(L.rowmeta[i]);
    for (int f = 0; f < nf; f++) {
      int R = f * nv + L.l2g[i];
      tmp.clear();
      unsigned dm = 0;
      for (int g = 0; g < nf; g++) dm |= unsigned(c->hmask[size_t(i) * nf + g] != 0) << g;
      for (int s = 0; s < len; s++) {
        int j = L.colidx[size_t(L.chunk_off[chunk]) + size_t(s) * pnp::kRows + lane];
        double K[9], B[9];
        for (int q = 0; q < NKS; q++)
          K[q] = hv[(size_t(L.chunk_off[chunk]) + size_t(s) * pnp::kRows) * NKS +
                    pnp::vin(NKS, q, lane)];
        expand_host(c->pat, K, dm, s == 0, B);
        for (int g = 0; g < nf; g++) {
          int v = pnp::pat_index(c->pat, f, g);
          if (v < 0) continue;
          tmp.push_back({g * nv + L.l2g[j], B[v]});
        }
      }
      std::sort(tmp.begin(), tmp.end());
      for (auto &pr : tmp) {
        col[cnt[R] + fill[R]] = pr.first;
        val[cnt[R] + fill[R]] = pr.second;
        fill[R]++;
      }
    }
  }
  for (int i = 0; i <= n; i++) rowptr[i] = cnt[i];
  return PNP_OK;
}

// ---------------------------------------------------------------------------------------------
// flags / device pointers / FD Jacobian / jacobian_apply / device CSR view
// ---------------------------------------------------------------------------------------------
static int check_flags(pnp_ctx *c, int32_t flags, int32_t allowed) {
  if (flags & ~allowed) return c->fail(PNP_E_ARG, "unsupported flags for this call");
  return PNP_OK;
}

extern "C" int pnp_residual_ex(pnp_ctx *c, const double *x, double *r, int32_t flags) {
  if (!c || !x || !r) return PNP_E_ARG;
  if (c->kind < 0) return c->fail(PNP_E_STATE, "no operator set");
  int rc;
  if ((rc = check_flags(c, flags, PNP_DEVICE_PTRS))) return rc;
  hipSetDevice(c->device);
  const bool dev = flags & PNP_DEVICE_PTRS;
  if (c->seq_on()) return seq_residual_abi(c, x, r, dev);
  if ((rc = c->upload_ext(x, c->nf, c->x.p, true, dev))) return rc;
  if ((rc = c->assemble(c->x.p, 0))) return rc;
  return c->download_ext(c->r.p, c->nf, r, dev);
}

extern "C" int pnp_jacobian_ex(pnp_ctx *c, const double *x, int32_t flags) {
  if (!c || !x) return PNP_E_ARG;
  if (c->kind < 0) return c->fail(PNP_E_STATE, "no operator set");
  int rc;
  if ((rc = check_flags(c, flags, PNP_DEVICE_PTRS | PNP_JAC_FD))) return rc;
  hipSetDevice(c->device);
  if (c->seq_on())
    return seq_jacobian_abi(c, x, flags & PNP_DEVICE_PTRS, c->fd_opt || (flags & PNP_JAC_FD));
  if ((rc = c->upload_ext(x, c->nf, c->x.p, true, flags & PNP_DEVICE_PTRS))) return rc;
  const int keep = c->fd_opt;
  if (flags & PNP_JAC_FD) c->fd_opt = 1;
  rc = c->assemble(c->x.p, 1);
  c->fd_opt = keep;
  if (rc) return rc;
  CK(hipStreamSynchronize(c->stream), "jacobian");
  return PNP_OK;
}

extern "C" int pnp_jacobian_apply(pnp_ctx *c, const double *x, const double *z, double *y,
                                  int32_t flags) {
  if (!c || !z || !y) return PNP_E_ARG;
  if (c->kind < 0) return c->fail(PNP_E_STATE, "no operator set");
  int rc;
  if ((rc = check_flags(c, flags, PNP_DEVICE_PTRS | PNP_JAC_FD))) return rc;
  hipSetDevice(c->device);
  const bool dev = flags & PNP_DEVICE_PTRS;
  if (x) {
    if ((rc = pnp_jacobian_ex(c, x, flags))) return rc;
  } else if (!c->assembled) {
    return c->fail(PNP_E_STATE, "no Jacobian assembled (pass x)");
  }
  if (c->seq_on()) {  // y = A z in BCRSMatrix::mv's order on the CSR view
    const size_t n = c->nseq();
    double *sz = c->sq(pnp_ctx::SQ_Z), *sy = c->sq(pnp_ctx::SQ_Y);
    CK(hipMemcpyAsync(sz, z, 8 * n, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream),
       "seq upload");
    CK(pnp::launch_seq_spmv(int(n), c->csr_rowptr.p, c->csr_col.p, c->csr_val.p, sz, sy, c->stream),
       "seq apply");
    CK(hipMemcpyAsync(y, sy, 8 * n, dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream),
       "seq download");
    CK(hipStreamSynchronize(c->stream), "seq apply");
    return PNP_OK;
  }
  // z with ghosts (the halo of a global vector is local: every rank holds it), y = A z
  if ((rc = c->upload_ext(z, c->nf, c->y.p, true, dev))) return rc;
  int nsp = 0;
  CK(pnp::launch_spmv(c->dl, c->nf, c->pat, c->vals.p, c->y.p, c->t.p, 0, nullptr, c->partials.p,
                      &nsp, c->stream),
     "jacobian apply");
  return c->download_ext(c->t.p, c->nf, y, dev);
}

static int seq_solve_abi(pnp_ctx *c, const double *rhs, double *z, const pnp_solve_opts &o,
                         pnp_solve_result &res, bool dev) {
  int rc;
  if ((rc = c->seq_build())) return rc;
  const size_t n = c->nseq();
  double *sb = c->sq(pnp_ctx::SQ_B), *sz = c->sq(pnp_ctx::SQ_Z);
  CK(hipMemcpyAsync(sb, rhs, 8 * n, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream),
     "seq upload");
  CK(hipMemsetAsync(sz, 0, 8 * n, c->stream), "seq upload");
  if ((rc = c->seq_krylov(o, sz, sb, res))) return rc;
  CK(hipMemcpyAsync(z, sz, 8 * n, dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream),
     "seq download");
  CK(hipStreamSynchronize(c->stream), "seq solve");
  return res.breakdown ? PNP_E_BREAKDOWN : PNP_OK;
}

extern "C" int pnp_linear_solve_ex(pnp_ctx *c, const double *rhs, double *z,
                                   const pnp_solve_opts *o, pnp_solve_result *res, int32_t flags) {
  if (!c || !rhs || !z || !o || !res) return PNP_E_ARG;
  int rc;
  if ((rc = check_flags(c, flags, PNP_DEVICE_PTRS))) return rc;
  hipSetDevice(c->device);
  std::memset(res, 0, sizeof *res);
  const bool dev = flags & PNP_DEVICE_PTRS;
  if (c->seq_on()) return seq_solve_abi(c, rhs, z, *o, *res, dev);
  if ((rc = c->upload_ext(rhs, c->nf, c->b.p, false, dev))) return rc;
  if ((rc = c->krylov(c->b.p, c->z.p, *o, *res))) return rc;
  if ((rc = c->download_ext(c->z.p, c->nf, z, dev))) return rc;
  return res->breakdown ? PNP_E_BREAKDOWN : PNP_OK;
}

extern "C" int pnp_jacobian_csr_device(pnp_ctx *c, pnp_csr_view *out) {
  if (!c || !out) return PNP_E_ARG;
  if (!c->assembled) return c->fail(PNP_E_STATE, "no Jacobian assembled");
  hipSetDevice(c->device);
  int rc;
  if ((rc = c->csr_values())) return rc;
  CK(hipStreamSynchronize(c->stream), "csr fill");
  out->n = c->nf * c->mesh.nv;
  out->nnz = c->csr_nnz;
  out->rowptr = c->csr_rowptr.p;
  out->col = c->csr_col.p;
  out->val = c->csr_val.p;
  return PNP_OK;
}

// ---------------------------------------------------------------------------------------------
// solves
// ---------------------------------------------------------------------------------------------
extern "C" int pnp_linear_solve(pnp_ctx *c, const double *rhs, double *z, const pnp_solve_opts *o,
                                pnp_solve_result *res) {
  if (!c || !rhs || !z || !o || !res) return PNP_E_ARG;
  hipSetDevice(c->device);
  std::memset(res, 0, sizeof *res);
  if (c->seq_on()) return seq_solve_abi(c, rhs, z, *o, *res, false);
  int rc;
  if ((rc = c->upload_ext(rhs, c->nf, c->b.p, false))) return rc;
  if ((rc = c->krylov(c->b.p, c->z.p, *o, *res))) return rc;
  if ((rc = c->download_ext(c->z.p, c->nf, z))) return rc;
  return res->breakdown ? PNP_E_BREAKDOWN : PNP_OK;
}

extern "C" int pnp_prec_apply(pnp_ctx *c, int32_t prec, const double *d, double *v) {
  if (!c || !d || !v || prec < PNP_PREC_NONE || prec > PNP_PREC_SSOR_NATURAL) return PNP_E_ARG;
  if (!c->assembled) return c->fail(PNP_E_STATE, "no Jacobian assembled");
  hipSetDevice(c->device);
  int rc;
  if (c->seq_on()) {
    if (prec != PNP_PREC_NONE && prec != PNP_PREC_JACOBI && prec != PNP_PREC_SSOR_NATURAL)
      return c->fail(PNP_E_ARG, "PNP_OPT_SEQ_ORDER: preconditioner must be NONE, JACOBI or SSOR_NATURAL");
    const size_t n = c->nseq();
    double *sb = c->sq(pnp_ctx::SQ_B), *sz = c->sq(pnp_ctx::SQ_Z);
    CK(hipMemcpyAsync(sb, d, 8 * n, hipMemcpyHostToDevice, c->stream), "seq upload");
    CK(hipMemsetAsync(sz, 0, 8 * n, c->stream), "seq upload");
    if ((rc = c->seq_prec(prec, sb, sz))) return rc;
    if (prec == PNP_PREC_SSOR_NATURAL && (rc = c->nat_check())) return rc;
    CK(hipMemcpyAsync(v, sz, 8 * n, hipMemcpyDeviceToHost, c->stream), "seq download");
    CK(hipStreamSynchronize(c->stream), "seq prec");
    return PNP_OK;
  }
  if ((rc = c->upload_ext(d, c->nf, c->b.p, false))) return rc;
  if (prec == PNP_PREC_ILU0 && (rc = c->ilu_factor())) return rc;
  if ((rc = c->precond(prec, c->b.p, c->z.p))) return rc;
  if (prec == PNP_PREC_SSOR_NATURAL && (rc = c->nat_check())) return rc;
  if (prec == PNP_PREC_ILU0 && (rc = c->ilu_flow_check())) return rc;
  return c->download_ext(c->z.p, c->nf, v);
}

extern "C" int pnp_set_option(pnp_ctx *c, int32_t option, int64_t value) {
  if (!c) return PNP_E_ARG;
  c->graphs_clear();
  if (option == PNP_OPT_GRAPH) {
    if (value < -1 || value > 1) return c->fail(PNP_E_ARG, "PNP_OPT_GRAPH takes -1, 0 or 1");
    c->graph_opt = int(value);
    return PNP_OK;
  }
  if (option == PNP_OPT_ILU_F32) {
    if (value < 0 || value > 3) return c->fail(PNP_E_ARG, "PNP_OPT_ILU_F32 takes 0 .. 3");
    if (c->ilu_f32 != int(value)) {
      c->ilu_f32 = int(value);
      if (c->split_of == 2) c->split_of = 0;  // re-split the factors in the new precision
    }
    return PNP_OK;
  }
  if (option == PNP_OPT_ILU_FLOW) {
    if (value < 0 || value > 2) return c->fail(PNP_E_ARG, "PNP_OPT_ILU_FLOW takes 0, 1 or 2");
    c->ilu_flow_opt = int(value);
    return PNP_OK;
  }
  if (option == PNP_OPT_NAT_FLOW) {
    if (value < -1 || value > 1) return c->fail(PNP_E_ARG, "PNP_OPT_NAT_FLOW takes -1, 0 or 1");
    c->nat_flow_opt = int(value);
    return PNP_OK;
  }
  if (option == PNP_OPT_AMG_FALLBACK) {
    if (value != 0 && value != 1) return c->fail(PNP_E_ARG, "PNP_OPT_AMG_FALLBACK takes 0 or 1");
    c->amg_fallback = int(value);
    return PNP_OK;
  }
  if (option == PNP_OPT_ILU_RETRY) {
    if (value != 0 && value != 1) return c->fail(PNP_E_ARG, "PNP_OPT_ILU_RETRY takes 0 or 1");
    c->ilu_retry = int(value);
    return PNP_OK;
  }
  if (option == PNP_OPT_BICG_TWORED) {
    if (value < -1 || value > 1) return c->fail(PNP_E_ARG, "PNP_OPT_BICG_TWORED takes -1, 0 or 1");
    c->twored_opt = int(value);
    return PNP_OK;
  }
  if (option == PNP_OPT_SEQ_ORDER) {
    if (value != 0 && value != 1) return c->fail(PNP_E_ARG, "PNP_OPT_SEQ_ORDER takes 0 or 1");
    if (value && (c->degree > 1 || c->dist))
      return c->fail(PNP_E_ARG, "PNP_OPT_SEQ_ORDER: P1 contexts of one rank only");
    if (c->seq_opt != int(value)) {
      c->seq_opt = int(value);
      c->assembled = false;  // the next Jacobian is assembled in the newly selected form
      c->csr_vals_valid = false;
    }
    return PNP_OK;
  }
  if (option == PNP_OPT_JAC_FD) {
    if (value != 0 && value != 1) return c->fail(PNP_E_ARG, "PNP_OPT_JAC_FD takes 0 or 1");
    c->fd_opt = int(value);
    return PNP_OK;
  }
  if (option == PNP_OPT_ILU_FUSED_FACTOR) {
    if (value != 0 && value != 1) return c->fail(PNP_E_ARG, "PNP_OPT_ILU_FUSED_FACTOR takes 0 or 1");
    c->ilu_fused = int(value);
    c->lu_valid = false;
    if (c->split_of == 2) c->split_of = 0;
    return PNP_OK;
  }
  return c->fail(PNP_E_ARG, "unknown option");
}

extern "C" int pnp_set_create_option(int32_t option, int64_t value) {
  if (option == PNP_CREATE_ABSORB_THIN_COLOR) {
    if (value < -1 || value > 1) {
      g_err = "PNP_CREATE_ABSORB_THIN_COLOR takes -1, 0 or 1";
      return PNP_E_ARG;
    }
    pnp::g_absorb_thin_color.store(int(value));
    return PNP_OK;
  }
  g_err = "unknown creation option";
  return PNP_E_ARG;
}

extern "C" int pnp_get_create_option(int32_t option, int64_t *value) {
  if (!value) return PNP_E_ARG;
  if (option == PNP_CREATE_ABSORB_THIN_COLOR) {
    *value = pnp::g_absorb_thin_color.load();
    return PNP_OK;
  }
  g_err = "unknown creation option";
  return PNP_E_ARG;
}

extern "C" int pnp_get_option(pnp_ctx *c, int32_t option, int64_t *value) {
  if (!c || !value) return PNP_E_ARG;
  if (option == PNP_OPT_ILU_F32) {
    *value = c->ilu_f32;
    return PNP_OK;
  }
  if (option == PNP_OPT_ILU_FUSED_FACTOR) {
    *value = c->ilu_fused;
    return PNP_OK;
  }
  if (option == PNP_OPT_GRAPH) {
    *value = c->graph_opt;
    return PNP_OK;
  }
  if (option == PNP_OPT_JAC_FD) {
    *value = c->fd_opt;
    return PNP_OK;
  }
  if (option == PNP_OPT_BICG_TWORED) {
    *value = c->twored_opt;
    return PNP_OK;
  }
  if (option == PNP_OPT_ILU_FLOW) {
    *value = c->ilu_flow_opt;
    return PNP_OK;
  }
  if (option == PNP_OPT_AMG_FALLBACK) {
    *value = c->amg_fallback;
    return PNP_OK;
  }
  if (option == PNP_OPT_ILU_RETRY) {
    *value = c->ilu_retry;
    return PNP_OK;
  }
  if (option == PNP_OPT_SEQ_ORDER) {
    *value = c->seq_opt;
    return PNP_OK;
  }
  return c->fail(PNP_E_ARG, "unknown option");
}

extern "C" int pnp_amg_configure(pnp_ctx *c, const pnp_amg_opts *o) {
  if (!c || !o) return PNP_E_ARG;
  if (o->smoother != PNP_PREC_SSOR && o->smoother != PNP_PREC_ILU0 &&
      o->smoother != PNP_PREC_JACOBI && o->smoother != PNP_PREC_SSOR_NATURAL)
    return c->fail(PNP_E_ARG, "AMG smoother must be SSOR, SSOR_NATURAL, ILU0 or JACOBI");
  if (o->coarse_target < 1 || o->coarse_target > pnp::kAmgMaxCoarse || o->max_levels < 2 ||
      o->max_levels > pnp::kAmgMaxLevels || !(o->omega > 0 && o->omega <= 2) ||
      o->coarse_sweeps < 1 || o->coarse_sweeps > 8 || o->level0_presmooth < -1 ||
      o->level0_presmooth > 1)
    return c->fail(PNP_E_ARG, "AMG options out of range");
  const bool rebuild = o->coarse_target != c->amg_opts.coarse_target ||
                       o->max_levels != c->amg_opts.max_levels;
  c->amg_opts = *o;
  if (rebuild) c->amg_built = false;
  c->amg_valid = false;
  return PNP_OK;
}

extern "C" int pnp_amg_info(pnp_ctx *c, pnp_amg_stats *st) {
  if (!c || !st) return PNP_E_ARG;
  std::memset(st, 0, sizeof *st);
  if (!c->amg_built) return c->fail(PNP_E_STATE, "AMG not set up (solve or apply with PNP_PREC_AMG)");
  st->levels = int(c->amg_h.size()) + 1;
  st->rows[0] = c->L.n_owned;
  st->blocks[0] = c->L.nblocks;
  for (size_t k = 0; k < c->amg_h.size() && k + 1 < 16; k++) {
    st->rows[k + 1] = c->amg_h[k].nb;
    st->blocks[k + 1] = (int64_t)c->amg_h[k].col.size();
  }
  st->omega = c->amg_opts.omega;
  st->smoother = c->amg_opts.smoother;
  return PNP_OK;
}

extern "C" int pnp_amg_aggregates(pnp_ctx *c, int32_t level, int32_t *agg) {
  if (!c || !agg || level < 0) return PNP_E_ARG;
  if (!c->amg_built) return c->fail(PNP_E_STATE, "AMG not set up");
  if (level >= int(c->amg_h.size())) return c->fail(PNP_E_ARG, "no such AMG level");
  const std::vector<int> &a = c->amg_h[level].agg;
  if (level == 0) {  // global vertex numbering, -1 for vertices this rank does not own
    for (int g = 0; g < c->mesh.nv; g++) agg[g] = -1;
    for (int i = 0; i < c->L.n_owned; i++) agg[c->L.l2g[i]] = a[i];
  } else {
    std::copy(a.begin(), a.end(), agg);
  }
  return PNP_OK;
}

extern "C" int pnp_ion_flux(pnp_ctx *c, const double *x, int32_t nsurf, double *ip, double *im) {
  if (!c || !ip || !im || nsurf < 0 || nsurf > 256) return PNP_E_ARG;
  hipSetDevice(c->device);
  const double *xd = c->x.p;
  int rc;
  if (x) {
    if ((rc = c->upload_ext(x, 3, c->fluxx.p, true))) return rc;
    xd = c->fluxx.p;
  } else if (c->nf != 3) {
    return c->fail(PNP_E_STATE, "ion flux of the context state needs a 3-field (PNP) operator");
  }
  const int ns = int(c->fseg_group.size());
  if (c->degree > 1)
    CK(pnp::launch_pk_ion_flux(c->dl, c->pkd, ns, c->d_fseg.p, xd, c->params.cylindrical,
                               c->params.pi, c->fluxout.p, c->stream),
       "ion flux");
  else
    CK(pnp::launch_ion_flux(ns, c->d_fseg.p, c->d_xy.p, xd, c->params.cylindrical, c->params.pi,
                            c->fluxout.p, c->stream),
       "ion flux");
  std::vector<double> out(2 * size_t(ns)), acc(2 * size_t(nsurf), 0.0);
  if (ns) {
    CK(hipMemcpyAsync(out.data(), c->fluxout.p, sizeof(double) * out.size(),
                      hipMemcpyDeviceToHost, c->stream),
       "ion flux");
  }
  CK(hipStreamSynchronize(c->stream), "ion flux");
  for (int k = 0; k < ns; k++) {  // global segment order: independent of the launch
    const int g = c->fseg_group[k];
    if (g < 0 || g >= nsurf) return c->fail(PNP_E_ARG, "boundary group outside [0, nsurf)");
    acc[2 * size_t(g)] += out[2 * size_t(k)];
    acc[2 * size_t(g) + 1] += out[2 * size_t(k) + 1];
  }
  if (c->dist && nsurf > 0) {
    CK(hipMemcpy(c->fluxred.p, acc.data(), sizeof(double) * acc.size(), hipMemcpyHostToDevice),
       "ion flux");
    if ((rc = c->allreduce_dev(c->fluxred.p, 2 * nsurf))) return rc;
    CK(hipStreamSynchronize(c->stream), "ion flux");
    CK(hipMemcpy(acc.data(), c->fluxred.p, sizeof(double) * acc.size(), hipMemcpyDeviceToHost),
       "ion flux");
  }
  for (int g = 0; g < nsurf; g++) {
    ip[g] = acc[2 * size_t(g)];
    im[g] = acc[2 * size_t(g) + 1];
  }
  return PNP_OK;
}

// PDELab Newton in the reference's order (PNP_OPT_SEQ_ORDER; the oracle's orc_newton statements):
// external layout, GridOperator residual / Jacobian in element order, ISTL solves in their order,
// defect = sqrt(<r, r>) summed sequentially, u -= lambda z
static int seq_newton(pnp_ctx *c, double *u, const pnp_newton_opts *o, pnp_newton_result *res) {
  int rc;
  if ((rc = c->seq_build())) return rc;
  double t_start = now_s();
  const size_t n = c->nseq();
  double *x = c->sq(pnp_ctx::SQ_X), *r = c->sq(pnp_ctx::SQ_R), *z = c->sq(pnp_ctx::SQ_Z),
         *prevu = c->sq(pnp_ctx::SQ_PREVU);
  CK(hipMemcpyAsync(x, u, 8 * n, hipMemcpyHostToDevice, c->stream), "seq upload");
  double ta = now_s();
  if ((rc = c->seq_residual(x, r))) return rc;
  double defect = std::sqrt(c->seq_dot(r, r, rc));
  if (rc) return rc;
  res->assemble_seconds += now_s() - ta;
  res->first_defect = defect;
  double prev_defect = defect;
  res->status = PNP_OK;
  const bool fd = c->fd_opt != 0;
  for (;;) {
    res->converged = (defect < o->abs_limit || defect < res->first_defect * o->reduction) ? 1 : 0;
    if (res->converged) break;
    if (res->iterations >= o->maxit) {
      res->status = PNP_E_NOT_CONVERGED;
      break;
    }
    ta = now_s();
    if ((rc = c->seq_jacobian(x, fd))) return rc;
    CK(hipStreamSynchronize(c->stream), "seq jacobian");
    res->assemble_seconds += now_s() - ta;
    const double stop_defect = std::max(res->first_defect * o->reduction, o->abs_limit);
    double lin_red;
    if (stop_defect / (10 * defect) > defect * defect / (prev_defect * prev_defect))
      lin_red = stop_defect / (10 * defect);
    else
      lin_red = std::min(o->min_linear_reduction, defect * defect / (prev_defect * prev_defect));
    prev_defect = defect;
    CK(hipMemsetAsync(z, 0, 8 * n, c->stream), "seq z");
    pnp_solve_opts lo = o->linear;
    lo.reduction = lin_red;
    pnp_solve_result sr{};
    double ts = now_s();
    if ((rc = c->seq_krylov(lo, z, r, sr))) return rc;  // r: overwritten by the solve's residual
    res->solve_seconds += now_s() - ts;
    res->linear_iterations += sr.iterations;
    const int step_its = sr.iterations;
    if (sr.breakdown) {
      res->status = PNP_E_BREAKDOWN;
      break;
    }
    if (!sr.converged) {
      res->status = PNP_E_NOT_CONVERGED;
      break;
    }
    // hackbuschReuskenAcceptBest
    double lambda = 1.0, best_lambda = 0.0, best_defect = defect;
    CK(hipMemcpyAsync(prevu, x, 8 * n, hipMemcpyDeviceToDevice, c->stream), "seq prevu");
    int i = 0;
    bool ls_fail = false;
    for (;;) {
      CK(pnp::launch_seq_aymx(int(n), lambda, x, z, c->stream), "seq update");
      ta = now_s();
      if ((rc = c->seq_residual(x, r))) return rc;
      defect = std::sqrt(c->seq_dot(r, r, rc));
      if (rc) return rc;
      res->assemble_seconds += now_s() - ta;
      if (defect <= (1.0 - lambda / 4) * prev_defect) break;
      if (defect < best_defect) {
        best_defect = defect;
        best_lambda = lambda;
      }
      if (++i >= o->line_search_maxit) {
        if (best_lambda == 0.0) {
          ls_fail = true;
          break;
        }
        if (best_lambda != lambda) {
          CK(hipMemcpyAsync(x, prevu, 8 * n, hipMemcpyDeviceToDevice, c->stream), "seq prevu");
          CK(pnp::launch_seq_aymx(int(n), best_lambda, x, z, c->stream), "seq update");
          if ((rc = c->seq_residual(x, r))) return rc;
          defect = std::sqrt(c->seq_dot(r, r, rc));
          if (rc) return rc;
        }
        break;
      }
      lambda *= 0.5;
      CK(hipMemcpyAsync(x, prevu, 8 * n, hipMemcpyDeviceToDevice, c->stream), "seq prevu");
    }
    if (ls_fail) {
      res->status = PNP_E_NOT_CONVERGED;
      break;
    }
    res->iterations++;
    c->newton_its.push_back(step_its);
    c->newton_defects.push_back(defect);
  }
  res->defect = defect;
  CK(hipMemcpyAsync(u, x, 8 * n, hipMemcpyDeviceToHost, c->stream), "seq download");
  CK(hipStreamSynchronize(c->stream), "seq newton");
  res->elapsed = now_s() - t_start;
  return PNP_OK;
}

extern "C" int pnp_newton(pnp_ctx *c, double *u, const pnp_newton_opts *o, pnp_newton_result *res) {
  if (!c || !u || !o || !res) return PNP_E_ARG;
  if (c->kind < 0) return c->fail(PNP_E_STATE, "no operator set");
  hipSetDevice(c->device);
  std::memset(res, 0, sizeof *res);
  c->newton_its.clear();
  c->newton_defects.clear();
  if (c->seq_on()) return seq_newton(c, u, o, res);
  double t_start = now_s();
  int rc;
  long long n = c->nown();
  // PNP_OPT_ILU_RETRY: the factor precision a retry switched from, restored when this call ends
  int ilu_saved = -1;
  struct IluRestore {
    pnp_ctx *c;
    int &saved;
    ~IluRestore() {
      if (saved < 0) return;
      c->ilu_f32 = saved;
      if (c->split_of == 2) c->split_of = 0;
      c->lu_valid = false;
    }
  } ilu_restore{c, ilu_saved};
  if ((rc = c->upload_ext(u, c->nf, c->x.p, true))) return rc;
  double ta = now_s();
  if ((rc = c->assemble(c->x.p, 0))) return rc;
  double defect;
  if ((rc = c->norm(c->r.p, defect))) return rc;
  res->assemble_seconds += now_s() - ta;
  res->first_defect = defect;
  double prev_defect = defect;
  res->status = PNP_OK;
  for (;;) {
    res->converged = (defect < o->abs_limit || defect < res->first_defect * o->reduction) ? 1 : 0;
    if (res->converged) break;
    if (res->iterations >= o->maxit) {
      res->status = PNP_E_NOT_CONVERGED;
      break;
    }
    ta = now_s();
    if ((rc = c->assemble(c->x.p, 1))) return rc;  // reassemble every step (threshold 0)
    CK(hipStreamSynchronize(c->stream), "assemble");
    res->assemble_seconds += now_s() - ta;
    double stop_defect = std::max(res->first_defect * o->reduction, o->abs_limit);
    double lin_red;
    if (stop_defect / (10 * defect) > defect * defect / (prev_defect * prev_defect))
      lin_red = stop_defect / (10 * defect);
    else
      lin_red = std::min(o->min_linear_reduction, defect * defect / (prev_defect * prev_defect));
    prev_defect = defect;
    // z solves J z = r(u); r lives in c->r (owned rows); keep it in b for the solver
    CK(hipMemcpyAsync(c->b.p, c->r.p, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream),
       "rhs");
    pnp_solve_opts lo = o->linear;
    lo.reduction = lin_red;
    pnp_solve_result sr{};
    double ts = now_s();
    if ((rc = c->krylov(c->b.p, c->z.p, lo, sr))) return rc;
    res->linear_iterations += sr.iterations;
    int step_its = sr.iterations;
    if (lo.prec == PNP_PREC_AMG && c->amg_fallback && (sr.breakdown || !sr.converged)) {
      // AMG fallback: the V-cycle of a non-symmetric system can fail where its level-0
      // smoother alone converges (a far-from-converged state); redo this step's solve with the
      // smoother as the preconditioner
      lo.prec = c->amg_opts.smoother;
      CK(hipMemcpyAsync(c->b.p, c->r.p, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream),
         "rhs");
      if ((rc = c->krylov(c->b.p, c->z.p, lo, sr))) return rc;
      res->linear_iterations += sr.iterations;
      step_its += sr.iterations;
      res->linear_fallbacks++;
    }
    const bool uses_ilu = lo.prec == PNP_PREC_ILU0 ||
                          (lo.prec == PNP_PREC_AMG && c->amg_opts.smoother == PNP_PREC_ILU0);
    if (c->ilu_retry && uses_ilu && c->ilu_f32 != 0 && (sr.breakdown || !sr.converged)) {
      // reduced-precision ILU(0) factors stalled this solve: re-solve with fp64 factors (ISTL's
      // SeqILU0) and keep them for the rest of this call
      if (ilu_saved < 0) ilu_saved = c->ilu_f32;
      c->ilu_f32 = 0;
      if (c->split_of == 2) c->split_of = 0;
      c->lu_valid = false;
      CK(hipMemcpyAsync(c->b.p, c->r.p, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream),
         "rhs");
      if ((rc = c->krylov(c->b.p, c->z.p, lo, sr))) return rc;
      res->linear_iterations += sr.iterations;
      step_its += sr.iterations;
      res->precision_retries++;
    }
    res->solve_seconds += now_s() - ts;
    if (sr.breakdown) {
      res->status = PNP_E_BREAKDOWN;
      break;
    }
    if (!sr.converged) {  // PDELab NewtonLinearSolverError
      res->status = PNP_E_NOT_CONVERGED;
      break;
    }
    // hackbuschReuskenAcceptBest line search
    double lambda = 1.0, best_lambda = 0.0, best_defect = defect;
    CK(hipMemcpyAsync(c->prevu.p, c->x.p, sizeof(double) * n, hipMemcpyDeviceToDevice, c->stream),
       "prevu");
    int i = 0;
    bool ls_fail = false;
    for (;;) {
      CK(pnp::launch_axpby(n, 1.0, c->prevu.p, -lambda, c->z.p, c->x.p, c->stream), "axpby");
      if ((rc = c->halo(c->x.p, c->nf))) return rc;
      ta = now_s();
      if ((rc = c->assemble(c->x.p, 0))) return rc;
      if ((rc = c->norm(c->r.p, defect))) return rc;
      res->assemble_seconds += now_s() - ta;
      if (std::isfinite(defect) && defect <= (1.0 - lambda / 4) * prev_defect) break;
      if (std::isfinite(defect) && defect < best_defect) {
        best_defect = defect;
        best_lambda = lambda;
      }
      if (++i >= o->line_search_maxit) {
        if (best_lambda == 0.0) {
          ls_fail = true;
          break;
        }
        if (best_lambda != lambda) {
          CK(pnp::launch_axpby(n, 1.0, c->prevu.p, -best_lambda, c->z.p, c->x.p, c->stream),
             "axpby");
          if ((rc = c->halo(c->x.p, c->nf))) return rc;
          if ((rc = c->assemble(c->x.p, 0))) return rc;
          if ((rc = c->norm(c->r.p, defect))) return rc;
        }
        break;
      }
      lambda *= 0.5;
    }
    if (ls_fail) {
      res->status = PNP_E_NOT_CONVERGED;
      break;
    }
    res->iterations++;
    c->newton_its.push_back(step_its);
    c->newton_defects.push_back(defect);
  }
  res->defect = defect;
  if ((rc = c->download_ext(c->x.p, c->nf, u))) return rc;
  res->elapsed = now_s() - t_start;
  return PNP_OK;
}

// owner-masked dot of two external-layout vectors (this rank's owned entries), allreduced
static int dot_ext(pnp_ctx *c, const double *a, const double *b, int nfields, int32_t flags,
                   double *out) {
  if (!c || !a || !b || !out || nfields < 1 || nfields > 3) return PNP_E_ARG;
  int rc;
  if ((rc = check_flags(c, flags, PNP_DEVICE_PTRS))) return rc;
  hipSetDevice(c->device);
  const bool dev = flags & PNP_DEVICE_PTRS;
  if ((rc = c->upload_ext(a, nfields, c->t.p, false, dev))) return rc;
  if (b != a && (rc = c->upload_ext(b, nfields, c->y.p, false, dev))) return rc;
  const long long n = (long long)c->L.n_owned * nfields;
  CK(pnp::launch_dot(n, c->t.p, b != a ? c->y.p : c->t.p, 0, c->partials.p, c->stream), "dot");
  CK(pnp::launch_reduce(c->partials.p, pnp::blas_nparts(n), 1, c->S.p + 1, c->stream), "dot");
  if (c->dist) {
    double *red = reinterpret_cast<double *>(reinterpret_cast<char *>(c->S.p + 1) +
                                             offsetof(pnp::Scalars, red));
    if ((rc = c->allreduce_dev(red, 1))) return rc;
  }
  CK(hipMemcpyAsync(c->hS + 1, c->S.p + 1, sizeof(pnp::Scalars), hipMemcpyDeviceToHost, c->stream),
     "dot readback");
  CK(hipStreamSynchronize(c->stream), "dot readback");
  *out = c->hS[1].red[0];
  return PNP_OK;
}

extern "C" int pnp_dot(pnp_ctx *c, const double *a, const double *b, int32_t nfields,
                       int32_t flags, double *out) {
  return dot_ext(c, a, b, nfields, flags, out);
}

extern "C" int pnp_norm(pnp_ctx *c, const double *a, int32_t nfields, int32_t flags, double *out) {
  const int rc = dot_ext(c, a, a, nfields, flags, out);
  if (rc == PNP_OK) *out = std::sqrt(*out);
  return rc;
}

extern "C" int pnp_newton_history(pnp_ctx *c, int32_t *its, double *defects, int32_t cap,
                                  int32_t *nsteps) {
  if (!c || !nsteps || cap < 0) return PNP_E_ARG;
  const int n = int(c->newton_its.size());
  *nsteps = n;
  for (int k = 0; k < std::min(n, int(cap)); k++) {
    if (its) its[k] = c->newton_its[k];
    if (defects) defects[k] = c->newton_defects[k];
  }
  return PNP_OK;
}

extern "C" int pnp_sync_vector(pnp_ctx *c, double *v, int32_t nfields) {
  if (!c || !v || nfields < 1 || nfields > 3) return PNP_E_ARG;
  if (!c->dist) return PNP_OK;
  hipSetDevice(c->device);
  size_t nv = size_t(c->mesh.nv), n = nv * nfields;
  std::vector<double> mine(n, 0.0);
  for (int i = 0; i < c->L.n_owned; i++)
    for (int f = 0; f < nfields; f++) mine[f * nv + c->L.l2g[i]] = v[f * nv + c->L.l2g[i]];
  CK(hipMemcpy(c->ext.p, mine.data(), sizeof(double) * n, hipMemcpyHostToDevice), "sync upload");
  int rc = c->allreduce_dev(c->ext.p, int(n));
  if (rc) return rc;
  CK(hipStreamSynchronize(c->stream), "sync");
  CK(hipMemcpy(v, c->ext.p, sizeof(double) * n, hipMemcpyDeviceToHost), "sync download");
  return PNP_OK;
}

extern "C" int pnp_initial_state(pnp_ctx *c, const double *phi_pb, double *x0) {
  if (!c || !x0) return PNP_E_ARG;
  if (c->degree > 1)
    pnp::pk_initial_state(c->tmesh, c->pks, c->params, phi_pb, x0);
  else
    pnp::initial_state(c->mesh, c->params, phi_pb, x0);
  return PNP_OK;
}

extern "C" int pnp_space(pnp_ctx *c, pnp_space_info *info, double *xy, int32_t *enode) {
  if (!c || !info) return PNP_E_ARG;
  const bool pk = c->degree > 1;
  info->degree = c->degree;
  info->nnodes = c->mesh.nv;
  info->nt = pk ? c->tmesh.nt : c->mesh.nt;
  info->nlocal = pk ? c->pks.nl : 3;
  if (xy) std::memcpy(xy, c->mesh.xy.data(), sizeof(double) * c->mesh.xy.size());
  if (enode) {
    const std::vector<int> &en = pk ? c->pks.enode : c->mesh.tri;
    std::memcpy(enode, en.data(), sizeof(int) * en.size());
  }
  return PNP_OK;
}

// ---------------------------------------------------------------------------------------------
// device-resident hot path (benchmarks)
// ---------------------------------------------------------------------------------------------
extern "C" int pnp_state_set(pnp_ctx *c, const double *x) {
  if (!c || !x) return PNP_E_ARG;
  if (c->kind < 0) return c->fail(PNP_E_STATE, "no operator set");
  hipSetDevice(c->device);
  int rc = c->upload_ext(x, c->nf, c->x.p, true);
  if (rc) return rc;
  CK(hipStreamSynchronize(c->stream), "state_set");
  return PNP_OK;
}

extern "C" int pnp_state_get(pnp_ctx *c, double *x) {
  if (!c || !x) return PNP_E_ARG;
  hipSetDevice(c->device);
  return c->download_ext(c->x.p, c->nf, x);
}

extern "C" int pnp_assemble_state(pnp_ctx *c, int32_t n) {
  if (!c) return PNP_E_ARG;
  hipSetDevice(c->device);
  const int jac = n >= 0 ? 1 : 0;  // n < 0: |n| residual-only assemblies (line-search kernel)
  for (int k = 0; k < (n >= 0 ? n : -n); k++) {
    int rc = c->assemble(c->x.p, jac);
    if (rc) return rc;
  }
  CK(hipStreamSynchronize(c->stream), "assemble_state");
  return PNP_OK;
}

extern "C" int pnp_assemble_state_timed(pnp_ctx *c, int32_t n, double *ms) {
  if (!c || !ms || n == 0) return PNP_E_ARG;
  hipSetDevice(c->device);
  // one event pair around the whole batch (no per-launch events inside it): the device time of
  // |n| back-to-back launches, as a kernel trace sees them
  const bool timing = c->timing;
  c->timing = false;
  hipEvent_t e0 = c->ev_get(), e1 = c->ev_get();
  hipEventRecord(e0, c->stream);
  int rc = PNP_OK;
  for (int k = 0; k < (n >= 0 ? n : -n) && rc == PNP_OK; k++) rc = c->assemble(c->x.p, n >= 0);
  hipEventRecord(e1, c->stream);
  c->timing = timing;
  const hipError_t e = hipStreamSynchronize(c->stream);
  float t = 0;
  if (rc == PNP_OK && e == hipSuccess) hipEventElapsedTime(&t, e0, e1);
  c->ev_pool.push_back(e0);
  c->ev_pool.push_back(e1);
  if (rc) return rc;
  CK(e, "assemble_state_timed");
  *ms = t;
  return PNP_OK;
}

extern "C" int pnp_bicgstab_iterations(pnp_ctx *c, int32_t n, int32_t prec, pnp_solve_result *res) {
  if (!c || !res || n <= 0) return PNP_E_ARG;
  hipSetDevice(c->device);
  std::memset(res, 0, sizeof *res);
  pnp_solve_opts o{};
  o.prec = prec;
  o.maxit = n;
  CK(hipMemcpyAsync(c->b.p, c->r.p, sizeof(double) * c->nown(), hipMemcpyDeviceToDevice,
                    c->stream),
     "rhs");
  c->amg_symmetric = false;  // as in krylov(): BiCGSTAB
  c->after_solve = true;
  int rc = c->bicgstab(c->b.p, c->z.p, o, *res, n);
  c->amg_symmetric = true;
  return rc;
}

extern "C" int pnp_probe_slot_stores(pnp_ctx *c, int32_t tile_elems, int32_t reps,
                                     pnp_store_probe *out) {
  if (!c || !out || tile_elems <= 0 || reps <= 0) return PNP_E_ARG;
  if (c->degree < 2) return c->fail(PNP_E_ARG, "pnp_probe_slot_stores: P_k contexts only");
  hipSetDevice(c->device);
  std::memset(out, 0, sizeof *out);
  const int nl = c->pks.nl, no = c->L.n_owned;
  // pk_build's local elements: ascending global id, every element with an owned node
  std::vector<int> first(no, -1), last(no, -1);
  int ne = 0;
  for (int e = 0; e < c->tmesh.nt; e++) {
    const int *g = &c->pks.enode[size_t(e) * nl];
    bool mine = false;
    for (int a = 0; a < nl; a++) {
      const int l = c->L.g2l[g[a]];
      mine = mine || (l >= 0 && l < no);
    }
    if (!mine) continue;
    for (int a = 0; a < nl; a++) {
      const int l = c->L.g2l[g[a]];
      if (l < 0 || l >= no) continue;
      if (first[l] < 0) first[l] = ne;
      last[l] = ne;
    }
    ne++;
  }
  std::vector<int> tile(no), tsort(no), rnd(no);
  long long slots = 0;
  for (int r = 0; r < no; r++) {
    tile[r] = tsort[r] = rnd[r] = r;
    slots += pnp::meta_len(c->L.rowmeta[r]);
    out->rows_whole += first[r] / tile_elems == last[r] / tile_elems;
  }
  std::stable_sort(tile.begin(), tile.end(), [&](int a, int b) { return first[a] < first[b]; });
  std::stable_sort(tsort.begin(), tsort.end(),
                   [&](int a, int b) { return first[a] / tile_elems < first[b] / tile_elems; });
  std::mt19937 rng(20261018);
  std::shuffle(rnd.begin(), rnd.end(), rng);
  const std::vector<int> *hv[3] = {&tile, &tsort, &rnd};
  DBuf<int> d_ord[3];
  DBuf<double> val;
  for (int k = 0; k < 3; k++) {
    CK(d_ord[k].alloc(std::max(1, no)), "probe order");
    CK(hipMemcpy(d_ord[k].p, hv[k]->data(), sizeof(int) * no, hipMemcpyHostToDevice), "probe order");
  }
  CK(val.alloc(std::max<size_t>(1, size_t(c->L.chunk_off[c->L.nchunks]))), "probe slots");
  const int *orders[4] = {nullptr, d_ord[0].p, d_ord[1].p, d_ord[2].p};
  double *res[4] = {&out->us_sell, &out->us_tile, &out->us_tile_sorted, &out->us_random};
  for (int k = 0; k < 4; k++) {
    for (int w = 0; w < 2; w++) CK(pnp::launch_slot_store_probe(c->dl, orders[k], val.p, c->stream), "probe");
    hipEvent_t e0 = c->ev_get(), e1 = c->ev_get();
    hipEventRecord(e0, c->stream);
    for (int i = 0; i < reps; i++) CK(pnp::launch_slot_store_probe(c->dl, orders[k], val.p, c->stream), "probe");
    hipEventRecord(e1, c->stream);
    const hipError_t e = hipStreamSynchronize(c->stream);
    float t = 0;
    if (e == hipSuccess) hipEventElapsedTime(&t, e0, e1);
    c->ev_pool.push_back(e0);
    c->ev_pool.push_back(e1);
    CK(e, "probe");
    *res[k] = 1e3 * t / reps;
  }
  out->slot_bytes = 8 * slots;
  out->rows = no;
  out->tiles = (ne + tile_elems - 1) / tile_elems;
  out->elements = ne;
  return PNP_OK;
}

extern "C" int pnp_cache_scrub(pnp_ctx *c, int64_t bytes) {
  if (!c || bytes < 0) return PNP_E_ARG;
  hipSetDevice(c->device);
  const size_t n = size_t(bytes) / 8;
  if (c->scrub.n < n + 1) CK(c->scrub.alloc(n + 1), "scrub buffer");
  CK(pnp::launch_scrub(c->scrub.p, (long long)n, c->scrub.p + n, c->stream), "scrub");
  CK(hipStreamSynchronize(c->stream), "scrub");
  return PNP_OK;
}

extern "C" int pnp_timers_enable(pnp_ctx *c, int32_t on) {
  if (!c) return PNP_E_ARG;
  c->timing = on != 0;
  return PNP_OK;
}

extern "C" int pnp_timers_get(pnp_ctx *c, pnp_timers *t) {
  if (!c || !t) return PNP_E_ARG;
  c->timers_flush();
  t->assemble_ms = c->t_ms[T_ASM];
  t->spmv_ms = c->t_ms[T_SPMV];
  t->prec_ms = c->t_ms[T_PREC];
  t->blas_ms = c->t_ms[T_BLAS];
  t->halo_ms = c->t_ms[T_HALO];
  t->allreduce_ms = c->t_ms[T_ALLRED];
  t->assemble_launches = c->t_n[T_ASM];
  t->spmv_launches = c->t_n[T_SPMV];
  t->prec_launches = c->t_n[T_PREC];
  t->blas_launches = c->t_n[T_BLAS];
  t->factor_ms = c->t_ms[T_FACT];
  t->factor_launches = c->t_n[T_FACT];
  return PNP_OK;
}

extern "C" int pnp_timers_reset(pnp_ctx *c) {
  if (!c) return PNP_E_ARG;
  c->timers_flush();
  for (int k = 0; k < T_NCAT; k++) {
    c->t_ms[k] = 0;
    c->t_n[k] = 0;
  }
  return PNP_OK;
}

// ---------------------------------------------------------------------------------------------
// host-only setup / inspection
// ---------------------------------------------------------------------------------------------
struct pnp_layout_buf {
  pnp::Fans fans;
  pnp::LocalLayout L;
  std::vector<int> chunk_off32;
};

extern "C" int pnp_setup_boundary(const pnp_mesh *mesh, const pnp_params *params, int32_t nfields,
                                  int32_t field0, uint8_t *mask, double *load) {
  if (!params || nfields < 1 || field0 < 0 || field0 + nfields > 3) return PNP_E_ARG;
  pnp::Mesh m;
  std::string err;
  if (!mesh_from_view(mesh, m, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  pnp::Params P;
  params_from(params, P);
  for (int s = 0; s < m.nb; s++)
    if (m.bgroup[s] < 0 || m.bgroup[s] >= int(P.surf.size())) return PNP_E_ARG;
  std::vector<uint8_t> mk;
  std::vector<double> ld;
  pnp::dirichlet_mask(m, P, nfields, field0, mk);
  pnp::neumann_load(m, P, nfields, field0, ld);
  for (int v = 0; v < m.nv; v++)
    for (int f = 0; f < nfields; f++) {
      if (mask) mask[size_t(f) * m.nv + v] = mk[size_t(v) * nfields + f];
      if (load) load[size_t(f) * m.nv + v] = ld[size_t(v) * nfields + f];
    }
  return PNP_OK;
}

extern "C" int pnp_setup_initial_state(const pnp_mesh *mesh, const pnp_params *params,
                                       const double *phi_pb, double *x0) {
  if (!params || !x0) return PNP_E_ARG;
  pnp::Mesh m;
  std::string err;
  if (!mesh_from_view(mesh, m, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  pnp::Params P;
  params_from(params, P);
  for (int s = 0; s < m.nb; s++)
    if (m.bgroup[s] < 0 || m.bgroup[s] >= int(P.surf.size())) return PNP_E_ARG;
  pnp::initial_state(m, P, phi_pb, x0);
  return PNP_OK;
}

extern "C" int pnp_layout_build(const pnp_mesh *mesh, int32_t rank, int32_t nranks,
                                pnp_layout_buf **out) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks) return PNP_E_ARG;
  pnp::Mesh m;
  std::string err;
  if (!mesh_from_view(mesh, m, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  auto b = std::make_unique<pnp_layout_buf>();
  if (!pnp::build_fans(m, b->fans, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  std::vector<int> part;
  pnp::rcb_partition(m, nranks, part);
  if (!pnp::build_local_layout(m, b->fans, part, rank, nranks, b->L, err)) {
    g_err = err;
    return PNP_E_MESH;
  }
  *out = b.release();
  return PNP_OK;
}

extern "C" int pnp_layout_view(const pnp_layout_buf *b, pnp_layout *v) {
  if (!b || !v) return PNP_E_ARG;
  const pnp::LocalLayout &L = b->L;
  v->n_owned = L.n_owned;
  v->n_ghost = L.n_ghost;
  v->ncolors = int(L.color_ptr.size()) - 1;
  v->nchunks = L.nchunks;
  v->nnbr = int(L.nbr_ranks.size());
  v->max_slots = b->fans.max_slots;
  v->nslots = L.nslots;
  v->nblocks = L.nblocks;
  v->l2g = L.l2g.data();
  v->color_ptr = L.color_ptr.data();
  v->color_idx = L.color_idx.data();
  v->rowcolor = L.rowcolor.data();
  v->chunk_len = L.chunk_len.data();
  v->chunk_off = L.chunk_off.data();
  v->colidx = L.colidx.data();
  v->rowmeta = L.rowmeta.data();
  v->nbr_ranks = L.nbr_ranks.data();
  v->recv_ptr = L.recv_ptr.data();
  v->send_ptr = L.send_ptr.data();
  v->send_idx = L.send_idx.data();
  v->color_conflicts = L.conflicts;
  return PNP_OK;
}

extern "C" void pnp_layout_free(pnp_layout_buf *b) { delete b; }
