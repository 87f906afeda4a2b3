"""Host-side mirror of the reference's PDELab/ISTL surface over libpnp_amd.so (ctypes).

This is the Python face of the C ABI in include/pnp_capi.h.  It mirrors the reference's
objects and call sequence (src/stationary_pnp_from_pb.hh:93-369):

    Sysparams / readConfigFile        -> read_config()           (src/sysparams.cc:16-98)
    GmshReader + UGGrid               -> Mesh.read_gmsh(), Mesh.refine()
    GridOperator(GFS, CC, LOP)        -> Context.set_operator(OP_PNP | OP_PB | ...)
    go.residual(u, r) / go.jacobian   -> Context.residual(x) / Context.jacobian(x)
    ISTLBackend_NOVLP_BCGS_*.apply    -> Context.linear_solve(rhs, prec=...)
    Newton::apply                     -> Context.newton(u, ...)
    interpolate(BCExtension)          -> Context.initial_state(phi_pb)

Everything numeric runs in the HIP kernels of libpnp_amd.so; there is no Python or CPU fallback:
if the shared library is missing or the GPU is absent, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(os.path.dirname(HERE))          # dune-pnp_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
LIB_PATH = os.environ.get("PNP_AMD_LIB") or os.path.join(PKG_ROOT, "libpnp_amd.so")
HEADER = os.path.join(REPO_ROOT, "include", "pnp_capi.h")

OK, E_ARG, E_HIP, E_RCCL, E_BREAKDOWN, E_NOT_CONVERGED, E_IO, E_MESH, E_STATE = \
    0, -1, -2, -3, -4, -5, -6, -7, -8
OP_PNP, OP_PNP_IMPLICIT_EULER, OP_PB, OP_DIFF, OP_DIFF_IMPLICIT_EULER, OP_POISSON = range(6)
PREC_NONE, PREC_SSOR, PREC_ILU0, PREC_JACOBI, PREC_AMG, PREC_SSOR_NATURAL = range(6)
METHOD_BICGSTAB, METHOD_CG = 0, 1
(OPT_ILU_F32, OPT_ILU_FUSED_FACTOR, OPT_JAC_FD, OPT_BICG_TWORED, OPT_AMG_FALLBACK,
 OPT_GRAPH, OPT_SEQ_ORDER, OPT_ILU_FLOW, OPT_NAT_FLOW, OPT_ILU_RETRY) = 1, 2, 3, 4, 5, 6, 7, 8, 9, 10
DEVICE_PTRS, JAC_FD = 1, 2
CREATE_ABSORB_THIN_COLOR = 1
PREC_BY_NAME = {"none": PREC_NONE, "nonprec": PREC_NONE, "ssor": PREC_SSOR, "ilu0": PREC_ILU0,
                "jacobi": PREC_JACOBI, "amg": PREC_AMG, "ssor_natural": PREC_SSOR_NATURAL}
MAX_SURFACES = 64


class PnpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"pnp error {code}: {msg}")
        self.code = code


# ------------------------------------------------------------------------------------------------
# ctypes structures (must match include/pnp_capi.h)
# ------------------------------------------------------------------------------------------------
class _Mesh(C.Structure):
    _fields_ = [("nv", C.c_int32), ("coords", C.c_void_p), ("nt", C.c_int32),
                ("tri", C.c_void_p), ("nbseg", C.c_int32), ("bseg", C.c_void_p),
                ("bseg_group", C.c_void_p)]


class _Surface(C.Structure):
    _fields_ = [("coulomb_btype", C.c_int32), ("coulomb_flux", C.c_double),
                ("coulomb_potential", C.c_double), ("plus_btype", C.c_int32),
                ("plus_flux", C.c_double), ("plus_concentration", C.c_double),
                ("minus_btype", C.c_int32), ("minus_flux", C.c_double),
                ("minus_concentration", C.c_double)]


class _Params(C.Structure):
    _fields_ = [("l_b", C.c_double), ("c0", C.c_double), ("tau", C.c_double), ("pi", C.c_double),
                ("cylindrical", C.c_int32), ("n_surfaces", C.c_int32), ("surfaces", C.c_void_p)]


class _Config(C.Structure):
    _fields_ = [("meshfile", C.c_char * 1024), ("n_surfaces", C.c_int32),
                ("verbosity", C.c_int32), ("cylindrical", C.c_int32),
                ("linear_solver_iterations", C.c_int32), ("l_b", C.c_double),
                ("newton_reassemble_threshold", C.c_double), ("newton_reduction", C.c_double),
                ("newton_min_linear_reduction", C.c_double), ("newton_max_iterations", C.c_int32),
                ("newton_line_search_max_iteration", C.c_int32), ("c0", C.c_double),
                ("tau", C.c_double), ("output_freq", C.c_int32), ("n_steps", C.c_int32),
                ("potential_update_freq", C.c_int32), ("surfaces", _Surface * MAX_SURFACES),
                ("defaulted", C.c_uint32)]


_EXCHANGE_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_int32),
                           C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                           C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(C.c_int64))
_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.POINTER(C.c_double), C.c_int32)


class _HostTransport(C.Structure):
    _fields_ = [("user", C.c_void_p), ("exchange", _EXCHANGE_FN),
                ("allreduce_sum", _ALLREDUCE_FN)]


class _Comm(C.Structure):
    _fields_ = [("rank", C.c_int32), ("size", C.c_int32), ("rccl_unique_id", C.c_void_p),
                ("local_group", C.c_char_p), ("host", C.POINTER(_HostTransport))]


class TorchDistTransport:
    """A host transport (pnp_comm.host) over an initialised torch.distributed process group (gloo):
    point-to-point halo exchange, all_reduce sums.  For ranks that cannot use RCCL -- several
    processes on one GPU (tests/test_gpu_dist_host.py, `bench.py --transport host`)."""

    def __init__(self, dist=None):
        import torch
        if dist is None:
            import torch.distributed as dist
        self.dist, self.torch = dist, torch
        self.calls = {"exchange": 0, "allreduce": 0}

    def exchange(self, peers, sends, rcounts):
        self.calls["exchange"] += 1
        reqs, outs = [], []
        for q, peer in enumerate(peers):
            buf = self.torch.empty(int(rcounts[q]), dtype=self.torch.float64)
            outs.append(buf)
            if len(sends[q]):
                reqs.append(self.dist.isend(self.torch.from_numpy(sends[q]), peer))
            if rcounts[q]:
                reqs.append(self.dist.irecv(buf, peer))
        for r in reqs:
            r.wait()
        return [o.numpy() for o in outs]

    def allreduce_sum(self, buf):
        self.calls["allreduce"] += 1
        self.dist.all_reduce(self.torch.from_numpy(buf))  # shares the staging memory


def _host_transport(obj):
    """pnp_host_transport over a Python object with
         exchange(nbr, sends, recv_counts) -> list of received arrays  (sends: list of arrays)
         allreduce_sum(buf)  (in place, a float64 numpy array)
    e.g. tools / tests built on torch.distributed (gloo).  Exceptions become a failed call."""
    def exchange(_u, nq, nbr, sbuf, soff, scnt, rbuf, roff, rcnt):
        try:
            peers = [nbr[q] for q in range(nq)]
            sends = [np.ctypeslib.as_array(sbuf, shape=(max(1, soff[q] + scnt[q]),))
                     [soff[q]:soff[q] + scnt[q]].copy() for q in range(nq)]
            got = obj.exchange(peers, sends, [rcnt[q] for q in range(nq)])
            for q in range(nq):
                if rcnt[q]:
                    dst = np.ctypeslib.as_array(rbuf, shape=(roff[q] + rcnt[q],))
                    dst[roff[q]:roff[q] + rcnt[q]] = got[q]
            return 0
        except Exception:  # noqa: BLE001 -- reported to the library as a failed exchange
            import traceback
            traceback.print_exc()
            return 1

    def allreduce(_u, buf, k):
        try:
            obj.allreduce_sum(np.ctypeslib.as_array(buf, shape=(k,)))
            return 0
        except Exception:  # noqa: BLE001
            import traceback
            traceback.print_exc()
            return 1
    fx, fa = _EXCHANGE_FN(exchange), _ALLREDUCE_FN(allreduce)
    return _HostTransport(None, fx, fa), (fx, fa)


class _Info(C.Structure):
    _fields_ = [("nv_global", C.c_int32), ("nv_owned", C.c_int32), ("nv_ghost", C.c_int32),
                ("nfields", C.c_int32), ("ncolors", C.c_int32), ("nchunks", C.c_int32),
                ("max_slots", C.c_int32), ("nranks", C.c_int32), ("nblocks", C.c_int64),
                ("nnz_reduced", C.c_int64), ("nslots", C.c_int64), ("device_bytes", C.c_int64),
                ("nks", C.c_int32), ("nvb", C.c_int32), ("lslots", C.c_int64),
                ("uslots", C.c_int64), ("ilu_f32", C.c_int32), ("degree", C.c_int32),
                ("color_conflicts", C.c_int64), ("transport", C.c_int32),
                ("nat_flow_applies", C.c_int64), ("nat_level_applies", C.c_int64),
                ("ilu_flow_applies", C.c_int64), ("lslots_live", C.c_int64),
                ("uslots_live", C.c_int64), ("lsx_entries", C.c_int64),
                ("usx_entries", C.c_int64)]


class _SpaceInfo(C.Structure):
    _fields_ = [("degree", C.c_int32), ("nnodes", C.c_int32), ("nt", C.c_int32),
                ("nlocal", C.c_int32)]


class _StoreProbe(C.Structure):
    _fields_ = [("us_sell", C.c_double), ("us_tile", C.c_double), ("us_tile_sorted", C.c_double),
                ("us_random", C.c_double),
                ("slot_bytes", C.c_int64), ("rows", C.c_int64), ("rows_whole", C.c_int64),
                ("tiles", C.c_int64), ("elements", C.c_int64)]


class _OpArgs(C.Structure):
    _fields_ = [("kind", C.c_int32), ("dt", C.c_double), ("z", C.c_double),
                ("field", C.c_int32), ("phi", C.c_void_p), ("cp", C.c_void_p),
                ("cm", C.c_void_p), ("x_old", C.c_void_p), ("c_extra", C.c_void_p)]


class _SolveOpts(C.Structure):
    _fields_ = [("prec", C.c_int32), ("reduction", C.c_double), ("maxit", C.c_int32),
                ("check_every", C.c_int32), ("method", C.c_int32)]


class _SolveResult(C.Structure):
    _fields_ = [("converged", C.c_int32), ("iterations", C.c_int32), ("breakdown", C.c_int32),
                ("it_half", C.c_double), ("defect0", C.c_double), ("defect", C.c_double),
                ("reduction", C.c_double), ("elapsed", C.c_double)]


class _AmgOpts(C.Structure):
    _fields_ = [("smoother", C.c_int32), ("coarse_target", C.c_int32), ("max_levels", C.c_int32),
                ("omega", C.c_double), ("coarse_sweeps", C.c_int32),
                ("level0_presmooth", C.c_int32)]


class _AmgStats(C.Structure):
    _fields_ = [("levels", C.c_int32), ("smoother", C.c_int32), ("rows", C.c_int32 * 16),
                ("blocks", C.c_int64 * 16), ("omega", C.c_double)]


class _NewtonOpts(C.Structure):
    _fields_ = [("reduction", C.c_double), ("abs_limit", C.c_double),
                ("min_linear_reduction", C.c_double), ("maxit", C.c_int32),
                ("line_search_maxit", C.c_int32), ("linear", _SolveOpts)]


class _NewtonResult(C.Structure):
    _fields_ = [("converged", C.c_int32), ("iterations", C.c_int32),
                ("linear_iterations", C.c_int32), ("status", C.c_int32),
                ("first_defect", C.c_double), ("defect", C.c_double), ("elapsed", C.c_double),
                ("assemble_seconds", C.c_double), ("solve_seconds", C.c_double),
                ("linear_fallbacks", C.c_int32), ("precision_retries", C.c_int32)]


class _Timers(C.Structure):
    _fields_ = [("assemble_ms", C.c_double), ("spmv_ms", C.c_double), ("prec_ms", C.c_double),
                ("blas_ms", C.c_double), ("halo_ms", C.c_double), ("allreduce_ms", C.c_double),
                ("assemble_launches", C.c_int64), ("spmv_launches", C.c_int64),
                ("prec_launches", C.c_int64), ("blas_launches", C.c_int64),
                ("factor_ms", C.c_double), ("factor_launches", C.c_int64)]


class _CsrView(C.Structure):
    _fields_ = [("n", C.c_int32), ("nnz", C.c_int64), ("rowptr", C.c_void_p), ("col", C.c_void_p),
                ("val", C.c_void_p)]


class _Layout(C.Structure):
    _fields_ = [("n_owned", C.c_int32), ("n_ghost", C.c_int32), ("ncolors", C.c_int32),
                ("nchunks", C.c_int32), ("nnbr", C.c_int32), ("max_slots", C.c_int32),
                ("nslots", C.c_int64), ("nblocks", C.c_int64),
                ("l2g", C.POINTER(C.c_int32)), ("color_ptr", C.POINTER(C.c_int32)),
                ("color_idx", C.POINTER(C.c_int32)), ("rowcolor", C.POINTER(C.c_uint8)),
                ("chunk_len", C.POINTER(C.c_int32)), ("chunk_off", C.POINTER(C.c_int32)),
                ("colidx", C.POINTER(C.c_int32)), ("rowmeta", C.POINTER(C.c_uint64)),
                ("nbr_ranks", C.POINTER(C.c_int32)), ("recv_ptr", C.POINTER(C.c_int32)),
                ("send_ptr", C.POINTER(C.c_int32)), ("send_idx", C.POINTER(C.c_int32)),
                ("color_conflicts", C.c_int64)]


_LIB = None


def lib():
    """Load libpnp_amd.so; raises if it has not been built (no silent fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise PnpError(E_IO, f"{LIB_PATH} not built (run __graft_entry__.build() or make -C "
                                 f"dune-pnp_amd)")
        L = C.CDLL(LIB_PATH)
        L.pnp_last_error.restype = C.c_char_p
        L.pnp_last_error.argtypes = [C.c_void_p]
        L.pnp_create.argtypes = [C.POINTER(_Mesh), C.POINTER(_Params), C.c_int32,
                                 C.POINTER(_Comm), C.POINTER(C.c_void_p)]
        L.pnp_create_pk.argtypes = [C.POINTER(_Mesh), C.POINTER(_Params), C.c_int32, C.c_int32,
                                    C.POINTER(_Comm), C.POINTER(C.c_void_p)]
        for name in ("pnp_destroy", "pnp_mesh_free", "pnp_layout_free"):
            getattr(L, name).restype = None
            getattr(L, name).argtypes = [C.c_void_p]
        _LIB = L
    return _LIB


def _check(rc, ctx=None):
    if rc != OK:
        msg = lib().pnp_last_error(ctx)
        raise PnpError(rc, (msg or b"").decode())


def _ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


# ------------------------------------------------------------------------------------------------
# mesh + config
# ------------------------------------------------------------------------------------------------
class Mesh:
    """Triangle mesh + boundary segments (what GmshReader hands the reference)."""

    def __init__(self, xy, tri, bseg, bgroup):
        self.xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 2)
        self.tri = np.ascontiguousarray(tri, dtype=np.int32).reshape(-1, 3)
        self.bseg = np.ascontiguousarray(bseg, dtype=np.int32).reshape(-1, 2)
        self.bgroup = np.ascontiguousarray(bgroup, dtype=np.int32).reshape(-1)

    nv = property(lambda s: s.xy.shape[0])
    nt = property(lambda s: s.tri.shape[0])
    nb = property(lambda s: s.bseg.shape[0])

    def c(self):
        return _Mesh(self.nv, self.xy.ctypes.data, self.nt, self.tri.ctypes.data, self.nb,
                     self.bseg.ctypes.data, self.bgroup.ctypes.data)

    @staticmethod
    def _from_buf(buf):
        v = _Mesh()
        _check(lib().pnp_mesh_view(buf, C.byref(v)))
        xy = np.ctypeslib.as_array(C.cast(v.coords, C.POINTER(C.c_double)), (v.nv * 2,)).copy()
        tri = np.ctypeslib.as_array(C.cast(v.tri, C.POINTER(C.c_int32)), (v.nt * 3,)).copy()
        if v.nbseg:
            bs = np.ctypeslib.as_array(C.cast(v.bseg, C.POINTER(C.c_int32)), (v.nbseg * 2,)).copy()
            bg = np.ctypeslib.as_array(C.cast(v.bseg_group, C.POINTER(C.c_int32)),
                                       (v.nbseg,)).copy()
        else:
            bs, bg = np.zeros(0, np.int32), np.zeros(0, np.int32)
        lib().pnp_mesh_free(buf)
        return Mesh(xy, tri, bs, bg)

    @staticmethod
    def read_gmsh(path):
        buf = C.c_void_p()
        _check(lib().pnp_mesh_read_gmsh(path.encode(), C.byref(buf)))
        return Mesh._from_buf(buf)

    @staticmethod
    def from_geo(path, size_scale=1.0):
        """gmsh's preprocessing of a .geo geometry, natively (pnp_mesh_from_geo)."""
        buf = C.c_void_p()
        _check(lib().pnp_mesh_from_geo(path.encode(), C.c_double(size_scale), C.byref(buf)))
        return Mesh._from_buf(buf)

    @staticmethod
    def load(meshfile, size_scale=1.0):
        """The mesh a config names: the .msh if it exists, else the .geo of the same name meshed
        here (the reference's workflow runs gmsh on the .geo first, e.g.
        test/pore_without_dna/pore.cfg:21 names a .msh that only exists as a .geo)."""
        if os.path.exists(meshfile):
            return Mesh.read_gmsh(meshfile)
        geo = os.path.splitext(meshfile)[0] + ".geo"
        if os.path.exists(geo):
            return Mesh.from_geo(geo, size_scale)
        return Mesh.read_gmsh(meshfile)  # raises the reader's error

    def write_gmsh(self, path):
        m = self.c()
        _check(lib().pnp_mesh_write_gmsh(C.byref(m), path.encode()))

    def refine(self, k):
        if k == 0:
            return self
        buf = C.c_void_p()
        m = self.c()
        _check(lib().pnp_mesh_refine(C.byref(m), int(k), C.byref(buf)))
        return Mesh._from_buf(buf)


@dataclass
class Surface:
    cb: int = 1
    cflux: float = 0.0
    cpot: float = 0.0
    pb: int = 1
    pflux: float = 0.0
    pconc: float = 0.0
    mb: int = 1
    mflux: float = 0.0
    mconc: float = 0.0


@dataclass
class Config:
    meshfile: str
    system: dict
    surfaces: list
    defaulted_mask: int


_SYSTEM_KEYS = ["verbosity", "cylindrical", "l_b", "linearSolverIterations",
                "newtonReassembleThreshold", "newtonReduction", "newtonMinLinearReduction",
                "newtonMaxIterations", "newtonLineSearchMaxIteration", "c0", "tau", "outputFreq",
                "nSteps", "potentialUpdateFreq"]


def read_config(path) -> Config:
    c = _Config()
    _check(lib().pnp_config_read(str(path).encode(), C.byref(c)))
    system = {"verbosity": c.verbosity, "cylindrical": c.cylindrical, "l_b": c.l_b,
              "linearSolverIterations": c.linear_solver_iterations,
              "newtonReassembleThreshold": c.newton_reassemble_threshold,
              "newtonReduction": c.newton_reduction,
              "newtonMinLinearReduction": c.newton_min_linear_reduction,
              "newtonMaxIterations": c.newton_max_iterations,
              "newtonLineSearchMaxIteration": c.newton_line_search_max_iteration,
              "c0": c.c0, "tau": c.tau, "outputFreq": c.output_freq, "nSteps": c.n_steps,
              "potentialUpdateFreq": c.potential_update_freq, "n_surfaces": c.n_surfaces}
    surfs = []
    for i in range(c.n_surfaces):
        s = c.surfaces[i]
        surfs.append(Surface(s.coulomb_btype, s.coulomb_flux, s.coulomb_potential, s.plus_btype,
                             s.plus_flux, s.plus_concentration, s.minus_btype, s.minus_flux,
                             s.minus_concentration))
    return Config(c.meshfile.decode(), system, surfs, int(c.defaulted))


def defaulted_keys(cfg: Config):
    return [k for i, k in enumerate(_SYSTEM_KEYS) if (cfg.defaulted_mask >> i) & 1]


class Params:
    def __init__(self, surfaces, l_b=1.0, c0=0.06, tau=1.0, cylindrical=0, pi=3.1415):
        arr = (_Surface * max(1, len(surfaces)))()
        for i, s in enumerate(surfaces):
            arr[i] = _Surface(s.cb, s.cflux, s.cpot, s.pb, s.pflux, s.pconc, s.mb, s.mflux,
                              s.mconc)
        self._arr = arr
        self.c = _Params(l_b, c0, tau, pi, int(cylindrical), len(surfaces),
                         C.cast(arr, C.c_void_p).value)
        self.surfaces = surfaces

    @staticmethod
    def from_config(cfg: Config, pi=3.1415):
        s = cfg.system
        return Params(cfg.surfaces, l_b=s["l_b"], c0=s["c0"], tau=s["tau"],
                      cylindrical=s["cylindrical"], pi=pi)


# ------------------------------------------------------------------------------------------------
# host-only setup
# ------------------------------------------------------------------------------------------------
def setup_boundary(mesh: Mesh, params: Params, nfields, field0=0):
    mask = np.zeros(nfields * mesh.nv, dtype=np.uint8)
    load = np.zeros(nfields * mesh.nv, dtype=np.float64)
    m = mesh.c()
    _check(lib().pnp_setup_boundary(C.byref(m), C.byref(params.c), int(nfields), int(field0),
                                    _ptr(mask), _ptr(load)))
    return mask, load


def setup_initial_state(mesh: Mesh, params: Params, phi_pb):
    phi = np.ascontiguousarray(phi_pb, dtype=np.float64)
    x0 = np.zeros(3 * mesh.nv)
    m = mesh.c()
    _check(lib().pnp_setup_initial_state(C.byref(m), C.byref(params.c), _ptr(phi), _ptr(x0)))
    return x0


class Layout:
    """The partition/local layout pnp_create builds (host-only, for inspection/tests)."""

    def __init__(self, mesh: Mesh, rank=0, nranks=1):
        buf = C.c_void_p()
        m = mesh.c()
        _check(lib().pnp_layout_build(C.byref(m), int(rank), int(nranks), C.byref(buf)))
        v = _Layout()
        _check(lib().pnp_layout_view(buf, C.byref(v)))

        def arr(p, n, dt=np.int32):
            return np.ctypeslib.as_array(p, (n,)).astype(dt).copy() if n else np.zeros(0, dt)
        self.n_owned, self.n_ghost = v.n_owned, v.n_ghost
        self.ncolors, self.nchunks, self.max_slots = v.ncolors, v.nchunks, v.max_slots
        self.nslots, self.nblocks = v.nslots, v.nblocks
        self.l2g = arr(v.l2g, v.n_owned + v.n_ghost)
        self.color_ptr = arr(v.color_ptr, v.ncolors + 1)
        self.color_idx = arr(v.color_idx, v.n_owned)
        self.rowcolor = arr(v.rowcolor, v.n_owned + v.n_ghost, np.uint8)
        self.chunk_len = arr(v.chunk_len, v.nchunks)
        self.chunk_off = arr(v.chunk_off, v.nchunks + 1)
        self.colidx = arr(v.colidx, v.nslots)
        self.rowmeta = arr(v.rowmeta, v.n_owned, np.uint64)
        self.nbr_ranks = arr(v.nbr_ranks, v.nnbr)
        self.recv_ptr = arr(v.recv_ptr, v.nnbr + 1)
        self.send_ptr = arr(v.send_ptr, v.nnbr + 1)
        self.send_idx = arr(v.send_idx, int(self.send_ptr[-1]) if v.nnbr else 0)
        self.color_conflicts = int(v.color_conflicts)
        lib().pnp_layout_free(buf)

    def row_len(self, i):
        return int(self.rowmeta[i] & np.uint64(63))

    def row_cols(self, i):
        c, lane = divmod(i, 64)
        L = self.row_len(i)
        return [int(self.colidx[self.chunk_off[c] + s * 64 + lane]) for s in range(L)]


# ------------------------------------------------------------------------------------------------
# GPU context
# ------------------------------------------------------------------------------------------------
def set_create_option(option, value):
    """Process-wide option read by every later Context / Layout creation (pnp_set_create_option)."""
    _check(lib().pnp_set_create_option(option, C.c_int64(value)))


def get_create_option(option):
    v = C.c_int64(0)
    _check(lib().pnp_get_create_option(option, C.byref(v)))
    return v.value


def rccl_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    _check(lib().pnp_rccl_unique_id(buf))
    return buf.raw


class Context:
    """One GPU (one rank): mesh + parameters resident in HBM, one operator at a time."""

    def __init__(self, mesh: Mesh, params: Params, device=0, rank=0, size=1, unique_id=None,
                 local_group=None, degree=1, host_transport=None):
        """degree 2 / 3: the Lagrange P_k space (pnp_create_pk, the reference's PDEGREE); its
        vectors have nfields x nn entries over the nodes of space().  host_transport: an object
        with exchange / allreduce_sum (see _host_transport) -- the host-staged transport
        (pnp_comm.host) for ranks in separate processes without RCCL."""
        self.mesh, self.params = mesh, params
        self._uid = C.create_string_buffer(unique_id, 128) if unique_id else None
        self._grp = local_group.encode() if local_group else None
        self._ht = None
        if host_transport is not None:
            ht, keep = _host_transport(host_transport)
            self._ht = (ht, keep)  # callbacks must outlive the context
        comm = _Comm(rank, size, C.cast(self._uid, C.c_void_p).value if self._uid else None,
                     self._grp, C.pointer(self._ht[0]) if self._ht else None)
        h = C.c_void_p()
        m = mesh.c()
        _check(lib().pnp_create_pk(C.byref(m), C.byref(params.c), int(degree), int(device),
                                   C.byref(comm), C.byref(h)))
        self.h = h
        self.degree = int(degree)
        self.nn = self.info()["nv_global"]  # DOF nodes (= mesh.nv for degree 1)
        self.nf = 0
        self.rank, self.size = rank, size

    def close(self):
        if getattr(self, "h", None):
            lib().pnp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ck(self, rc):
        _check(rc, self.h)

    def info(self):
        i = _Info()
        self._ck(lib().pnp_get_info(self.h, C.byref(i)))
        return {k: getattr(i, k) for k, _ in _Info._fields_}

    def space(self):
        """(xy [nn, 2], enode [nt, nlocal]) of the context's Lagrange space (pnp_space)."""
        si = _SpaceInfo()
        self._ck(lib().pnp_space(self.h, C.byref(si), None, None))
        xy = np.zeros((si.nnodes, 2))
        en = np.zeros((si.nt, si.nlocal), dtype=np.int32)
        self._ck(lib().pnp_space(self.h, C.byref(si), _ptr(xy), _ptr(en)))
        return xy, en

    def set_operator(self, kind, dt=0.0, z=0.0, field=0, phi=None, cp=None, cm=None, x_old=None,
                     c_extra=None):
        keep = [np.ascontiguousarray(a, dtype=np.float64) if a is not None else None
                for a in (phi, cp, cm, x_old, c_extra)]
        a = _OpArgs(kind, dt, z, field, *[None if k is None else k.ctypes.data for k in keep])
        self._ck(lib().pnp_set_operator(self.h, C.byref(a)))
        self.nf = 3 if kind in (OP_PNP, OP_PNP_IMPLICIT_EULER) else 1
        self._op_keep = keep

    def _vec(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        if x.size != self.nf * self.nn:
            raise PnpError(E_ARG, f"vector of size {x.size}, expected {self.nf * self.nn}")
        return x

    def residual(self, x):
        x = self._vec(x)
        r = np.zeros_like(x)
        self._ck(lib().pnp_residual(self.h, _ptr(x), _ptr(r)))
        return r

    def jacobian(self, x, export=True, fd=False):
        """Assemble J(x) (fd: the reference's forward-difference Jacobian, PNP_JAC_FD)."""
        x = self._vec(x)
        self._ck(lib().pnp_jacobian_ex(self.h, _ptr(x), JAC_FD if fd else 0))
        if not export:
            return None
        return self.jacobian_export()

    def jacobian_export(self):
        import scipy.sparse as sp
        nnz = C.c_int64()
        self._ck(lib().pnp_jacobian_export(self.h, C.byref(nnz), None, None, None))
        n = self.nf * self.nn
        rp = np.zeros(n + 1, dtype=np.int32)
        col = np.zeros(nnz.value, dtype=np.int32)
        val = np.zeros(nnz.value, dtype=np.float64)
        self._ck(lib().pnp_jacobian_export(self.h, C.byref(nnz), _ptr(rp), _ptr(col), _ptr(val)))
        return sp.csr_matrix((val, col, rp), shape=(n, n))

    def jacobian_apply(self, z, x=None, fd=False):
        """GridOperator::jacobian_apply: J(x) z (x None: the last assembled Jacobian)."""
        z = self._vec(z)
        xv = None if x is None else self._vec(x)
        y = np.zeros_like(z)
        self._ck(lib().pnp_jacobian_apply(self.h, _ptr(xv), _ptr(z), _ptr(y), JAC_FD if fd else 0))
        return y

    # raw device-pointer calls (PNP_DEVICE_PTRS): integer addresses of device buffers, e.g. a
    # torch tensor's data_ptr()
    def residual_dev(self, x_ptr, r_ptr):
        self._ck(lib().pnp_residual_ex(self.h, C.c_void_p(x_ptr), C.c_void_p(r_ptr), DEVICE_PTRS))

    def jacobian_dev(self, x_ptr, fd=False):
        self._ck(lib().pnp_jacobian_ex(self.h, C.c_void_p(x_ptr),
                                       DEVICE_PTRS | (JAC_FD if fd else 0)))

    def jacobian_apply_dev(self, x_ptr, z_ptr, y_ptr, fd=False):
        self._ck(lib().pnp_jacobian_apply(self.h, C.c_void_p(x_ptr) if x_ptr else None,
                                          C.c_void_p(z_ptr), C.c_void_p(y_ptr),
                                          DEVICE_PTRS | (JAC_FD if fd else 0)))

    def linear_solve_dev(self, rhs_ptr, z_ptr, prec=PREC_NONE, reduction=1e-8, maxit=20000,
                         check_every=8, method=0):
        o = _SolveOpts(prec, reduction, maxit, check_every, method)
        r = _SolveResult()
        rc = lib().pnp_linear_solve_ex(self.h, C.c_void_p(rhs_ptr), C.c_void_p(z_ptr), C.byref(o),
                                       C.byref(r), DEVICE_PTRS)
        if rc not in (OK, E_BREAKDOWN):
            self._ck(rc)
        return {k: getattr(r, k) for k, _ in _SolveResult._fields_}

    def jacobian_csr_device(self):
        """Device CSR view of the last assembled Jacobian: dict of n, nnz and device addresses."""
        v = _CsrView()
        self._ck(lib().pnp_jacobian_csr_device(self.h, C.byref(v)))
        return {"n": v.n, "nnz": v.nnz, "rowptr": v.rowptr, "col": v.col, "val": v.val}

    def linear_solve(self, rhs, prec=PREC_NONE, reduction=1e-8, maxit=20000, check_every=8,
                     method=0):
        """method 0: ISTL BiCGSTABSolver, 1: ISTL CGSolver (METHOD_CG)."""
        rhs = self._vec(rhs)
        z = np.zeros_like(rhs)
        o = _SolveOpts(prec, reduction, maxit, check_every, method)
        r = _SolveResult()
        rc = lib().pnp_linear_solve(self.h, _ptr(rhs), _ptr(z), C.byref(o), C.byref(r))
        if rc not in (OK, E_BREAKDOWN):
            self._ck(rc)
        return z, {k: getattr(r, k) for k, _ in _SolveResult._fields_}

    def prec_apply(self, d, prec):
        """v = M^{-1} d for one preconditioner application on the last assembled Jacobian."""
        d = self._vec(d)
        v = np.zeros_like(d)
        self._ck(lib().pnp_prec_apply(self.h, int(prec), _ptr(d), _ptr(v)))
        return v

    def amg_configure(self, smoother=PREC_SSOR, coarse_target=1024, max_levels=12, omega=0.8,
                      coarse_sweeps=2, level0_presmooth=-1):
        """Options of PREC_AMG (the reference's CG_AMG_SSOR preconditioner); see pnp_capi.h."""
        o = _AmgOpts(int(smoother), int(coarse_target), int(max_levels), float(omega),
                     int(coarse_sweeps), int(level0_presmooth))
        self._ck(lib().pnp_amg_configure(self.h, C.byref(o)))

    def amg_info(self):
        st = _AmgStats()
        self._ck(lib().pnp_amg_info(self.h, C.byref(st)))
        n = st.levels
        return {"levels": n, "rows": list(st.rows[:n]), "blocks": list(st.blocks[:n]),
                "smoother": st.smoother, "omega": st.omega}

    def amg_aggregates(self, level):
        """level 0: aggregate per global vertex (-1: not owned); level l: per level-l row."""
        info = self.amg_info()
        n = self.nn if level == 0 else info["rows"][level]
        agg = np.zeros(n, dtype=np.int32)
        self._ck(lib().pnp_amg_aggregates(self.h, int(level), _ptr(agg)))
        return agg

    def ion_flux(self, x=None, nsurf=None):
        """calcIonFlux (src/ionFlux.hh:8-96): per-surface (ip, im) of x = [phi|c+|c-] (or of
        the context's state when x is None)."""
        n = int(nsurf if nsurf is not None else len(self.params.surfaces))
        ip = np.zeros(n)
        im = np.zeros(n)
        xv = None if x is None else np.ascontiguousarray(x, dtype=np.float64)
        if xv is not None and xv.size != 3 * self.nn:
            raise PnpError(E_ARG, "ion_flux needs a 3-field state")
        self._ck(lib().pnp_ion_flux(self.h, _ptr(xv), n, _ptr(ip), _ptr(im)))
        return ip, im

    def newton(self, u, reduction=1e-9, abs_limit=1e-12, min_linear_reduction=1e-8, maxit=50,
               line_search_maxit=500, prec=PREC_NONE, linear_maxit=20000, check_every=8,
               method=0):
        u = self._vec(u).copy()
        o = _NewtonOpts(reduction, abs_limit, min_linear_reduction, maxit, line_search_maxit,
                        _SolveOpts(prec, 0.0, linear_maxit, check_every, method))
        r = _NewtonResult()
        self._ck(lib().pnp_newton(self.h, _ptr(u), C.byref(o), C.byref(r)))
        return u, {k: getattr(r, k) for k, _ in _NewtonResult._fields_}

    def dot(self, a, b, nfields=None):
        """Collective: owner-masked global scalar product of two external-layout vectors."""
        a = np.ascontiguousarray(a, dtype=np.float64)
        b = np.ascontiguousarray(b, dtype=np.float64)
        out = C.c_double(0)
        self._ck(lib().pnp_dot(self.h, _ptr(a), _ptr(b), nfields or (a.size // self.nn), 0,
                               C.byref(out)))
        return out.value

    def norm(self, a, nfields=None):
        a = np.ascontiguousarray(a, dtype=np.float64)
        out = C.c_double(0)
        self._ck(lib().pnp_norm(self.h, _ptr(a), nfields or (a.size // self.nn), 0, C.byref(out)))
        return out.value

    def newton_history(self):
        """Per-step record of the last newton(): (linear iterations, defect after the step)."""
        n = C.c_int32(0)
        self._ck(lib().pnp_newton_history(self.h, None, None, 0, C.byref(n)))
        its = np.zeros(n.value, dtype=np.int32)
        dfs = np.zeros(n.value)
        self._ck(lib().pnp_newton_history(self.h, _ptr(its), _ptr(dfs), n.value, C.byref(n)))
        return its, dfs

    def sync_vector(self, v, nfields=None):
        """Collective: global vector from every rank's owned entries (no-op on one GPU)."""
        nf = nfields or (v.size // self.nn)
        v = np.ascontiguousarray(v, dtype=np.float64).copy()
        self._ck(lib().pnp_sync_vector(self.h, _ptr(v), int(nf)))
        return v

    def initial_state(self, phi_pb):
        phi = np.ascontiguousarray(phi_pb, dtype=np.float64)
        x0 = np.zeros(3 * self.nn)
        self._ck(lib().pnp_initial_state(self.h, _ptr(phi), _ptr(x0)))
        return x0

    # device-resident hot path ------------------------------------------------------------------
    def state_set(self, x):
        x = self._vec(x)
        self._ck(lib().pnp_state_set(self.h, _ptr(x)))

    def state_get(self):
        x = np.zeros(self.nf * self.nn)
        self._ck(lib().pnp_state_get(self.h, _ptr(x)))
        return x

    def assemble_state(self, n=1):
        self._ck(lib().pnp_assemble_state(self.h, int(n)))

    def assemble_state_timed(self, n=1):
        """n assemblies of the state; returns their device time (s) from one event pair."""
        ms = C.c_double()
        self._ck(lib().pnp_assemble_state_timed(self.h, int(n), C.byref(ms)))
        return ms.value / 1e3

    def bicgstab_iterations(self, n, prec=PREC_NONE):
        r = _SolveResult()
        self._ck(lib().pnp_bicgstab_iterations(self.h, int(n), int(prec), C.byref(r)))
        return {k: getattr(r, k) for k, _ in _SolveResult._fields_}

    def set_option(self, option, value):
        self._ck(lib().pnp_set_option(self.h, int(option), C.c_int64(int(value))))

    def get_option(self, option):
        v = C.c_int64()
        self._ck(lib().pnp_get_option(self.h, int(option), C.byref(v)))
        return v.value

    def probe_slot_stores(self, tile_elems=256, reps=20):
        """pnp_probe_slot_stores (P_k contexts): the SELL slot stores of one Jacobian in SELL,
        spatial-tile and random row order; dict of the pnp_store_probe fields."""
        o = _StoreProbe()
        self._ck(lib().pnp_probe_slot_stores(self.h, int(tile_elems), int(reps), C.byref(o)))
        return {k: getattr(o, k) for k, _ in _StoreProbe._fields_}

    def cache_scrub(self, nbytes=1 << 30):
        """Evict the caches (read nbytes of scratch on the context's stream) before a cold timing."""
        self._ck(lib().pnp_cache_scrub(self.h, C.c_int64(int(nbytes))))

    def timers(self, enable=None, reset=False):
        if enable is not None:
            self._ck(lib().pnp_timers_enable(self.h, int(bool(enable))))
        if reset:
            self._ck(lib().pnp_timers_reset(self.h))
        t = _Timers()
        self._ck(lib().pnp_timers_get(self.h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in _Timers._fields_}


def header_symbols():
    """Function names declared in include/pnp_capi.h."""
    import re
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char \*)\s*(pnp_\w+)\s*\(", txt, re.M)))
