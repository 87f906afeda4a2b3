"""The sweep variants against each other, -m gpu: the LDS-staged ILU(0) sweeps (k_ilu0_solve_lds,
the default) against the direct-gather sweeps (PNP_ILU_LDS=0), and the longest-first lane order of
the split L / U storage (the default) against the identity order (PNP_SPLIT_SORT=0).  The knobs
are read once per process, so each variant runs in a child process.  Every variant keeps each
row's slot order and arithmetic, so preconditioner applications (ILU(0) with fp32 and fp64
factors, fp32 and fp64, and bf16 factors with the single-precision intermediate, the
multicolour SSOR), BiCGSTAB iterates and counts, the AMG's ILU(0)-smoothed cycle and
a PB -> PNP Newton must be bitwise the same, on one rank and on 3 partitioned ranks."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = r"""
import hashlib, json, sys
import numpy as np
sys.path.insert(0, HERE)
import conftest  # noqa: F401  (puts the package on the path)
from test_gpu import golden
from test_gpu_multirank import run_ranks
import pnp_amd as P
out = {}
def h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()
for name in ("pore_small_k0", "cylinder_k0"):
    z, mesh, par, orc = golden(name)
    x = z["newton_pnp_x0"]
    ctx = P.Context(mesh, par)
    ctx.set_operator(P.OP_PNP)
    ctx.jacobian(x, export=False)
    rhs = ctx.residual(x)
    out[f"{name}ssor"] = h(ctx.prec_apply(rhs, P.PREC_SSOR))
    sol, res = ctx.linear_solve(rhs, prec=P.PREC_SSOR, reduction=1e-10, maxit=20000)
    out[f"{name}ssor_solve"] = [h(sol), res["iterations"]]
    for f32 in (3, 1, 0):
        ctx.set_option(P.OPT_ILU_F32, f32)
        out[f"{name}apply{f32}"] = h(ctx.prec_apply(rhs, P.PREC_ILU0))
        sol, res = ctx.linear_solve(rhs, prec=P.PREC_ILU0, reduction=1e-10, maxit=20000)
        out[f"{name}solve{f32}"] = [h(sol), res["iterations"], res["it_half"]]
    ctx.set_option(P.OPT_ILU_F32, 1)
    ctx.amg_configure(smoother=P.PREC_ILU0)
    sol, res = ctx.linear_solve(rhs, prec=P.PREC_AMG, reduction=1e-10, maxit=20000)
    out[f"{name}amg"] = [h(sol), res["iterations"]]
    ctx.set_operator(P.OP_PB)
    phi, rpb = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_ILU0)
    x0 = ctx.initial_state(phi)
    ctx.set_operator(P.OP_PNP)
    u, res = ctx.newton(x0, prec=P.PREC_ILU0)
    out[f"{name}newton"] = [h(u), res["linear_iterations"]]
z, mesh, par, orc = golden("pore_small_k0")
x = z["newton_pnp_x0"]
def fn(c, r):
    c.set_operator(P.OP_PNP)
    c.jacobian(x, export=False)
    b = c.sync_vector(c.residual(x))
    sol, res = c.linear_solve(b, prec=P.PREC_ILU0, reduction=1e-10, maxit=20000)
    return h(c.sync_vector(sol)), res["iterations"]
out["ranks3"] = run_ranks(3, mesh, par, fn)
print("RESULT " + json.dumps(out))
"""


def run(**knobs):
    env = dict(os.environ, **{k: str(v) for k, v in knobs.items()})
    code = CHILD.replace("HERE", repr(HERE))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300, cwd=HERE)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_sweep_variants_are_bitwise_equal():
    ref = run()
    assert run(PNP_ILU_LDS=0) == ref
    for b in (3, 4, 8):  # slot batches (the default is 2 on these meshes, 3 past 1.5 M rows)
        assert run(PNP_ILU_LDS_B=b) == ref, b
    assert run(PNP_SPLIT_SORT=0) == ref
    assert run(PNP_SPLIT_SORT=0, PNP_ILU_LDS=0) == ref


def test_layout_counts_in_pnp_info():
    """pnp_info's split-storage counts (tools/ilu_bytes.py reads them): every owned coupling of two
    colours is one live L or U slot, the diagonal one U slot per row, same-colour pairs none; each
    staged list entry serves at least one live off-diagonal slot"""
    import conftest  # noqa: F401
    import pnp_amd as P
    from test_gpu import golden
    for name in ("pore_small_k0", "cylinder_k0"):
        z, mesh, par, orc = golden(name)
        ctx = P.Context(mesh, par)
        ctx.set_operator(P.OP_PNP)
        info = ctx.info()
        ctx.close()
        rows = info["nv_owned"]
        assert info["lslots_live"] + info["uslots_live"] + 2 * info["color_conflicts"] == \
            info["nblocks"], info
        assert info["lslots_live"] <= info["lslots"] and info["uslots_live"] <= info["uslots"]
        assert 0 < info["lsx_entries"] <= info["lslots_live"]
        assert 0 < info["usx_entries"] <= info["uslots_live"] - rows
