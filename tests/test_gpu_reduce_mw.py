"""The multi-workgroup reduction (linalg.hip k_reduce_mw, round 6; -m gpu): long partial arrays --
the SpMV's two partials per 256-row block, ~23,000 at config 5 -- are summed by G workgroups over
contiguous slices whose sums the last-ticket workgroup adds in slice order.  Config 5 is the only
system that reaches the default threshold (8,192 partials), so here PNP_RED_MW_MIN=1 (a test hook,
read once per process) routes every reduction with at least two slices through it on the config-3
system (2.2 M DOF, ~5,800 SpMV partials, 4 slices), in a child process.  Asserted against the
one-workgroup reduction in this process: BiCGSTAB + ILU(0) on the same system converges to the
same tolerance, with half-step counts within the chaotic spread of the iteration (10 %), solutions
that differ by at most the two solves' residual tolerances, and the initial defect (one reduction
of the same partials in another order) equal to 1e-14 relative."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import pnp_amd as P
from conftest import DATA

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _solve(out_path=None):
    cfg = P.read_config(os.path.join(DATA, "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PNP)
    rng = np.random.default_rng(20261018)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    J = ctx.jacobian(x)
    b = ctx.residual(x)
    z, res = ctx.linear_solve(b, prec=P.PREC_ILU0, reduction=1e-8, maxit=5000)
    ctx.close()
    rel = float(np.linalg.norm(J @ z - b) / np.linalg.norm(b))
    out = {"it_half": res["it_half"], "defect0": res["defect0"], "converged": res["converged"],
           "rel": rel}
    if out_path:
        np.save(out_path, z)
        print("RESULT " + json.dumps(out), flush=True)
    return out, z, J, b


def test_multi_workgroup_reduction_matches_the_one_workgroup_sum(tmp_path):
    ref, zref, J, b = _solve()
    env = dict(os.environ, PNP_RED_MW_MIN="1")
    pkg = os.path.join(os.path.dirname(HERE), "dune-pnp_amd", "python")
    code = (f"import sys; sys.path[:0] = [{HERE!r}, {pkg!r}]; import test_gpu_reduce_mw as T; "
            f"T._solve({str(tmp_path / 'z.npy')!r})")
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300, cwd=HERE)
    assert p.returncode == 0, p.stderr[-2000:]
    mw = json.loads(next(ln for ln in p.stdout.splitlines() if ln.startswith("RESULT "))[7:])
    z = np.load(tmp_path / "z.npy")
    assert ref["converged"] == 1 and mw["converged"] == 1
    assert ref["rel"] <= 1.001e-8 and mw["rel"] <= 1.001e-8
    assert abs(mw["defect0"] - ref["defect0"]) <= 1e-14 * ref["defect0"]
    assert abs(mw["it_half"] - ref["it_half"]) <= 0.1 * ref["it_half"] + 0.5
    # both solutions meet the 1e-8 residual reduction, so they differ by at most twice that in
    # the residual norm (the solution error itself is scaled by the condition number: 2.6e-4
    # relative in the max norm on this system)
    assert np.linalg.norm(J @ (z - zref)) <= 2.01e-8 * np.linalg.norm(b)
