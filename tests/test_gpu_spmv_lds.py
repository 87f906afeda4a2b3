"""The LDS-staged SpMV (k_spmv_lds, the default) against the direct-gather k_spmv
(PNP_SPMV_LDS=0), -m gpu.  The kernel is chosen once per process, so each variant runs in a child
process; the LDS kernel keeps the direct kernel's arithmetic order (even / odd slot sums, dot
partials per 128 rows with the same trees), so the Jacobian-vector products, the BiCGSTAB
iterates and the iteration counts must be bitwise the same -- on one rank and on 3 partitioned
ranks (halo-split SpMV)."""
import hashlib
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
z, mesh, par, orc = golden("pore_small_k0")
x = z["newton_pnp_x0"]
out = {}
def h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()
ctx = P.Context(mesh, par)
ctx.set_operator(P.OP_PNP)
ctx.jacobian(x, export=False)
rhs = ctx.residual(x)
out["apply"] = h(ctx.jacobian_apply(rhs))
for prec in (P.PREC_NONE, P.PREC_ILU0, P.PREC_AMG):
    sol, res = ctx.linear_solve(rhs, prec=prec, reduction=1e-10, maxit=20000)
    out[f"solve{prec}"] = [h(sol), res["iterations"], res["it_half"]]
def fn(c, r):
    c.set_operator(P.OP_PNP)
    c.jacobian(x, export=False)
    b = c.sync_vector(c.residual(x))
    sol, res = c.linear_solve(b, prec=P.PREC_ILU0, reduction=1e-10, maxit=20000)
    return h(c.sync_vector(sol)), res["iterations"]
out["ranks3"] = run_ranks(3, mesh, par, fn)
print("RESULT " + json.dumps(out))
"""


def run(lds):
    env = dict(os.environ, PNP_SPMV_LDS=str(lds))
    code = CHILD.replace("HERE", repr(HERE))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300, cwd=HERE)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_lds_spmv_bitwise_equals_direct_spmv():
    a, b = run(1), run(0)
    assert a == b
