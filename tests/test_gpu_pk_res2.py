"""The two-pass P_k assembly (element pass + ordered per-row gather: k_pk_elem_res /
k_pk_res_gather for residual-only launches, k_pk_elem_jac / k_pk_jac_gather for the analytic
Jacobian, the defaults) against the row walk (k_pk_row, PNP_PK_RES2=0 PNP_PK_JAC2=0), -m gpu.  The
knobs are read once per process, so each variant runs in a child process.  Both evaluate the row
walk's statements per element row and sum a row's elements in the same ascending order, so every
residual and Jacobian -- the four scalar operators at k = 2 and 3, including the implicit-Euler
operator's old-time mass term -- and a P2 PB Newton solve must be bitwise the same."""
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
import pnp_amd as P
from test_gpu_pk import setup, KINDS
def h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()
out = {}
for name in ("pore_small", "cylinder"):
    for k in (2, 3):
        mesh, ctx, orc = setup(name, k)
        nn = ctx.nn
        rng = np.random.default_rng(7 + k)
        for kind in ("pb", "poisson", "diff", "diff_ie"):
            kw = {}
            if kind.startswith("diff"):
                kw = dict(z=-1.0, phi=rng.uniform(-1, 1, nn), field=2)
                if kind == "diff_ie":
                    kw.update(dt=0.37, x_old=rng.uniform(0.0, 0.1, nn))
            if kind == "poisson":
                kw = dict(cp=rng.uniform(0.0, 0.1, nn), cm=rng.uniform(0.0, 0.1, nn))
            ctx.set_operator(KINDS[kind][0], **kw)
            x = rng.uniform(-1, 1, nn) if kind in ("pb", "poisson") else rng.uniform(0, 0.1, nn)
            J = ctx.jacobian(x).tocsr()
            out[f"{name}/{k}/{kind}"] = [h(ctx.residual(x)), h(J.data), h(J.indices)]
        if k == 2:  # P3 matrices are indefinite (quirk Q10): no preconditioned Newton there
            ctx.set_operator(P.OP_PB)
            u, res = ctx.newton(np.zeros(nn), prec=P.PREC_SSOR)
            out[f"{name}/{k}/newton"] = [h(u), res["linear_iterations"], res["converged"]]
        ctx.close()
print("RESULT " + json.dumps(out))
"""


def run(two_pass):
    env = dict(os.environ, PNP_PK_RES2=str(two_pass), PNP_PK_JAC2=str(two_pass))
    code = CHILD.replace("HERE", repr(HERE))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300, cwd=HERE)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_two_pass_residual_bitwise_equals_row_walk():
    a, b = run(1), run(0)
    assert a == b
