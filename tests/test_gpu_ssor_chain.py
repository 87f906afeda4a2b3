"""Natural-order SSOR tails as chains (PNP_NAT_CHAIN, ssor_natural.hip k_ssor_nat_chain), -m gpu:
the chain kernel runs the level kernel's arithmetic per row, so applications, BiCGSTAB solves and
PB / PNP Newton must be BITWISE the dataflow-units-only schedule's (PNP_NAT_CHAIN=0) -- with the
default threshold (the resident-group capacity), with one that makes every level a tail level (the
whole sweep as chains, groups shared past the capacity), with a small one (head as dataflow units,
tail as chains), and on the config-3 system.  The knob is read once per process: each setting runs
in a child process."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CHILD = r"""
import hashlib, json, os, sys
import numpy as np
sys.path.insert(0, HERE)
import conftest  # noqa: F401
from conftest import DATA
from test_gpu import golden
import pnp_amd as P
out = {}
def h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()
for name in ("pore_small_k0", "cylinder_k0", "pore_pnp_k0"):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    for kind in ("pnp", "pb"):
        if kind == "pnp":
            x = z["newton_pnp_x0"] if "newton_pnp_x0" in z else z["pnp_x"]
            ctx.set_operator(P.OP_PNP)
        else:
            x = z["pb_x"]
            ctx.set_operator(P.OP_PB)
        ctx.jacobian(x, export=False)
        rhs = ctx.residual(x)
        out[f"{name}{kind}apply"] = h(ctx.prec_apply(rhs, P.PREC_SSOR_NATURAL))
        sol, res = ctx.linear_solve(rhs, prec=P.PREC_SSOR_NATURAL, reduction=1e-10, maxit=5000)
        out[f"{name}{kind}solve"] = [h(sol), res["it_half"]]
    ctx.set_operator(P.OP_PB)
    u, r = ctx.newton(np.zeros(mesh.nv), prec=P.PREC_SSOR_NATURAL)
    out[f"{name}pbnewton"] = [h(u), r["linear_iterations"]]
    ctx.close()
if os.environ.get("FULL") == "1":
    cfg = P.read_config(os.path.join(DATA, "pore_pnp/pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    rng = np.random.default_rng(20261015)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    for kind, op in (("pnp", P.OP_PNP), ("pb", P.OP_PB)):
        ctx.set_operator(op)
        xx = x if kind == "pnp" else x[:nv]
        ctx.jacobian(xx, export=False)
        rhs = ctx.residual(xx)
        out[f"full{kind}apply"] = h(ctx.prec_apply(rhs, P.PREC_SSOR_NATURAL))
        sol, res = ctx.linear_solve(rhs, prec=P.PREC_SSOR_NATURAL, reduction=1e-12, maxit=12)
        out[f"full{kind}solve"] = [h(sol), res["it_half"]]
    ctx.close()
print("RESULT " + json.dumps(out))
"""


def run(**knobs):
    env = dict(os.environ, **{k: str(v) for k, v in knobs.items()})
    code = CHILD.replace("HERE", repr(HERE))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=400, cwd=HERE)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_chain_tails_are_bitwise_the_dataflow_schedule():
    ref = run(FULL=1, PNP_NAT_CHAIN=0)
    assert run(FULL=1) == ref  # the default threshold
    assert run(FULL=1, PNP_NAT_CHAIN=1 << 30) == ref  # every level a tail level: all chains
    assert run(FULL=1, PNP_NAT_CHAIN=2048) == ref
