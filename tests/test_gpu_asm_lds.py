"""The LDS-staged assembly walk (k_assemble_ga<..., LDSG=1>: fan neighbours' coordinates, dofs
and frozen fields gathered once per workgroup into LDS) against the direct-gather walk, -m gpu.
The walk is chosen once per process (PNP_ASM_LDS=1 / 0; unset: the LDS walk past the Infinity
Cache, i.e. at config 5), so each variant runs in a child process.  Only where the neighbour
values come from differs, so residuals, Jacobians and the BiCGSTAB trajectory on them must be
bitwise the same, for every operator (NK = 5, 6, 1) on two meshes, residual-only and fused."""
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
from test_gpu import golden, set_ops
import pnp_amd as P
def h(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()
out = {}
for name, kinds in (("pore_small_k0", ("pnp", "pnp_ie", "pb", "diff", "poisson")),
                    ("cylinder_k0", ("pnp", "pb"))):
    z, mesh, par, orc = golden(name)
    ctx = P.Context(mesh, par)
    for kind in kinds:
        set_ops(z, ctx, orc, kind)
        x = z[kind + "_x"]
        r = ctx.residual(x)  # residual-only launch
        J = ctx.jacobian(x)  # fused residual + Jacobian launch
        entry = [h(r), h(J.data), h(J.indices)]
        if kind == "pnp":
            sol, res = ctx.linear_solve(r, prec=P.PREC_ILU0, reduction=1e-10, maxit=20000)
            entry += [h(sol), res["iterations"]]
        out[name + "/" + kind] = entry
    ctx.close()
print("RESULT " + json.dumps(out))
"""


def run(lds):
    env = dict(os.environ, PNP_ASM_LDS=str(lds))
    code = CHILD.replace("HERE", repr(HERE))
    p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=300, cwd=HERE)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_lds_assembly_bitwise_equals_direct_assembly():
    a, b = run(1), run(0)
    assert a.keys() == b.keys() and len(a) == 7
    for k in a:
        assert a[k] == b[k], k
