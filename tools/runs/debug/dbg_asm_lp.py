"""A/B debug: Jacobian of the persistent LDS walk vs the direct walk on pore_small_k0 (PNP)."""
import os, subprocess, sys, json
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
code = r"""
import sys, numpy as np
sys.path.insert(0, %r); sys.path.insert(0, %r)
import conftest
from test_gpu import golden, set_ops
import pnp_amd as P
z, mesh, par, orc = golden("pore_small_k0")
ctx = P.Context(mesh, par)
set_ops(z, ctx, orc, "pnp")
J = ctx.jacobian(z["pnp_x"]).tocsr()
np.save(sys.argv[1], np.stack([J.indptr[:-1].astype(float)[:1], J.indptr[:1].astype(float)]))
np.savez(sys.argv[1], data=J.data, indices=J.indices, indptr=J.indptr)
""" % (os.path.join(ROOT, "tests"), os.path.join(ROOT, "dune-pnp_amd", "python"))
outs = []
for env in ({"PNP_ASM_LDS": "1"}, {"PNP_ASM_LDS": "0"}):
    f = "/tmp/j_%s.npz" % env["PNP_ASM_LDS"]
    subprocess.run([sys.executable, "-c", code, f], env=dict(os.environ, **env), check=True)
    outs.append(np.load(f))
a, b = outs
assert (a["indices"] == b["indices"]).all()
d = np.abs(a["data"] - b["data"])
rel = d / np.maximum(np.abs(b["data"]), 1e-300)
bad = np.nonzero(d)[0]
print("differing entries", len(bad), "of", len(d), "max abs", d.max(), "max rel", rel.max())
rows = np.searchsorted(b["indptr"], bad, side="right") - 1
print("rows", sorted(set((rows % 3048).tolist()))[:40], "fields", sorted(set((rows // 3048).tolist())))
print("cols", sorted(set(b["indices"][bad].tolist()))[:20])
