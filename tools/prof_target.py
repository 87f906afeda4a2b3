"""Profiling target: config-3 PNP (pore_pnp k=4), synthetic seeded state, a few fused
assemblies and BiCGSTAB(+SSOR) iterations.  Run under rocprofv3 (tools/gpu_run.sh)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

refine = int(sys.argv[1]) if len(sys.argv) > 1 else 4
nasm = int(sys.argv[2]) if len(sys.argv) > 2 else 10
nit = int(sys.argv[3]) if len(sys.argv) > 3 else 10
prec = P.PREC_BY_NAME[sys.argv[4]] if len(sys.argv) > 4 else P.PREC_SSOR
cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(refine)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PNP)
rng = np.random.default_rng(20261015)
nv = mesh.nv
x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                    0.06 * rng.uniform(0.5, 1.5, nv)])
ctx.state_set(x)
ctx.assemble_state(nasm)
res = ctx.bicgstab_iterations(nit, prec)
print("info", ctx.info())
print("bicgstab", res)
