"""A/B of assembly variants in ONE process (cdna_hip_programming.md §5.4 rule 24): the
variant is chosen at first launch from PNP_ASM_WAVES, so run this script once per variant
inside one gpurun call, interleaved, and compare medians."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PNP)
rng = np.random.default_rng(20261015)
nv = mesh.nv
x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                    0.06 * rng.uniform(0.5, 1.5, nv)])
import hashlib  # noqa: E402
J = ctx.jacobian(x)
jh = hashlib.sha1(np.ascontiguousarray(J.data).tobytes()).hexdigest()[:12]
ctx.state_set(x)
ctx.assemble_state(5)
res = []
for rep in range(10):
    ctx.timers(enable=True, reset=True)
    ctx.assemble_state(20)
    t = ctx.timers(enable=False)
    res.append(t["assemble_ms"] / t["assemble_launches"] * 1e3)
resid = []
for rep in range(5):
    ctx.timers(enable=True, reset=True)
    ctx.assemble_state(-20)
    t = ctx.timers(enable=False)
    resid.append(t["assemble_ms"] / t["assemble_launches"] * 1e3)
ctx.assemble_state(1)
ctx.timers(enable=True, reset=True)
ctx.bicgstab_iterations(20, P.PREC_SSOR)
t = ctx.timers(enable=False)
ctx.bicgstab_iterations(2, P.PREC_ILU0)  # factorise
ilu, iltot = [], []
for rep in range(5):
    ctx.timers(enable=True, reset=True)
    ctx.bicgstab_iterations(10, P.PREC_ILU0)
    ti = ctx.timers(enable=False)
    ilu.append(ti['prec_ms'] / ti['prec_launches'] * 1e3)
    iltot.append((ti['prec_ms'] + ti['spmv_ms'] + ti['blas_ms']) / 10 * 1e3)
knobs = " ".join(f"{k[4:].lower()}={v}" for k, v in sorted(os.environ.items())
                 if k.startswith("PNP_") and k != "PNP_AMD_LIB")
print(f"{knobs or 'default'} jac={jh} assemble_us median={np.median(res):.2f} "
      f"min={np.min(res):.2f} residual_only_us={np.median(resid):.2f}  spmv_us={t['spmv_ms'] / t['spmv_launches'] * 1e3:.2f} "
      f"sgs_apply_us={t['prec_ms'] / t['prec_launches'] * 1e3:.2f} "
      f"ilu_apply_us={np.median(ilu):.2f} ilu_bicgstab_us_per_it={np.median(iltot):.1f} "
      f"blas_ms_per_it={t['blas_ms'] / 20:.4f}")
