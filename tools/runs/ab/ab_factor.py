"""A/B of the ILU(0) factorisation: fused (one launch per colour, expand + split folded in) vs the
three-pass path, config 3, device time from the context's HIP events (T_FACT covers the
factorisation and the split).  usage: python tools/ab_factor.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(int(sys.argv[1]) if len(sys.argv) > 1 else 4)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PB)
phi, _ = ctx.newton(np.zeros(mesh.nv), reduction=1e-9, prec=P.PREC_SSOR)
x0 = ctx.initial_state(phi)
ctx.set_operator(P.OP_PNP)
ctx.state_set(x0)
for rnd in range(2):
    for fused in (0, 1):
        for f32 in (0, 1):
            ctx.set_option(P.OPT_ILU_FUSED_FACTOR, fused)
            ctx.set_option(P.OPT_ILU_F32, f32)
            ctx.assemble_state(1)
            ctx.bicgstab_iterations(1, P.PREC_ILU0)  # warm
            ctx.timers(enable=True, reset=True)
            for _ in range(5):
                ctx.assemble_state(1)
                ctx.bicgstab_iterations(1, P.PREC_ILU0)
            t = ctx.timers(enable=False)
            print(f"round {rnd} fused {fused} f32 {f32}: factorisation {t['factor_ms'] / 5:.3f} ms "
                  f"({t['factor_launches'] // 5} timed sections)", flush=True)
