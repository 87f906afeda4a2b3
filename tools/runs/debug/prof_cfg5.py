"""Assembly-only driver for profiling config 5 (test/pore_without_dna, the .geo meshed natively at
size scale 0.85, refined k) -- run under rocprofv3 (kernel trace / PMC passes).
usage: python tools/prof_cfg5.py [k=6] [launches=20]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
import pnp_amd as P  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = P.read_config(os.path.join(ROOT, "data", "pore_without_dna", "pore.cfg"))
mesh = P.Mesh.load(cfg.meshfile, size_scale=0.85).refine(k)
ctx = P.Context(mesh, P.Params.from_config(cfg))
ctx.set_operator(P.OP_PNP)
rng = np.random.default_rng(20261015)
nv = mesh.nv
x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                    0.06 * rng.uniform(0.5, 1.5, nv)])
ctx.state_set(x)
ctx.assemble_state(3)
ctx.timers(enable=True, reset=True)
ctx.assemble_state(n)
t = ctx.timers(enable=False)
info = ctx.info()
print(f"k={k} nv={nv} nt={mesh.nt} colors={info['ncolors']} blocks={info['nblocks']} "
      f"slots={info['nslots']} assemble_us={t['assemble_ms'] / t['assemble_launches'] * 1e3:.2f}",
      flush=True)
