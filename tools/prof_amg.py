"""Where a BiCGSTAB + AMG(ILU(0) smoother) iteration's time goes at config 3 (PNP, pore_pnp k=4).
Run mode (under rocprofv3 --kernel-trace): assembles the PNP Jacobian at a random admissible state,
sets up the AMG, warms up, then runs N iterations between two marker k_scrub launches and prints
the event-timed ms per iteration.  Split mode: reads the kernel trace and prints, per kernel, the
launches and device time per iteration between the markers, with each kernel's grid size (the
level it works on), and the gaps (time between launches) per iteration.
usage: python tools/prof_amg.py run [iters=40]
       python tools/prof_amg.py split <kernel_trace.csv> [iters=40]"""
import collections
import csv
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MARK = 64 << 20


def run(iters):
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
    import pnp_amd as P
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PNP)
    rng = np.random.default_rng(20261018)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ctx.state_set(x)
    ctx.assemble_state(1)
    ctx.amg_configure(smoother=P.PREC_ILU0)
    ctx.bicgstab_iterations(5, P.PREC_AMG)
    ctx.cache_scrub(MARK)
    t0 = time.perf_counter()
    ctx.bicgstab_iterations(iters, P.PREC_AMG)
    dt = time.perf_counter() - t0
    ctx.cache_scrub(MARK)
    print(json.dumps({"iters": iters, "ms_per_iter_wall": 1e3 * dt / iters,
                      "amg_rows": ctx.amg_info()["rows"]}), flush=True)


def split(path, iters):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k_scrub" in r["Kernel_Name"]]
    a, b = marks[-2], marks[-1]
    seg = rows[a + 1:b]
    acc = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in seg:
        n = r["Kernel_Name"].replace("void pnp::(anonymous namespace)::", "")
        n = n.replace("pnp::(anonymous namespace)::", "").split("(")[0][:70]
        key = f"{n} grid={r['Grid_Size_X']}"
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        acc[key][0] += 1
        acc[key][1] += d
        busy += d
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e3
    print(f"iterations {iters}: span {span / iters:.1f} us/it, busy {busy / iters:.1f} us/it, "
          f"gaps {(span - busy) / iters:.1f} us/it, launches {len(seg) / iters:.1f}/it")
    for k, (n, t) in sorted(acc.items(), key=lambda kv: -kv[1][1]):
        print(f"{t / iters:8.1f} us/it  {n / iters:5.1f} launches/it  {t / n:7.2f} us each  {k}")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 40)
    else:
        split(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
