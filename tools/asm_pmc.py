"""Counter passes on the config-3 PNP assembly, warm against in situ.

Target (`python tools/asm_pmc.py run`): the bench's config-3 system (pore_pnp k=4, 2.2 M DOF,
the Boltzmann-like random state of tools/ab_newton_asm.py), then three phases separated by marker
cache scrubs (k_scrub, 64 MiB):
  warm     10 assemblies back to back (after 2 untimed ones), bench.py's `value` regime;
  in_situ  10 x (20 BiCGSTAB + ILU(0) iterations, then one assembly), as Newton runs it;
  cold     10 x (1 GiB scrub, then one assembly).
Run it under rocprofv3 once per counter set (`--pmc <set> --kernel-trace`, the program after --).

Split (`python tools/asm_pmc.py split <out.json> <counter_collection.csv>...`): every dispatch of
k_assemble_ga<0, ...> is attributed to its phase by its position in the fixed sequence; per phase
and counter
the mean per launch, plus derived bytes (FETCH_SIZE x 2 as calibrated, WRITE_SIZE, TCC_EA0 requests
x 64 B / 128 B) and the L2 hit rate.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MARK = 64 << 20
SCRUB = 1 << 30


def run():
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "dune-pnp_amd", "python"))
    import pnp_amd as P
    cfg = P.read_config(os.path.join(ROOT, "data", "pore_pnp", "pore.cfg"))
    mesh = P.Mesh.read_gmsh(cfg.meshfile).refine(4)
    ctx = P.Context(mesh, P.Params.from_config(cfg))
    ctx.set_operator(P.OP_PNP)
    rng = np.random.default_rng(20261017)
    nv = mesh.nv
    x = np.concatenate([rng.uniform(-1, 1, nv), 0.06 * rng.uniform(0.5, 1.5, nv),
                        0.06 * rng.uniform(0.5, 1.5, nv)])
    ctx.state_set(x)
    ctx.assemble_state(2)
    ctx.bicgstab_iterations(2, P.PREC_ILU0)
    ctx.assemble_state(2)
    ctx.assemble_state(10)  # warm
    ctx.cache_scrub(MARK)
    for _ in range(10):  # in situ
        ctx.bicgstab_iterations(20, P.PREC_ILU0)
        ctx.assemble_state(1)
    ctx.cache_scrub(MARK)
    for _ in range(10):  # cold
        ctx.cache_scrub(SCRUB)
        ctx.assemble_state(1)
    ctx.cache_scrub(MARK)
    ctx.close()
    print("asm_pmc: done", flush=True)


def split(out_path, paths):
    phases = ("warm", "in_situ", "cold")
    acc = {p: collections.defaultdict(list) for p in phases}
    for path in paths:
        rows = list(csv.DictReader(open(path)))
        disp = collections.OrderedDict()
        for r in rows:
            disp.setdefault(int(r["Dispatch_Id"]), []).append(r)
        order = sorted(disp)
        # attribute by position: assembly dispatches in order; the first 2+2+10 are warm-up/warm,
        # then 10 in situ, then 10 cold (the target's fixed sequence)
        asm = [did for did in order if "k_assemble_ga<0" in disp[did][0]["Kernel_Name"]]
        if len(asm) < 34:
            raise SystemExit(f"{path}: {len(asm)} assembly dispatches, expected 34")
        seq = asm[-34:]
        groups = {"warm": seq[4:14], "in_situ": seq[14:24], "cold": seq[24:34]}
        for p, ids in groups.items():
            for did in ids:
                for r in disp[did]:
                    acc[p][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"kernel": "k_assemble_ga<0, ...> (config 3, OP_PNP)", "phases": {}}
    for p in phases:
        d = {k: sum(v) / len(v) for k, v in acc[p].items()}
        der = {}
        if "FETCH_SIZE" in d:
            der["read_bytes_fetch_x2"] = 2 * d["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in d:
            der["write_bytes"] = d["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            der["l2_hit_rate"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        out["phases"][p] = {"counters_mean_per_launch": d, "derived": der,
                            "launches": max((len(v) for v in acc[p].values()), default=0)}
        print(p, json.dumps({k: round(v, 1) for k, v in d.items()}), json.dumps(der))
    json.dump(out, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run()
    else:
        split(sys.argv[2], sys.argv[3:])
