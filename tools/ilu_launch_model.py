"""The ILU(0) application's per-launch model: for each colour
launch of config 3, the bytes it moves (rocprofv3 --pmc FETCH_SIZE x 2 + WRITE_SIZE, KB, from
tools/pmc_kernels.py JSON, split by kernel and grid) against its trace time (the BiCGSTAB split of
tools/bicg_split.py), and the least-squares line  time = fixed + bytes / marginal bandwidth.
Beside it the measured floor of a launch of the same shape (tools/micro/launch_floor).
usage: python tools/ilu_launch_model.py <fetch.json> <write.json> <bicg_split.json>
       <launch_floor.log> [out.json]"""
import json
import sys

import numpy as np


def main():
    fetch, write, split = (json.load(open(p)) for p in sys.argv[1:4])
    floor = [json.loads(ln) for ln in open(sys.argv[4]) if ln.startswith("{")]
    floor = next(f for f in floor if f["workgroups"] == 800)
    phase = next(p for p in split["phases"] if p["config"] == 3)
    rows = []
    for k in phase["kernels"]:
        if "k_ilu0_solve_lds" not in k["kernel"]:
            continue
        g = str(k["grid"])
        name = next((n for n in fetch if n.startswith(k["kernel"])), None)
        if name is None or g not in fetch[name]:
            continue
        b = 2 * fetch[name][g]["FETCH_SIZE"] * 1024 + write[name][g]["WRITE_SIZE"] * 1024
        rows.append({"kernel": k["kernel"], "grid": k["grid"], "bytes": b, "trace_us": k["avg_us"]})
    x = np.array([r["bytes"] for r in rows]) / 1e6
    t = np.array([r["trace_us"] for r in rows])
    (a, s), *_ = np.linalg.lstsq(np.vstack([np.ones_like(x), x]).T, t, rcond=None)
    out = {"launches": rows, "fixed_us_per_launch": float(a),
           "marginal_gbs": float(1e3 / s), "max_fit_error_us": float(np.max(np.abs(a + s * x - t))),
           "launch_floor_us_800wg": {"empty": floor["empty_us"],
                                     "own_load_store": floor["own load+store_us"],
                                     "dependent_gather": floor["+ dependent gather_us"]},
           "sources": sys.argv[1:5]}
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 5:
        json.dump(out, open(sys.argv[5], "w"), indent=1)


if __name__ == "__main__":
    main()
