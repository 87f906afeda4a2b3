"""Split the assembly launches of a rocprofv3 --kernel-trace run of bench.py into the three regimes
the bench line reports, by the kernel dispatched right before each one on the same stream:
  warm     -- third or later of a back-to-back run of assemblies (bench.py's timed region 1 and its
              event passes run after two untimed launches: the first two after a solve bring the
              write stream back into the Infinity Cache)
  rewarm   -- second of a back-to-back run
  in_situ  -- after a BiCGSTAB kernel (as pnp_newton runs it: `roofline_in_situ`)
  cold     -- after the 1 GiB k_scrub read (`roofline_cold`)
and print per-regime launch counts and average / min / max durations, so each `frac` of the line
follows from the committed profile (bytes per launch / average duration / 8 TB/s).
usage: python tools/asm_regimes.py <run_kernel_trace.csv> <B_asm bytes> [out.json] [kernel substr]
       [grid size in threads: only launches of this grid, e.g. 738048 = config 3]"""
import collections
import csv
import json
import sys

path, b_asm = sys.argv[1], float(sys.argv[2])
out_path = sys.argv[3] if len(sys.argv) > 3 else None
key = sys.argv[4] if len(sys.argv) > 4 and sys.argv[4] else "k_assemble_ga<0, 1, 3, 9, 6"
grid = sys.argv[5] if len(sys.argv) > 5 else None
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
last = {}
run = {}
acc = collections.defaultdict(list)
for r in rows:
    q = (r["Agent_Id"], r["Queue_Id"])
    name = r["Kernel_Name"]
    if key in name and grid and r["Grid_Size_X"] != grid:
        name = "(other grid) " + name  # another system's assembly: a predecessor like any kernel
    if key in name and not name.startswith("(other grid)"):
        prev = last.get(q, "")
        if prev.startswith("(other grid)"):
            prev = "another system's assembly"
        run[q] = run.get(q, 0) + 1 if key in prev else 0
        if key in prev:
            reg = "warm" if run[q] >= 2 else "rewarm"
        elif "k_scrub" in prev:
            reg = "cold"
        elif any(k in prev for k in ("k_update", "k_reduce", "k_spmv", "k_ilu0", "k_dot")):
            reg = "in_situ"
        else:
            reg = "other"
        acc[reg].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    if "__amd_rocclr" not in name:  # runtime copies / fills (scalar read-backs) do not count
        last[q] = name
res = {"kernel": key, "grid_threads": grid, "bytes_per_launch": b_asm, "peak_gbs": 8000.0,
       "source": path, "regimes": {}}
for reg, v in acc.items():
    avg = sum(v) / len(v)
    res["regimes"][reg] = {"launches": len(v), "avg_us": avg, "min_us": min(v), "max_us": max(v),
                           "achieved_gbs": b_asm / (avg * 1e-6) / 1e9,
                           "frac": b_asm / (avg * 1e-6) / 1e9 / 8000.0}
    print(f"{reg:8s} n={len(v):3d} avg {avg:7.2f} us  min {min(v):7.2f}  max {max(v):7.2f}  "
          f"frac {res['regimes'][reg]['frac']:.3f}")
if out_path:
    json.dump(res, open(out_path, "w"), indent=1)
