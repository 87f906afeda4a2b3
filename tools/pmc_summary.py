"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_run.sh steps pmcf, pmcw)
into per-kernel per-launch HBM-side bytes, with the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts 64 B per 128-B request,
so it is doubled; WRITE_SIZE is taken as is.  FETCH_SIZE is in KB (rocprofv3 derived metric).
usage: python tools/pmc_summary.py <fetch run_counter_collection.csv> <write csv> <out.json>
       [bicgstab iterations of the profiled run (bench.py's per-iteration BLAS bytes)]"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


f, nf = per_kernel(sys.argv[1], "FETCH_SIZE")
w, nw = per_kernel(sys.argv[2], "WRITE_SIZE")
out = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes with "
                 "--kernel-trace (tools/gpu_run.sh pmcf/pmcw on tools/prof_target.py, config 3, "
                 "ILU0); FETCH_SIZE x2 (gfx950 correction), both KB -> bytes x1024",
       "kernels": {},
       "bicgstab_iterations": int(sys.argv[4]) if len(sys.argv) > 4 else None}
for k in sorted(set(f) | set(w)):
    fb = 2 * 1024 * f.get(k, 0.0)
    wb = 1024 * w.get(k, 0.0)
    out["kernels"][k] = {"fetch_bytes_x2": fb, "write_bytes": wb, "traffic_bytes": fb + wb,
                         "launches_fetch": nf.get(k, 0), "launches_write": nw.get(k, 0)}
json.dump(out, open(sys.argv[3], "w"), indent=1)
for k, v in out["kernels"].items():
    if v["traffic_bytes"] > 1e7:
        print(f"{k[:70]:70s} fetch*2 {v['fetch_bytes_x2'] / 1e6:8.1f} MB  write {v['write_bytes'] / 1e6:8.1f} MB")
