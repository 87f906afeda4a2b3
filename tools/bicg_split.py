"""Per-config, per-kernel BiCGSTAB split of a rocprofv3 --kernel-trace run of tools/prof_bicg.py
(VERDICT round 4, next #1): the trace's launches between each pair of k_scrub markers belong to
one phase (one config), in the order prof_bicg.py printed them.  Per phase and kernel class
(SpMV, ILU(0) apply, BLAS = vector updates + reductions) the trace's device time per unit (per
SpMV, per preconditioner application, per iteration) is set beside the library's event timers of
the same pass and the stored-format bytes, so each fraction the bench line reports follows from
the committed trace:
    frac = bytes per unit / (trace time per unit) / 8 TB/s
Event pairs bracket a unit's launches and the gaps between them, so event time >= trace time;
the `gap_share` column is (event - trace) / event.
usage: python tools/bicg_split.py <run_kernel_trace.csv> <prof_bicg.py stdout> [out.json]"""
import collections
import csv
import json
import sys

PEAK = 8000.0
CLASSES = (("spmv", ("k_spmv",)), ("ilu0_apply", ("k_ilu0",)),
           ("blas_per_iter", ("k_update", "k_reduce", "k_dot")))


def cls_of(name):
    for c, keys in CLASSES:
        if any(k in name for k in keys):
            return c
    return None


def short(name):
    n = name.replace("void pnp::(anonymous namespace)::", "").replace("pnp::(anonymous namespace)::", "")
    return n.split("(")[0]


def main():
    trace, log = sys.argv[1], sys.argv[2]
    out_path = sys.argv[3] if len(sys.argv) > 3 else None
    phases_meta = [json.loads(ln) for ln in open(log) if ln.startswith("{")]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "k_scrub" in r["Kernel_Name"]]
    if len(marks) < 2 * len(phases_meta):
        sys.exit(f"{len(marks)} markers for {len(phases_meta)} phases")
    res = {"source": {"trace": trace, "log": log}, "peak_gbs": PEAK, "phases": []}
    for k, meta in enumerate(phases_meta):
        a, b = marks[2 * k], marks[2 * k + 1]
        per = collections.defaultdict(list)
        tot = collections.defaultdict(float)
        for r in rows[a + 1:b]:
            name = r["Kernel_Name"]
            c = cls_of(name)
            if c is None:
                continue
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
            per[(c, short(name), r["Grid_Size_X"])].append(d)
            tot[c] += d
        nit, tm, by = meta["iterations"], meta["timers"], meta["bytes"]
        units = {"spmv": max(1, tm["spmv_launches"]), "ilu0_apply": max(1, tm["prec_launches"]),
                 "blas_per_iter": nit}
        ev_ms = {"spmv": tm["spmv_ms"], "ilu0_apply": tm["prec_ms"], "blas_per_iter": tm["blas_ms"]}
        byt = {"spmv": by["spmv_stored"], "ilu0_apply": by["ilu_stored"], "blas_per_iter": by["blas"]}
        ph = {"config": meta["config"], "dofs": meta["dofs"], "iterations": nit, "classes": {},
              "kernels": []}
        print(f"config {meta['config']} ({meta['dofs']} DOF), {nit} iterations")
        for c, _ in CLASSES:
            t_us = tot[c] / units[c]
            e_us = 1e3 * ev_ms[c] / units[c]
            f_t = byt[c] / (t_us * 1e-6) / 1e9 / PEAK if t_us > 0 else None
            f_e = byt[c] / (e_us * 1e-6) / 1e9 / PEAK if e_us > 0 else None
            ph["classes"][c] = {"units": units[c], "bytes_per_unit": byt[c],
                                "trace_us_per_unit": t_us, "event_us_per_unit": e_us,
                                "gap_share": (e_us - t_us) / e_us if e_us > 0 else None,
                                "frac_trace": f_t, "frac_event": f_e}
            print(f"  {c:14s} trace {t_us:8.2f} us  events {e_us:8.2f} us  "
                  f"frac trace {f_t or 0:.3f} events {f_e or 0:.3f}")
        for (c, n, g), v in sorted(per.items()):
            ph["kernels"].append({"class": c, "kernel": n, "grid": int(g), "launches": len(v),
                                  "avg_us": sum(v) / len(v), "min_us": min(v), "max_us": max(v)})
            print(f"    {n[:60]:60s} grid {g:>9s} n={len(v):4d} avg {sum(v) / len(v):7.2f} us")
        res["phases"].append(ph)
    if out_path:
        json.dump(res, open(out_path, "w"), indent=1)


if __name__ == "__main__":
    main()
