"""Split a rocprofv3 kernel trace of natural-SSOR applications (PNP_NAT_CHAIN set) into its four
launches per application -- forward head (k_ssor_nat_flow or _pipe), forward chains (k_ssor_nat_chain),
backward head, backward chains -- and print the average and spread of each, per run segment
(a segment = consecutive applications with the same grid sizes).
usage: python tools/nat_split.py <kernel_trace.csv>"""
import csv
import statistics as st
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = [(r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r.get("Grid_Size_X", r.get("Grid_Size", "")))
           for r in rows if any(k in r["Kernel_Name"] for k in ("k_ssor_nat_flow", "k_ssor_nat_pipe", "k_ssor_nat_chain"))]
    apps, cur = [], []
    for name, dur, grid in seq:
        kind = "chain" if "k_ssor_nat_chain" in name else "flow"
        cur.append((kind, dur, grid))
        if len(cur) == 4:
            apps.append(cur)
            cur = []
    segs = []
    for a in apps:
        key = tuple(g for _, _, g in a)
        if not segs or segs[-1][0] != key:
            segs.append((key, []))
        segs[-1][1].append(a)
    for key, group in segs:
        parts = list(zip(*[[d / 1e3 for _, d, _ in a] for a in group]))
        tot = [sum(d for _, d, _ in a) / 1e3 for a in group]
        desc = " ".join(f"{lab} {st.mean(p):.1f} [{min(p):.1f}-{max(p):.1f}]"
                        for lab, p in zip(("fwd-head", "fwd-chain", "bwd-head", "bwd-chain"), parts))
        print(f"grids {key}: {len(group)} applications, total {st.mean(tot):.1f} us "
              f"[{min(tot):.1f}-{max(tot):.1f}]; {desc}")


if __name__ == "__main__":
    main(sys.argv[1])
