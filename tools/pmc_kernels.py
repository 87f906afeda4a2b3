"""Per-kernel means of the counters of a rocprofv3 --pmc run (run_counter_collection.csv), split
by grid size, as JSON: {kernel: {grid: {counter: mean per dispatch, "dispatches": n}}}.
usage: python tools/pmc_kernels.py <counter_collection.csv> [name filter] [out.json]"""
import collections
import csv
import json
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"].replace("void pnp::(anonymous namespace)::", "").replace(
            "pnp::(anonymous namespace)::", "").split("(")[0]
        if filt not in n:
            continue
        acc[(n, r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = collections.defaultdict(dict)
    for (n, g), d in sorted(acc.items()):
        row = {k: sum(v) / len(v) for k, v in d.items()}
        row["dispatches"] = max(len(v) for v in d.values())
        out[n][g] = row
        print(n, g, {k: round(v) for k, v in row.items()})
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
