"""Join tools/micro/fetch_calib's known byte counts with rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE
passes into per-access-pattern correction factors (factor = known bytes / counter bytes, the number
to multiply a counter by before comparing it with a byte count).  Test infrastructure, not product.
usage: python tools/fetch_calib_summary.py <fetch_calib stdout> <FETCH csv> <WRITE csv> <out.json>"""
import collections
import csv
import json
import sys


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[r["Kernel_Name"].split("(")[0].strip()].append(1024.0 * float(r["Counter_Value"]))
    return acc


known = {}
for line in open(sys.argv[1]):
    line = line.strip()
    if line.startswith("{"):
        d = json.loads(line)
        known[d.pop("kernel")] = d
fetch = per_kernel(sys.argv[2], "FETCH_SIZE")
write = per_kernel(sys.argv[3], "WRITE_SIZE")
out = {"method": "tools/micro/fetch_calib.hip: each kernel touches a known set of 128-B lines of a "
                 "2 GiB buffer once per launch; rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in "
                 "separate passes; factor = known bytes / counter bytes (KB x 1024), mean over launches",
       "patterns": {}}
for k, d in known.items():
    row = dict(d)
    if "known_bytes" in d and fetch.get(k):
        fb = sum(fetch[k]) / len(fetch[k])
        row["fetch_size_bytes"] = fb
        row["factor"] = d["known_bytes"] / fb if fb else None
        if "data_lines_bytes" in d:
            # index bytes stream at 4 B per lane: remove them at the s4 factor, leaving the gather's
            s4 = known.get("s4", {})
            s4f = (s4["known_bytes"] / (sum(fetch["s4"]) / len(fetch["s4"]))) if fetch.get("s4") else None
            if s4f:
                gather_counter = fb - d["index_bytes"] / s4f
                row["gather_factor"] = d["data_lines_bytes"] / gather_counter if gather_counter > 0 else None
    if "known_write_bytes" in d and write.get(k):
        wb = sum(write[k]) / len(write[k])
        row["write_size_bytes"] = wb
        row["factor"] = d["known_write_bytes"] / wb if wb else None
    out["patterns"][k] = row
json.dump(out, open(sys.argv[4], "w"), indent=1)
for k, r in out["patterns"].items():
    print(f"{k:5s} factor {r.get('factor')}  gather_factor {r.get('gather_factor')}")
