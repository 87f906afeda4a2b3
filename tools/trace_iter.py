"""Print one Krylov iteration of a rocprofv3 kernel trace: per-launch duration and the idle
gap before it (diagnostic for launch-rate / dependency bubbles).

usage: python tools/trace_iter.py run_kernel_trace.csv [kernel-substring-of-iteration-start]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
key = sys.argv[2] if len(sys.argv) > 2 else "ilu0_solve<3"
seq = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
               r["Grid_Size_X"], r["VGPR_Count"]) for r in rows), key=lambda t: t[1])
idx = [i for i, t in enumerate(seq) if key in t[0]]
mid = idx[len(idx) // 2]
# back up to the start of the iteration (the update_p launch before it)
start = mid
while start > 0 and "update_p" not in seq[start][0]:
    start -= 1
tot_busy = tot_gap = 0.0
prev = None
for k in range(start, min(start + 40, len(seq))):
    n, s, e, g, v = seq[k]
    if k > start and "update_p" in n:
        break
    d = (e - s) / 1e3
    gap = (s - prev) / 1e3 if prev else 0.0
    tot_busy += d
    tot_gap += max(gap, 0.0)
    name = n.split("::")[-1][:48]
    print(f"{d:8.2f} us  gap {gap:6.2f}  grid {g:>8}  vgpr {v:>3}  {name}")
    prev = e
print(f"busy {tot_busy:.1f} us  gaps {tot_gap:.1f} us")
