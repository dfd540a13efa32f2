"""k_sq_step durations and launch gaps from a rocprofv3 kernel trace (csv)."""
import collections
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_sq_step" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
by = collections.defaultdict(list)
for r, d in zip(rows, dur):
    by[int(r["Grid_Size_X"] if "Grid_Size_X" in r else r["Grid_Size"])].append(d)
print(f"k_sq_step launches {len(dur)}  mean {statistics.mean(dur):.2f} us  min {min(dur):.2f}  max {max(dur):.2f}")
ks = sorted(by)
for k in ks[:3] + ks[-3:]:
    print(f"  grid {k}: n {len(by[k])} mean {statistics.mean(by[k]):.2f} min {min(by[k]):.2f}")
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
gaps = [g for g in gaps if g < 1000]
print(f"gap mean {statistics.mean(gaps):.2f} us  median {statistics.median(gaps):.2f}")
