"""Per-position average duration of the k_conv3x3 launches of a step (rocprof kernel trace)."""
import collections
import csv
import gzip
import sys

rows = list(csv.DictReader(gzip.open(sys.argv[1], "rt")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = sys.argv[2] if len(sys.argv) > 2 else "k_conv3x3<0>"
n = int(sys.argv[3]) if len(sys.argv) > 3 else 22
seq = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
steps = len(seq) // n
per = collections.defaultdict(list)
for s in range(steps - 8, steps):
    for i in range(n):
        per[i].append(seq[s * n + i])
print(name, [round(sum(per[i]) / len(per[i]), 1) for i in range(n)])
