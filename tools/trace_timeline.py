"""Print one training step of a rocprofv3 kernel trace as a timeline (start offset, duration, stream,
kernel), from the Nth occurrence of a marker kernel to the next one.

    python tools/trace_timeline.py kernel_trace.csv[.gz] [--marker k_hard_voxelize_or_first] [--step 5]
"""
import argparse
import csv
import gzip


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_adamw")
    ap.add_argument("--step", type=int, default=5)
    ap.add_argument("--grep", default=None)
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    rows = list(csv.DictReader(op(a.trace, "rt")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    i0, i1 = idx[a.step], idx[a.step + 1]
    t0 = int(rows[i0]["End_Timestamp"])
    busy_end = t0
    for r in rows[i0 + 1:i1 + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0][:70]
        if a.grep and a.grep not in name:
            continue
        gap = (s - busy_end) / 1e3
        busy_end = max(busy_end, e)
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {gap:7.1f} q{r['Queue_Id']:>2} g{r['Grid_Size_X']:>8} {name}")


if __name__ == "__main__":
    main()
