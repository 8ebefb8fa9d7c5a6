"""Where one training step's wall time goes, from a rocprofv3 kernel trace: per-stream kernel busy time, the
union of all kernel intervals (GPU busy), idle gaps (no kernel running anywhere) and the largest of them with
the kernels either side, averaged over steps delimited by a marker kernel.

    python tools/step_streams.py kernel_trace.csv[.gz] [--marker k_adamw] [--steps 4] [--top 12]
"""
import argparse
import collections
import csv
import gzip


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="k_adamw")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    op = gzip.open if a.trace.endswith(".gz") else open
    rows = list(csv.DictReader(op(a.trace, "rt")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    skey = "Stream_Id" if "Stream_Id" in rows[0] else ("Queue_Id" if "Queue_Id" in rows[0] else None)
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    steps = list(zip(idx[-a.steps - 1:-1], idx[-a.steps:]))
    per_stream = collections.defaultdict(float)
    walls, unions, gaps = [], [], []
    for i0, i1 in steps:
        t0, t1 = int(rows[i0]["End_Timestamp"]), int(rows[i1]["End_Timestamp"])
        walls.append(t1 - t0)
        cur_end, busy, prev = t0, 0, rows[i0]
        for r in rows[i0 + 1:i1 + 1]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            per_stream[r[skey] if skey else "?"] += e - s
            if s > cur_end:
                gaps.append((s - cur_end, prev["Kernel_Name"].split("(")[0][:60], r["Kernel_Name"].split("(")[0][:60],
                             (s - t0) / 1e3))
            busy += max(0, e - max(s, cur_end))
            if e > cur_end:
                cur_end, prev = e, r
        unions.append(busy)
    n = len(steps)
    print(f"steps {n}: wall {sum(walls) / n / 1e6:.3f} ms/step, GPU busy (union of kernels) "
          f"{sum(unions) / n / 1e6:.3f} ms/step, idle {(sum(walls) - sum(unions)) / n / 1e6:.3f} ms/step")
    for k, v in sorted(per_stream.items(), key=lambda kv: -kv[1]):
        print(f"  stream {k}: kernel time {v / n / 1e6:.3f} ms/step")
    gaps.sort(key=lambda g: -g[0])
    print(f"largest idle gaps (us, after -> before, ms into the step), of {len(gaps) / n:.0f} per step:")
    for g, p, q, at in gaps[:a.top]:
        print(f"  {g / 1e3:8.1f}  at {at:7.3f}  {p} -> {q}")
    hist = collections.Counter()
    for g, *_ in gaps:
        hist["<5us" if g < 5e3 else "5-20us" if g < 2e4 else "20-100us" if g < 1e5 else ">100us"] += g
    print("idle by gap size (ms/step):", {k: round(v / n / 1e6, 3) for k, v in hist.items()})


if __name__ == "__main__":
    main()
