"""Summarise a rocprofv3 --kernel-trace CSV over the LAST n training steps.

Steps are delimited by the voxelisation key kernel (rpc::vox::k_keys, launched once at the
start of every step), so warm-up / MIOpen find-mode kernels are excluded.

    python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv --steps 8 [--top 40]
"""
import argparse
import collections
import csv
import re


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = n.replace("void ", "")
    return n[:100]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--marker", default="k_keys")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(starts) < a.steps + 1:
        raise SystemExit(f"only {len(starts)} step markers")
    lo, hi = starts[-a.steps - 1], starts[-1]
    sel = rows[lo:hi]
    t0, t1 = int(sel[0]["Start_Timestamp"]), int(rows[hi]["Start_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0.0])
    busy = 0.0
    for r in sel:
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += d
        busy += d
    wall = (t1 - t0) / a.steps
    print(f"steps {a.steps}: wall/step {wall / 1e6:.3f} ms, kernel busy/step {busy / a.steps / 1e6:.3f} ms, "
          f"kernels/step {len(sel) / a.steps:.0f}")
    print(f"{'ms/step':>9} {'%busy':>6} {'calls/st':>8} {'avg us':>9}  kernel")
    for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{d / a.steps / 1e6:9.3f} {100 * d / busy:6.2f} {c / a.steps:8.1f} {d / c / 1e3:9.1f}  {k}")


if __name__ == "__main__":
    main()
