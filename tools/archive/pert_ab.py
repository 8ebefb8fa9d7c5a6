"""A/B numerics of the perturber kernels: run the golden perturber_* cases (train forward +
backward) and print the max |error| of every output against the float64 fixture, so two builds
of librpc_hip.so (RPC_HIP_LIB=...) can be compared line by line.

    python tools/pert_ab.py [tag ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_perturber import NAMES, _load, _params  # noqa: E402

from robustpointclouds_amd import perturb as P  # noqa: E402


def run(tag):
    d = _load(tag)
    F, hidden = int(d["F"]), [int(h) for h in d["hidden"]]
    dev = torch.device("cuda")
    ps = _params(d, F, hidden, dev)
    for k, p in enumerate(ps):
        if p is not None and NAMES[k] is not None:
            p.requires_grad_(True)
    cfg = P.make_cfg(F, hidden, True, True, 0.2)
    out, lvec, _ = P.PerturberFn.apply(torch.from_numpy(d["x"]).to(dev), cfg, *ps)
    G, c = torch.from_numpy(d["G"]).to(dev), torch.from_numpy(d["c"]).to(dev)
    ((out * G).sum() + (lvec * c).sum()).backward()
    rows = [("out", np.abs(out.detach().cpu().numpy() - d["out"]).max() / max(np.abs(d["out"]).max(), 1e-30))]
    for k, name in enumerate(NAMES):
        if name is not None and ps[k] is not None and ps[k].grad is not None:
            r = d["d" + name]
            rows.append((name, np.abs(ps[k].grad.cpu().numpy() - r).max() / max(np.abs(r).max(), 1e-30)))
    lib = os.environ.get("RPC_HIP_LIB", "in-tree")
    print(f"[{tag}] lib={lib} N={d['x'].shape[0]}")
    print("  " + " ".join(f"{n}:{e:.2e}" for n, e in rows))


if __name__ == "__main__":
    for t in sys.argv[1:] or ["3class", "car_small", "nus"]:
        run(t)
