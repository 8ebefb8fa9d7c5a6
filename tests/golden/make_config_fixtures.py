"""Extract the reference configs' top-level settings as DATA (JSON fixtures) for the plugin-surface
tests (tests/test_plugin_surface.py). Run in the container that holds the reference:

    python tests/golden/make_config_fixtures.py /root/reference

The config files are parsed with `ast` and only literal expressions are evaluated (dict(...) calls,
lists, tuples, numbers, strings and constant arithmetic such as 1.0 / 9.0) — nothing in them is
executed. `_base_` inheritance is not resolved: the bases live in the un-vendored mmdetection3d
checkout, so a fixture holds exactly what the reference file itself writes.
"""
from __future__ import annotations

import ast
import json
import operator
import os
import sys

CONFIGS = {
    "kitti3class": "configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py",
    "kitti_car": "configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-car.py",
    "nuscenes": "configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py",
}
KEYS = ("custom_imports", "model", "custom_hooks", "optim_wrapper", "param_scheduler", "train_cfg",
        "point_cloud_range")
_BIN = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul, ast.Div: operator.truediv}


def _eval(node):
    if isinstance(node, ast.Constant):
        return node.value
    if isinstance(node, (ast.List, ast.Tuple)):
        return [_eval(e) for e in node.elts]
    if isinstance(node, ast.Dict):
        return {_eval(k): _eval(v) for k, v in zip(node.keys, node.values)}
    if isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and node.func.id == "dict" and not node.args:
        return {kw.arg: _eval(kw.value) for kw in node.keywords}
    if isinstance(node, ast.BinOp) and type(node.op) in _BIN:
        return _BIN[type(node.op)](_eval(node.left), _eval(node.right))
    if isinstance(node, ast.UnaryOp) and isinstance(node.op, ast.USub):
        return -_eval(node.operand)
    raise ValueError(f"non-literal config expression at line {node.lineno}")


def extract(path):
    tree = ast.parse(open(path).read(), filename=path)
    out = {}
    for st in tree.body:
        if isinstance(st, ast.Assign) and len(st.targets) == 1 and isinstance(st.targets[0], ast.Name):
            name = st.targets[0].id
            if name in KEYS:
                out[name] = _eval(st.value)
    return out


def main(ref_root):
    here = os.path.dirname(os.path.abspath(__file__))
    for tag, rel in CONFIGS.items():
        d = extract(os.path.join(ref_root, rel))
        d["_source"] = rel
        with open(os.path.join(here, f"config_{tag}.json"), "w") as f:
            json.dump(d, f, indent=1, sort_keys=True)
        print(tag, sorted(d))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
