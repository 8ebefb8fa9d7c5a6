"""Build librpc_hip.so (the C-ABI kernel library) in-tree for gfx950.

    python -m robustpointclouds_amd._build          # incremental
    python -m robustpointclouds_amd._build --force  # rebuild everything

Each csrc/*.hip is compiled to an object with hipcc (in parallel), then linked into
robustpointclouds_amd/_lib/librpc_hip.so. The .so is git-ignored but travels to the GPU
box with the gpurun snapshot. No fast-math: voxelisation needs IEEE division.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_lib", "obj")
LIB = os.path.join(HERE, "_lib", "librpc_hip.so")
INCLUDE = os.path.join(ROOT, "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RPC_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-I", CSRC,
         "-Wno-unused-result", "-munsafe-fp-atomics"]


def _git_describe() -> str:
    try:
        return subprocess.check_output(["git", "-C", ROOT, "describe", "--always", "--dirty"],
                                       stderr=subprocess.DEVNULL, text=True).strip()
    except Exception:
        return "unknown"


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, os.path.basename(src) + ".o")
    deps = [src] + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [HIPCC, *FLAGS, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
    return obj


def build(force: bool = False, jobs: int | None = None) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    ver = os.path.join(OBJ, "version.cpp")
    with open(ver, "w") as f:
        f.write('extern "C" const char* rpc_version(void) { return "rpc_hip %s %s"; }\n'
                % (_git_describe(), ARCH))
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4) // 2), 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    # a kernel template whose host pass failed (hipcc defers device-code diagnostics in the host pass and can
    # drop the kernel silently) leaves its launch stub undefined: fail the build, not the first dlopen
    for o in objs:
        r = subprocess.run(["nm", "-C", "--undefined-only", o], capture_output=True, text=True)
        bad = [ln.strip() for ln in r.stdout.splitlines() if "__device_stub__" in ln]
        if bad:
            raise RuntimeError(f"{os.path.basename(o)}: kernels without a host launch stub:\n" + "\n".join(bad[:8]))
    vobj = os.path.join(OBJ, "version.o")
    subprocess.run(["g++", "-O2", "-fPIC", "-c", ver, "-o", vobj], check=True)
    tmp = LIB + ".tmp"
    r = subprocess.run([HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp, *objs, vobj],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
