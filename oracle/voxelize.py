"""PARITY ORACLE — TEST INFRASTRUCTURE ONLY. ctypes loader for oracle/voxelize_ref.c."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "voxelize_ref.c")
LIB = os.path.join(HERE, "_build", "libvoxref.so")
_lib = None


def build(force: bool = False) -> str:
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        # no -ffast-math: IEEE float division/floor like the reference
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", LIB, SRC, "-lm"], check=True)
    return LIB


def _load():
    global _lib
    if _lib is None:
        build()
        lib = C.CDLL(LIB)
        fp = C.POINTER(C.c_float)
        ip = C.POINTER(C.c_int)
        lib.oracle_hard_voxelize.restype = C.c_int
        lib.oracle_hard_voxelize.argtypes = [fp, C.c_int, C.c_int, fp, fp, C.c_int, C.c_int, fp, ip, ip]
        _lib = lib
    return _lib


def hard_voxelize(points: np.ndarray, voxel_size, pc_range, max_points: int, max_voxels: int):
    """One frame -> (voxels [V, max_points, F], coors [V, 3] zyx, num_points [V])."""
    lib = _load()
    pts = np.ascontiguousarray(points, dtype=np.float32)
    n, F = pts.shape
    vs = np.asarray(voxel_size, np.float32)
    rg = np.asarray(pc_range, np.float32)
    vox = np.zeros((max_voxels, max_points, F), np.float32)
    coors = np.zeros((max_voxels, 3), np.int32)
    npts = np.zeros((max_voxels,), np.int32)
    fp = C.POINTER(C.c_float)
    ip = C.POINTER(C.c_int)
    V = lib.oracle_hard_voxelize(pts.ctypes.data_as(fp), n, F, vs.ctypes.data_as(fp), rg.ctypes.data_as(fp),
                                 max_points, max_voxels, vox.ctypes.data_as(fp), coors.ctypes.data_as(ip),
                                 npts.ctypes.data_as(ip))
    if V < 0:
        raise MemoryError("oracle_hard_voxelize")
    return vox[:V], coors[:V], npts[:V]


def voxelize_frames(frames, voxel_size, pc_range, max_points, max_voxels):
    """Det3DDataPreprocessor.voxelize (hard): per frame, pad batch id, concatenate."""
    vs, cs, ns = [], [], []
    for i, f in enumerate(frames):
        v, c, n = hard_voxelize(f, voxel_size, pc_range, max_points, max_voxels)
        vs.append(v)
        cs.append(np.concatenate([np.full((c.shape[0], 1), i, np.int32), c], 1))
        ns.append(n)
    return np.concatenate(vs), np.concatenate(cs), np.concatenate(ns)


def hard_voxelize_py(points, voxel_size, pc_range, max_points, max_voxels):
    """Independent pure-Python loop (small inputs only) used to check the C restatement."""
    pts = np.asarray(points, np.float32)
    vs = np.asarray(voxel_size, np.float32)
    rg = np.asarray(pc_range, np.float32)
    grid = [int(np.round(np.float32(rg[3 + j] - rg[j]) / vs[j])) for j in range(3)]
    table = {}
    voxels, coors, npts = [], [], []
    for p in pts:
        c = []
        ok = True
        for j in range(3):
            cf = np.floor(np.float32(np.float32(p[j] - rg[j]) / vs[j]))
            if not (cf >= 0 and cf < grid[j]):
                ok = False
                break
            c.append(int(cf))
        if not ok:
            continue
        key = (c[2], c[1], c[0])
        if key not in table:
            if len(voxels) >= max_voxels:
                continue
            table[key] = len(voxels)
            voxels.append(np.zeros((max_points, pts.shape[1]), np.float32))
            coors.append(key)
            npts.append(0)
        v = table[key]
        if npts[v] < max_points:
            voxels[v][npts[v]] = p
            npts[v] += 1
    F = pts.shape[1]
    if not voxels:
        return np.zeros((0, max_points, F), np.float32), np.zeros((0, 3), np.int32), np.zeros(0, np.int32)
    return np.stack(voxels), np.array(coors, np.int32), np.array(npts, np.int32)
