"""CPU simulation for the sparse-encoder block-union design: per 128-row block of each
layer's rulebook, how many distinct source rows the block's valid pairs reference (U) against the pairs
themselves, in the HIP row order (first appearance) and in spatially bricked orders."""
import sys

import numpy as np

sys.path.insert(0, ".")
from oracle import voxelize as ov  # noqa: E402
from robustpointclouds_amd.synthetic import KITTI_PC_RANGE, KITTI_VOXEL_SIZE, kitti_batch  # noqa: E402


def keys(c, shp):
    B, D, H, W = shp
    c = c.astype(np.int64)
    return ((c[:, 0] * D + c[:, 1]) * H + c[:, 2]) * W + c[:, 3]


def subm_nbr(c, shp):
    B, D, H, W = shp
    k = keys(c, shp)
    o = np.argsort(k)
    sk = k[o]
    nbr = np.full((len(c), 27), -1, np.int64)
    i = 0
    for a in (-1, 0, 1):
        for b in (-1, 0, 1):
            for d in (-1, 0, 1):
                n = c + np.array([0, a, b, d])
                ok = (n[:, 1] >= 0) & (n[:, 1] < D) & (n[:, 2] >= 0) & (n[:, 2] < H) & (n[:, 3] >= 0) & (n[:, 3] < W)
                nk = keys(n, shp)
                pos = np.clip(np.searchsorted(sk, nk), 0, len(sk) - 1)
                hit = ok & (sk[pos] == nk)
                nbr[hit, i] = o[pos[hit]]
                i += 1
    return nbr


def strided(c, shp_out, ksz, stride, pad):
    """HIP first-appearance output order (a cell's head = smallest r*K + k) + nbr_out [n_out][K]"""
    K = ksz[0] * ksz[1] * ksz[2]
    cand = []
    t = 0
    rows, ks, oc = [], [], []
    kk = 0
    for a in range(ksz[0]):
        for b in range(ksz[1]):
            for d in range(ksz[2]):
                n = c[:, 1:] + np.array(pad) - np.array([a, b, d])
                ok = np.all(n >= 0, 1) & np.all(n % np.array(stride) == 0, 1)
                o = n // np.array(stride)
                ok &= (o[:, 0] < shp_out[1]) & (o[:, 1] < shp_out[2]) & (o[:, 2] < shp_out[3])
                r = np.nonzero(ok)[0]
                rows.append(r)
                ks.append(np.full(len(r), kk))
                oc.append(np.concatenate([c[r, :1], o[ok]], 1))
                kk += 1
    rows, ks, oc = np.concatenate(rows), np.concatenate(ks), np.concatenate(oc)
    t = rows * K + ks
    kk_ = keys(oc, shp_out)
    order = np.lexsort((t, kk_))
    first = np.ones(len(order), bool)
    first[1:] = kk_[order][1:] != kk_[order][:-1]
    heads = order[first]
    heads = heads[np.argsort(t[heads])]                 # numbered in head order
    cell_id = {}
    ukey = kk_[heads]
    idx = np.argsort(ukey)
    pos = np.searchsorted(ukey[idx], kk_)
    out_row = idx[pos]
    nbr = np.full((len(heads), K), -1, np.int64)
    nbr[out_row, ks] = rows
    return oc[heads], nbr


def stats(nbr, perm=None, BMR=128):
    n = nbr.shape[0]
    if perm is not None:
        nbr = nbr[perm]
    U, P = [], []
    for r0 in range(0, n, BMR):
        blk = nbr[r0:r0 + BMR]
        v = blk[blk >= 0]
        U.append(len(np.unique(v)))
        P.append(len(v))
    U, P = np.array(U), np.array(P)
    return U.mean(), U.max(), P.mean(), np.percentile(U, 99)


def brick_perm(c, bz, by, bx):
    k = np.lexsort((c[:, 3] % bx, c[:, 2] % by, c[:, 1] % bz, c[:, 3] // bx, c[:, 2] // by, c[:, 1] // bz, c[:, 0]))
    return k


def main():
    pts, _, _ = kitti_batch(6, seed0=0, num_classes=3)
    v, c, n = ov.voxelize_frames(pts, KITTI_VOXEL_SIZE, KITTI_PC_RANGE, 5, 16000)
    c = c.astype(np.int64)
    shp = (6, 41, 1600, 1408)
    levels = []
    levels.append(("L0 subm", c, shp, subm_nbr(c, shp)))
    plan = [((21, 800, 704), (1, 1, 1)), ((11, 400, 352), (1, 1, 1)), ((5, 200, 176), (0, 1, 1))]
    cur = c
    for so, pad in plan:
        so = (6,) + so
        oc, nb = strided(cur, so, (3, 3, 3), (2, 2, 2), pad)
        levels.append((f"spconv->{so[1:]}", oc, so, nb))
        levels.append((f"subm {so[1:]}", oc, so, subm_nbr(oc, so)))
        cur = oc
    for name, cc, sh, nb in levels:
        print(f"{name:28s} rows {nb.shape[0]:7d} valid/row {float((nb >= 0).sum(1).mean()):5.2f}")
        for tag, perm in (("first-appearance", None), ("brick 2x4x16", brick_perm(cc, 2, 4, 16)),
                          ("brick 4x4x8", brick_perm(cc, 4, 4, 8)), ("brick 1x8x16", brick_perm(cc, 1, 8, 16)),
                          ("brick 2x8x8", brick_perm(cc, 2, 8, 8)), ("brick 3x6x8", brick_perm(cc, 3, 6, 8))):
            if "subm" not in name and perm is not None:
                continue
            um, ux, pm, u99 = stats(nb, perm)
            print(f"   {tag:18s} U mean {um:6.1f} p99 {u99:6.0f} max {ux:5d}  pairs/blk {pm:7.1f}  ratio {pm / um:5.2f}")


if __name__ == "__main__":
    main()
