"""rpc_bn_finalize (the BatchNorm statistics of every sparse / dense / VFE layer) against a float64 restatement
of its arithmetic, both modes, float and double partial rows (RPC_BN_PART_F64), channel counts that are not a
multiple of the kernel's 16-channel blocks and partial-row counts on both sides of its 8-row unroll."""
import numpy as np
import pytest
import torch

from robustpointclouds_amd import _ffi

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _ref(part, C, N, mode, gamma, beta, eps, mom, rm, rv, fbn):
    s1, s2 = part[:, :C].sum(0), part[:, C:].sum(0)
    if mode == 0:
        mean = s1 / N
        var = np.maximum(s2 / N - mean * mean, 0)
        invstd = 1.0 / np.sqrt(var.astype(np.float32) + np.float32(eps))
        bn = np.concatenate([gamma * invstd, beta, mean, invstd])
        uvar = var * N / (N - 1)
        return bn, (1 - mom) * rm + mom * mean, (1 - mom) * rv + mom * uvar
    bn = np.concatenate([gamma * fbn[3 * C:], s1 / N, s2 / N, fbn[2 * C:3 * C], fbn[3 * C:]])
    return bn, s2, s1


@pytest.mark.parametrize("C", [5, 16, 48, 128, 256])
@pytest.mark.parametrize("nblk", [1, 7, 515, 4700])
@pytest.mark.parametrize("f64", [False, True])
def test_bn_finalize_matches_float64(C, nblk, f64):
    lib = _ffi.load()
    rng = np.random.default_rng(C * 10007 + nblk)
    N = nblk * 64
    dt = np.float64 if f64 else np.float32
    s = rng.normal(0.5, 1.0, (nblk, C)).astype(dt)
    part = np.concatenate([s, (s * s + rng.uniform(0.5, 2.0, (nblk, C))).astype(dt)], 1)
    gamma = rng.uniform(0.5, 1.5, C).astype(np.float32)
    beta = rng.uniform(-0.2, 0.2, C).astype(np.float32)
    fbn = np.concatenate([gamma, beta, rng.normal(0, 1, C), rng.uniform(0.5, 2, C)]).astype(np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
    st = _ffi.stream_of(t(gamma))
    for mode in (0, 1):
        rm, rv = t(np.zeros(C, np.float32)), t(np.ones(C, np.float32))
        bn = torch.zeros(5 * C, dtype=torch.float32, device=DEV)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        pp, g, b, f = t(part), t(gamma), t(beta), t(fbn)
        _ffi.check(lib.rpc_bn_finalize(_ffi.ptr(pp), nblk, C, N, mode | (4 if f64 else 0), _ffi.ptr(g), _ffi.ptr(b),
                                       1e-3, 0.01, _ffi.ptr(rm), _ffi.ptr(rv), _ffi.ptr(f), _ffi.ptr(bn),
                                       _ffi.ptr(dg), _ffi.ptr(db), None, st), "rpc_bn_finalize")
        torch.cuda.synchronize()
        want = _ref(part.astype(np.float64), C, N, mode, gamma.astype(np.float64), beta.astype(np.float64), 1e-3, 0.01,
                    np.zeros(C), np.ones(C), fbn.astype(np.float64))
        nb = 4 * C if mode == 0 else 5 * C
        np.testing.assert_allclose(bn.cpu().numpy()[:nb], want[0], rtol=2e-6, atol=1e-6)
        if mode == 0:
            np.testing.assert_allclose(rm.cpu().numpy(), want[1], rtol=2e-6, atol=1e-7)
            np.testing.assert_allclose(rv.cpu().numpy(), want[2], rtol=2e-6, atol=1e-7)
        else:
            np.testing.assert_allclose(dg.cpu().numpy(), want[1], rtol=2e-6)
            np.testing.assert_allclose(db.cpu().numpy(), want[2], rtol=2e-6)
