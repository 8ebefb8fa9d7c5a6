"""clip_grad_norm_ + AdamW as two HIP kernels.

mmengine's OptimWrapper for the reference configs
(configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:130-140:
AdamW lr 1e-4, betas (0.9, 0.999), weight_decay 1e-3, clip_grad max_norm 0.5, paramwise
custom_keys {'adversary': lr_mult 2.0}) runs torch.nn.utils.clip_grad_norm_ and then
torch.optim.AdamW — a few dozen small launches plus ~1 ms of Python per step. `ClipAdamW` keeps a
device table of (param, exp_avg, exp_avg_sq, numel, group, step) once, uploads the step's gradient
addresses (one pinned host->device copy) and runs csrc/step_tail.hip `rpc_clip_adamw`: a
deterministic global-norm pass and one fused clip + AdamW pass over fixed-size chunks.
It exposes the torch-optimizer surface the trainer and LR schedule use (`param_groups` with 'lr',
`step()`, `zero_grad()`, `state_dict()` / `load_state_dict()`).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _ffi

CHUNK = 16384  # RPC_OPTIM_CHUNK


class ClipAdamW:
    def __init__(self, param_groups, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-3, max_norm=0.5):
        self.param_groups = []
        for g in param_groups:
            g = dict(g)
            g["params"] = list(g["params"])
            g.setdefault("lr", lr)
            g.setdefault("initial_lr", g["lr"])
            self.param_groups.append(g)
        if len(self.param_groups) > 4:
            raise ValueError("at most 4 parameter groups")
        self.betas, self.eps, self.weight_decay, self.max_norm = betas, eps, weight_decay, max_norm
        self.params = [p for g in self.param_groups for p in g["params"]]
        gid = [i for i, g in enumerate(self.param_groups) for _ in g["params"]]
        if not self.params:
            raise ValueError("no parameters")
        dev = self.params[0].device
        if dev.type != "cuda":
            raise RuntimeError("ClipAdamW runs on the HIP kernels only (no CPU path)")
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev:
                raise RuntimeError("ClipAdamW needs contiguous fp32 parameters on one device")
        self.device = dev
        numel = [p.numel() for p in self.params]
        # moments in two flat buffers (torch's state['exp_avg'/'exp_avg_sq'] are views of them); every
        # view starts on a 256-byte boundary so the kernels' 16-byte vector path applies to all of them
        # (unpadded, the first tensor whose size is not a multiple of 4 — a head bias — pushed every
        # later tensor onto the scalar path)
        padded = [(n + 63) // 64 * 64 for n in numel]
        total = int(sum(padded))
        self.exp_avg = torch.zeros(total, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(total, dtype=torch.float32, device=dev)
        offs = np.concatenate([[0], np.cumsum(padded)[:-1]]).astype(np.int64)
        self._m_views = [self.exp_avg[o:o + n].view_as(p) for o, n, p in zip(offs, numel, self.params)]
        self._v_views = [self.exp_avg_sq[o:o + n].view_as(p) for o, n, p in zip(offs, numel, self.params)]
        self.steps = torch.zeros(len(self.params), dtype=torch.float32, device=dev)
        ctens, cstart = [], []
        for t, n in enumerate(numel):
            for s in range(0, n, CHUNK):
                ctens.append(t)
                cstart.append(s)
        self.nchunks = len(ctens)
        i64 = lambda v: torch.tensor(v, dtype=torch.int64, device=dev)
        i32 = lambda v: torch.tensor(v, dtype=torch.int32, device=dev)
        self._pptr = i64([p.data_ptr() for p in self.params])
        self._mptr = i64([m.data_ptr() for m in self._m_views])
        self._vptr = i64([v.data_ptr() for v in self._v_views])
        self._numel, self._group = i32(numel), i32(gid)
        self._ctens, self._cstart = i32(ctens), i32(cstart)
        self._gptr_host = torch.zeros(len(self.params), dtype=torch.int64, pin_memory=True)
        self._gptr_np = self._gptr_host.numpy()
        self._gptr = torch.zeros(len(self.params), dtype=torch.int64, device=dev)
        lib = _ffi.load()
        self._wsz = lib.rpc_clip_adamw_workspace_size(self.nchunks)
        self._ws = _ffi.workspace(self._wsz, dev)
        self.norm = torch.zeros(2, dtype=torch.float32, device=dev)
        self._hyper = _ffi.RpcAdamWHyper()
        self._gptr_event = None

    @torch.no_grad()
    def step(self):
        """clip_grad_norm_(max_norm) then one AdamW step. Returns the device [2] tensor
        (total gradient norm, clip coefficient)."""
        lib = _ffi.load()
        if self._gptr_event is not None:   # last step's host->device copy of the pinned buffer is done
            self._gptr_event.synchronize()
        g_np = self._gptr_np
        for i, p in enumerate(self.params):
            g = p.grad
            if g is None:
                g_np[i] = 0
                continue
            if g.dtype != torch.float32 or not g.is_contiguous():
                raise RuntimeError("ClipAdamW needs contiguous fp32 gradients")
            g_np[i] = g.data_ptr()
        self._gptr.copy_(self._gptr_host, non_blocking=True)
        h = self._hyper
        for i, g in enumerate(self.param_groups):
            h.lr[i] = float(g["lr"])
        h.beta1, h.beta2 = self.betas
        h.eps, h.weight_decay = self.eps, self.weight_decay
        st = _ffi.stream_of(self.norm)
        _ffi.check(lib.rpc_clip_adamw(_ffi.ptr(self._pptr), _ffi.ptr(self._gptr), _ffi.ptr(self._mptr),
                                      _ffi.ptr(self._vptr), _ffi.ptr(self._numel), _ffi.ptr(self._group),
                                      _ffi.ptr(self._ctens), _ffi.ptr(self._cstart), self.nchunks, len(self.params),
                                      _ffi.ptr(self.steps), C.byref(h), float(self.max_norm or 0.0),
                                      _ffi.ptr(self.norm), _ffi.ptr(self._ws), self._wsz, st), "rpc_clip_adamw")
        # the host pointer buffer is rewritten next step: order that after this copy
        self._gptr_event = torch.cuda.Event()
        self._gptr_event.record(torch.cuda.current_stream(self.device))
        return self.norm

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    # ------------------------------------------------------------------ checkpoints (torch layout)
    def state_dict(self):
        state = {i: dict(step=self.steps[i].detach().clone().cpu(), exp_avg=self._m_views[i].detach().clone(),
                         exp_avg_sq=self._v_views[i].detach().clone()) for i in range(len(self.params))}
        groups, k = [], 0
        for g in self.param_groups:
            d = {kk: v for kk, v in g.items() if kk != "params"}
            d.update(params=list(range(k, k + len(g["params"]))), betas=self.betas, eps=self.eps,
                     weight_decay=self.weight_decay)
            k += len(g["params"])
            groups.append(d)
        return dict(state=state, param_groups=groups)

    @torch.no_grad()
    def load_state_dict(self, sd):
        for i, s in sd["state"].items():
            i = int(i)
            self._m_views[i].copy_(s["exp_avg"])
            self._v_views[i].copy_(s["exp_avg_sq"])
            self.steps[i] = float(s["step"])
        for g, d in zip(self.param_groups, sd["param_groups"]):
            g["lr"] = d["lr"]
            g["initial_lr"] = d.get("initial_lr", d["lr"])


class OptimWrapper:
    """The mmengine `OptimWrapper` / `AmpOptimWrapper` surface a model's `train_step` calls
    (`optim_context`, `update_params`, plus `backward` / `step` / `zero_grad` / `param_groups`),
    over `ClipAdamW` on a ROCm device (clip_grad fused into the step) or torch AdamW +
    clip_grad_norm_ on the host. `amp_dtype` (AmpOptimWrapper) turns autocast on in
    `optim_context`, which selects the bf16 perf engines (base_model.select_engines)."""

    def __init__(self, optimizer, clip_grad=None, amp_dtype=None):
        self.optimizer = optimizer
        self.clip_grad = dict(clip_grad) if clip_grad else None
        if self.clip_grad and float(self.clip_grad.get("norm_type", 2)) != 2.0:
            raise ValueError("clip_grad: only the L2 norm (norm_type 2) of the reference configs is supported")
        self.amp_dtype = amp_dtype
        self.grad_norm = None

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    def optim_context(self, model):
        import contextlib
        if self.amp_dtype is None:
            return contextlib.nullcontext()
        return torch.autocast("cuda", dtype=self.amp_dtype)

    def backward(self, loss):
        loss.backward()

    def step(self):
        if isinstance(self.optimizer, ClipAdamW):
            self.grad_norm = self.optimizer.step()[0]
            return
        if self.clip_grad:
            params = [p for g in self.optimizer.param_groups for p in g["params"] if p.grad is not None]
            self.grad_norm = torch.nn.utils.clip_grad_norm_(params, float(self.clip_grad["max_norm"]))
        self.optimizer.step()

    def zero_grad(self):
        self.optimizer.zero_grad(set_to_none=True)

    def update_params(self, loss):
        self.backward(loss)
        self.step()
        self.zero_grad()

    def state_dict(self):
        return self.optimizer.state_dict()

    def load_state_dict(self, sd):
        self.optimizer.load_state_dict(sd)
