"""ctypes binding of librpc_hip.so (declared in include/rpc_hip.h).

The product path has no fallback: if the library is missing or cannot be loaded, every
op raises. Device buffers are torch tensors; only raw pointers and sizes cross the ABI.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch

# RPC_HIP_LIB: load another build of the same library (A/B measurements in tools/); default in-tree
_LIB_PATH = os.environ.get("RPC_HIP_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                         "librpc_hip.so")
_lock = threading.Lock()
_lib = None

RPC_ERRORS = {1: "bad argument", 2: "workspace too small", 3: "unsupported width combination",
              4: "HIP runtime error"}
PERTURBER_NPARAMS = 36

vp = C.c_void_p
i32 = C.c_int
sz = C.c_size_t
fp = C.POINTER(C.c_float)
ip = C.POINTER(C.c_int)


class PerturberCfg(C.Structure):
    _fields_ = [("F", C.c_int), ("hidden", C.c_int * 3), ("use_attention", C.c_int),
                ("training", C.c_int), ("sensor_error_bound", C.c_float), ("bn_eps", C.c_float),
                ("bn_momentum", C.c_float), ("vfe_features", C.c_int), ("wgrad_split_bf16", C.c_int),
                ("act16", C.c_int)]


class RpcHardVfeCfg(C.Structure):
    """include/rpc_hip.h RpcHardVfeCfg."""
    _fields_ = [("F", C.c_int), ("T", C.c_int), ("nlayers", C.c_int), ("channels", C.c_int * 4),
                ("with_cluster_center", C.c_int), ("with_voxel_center", C.c_int), ("with_distance", C.c_int),
                ("training", C.c_int), ("voxel_size", C.c_float * 3), ("pc_range_min", C.c_float * 3),
                ("bn_eps", C.c_float), ("bn_momentum", C.c_float)]


class RpcHeadCfg(C.Structure):
    """include/rpc_hip.h RpcHeadCfg (field order and types must match)."""
    _fields_ = [("B", C.c_int), ("H", C.c_int), ("W", C.c_int), ("S", C.c_int), ("R", C.c_int), ("C", C.c_int),
                ("NA", C.c_int), ("assigner_per_size", C.c_int), ("assign_per_class", C.c_int),
                ("use_dir", C.c_int), ("diff_rad_by_sin", C.c_int),
                ("pos_iou_thr", C.c_float * 4), ("neg_iou_thr", C.c_float * 4), ("min_pos_iou", C.c_float * 4),
                ("dir_offset", C.c_float), ("dir_limit_offset", C.c_float), ("pos_weight", C.c_float),
                ("beta", C.c_float), ("gamma", C.c_float), ("alpha", C.c_float),
                ("lw_cls", C.c_float), ("lw_bbox", C.c_float), ("lw_dir", C.c_float),
                ("z_bf16", C.c_int), ("z_sb", C.c_longlong), ("z_shw", C.c_longlong), ("z_sn", C.c_longlong),
                ("dz_bf16", C.c_int), ("dz_sb", C.c_longlong), ("dz_shw", C.c_longlong), ("dz_sn", C.c_longlong),
                ("dz_nwrite", C.c_int)]


class RpcAdamWHyper(C.Structure):
    _fields_ = [("lr", C.c_float * 4), ("beta1", C.c_float), ("beta2", C.c_float), ("eps", C.c_float),
                ("weight_decay", C.c_float)]


class RpcStrongCfg(C.Structure):
    _fields_ = [("epoch_scaling", C.c_double), ("complexity", C.c_double), ("max_scaling", C.c_double),
                ("adversarial_loss_weight", C.c_double), ("momentum_alpha", C.c_float), ("dynamic", C.c_int), ("curriculum", C.c_int),
                ("history_count", C.c_longlong)]


class RpcAugFrame(C.Structure):
    _fields_ = [("flip_h", C.c_int), ("flip_v", C.c_int), ("rot", C.c_float), ("cosr", C.c_float),
                ("sinr", C.c_float), ("scale", C.c_float), ("tx", C.c_float), ("ty", C.c_float), ("tz", C.c_float)]


class RpcDenseWprep(C.Structure):
    """include/rpc_hip.h RpcDenseWprep."""
    _fields_ = [("W", C.c_void_p), ("w_fwd", C.c_void_p), ("w_dgrad", C.c_void_p), ("kind", C.c_int),
                ("ci", C.c_int), ("co", C.c_int), ("taps", C.c_int), ("flip", C.c_int), ("co_src", C.c_int)]


class RpcSpconvWprep(C.Structure):
    """include/rpc_hip.h RpcSpconvWprep."""
    _fields_ = [("W", C.c_void_p), ("bt", C.c_void_p), ("kvol", C.c_int), ("ci", C.c_int), ("co", C.c_int),
                ("dgrad", C.c_int), ("fmt", C.c_int)]


class RpcSparseLayer(C.Structure):
    """include/rpc_hip.h RpcSparseLayer (one sparse conv of the rpc_sparse_backward layer table)."""
    _fields_ = [("kind", C.c_int), ("ci", C.c_int), ("co", C.c_int), ("kvol", C.c_int), ("n_in", C.c_int),
                ("n_out", C.c_int), ("bf16", C.c_int), ("mat", C.c_int), ("res", C.c_int),
                ("nbr", C.c_void_p), ("nbr_in", C.c_void_p), ("z", C.c_void_p), ("bn", C.c_void_p),
                ("out", C.c_void_p), ("h_in", C.c_void_p), ("src", C.c_void_p), ("src_bn", C.c_void_p),
                ("W", C.c_void_p), ("gamma", C.c_void_p), ("beta", C.c_void_p), ("btd", C.c_void_p),
                ("dW", C.c_void_p), ("dgamma", C.c_void_p), ("dbeta", C.c_void_p), ("h_fmt", C.c_int),
                ("fin_ticket", C.c_void_p)]


class RpcBnFin(C.Structure):
    """include/rpc_hip.h RpcBnFin (BatchNorm finalize fused into rpc_spconv_gemm_bf16_fin)."""
    _fields_ = [("ticket", C.c_void_p), ("gpart", C.c_void_p), ("mode", C.c_int), ("gamma", C.c_void_p),
                ("beta", C.c_void_p), ("eps", C.c_float), ("momentum", C.c_float), ("running_mean", C.c_void_p),
                ("running_var", C.c_void_p), ("fbn", C.c_void_p), ("bn", C.c_void_p), ("dgamma", C.c_void_p),
                ("dbeta", C.c_void_p)]


class RpcCenterCfg(C.Structure):
    """include/rpc_hip.h RpcCenterCfg."""
    _fields_ = [("B", C.c_int), ("H", C.c_int), ("W", C.c_int), ("ntasks", C.c_int), ("ncls_total", C.c_int),
                ("task_ncls", C.c_int * 8), ("max_objs", C.c_int), ("min_radius", C.c_int),
                ("out_size_factor", C.c_int), ("norm_bbox", C.c_int), ("voxel_x", C.c_float), ("voxel_y", C.c_float),
                ("pc_x", C.c_float), ("pc_y", C.c_float), ("gaussian_overlap", C.c_double),
                ("code_weights", C.c_float * 10), ("loss_cls_weight", C.c_float), ("loss_bbox_weight", C.c_float),
                ("hm_pitch", C.c_int), ("box_pitch", C.c_int)]


# name -> (restype, argtypes); every symbol here must be exported by the .so
SIGNATURES = {
    "rpc_version": (C.c_char_p, []),
    "rpc_hard_voxelize_workspace_size": (sz, [i32, i32]),
    "rpc_hard_voxelize": (i32, [vp, i32, i32, vp, i32, fp, fp, i32, i32, vp, vp, vp, vp, vp, sz, vp]),
    "rpc_vfe_mean_forward": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "rpc_vfe_mean_backward": (i32, [vp, vp, i32, i32, i32, i32, vp, vp]),
    "rpc_hard_vfe_workspace_size": (sz, [C.POINTER(RpcHardVfeCfg), i32]),
    "rpc_hard_vfe_forward": (i32, [C.POINTER(RpcHardVfeCfg), C.POINTER(vp), vp, vp, vp, i32, vp, vp, sz, vp]),
    "rpc_hard_vfe_backward": (i32, [C.POINTER(RpcHardVfeCfg), C.POINTER(vp), vp, vp, vp, i32, vp, vp,
                                    C.POINTER(vp), vp, sz, vp]),
    "rpc_perturber_workspace_size": (sz, [C.POINTER(PerturberCfg), i32, i32]),
    "rpc_perturber_forward": (i32, [C.POINTER(PerturberCfg), C.POINTER(vp), vp, i32, i32, vp, vp, vp,
                                    vp, vp, sz, vp]),
    "rpc_perturber_backward": (i32, [C.POINTER(PerturberCfg), C.POINTER(vp), vp, i32, i32, vp, vp, vp,
                                     C.POINTER(vp), vp, sz, vp]),
    "rpc_subm_rulebook": (i32, [vp, i32, ip, ip, vp, vp, vp]),
    "rpc_spconv_rulebook_workspace_size": (sz, [i32, i32]),
    "rpc_spconv_rulebook_count": (i32, [vp, i32, ip, ip, ip, ip, vp, vp, vp, sz, vp]),
    "rpc_spconv_rulebook_build": (i32, [vp, i32, ip, ip, ip, ip, vp, i32, vp, vp, vp, vp, vp]),
    "rpc_spconv_gemm_blocks": (i32, [i32]),
    "rpc_spconv_forward": (i32, [vp, vp, i32, vp, i32, i32, vp, i32, vp, vp, vp]),
    "rpc_spconv_dgrad": (i32, [vp, vp, vp, i32, vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp]),
    "rpc_spconv_wgrad_workspace_size": (sz, [i32, i32, i32, i32]),
    "rpc_spconv_wgrad": (i32, [vp, vp, i32, vp, i32, i32, vp, vp, vp, i32, vp, vp, sz, vp]),
    "rpc_bn_finalize_workspace_size": (sz, [i32]),
    "rpc_bn_finalize": (i32, [vp, i32, i32, i32, i32, vp, vp, C.c_float, C.c_float, vp, vp, vp, vp, vp, vp,
                              vp, vp]),
    "rpc_sparse_to_dense": (i32, [vp, vp, vp, i32, i32, ip, i32, vp, vp]),
    "rpc_sparse_dense_clear": (i32, [vp, i32, i32, ip, i32, vp, vp]),
    "rpc_dense_to_sparse_grad": (i32, [vp, vp, vp, vp, i32, i32, ip, i32, vp, vp, vp]),
    "rpc_to_bf16_rows": (i32, [vp, vp, i32, i32, i32, vp, vp]),
    "rpc_bnbwd_to_bf16_rows": (i32, [vp, vp, vp, i32, i32, vp, vp]),
    "rpc_spconv_bf16_weight_elems": (sz, [i32, i32, i32, i32]),
    "rpc_spconv_prep_weight_bf16": (i32, [vp, i32, i32, i32, i32, vp, vp]),
    "rpc_spconv_prep_weight_bf16_batch": (i32, [vp, i32, vp]),
    "rpc_spconv_gemm_bf16": (i32, [vp, i32, vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32, vp]),
    "rpc_spconv_gemm_bf16_n": (i32, [vp, i32, i32, vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32, vp]),
    "rpc_spconv_gemm_h16": (i32, [vp, i32, i32, i32, vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32, vp]),
    "rpc_to_h16_rows": (i32, [vp, vp, i32, i32, i32, i32, vp, vp, vp]),
    "rpc_spconv_wgrad_h16": (i32, [vp, i32, i32, vp, i32, i32, vp, i32, vp, vp, sz, vp]),
    "rpc_sparse_res_forward_h16": (i32, [vp, vp, vp, i32, i32, vp, vp, i32, vp, vp]),
    "rpc_bn_fin_groups": (i32, [i32]),
    "rpc_bn_fin_tickets": (i32, [i32]),
    "rpc_spconv_gemm_bf16_fin": (i32, [vp, i32, i32, vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, i32,
                                       C.POINTER(RpcBnFin), vp]),
    "rpc_sparse_tune": (i32, [i32, i32]),
    "rpc_spconv_gemm_res": (i32, [vp, i32, i32, vp, i32, i32, i32, vp, i32, vp, vp, vp, vp, vp, vp,
                                  C.POINTER(RpcBnFin), vp]),
    "rpc_spconv_wgrad_bf16_workspace_size": (sz, [i32, i32, i32, i32]),
    "rpc_spconv_wgrad_bf16": (i32, [vp, i32, vp, i32, i32, vp, i32, vp, vp, sz, vp]),
    "rpc_sparse_backward_workspace_size": (sz, [vp, i32]),
    "rpc_sparse_backward": (i32, [vp, i32, vp, vp, ip, i32, vp, vp, sz, vp, vp]),
    "rpc_dense_conv": (i32, [i32, vp, i32, i32, vp, i32, vp, i32, i32, i32, vp, ip, ip, ip, vp]),
    "rpc_dense_conv_blocks": (i32, [i32, ip]),
    "rpc_dense_conv_s1_kernel": (i32, [i32, i32, ip]),
    "rpc_dense_conv_part_rows": (i32, [i32, i32, ip]),
    "rpc_dense_conv_bnbwd": (i32, [vp, i32, i32, vp, i32, vp, i32, vp, vp, vp, ip, vp]),
    "rpc_dense_tune": (i32, [i32, i32]),
    "rpc_dense_wgrad_workspace_size": (sz, [i32, ip, i32, i32]),
    "rpc_dense_wgrad": (i32, [i32, i32, vp, i32, i32, vp, i32, i32, ip, ip, ip, vp, vp, sz, vp]),
    "rpc_dense_bn_apply": (i32, [vp, i32, i32, vp, vp, i32, i32, vp]),
    "rpc_dense_bnbwd_blocks": (i32, [i32]),
    "rpc_dense_bnbwd_stats": (i32, [vp, i32, i32, vp, i32, i32, vp, vp, vp]),
    "rpc_dense_bnbwd_apply": (i32, [vp, i32, i32, vp, i32, i32, vp, vp, vp, vp]),
    "rpc_dense_wprep": (i32, [vp, i32, i32, i32, i32, i32, vp, vp, vp]),
    "rpc_dense_wprep_batch": (i32, [vp, i32, vp]),
    "rpc_dense_conv_f32": (i32, [i32, vp, i32, i32, vp, i32, vp, i32, i32, i32, vp, ip, ip, ip, vp]),
    "rpc_dense_conv_blocks_f32": (i32, [i32, ip]),
    "rpc_dense_wgrad_workspace_size_f32": (sz, [i32, ip, i32, i32]),
    "rpc_dense_wgrad_f32": (i32, [i32, i32, vp, i32, i32, vp, i32, i32, ip, ip, ip, vp, vp, sz, vp]),
    "rpc_dense_bn_apply_f32": (i32, [vp, i32, i32, vp, vp, i32, i32, vp]),
    "rpc_dense_bnbwd_stats_f32": (i32, [vp, i32, i32, vp, i32, i32, vp, vp, vp]),
    "rpc_dense_bnbwd_apply_f32": (i32, [vp, i32, i32, vp, i32, i32, vp, vp, vp, vp]),
    "rpc_dense_wprep_batch_f32": (i32, [vp, i32, vp]),
    "rpc_loss_tail_forward": (i32, [vp, vp, C.c_float, vp, vp]),
    "rpc_loss_tail_backward": (i32, [vp, C.c_float, vp, vp, vp, vp]),
    "rpc_center_tail_forward": (i32, [vp, i32, vp, C.c_float, C.c_float, vp, vp]),
    "rpc_center_tail_backward": (i32, [vp, i32, C.c_float, C.c_float, vp, vp, vp, vp]),
    "rpc_clip_adamw_workspace_size": (sz, [i32]),
    "rpc_clip_adamw": (i32, [vp, vp, vp, vp, vp, vp, vp, vp, i32, i32, vp, C.POINTER(RpcAdamWHyper), C.c_float, vp,
                             vp, sz, vp]),
    "rpc_strong_perturb_workspace_size": (sz, []),
    "rpc_strong_perturb_forward": (i32, [C.POINTER(RpcStrongCfg), vp, vp, vp, C.c_longlong, vp, vp, vp, vp, vp, sz,
                                         vp]),
    "rpc_strong_perturb_backward": (i32, [vp, C.c_longlong, vp, vp, vp, vp, vp, vp]),
    "rpc_augment_points_workspace_size": (sz, [i32, i32]),
    "rpc_augment_points": (i32, [vp, i32, i32, vp, i32, vp, fp, i32, C.c_ulonglong, vp, vp, vp, sz, vp]),
    "rpc_augment_boxes": (i32, [vp, vp, i32, i32, vp, fp, vp]),
    "rpc_head_pack": (i32, [vp, i32, i32, vp, vp, i32, i32, C.c_longlong, vp]),
    "rpc_head_unpack_workspace_size": (sz, []),
    "rpc_head_unpack_grad": (i32, [vp, i32, i32, i32, vp, i32, C.c_longlong, vp, vp, sz, vp]),
    "rpc_dcn_prep_weight": (i32, [vp, vp, vp, vp]),
    "rpc_dcn_forward": (i32, [vp, i32, vp, i32, vp, vp, vp, i32, i32, i32, i32, vp]),
    "rpc_dcn_backward_workspace_size": (sz, [i32, i32, i32]),
    "rpc_dcn_backward": (i32, [vp, i32, vp, i32, vp, vp, vp, i32, vp, vp, i32, vp, vp, i32, i32, i32, vp, sz, vp]),
    "rpc_dcn_forward_f32": (i32, [vp, i32, vp, i32, vp, vp, vp, i32, i32, i32, i32, vp]),
    "rpc_dcn_backward_f32": (i32, [vp, i32, vp, i32, vp, vp, vp, i32, vp, vp, i32, vp, vp, i32, i32, i32, vp, sz,
                                   vp]),
    "rpc_dcn_backward_ex": (i32, [vp, i32, vp, i32, vp, vp, vp, i32, vp, vp, i32, i32, vp, vp, i32, i32, i32, vp, sz,
                                  vp]),
    "rpc_dcn_backward_f32_ex": (i32, [vp, i32, vp, i32, vp, vp, vp, i32, vp, vp, i32, i32, vp, vp, i32, i32, i32, vp,
                                      sz, vp]),
    "rpc_head_pack_f32": (i32, [vp, i32, i32, vp, vp, i32, i32, C.c_longlong, vp]),
    "rpc_head_unpack_grad_f32": (i32, [vp, i32, i32, i32, vp, i32, C.c_longlong, vp, vp, sz, vp]),
    "rpc_sparse_res_forward": (i32, [vp, vp, vp, i32, i32, vp, vp, vp]),
    "rpc_sparse_res_backward": (i32, [vp, vp, vp, vp, vp, i32, i32, vp, vp, vp]),
    "rpc_center_head_workspace_size": (sz, [C.POINTER(RpcCenterCfg), i32]),
    "rpc_center_head_loss_forward": (i32, [C.POINTER(RpcCenterCfg), vp, vp, i32, vp, vp, vp, vp, sz, vp]),
    "rpc_center_head_loss_backward": (i32, [C.POINTER(RpcCenterCfg), vp, vp, vp, vp, vp, vp, sz, vp]),
    "rpc_center_head_targets": (i32, [C.POINTER(RpcCenterCfg), i32, vp, C.POINTER(vp), C.POINTER(vp),
                                      C.POINTER(vp), C.POINTER(vp)]),
    "rpc_stream_create": (i32, [i32, C.POINTER(vp)]),
    "rpc_stream_priority_range": (i32, [C.POINTER(i32), C.POINTER(i32)]),
    "rpc_anchor_head_workspace_size": (sz, [C.POINTER(RpcHeadCfg), i32]),
    "rpc_anchor_head_loss_forward": (i32, [C.POINTER(RpcHeadCfg), vp, vp, vp, i32, vp, vp, vp, vp, vp, sz, vp]),
    "rpc_anchor_head_loss_backward": (i32, [C.POINTER(RpcHeadCfg), vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, vp,
                                            sz, vp]),
}


def lib_path() -> str:
    return _LIB_PATH


def load():
    """Load (once) and return the ctypes library; raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"librpc_hip.so not built ({_LIB_PATH}); run "
                               "`python -m robustpointclouds_amd._build` — there is no CPU fallback")
        lib = C.CDLL(_LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def bump_batches(bns) -> None:
    """num_batches_tracked += 1 for a list of BatchNorm modules: one multi-tensor kernel instead of one
    add kernel (and one Module.__setattr__ / register_buffer round trip) per module."""
    ts = [m.num_batches_tracked for m in bns if getattr(m, "num_batches_tracked", None) is not None]
    if ts:
        torch._foreach_add_(ts, 1)


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: rpc error {rc} ({RPC_ERRORS.get(rc, '?')})")


def ptr(t: torch.Tensor | None):
    return None if t is None else C.c_void_p(t.data_ptr())


def stream_of(t: torch.Tensor):
    if not t.is_cuda:
        raise RuntimeError("rpc_hip ops run on the GPU only (no CPU fallback); got a CPU tensor")
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


# RPC_SIDE_PRIORITY=1: side-work streams (batch prefetch, sparse rulebooks / weight gradients) are HIP
# streams at the device's least priority, so the training stream's kernels are dispatched first
SIDE_PRIORITY = os.environ.get("RPC_SIDE_PRIORITY", "0") != "0"
_side_streams: list = []


def side_stream(device) -> torch.cuda.Stream:
    """A stream for work off the step's critical path (torch.cuda.Stream, or with RPC_SIDE_PRIORITY a
    least-priority HIP stream wrapped as torch.cuda.ExternalStream; never destroyed)."""
    if not SIDE_PRIORITY:
        return torch.cuda.Stream(device)
    lib = load()
    out = C.c_void_p()
    with torch.cuda.device(device):
        check(lib.rpc_stream_create(1, C.byref(out)), "rpc_stream_create")
    s = torch.cuda.ExternalStream(out.value, device=device)
    _side_streams.append(s)
    return s


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


_ARMED: dict = {}


def float_arr(vals):
    return (C.c_float * len(vals))(*[float(v) for v in vals])


def int_arr(vals):
    return (C.c_int * len(vals))(*[int(v) for v in vals])
