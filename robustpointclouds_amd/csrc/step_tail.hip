// Step tail, for gfx950: the loss combination of AdversarialVoxelNet.loss + mmengine parse_losses
// (§8(a) rows a9, a10) and the optimizer update (clip_grad_norm_ + AdamW, row a10).
//
// Loss tail — models/detectors/adversarial_voxelnet.py:187-421 with upstream's list-valued
// Anchor3DHead losses (SURVEY.md finding 3: no Tensor-valued 'loss' entry, so det_loss_total = 0
// and loss_adversarial = 0.01 * (loss_intensity + loss_bias + loss_imbalance)), then mmengine
// `BaseModel.parse_losses` (total = sum of every 'loss' key in dict order). One single-wave kernel
// forward, one backward (the Jacobian is constant except the l2 multiplier tier, :401-411), instead
// of ~40 scalar torch kernels and their autograd nodes.
//   out[0..2]  loss_cls, loss_bbox, loss_dir           (head, identity)
//   out[3]     loss_adversarial = 0.01 * (out4 + out5 + out6)
//   out[4..6]  loss_intensity = 3 I, loss_bias = 10 B, loss_imbalance = 10 S
//   out[7]     loss_l2_regularization = reg_coef * mult(l2) * l2
//   out[8]     perturbation_l2_norm = l2 (no gradient)
//   out[9]     total = out0 + out1 + out2 + out3 + out4 + out5 + out6 + out7 (parse_losses order)
//
// Optimizer — mmengine OptimWrapper with clip_grad=dict(max_norm=0.5) and AdamW
// (configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:130-140; paramwise
// lr_mult 2.0 for the adversary): torch.nn.utils.clip_grad_norm_ (global L2 norm, coef =
// max_norm / (norm + 1e-6) clamped to 1) followed by torch's AdamW update (decoupled weight decay,
// bias-corrected moments) — over a table of tensors split into fixed-size chunks (multi-tensor
// apply). Pass 1: per-chunk sums of g^2 in double, reduced in chunk order by the last-arriving
// block (deterministic) -> norm, coef. Pass 2: every chunk applies coef and the AdamW update in
// one read of (p, g, m, v) and one write of (p, m, v), float4-vectorised.
#include <hip/hip_runtime.h>

#include "common.h"

namespace rpc {
namespace tail {

__global__ __launch_bounds__(64) void k_loss_tail_fwd(const float* __restrict__ head, const float* __restrict__ pert,
                                                      float reg_coef, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const float l2 = pert[0];
  const float li = 3.0f * pert[1], lb = 10.0f * pert[2], lm = 10.0f * pert[3];
  const float adv = 0.0f + 0.01f * ((li + lb) + lm);
  const float mult = l2 < 0.001f ? 0.01f : (l2 < 0.005f ? 0.1f : (l2 < 0.01f ? 0.3f : 1.0f));
  const float reg = reg_coef * mult * l2;
  out[0] = head[0];
  out[1] = head[1];
  out[2] = head[2];
  out[3] = adv;
  out[4] = li;
  out[5] = lb;
  out[6] = lm;
  out[7] = reg;
  out[8] = l2;
  out[9] = ((((((head[0] + head[1]) + head[2]) + adv) + li) + lb) + lm) + reg;
}

__global__ __launch_bounds__(64) void k_loss_tail_bwd(const float* __restrict__ pert, float reg_coef,
                                                      const float* __restrict__ g, float* __restrict__ ghead,
                                                      float* __restrict__ gpert) {
  if (threadIdx.x != 0) return;
  const float l2 = pert[0];
  const float mult = l2 < 0.001f ? 0.01f : (l2 < 0.005f ? 0.1f : (l2 < 0.01f ? 0.3f : 1.0f));
  const float gt = g[9];
  for (int k = 0; k < 3; ++k) ghead[k] = g[k] + gt;
  const float gadv = g[3] + gt;  // d total / d adv = 1
  gpert[0] = (reg_coef * mult) * (g[7] + gt);
  gpert[1] = 3.0f * (g[4] + gt + 0.01f * gadv);
  gpert[2] = 10.0f * (g[5] + gt + 0.01f * gadv);
  gpert[3] = 10.0f * (g[6] + gt + 0.01f * gadv);
}

// Loss tail of AdversarialCenterPoint.loss_by_feat_single (plugin detectors/adversarial_centerpoint.py, restating
// models/detectors/adversarial_centerpoint.py:203-257 with the documented l2 fix) + parse_losses, over the CenterHead's
// packed task losses v[n] (task t: heatmap 2t, bbox 2t + 1):
//   det = (0 + w_0) + w_1 + ...,  w_i = isfinite(c_i) ? c_i : 0,  c_i = clamp(v_i, 0, 100) (torch: NaN stays NaN)
//   out[0..n)  v (identity)
//   out[n]     loss_adversarial = det > 0 ? det * negw : 0          (negw = -min(w * epoch / 10, w))
//   out[n+1]   loss_l2_regularization = l2 * rw
//   out[n+2]   perturbation_l2_norm = l2 (no gradient)
//   out[n+3]   total = ((v_0 + v_1 + ... + v_{n-1}) + out[n]) + out[n+1]   (parse_losses, dict order)
// Single lane, the torch composition's fp32 operation order: its values bit for bit, instead of ~60 scalar torch
// kernels forward and ~40 backward.
__device__ __forceinline__ float torch_clamp(float v, float lo, float hi) {
  return v != v ? v : fminf(fmaxf(v, lo), hi);
}
__device__ __forceinline__ float center_det(const float* __restrict__ v, int n) {
  float det = 0.0f;
  for (int i = 0; i < n; ++i) {
    const float c = torch_clamp(v[i], 0.0f, 100.0f);
    det = __fadd_rn(det, isfinite(c) ? c : 0.0f);
  }
  return det;
}
__global__ __launch_bounds__(64) void k_center_tail_fwd(const float* __restrict__ v, int n, const float* __restrict__ l2p,
                                                        float negw, float rw, float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const float det = center_det(v, n);
  const float adv = det > 0.0f ? __fmul_rn(det, negw) : 0.0f;
  const float l2 = *l2p, reg = __fmul_rn(l2, rw);
  float total = n > 0 ? v[0] : 0.0f;
  for (int i = 0; i < n; ++i) out[i] = v[i];
  for (int i = 1; i < n; ++i) total = __fadd_rn(total, v[i]);
  total = __fadd_rn(__fadd_rn(total, adv), reg);
  out[n] = adv;
  out[n + 1] = reg;
  out[n + 2] = l2;
  out[n + 3] = total;
}
__global__ __launch_bounds__(64) void k_center_tail_bwd(const float* __restrict__ v, int n, float negw, float rw,
                                                        const float* __restrict__ g, float* __restrict__ gv,
                                                        float* __restrict__ gl2) {
  const float gt = g[n + 3];
  const float det = center_det(v, n);
  const float ddet = det > 0.0f ? __fmul_rn(__fadd_rn(g[n], gt), negw) : 0.0f;
  for (int i = threadIdx.x; i < n; i += 64) {
    const float c = torch_clamp(v[i], 0.0f, 100.0f);
    const bool pass = isfinite(c) && v[i] >= 0.0f && v[i] <= 100.0f;   // clamp's gradient mask is inclusive
    gv[i] = __fadd_rn(__fadd_rn(g[i], gt), pass ? ddet : 0.0f);
  }
  if (threadIdx.x == 0) *gl2 = __fmul_rn(__fadd_rn(g[n + 1], gt), rw);
}

// ------------------------------------------------------------------ clip_grad_norm_ + AdamW
constexpr int kChunk = RPC_OPTIM_CHUNK;
constexpr int OBLK = 256;

__global__ __launch_bounds__(OBLK) void k_sqnorm(const long long* __restrict__ gptr, const int* __restrict__ numel,
                                                 const int* __restrict__ ctensor, const int* __restrict__ cstart,
                                                 int nchunks, float max_norm, double* __restrict__ part,
                                                 unsigned* __restrict__ ticket, float* __restrict__ out,
                                                 int ntensors, float* __restrict__ steps) {
  __shared__ double sh[OBLK / 64];
  __shared__ int last;
  const int c = blockIdx.x, t = ctensor[c], s0 = cstart[c];
  const int n = min(kChunk, numel[t] - s0);
  const float* g = (const float*)gptr[t];
  double acc = 0.0;
  if (g) {
    g += s0;
    int i0 = 0;
    // four float4 in flight per thread, four partial sums; a gradient view at an odd offset (DDP bucket)
    // is read with scalar loads in the same loop
    const bool gvec = (((uintptr_t)g) & 15) == 0;
    auto ldg4 = [&](int q) -> float4 {
      return gvec ? ((const float4*)g)[q] : make_float4(g[4 * q], g[4 * q + 1], g[4 * q + 2], g[4 * q + 3]);
    };
    {
      const int n4 = n >> 2;
      double a[4] = {0.0, 0.0, 0.0, 0.0};
      int q = threadIdx.x;
      for (; q + 3 * OBLK < n4; q += 4 * OBLK) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = ldg4(q + u * OBLK);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          a[u] += ((double)v[u].x * v[u].x + (double)v[u].y * v[u].y) + ((double)v[u].z * v[u].z + (double)v[u].w * v[u].w);
      }
      for (; q < n4; q += OBLK) {
        const float4 v = ldg4(q);
        a[0] += ((double)v.x * v.x + (double)v.y * v.y) + ((double)v.z * v.z + (double)v.w * v.w);
      }
      acc = (a[0] + a[1]) + (a[2] + a[3]);
      i0 = n4 << 2;
    }
    for (int i = i0 + threadIdx.x; i < n; i += OBLK) {
      const float v = g[i];
      acc += (double)v * (double)v;
    }
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[c] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
  if (!last_block_arrive_2d(ticket, &last, nchunks)) return;
  {
    // the last block: all its threads read the partials (about two each, in flight together), then
    // the four waves are combined in order (was one wave walking ~7 dependent loads per lane)
    double s = 0.0;
    for (int k = threadIdx.x; k < nchunks; k += OBLK) s += part[k];
    s = wave_sum(s);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
  }
  if (threadIdx.x < 64) {
    const double s = ((sh[0] + sh[1]) + sh[2]) + sh[3];
    if (threadIdx.x == 0) {
      const float norm = (float)sqrt(s);
      float coef = 1.0f;
      if (max_norm > 0.0f) {
        coef = max_norm / (norm + 1e-6f);
        coef = coef < 1.0f ? coef : 1.0f;
      }
      out[0] = norm;
      out[1] = coef;
    }
    // optimizer step counters (torch state['step']): only tensors that have a gradient advance
    for (int t = threadIdx.x; t < ntensors; t += 64)
      if (gptr[t]) steps[t] += 1.0f;
  }
}

struct AdamArgs {  // by value as a kernel argument
  RpcAdamWHyper h;
};

__device__ __forceinline__ void adamw1(float& p, float g, float& m, float& v, float lr, float step_size,
                                       float bc2_sqrt, const RpcAdamWHyper& h) {
  p = p - lr * h.weight_decay * p;
  m = h.beta1 * m + (1.0f - h.beta1) * g;
  v = h.beta2 * v + (1.0f - h.beta2) * g * g;
  const float denom = sqrtf(v) / bc2_sqrt + h.eps;
  p = p - step_size * m / denom;
}

__global__ __launch_bounds__(OBLK) void k_adamw(const long long* __restrict__ pptr, const long long* __restrict__ gptr,
                                                const long long* __restrict__ mptr, const long long* __restrict__ vptr,
                                                const int* __restrict__ numel, const int* __restrict__ group,
                                                const int* __restrict__ ctensor, const int* __restrict__ cstart,
                                                AdamArgs a, const float* __restrict__ clip,
                                                const float* __restrict__ steps) {
  const int c = blockIdx.x, t = ctensor[c], s0 = cstart[c];
  const float* g = (const float*)gptr[t];
  if (!g) return;  // parameter without a gradient: untouched (torch skips it)
  const int n = min(kChunk, numel[t] - s0);
  float* p = (float*)pptr[t] + s0;
  float* m = (float*)mptr[t] + s0;
  float* v = (float*)vptr[t] + s0;
  g += s0;
  const float coef = clip ? clip[1] : 1.0f;
  const float lr = a.h.lr[group[t]];
  const float step = steps[t];
  const float step_size = lr / (1.0f - powf(a.h.beta1, step));
  const float bc2_sqrt = sqrtf(1.0f - powf(a.h.beta2, step));
  // p / m / v are 16-byte aligned (the moments' views are padded, optim.py); a gradient that is a view
  // into a DDP bucket at an odd offset is read with scalar loads inside the vector loop
  const bool vec = ((((uintptr_t)p | (uintptr_t)m | (uintptr_t)v) & 15) == 0);
  const bool gvec = (((uintptr_t)g) & 15) == 0;
  auto ldg4 = [&](int q) -> float4 {
    return gvec ? ((const float4*)g)[q] : make_float4(g[4 * q], g[4 * q + 1], g[4 * q + 2], g[4 * q + 3]);
  };
  int i0 = 0;
  if (vec) {
    const int n4 = n >> 2;
    int q = threadIdx.x;
    // four float4 of each operand in flight per thread (a 16384-element chunk is 16 float4 per thread:
    // one load round trip per float4 made the pass latency-bound at ~2.9 TB/s)
    for (; q + 3 * OBLK < n4; q += 4 * OBLK) {
      float4 pp[4], gg[4], mm[4], vv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        pp[u] = ((float4*)p)[q + u * OBLK];
        gg[u] = ldg4(q + u * OBLK);
        mm[u] = ((float4*)m)[q + u * OBLK];
        vv[u] = ((float4*)v)[q + u * OBLK];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        adamw1(pp[u].x, gg[u].x * coef, mm[u].x, vv[u].x, lr, step_size, bc2_sqrt, a.h);
        adamw1(pp[u].y, gg[u].y * coef, mm[u].y, vv[u].y, lr, step_size, bc2_sqrt, a.h);
        adamw1(pp[u].z, gg[u].z * coef, mm[u].z, vv[u].z, lr, step_size, bc2_sqrt, a.h);
        adamw1(pp[u].w, gg[u].w * coef, mm[u].w, vv[u].w, lr, step_size, bc2_sqrt, a.h);
        ((float4*)p)[q + u * OBLK] = pp[u];
        ((float4*)m)[q + u * OBLK] = mm[u];
        ((float4*)v)[q + u * OBLK] = vv[u];
      }
    }
    for (; q < n4; q += OBLK) {
      float4 pp = ((float4*)p)[q], gg = ldg4(q), mm = ((float4*)m)[q], vv = ((float4*)v)[q];
      adamw1(pp.x, gg.x * coef, mm.x, vv.x, lr, step_size, bc2_sqrt, a.h);
      adamw1(pp.y, gg.y * coef, mm.y, vv.y, lr, step_size, bc2_sqrt, a.h);
      adamw1(pp.z, gg.z * coef, mm.z, vv.z, lr, step_size, bc2_sqrt, a.h);
      adamw1(pp.w, gg.w * coef, mm.w, vv.w, lr, step_size, bc2_sqrt, a.h);
      ((float4*)p)[q] = pp;
      ((float4*)m)[q] = mm;
      ((float4*)v)[q] = vv;
    }
    i0 = n4 << 2;
  }
  for (int i = i0 + threadIdx.x; i < n; i += OBLK) {
    float pp = p[i], mm = m[i], vv = v[i];
    adamw1(pp, g[i] * coef, mm, vv, lr, step_size, bc2_sqrt, a.h);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

}  // namespace tail
}  // namespace rpc

using namespace rpc;
using namespace rpc::tail;

extern "C" int rpc_loss_tail_forward(const float* head_losses, const float* pert_losses, float reg_coef, float* out,
                                     void* stream) {
  if (!head_losses || !pert_losses || !out) return RPC_ERR_ARG;
  hipLaunchKernelGGL(k_loss_tail_fwd, dim3(1), dim3(64), 0, (hipStream_t)stream, head_losses, pert_losses, reg_coef,
                     out);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_loss_tail_backward(const float* pert_losses, float reg_coef, const float* grad_out,
                                      float* grad_head, float* grad_pert, void* stream) {
  if (!pert_losses || !grad_out || !grad_head || !grad_pert) return RPC_ERR_ARG;
  hipLaunchKernelGGL(k_loss_tail_bwd, dim3(1), dim3(64), 0, (hipStream_t)stream, pert_losses, reg_coef, grad_out,
                     grad_head, grad_pert);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_center_tail_forward(const float* task_losses, int n, const float* l2, float negw, float rw,
                                       float* out, void* stream) {
  if (!task_losses || !l2 || !out || n < 0 || n > 256) return RPC_ERR_ARG;
  hipLaunchKernelGGL(k_center_tail_fwd, dim3(1), dim3(64), 0, (hipStream_t)stream, task_losses, n, l2, negw, rw, out);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_center_tail_backward(const float* task_losses, int n, float negw, float rw, const float* grad_out,
                                        float* grad_losses, float* grad_l2, void* stream) {
  if (!task_losses || !grad_out || !grad_losses || !grad_l2 || n < 0 || n > 256) return RPC_ERR_ARG;
  hipLaunchKernelGGL(k_center_tail_bwd, dim3(1), dim3(64), 0, (hipStream_t)stream, task_losses, n, negw, rw, grad_out,
                     grad_losses, grad_l2);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" size_t rpc_clip_adamw_workspace_size(int nchunks) {
  return (size_t)(nchunks > 0 ? nchunks : 1) * sizeof(double) + 256;
}

extern "C" int rpc_clip_adamw(const long long* param_ptrs, const long long* grad_ptrs, const long long* exp_avg_ptrs,
                              const long long* exp_avg_sq_ptrs, const int* numel, const int* group,
                              const int* chunk_tensor, const int* chunk_start, int nchunks, int ntensors,
                              float* steps, const RpcAdamWHyper* hyper, float max_norm, float* norm_out,
                              void* workspace, size_t ws_bytes, void* stream) {
  if (!param_ptrs || !grad_ptrs || !exp_avg_ptrs || !exp_avg_sq_ptrs || !numel || !group || !chunk_tensor ||
      !chunk_start || !steps || !hyper || !norm_out || !workspace || nchunks < 0 || ntensors < 0)
    return RPC_ERR_ARG;
  if (ws_bytes < rpc_clip_adamw_workspace_size(nchunks)) return RPC_ERR_WORKSPACE;
  if (nchunks == 0) return RPC_OK;
  hipStream_t st = (hipStream_t)stream;
  double* part = (double*)workspace;
  unsigned* ticket = (unsigned*)((char*)workspace + (size_t)nchunks * sizeof(double));
  RPC_CHECK(hipMemsetAsync(ticket, 0, sizeof(unsigned), st));
  hipLaunchKernelGGL(k_sqnorm, dim3(nchunks), dim3(OBLK), 0, st, grad_ptrs, numel, chunk_tensor, chunk_start, nchunks,
                     max_norm, part, ticket, norm_out, ntensors, steps);
  RPC_LAUNCH_CHECK();
  AdamArgs a{*hyper};
  hipLaunchKernelGGL(k_adamw, dim3(nchunks), dim3(OBLK), 0, st, param_ptrs, grad_ptrs, exp_avg_ptrs, exp_avg_sq_ptrs,
                     numel, group, chunk_tensor, chunk_start, a, (const float*)norm_out, (const float*)steps);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
