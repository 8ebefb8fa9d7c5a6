// §8(f3): CenterHead training targets and losses (AdversarialCenterPoint, BASELINE config 4), gfx950.
//
// Upstream mmdet3d CenterHead.get_targets_single / loss_by_feat (restated in oracle/center_head.py):
//   k_targets   one block per frame: each GT's task slot k (class order within the task, then GT
//               order), gaussian_radius in the reference's float32 op order, centre cell, ind/mask and
//               the 10-value anno box; the draw list for the heatmap
//   k_draw      one block per GT: the float64 gaussian of draw_heatmap_gaussian cast to float32 and
//               max-combined into the target heatmap with an integer atomicMax (values >= 0, so the
//               bit patterns order like the floats; max is order-free -> deterministic)
//   k_focal     clamp_sigmoid + GaussianFocalLoss per heatmap element, per-block per-task partials of
//               the loss sum and of the eq(1) count (num_pos)
//   k_l1        the L1 loss of the boxes gathered at ind, per-block partials; its last-arriving
//               block reduces both partial sets in block order and writes the losses + normalisers
// Backward: k_focal_bwd (every heatmap element) and k_l1_bwd (scatter at the gathered cells).
#include <hip/hip_runtime.h>
#include <math.h>

#include "common.h"

#pragma clang fp contract(off)  // the reference's float32 op order (no fused multiply-adds)

namespace rpc {
namespace ctr {

constexpr int BLK = 256;
constexpr int NBF = 512;   // focal partial rows (max blocks)
constexpr int NBL = 64;    // L1 partial rows (max blocks)
constexpr int MT = RPC_CENTER_MAX_TASKS;

struct WS {
  unsigned* ticket;
  float* tgt;      // [B][H][W][ncls]
  int* ind;        // [B][T][MO]
  int* mask;       // [B][T][MO]
  float* anno;     // [B][T][MO][10]
  int4* draw;      // [B][maxg]: global class (-1 none), cx, cy, radius
  float* pf;       // [NBF][2T]
  float* pl;       // [NBL][2T]
  float* den;      // [2T]: heatmap, bbox denominators
};

static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

static inline size_t carve(const RpcCenterCfg& c, int maxg, char* base, WS* w) {
  const size_t cells = (size_t)c.B * c.H * c.W;
  const size_t slots = (size_t)c.B * c.ntasks * c.max_objs;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    char* p = base ? base + off : nullptr;
    off += al256(bytes);
    return p;
  };
  char* t = take(256);
  char* tg = take(cells * c.ncls_total * sizeof(float));
  char* in = take(slots * sizeof(int));
  char* mk = take(slots * sizeof(int));
  char* an = take(slots * 10 * sizeof(float));
  char* pf = take((size_t)NBF * 2 * MT * sizeof(float));
  char* pl = take((size_t)NBL * 2 * MT * sizeof(float));
  char* dn = take(2 * MT * sizeof(float));
  char* dr = take((size_t)c.B * (maxg > 0 ? maxg : 1) * sizeof(int4));   // last: the only max_gts-sized region
  if (w) *w = WS{(unsigned*)t, (float*)tg, (int*)in, (int*)mk, (float*)an, (int4*)dr, (float*)pf, (float*)pl, (float*)dn};
  return off;
}

__device__ __forceinline__ int task_of(const RpcCenterCfg& c, int g, int* first) {
  int f = 0;
  for (int t = 0; t < c.ntasks; ++t) {
    if (g < f + c.task_ncls[t]) {
      *first = f;
      return t;
    }
    f += c.task_ncls[t];
  }
  *first = f;
  return -1;
}

// gaussian_radius((length, width), min_overlap) in float32 with the python constants rounded once
__device__ float gaussian_radius(float height, float width, double mo) {
  const float k1m = (float)(1.0 - mo), k1p = (float)(1.0 + mo), k4a3 = (float)(4.0 * (4.0 * mo));
  const float km2 = (float)(-2.0 * mo), kmo1 = (float)(mo - 1.0);
  const float b1 = height + width;
  const float c1 = ((width * height) * k1m) / k1p;
  const float sq1 = __fsqrt_rn(b1 * b1 - 4.0f * c1);
  const float r1 = (b1 + sq1) / 2.0f;
  const float b2 = 2.0f * (height + width);
  const float c2 = (k1m * width) * height;
  const float sq2 = __fsqrt_rn(b2 * b2 - 16.0f * c2);
  const float r2 = (b2 + sq2) / 2.0f;
  const float b3 = km2 * (height + width);
  const float c3 = (kmo1 * width) * height;
  const float sq3 = __fsqrt_rn(b3 * b3 - k4a3 * c3);
  const float r3 = (b3 + sq3) / 2.0f;
  float r = r1;
  if (r2 < r) r = r2;
  if (r3 < r) r = r3;
  return r;
}

__global__ __launch_bounds__(BLK) void k_targets(RpcCenterCfg c, const float* __restrict__ boxes,
                                                 const long long* __restrict__ labels, int maxg, WS w) {
  const int b = blockIdx.x, T = c.ntasks, MO = c.max_objs;
  const size_t sb = (size_t)b * T * MO;
  for (int i = threadIdx.x; i < T * MO; i += BLK) {
    w.ind[sb + i] = 0;
    w.mask[sb + i] = 0;
#pragma unroll
    for (int q = 0; q < 10; ++q) w.anno[(sb + i) * 10 + q] = 0.0f;
  }
  for (int m = threadIdx.x; m < maxg; m += BLK) w.draw[(size_t)b * maxg + m] = make_int4(-1, 0, 0, 0);
  __syncthreads();
  const long long* lb = labels + (size_t)b * maxg;
  for (int m = threadIdx.x; m < maxg; m += BLK) {
    const long long l = lb[m];
    if (l < 0 || l >= c.ncls_total) continue;
    int first;
    const int t = task_of(c, (int)l, &first);
    int k = 0;
    for (int j = 0; j < maxg; ++j) {
      const long long lj = lb[j];
      k += (lj >= first && lj < l) || (lj == l && j < m);
    }
    if (k >= MO) continue;
    const float* bx = boxes + ((size_t)b * maxg + m) * 9;
    const float osf = (float)c.out_size_factor;
    const float width = (bx[3] / c.voxel_x) / osf;
    const float length = (bx[4] / c.voxel_y) / osf;
    if (!(width > 0.0f && length > 0.0f)) continue;
    const float rf = gaussian_radius(length, width, c.gaussian_overlap);
    int radius = (int)rf;
    if (radius < c.min_radius) radius = c.min_radius;
    const float coor_x = ((bx[0] - c.pc_x) / c.voxel_x) / osf;
    const float coor_y = ((bx[1] - c.pc_y) / c.voxel_y) / osf;
    const int cx = (int)coor_x, cy = (int)coor_y;
    if (!(cx >= 0 && cx < c.W && cy >= 0 && cy < c.H)) continue;
    const size_t slot = sb + (size_t)t * MO + k;
    w.ind[slot] = cy * c.W + cx;
    w.mask[slot] = 1;
    float* an = w.anno + slot * 10;
    an[0] = coor_x - (float)cx;
    an[1] = coor_y - (float)cy;
    an[2] = bx[2] + bx[5] * 0.5f;                       // gravity centre z
    an[3] = c.norm_bbox ? logf(bx[3]) : bx[3];
    an[4] = c.norm_bbox ? logf(bx[4]) : bx[4];
    an[5] = c.norm_bbox ? logf(bx[5]) : bx[5];
    an[6] = sinf(bx[6]);
    an[7] = cosf(bx[6]);
    an[8] = bx[7];
    an[9] = bx[8];
    w.draw[(size_t)b * maxg + m] = make_int4((int)l, cx, cy, radius);
  }
}

// draw_heatmap_gaussian: gaussian_2d((d, d), sigma = d / 6) in float64, window clipped at the map
__global__ __launch_bounds__(64) void k_draw(RpcCenterCfg c, int maxg, WS w) {
  const int e = blockIdx.x, b = e / maxg;
  const int4 d = w.draw[e];
  if (d.x < 0) return;
  const int r = d.w, x = d.y, y = d.z;
  const int left = min(x, r), right = min(c.W - x, r + 1);
  const int top = min(y, r), bottom = min(c.H - y, r + 1);
  const int nx = left + right, ny = top + bottom;
  const double sigma = (double)(2 * r + 1) / 6.0;
  const double den = 2.0 * sigma * sigma;
  const double thr = 2.220446049250313e-16;   // np.finfo(float64).eps * h.max() (h.max() = 1)
  for (int i = threadIdx.x; i < nx * ny; i += 64) {
    const int iy = i / nx, ix = i - iy * nx;
    const double gy = (double)(iy - top), gx = (double)(ix - left);
    double h = exp(-(gx * gx + gy * gy) / den);
    if (h < thr) h = 0.0;
    const float v = (float)h;
    const int yy = y - top + iy, xx = x - left + ix;
    int* dst = (int*)&w.tgt[(((size_t)b * c.H + yy) * c.W + xx) * c.ncls_total + d.x];
    atomicMax(dst, __float_as_int(v));
  }
}

__device__ __forceinline__ void block_rows(float (*acc)[MT], float* out_row, int T) {
  // acc[2][MT] per thread -> block sums (wave shuffles, then waves in order)
  __shared__ float sh[BLK / 64][2 * MT];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const float v = wave_sum(acc[q][t]);
      if (lane == 0) sh[wv][q * MT + t] = v;
    }
  __syncthreads();
  if (threadIdx.x < 2 * T) {
    const int q = threadIdx.x / T, t = threadIdx.x - q * T;
    float s = 0.0f;
    for (int k = 0; k < BLK / 64; ++k) s += sh[k][q * MT + t];
    out_row[q * T + t] = s;
  }
}

__device__ __forceinline__ float focal_elem(float x, float g, float* dldx) {
  const float s = 1.0f / (1.0f + expf(-x));
  const float lo = 1e-4f, hi = 1.0f - 1e-4f;
  const float p = fminf(fmaxf(s, lo), hi);
  const float eps = 1e-12f;
  const float pos = g == 1.0f ? 1.0f : 0.0f;
  const float omg = 1.0f - g;
  const float negw = powf(omg, 4.0f);
  const float lp = logf(p + eps), ln = logf((1.0f - p) + eps);
  const float loss = (-lp * ((1.0f - p) * (1.0f - p))) * pos + (-ln * (p * p)) * negw;
  if (dldx) {
    const float dpos = -((1.0f - p) * (1.0f - p)) / (p + eps) + 2.0f * (1.0f - p) * lp;
    const float dneg = (p * p) / ((1.0f - p) + eps) - 2.0f * p * ln;
    const float dp = dpos * pos + dneg * negw;
    const bool pass = s >= lo && s <= hi;
    *dldx = pass ? dp * (s * (1.0f - s)) : 0.0f;
  }
  return loss;
}

__global__ __launch_bounds__(BLK) void k_focal(RpcCenterCfg c, const float* __restrict__ hm, WS w) {
  float acc[2][MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[0][t] = acc[1][t] = 0.0f;
  const long long n = (long long)c.B * c.H * c.W * c.ncls_total;
  for (long long e = (long long)blockIdx.x * BLK + threadIdx.x; e < n; e += (long long)gridDim.x * BLK) {
    const long long p = e / c.ncls_total;
    const int g = (int)(e - p * c.ncls_total);
    int first;
    const int tt = task_of(c, g, &first);
    const float tv = w.tgt[e];
    const float l = focal_elem(hm[p * c.hm_pitch + g], tv, nullptr);
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      acc[0][t] += t == tt ? l : 0.0f;
      acc[1][t] += (t == tt && tv == 1.0f) ? 1.0f : 0.0f;
    }
  }
  block_rows(acc, w.pf + (size_t)blockIdx.x * 2 * c.ntasks, c.ntasks);
}

__global__ __launch_bounds__(BLK) void k_l1(RpcCenterCfg c, const float* __restrict__ box, int nbf, WS w,
                                            float* __restrict__ losses) {
  __shared__ int lastf;
  float acc[2][MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[0][t] = acc[1][t] = 0.0f;
  const int T = c.ntasks, MO = c.max_objs;
  const long long n = (long long)c.B * T * MO;
  for (long long e = (long long)blockIdx.x * BLK + threadIdx.x; e < n; e += (long long)gridDim.x * BLK) {
    if (!w.mask[e]) continue;
    const int b = (int)(e / ((long long)T * MO));
    const int tt = (int)((e / MO) % T);
    const size_t cell = (size_t)b * c.H * c.W + w.ind[e];
    const float* pr = box + cell * c.box_pitch + tt * 10;
    const float* an = w.anno + e * 10;
    float s = 0.0f;
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      const float wq = isnan(an[q]) ? 0.0f : c.code_weights[q];
      s += fabsf(pr[q] - an[q]) * wq;
    }
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      acc[0][t] += t == tt ? s : 0.0f;
      acc[1][t] += t == tt ? 1.0f : 0.0f;
    }
  }
  block_rows(acc, w.pl + (size_t)blockIdx.x * 2 * T, T);
  if (!last_block_arrive(w.ticket, &lastf)) return;
  if (threadIdx.x < T) {
    const int t = threadIdx.x;
    double fs = 0.0, fc = 0.0, ls = 0.0, lc = 0.0;
    for (int k = 0; k < nbf; ++k) {
      fs += (double)w.pf[k * 2 * T + t];
      fc += (double)w.pf[k * 2 * T + T + t];
    }
    for (int k = 0; k < (int)gridDim.x; ++k) {
      ls += (double)w.pl[k * 2 * T + t];
      lc += (double)w.pl[k * 2 * T + T + t];
    }
    const double eps = 1.1920928955078125e-07;
    const double avg = fc > 1.0 ? fc : 1.0;                      // max(num_pos, 1)
    const float dh = (float)(avg + eps);
    const float num = (float)lc;
    const float db = (num + 1e-4f) + (float)eps;
    w.den[t] = dh;
    w.den[T + t] = db;
    losses[2 * t] = ((float)fs / dh) * c.loss_cls_weight;
    losses[2 * t + 1] = c.loss_bbox_weight * ((float)ls / db);
  }
}

__global__ __launch_bounds__(BLK) void k_focal_bwd(RpcCenterCfg c, const float* __restrict__ hm,
                                                   const float* __restrict__ gl, WS w, float* __restrict__ dhm) {
  const long long n = (long long)c.B * c.H * c.W * c.ncls_total;
  for (long long e = (long long)blockIdx.x * BLK + threadIdx.x; e < n; e += (long long)gridDim.x * BLK) {
    const long long p = e / c.ncls_total;
    const int g = (int)(e - p * c.ncls_total);
    int first;
    const int t = task_of(c, g, &first);
    float d;
    focal_elem(hm[p * c.hm_pitch + g], w.tgt[e], &d);
    dhm[p * c.hm_pitch + g] = d * ((gl[2 * t] * c.loss_cls_weight) / w.den[t]);
  }
}

__global__ __launch_bounds__(BLK) void k_l1_bwd(RpcCenterCfg c, const float* __restrict__ box,
                                                const float* __restrict__ gl, WS w, float* __restrict__ dbox) {
  const int T = c.ntasks, MO = c.max_objs;
  const long long n = (long long)c.B * T * MO;
  for (long long e = (long long)blockIdx.x * BLK + threadIdx.x; e < n; e += (long long)gridDim.x * BLK) {
    if (!w.mask[e]) continue;
    const int b = (int)(e / ((long long)T * MO));
    const int t = (int)((e / MO) % T);
    const size_t cell = (size_t)b * c.H * c.W + w.ind[e];
    const float* pr = box + cell * c.box_pitch + t * 10;
    const float* an = w.anno + e * 10;
    const float gs = (gl[2 * t + 1] * c.loss_bbox_weight) / w.den[T + t];
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      if (isnan(an[q])) continue;
      const float d = pr[q] - an[q];
      const float sg = d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
      atomicAdd(&dbox[cell * c.box_pitch + t * 10 + q], sg * (c.code_weights[q] * gs));
    }
  }
}

static int check_cfg(const RpcCenterCfg* c) {
  if (!c || c->B < 1 || c->H < 1 || c->W < 1 || c->ntasks < 1 || c->ntasks > MT || c->max_objs < 1) return 0;
  int s = 0;
  for (int t = 0; t < c->ntasks; ++t) {
    if (c->task_ncls[t] < 1) return 0;
    s += c->task_ncls[t];
  }
  if (s != c->ncls_total || c->hm_pitch < c->ncls_total || c->box_pitch < 10 * c->ntasks) return 0;
  if (c->out_size_factor < 1 || !(c->voxel_x > 0.0f) || !(c->voxel_y > 0.0f)) return 0;
  return 1;
}

}  // namespace ctr
}  // namespace rpc

using namespace rpc;
using namespace rpc::ctr;

extern "C" size_t rpc_center_head_workspace_size(const RpcCenterCfg* cfg, int max_gts) {
  if (!check_cfg(cfg)) return 0;
  return carve(*cfg, max_gts, nullptr, nullptr);
}

extern "C" int rpc_center_head_targets(const RpcCenterCfg* cfg, int max_gts, const void* workspace,
                                       const float** heatmap, const int** ind, const int** mask, const float** anno) {
  if (!check_cfg(cfg) || !workspace) return RPC_ERR_ARG;
  WS w;
  carve(*cfg, max_gts, (char*)workspace, &w);
  if (heatmap) *heatmap = w.tgt;
  if (ind) *ind = w.ind;
  if (mask) *mask = w.mask;
  if (anno) *anno = w.anno;
  return RPC_OK;
}

extern "C" int rpc_center_head_loss_forward(const RpcCenterCfg* cfg, const float* gt_boxes,
                                            const long long* gt_labels, int max_gts, const float* hm,
                                            const float* box, float* losses, void* workspace, size_t ws_bytes,
                                            void* stream) {
  if (!check_cfg(cfg) || max_gts < 0 || !hm || !box || !losses || !workspace) return RPC_ERR_ARG;
  if (max_gts > 0 && (!gt_boxes || !gt_labels)) return RPC_ERR_ARG;
  const RpcCenterCfg& c = *cfg;
  if (ws_bytes < carve(c, max_gts, nullptr, nullptr)) return RPC_ERR_WORKSPACE;
  WS w;
  carve(c, max_gts, (char*)workspace, &w);
  hipStream_t st = (hipStream_t)stream;
  // ticket + target heatmap are contiguous from the workspace start
  RPC_CHECK(hipMemsetAsync(workspace, 0, (size_t)((char*)w.ind - (char*)workspace), st));
  hipLaunchKernelGGL(k_targets, dim3(c.B), dim3(BLK), 0, st, c, gt_boxes, gt_labels, max_gts, w);
  if (max_gts > 0) hipLaunchKernelGGL(k_draw, dim3(c.B * max_gts), dim3(64), 0, st, c, max_gts, w);
  const long long n = (long long)c.B * c.H * c.W * c.ncls_total;
  const int nbf = grid_for(n, BLK * 4, NBF);
  hipLaunchKernelGGL(k_focal, dim3(nbf), dim3(BLK), 0, st, c, hm, w);
  const int nbl = grid_for((long long)c.B * c.ntasks * c.max_objs, BLK, NBL);
  hipLaunchKernelGGL(k_l1, dim3(nbl), dim3(BLK), 0, st, c, box, nbf, w, losses);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_center_head_loss_backward(const RpcCenterCfg* cfg, const float* hm, const float* box,
                                             const float* grad_losses, float* dhm, float* dbox, void* workspace,
                                             size_t ws_bytes, void* stream) {
  if (!check_cfg(cfg) || !hm || !box || !grad_losses || !dhm || !dbox || !workspace) return RPC_ERR_ARG;
  const RpcCenterCfg& c = *cfg;
  if (ws_bytes < carve(c, 0, nullptr, nullptr)) return RPC_ERR_WORKSPACE;
  WS w;
  carve(c, 0, (char*)workspace, &w);   // the draw list (last region) is not read by the backward
  hipStream_t st = (hipStream_t)stream;
  const long long cells = (long long)c.B * c.H * c.W;
  const long long n = cells * c.ncls_total;
  hipLaunchKernelGGL(k_focal_bwd, dim3(grid_for(n, BLK, 2048)), dim3(BLK), 0, st, c, hm, grad_losses, w, dhm);
  RPC_CHECK(hipMemsetAsync(dbox, 0, (size_t)cells * c.box_pitch * sizeof(float), st));
  hipLaunchKernelGGL(k_l1_bwd, dim3(grid_for((long long)c.B * c.ntasks * c.max_objs, BLK, NBL)), dim3(BLK), 0, st, c,
                     box, grad_losses, w, dbox);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

// ------------------------------------------------------------------ head output packing
// The final 3x3 convolutions of the task heads run on the dense engine with their outputs padded to
// 64 channels (bf16 z); their bias is added here while the n real channels are packed into the fp32
// head buffers the loss reads (hm / box at a channel offset). Backward: the fp32 gradient slice
// becomes the bf16 dz image (padding channels zero) and dbias (fixed-order two-level sums).
namespace rpc {
namespace ctr {
constexpr int PACK_NB = 256;

// F32: fp32 z / dz images (parity mode), else bf16
template <bool F32>
__global__ __launch_bounds__(BLK) void k_pack(const void* __restrict__ zv, int zp, int n,
                                              const float* __restrict__ bias, float* __restrict__ out, int op,
                                              int ooff, long long cells) {
  const long long e = (long long)blockIdx.x * BLK + threadIdx.x;
  if (e >= cells * n) return;
  const long long p = e / n;
  const int c = (int)(e - p * n);
  const float v = F32 ? ((const float*)zv)[p * zp + c]
                      : __uint_as_float((unsigned)((const unsigned short*)zv)[p * zp + c] << 16);
  out[p * op + ooff + c] = v + bias[c];
}

template <bool F32>
__global__ __launch_bounds__(BLK) void k_unpack(const float* __restrict__ d, int dp, int doff, int n,
                                                void* __restrict__ dzv, int zp, long long cells,
                                                float* __restrict__ part) {
  __shared__ float sh[BLK / 64][16];
  const long long per = (cells + gridDim.x - 1) / gridDim.x;
  const long long p0 = (long long)blockIdx.x * per, p1 = min(cells, p0 + per);
  float acc[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) acc[c] = 0.0f;
  for (long long p = p0 + threadIdx.x; p < p1; p += BLK) {
    for (int c = 0; c < zp; c += 8) {
      if (F32) {
        float v[8];
#pragma unroll
        for (int h = 0; h < 8; ++h) v[h] = c + h < n ? d[p * dp + doff + c + h] : 0.0f;
        float4* o = (float4*)((float*)dzv + p * zp + c);
        o[0] = make_float4(v[0], v[1], v[2], v[3]);
        o[1] = make_float4(v[4], v[5], v[6], v[7]);
        continue;
      }
      unsigned w[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const int c0 = c + 2 * h;
        const float a = c0 < n ? d[p * dp + doff + c0] : 0.0f;
        const float b = c0 + 1 < n ? d[p * dp + doff + c0 + 1] : 0.0f;
        w[h] = (unsigned)__builtin_bit_cast(unsigned short, (__bf16)a) |
               ((unsigned)__builtin_bit_cast(unsigned short, (__bf16)b) << 16);
      }
      *(uint4*)((unsigned short*)dzv + p * zp + c) = make_uint4(w[0], w[1], w[2], w[3]);
    }
#pragma unroll
    for (int c = 0; c < 16; ++c)
      if (c < n) acc[c] += d[p * dp + doff + c];
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    const float v = wave_sum(acc[c]);
    if (lane == 0) sh[wv][c] = v;
  }
  __syncthreads();
  if (threadIdx.x < n) {
    float s = 0.0f;
    for (int k = 0; k < BLK / 64; ++k) s += sh[k][threadIdx.x];
    part[(size_t)blockIdx.x * n + threadIdx.x] = s;
  }
}
static int head_pack(bool f32, const void* z, int zp, int n, const float* bias, float* out, int op, int ooff,
                     long long cells, void* stream) {
  if (!z || !bias || !out || n < 1 || n > 16 || zp < n || op < ooff + n || cells < 0) return RPC_ERR_ARG;
  if (cells == 0) return RPC_OK;
  const dim3 grid((unsigned)((cells * n + BLK - 1) / BLK));
  if (f32)
    hipLaunchKernelGGL(k_pack<true>, grid, dim3(BLK), 0, (hipStream_t)stream, z, zp, n, bias, out, op, ooff, cells);
  else
    hipLaunchKernelGGL(k_pack<false>, grid, dim3(BLK), 0, (hipStream_t)stream, z, zp, n, bias, out, op, ooff, cells);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

static int head_unpack(bool f32, const float* dout, int dp, int doff, int n, void* dz, int zp, long long cells,
                       float* dbias, void* workspace, size_t ws_bytes, void* stream) {
  if (!dout || !dz || !dbias || !workspace || n < 1 || n > 16 || zp < n || (zp & 7) || dp < doff + n || cells < 1)
    return RPC_ERR_ARG;
  if (ws_bytes < (size_t)PACK_NB * 16 * sizeof(float)) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int nb = (int)(cells < PACK_NB * 64 ? (cells + 63) / 64 : PACK_NB);
  if (f32)
    hipLaunchKernelGGL(k_unpack<true>, dim3(nb), dim3(BLK), 0, st, dout, dp, doff, n, dz, zp, cells, (float*)workspace);
  else
    hipLaunchKernelGGL(k_unpack<false>, dim3(nb), dim3(BLK), 0, st, dout, dp, doff, n, dz, zp, cells,
                       (float*)workspace);
  RPC_LAUNCH_CHECK();
  slab_reduce((const float*)workspace, nb, n, dbias, st);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
}  // namespace ctr
}  // namespace rpc

extern "C" int rpc_head_pack(const void* z, int zp, int n, const float* bias, float* out, int op, int ooff,
                             long long cells, void* stream) {
  return head_pack(false, z, zp, n, bias, out, op, ooff, cells, stream);
}

extern "C" int rpc_head_pack_f32(const float* z, int zp, int n, const float* bias, float* out, int op, int ooff,
                                 long long cells, void* stream) {
  return head_pack(true, z, zp, n, bias, out, op, ooff, cells, stream);
}

extern "C" size_t rpc_head_unpack_workspace_size(void) { return (size_t)PACK_NB * 16 * sizeof(float); }

extern "C" int rpc_head_unpack_grad(const float* dout, int dp, int doff, int n, void* dz, int zp, long long cells,
                                    float* dbias, void* workspace, size_t ws_bytes, void* stream) {
  return head_unpack(false, dout, dp, doff, n, dz, zp, cells, dbias, workspace, ws_bytes, stream);
}

extern "C" int rpc_head_unpack_grad_f32(const float* dout, int dp, int doff, int n, float* dz, int zp,
                                        long long cells, float* dbias, void* workspace, size_t ws_bytes,
                                        void* stream) {
  return head_unpack(true, dout, dp, doff, n, dz, zp, cells, dbias, workspace, ws_bytes, stream);
}
