// §8(f1) / row a8: Anchor3DHead training targets and losses on the GPU, for gfx950.
//
// Restates upstream mmdet3d v1.x `Anchor3DHead.loss_by_feat` with `AnchorTrainMixin.anchor_target_3d`
// (Max3DIoUAssigner = mmdet MaxIoUAssigner over BboxOverlapsNearest3D, sampling-free), mmcv
// `sigmoid_focal_loss` (forward and analytic backward of its CUDA kernel), mmdet `SmoothL1Loss` with
// `add_sin_difference`, `get_direction_target` + `CrossEntropyLoss`, as configured at
// configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:38-69 (head), :86-112
// (assigners) and …-kitti-3d-car.py:18-39, called from models/detectors/adversarial_voxelnet.py:168.
//
// Four kernels, no host synchronisation:
//   k_gt_prep   nearest-BEV box + area of every ground truth box
//   k_gt_max    max IoU of every GT over the anchors of its assigner (MaxIoUAssigner's
//               gt_max_overlaps), wave max -> LDS -> one atomicMax per (block, GT); IoU >= 0 so the
//               float bits order as unsigned and the max is order-independent (deterministic)
//   k_loss_fwd  one thread per BEV location, all its anchors: assignment (pos / neg / ignore, low-
//               quality matches, later GTs overwrite), focal / SmoothL1 / direction-CE sums in double,
//               the assignment per anchor kept for the backward; per-frame positive counts by integer
//               atomics, per-block partial sums reduced in block order by the last-arriving block
//               (num_total_pos = sum_b max(pos_b, 1), loss = sum / (num_total_pos + eps) * weight)
//   k_loss_bwd  the analytic gradient of the three losses w.r.t. the head's raw outputs, scaled by
//               the upstream gradients and 1 / (num_total_pos + eps), plus per-block bias-gradient
//               partials (fixed-order slab reduce)
// The head conv outputs are read through (frame, location, channel) strides, so the same kernels
// serve the bf16 NHWC image of the HIP 1x1 GEMM (perf mode) and torch's fp32 NCHW conv output.
// Element-wise arithmetic is compiled without FMA contraction: the IoU / threshold comparisons
// are bit-identical to the CPU restatement (oracle/anchor_head.py) on the same anchors.
#include <hip/hip_runtime.h>

#include "common.h"

#pragma clang fp contract(off)

namespace rpc {
namespace head {

constexpr int BLK = 256;
constexpr float kFltMin = 1.1754943508222875e-38f;
constexpr float kEps = 1.1920928955078125e-07f;  // torch.finfo(float32).eps
constexpr float kPi = 3.14159265358979323846f;
constexpr int kMaxA = 8;  // anchors per location a k_gt_max thread keeps in registers

__device__ __forceinline__ float limit_period(float v, float off, float period) {
  return v - floorf(v / period + off) * period;
}

// BaseInstance3DBoxes.nearest_bev of (x, y, dx, dy, yaw): x1, y1, x2, y2
__device__ __forceinline__ void nearest_bev(float x, float y, float dx, float dy, float yaw, float* o) {
  const float nr = fabsf(limit_period(yaw, 0.5f, kPi));
  if (nr > kPi / 4.0f) {
    const float t = dx;
    dx = dy;
    dy = t;
  }
  o[0] = x - dx / 2.0f;
  o[1] = y - dy / 2.0f;
  o[2] = x + dx / 2.0f;
  o[3] = y + dy / 2.0f;
}

// mmdet bbox_overlaps(mode='iou', eps=1e-6) of gt g (x1,y1,x2,y2,area) and anchor a
__device__ __forceinline__ float iou(const float* g, const float* a, float area_a) {
  const float lx = fmaxf(g[0], a[0]), ly = fmaxf(g[1], a[1]);
  const float rx = fminf(g[2], a[2]), ry = fminf(g[3], a[3]);
  const float w = fmaxf(rx - lx, 0.0f), h = fmaxf(ry - ly, 0.0f);
  const float ov = w * h;
  const float un = fmaxf(g[4] + area_a - ov, 1e-6f);
  return ov / un;
}

// anchor a = s * R + r at BEV cell (h, w): (x, y, z, dx, dy, dz, yaw) from the generator's tables
__device__ __forceinline__ void anchor_box(const RpcHeadCfg& c, const float* tab, int h, int w, int s, int r,
                                           float* o) {
  const float* xc = tab;
  const float* yc = xc + c.S * c.W;
  const float* zc = yc + c.S * c.H;
  const float* sz = zc + c.S;
  const float* rot = sz + 3 * c.S;
  o[0] = xc[s * c.W + w];
  o[1] = yc[s * c.H + h];
  o[2] = zc[s];
  o[3] = sz[3 * s];
  o[4] = sz[3 * s + 1];
  o[5] = sz[3 * s + 2];
  o[6] = rot[r];
}

__device__ __forceinline__ int assigner_of(const RpcHeadCfg& c, int s) { return c.assigner_per_size ? s : 0; }

// gt j takes part in assigner i
__device__ __forceinline__ bool gt_in(const RpcHeadCfg& c, const float* gtb, int i) {
  const int lab = (int)gtb[5];
  return lab >= 0 && (!c.assign_per_class || lab == i);
}

__device__ __forceinline__ float load_z(const void* z, int bf16, long long off) {
  if (bf16) return __uint_as_float((unsigned)((const unsigned short*)z)[off] << 16);
  return ((const float*)z)[off];
}

__device__ __forceinline__ void store_z(void* z, int bf16, long long off, float v) {
  if (bf16)
    ((unsigned short*)z)[off] = __builtin_bit_cast(unsigned short, (__bf16)v);
  else
    ((float*)z)[off] = v;
}

// Head outputs of one thread's BEV cell: strided loads (any layout), or — for bf16 NHWC images
// (channel stride 1) — a row of an LDS tile holding the block's BLK consecutive cells, filled and
// drained with 16-byte coalesced accesses (the cells of a block are contiguous rows in HBM).
template <bool kTile>
struct ZRow {
  const void* z;
  int bf16;
  long long base, sn;
  unsigned short* t;
  __device__ __forceinline__ float get(int ch) const {
    if (kTile) return __uint_as_float((unsigned)t[ch] << 16);
    return load_z(z, bf16, base + (long long)ch * sn);
  }
};

// rows [loc0, loc0 + nrows) of frame b, channels [0, 8*nc8): image -> tile (pitch tp elements)
__device__ __forceinline__ void tile_load(unsigned short* tile, int tp, const void* z, long long sb, long long shw,
                                          int b, int loc0, int nrows, int nc8) {
  const unsigned short* src = (const unsigned short*)z + (long long)b * sb + (long long)loc0 * shw;
  for (int q = threadIdx.x; q < nrows * nc8; q += BLK) {
    const int r = q / nc8, c8 = q - r * nc8;
    *(uint4*)&tile[r * tp + 8 * c8] = *(const uint4*)(src + (long long)r * shw + 8 * c8);
  }
}

__device__ __forceinline__ void tile_store(const unsigned short* tile, int tp, void* dz, long long sb, long long shw,
                                           int b, int loc0, int nrows, int nc8) {
  unsigned short* dst = (unsigned short*)dz + (long long)b * sb + (long long)loc0 * shw;
  for (int q = threadIdx.x; q < nrows * nc8; q += BLK) {
    const int r = q / nc8, c8 = q - r * nc8;
    *(uint4*)(dst + (long long)r * shw + 8 * c8) = *(const uint4*)&tile[r * tp + 8 * c8];
  }
}

// ------------------------------------------------------------------ GT preparation
// gtb[b][j] = x1, y1, x2, y2, area, label (label -1: padding)
__global__ __launch_bounds__(64) void k_gt_prep(const float* __restrict__ boxes, const long long* __restrict__ labels,
                                                int M, float* __restrict__ gtb) {
  const int b = blockIdx.x;
  for (int j = threadIdx.x; j < M; j += 64) {
    const float* bx = boxes + ((long long)b * M + j) * 7;
    float o[4];
    nearest_bev(bx[0], bx[1], bx[3], bx[4], bx[6], o);
    float* g = gtb + ((long long)b * M + j) * 8;
    g[0] = o[0];
    g[1] = o[1];
    g[2] = o[2];
    g[3] = o[3];
    g[4] = (o[2] - o[0]) * (o[3] - o[1]);
    g[5] = (float)labels[(long long)b * M + j];
    g[6] = 0.0f;
    g[7] = 0.0f;
  }
}

// ------------------------------------------------------------------ per-GT max IoU
// grid (cdiv(H*W, BLK), NA, B); gmax[b][i][j] (float bits, zero-initialised by the launcher)
__global__ __launch_bounds__(BLK) void k_gt_max(RpcHeadCfg c, const float* __restrict__ tab,
                                                const float* __restrict__ gtb, int M, unsigned* __restrict__ gmax) {
  extern __shared__ float wmax[];  // [4][M]
  const int HW = c.H * c.W;
  const int loc = blockIdx.x * BLK + threadIdx.x, i = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int s0 = c.assigner_per_size ? i : 0, s1 = c.assigner_per_size ? i + 1 : c.S;
  // the assigner's anchors of this cell, statically indexed (registers, no scratch)
  const int na = loc < HW ? (s1 - s0) * c.R : 0;
  float bev[kMaxA][5];
  {
    const int h = loc < HW ? loc / c.W : 0, w = loc < HW ? loc - h * c.W : 0;
#pragma unroll
    for (int k = 0; k < kMaxA; ++k) {
      if (k < na) {
        float a[7];
        anchor_box(c, tab, h, w, s0 + k / c.R, k % c.R, a);
        nearest_bev(a[0], a[1], a[3], a[4], a[6], bev[k]);
        bev[k][4] = (bev[k][2] - bev[k][0]) * (bev[k][3] - bev[k][1]);
      }
    }
  }
  const float* G = gtb + (long long)b * M * 8;
  for (int j = 0; j < M; ++j) {
    float m = -1.0f;
    if (gt_in(c, G + 8 * j, i)) {
#pragma unroll
      for (int k = 0; k < kMaxA; ++k)
        if (k < na) m = fmaxf(m, iou(G + 8 * j, bev[k], bev[k][4]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) wmax[wv * M + j] = m;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < M; j += BLK) {
    const float m = fmaxf(fmaxf(wmax[j], wmax[M + j]), fmaxf(wmax[2 * M + j], wmax[3 * M + j]));
    if (m >= 0.0f) atomicMax(&gmax[((long long)b * c.NA + i) * M + j], __float_as_uint(m));
  }
}

// MaxIoUAssigner.assign_wrt_overlaps for one anchor: -1 ignore, 0 negative, j+1 positive for gt j
__device__ __forceinline__ int assign(const RpcHeadCfg& c, const float* G, int M, const unsigned* gm, int i,
                                      const float* bev, float area) {
  float best = -1.0f;
  int arg = -1, lowq = -1;
  bool any = false;
  for (int j = 0; j < M; ++j) {
    if (!gt_in(c, G + 8 * j, i)) continue;
    any = true;
    const float v = iou(G + 8 * j, bev, area);
    if (v > best) {
      best = v;
      arg = j;
    }
    const float g = __uint_as_float(gm[j]);
    if (g >= c.min_pos_iou[i] && v == g) lowq = j;
  }
  if (!any) return 0;
  int a = -1;
  if (best >= 0.0f && best < c.neg_iou_thr[i]) a = 0;
  if (best >= c.pos_iou_thr[i]) a = arg + 1;
  if (lowq >= 0) a = lowq + 1;
  return a;
}

// DeltaXYZWLHRBBoxCoder.encode(anchor, gt)
__device__ __forceinline__ void encode(const float* a, const float* g, float* t) {
  const float za = a[2] + a[5] / 2.0f, zg = g[2] + g[5] / 2.0f;
  const float diag = sqrtf(a[4] * a[4] + a[3] * a[3]);
  t[0] = (g[0] - a[0]) / diag;
  t[1] = (g[1] - a[1]) / diag;
  t[2] = (zg - za) / a[5];
  t[3] = logf(g[3] / a[3]);
  t[4] = logf(g[4] / a[4]);
  t[5] = logf(g[5] / a[5]);
  t[6] = g[6] - a[6];
}

__device__ __forceinline__ int dir_target(const RpcHeadCfg& c, float t6, float a6) {
  const float rot = t6 + a6;
  const float off = limit_period(rot - c.dir_offset, c.dir_limit_offset, 2.0f * kPi);
  int d = (int)floorf(off / kPi);
  return d < 0 ? 0 : (d > 1 ? 1 : d);
}

// focal-loss modulating factor: the configs' gamma = 2 as one product (pow of ocml is ~100 instructions)
__device__ __forceinline__ float pow_gamma(float x, float gamma) { return gamma == 2.0f ? x * x : powf(x, gamma); }

__device__ __forceinline__ float smooth_l1(float d, float beta) {
  const float a = fabsf(d);
  return a < beta ? 0.5f * a * a / beta : a - 0.5f * beta;
}

__device__ __forceinline__ float smooth_l1_grad(float d, float beta) {
  const float a = fabsf(d);
  if (a < beta) return d / beta;
  return d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f);
}

struct Loc {
  int b, loc, h, w;
  long long zbase;
};

__device__ __forceinline__ Loc locate(const RpcHeadCfg& c, int b, int loc) {
  Loc l;
  l.b = b;
  l.loc = loc;
  l.h = loc / c.W;
  l.w = loc - l.h * c.W;
  l.zbase = (long long)b * c.z_sb + (long long)loc * c.z_shw;
  return l;
}

// ------------------------------------------------------------------ forward: assignment + loss sums
// grid (cdiv(H*W, BLK), B). part[blk] = (cls, bbox, dir) double; cnt[b] positives; ticket; out[4]
template <bool kTile>
__global__ __launch_bounds__(BLK) void k_loss_fwd(RpcHeadCfg c, const float* __restrict__ tab,
                                                  const float* __restrict__ gtb, const float* __restrict__ boxes, int M,
                                                  const unsigned* __restrict__ gmax, const void* __restrict__ z,
                                                  const float* __restrict__ bias, int* __restrict__ asg,
                                                  double* __restrict__ part, int* __restrict__ cnt,
                                                  unsigned* __restrict__ ticket, float* __restrict__ out) {
  __shared__ double sred[3][4];
  __shared__ int spos[4];
  __shared__ int last_flag;
  const int HW = c.H * c.W, A = c.S * c.R, C = c.C;
  const int loc = blockIdx.x * BLK + threadIdx.x, b = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nblk = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
  double lc = 0.0, lb = 0.0, ld = 0.0;
  int npos = 0;
  extern __shared__ __attribute__((aligned(16))) unsigned short ztile[];
  const int N = A * (C + 7 + (c.use_dir ? 2 : 0)), nc8 = (N + 7) / 8, tp = 8 * nc8;
  const int loc0 = blockIdx.x * BLK, nrows = min(BLK, HW - loc0);
  if (kTile) {
    tile_load(ztile, tp, z, c.z_sb, c.z_shw, b, loc0, nrows, nc8);
    __syncthreads();
  }
  if (loc < HW) {
    const Loc L = locate(c, b, loc);
    const ZRow<kTile> zr{z, c.z_bf16, L.zbase, c.z_sn, ztile + threadIdx.x * tp};
    const float* G = gtb + (long long)b * M * 8;
    const int reg0 = A * C, dir0 = A * C + A * 7;
    for (int a = 0; a < A; ++a) {
      const int s = a / c.R, r = a - s * c.R, i = assigner_of(c, s);
      float an[7], bev[4];
      anchor_box(c, tab, L.h, L.w, s, r, an);
      nearest_bev(an[0], an[1], an[3], an[4], an[6], bev);
      const float area = (bev[2] - bev[0]) * (bev[3] - bev[1]);
      const int g = assign(c, G, M, gmax + ((long long)b * c.NA + i) * M, i, bev, area);
      asg[((long long)b * HW + loc) * A + a] = g;
      const bool pos = g > 0;
      const float lw = pos ? (c.pos_weight > 0.0f ? c.pos_weight : 1.0f) : (g == 0 ? 1.0f : 0.0f);
      const int label = pos ? (int)G[8 * (g - 1) + 5] : C;
      float fc = 0.0f;
      for (int k = 0; k < C; ++k) {
        const int ch = a * C + k;
        const float x = zr.get(ch) + (bias ? bias[ch] : 0.0f);
        const float p = 1.0f / (1.0f + expf(-x));
        float f;
        if (label == k)
          f = -c.alpha * pow_gamma(1.0f - p, c.gamma) * logf(fmaxf(p, kFltMin));
        else
          f = -(1.0f - c.alpha) * pow_gamma(p, c.gamma) * logf(fmaxf(1.0f - p, kFltMin));
        fc += f * lw;
      }
      lc += (double)fc;
      if (pos) {
        ++npos;
        float t[7], pr[7];
        encode(an, boxes + ((long long)b * M + (g - 1)) * 7, t);
        for (int k = 0; k < 7; ++k) {
          const int ch = reg0 + a * 7 + k;
          pr[k] = zr.get(ch) + (bias ? bias[ch] : 0.0f);
        }
        float sb = 0.0f;
        for (int k = 0; k < 7; ++k) {
          float p = pr[k], q = t[k];
          if (k == 6 && c.diff_rad_by_sin) {
            p = sinf(pr[6]) * cosf(t[6]);
            q = cosf(pr[6]) * sinf(t[6]);
          }
          sb += smooth_l1(p - q, c.beta);
        }
        lb += (double)sb;
        if (c.use_dir) {
          const int dt = dir_target(c, t[6], an[6]);
          float d[2];
          for (int k = 0; k < 2; ++k) {
            const int ch = dir0 + a * 2 + k;
            d[k] = zr.get(ch) + (bias ? bias[ch] : 0.0f);
          }
          const float m = fmaxf(d[0], d[1]);
          const float lse = logf(expf(d[0] - m) + expf(d[1] - m));
          ld += (double)(lse - (d[dt] - m));
        }
      }
    }
  }
  lc = wave_sum(lc);
  lb = wave_sum(lb);
  ld = wave_sum(ld);
  int np = npos;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) np += __shfl_xor(np, o, 64);
  if (lane == 0) {
    sred[0][wv] = lc;
    sred[1][wv] = lb;
    sred[2][wv] = ld;
    spos[wv] = np;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 0; q < 3; ++q) part[(long long)bid * 3 + q] = ((sred[q][0] + sred[q][1]) + sred[q][2]) + sred[q][3];
    const int bp = ((spos[0] + spos[1]) + spos[2]) + spos[3];
    if (bp) atomicAdd(&cnt[b], bp);
  }
  if (!last_block_arrive_2d(ticket, &last_flag, nblk)) return;
  // last block: fixed-order reduction of the partials
  if (threadIdx.x < 64) {
    double s[3] = {0.0, 0.0, 0.0};
    for (int k = threadIdx.x; k < nblk; k += 64)
      for (int q = 0; q < 3; ++q) s[q] += part[(long long)k * 3 + q];
    for (int q = 0; q < 3; ++q) s[q] = wave_sum(s[q]);
    if (threadIdx.x == 0) {
      float np_tot = 0.0f;
      for (int k = 0; k < c.B; ++k) np_tot += (float)(cnt[k] > 1 ? cnt[k] : 1);
      const float den = np_tot + kEps;
      out[0] = (float)s[0] / den * c.lw_cls;
      out[1] = (float)s[1] / den * c.lw_bbox;
      out[2] = c.use_dir ? (float)s[2] / den * c.lw_dir : 0.0f;
      out[3] = np_tot;
    }
  }
}

// ------------------------------------------------------------------ backward: d loss / d head outputs
// g[3] = upstream gradients of (loss_cls, loss_bbox, loss_dir); stats[3] = num_total_pos.
// dz written through the dz strides (c.dz_*), channels [N, n_write) zeroed; bias partials [nblk][N].
template <bool kTile>
__global__ __launch_bounds__(BLK) void k_loss_bwd(RpcHeadCfg c, const float* __restrict__ tab,
                                                  const float* __restrict__ gtb, const float* __restrict__ boxes, int M,
                                                  const void* __restrict__ z, const float* __restrict__ bias,
                                                  const int* __restrict__ asg, const float* __restrict__ g,
                                                  const float* __restrict__ stats, void* __restrict__ dz,
                                                  float* __restrict__ bpart) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int HW = c.H * c.W, A = c.S * c.R, C = c.C;
  const int N = A * (C + 7 + (c.use_dir ? 2 : 0));
  float* sb = (float*)smem;  // [4][N] per-wave bias-gradient sums
  unsigned short* ztile = (unsigned short*)(smem + ((4 * N * sizeof(float) + 15) & ~15));
  // the LDS tile holds the N computed channels (rounded to 16-byte granules): at 72 channels x 256 cells
  // that is 37 KB and four blocks share a CU, so the 828-block grid runs in one round (the 128-wide
  // zero-padded tile of 70 KB ran 1.6 rounds); channels [8*nc8, n_write) are zero-stored directly
  const int nc8 = (N + 7) / 8, nw8 = c.dz_nwrite / 8, tp = 8 * nc8;
  const int loc0 = blockIdx.x * BLK, nrows = min(BLK, HW - loc0);
  const int loc = blockIdx.x * BLK + threadIdx.x, b = blockIdx.y;
  if (kTile) {
    tile_load(ztile, tp, z, c.z_sb, c.z_shw, b, loc0, nrows, nc8);
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int bid = blockIdx.y * gridDim.x + blockIdx.x;
  const bool live = loc < HW;
  const float den = stats[3] + kEps;
  const float s_cls = g[0] * c.lw_cls / den, s_box = g[1] * c.lw_bbox / den, s_dir = g[2] * c.lw_dir / den;
  const Loc L = locate(c, b, live ? loc : 0);
  const long long dbase = (long long)b * c.dz_sb + (long long)(live ? loc : 0) * c.dz_shw;
  unsigned short* trow = ztile + threadIdx.x * tp;
  const ZRow<kTile> zr{z, c.z_bf16, L.zbase, c.z_sn, trow};
  // dz of this cell: into the tile row (written out coalesced at the end) or strided stores
  auto put = [&](int ch, float v) {
    if (kTile)
      trow[ch] = __builtin_bit_cast(unsigned short, (__bf16)v);
    else
      store_z(dz, c.dz_bf16, dbase + (long long)ch * c.dz_sn, v);
  };
  const float* G = gtb + (long long)b * M * 8;
  const int reg0 = A * C, dir0 = A * C + A * 7;
  for (int a = 0; a < A; ++a) {
    const int s = a / c.R, r = a - s * c.R;
    const int gi = live ? asg[((long long)b * HW + loc) * A + a] : -1;
    const bool pos = gi > 0;
    const float lw = pos ? (c.pos_weight > 0.0f ? c.pos_weight : 1.0f) : (gi == 0 ? 1.0f : 0.0f);
    const int label = pos ? (int)G[8 * (gi - 1) + 5] : C;
    for (int k = 0; k < C; ++k) {
      const int ch = a * C + k;
      float d = 0.0f;
      if (live) {
        const float x = zr.get(ch) + (bias ? bias[ch] : 0.0f);
        const float p = 1.0f / (1.0f + expf(-x));
        float gr;
        if (label == k)
          gr = -c.alpha * pow_gamma(1.0f - p, c.gamma) * (1.0f - p - c.gamma * p * logf(fmaxf(p, kFltMin)));
        else
          gr = -(1.0f - c.alpha) * pow_gamma(p, c.gamma) * (c.gamma * (1.0f - p) * logf(fmaxf(1.0f - p, kFltMin)) - p);
        d = gr * lw * s_cls;
        put(ch, d);
      }
      const float t = wave_sum(d);
      if (lane == 0) sb[wv * N + ch] = t;
    }
    float an[7], tg[7], pr[7], dr[7] = {0, 0, 0, 0, 0, 0, 0}, dd[2] = {0.0f, 0.0f};
    if (live && pos) {
      anchor_box(c, tab, L.h, L.w, s, r, an);
      encode(an, boxes + ((long long)b * M + (gi - 1)) * 7, tg);
      for (int k = 0; k < 7; ++k) {
        const int ch = reg0 + a * 7 + k;
        pr[k] = zr.get(ch) + (bias ? bias[ch] : 0.0f);
      }
      for (int k = 0; k < 6; ++k) dr[k] = smooth_l1_grad(pr[k] - tg[k], c.beta) * s_box;
      if (c.diff_rad_by_sin) {
        const float sp = sinf(pr[6]), cp = cosf(pr[6]), st = sinf(tg[6]), ct = cosf(tg[6]);
        const float u = smooth_l1_grad(sp * ct - cp * st, c.beta);
        dr[6] = (u * (cp * ct) + u * (sp * st)) * s_box;
      } else {
        dr[6] = smooth_l1_grad(pr[6] - tg[6], c.beta) * s_box;
      }
      if (c.use_dir) {
        const int dt = dir_target(c, tg[6], an[6]);
        float d2[2];
        for (int k = 0; k < 2; ++k) {
          const int ch = dir0 + a * 2 + k;
          d2[k] = zr.get(ch) + (bias ? bias[ch] : 0.0f);
        }
        const float m = fmaxf(d2[0], d2[1]);
        const float e0 = expf(d2[0] - m), e1 = expf(d2[1] - m), se = e0 + e1;
        dd[0] = (e0 / se - (dt == 0 ? 1.0f : 0.0f)) * s_dir;
        dd[1] = (e1 / se - (dt == 1 ? 1.0f : 0.0f)) * s_dir;
      }
    }
    for (int k = 0; k < 7; ++k) {
      const int ch = reg0 + a * 7 + k;
      if (live) put(ch, dr[k]);
      const float t = wave_sum(dr[k]);
      if (lane == 0) sb[wv * N + ch] = t;
    }
    if (c.use_dir)
      for (int k = 0; k < 2; ++k) {
        const int ch = dir0 + a * 2 + k;
        if (live) put(ch, dd[k]);
        const float t = wave_sum(dd[k]);
        if (lane == 0) sb[wv * N + ch] = t;
      }
  }
  if (live)
    for (int ch = N; ch < (kTile ? 8 * nc8 : c.dz_nwrite); ++ch) put(ch, 0.0f);
  __syncthreads();
  if (kTile) {
    tile_store(ztile, tp, dz, c.dz_sb, c.dz_shw, b, loc0, nrows, nc8);
    const int nz = nw8 - nc8;
    if (nz > 0) {
      unsigned short* dst = (unsigned short*)dz + (long long)b * c.dz_sb + (long long)loc0 * c.dz_shw;
      for (int q = threadIdx.x; q < nrows * nz; q += BLK) {
        const int r = q / nz, g8 = nc8 + (q - r * nz);
        *(uint4*)(dst + (long long)r * c.dz_shw + 8 * g8) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
  for (int ch = threadIdx.x; ch < N; ch += BLK)
    bpart[(long long)bid * N + ch] = ((sb[ch] + sb[N + ch]) + sb[2 * N + ch]) + sb[3 * N + ch];
}

}  // namespace head
}  // namespace rpc

using namespace rpc;
using namespace rpc::head;

static inline int head_channels(const RpcHeadCfg* c) { return c->S * c->R * (c->C + 7 + (c->use_dir ? 2 : 0)); }
static inline unsigned cdiv_u(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

static size_t align256(size_t n) { return (n + 255) & ~(size_t)255; }

struct HeadWs {
  float* gtb;
  unsigned* gmax;
  int* cnt;
  unsigned* ticket;
  double* part;
  float* bpart;
  size_t zero_bytes;  // gmax + cnt + ticket, contiguous
  size_t total;
};

static HeadWs head_ws(const RpcHeadCfg* c, int M, void* base) {
  HeadWs w;
  const int HW = c->H * c->W;
  const long long nblk = (long long)cdiv_u(HW, BLK) * c->B;
  char* p = (char*)base;
  size_t off = 0;
  w.gmax = (unsigned*)(p + off);
  off += (size_t)c->B * c->NA * (M > 0 ? M : 1) * sizeof(unsigned);
  w.cnt = (int*)(p + off);
  off += (size_t)c->B * sizeof(int);
  w.ticket = (unsigned*)(p + off);
  off += sizeof(unsigned);
  w.zero_bytes = off;
  off = align256(off);
  w.gtb = (float*)(p + off);
  off = align256(off + (size_t)c->B * (M > 0 ? M : 1) * 8 * sizeof(float));
  w.part = (double*)(p + off);
  off = align256(off + (size_t)nblk * 3 * sizeof(double));
  w.bpart = (float*)(p + off);
  off = align256(off + (size_t)nblk * head_channels(c) * sizeof(float));
  w.total = off;
  return w;
}

// bf16 images with unit channel stride and 16-byte aligned rows take the LDS-tile path
static bool zrow_tile(const RpcHeadCfg& c, const void* z, const void* dz) {
  const int N = head_channels(&c);
  bool ok = c.z_bf16 && c.z_sn == 1 && c.z_shw % 8 == 0 && c.z_sb % 8 == 0 && ((uintptr_t)z & 15) == 0 &&
            c.z_shw >= 8 * ((N + 7) / 8);
  if (dz) ok = ok && c.dz_bf16 && c.dz_sn == 1 && c.dz_shw % 8 == 0 && c.dz_sb % 8 == 0 && c.dz_nwrite % 8 == 0 &&
               c.dz_shw >= c.dz_nwrite && ((uintptr_t)dz & 15) == 0;
  return ok;
}

static int head_cfg_ok(const RpcHeadCfg* c) {
  if (!c || c->B <= 0 || c->H <= 0 || c->W <= 0 || c->S <= 0 || c->R <= 0 || c->C <= 0) return 0;
  if (c->S > RPC_HEAD_MAX_SIZES || c->S * c->R > kMaxA) return 0;
  if (c->NA != (c->assigner_per_size ? c->S : 1)) return 0;
  return 1;
}

extern "C" size_t rpc_anchor_head_workspace_size(const RpcHeadCfg* cfg, int max_gts) {
  if (!head_cfg_ok(cfg) || max_gts < 0) return 0;
  return head_ws(cfg, max_gts, nullptr).total;
}

extern "C" int rpc_anchor_head_loss_forward(const RpcHeadCfg* cfg, const float* anchor_tab, const float* gt_boxes,
                                            const long long* gt_labels, int max_gts, const void* z, const float* bias,
                                            int* assigned, float* losses, void* workspace, size_t ws_bytes,
                                            void* stream) {
  if (!head_cfg_ok(cfg) || !anchor_tab || !z || !assigned || !losses || !workspace || max_gts < 0) return RPC_ERR_ARG;
  if (max_gts > 0 && (!gt_boxes || !gt_labels)) return RPC_ERR_ARG;
  const RpcHeadCfg c = *cfg;
  HeadWs w = head_ws(&c, max_gts, workspace);
  if (ws_bytes < w.total) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int HW = c.H * c.W, M = max_gts;
  RPC_CHECK(hipMemsetAsync(workspace, 0, w.zero_bytes, st));
  if (M > 0) {
    hipLaunchKernelGGL(k_gt_prep, dim3(c.B), dim3(64), 0, st, gt_boxes, gt_labels, M, w.gtb);
    RPC_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_gt_max, dim3(cdiv_u(HW, BLK), c.NA, c.B), dim3(BLK), 4 * M * sizeof(float), st, c,
                       anchor_tab, (const float*)w.gtb, M, w.gmax);
    RPC_LAUNCH_CHECK();
  }
  const bool tile = zrow_tile(c, z, nullptr);
  const int N = head_channels(&c);
  const size_t lds = tile ? (size_t)BLK * (8 * ((N + 7) / 8)) * sizeof(unsigned short) : 0;
  hipLaunchKernelGGL(tile ? k_loss_fwd<true> : k_loss_fwd<false>, dim3(cdiv_u(HW, BLK), c.B), dim3(BLK), lds, st, c,
                     anchor_tab, (const float*)w.gtb,
                     gt_boxes, M, (const unsigned*)w.gmax, z, bias, assigned, w.part, w.cnt, w.ticket, losses);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_anchor_head_loss_backward(const RpcHeadCfg* cfg, const float* anchor_tab, const float* gt_boxes,
                                             int max_gts, const void* z, const float* bias, const int* assigned,
                                             const float* grad_losses, const float* losses, void* dz,
                                             float* dbias, void* workspace, size_t ws_bytes, void* stream) {
  if (!head_cfg_ok(cfg) || !anchor_tab || !z || !assigned || !grad_losses || !losses || !dz || !workspace ||
      max_gts < 0)
    return RPC_ERR_ARG;
  const RpcHeadCfg c = *cfg;
  const int N = head_channels(&c);
  if (c.dz_nwrite < N) return RPC_ERR_ARG;
  HeadWs w = head_ws(&c, max_gts, workspace);
  if (ws_bytes < w.total) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int HW = c.H * c.W;
  const unsigned gx = cdiv_u(HW, BLK);
  const bool tile = zrow_tile(c, z, dz);
  const int tp = 8 * ((N + 7) / 8);
  const size_t lds = ((4 * N * sizeof(float) + 15) & ~(size_t)15) + (tile ? (size_t)BLK * tp * sizeof(unsigned short) : 0);
  hipLaunchKernelGGL(tile ? k_loss_bwd<true> : k_loss_bwd<false>, dim3(gx, c.B), dim3(BLK), lds, st, c, anchor_tab,
                     (const float*)w.gtb, gt_boxes, max_gts, z, bias, assigned, grad_losses, losses, dz, w.bpart);
  RPC_LAUNCH_CHECK();
  if (dbias) {
    slab_reduce(w.bpart, (int)(gx * c.B), N, dbias, st);
    RPC_LAUNCH_CHECK();
  }
  return RPC_OK;
}
