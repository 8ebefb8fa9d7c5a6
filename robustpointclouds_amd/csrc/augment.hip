// §8(f2): the training-pipeline point / box augmentations on the GPU, batched over frames (gfx950).
//
// Restates, for the transforms of configs/_base_/kitti-3d-car.py:42-68 that act on every frame
// (upstream mmdet3d v1.x transforms, not vendored here):
//   RandomFlip3D(flip_ratio_bev_horizontal)   points y -> -y (horizontal) / x -> -x (vertical);
//                                             boxes the same, yaw -> -yaw (+ pi for vertical)
//   GlobalRotScaleTrans(rot_range, scale)     [x y z] @ [[c s 0] [-s c 0] [0 0 1]], boxes: centre
//                                             likewise and yaw += angle; then * scale (points xyz,
//                                             box centre + dims); then + translation
//   PointsRangeFilter(point_cloud_range)      keep x > x0 & y > y0 & z > z0 & x < x1 & y < y1 & z < z1
//   ObjectRangeFilter(point_cloud_range)      keep boxes with BEV centre strictly inside, then
//                                             limit_yaw(offset 0.5, period 2 pi)
//   PointShuffle                              a random permutation of each frame's points
// The random parameters are drawn on the host in the reference's order (augment.py), so the device
// does only the per-point / per-box arithmetic:
//   K1 transform + in-range flag per point (frame by binary search over the offsets, as in a1);
//   K2 exclusive scan of the flags (hipCUB);  K3 compaction in point order + per-frame offsets; the
//   tail beyond the surviving points is filled with NaN so a1 (hard_voxelize) rejects it without a
//   host read of the new count;  K4 optional shuffle: 64-bit keys (frame, hash(seed, frame, rank))
//   radix-sorted, then a gather — a uniform permutation per frame, reproducible from the seed;
//   K5 boxes in place; dropped boxes become padding (label -1), the convention of pack_gt.
#include <hipcub/hipcub.hpp>
#include <math.h>

#include "common.h"

#pragma clang fp contract(off)

namespace rpc {
namespace aug {

constexpr int BLK = 256;
constexpr float kPiF = 3.14159265358979323846f;   // np.pi as a float32 tensor operand

__device__ __forceinline__ int frame_of(const int* off, int B, int p) {
  int lo = 0, hi = B;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (off[mid] <= p) lo = mid; else hi = mid;
  }
  return lo;
}

struct Range {
  float r[6];
};

// the transform chain of one point's xyz (in place)
__device__ __forceinline__ void xform(const RpcAugFrame& a, float& x, float& y, float& z) {
  if (a.flip_h) y = -y;
  if (a.flip_v) x = -x;
  // rotation: row vector @ rot_mat_T
  const float xr = x * a.cosr + y * (-a.sinr);
  const float yr = x * a.sinr + y * a.cosr;
  x = xr;
  y = yr;
  x = x * a.scale;
  y = y * a.scale;
  z = z * a.scale;
  x = x + a.tx;
  y = y + a.ty;
  z = z + a.tz;
}

__global__ __launch_bounds__(BLK) void k_points(const float* __restrict__ pts, int F, int P, const int* __restrict__ off,
                                                int B, const RpcAugFrame* __restrict__ fr, Range rg,
                                                float* __restrict__ tmp, int* __restrict__ flag) {
  const int p = blockIdx.x * BLK + threadIdx.x;
  if (p >= P) return;
  const int b = frame_of(off, B, p);
  const bool in_frame = p < off[B];
  const float* q = pts + (size_t)p * F;
  float x = q[0], y = q[1], z = q[2];
  xform(fr[b], x, y, z);
  float* o = tmp + (size_t)p * F;
  o[0] = x;
  o[1] = y;
  o[2] = z;
  for (int f = 3; f < F; ++f) o[f] = q[f];
  const bool keep = in_frame && x > rg.r[0] && y > rg.r[1] && z > rg.r[2] && x < rg.r[3] && y < rg.r[4] && z < rg.r[5];
  flag[p] = keep ? 1 : 0;
}

// compaction in point order; pos = exclusive scan of flag (P+1 entries); out_off[b] = pos[off[b]]
__global__ __launch_bounds__(BLK) void k_compact(const float* __restrict__ tmp, int F, int P,
                                                 const int* __restrict__ off, int B, const int* __restrict__ flag,
                                                 const int* __restrict__ pos, float* __restrict__ out,
                                                 int* __restrict__ out_off) {
  const int p = blockIdx.x * BLK + threadIdx.x;
  if (p <= B) out_off[p] = pos[off[p]];
  if (p >= P) return;
  const int n_keep = pos[P];
  if (flag[p]) {
    const float* s = tmp + (size_t)p * F;
    float* d = out + (size_t)pos[p] * F;
    for (int f = 0; f < F; ++f) d[f] = s[f];
  }
  if (p >= n_keep) {   // tail: NaN points are rejected by the voxeliser (no host read of n_keep)
    float* d = out + (size_t)p * F;
    for (int f = 0; f < F; ++f) d[f] = __builtin_nanf("");
  }
}

__device__ __forceinline__ unsigned hash3(unsigned long long seed, unsigned a, unsigned b) {
  unsigned long long h = seed ^ (0x9E3779B97F4A7C15ull * (a + 1)) ^ (0xC2B2AE3D27D4EB4Full * (b + 1));
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return (unsigned)h;
}

// key = (frame << 32) | hash(seed, frame, rank in frame); the NaN tail sorts last (frame B)
__global__ __launch_bounds__(BLK) void k_shuffle_keys(int P, const int* __restrict__ out_off, int B,
                                                      unsigned long long seed, unsigned long long* __restrict__ keys,
                                                      int* __restrict__ vals) {
  const int p = blockIdx.x * BLK + threadIdx.x;
  if (p >= P) return;
  int b = B;
  if (p < out_off[B]) b = frame_of(out_off, B, p);
  const unsigned r = b < B ? (unsigned)(p - out_off[b]) : (unsigned)p;
  keys[p] = ((unsigned long long)b << 32) | hash3(seed, (unsigned)b, r);
  vals[p] = p;
}

__global__ __launch_bounds__(BLK) void k_gather(const float* __restrict__ src, int F, int P, const int* __restrict__ idx,
                                                float* __restrict__ dst) {
  const int p = blockIdx.x * BLK + threadIdx.x;
  if (p >= P) return;
  const float* s = src + (size_t)idx[p] * F;
  float* d = dst + (size_t)p * F;
  for (int f = 0; f < F; ++f) d[f] = s[f];
}

__device__ __forceinline__ float limit_period(float v, float off, float period) {
  return v - floorf(v / period + off) * period;
}

// boxes [B][M][7] (x, y, z, dx, dy, dz, yaw), labels [B][M] int64, in place
__global__ __launch_bounds__(BLK) void k_boxes(float* __restrict__ boxes, long long* __restrict__ labels, int B, int M,
                                               const RpcAugFrame* __restrict__ fr, Range rg) {
  const int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= B * M) return;
  const int b = t / M;
  if (labels[t] < 0) return;
  float* bx = boxes + (size_t)t * 7;
  const RpcAugFrame a = fr[b];
  float x = bx[0], y = bx[1], z = bx[2], yaw = bx[6];
  if (a.flip_h) {
    y = -y;
    yaw = -yaw;
  }
  if (a.flip_v) {
    x = -x;
    yaw = -yaw + kPiF;
  }
  const float xr = x * a.cosr + y * (-a.sinr);
  const float yr = x * a.sinr + y * a.cosr;
  x = xr;
  y = yr;
  yaw = yaw + a.rot;
  x = x * a.scale;
  y = y * a.scale;
  z = z * a.scale;
  const float dx = bx[3] * a.scale, dy = bx[4] * a.scale, dz = bx[5] * a.scale;
  x = x + a.tx;
  y = y + a.ty;
  z = z + a.tz;
  const bool keep = x > rg.r[0] && y > rg.r[1] && x < rg.r[3] && y < rg.r[4];
  if (!keep) {
    labels[t] = -1;
    bx[3] = bx[4] = bx[5] = 1.0f;   // padding boxes keep unit size (pack_gt convention)
    return;
  }
  bx[0] = x;
  bx[1] = y;
  bx[2] = z;
  bx[3] = dx;
  bx[4] = dy;
  bx[5] = dz;
  bx[6] = limit_period(yaw, 0.5f, 2.0f * kPiF);
}

}  // namespace aug
}  // namespace rpc

using namespace rpc;
using namespace rpc::aug;

static size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

struct AugWs {
  size_t tmp, flag, pos, keys, keys2, vals, vals2, cub, cub_bytes, total;
};

static AugWs aug_ws(int F, int P) {
  AugWs w;
  size_t scan_b = 0, sort_b = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (const int*)nullptr, (int*)nullptr, P + 1, (hipStream_t)0);
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (const unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                     (const int*)nullptr, (int*)nullptr, P > 0 ? P : 1, 0, 64, (hipStream_t)0);
  size_t o = 0;
  w.tmp = o; o += al256(sizeof(float) * (size_t)(P > 0 ? P : 1) * F);
  w.flag = o; o += al256(sizeof(int) * (size_t)(P + 1));
  w.pos = o; o += al256(sizeof(int) * (size_t)(P + 1));
  w.keys = o; o += al256(sizeof(unsigned long long) * (size_t)(P > 0 ? P : 1));
  w.keys2 = o; o += al256(sizeof(unsigned long long) * (size_t)(P > 0 ? P : 1));
  w.vals = o; o += al256(sizeof(int) * (size_t)(P > 0 ? P : 1));
  w.vals2 = o; o += al256(sizeof(int) * (size_t)(P > 0 ? P : 1));
  w.cub_bytes = scan_b > sort_b ? scan_b : sort_b;
  w.cub = o; o += al256(w.cub_bytes);
  w.total = o;
  return w;
}

extern "C" size_t rpc_augment_points_workspace_size(int num_features, int total_points) {
  if (num_features < 3 || total_points < 0) return 0;
  return aug_ws(num_features, total_points).total;
}

extern "C" int rpc_augment_points(const float* points, int F, int P, const int* frame_offsets, int B,
                                  const RpcAugFrame* frames, const float* pc_range, int shuffle,
                                  unsigned long long seed, float* out_points, int* out_offsets, void* workspace,
                                  size_t ws_bytes, void* stream) {
  if (!points || F < 3 || P < 0 || !frame_offsets || B < 1 || !frames || !pc_range || !out_points || !out_offsets ||
      !workspace)
    return RPC_ERR_ARG;
  AugWs w = aug_ws(F, P);
  if (ws_bytes < w.total) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  char* base = (char*)workspace;
  float* tmp = (float*)(base + w.tmp);
  int* flag = (int*)(base + w.flag);
  int* pos = (int*)(base + w.pos);
  Range rg;
  for (int k = 0; k < 6; ++k) rg.r[k] = pc_range[k];
  const unsigned nb = (unsigned)((P + BLK) / BLK);   // covers P and the B+1 offsets (B < P or one block)
  RPC_CHECK(hipMemsetAsync(flag + P, 0, sizeof(int), st));
  if (P > 0) {
    hipLaunchKernelGGL(k_points, dim3(nb), dim3(BLK), 0, st, points, F, P, frame_offsets, B, frames, rg, tmp, flag);
    RPC_LAUNCH_CHECK();
  }
  size_t cb = w.cub_bytes;
  RPC_CHECK(hipcub::DeviceScan::ExclusiveSum(base + w.cub, cb, flag, pos, P + 1, st));
  const unsigned nc = (unsigned)(((P > B ? P : B + 1) + BLK) / BLK);
  hipLaunchKernelGGL(k_compact, dim3(nc), dim3(BLK), 0, st, tmp, F, P, frame_offsets, B, flag, pos, out_points,
                     out_offsets);
  RPC_LAUNCH_CHECK();
  if (shuffle && P > 0) {
    unsigned long long* keys = (unsigned long long*)(base + w.keys);
    unsigned long long* keys2 = (unsigned long long*)(base + w.keys2);
    int* vals = (int*)(base + w.vals);
    int* vals2 = (int*)(base + w.vals2);
    hipLaunchKernelGGL(k_shuffle_keys, dim3(nb), dim3(BLK), 0, st, P, (const int*)out_offsets, B, seed, keys, vals);
    RPC_LAUNCH_CHECK();
    cb = w.cub_bytes;
    RPC_CHECK(hipcub::DeviceRadixSort::SortPairs(base + w.cub, cb, keys, keys2, vals, vals2, P, 0, 64, st));
    RPC_CHECK(hipMemcpyAsync(tmp, out_points, sizeof(float) * (size_t)P * F, hipMemcpyDeviceToDevice, st));
    hipLaunchKernelGGL(k_gather, dim3(nb), dim3(BLK), 0, st, tmp, F, P, (const int*)vals2, out_points);
    RPC_LAUNCH_CHECK();
  }
  return RPC_OK;
}

extern "C" int rpc_augment_boxes(float* boxes, long long* labels, int B, int M, const RpcAugFrame* frames,
                                 const float* pc_range, void* stream) {
  if (B < 1 || M < 0 || !frames || !pc_range || (M > 0 && (!boxes || !labels))) return RPC_ERR_ARG;
  if (M == 0) return RPC_OK;
  Range rg;
  for (int k = 0; k < 6; ++k) rg.r[k] = pc_range[k];
  hipLaunchKernelGGL(k_boxes, dim3((unsigned)((B * M + BLK - 1) / BLK)), dim3(BLK), 0, (hipStream_t)stream, boxes,
                     labels, B, M, frames, rg);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
