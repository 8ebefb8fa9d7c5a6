// a1: bit-exact hard voxelisation of B frames in one pass (gfx950).
//
// Replaces mmcv.ops hard_voxelize_forward (upstream mmcv voxelization_cuda.cu), whose
// deterministic CUDA path finds each point's voxel slot with an O(N^2) scan over the
// earlier points and then assigns voxel ids in a single-thread serial kernel, one frame
// at a time from a Python loop (upstream Det3DDataPreprocessor.voxelize). Here:
//
//   K1  per point: integer voxel key (frame, z, y, x) or INVALID, coalesced loads;
//   K2  stable LSD radix sort of (key, point index)  -> points of a voxel are contiguous
//       and in point order, so a point's slot is the length of the equal-key run before
//       it (bounded look-back of max_points, no atomics);
//   K3  head flags (slot 0) scattered back to point order;
//   K4  exclusive scan of the head flags -> voxel rank in order of first appearance;
//   K5  per sorted point: write voxel slot, coors and num_points; drop voxels whose
//       rank >= max_voxels and points whose slot >= max_points; zero the unused slots.
//
// Every step is deterministic: same input -> same bytes, and equal to mmcv's CPU and CUDA
// kernels (first-appearance voxel order, the max_voxels cap, max_points in point order).
#include <hipcub/hipcub.hpp>

#include "common.h"

namespace rpc {
namespace vox {

constexpr int BLK = 256;

struct Grid {
  float vs[3];
  float mn[3];
  int g[3];           // x, y, z cells
  unsigned long long G;  // cells per frame
};

__global__ __launch_bounds__(BLK) void k_keys(const float* __restrict__ pts, int F, int P,
                                              const int* __restrict__ off, int B, Grid gr,
                                              unsigned long long inv,
                                              unsigned long long* __restrict__ keys,
                                              int* __restrict__ vals, int* __restrict__ head) {
  int p = blockIdx.x * BLK + threadIdx.x;
  if (p == 0) head[P] = 0;
  if (p >= P) return;
  // frame of p: binary search over the B+1 offsets (B is small, offsets stay in L1/L2)
  int lo = 0, hi = B;
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (__ldg(off + mid) <= p) lo = mid; else hi = mid;
  }
  const float* q = pts + (size_t)p * F;
  unsigned long long key = inv;
  bool ok = true;
  int c[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    // float32 arithmetic exactly as mmcv: floor((p - min) / vs); IEEE division.
    float cf = floorf((q[j] - gr.mn[j]) / gr.vs[j]);
    ok = ok && (cf >= 0.0f) && (cf < (float)gr.g[j]);  // NaN fails both tests
    c[j] = ok ? (int)cf : 0;
  }
  if (ok) {
    unsigned long long lin =
        ((unsigned long long)c[2] * gr.g[1] + (unsigned long long)c[1]) * gr.g[0] + c[0];
    key = (unsigned long long)lo * gr.G + lin;
  }
  keys[p] = key;
  vals[p] = p;
  head[p] = 0;
}

__device__ __forceinline__ int run_slot(const unsigned long long* __restrict__ k, int i,
                                        unsigned long long key, int maxp) {
  int s = 0;
  while (s < maxp && i - s - 1 >= 0 && k[i - s - 1] == key) ++s;
  return s;
}

__global__ __launch_bounds__(BLK) void k_heads(const unsigned long long* __restrict__ ks,
                                               const int* __restrict__ vs, int P,
                                               unsigned long long inv, int* __restrict__ head) {
  int i = blockIdx.x * BLK + threadIdx.x;
  if (i >= P) return;
  unsigned long long k = ks[i];
  if (k == inv) return;
  if (i == 0 || ks[i - 1] != k) head[vs[i]] = 1;
}

__global__ __launch_bounds__(BLK) void k_emit(const float* __restrict__ pts, int F, int P,
                                              const int* __restrict__ off, int B, Grid gr,
                                              unsigned long long inv,
                                              const unsigned long long* __restrict__ ks,
                                              const int* __restrict__ vs,
                                              const int* __restrict__ rank, int maxp, int maxv,
                                              float* __restrict__ voxels, int* __restrict__ coors,
                                              int* __restrict__ npts, int* __restrict__ vnum) {
  int i = blockIdx.x * BLK + threadIdx.x;
  if (i == 0) {
    int tot = 0;
    for (int b = 0; b < B; ++b) {
      int nb = rank[off[b + 1]] - rank[off[b]];
      nb = nb < maxv ? nb : maxv;
      vnum[b] = nb;
      tot += nb;
    }
    vnum[B] = tot;
  }
  if (i >= P) return;
  unsigned long long k = ks[i];
  if (k == inv) return;
  int s = run_slot(ks, i, k, maxp);
  if (s >= maxp) return;
  int hp = vs[i - s];
  int b = (int)(k / gr.G);
  unsigned long long lin = k - (unsigned long long)b * gr.G;
  int local = rank[hp] - rank[off[b]];
  if (local >= maxv) return;
  int voff = 0;
  for (int bb = 0; bb < b; ++bb) {
    int nb = rank[off[bb + 1]] - rank[off[bb]];
    voff += nb < maxv ? nb : maxv;
  }
  long long gv = (long long)voff + local;
  const float* src = pts + (size_t)vs[i] * F;
  float* dst = voxels + ((size_t)gv * maxp + s) * F;
  for (int f = 0; f < F; ++f) dst[f] = src[f];
  if (s == 0) {
    int cx = (int)(lin % (unsigned long long)gr.g[0]);
    unsigned long long t = lin / (unsigned long long)gr.g[0];
    int cy = (int)(t % (unsigned long long)gr.g[1]);
    int cz = (int)(t / (unsigned long long)gr.g[1]);
    int* c = coors + gv * 4;
    c[0] = b;
    c[1] = cz;
    c[2] = cy;
    c[3] = cx;
  }
  bool last = (s == maxp - 1) || (i + 1 >= P) || (ks[i + 1] != k);
  if (last) {
    npts[gv] = s + 1;
    for (int t = s + 1; t < maxp; ++t) {
      float* z = voxels + ((size_t)gv * maxp + t) * F;
      for (int f = 0; f < F; ++f) z[f] = 0.0f;
    }
  }
}

static inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

struct WsLayout {
  size_t keys_in, keys_out, vals_in, vals_out, head, rank, sort_tmp, scan_tmp, total;
  size_t sort_bytes, scan_bytes;
};

static int layout(int P, WsLayout* L, hipStream_t st) {
  size_t sort_b = 0, scan_b = 0;
  RPC_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_b, (unsigned long long*)nullptr,
                                               (unsigned long long*)nullptr, (int*)nullptr,
                                               (int*)nullptr, P, 0, 64, st));
  RPC_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (int*)nullptr, (int*)nullptr,
                                             P + 1, st));
  size_t o = 0;
  L->keys_in = o; o += al(sizeof(unsigned long long) * (size_t)P);
  L->keys_out = o; o += al(sizeof(unsigned long long) * (size_t)P);
  L->vals_in = o; o += al(sizeof(int) * (size_t)P);
  L->vals_out = o; o += al(sizeof(int) * (size_t)P);
  L->head = o; o += al(sizeof(int) * (size_t)(P + 1));
  L->rank = o; o += al(sizeof(int) * (size_t)(P + 1));
  L->sort_tmp = o; o += al(sort_b);
  L->scan_tmp = o; o += al(scan_b);
  L->sort_bytes = sort_b;
  L->scan_bytes = scan_b;
  L->total = o;
  return RPC_OK;
}

}  // namespace vox
}  // namespace rpc

using namespace rpc;
using namespace rpc::vox;

extern "C" size_t rpc_hard_voxelize_workspace_size(int total_points, int batch) {
  (void)batch;
  if (total_points < 1) total_points = 1;
  WsLayout L;
  if (layout(total_points, &L, 0) != RPC_OK) return 0;
  return L.total;
}

extern "C" int rpc_hard_voxelize(const float* points, int F, int P, const int* frame_offsets,
                                 int B, const float* voxel_size, const float* coors_range,
                                 int max_points, int max_voxels, float* voxels, int* coors,
                                 int* num_points, int* voxel_num, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  if (F < 3 || B < 1 || max_points < 1 || max_voxels < 1 || P < 0 || !frame_offsets ||
      !voxel_size || !coors_range || !voxel_num)
    return RPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (P == 0) {
    RPC_CHECK(hipMemsetAsync(voxel_num, 0, sizeof(int) * (B + 1), st));
    return RPC_OK;
  }
  if (!points || !voxels || !coors || !num_points || !workspace) return RPC_ERR_ARG;
  Grid gr;
  for (int j = 0; j < 3; ++j) {
    gr.vs[j] = voxel_size[j];
    gr.mn[j] = coors_range[j];
    // host float arithmetic as mmcv: round((max - min) / vs)
    float span = coors_range[3 + j] - coors_range[j];
    gr.g[j] = (int)roundf(span / voxel_size[j]);
    if (gr.g[j] <= 0) return RPC_ERR_ARG;
  }
  gr.G = (unsigned long long)gr.g[0] * gr.g[1] * gr.g[2];
  unsigned long long inv = (unsigned long long)B * gr.G;
  int end_bit = 64 - __builtin_clzll(inv);
  WsLayout L;
  int rc = layout(P, &L, st);
  if (rc) return rc;
  if (workspace_bytes < L.total) return RPC_ERR_WORKSPACE;
  char* ws = (char*)workspace;
  auto* kin = (unsigned long long*)(ws + L.keys_in);
  auto* kout = (unsigned long long*)(ws + L.keys_out);
  int* vin = (int*)(ws + L.vals_in);
  int* vout = (int*)(ws + L.vals_out);
  int* head = (int*)(ws + L.head);
  int* rank = (int*)(ws + L.rank);
  int nb = (P + BLK - 1) / BLK;
  hipLaunchKernelGGL(k_keys, dim3(nb), dim3(BLK), 0, st, points, F, P, frame_offsets, B, gr, inv,
                     kin, vin, head);
  RPC_LAUNCH_CHECK();
  size_t sb = L.sort_bytes;
  RPC_CHECK(hipcub::DeviceRadixSort::SortPairs(ws + L.sort_tmp, sb, kin, kout, vin, vout, P, 0,
                                               end_bit, st));
  hipLaunchKernelGGL(k_heads, dim3(nb), dim3(BLK), 0, st, kout, vout, P, inv, head);
  RPC_LAUNCH_CHECK();
  size_t cb = L.scan_bytes;
  RPC_CHECK(hipcub::DeviceScan::ExclusiveSum(ws + L.scan_tmp, cb, head, rank, P + 1, st));
  hipLaunchKernelGGL(k_emit, dim3(nb), dim3(BLK), 0, st, points, F, P, frame_offsets, B, gr, inv,
                     kout, vout, rank, max_points, max_voxels, voxels, coors, num_points,
                     voxel_num);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
