// a5: HardSimpleVFE (upstream mmdet3d voxel_encoders/voxel_encoder.py), used at
// models/detectors/adversarial_voxelnet.py:135-137. Memory-bound: one pass over the
// voxel slots, summed in slot order (0..max_points-1) then one IEEE division, which is
// the order torch's CPU reduction uses, so the result is bit-exact with it.
#include "common.h"

namespace rpc {
namespace vfe {
constexpr int BLK = 256;

__global__ __launch_bounds__(BLK) void k_fwd(const float* __restrict__ vox,
                                             const int* __restrict__ np, int V, int P, int F,
                                             int VF, float* __restrict__ out) {
  int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= V * VF) return;
  int v = t / VF, f = t - v * VF;
  const float* p = vox + (size_t)v * P * F + f;
  float s = p[0];
  for (int j = 1; j < P; ++j) s += p[(size_t)j * F];
  out[t] = s / (float)np[v];
}

__global__ __launch_bounds__(BLK) void k_bwd(const float* __restrict__ dout,
                                             const int* __restrict__ np, int V, int P, int F,
                                             int VF, float* __restrict__ dvox) {
  long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  if (t >= (long long)V * P * F) return;
  int f = (int)(t % F);
  int v = (int)(t / ((long long)P * F));
  dvox[t] = f < VF ? dout[(size_t)v * VF + f] / (float)np[v] : 0.0f;
}
}  // namespace vfe
}  // namespace rpc

extern "C" int rpc_vfe_mean_forward(const float* voxels, const int* num_points, int V, int P,
                                    int F, int VF, float* out, void* stream) {
  if (V < 0 || P < 1 || F < 1 || VF < 1 || VF > F) return RPC_ERR_ARG;
  if (V == 0) return RPC_OK;
  if (!voxels || !num_points || !out) return RPC_ERR_ARG;
  long long n = (long long)V * VF;
  hipLaunchKernelGGL(rpc::vfe::k_fwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, voxels, num_points, V, P, F, VF, out);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_vfe_mean_backward(const float* dout, const int* num_points, int V, int P, int F,
                                     int VF, float* dvoxels, void* stream) {
  if (V < 0 || P < 1 || F < 1 || VF < 1 || VF > F) return RPC_ERR_ARG;
  if (V == 0) return RPC_OK;
  if (!dout || !num_points || !dvoxels) return RPC_ERR_ARG;
  long long n = (long long)V * P * F;
  hipLaunchKernelGGL(rpc::vfe::k_bwd, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, dout, num_points, V, P, F, VF, dvoxels);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
