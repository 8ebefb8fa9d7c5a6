// §8(f4): the StrongAdversarialVoxelNet perturbation step (BASELINE config 5), for gfx950.
//
// models/detectors/strong_adversarial_voxelnet.py:109-192 (update_adversarial_strength +
// apply_enhanced_perturbations), applied to the HardSimpleVFE output [V, F]:
//   scaling   = min(epoch_scaling * boost * complexity, max_scaling)                   (:109-139)
//               boost = 2 / 1.5 / 1 when mean |l2| of the last 50 steps is < 0.1 / < 0.3 / else,
//               only once more than 50 steps are recorded
//   scaled    = (adversary(x) - x) * scaling [+ momentum_alpha * last_scaled]           (:157-175)
//   perturbed = x + scaled ;  l2 = ||scaled||_2 (Frobenius) appended to the history     (:177-186)
// One launch: every block derives `scaling` from the device-side history ring (no .item() host
// read, unlike :180), applies the combine over a grid-stride range and writes a double partial of
// sum scaled^2; the last-arriving block reduces the partials in block order, writes l2 and pushes
// it into the ring. The backward is the analytic one of the same expression (momentum term and
// scaling carry no gradient, as in the reference where both are detached / Python floats).
#include <hip/hip_runtime.h>
#include <math.h>

#include "common.h"

#pragma clang fp contract(off)  // the reference's float32 op order (no fused multiply-adds)

namespace rpc {
namespace strong {

constexpr int BLK = 256;
constexpr int GRID = 512;

// the reference computes the scaling in Python floats (double) and multiplies a float32 tensor
// by it (-> the scaling rounded to float32)
__device__ __forceinline__ double strong_scaling(const RpcStrongCfg& c, const float* hist) {
  double s = c.epoch_scaling;
  if (c.history_count > 50) {
    // np.mean of |x| over the 50 most recent entries (ring of RPC_STRONG_RING, newest at count-1)
    double m = 0.0;
    for (int k = 0; k < 50; ++k) {
      const long long idx = (long long)c.history_count - 50 + k;
      m += fabs((double)hist[idx % RPC_STRONG_RING]);
    }
    const double avg = m / 50.0;
    s *= avg < 0.1 ? 2.0 : (avg < 0.3 ? 1.5 : 1.0);
  }
  if (c.curriculum) s *= c.complexity;
  return s < c.max_scaling ? s : c.max_scaling;
}

__global__ __launch_bounds__(BLK) void k_strong_fwd(RpcStrongCfg c, const float* __restrict__ x,
                                                    const float* __restrict__ adv, const float* __restrict__ last,
                                                    long long n, float* __restrict__ perturbed,
                                                    float* __restrict__ scaled, float* __restrict__ hist,
                                                    float* __restrict__ state, double* __restrict__ part,
                                                    unsigned* __restrict__ ticket) {
  __shared__ double sh[BLK / 64];
  __shared__ int lastf;
  const double sd = c.dynamic ? strong_scaling(c, hist) : 1.0;
  const float s = (float)sd;
  double acc = 0.0;
  for (long long i = (long long)blockIdx.x * BLK + threadIdx.x; i < n; i += (long long)gridDim.x * BLK) {
    const float xv = x[i];
    float v = (adv[i] - xv) * s;
    if (last) v = v + c.momentum_alpha * last[i];
    scaled[i] = v;
    perturbed[i] = xv + v;
    acc += (double)v * (double)v;
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = ((sh[0] + sh[1]) + sh[2]) + sh[3];
  if (!last_block_arrive(ticket, &lastf)) return;
  if (threadIdx.x < 64) {
    double t = 0.0;
    for (int k = threadIdx.x; k < (int)gridDim.x; k += 64) t += part[k];
    t = wave_sum(t);
    if (threadIdx.x == 0) {
      const float l2 = (float)sqrt(t);
      state[0] = s;                                   // current scaling
      state[1] = l2;
      state[2] = (float)(c.adversarial_loss_weight * sd);   // dynamic weight (Python float product)
      hist[c.history_count % RPC_STRONG_RING] = l2;
    }
  }
}

// g_s = g_p + g_l2 * scaled / l2 ; g_adv = g_s * s ; g_x = g_p - g_s * s
__global__ __launch_bounds__(BLK) void k_strong_bwd(const float* __restrict__ scaled, long long n,
                                                    const float* __restrict__ state, const float* __restrict__ gp,
                                                    const float* __restrict__ gl2, float* __restrict__ gx,
                                                    float* __restrict__ gadv) {
  const float s = state[0], l2 = state[1];
  const float gn = (gl2 && l2 > 0.0f) ? gl2[0] / l2 : 0.0f;
  for (long long i = (long long)blockIdx.x * BLK + threadIdx.x; i < n; i += (long long)gridDim.x * BLK) {
    const float g = gp ? gp[i] : 0.0f;
    const float gs = g + gn * scaled[i];
    if (gadv) gadv[i] = gs * s;
    if (gx) gx[i] = g - gs * s;
  }
}

}  // namespace strong
}  // namespace rpc

using namespace rpc;
using namespace rpc::strong;

extern "C" size_t rpc_strong_perturb_workspace_size(void) { return GRID * sizeof(double) + 256; }

extern "C" int rpc_strong_perturb_forward(const RpcStrongCfg* cfg, const float* x, const float* adv_out,
                                          const float* last_scaled, long long n, float* perturbed, float* scaled,
                                          float* history, float* state, void* workspace, size_t ws_bytes,
                                          void* stream) {
  if (!cfg || !x || !adv_out || !perturbed || !scaled || !history || !state || !workspace || n < 0) return RPC_ERR_ARG;
  if (ws_bytes < rpc_strong_perturb_workspace_size()) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  double* part = (double*)workspace;
  unsigned* ticket = (unsigned*)((char*)workspace + GRID * sizeof(double));
  RPC_CHECK(hipMemsetAsync(ticket, 0, sizeof(unsigned), st));
  const int g = grid_for(n, BLK, GRID);
  hipLaunchKernelGGL(k_strong_fwd, dim3(g), dim3(BLK), 0, st, *cfg, x, adv_out, last_scaled, n, perturbed, scaled,
                     history, state, part, ticket);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_strong_perturb_backward(const float* scaled, long long n, const float* state,
                                           const float* grad_perturbed, const float* grad_l2, float* grad_x,
                                           float* grad_adv_out, void* stream) {
  if (!scaled || !state || n < 0) return RPC_ERR_ARG;
  if (n == 0) return RPC_OK;
  hipLaunchKernelGGL(k_strong_bwd, dim3(grid_for(n, BLK, 2048)), dim3(BLK), 0, (hipStream_t)stream, scaled, n, state,
                     grad_perturbed, grad_l2, grad_x, grad_adv_out);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
