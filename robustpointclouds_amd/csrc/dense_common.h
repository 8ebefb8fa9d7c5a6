// Shared by the dense BEV engine's bf16 (dense_conv.hip, perf mode) and fp32 (dense_f32.hip,
// parity mode) kernels: the pixel maps that turn a GEMM row + tap into a source pixel, the
// XCD-aware block remap and the fixed-order weight-gradient slab reduction.
#pragma once
#include <hip/hip_runtime.h>

namespace rpc {
namespace dn {

struct Img {
  int B, H, W;
};

// M_D2P (internal, bf16 only): the data gradient of S2 split by input-pixel parity
enum { M_S1 = 0, M_S2 = 1, M_D2 = 2, M_P1 = 3, M_U2 = 4, M_G2 = 5, M_D2P = 6 };

template <int MAP>
__host__ __device__ constexpr int taps_of() {
  return (MAP == M_P1 || MAP == M_U2) ? 1 : ((MAP == M_G2 || MAP == M_D2P) ? 4 : 9);
}

// weight-gradient "taps": U2 has one GEMM per output parity, each with its own weight slice
template <int MAP>
__host__ __device__ constexpr int wtaps_of() {
  return MAP == M_U2 ? 4 : taps_of<MAP>();
}

inline int map_wtaps(int map) {
  switch (map) {
    case M_P1: return 1;
    case M_U2:
    case M_G2: return 4;
    default: return 9;
  }
}

// K-operand source pixel of GEMM row pixel (b, y, x) for tap t in image S (-1: zero row)
template <int MAP>
__device__ __forceinline__ int src_row(int b, int y, int x, int t, const Img& S) {
  int sy, sx;
  if (MAP == M_S1) {
    sy = y + t / 3 - 1;
    sx = x + t % 3 - 1;
  } else if (MAP == M_S2) {
    sy = 2 * y + t / 3 - 1;
    sx = 2 * x + t % 3 - 1;
  } else if (MAP == M_D2) {
    const int oy = y + 1 - t / 3, ox = x + 1 - t % 3;
    if ((oy | ox) < 0 || ((oy | ox) & 1)) return -1;
    sy = oy >> 1;
    sx = ox >> 1;
  } else if (MAP == M_G2) {
    sy = 2 * y + (t >> 1);
    sx = 2 * x + (t & 1);
  } else {
    sy = y;
    sx = x;
  }
  if (sy < 0 || sy >= S.H || sx < 0 || sx >= S.W) return -1;
  return (b * S.H + sy) * S.W + sx;
}

// output pixel of GEMM row m = (b, y, x) (U2: parity par of the 2x upsampled image O)
template <int MAP>
__device__ __forceinline__ int out_row(int m, int b, int y, int x, int par, const Img& O) {
  if (MAP == M_U2) return (b * O.H + 2 * y + (par >> 1)) * O.W + 2 * x + (par & 1);
  return m;
}

// bijective XCD-aware remap of a 1-D block index (consecutive tiles -> the same XCD's L2)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// fixed-order chunk reduction (4 interleaved lanes) fused with the store to torch layout
// (kind 0: [co][ci][t], kind 1: [ci][co][t]): the reduced [T][CI][CO] element goes straight to dW
template <int DUMMY = 0>
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ part, int chunks, int kind, int CI,
                                                      int CO, int T, float* __restrict__ dW) {
  __shared__ double sh[4][64];
  const long long total = (long long)T * CI * CO;
  const int o = threadIdx.x & 63, q = threadIdx.x >> 6;
  const long long e = (long long)blockIdx.x * 64 + o;
  double s = 0.0;
  if (e < total) {
    // 8 chunks in flight per lane, predicated (no remainder loop that waits out one round trip per
    // chunk); same ascending order per lane, missing chunks add 0.0
    for (int c = q; c < chunks; c += 32) {
      float a[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {  // clamped address + select (a conditional load waits for itself)
        const float v = part[(long long)min(c + 4 * k, chunks - 1) * total + e];
        a[k] = c + 4 * k < chunks ? v : 0.0f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) s += (double)a[k];
    }
  }
  sh[q][o] = s;
  __syncthreads();
  if (q != 0 || e >= total) return;
  const float v = (float)(((sh[0][o] + sh[1][o]) + sh[2][o]) + sh[3][o]);
  const int t = (int)(e / ((long long)CI * CO));
  const int rem = (int)(e - (long long)t * CI * CO), ci = rem / CO, co = rem - ci * CO;
  if (kind == 0) dW[((size_t)co * CI + ci) * T + t] = v;
  else dW[((size_t)ci * CO + co) * T + t] = v;
}

// CUs of the current device (grid sizing in whole rounds of resident blocks)
inline int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

inline unsigned cdivu(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

}  // namespace dn
}  // namespace rpc
