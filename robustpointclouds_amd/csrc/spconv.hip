// a6: SECOND sparse middle encoder (upstream mmdet3d SparseEncoder over spconv) on gfx950.
//
// Sparse tensor = rows of features [N, C] (row-major) + coors [N, 4] (b, z, y, x).
//
// Rulebooks ("indice_key" in spconv) are neighbour maps built with a DENSE int32 index
// grid per resolution level: 288 GB of HBM makes a direct [B, D, H, W] table (2.2 GB at
// level 0 for B = 6) cheaper than hashing. The grid stays all -1 between calls: each
// builder scatters the row ids it needs and clears exactly those cells again.
//   SubM (stride 1, centred):   nbr[r, k] = row of coors[r] + (k - centre), or -1
//   SparseConv (strided):       output sites = { (c + pad - k) / stride } over inputs c and
//                               offsets k; ordered by their first candidate (i*K + k),
//                               found with an atomicMin on the grid and a scan — no sort,
//                               deterministic. nbr_out[o, k] = i and nbr_in[i, k] = o.
//
// Compute: output-stationary implicit GEMM on fp32 MFMA (v_mfma_f32_16x16x4_f32, exact
// k-ordered fma):  out[r, :] = sum_k A_k[r, :] . B_k, with A_k rows gathered by the
// neighbour map straight into LDS and transformed on load:
//   forward   A = relu(bn_prev(z_prev)) (or the raw VFE features), B = W[k] [CI, CO]
//   dgrad     A = dz = g*invstd*(dy - mean(dy) - xhat*mean(dy*xhat)), B = W[k]^T
// with offsets whose 64-row tile has no neighbour skipped. The epilogue writes z (pre-BN,
// kept for backward) and per-block BatchNorm partial sums; the dgrad epilogue applies the
// previous layer's ReLU mask and its BatchNorm-backward partial sums. Weight gradients
//   dW[k] = sum_r A_k[r, :]^T dz[r, :]
// are split over row chunks into partial slabs reduced in a fixed order. Nothing uses
// float atomics: results are bit-for-bit reproducible run to run.
#include <hipcub/hipcub.hpp>
#include <string.h>

#include <hip/hip_bf16.h>

#include "common.h"
#include "dense_common.h"

namespace rpc {
namespace sp {

constexpr int BLK = 256;
constexpr int BM = 64;      // rows per GEMM tile
constexpr int MAXK = 27;

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct Shape {
  int B, D, H, W;
};
struct KGeom {
  int k[3], s[3], p[3];
  int K;
};

__device__ __forceinline__ long long cell(const Shape& s, int b, int z, int y, int x) {
  return (((long long)b * s.D + z) * s.H + y) * s.W + x;
}

__global__ void k_grid_set(const int* __restrict__ coors, int N, Shape s, int* __restrict__ grid,
                           int clear) {
  int r = blockIdx.x * BLK + threadIdx.x;
  if (r >= N) return;
  const int* c = coors + 4 * r;
  grid[cell(s, c[0], c[1], c[2], c[3])] = clear ? -1 : r;
}

__global__ void k_subm_nbr(const int* __restrict__ coors, int N, Shape s, KGeom g,
                           const int* __restrict__ grid, int* __restrict__ nbr) {
  // 32-bit (row, offset) index: N * K < 2^31 is checked on the host
  const int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= N * g.K) return;
  const int r = t / g.K, k = t - r * g.K;
  int kx = k % g.k[2], ky = (k / g.k[2]) % g.k[1], kz = k / (g.k[2] * g.k[1]);
  const int* c = coors + 4 * r;
  int z = c[1] + kz - g.k[0] / 2, y = c[2] + ky - g.k[1] / 2, x = c[3] + kx - g.k[2] / 2;
  int v = -1;
  if (z >= 0 && z < s.D && y >= 0 && y < s.H && x >= 0 && x < s.W) v = grid[cell(s, c[0], z, y, x)];
  nbr[t] = v;
}

// output coordinate of input c through kernel offset k, or false
__device__ __forceinline__ bool out_of(const int* c, int k, const KGeom& g, const Shape& so, int& oz,
                                       int& oy, int& ox) {
  int kk[3] = {k / (g.k[2] * g.k[1]), (k / g.k[2]) % g.k[1], k % g.k[2]};
  int o[3];
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    int n = c[1 + a] + g.p[a] - kk[a];
    if (n < 0 || n % g.s[a]) return false;
    o[a] = n / g.s[a];
  }
  if (o[0] >= so.D || o[1] >= so.H || o[2] >= so.W) return false;
  oz = o[0];
  oy = o[1];
  ox = o[2];
  return true;
}

__global__ void k_cand_min(const int* __restrict__ coors, int N, KGeom g, Shape so,
                           unsigned* __restrict__ grid) {
  // 32-bit (row, offset) index: N * K < 2^31 is checked on the host
  const int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= N * g.K) return;
  const int r = t / g.K, k = t - r * g.K;
  const int* c = coors + 4 * r;
  int oz, oy, ox;
  if (!out_of(c, k, g, so, oz, oy, ox)) return;
  atomicMin(grid + cell(so, c[0], oz, oy, ox), (unsigned)t);
}

__global__ void k_cand_head(const int* __restrict__ coors, int N, KGeom g, Shape so,
                            const unsigned* __restrict__ grid, int* __restrict__ flag) {
  const int t = blockIdx.x * BLK + threadIdx.x;
  const int n = N * g.K;
  if (t == 0) flag[n] = 0;
  if (t >= n) return;
  const int r = t / g.K, k = t - r * g.K;
  const int* c = coors + 4 * r;
  int oz, oy, ox, f = 0;
  if (out_of(c, k, g, so, oz, oy, ox)) f = grid[cell(so, c[0], oz, oy, ox)] == (unsigned)t;
  flag[t] = f;
}

// Per-row forms of k_cand_head / k_out_assign: one thread per input row walks its K candidates in
// offset order, so the exclusive scan that numbers the output cells runs over N + 1 per-row head counts
// instead of N*K + 1 flags (the same first-appearance order: a cell's head is its smallest r*K + k).
// (the head offsets of each row are kept as a bit mask, K <= 27: the assign pass rewrites grid cells, so
// it cannot re-test them against candidate indices)
__global__ void k_row_heads(const int* __restrict__ coors, int N, KGeom g, Shape so, const unsigned* __restrict__ grid,
                            int* __restrict__ cnt, unsigned* __restrict__ hmask) {
  // 32 lanes per row, one per offset (K <= 27): the row's bits come out of the wave's ballot
  const long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  const int r = (int)(t >> 5), k = (int)(t & 31);
  if (r == N && k == 0) cnt[N] = 0;
  bool head = false;
  if (r < N && k < g.K) {
    const int* c = coors + 4 * r;
    int oz, oy, ox;
    head = out_of(c, k, g, so, oz, oy, ox) && grid[cell(so, c[0], oz, oy, ox)] == (unsigned)(r * g.K + k);
  }
  const unsigned m = (unsigned)(__ballot(head) >> (threadIdx.x & 32));
  if (r < N && k == 0) {
    cnt[r] = __popc(m);
    hmask[r] = m;
  }
}

__global__ void k_row_assign(const int* __restrict__ coors, int N, KGeom g, Shape so, const int* __restrict__ pos,
                             const unsigned* __restrict__ hmask, int* __restrict__ grid, int* __restrict__ coors_out) {
  const int r = blockIdx.x * BLK + threadIdx.x;
  if (r >= N) return;
  const int* c = coors + 4 * r;
  int o = pos[r];
  for (unsigned m = hmask[r]; m; m &= m - 1) {
    const int k = __ffs(m) - 1;
    int oz, oy, ox;
    out_of(c, k, g, so, oz, oy, ox);
    int* gc = grid + cell(so, c[0], oz, oy, ox);
    *gc = o;
    int* co = coors_out + 4 * o;
    co[0] = c[0];
    co[1] = oz;
    co[2] = oy;
    co[3] = ox;
    ++o;
  }
}

__global__ void k_out_assign(const int* __restrict__ coors, int N, KGeom g, Shape so,
                             const int* __restrict__ flag, const int* __restrict__ pos,
                             int* __restrict__ grid, int* __restrict__ coors_out) {
  const int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= N * g.K || !flag[t]) return;
  const int r = t / g.K, k = t - r * g.K;
  const int* c = coors + 4 * r;
  int oz, oy, ox;
  out_of(c, k, g, so, oz, oy, ox);
  int o = pos[t];
  grid[cell(so, c[0], oz, oy, ox)] = o;
  int* co = coors_out + 4 * o;
  co[0] = c[0];
  co[1] = oz;
  co[2] = oy;
  co[3] = ox;
}

__global__ void k_nbr_fill(const int* __restrict__ coors, int N, KGeom g, Shape so,
                           const int* __restrict__ grid, int* __restrict__ nbr_out,
                           int* __restrict__ nbr_in) {
  // 32-bit (row, offset) index: N * K < 2^31 is checked on the host
  const int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= N * g.K) return;
  const int r = t / g.K, k = t - r * g.K;
  const int* c = coors + 4 * r;
  int oz, oy, ox, o = -1;
  if (out_of(c, k, g, so, oz, oy, ox)) {
    o = grid[cell(so, c[0], oz, oy, ox)];
    nbr_out[(long long)o * g.K + k] = r;
  }
  nbr_in[t] = o;
}

// ------------------------------------------------------------------ implicit GEMM
enum { A_RAW = 0, A_BNRELU = 1, A_BNBWD = 2 };
enum { E_FWD = 0, E_DGRAD = 1, E_PLAIN = 2 };

struct GemmArgs {
  const float* a;       // A source rows [Nsrc, CI] (z of the previous layer, raw, or dy)
  const float* a2;      // A_BNBWD: z of the same layer [Nsrc, CI]
  const float* abn;     // A_BNRELU: scale[CI], beta[CI], mean[CI] (pre = (x - mean) * scale + beta);
                        // A_BNBWD : gi = g*invstd [CI], m1 [CI], m2 [CI], mean [CI], invstd [CI]
  const int* nbr;       // [Nout, K] neighbour map
  int K, rev;           // rev: use column K-1-k (SubM transpose)
  const float* W;       // [K][CIw][COw]
  int transW;           // B_k = W[k]^T (dgrad)
  int CIw, COw;         // weight dims as stored
  int Nout;
  float* out;           // [Nout, CO] (CO = real output width)
  int CO_real;
  // epilogue
  const float* ez;      // E_DGRAD: z of the output layer (previous layer in forward order) [Nout, CO]
  const float* ebn;     // E_DGRAD: scale, beta, mean, invstd of that layer [4*CO]
  float* part;          // [nblk][2*CO] partial column sums (may be null)
};

template <int CI, int CO, int AT, int ET>
__global__ __launch_bounds__(BLK) void k_gemm(GemmArgs g) {
  constexpr int CIP = (CI + 3) / 4 * 4;             // MFMA K steps of 4 (CI = 5: zero column 5..7)
  constexpr int AS = CIP + 2;                      // LDS row stride of A (bank spread)
  constexpr int BS = (CO % 32 == 0) ? CO + 16 : CO;
  constexpr int NT = CO / 16;
  __shared__ float sA[BM * AS];
  __shared__ float sB[CIP * BS];
  __shared__ int sN[BM * MAXK];
  __shared__ unsigned kmask;
  __shared__ float sP[4][2 * CO];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lb = dn::xcd_remap(blockIdx.x, gridDim.x);   // XCD-contiguous row blocks (L2-local gathers)
  const int r0 = lb * BM;
  const int K = g.K;
  if (tid == 0) kmask = 0;
  __syncthreads();
  unsigned my = 0;
  {
    // all of the thread's neighbour-index loads in flight before the first LDS store
    constexpr int PN = (BM * MAXK + BLK - 1) / BLK;
    int nv[PN];
#pragma unroll
    for (int i = 0; i < PN; ++i) {
      const int q = tid + i * BLK, r = q / K, k = q - r * K;
      const int kc = g.rev ? K - 1 - k : k;
      nv[i] = (q < BM * K && r0 + r < g.Nout) ? g.nbr[(long long)(r0 + r) * K + kc] : -1;
    }
#pragma unroll
    for (int i = 0; i < PN; ++i) {
      const int q = tid + i * BLK, r = q / K, k = q - r * K;
      if (q >= BM * K) continue;
      sN[r * MAXK + k] = nv[i];
      if (nv[i] >= 0) my |= 1u << k;
    }
  }
  if (my) atomicOr(&kmask, my);
  __syncthreads();
  const unsigned mask = kmask;
  f32x4 acc[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  constexpr int PA = (BM * CIP + BLK - 1) / BLK, PB = (CIP * CO + BLK - 1) / BLK;
  constexpr int GA = PA < 8 ? PA : 8, GB = PB < 8 ? PB : 8;   // loads in flight per group (registers)
  // two-level sums (r05): each offset's CI-term product is accumulated from zero and then added to the running
  // total, so a sum runs over ~CI/4 + K MFMA / add steps instead of K*CI/4 in one chain: the fp32 encoder output
  // went 2.1e-6 from float64 with one chain against torch-CPU fp32's 7.8e-7 (blocked sums), and the CenterPoint
  // step's gradients are conditioned enough to carry that 3x (tests/test_gpu_e2e_parity_centerpoint.py)
  auto mfma_k = [&]() {
    const float* pa = sA + (w * 16 + (lane & 15)) * AS + (lane >> 4);
    const float* pb = sB + (lane >> 4) * BS + (lane & 15);
    f32x4 c[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) c[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int kk = 0; kk < CIP / 4; ++kk) {
      float a = pa[kk * 4];
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        float b = pb[kk * 4 * BS + n * 16];
        c[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c[n], 0, 0, 0);
      }
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] += c[n];
  };
  if constexpr (PA <= 8 && PB <= 8) {
    // narrow layers (every register-held operand fits one group): the next offset's gathers and weight
    // tile are loaded into registers while the MFMAs of the current one run (one exposed round trip per
    // offset was the whole cost of these layers)
    float xa[PA], za[PA], wb[PB];
    auto load = [&](int k) {
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int q = tid + j * BLK, r = q / CIP, c = q - r * CIP;
        const int src = (q < BM * CIP && c < CI) ? sN[r * MAXK + k] : -1;
        xa[j] = src >= 0 ? g.a[(long long)src * CI + c] : 0.0f;
        za[j] = (AT == A_BNBWD && src >= 0) ? g.a2[(long long)src * CI + c] : 0.0f;
      }
      const float* Wk = g.W + (long long)k * g.CIw * g.COw;
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int q = tid + j * BLK, c = q / CO, n = q - c * CO;
        float v = 0.0f;
        if (q < CIP * CO) {
          if (!g.transW) { if (c < g.CIw && n < g.COw) v = Wk[c * g.COw + n]; }
          else { if (n < g.CIw && c < g.COw) v = Wk[n * g.COw + c]; }
        }
        wb[j] = v;
      }
    };
    auto stage = [&](int k) {
#pragma unroll
      for (int j = 0; j < PA; ++j) {
        const int q = tid + j * BLK, r = q / CIP, c = q - r * CIP;
        if (q >= BM * CIP) continue;
        const int src = c < CI ? sN[r * MAXK + k] : -1;
        float v = 0.0f;
        if (src >= 0) {
          const float x = xa[j];
          if (AT == A_BNRELU) v = fmaxf(fmaf(x - g.abn[2 * CI + c], g.abn[c], g.abn[CI + c]), 0.0f);
          else if (AT == A_BNBWD) {
            const float zz = za[j];
            const float xh = (zz - g.abn[3 * CI + c]) * g.abn[4 * CI + c];
            v = g.abn[c] * (x - g.abn[CI + c] - xh * g.abn[2 * CI + c]);
          } else v = x;
        }
        sA[r * AS + c] = v;
      }
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int q = tid + j * BLK, c = q / CO, n = q - c * CO;
        if (q < CIP * CO) sB[c * BS + n] = wb[j];
      }
    };
    auto next_k = [&](int k) {   // first offset > k with a neighbour in the block (K when none)
      const unsigned rest = k < 0 ? mask : (mask & ~((2u << k) - 1u));
      return rest ? __ffs(rest) - 1 : K;
    };
    int k = next_k(-1);
    if (k < K) load(k);
    while (k < K) {
      __syncthreads();   // the previous offset's MFMAs are done with sA / sB
      stage(k);
      __syncthreads();
      const int kn = next_k(k);
      if (kn < K) load(kn);
      mfma_k();
      k = kn;
    }
  } else {
    for (int k = 0; k < K; ++k) {
      if (!((mask >> k) & 1u)) continue;
      __syncthreads();
      // gather A_k (BM rows x CI, transformed on load) and B_k = W[k] (CI x CO) or W[k]^T (zero-padded
      // beyond the stored width): every global load of the thread is issued before the first LDS store
      // (as strided load -> store loops each load waited out its own round trip, ~5 per offset)
  #pragma unroll 1
      for (int i0 = 0; i0 < PA; i0 += GA) {
        float xa[GA], za[GA];
  #pragma unroll
        for (int j = 0; j < GA; ++j) {
          const int q = tid + (i0 + j) * BLK, r = q / CIP, c = q - r * CIP;
          const int src = (q < BM * CIP && c < CI) ? sN[r * MAXK + k] : -1;
          xa[j] = src >= 0 ? g.a[(long long)src * CI + c] : 0.0f;
          za[j] = (AT == A_BNBWD && src >= 0) ? g.a2[(long long)src * CI + c] : 0.0f;
        }
  #pragma unroll
        for (int j = 0; j < GA; ++j) {
          const int q = tid + (i0 + j) * BLK, r = q / CIP, c = q - r * CIP;
          if (q >= BM * CIP) continue;
          const int src = c < CI ? sN[r * MAXK + k] : -1;
          float v = 0.0f;
          if (src >= 0) {
            const float x = xa[j];
            if (AT == A_BNRELU) v = fmaxf(fmaf(x - g.abn[2 * CI + c], g.abn[c], g.abn[CI + c]), 0.0f);
            else if (AT == A_BNBWD) {
              const float zz = za[j];
              const float xh = (zz - g.abn[3 * CI + c]) * g.abn[4 * CI + c];
              v = g.abn[c] * (x - g.abn[CI + c] - xh * g.abn[2 * CI + c]);
            } else v = x;
          }
          sA[r * AS + c] = v;
        }
      }
      const float* Wk = g.W + (long long)k * g.CIw * g.COw;
  #pragma unroll 1
      for (int i0 = 0; i0 < PB; i0 += GB) {
        float wb[GB];
  #pragma unroll
        for (int j = 0; j < GB; ++j) {
          const int q = tid + (i0 + j) * BLK, c = q / CO, n = q - c * CO;
          float v = 0.0f;
          if (q < CIP * CO) {
            if (!g.transW) { if (c < g.CIw && n < g.COw) v = Wk[c * g.COw + n]; }
            else { if (n < g.CIw && c < g.COw) v = Wk[n * g.COw + c]; }
          }
          wb[j] = v;
        }
  #pragma unroll
        for (int j = 0; j < GB; ++j) {
          const int q = tid + (i0 + j) * BLK, c = q / CO, n = q - c * CO;
          if (q < CIP * CO) sB[c * BS + n] = wb[j];
        }
      }
      __syncthreads();
      mfma_k();
    }
  }
  // epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + reg
  float s1[NT], s2[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    s1[n] = s2[n] = 0.0f;
    int col = n * 16 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int row = r0 + w * 16 + (lane >> 4) * 4 + j;
      float v = acc[n][j];
      if (row < g.Nout && col < g.CO_real) {
        if (ET == E_DGRAD) {
          float zz = g.ez[(long long)row * CO + col];
          float h = fmaxf(fmaf(zz - g.ebn[2 * CO + col], g.ebn[col], g.ebn[CO + col]), 0.0f);
          v = h > 0.0f ? v : 0.0f;
          float xh = (zz - g.ebn[2 * CO + col]) * g.ebn[3 * CO + col];
          s1[n] += v;
          s2[n] += v * xh;
        } else {
          s1[n] += v;
          s2[n] += v * v;
        }
        g.out[(long long)row * g.CO_real + col] = v;
      }
    }
  }
  if (ET == E_PLAIN || g.part == nullptr) return;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    s1[n] += __shfl_xor(s1[n], 16, 64);
    s1[n] += __shfl_xor(s1[n], 32, 64);
    s2[n] += __shfl_xor(s2[n], 16, 64);
    s2[n] += __shfl_xor(s2[n], 32, 64);
    if (lane < 16) {
      sP[w][n * 16 + lane] = s1[n];
      sP[w][CO + n * 16 + lane] = s2[n];
    }
  }
  __syncthreads();
  for (int j = tid; j < 2 * CO; j += BLK)
    g.part[(long long)lb * 2 * CO + j] = sP[0][j] + sP[1][j] + sP[2][j] + sP[3][j];
}

// ------------------------------------------------------------------ weight gradient
// dW[k][c][n] = sum_r A_k[r, c] * D[r, n]; block = (row chunk, k). A_k gathered through
// nbr[:, k] with the forward A transform; D = dz of the output rows (BN backward on load).
struct WgradArgs {
  const float* a;     // forward A source [Nsrc, CI]
  const float* abn;   // forward A transform (A_BNRELU) scale, beta, mean
  const int* nbr;     // [Nout, K]
  int K, Nout, rows_per;
  const float* dy;    // [Nout, CO]
  const float* z;     // [Nout, CO]
  const float* dbn;   // gi, m1, m2, mean, invstd [5*CO]
  float* part;        // [chunks][K][CI][CO]
};

template <int CI, int CO, int AT>
__global__ __launch_bounds__(BLK) void k_wgrad(WgradArgs g) {
  // C[CI x CO] += A^T[CI x rows] D[rows x CO]; MFMA 16x16x4: M = CI, N = CO, K = rows
  constexpr int RT = 64;                     // rows per LDS tile
  constexpr int AS = CI + 4, DS = CO + 4;
  constexpr int MT = (CI + 15) / 16, NT = CO / 16;
  constexpr int TILES = MT * NT;
  constexpr int TPW = (TILES + 3) / 4;       // tiles per wave
  __shared__ float sA[RT * AS];
  __shared__ float sD[RT * DS];
  __shared__ int sN[RT];
  __shared__ int any;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int k = blockIdx.y, chunk = blockIdx.x;
  const int rb0 = chunk * g.rows_per, rb1 = min(g.Nout, rb0 + g.rows_per);
  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int rb = rb0; rb < rb1; rb += RT) {
    __syncthreads();
    if (tid == 0) any = 0;
    __syncthreads();
    if (tid < RT) {
      int r = rb + tid;
      int v = r < rb1 ? g.nbr[(long long)r * g.K + k] : -1;
      sN[tid] = v;
      if (v >= 0) any = 1;
    }
    __syncthreads();
    if (!any) continue;
    for (int q = tid; q < RT * CI; q += BLK) {
      int r = q / CI, c = q - r * CI;
      int src = sN[r];
      float v = 0.0f;
      if (src >= 0) {
        float x = g.a[(long long)src * CI + c];
        v = AT == A_BNRELU ? fmaxf(fmaf(x - g.abn[2 * CI + c], g.abn[c], g.abn[CI + c]), 0.0f) : x;
      }
      sA[r * AS + c] = v;
    }
    for (int q = tid; q < RT * CO; q += BLK) {
      int r = q / CO, n = q - r * CO;
      int row = rb + r;
      float v = 0.0f;
      if (row < rb1 && sN[r] >= 0) {
        float d = g.dy[(long long)row * CO + n];
        float zz = g.z[(long long)row * CO + n];
        float xh = (zz - g.dbn[3 * CO + n]) * g.dbn[4 * CO + n];
        v = g.dbn[n] * (d - g.dbn[CO + n] - xh * g.dbn[2 * CO + n]);
      }
      sD[r * DS + n] = v;
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      int tile = w + 4 * t;
      if (tile >= TILES) break;
      int m = tile / NT, n = tile - m * NT;
      int ci = m * 16 + (lane & 15);
      const float* pa = sA + (lane >> 4) * AS + (ci < CI ? ci : 0);
      const float* pd = sD + (lane >> 4) * DS + n * 16 + (lane & 15);
      f32x4 c = (f32x4){0.f, 0.f, 0.f, 0.f};   // two-level sums (as k_gemm): per 64-row tile, then the total
#pragma unroll 4
      for (int kk = 0; kk < RT / 4; ++kk) {
        float a = ci < CI ? pa[kk * 4 * AS] : 0.0f;
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, pd[kk * 4 * DS], c, 0, 0, 0);
      }
      acc[t] += c;
    }
  }
  float* out = g.part + ((long long)chunk * g.K + k) * CI * CO;
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    int tile = w + 4 * t;
    if (tile >= TILES) break;
    int m = tile / NT, n = tile - m * NT;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int ci = m * 16 + (lane >> 4) * 4 + j, col = n * 16 + (lane & 15);
      if (ci < CI) out[ci * CO + col] = acc[t][j];
    }
  }
}


// ------------------------------------------------------------------ BatchNorm finalize
// One block per channel c: every thread sums its strided share of the nblk partial rows of both
// columns c (sum) and C + c (sum of squares / of dy*xhat) with four rows in flight, then a
// fixed-order reduction (wave shuffles, then the four waves in order) in double; thread 0 writes
// the channel's parameters. No cross-block step (no ticket, no workspace):
// mode 0 (forward): bn = scale (= gamma*invstd), beta, mean, invstd ; running stats updated.
// mode 1 (backward): bnb = gi, m1, m2, mean, invstd ; dgamma, dbeta written.
template <typename P>
__global__ __launch_bounds__(BLK) void k_bn_finalize(const P* __restrict__ part, int nblk, int C, int N,
                                                     int mode, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     float mom, float* __restrict__ rmean,
                                                     float* __restrict__ rvar, const float* __restrict__ fbn,
                                                     float* __restrict__ bn, float* __restrict__ dgamma,
                                                     float* __restrict__ dbeta) {
  __shared__ double sh[2][BLK / 64];
  const int c = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long long C2 = 2 * C;
  double s1 = 0.0, s2 = 0.0;
  int r = threadIdx.x;
  for (; r + 3 * BLK < nblk; r += 4 * BLK) {
    const P* p = part + r * C2 + c;
    const P a0 = p[0], b0 = p[C], a1 = p[BLK * C2], b1 = p[BLK * C2 + C];
    const P a2 = p[2 * BLK * C2], b2 = p[2 * BLK * C2 + C], a3 = p[3 * BLK * C2], b3 = p[3 * BLK * C2 + C];
    s1 += (double)a0;
    s1 += (double)a1;
    s1 += (double)a2;
    s1 += (double)a3;
    s2 += (double)b0;
    s2 += (double)b1;
    s2 += (double)b2;
    s2 += (double)b3;
  }
  for (; r < nblk; r += BLK) {
    s1 += (double)part[r * C2 + c];
    s2 += (double)part[r * C2 + C + c];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if (lane == 0) {
    sh[0][w] = s1;
    sh[1][w] = s2;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  s1 = ((sh[0][0] + sh[0][1]) + sh[0][2]) + sh[0][3];
  s2 = ((sh[1][0] + sh[1][1]) + sh[1][2]) + sh[1][3];
  if (mode == 0) {
    const double mean = s1 / N;
    double var = s2 / N - mean * mean;
    if (var < 0) var = 0;
    const float invstd = 1.0f / sqrtf((float)var + eps);
    // BN applied as (z - mean) * scale + beta: no cancellation between z*scale and a shift
    bn[c] = gamma[c] * invstd;
    bn[C + c] = beta[c];
    bn[2 * C + c] = (float)mean;
    bn[3 * C + c] = invstd;
    const double uvar = N > 1 ? var * N / (N - 1) : var;
    rmean[c] = (1.0f - mom) * rmean[c] + mom * (float)mean;
    rvar[c] = (1.0f - mom) * rvar[c] + mom * (float)uvar;
  } else {
    // fbn: forward scale, beta, mean, invstd of this layer
    bn[c] = gamma[c] * fbn[3 * C + c];
    bn[C + c] = (float)(s1 / N);
    bn[2 * C + c] = (float)(s2 / N);
    bn[3 * C + c] = fbn[2 * C + c];
    bn[4 * C + c] = fbn[3 * C + c];
    if (dgamma) dgamma[c] = (float)s2;
    if (dbeta) dbeta[c] = (float)s1;
  }
}

// ------------------------------------------------------------------ dense BEV
// forward: dense[b, c*D + z, y, x] = relu(bn(z_rows[r, c])) ; backward: gather + ReLU mask +
// BatchNorm-backward partial sums (one 64-row tile per block, like the GEMM epilogue)
// dense index of (row coords, channel c): NCHW [B][C*D][H][W] (channel c*D + z) or NHWC
// [B][H][W][C*D] (the channels_last image the MIOpen NHWC convolutions consume directly)
template <bool NHWC>
__device__ __forceinline__ long long dense_index(const int* co, int c, int C, const Shape& s) {
  if (NHWC) return (((long long)co[0] * s.H + co[2]) * s.W + co[3]) * ((long long)C * s.D) + (long long)c * s.D + co[1];
  return (((long long)co[0] * C + c) * s.D + co[1]) * s.H * s.W + (long long)co[2] * s.W + co[3];
}

__device__ __forceinline__ void store_val(float* p, float v) { *p = v; }
__device__ __forceinline__ void store_val(__hip_bfloat16* p, float v) { *p = __float2bfloat16(v); }
__device__ __forceinline__ float load_val(const float* p) { return *p; }
__device__ __forceinline__ float load_val(const __hip_bfloat16* p) { return __bfloat162float(*p); }

template <typename T, bool NHWC>
__global__ __launch_bounds__(BLK) void k_to_dense(const float* __restrict__ z, const float* __restrict__ bn,
                                                  const int* __restrict__ coors, int N, int C, Shape s,
                                                  T* __restrict__ dense) {
  long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  if (t >= (long long)N * C) return;
  int r = (int)(t / C), c = (int)(t - (long long)r * C);
  float h = fmaxf(fmaf(z[t] - bn[2 * C + c], bn[c], bn[C + c]), 0.0f);
  store_val(dense + dense_index<NHWC>(coors + 4 * r, c, C, s), h);
}

constexpr int FBLK = 1024;   // k_from_dense: 1024 threads = 1024 / C row lanes over the block's 64 rows
// C % 4 == 0 form: 4 channels of a row per thread, float4 operand loads, 32-bit indexing (the scalar
// form's time went to a 64-bit division per element); same arithmetic per element
template <typename T, bool NHWC>
__global__ __launch_bounds__(BLK) void k_to_dense_v4(const float* __restrict__ z, const float* __restrict__ bn,
                                                     const int* __restrict__ coors, int N, int C, Shape s,
                                                     T* __restrict__ dense) {
  const int C4 = C >> 2;
  const int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= N * C4) return;
  const int r = t / C4, c = (t - r * C4) * 4;
  const float4 zv = *(const float4*)(z + (size_t)r * C + c);
  const float4 mu = *(const float4*)(bn + 2 * C + c), sc = *(const float4*)(bn + c), be = *(const float4*)(bn + C + c);
  const float zz[4] = {zv.x, zv.y, zv.z, zv.w}, m[4] = {mu.x, mu.y, mu.z, mu.w}, a[4] = {sc.x, sc.y, sc.z, sc.w},
              b[4] = {be.x, be.y, be.z, be.w};
  const int4 co = *(const int4*)(coors + 4 * r);
  const int cr[4] = {co.x, co.y, co.z, co.w};
#pragma unroll
  for (int j = 0; j < 4; ++j)
    store_val(dense + dense_index<NHWC>(cr, c + j, C, s), fmaxf(fmaf(zz[j] - m[j], a[j], b[j]), 0.0f));
}
// the cells k_to_dense_v4 wrote for these coordinates set back to 0 (rpc_sparse_dense_clear): a persistent
// dense image is re-cleared where the previous step scattered instead of zero-filled whole
template <typename T, bool NHWC>
__global__ __launch_bounds__(BLK) void k_dense_clear_v4(const int* __restrict__ coors, int N, int C, Shape s,
                                                        T* __restrict__ dense) {
  const int C4 = C >> 2;
  const int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= N * C4) return;
  const int r = t / C4, c = (t - r * C4) * 4;
  const int4 co = *(const int4*)(coors + 4 * r);
  const int cr[4] = {co.x, co.y, co.z, co.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) store_val(dense + dense_index<NHWC>(cr, c + j, C, s), 0.0f);
}
// any C / any N (rpc_sparse_dense_clear when C % 4 != 0 or N * C / 4 does not fit an int): one element per thread,
// 64-bit element index, like k_to_dense's scalar form
template <typename T, bool NHWC>
__global__ __launch_bounds__(BLK) void k_dense_clear(const int* __restrict__ coors, long long N, int C, Shape s,
                                                     T* __restrict__ dense) {
  const long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  if (t >= N * C) return;
  const long long r = t / C;
  const int c = (int)(t - r * C);
  const int cr[4] = {coors[4 * r], coors[4 * r + 1], coors[4 * r + 2], coors[4 * r + 3]};
  store_val(dense + dense_index<NHWC>(cr, c, C, s), 0.0f);
}
template <typename T, bool NHWC>
__global__ __launch_bounds__(FBLK) void k_from_dense(const T* __restrict__ gd, const float* __restrict__ z,
                                                    const float* __restrict__ bn, const int* __restrict__ coors,
                                                    int N, int C, Shape s, float* __restrict__ dy,
                                                    float* __restrict__ part) {
  // block: BM rows; threads laid out (row lane, channel) so that each row's gather and the dy
  // store are coalesced; row lanes combined in lane order (C <= 256)
  __shared__ float sh[2][FBLK];
  const int r0 = blockIdx.x * BM, r1 = min(N, r0 + BM);
  const int nl = FBLK / C;                       // >= 1 row lanes
  const int rl = threadIdx.x / C, c = threadIdx.x - rl * C;
  float s1 = 0.0f, s2 = 0.0f;
  if (rl < nl) {
    const float mu = bn[2 * C + c], sc = bn[c], sh0 = bn[C + c], is = bn[3 * C + c];
    // four rows per round: their z values and dense gathers are in flight together
    constexpr int RR = 4;
    for (int rb = r0 + rl; rb < r1; rb += RR * nl) {
      float zz[RR], gv[RR];
#pragma unroll
      for (int u = 0; u < RR; ++u) {
        const int r = rb + u * nl;
        zz[u] = r < r1 ? z[(long long)r * C + c] : 0.0f;
        gv[u] = r < r1 ? load_val(gd + dense_index<NHWC>(coors + 4 * r, c, C, s)) : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < RR; ++u) {
        const int r = rb + u * nl;
        if (r >= r1) continue;
        const float h = fmaxf(fmaf(zz[u] - mu, sc, sh0), 0.0f);
        const float v = h > 0.0f ? gv[u] : 0.0f;
        dy[(long long)r * C + c] = v;
        s1 += v;
        s2 += v * ((zz[u] - mu) * is);
      }
    }
  }
  sh[0][threadIdx.x] = s1;
  sh[1][threadIdx.x] = s2;
  __syncthreads();
  if (rl == 0) {
    float t1 = sh[0][c], t2 = sh[1][c];
    for (int k = 1; k < nl; ++k) {
      t1 += sh[0][k * C + c];
      t2 += sh[1][k * C + c];
    }
    part[(long long)blockIdx.x * 2 * C + c] = t1;
    part[(long long)blockIdx.x * 2 * C + C + c] = t2;
  }
}

// fp16 rows: finite values beyond the fp16 range saturate to +-65504 (inf / NaN pass through)
__device__ __forceinline__ float sat_f16(float f) {
  return (fabsf(f) > 65504.0f && fabsf(f) < __builtin_inff()) ? copysignf(65504.0f, f) : f;
}

// ------------------------------------------------------------------ SparseBasicBlock residual
// forward: out = relu(bn(z) + res) (res optional), fp32 rows and optionally bf16 rows [n][round8(C)]
// (upstream mmdet3d SparseBasicBlock.forward: norm2, + identity, relu; also materialises a plain
// relu(bn(z)) output that a block reads as its identity)
template <int FMT>   // hb: bf16 (0) or fp16 (1) rows
__global__ __launch_bounds__(BLK) void k_res_fwd(const float* __restrict__ z, const float* __restrict__ bn,
                                                 const float* __restrict__ res, int N, int C, int CP,
                                                 float* __restrict__ out, unsigned short* __restrict__ hb,
                                                 unsigned short* __restrict__ hb2) {
  const long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  if (t >= (long long)N * CP) return;
  const int r = (int)(t / CP), c = (int)(t - (long long)r * CP);
  float v = 0.0f;
  if (c < C) {
    const long long i = (long long)r * C + c;
    v = fmaf(z[i] - bn[2 * C + c], bn[c], bn[C + c]);
    if (res) v = v + res[i];
    v = fmaxf(v, 0.0f);
    out[i] = v;
  }
  if (hb) {
    if (FMT) {
      _Float16 h = (_Float16)sat_f16(v);
      hb[t] = __builtin_bit_cast(unsigned short, h);
      if (hb2) {
        __bf16 b = (__bf16)v;
        hb2[t] = __builtin_bit_cast(unsigned short, b);
      }
    } else {
      __bf16 b = (__bf16)v;
      hb[t] = __builtin_bit_cast(unsigned short, b);
    }
  }
}

// the same for C % 8 == 0, one thread per (row, 8 channels): two 16-byte loads per operand, one 16-byte
// store per 16-bit row image, 32-bit index math (the per-element kernel above divided a 64-bit index per
// element and moved 4 bytes per access: 74 us per 128-channel CenterPoint layer). Same arithmetic per
// element, so the same bits.
template <int FMT>
__global__ __launch_bounds__(BLK) void k_res_fwd_v8(const float* __restrict__ z, const float* __restrict__ bn,
                                                    const float* __restrict__ res, int N, int C,
                                                    float* __restrict__ out, unsigned short* __restrict__ hb,
                                                    unsigned short* __restrict__ hb2) {
  const int G = C >> 3;
  const int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= N * G) return;
  const int r = t / G, cg = t - r * G, c0 = cg * 8;
  const int i = r * C + c0;
  float zv[8], rv[8], v[8];
  *(float4*)&zv[0] = *(const float4*)(z + i);
  *(float4*)&zv[4] = *(const float4*)(z + i + 4);
  if (res) {
    *(float4*)&rv[0] = *(const float4*)(res + i);
    *(float4*)&rv[4] = *(const float4*)(res + i + 4);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = c0 + j;
    float x = fmaf(zv[j] - bn[2 * C + c], bn[c], bn[C + c]);
    if (res) x = x + rv[j];
    v[j] = fmaxf(x, 0.0f);
  }
  *(float4*)(out + i) = *(const float4*)&v[0];
  *(float4*)(out + i + 4) = *(const float4*)&v[4];
  if (hb) {
    unsigned short h[8], b2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (FMT) {
        h[j] = __builtin_bit_cast(unsigned short, (_Float16)sat_f16(v[j]));
        b2[j] = __builtin_bit_cast(unsigned short, (__bf16)v[j]);
      } else {
        h[j] = __builtin_bit_cast(unsigned short, (__bf16)v[j]);
      }
    }
    *(uint4*)(hb + i) = *(const uint4*)h;
    if (FMT && hb2) *(uint4*)(hb2 + i) = *(const uint4*)b2;
  }
}

// backward: m = (g1 + g2) * (out > 0) and the BatchNorm-backward partial sums of the layer that
// produced z (sum m, sum m * xhat) per BM rows, laid out like k_from_dense (C <= 256)
__global__ __launch_bounds__(BLK) void k_res_bwd(const float* __restrict__ g1, const float* __restrict__ g2,
                                                 const float* __restrict__ out, const float* __restrict__ z,
                                                 const float* __restrict__ bn, int N, int C,
                                                 float* __restrict__ m, float* __restrict__ part) {
  __shared__ float sh[2][BLK];
  const int r0 = blockIdx.x * BM, r1 = min(N, r0 + BM);
  const int nl = BLK / C;
  const int rl = threadIdx.x / C, c = threadIdx.x - rl * C;
  float s1 = 0.0f, s2 = 0.0f;
  if (rl < nl) {
    const float mu = bn[2 * C + c], is = bn[3 * C + c];
    for (int r = r0 + rl; r < r1; r += nl) {
      const long long i = (long long)r * C + c;
      float g = g1[i];
      if (g2) g = g + g2[i];
      const float v = out[i] > 0.0f ? g : 0.0f;
      m[i] = v;
      s1 += v;
      s2 += v * ((z[i] - mu) * is);
    }
  }
  sh[0][threadIdx.x] = s1;
  sh[1][threadIdx.x] = s2;
  __syncthreads();
  if (rl == 0) {
    float t1 = sh[0][c], t2 = sh[1][c];
    for (int k = 1; k < nl; ++k) {
      t1 += sh[0][k * C + c];
      t2 += sh[1][k * C + c];
    }
    part[(long long)blockIdx.x * 2 * C + c] = t1;
    part[(long long)blockIdx.x * 2 * C + C + c] = t2;
  }
}


// the same for C % 4 == 0 (C <= 128): thread = (row lane, 4 channels) with 16-byte accesses and 8 rows per
// thread, all 8 rows' loads in flight; a block covers 8 * BLK / (C / 4) rows = one or more BM-row partial
// groups (the layout rpc_bn_finalize reads). Partial sums: shuffles over the row lanes of a wave (fixed xor
// order), then the 4 waves in order through LDS — deterministic. (One row per thread and one LDS
// reduction per 64 rows ran the 16-channel CenterPoint layers at ~1.1 TB/s.)
__global__ __launch_bounds__(BLK) void k_res_bwd_v4(const float* __restrict__ g1, const float* __restrict__ g2,
                                                    const float* __restrict__ out, const float* __restrict__ z,
                                                    const float* __restrict__ bn, int N, int C,
                                                    float* __restrict__ m, float* __restrict__ part) {
  constexpr int RPT = 8;                                 // rows per thread
  __shared__ float sh[2][RPT][BLK / 64][128];
  const int Q = C >> 2, nl = BLK / Q;                    // row lanes per pass
  const int rows_blk = RPT * nl, ng = rows_blk / BM;     // rows and BM-row partial groups per block
  const int rb = blockIdx.x * rows_blk;
  const int rl = threadIdx.x / Q, cq = threadIdx.x - rl * Q, c0 = cq * 4;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float4 mu4 = *(const float4*)(bn + 2 * C + c0), is4 = *(const float4*)(bn + 3 * C + c0);
  const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w}, is[4] = {is4.x, is4.y, is4.z, is4.w};
  float4 ga[RPT], gb[RPT], o[RPT], zz[RPT];
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = rb + rl + nl * j;
    const int i = (r < N ? r : 0) * C + c0;
    ga[j] = *(const float4*)(g1 + i);
    gb[j] = g2 ? *(const float4*)(g2 + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    o[j] = *(const float4*)(out + i);
    zz[j] = *(const float4*)(z + i);
  }
  float s1[RPT][4], s2[RPT][4];   // per row slot; slots of one BM group are combined below
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int r = rb + rl + nl * j;
    const float gg[4] = {ga[j].x + gb[j].x, ga[j].y + gb[j].y, ga[j].z + gb[j].z, ga[j].w + gb[j].w};
    const float oo[4] = {o[j].x, o[j].y, o[j].z, o[j].w}, zv[4] = {zz[j].x, zz[j].y, zz[j].z, zz[j].w};
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = (r < N && oo[q] > 0.0f) ? gg[q] : 0.0f;
      s1[j][q] = v[q];
      s2[j][q] = v[q] * ((zv[q] - mu[q]) * is[q]);
    }
    if (r < N) *(float4*)(m + r * C + c0) = make_float4(v[0], v[1], v[2], v[3]);
  }
  // row slot j of this thread lies in group (nl * j) / BM; sum the slots of each group in slot order
  float t1[RPT][4], t2[RPT][4];
#pragma unroll
  for (int g = 0; g < RPT; ++g)
#pragma unroll
    for (int q = 0; q < 4; ++q) t1[g][q] = t2[g][q] = 0.0f;
#pragma unroll
  for (int j = 0; j < RPT; ++j) {
    const int g = (nl * j) / BM;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      t1[g][q] += s1[j][q];
      t2[g][q] += s2[j][q];
    }
  }
  // over the row lanes of the wave (lanes differing in the bits above log2(Q)), fixed xor order
#pragma unroll
  for (int g = 0; g < RPT; ++g) {
    if (g >= ng) continue;   // uniform
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      for (int msk = Q; msk < 64; msk <<= 1) {
        t1[g][q] += __shfl_xor(t1[g][q], msk, 64);
        t2[g][q] += __shfl_xor(t2[g][q], msk, 64);
      }
    }
  }
  if (lane < Q) {
#pragma unroll
    for (int g = 0; g < RPT; ++g) {
      if (g >= ng) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        sh[0][g][w][c0 + q] = t1[g][q];
        sh[1][g][w][c0 + q] = t2[g][q];
      }
    }
  }
  __syncthreads();
  const int gb0 = blockIdx.x * ng, ngr = (N + BM - 1) / BM;
  for (int e = threadIdx.x; e < ng * C; e += BLK) {
    const int g = e / C, c = e - g * C;
    if (gb0 + g >= ngr) continue;
    float a1 = 0.0f, a2 = 0.0f;
    for (int ww = 0; ww < BLK / 64; ++ww) {
      a1 += sh[0][g][ww][c];
      a2 += sh[1][g][ww][c];
    }
    part[(long long)(gb0 + g) * 2 * C + c] = a1;
    part[(long long)(gb0 + g) * 2 * C + C + c] = a2;
  }
}

// Weight gradient of the narrow input layer (CI * CO <= 128, the 4/5 -> 16 conv_input): every
// block takes a chunk of rows for ALL K offsets, so the BatchNorm-backward dz tile is formed once
// (not once per offset) and the K gathered x tiles sit side by side in LDS. Thread (k, ci, half)
// keeps the CO sums of dW[k][ci][:] in registers over its half of the tile rows; the dz row it
// reads is the same for all lanes of the wave (an LDS broadcast).
// NT threads: one (k, ci, half) triple each (512 for CI = 5: 27 x 5 x 2 = 270 > 256)
template <int CI, int CO, int AT>
constexpr int wn_threads() { return MAXK * CI * 2 <= BLK ? BLK : 2 * BLK; }
template <int CI, int CO, int AT, int NT = wn_threads<CI, CO, AT>()>
__global__ __launch_bounds__(NT) void k_wgrad_narrow(WgradArgs g) {
  constexpr int RT = 64;
  __shared__ __attribute__((aligned(16))) float sA[MAXK * RT * CI];
  __shared__ __attribute__((aligned(16))) float sD[RT * CO];
  __shared__ int sN[RT * MAXK];
  __shared__ float sH[NT / 2][CO];
  const int tid = threadIdx.x, K = g.K;
  const int rb0 = blockIdx.x * g.rows_per, rb1 = min(g.Nout, rb0 + g.rows_per);
  const int pair = tid >> 1, half = tid & 1;          // (k, ci) pair, row parity
  const int kk = pair / CI, ci = pair - kk * CI;
  const bool own = pair < K * CI;
  float acc[CO];
#pragma unroll
  for (int n = 0; n < CO; ++n) acc[n] = 0.f;
  // every staging loop below issues all of its thread's global loads before the first LDS store (one
  // round trip per phase; as plain strided loops each load waited for the store before it: ~18 exposed
  // latencies per 64-row sub-tile)
  constexpr int PN = (RT * MAXK + NT - 1) / NT, PD = (RT * CO + NT - 1) / NT;
  for (int rb = rb0; rb < rb1; rb += RT) {
    __syncthreads();
    {
      int nv[PN];
#pragma unroll
      for (int i = 0; i < PN; ++i) {
        const int q = tid + i * NT;
        const int r = q / K, k = q - r * K, row = rb + r;
        nv[i] = (q < RT * K && row < rb1) ? g.nbr[(long long)row * K + k] : -1;
      }
#pragma unroll
      for (int i = 0; i < PN; ++i)
        if (tid + i * NT < RT * K) sN[tid + i * NT] = nv[i];
      float dv[PD], zv[PD];
#pragma unroll
      for (int i = 0; i < PD; ++i) {
        const int q = tid + i * NT, r = q / CO, n = q - r * CO, row = rb + r;
        const bool ok = q < RT * CO && row < rb1;
        dv[i] = ok ? g.dy[(long long)row * CO + n] : 0.0f;
        zv[i] = ok ? g.z[(long long)row * CO + n] : 0.0f;
      }
#pragma unroll
      for (int i = 0; i < PD; ++i) {
        const int q = tid + i * NT, r = q / CO, n = q - r * CO, row = rb + r;
        if (q >= RT * CO) continue;
        float v = 0.0f;
        if (row < rb1) {
          const float xh = (zv[i] - g.dbn[3 * CO + n]) * g.dbn[4 * CO + n];
          v = g.dbn[n] * (dv[i] - g.dbn[CO + n] - xh * g.dbn[2 * CO + n]);
        }
        sD[q] = v;
      }
    }
    __syncthreads();
    if (CI == 4) {   // one 16-B gather per (offset, row)
      float4 gv[PN];
#pragma unroll
      for (int i = 0; i < PN; ++i) {
        const int q = tid + i * NT, k = q / RT, r = q - k * RT;
        const int src = q < K * RT ? sN[r * K + k] : -1;
        gv[i] = src >= 0 ? *(const float4*)(g.a + (long long)src * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int i = 0; i < PN; ++i) {
        const int q = tid + i * NT;
        if (q >= K * RT) continue;
        const int k = q / RT, r = q - k * RT;
        float4 v = gv[i];
        if (AT == A_BNRELU && sN[r * K + k] >= 0) {
          v.x = fmaxf(fmaf(v.x - g.abn[8], g.abn[0], g.abn[4]), 0.0f);
          v.y = fmaxf(fmaf(v.y - g.abn[9], g.abn[1], g.abn[5]), 0.0f);
          v.z = fmaxf(fmaf(v.z - g.abn[10], g.abn[2], g.abn[6]), 0.0f);
          v.w = fmaxf(fmaf(v.w - g.abn[11], g.abn[3], g.abn[7]), 0.0f);
        }
        *(float4*)&sA[q * 4] = v;
      }
    } else {
      for (int q = tid; q < K * RT * CI; q += NT) {
        const int k = q / (RT * CI), rem = q - k * (RT * CI), r = rem / CI, c = rem - r * CI;
        const int src = sN[r * K + k];
        float v = 0.0f;
        if (src >= 0) {
          const float x = g.a[(long long)src * CI + c];
          v = AT == A_BNRELU ? fmaxf(fmaf(x - g.abn[2 * CI + c], g.abn[c], g.abn[CI + c]), 0.0f) : x;
        }
        sA[q] = v;
      }
    }
    __syncthreads();
    if (own) {
      const float* pa = sA + kk * RT * CI + ci;
#pragma unroll 4
      for (int r = half; r < RT; r += 2) {
        const float a = pa[r * CI];
        const float4* pd = (const float4*)(sD + r * CO);
#pragma unroll
        for (int n4 = 0; n4 < CO / 4; ++n4) {
          const float4 d = pd[n4];
          acc[4 * n4 + 0] = fmaf(a, d.x, acc[4 * n4 + 0]);
          acc[4 * n4 + 1] = fmaf(a, d.y, acc[4 * n4 + 1]);
          acc[4 * n4 + 2] = fmaf(a, d.z, acc[4 * n4 + 2]);
          acc[4 * n4 + 3] = fmaf(a, d.w, acc[4 * n4 + 3]);
        }
      }
    }
  }
  // fixed-order combine of the two row parities
  __syncthreads();
  if (half == 1) {
#pragma unroll
    for (int n = 0; n < CO; ++n) sH[pair][n] = acc[n];
  }
  __syncthreads();
  if (half == 0 && own) {
    float* out = g.part + ((long long)blockIdx.x * K + kk) * CI * CO + ci * CO;
#pragma unroll
    for (int n = 0; n < CO; ++n) out[n] = acc[n] + sH[pair][n];
  }
}

// ------------------------------------------------------------------ narrow input layer (conv_input, CI 4 / 5 -> 16)
// The fp32 input layer as row passes instead of the 16 x 16 MFMA GEMM (4 of whose 16 K columns were real and
// which walked the K offsets one barrier pair each: 21.8 / 76 us forward, 52 / 194 us data gradient on the
// metric's / CenterPoint's layer 0). Block = 64 rows (one BatchNorm partial row, the GEMM's BM), thread = (row,
// quarter q of the 16 output / dz channels); the block's neighbour indices and the K weight taps are staged in
// LDS once; the gathers go out 9 offsets at a time with unconditional (clamped) loads, so each thread waits
// three round trips instead of one per offset. Per offset the CI (forward) / 4-channel (data gradient)
// products are summed first and then added to the running total (the GEMM's two-level order).
constexpr int L0R = 64, L0T = 256, L0G = 9;   // rows per block (= BM), threads, offsets per gather group
template <int CI>
__global__ __launch_bounds__(L0T) void k_l0_fwd(const float* __restrict__ x, const int* __restrict__ nbr, int K,
                                                const float* __restrict__ W, int n_out, float* __restrict__ z,
                                                float* __restrict__ part) {
  constexpr int CO = 16;
  __shared__ float sW[MAXK * CI * CO];
  __shared__ int sN[L0R * MAXK];
  __shared__ float sP[L0T / 64][2][CO];
  const int tid = threadIdx.x, r = tid >> 2, q = tid & 3, lane = tid & 63, w = tid >> 6;
  const int r0 = blockIdx.x * L0R, nr = min(L0R, n_out - r0);
  for (int i = tid; i < K * CI * CO; i += L0T) sW[i] = W[i];
  for (int i = tid; i < L0R * K; i += L0T) sN[i] = i < nr * K ? nbr[(long long)r0 * K + i] : -1;
  __syncthreads();
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += L0G) {
    int src[L0G];
    float xv[L0G][CI];
#pragma unroll
    for (int u = 0; u < L0G; ++u) {
      src[u] = k0 + u < K ? sN[r * K + k0 + u] : -1;
      const long long s = src[u] < 0 ? 0 : src[u];
#pragma unroll
      for (int c = 0; c < CI; ++c) xv[u][c] = x[s * CI + c];
    }
#pragma unroll
    for (int u = 0; u < L0G; ++u) {
      if (src[u] < 0) continue;
      const float* wk = sW + (k0 + u) * CI * CO + q * 4;
      float t[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < CI; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) t[j] = fmaf(xv[u][c], wk[c * CO + j], t[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] += t[j];
    }
  }
  const bool live = r < nr;
  if (live) *(float4*)(z + (long long)(r0 + r) * CO + q * 4) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  if (part == nullptr) return;
  float s1[4], s2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s1[j] = live ? acc[j] : 0.f;
    s2[j] = live ? acc[j] * acc[j] : 0.f;
  }
#pragma unroll
  for (int o = 4; o < 64; o <<= 1)   // the wave's 16 rows of this quarter, fixed xor order
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s1[j] += __shfl_xor(s1[j], o, 64);
      s2[j] += __shfl_xor(s2[j], o, 64);
    }
  if (lane < 4) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sP[w][0][q * 4 + j] = s1[j];
      sP[w][1][q * 4 + j] = s2[j];
    }
  }
  __syncthreads();
  if (tid < 2 * CO) {
    const int which = tid / CO, c = tid - which * CO;
    part[(long long)blockIdx.x * 2 * CO + tid] =
        ((sP[0][which][c] + sP[1][which][c]) + sP[2][which][c]) + sP[3][which][c];
  }
}

// data gradient of the input layer: din[r][n] = sum_k sum_o dz[nbr(r, k)][o] W[k][n][o] (n < CI), dz formed on
// load from (dy, z, bnb) of the 16-channel layer as k_gemm's A_BNBWD does; thread (row, quarter q of the 16 dz
// channels), the 4 quarters added in a fixed xor order
template <int CI>
__global__ __launch_bounds__(L0T) void k_l0_dgrad(const float* __restrict__ dy, const float* __restrict__ zz,
                                                  const float* __restrict__ bnb, const int* __restrict__ nbr, int K,
                                                  int rev, const float* __restrict__ W, int n_in,
                                                  float* __restrict__ din) {
  constexpr int CO = 16;
  __shared__ float sW[MAXK * CI * CO];
  __shared__ int sN[L0R * MAXK];
  const int tid = threadIdx.x, r = tid >> 2, q = tid & 3;
  const int r0 = blockIdx.x * L0R, nr = min(L0R, n_in - r0);
  for (int i = tid; i < K * CI * CO; i += L0T) sW[i] = W[i];
  for (int i = tid; i < L0R * K; i += L0T) {
    const int rr = i / K, k = i - rr * K;
    sN[i] = rr < nr ? nbr[(long long)(r0 + rr) * K + (rev ? K - 1 - k : k)] : -1;
  }
  float gi[4], m1[4], m2[4], mu[4], is[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int c = q * 4 + j;
    gi[j] = bnb[c];
    m1[j] = bnb[CO + c];
    m2[j] = bnb[2 * CO + c];
    mu[j] = bnb[3 * CO + c];
    is[j] = bnb[4 * CO + c];
  }
  __syncthreads();
  float acc[CI];
#pragma unroll
  for (int n = 0; n < CI; ++n) acc[n] = 0.f;
  for (int k0 = 0; k0 < K; k0 += L0G) {
    int src[L0G];
    float4 dv[L0G], zv[L0G];
#pragma unroll
    for (int u = 0; u < L0G; ++u) {
      src[u] = k0 + u < K ? sN[r * K + k0 + u] : -1;
      const long long s = src[u] < 0 ? 0 : src[u];
      dv[u] = *(const float4*)(dy + s * CO + q * 4);
      zv[u] = *(const float4*)(zz + s * CO + q * 4);
    }
#pragma unroll
    for (int u = 0; u < L0G; ++u) {
      if (src[u] < 0) continue;
      const float d4[4] = {dv[u].x, dv[u].y, dv[u].z, dv[u].w}, z4[4] = {zv[u].x, zv[u].y, zv[u].z, zv[u].w};
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xh = (z4[j] - mu[j]) * is[j];
        v[j] = gi[j] * (d4[j] - m1[j] - xh * m2[j]);
      }
      const float* wk = sW + (k0 + u) * CI * CO + q * 4;
#pragma unroll
      for (int n = 0; n < CI; ++n) {
        float t = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) t = fmaf(v[j], wk[n * CO + j], t);
        acc[n] += t;
      }
    }
  }
#pragma unroll
  for (int n = 0; n < CI; ++n) {
    acc[n] += __shfl_xor(acc[n], 1, 64);
    acc[n] += __shfl_xor(acc[n], 2, 64);
  }
  if (q == 0 && r < nr) {
#pragma unroll
    for (int n = 0; n < CI; ++n) din[(long long)(r0 + r) * CI + n] = acc[n];
  }
}

// ------------------------------------------------------------------ dispatch
template <int CI, int CO>
static void launch_gemm_t(int at, int et, const GemmArgs& a, int nblk, hipStream_t st) {
#define G(AT, ET) hipLaunchKernelGGL((k_gemm<CI, CO, AT, ET>), dim3(nblk), dim3(BLK), 0, st, a)
  if (at == A_RAW && et == E_FWD) G(A_RAW, E_FWD);
  else if (at == A_BNRELU && et == E_FWD) G(A_BNRELU, E_FWD);
  else if (at == A_BNBWD && et == E_DGRAD) G(A_BNBWD, E_DGRAD);
  else if (at == A_BNBWD && et == E_PLAIN) G(A_BNBWD, E_PLAIN);
#undef G
}

static int launch_gemm(int CI, int CO, int at, int et, const GemmArgs& a, int nblk, hipStream_t st) {
#define C2(ci, co) if (CI == ci && CO == co) { launch_gemm_t<ci, co>(at, et, a, nblk, st); return RPC_OK; }
  // forward pairs (CI, CO) of SparseEncoder and their dgrad transposes (CO, CI->pad16)
  C2(4, 16) C2(5, 16) C2(16, 16) C2(16, 32) C2(32, 32) C2(32, 64) C2(64, 64) C2(64, 128)
  C2(32, 16) C2(64, 32) C2(128, 64)
  C2(64, 16) C2(16, 64)   // 64-channel voxel features (HardVFE [.., 64]) into conv_input, and its dgrad
  C2(128, 128)            // nuScenes CenterPoint encoder_channels (..., (128, 128)) + conv_out, and dgrads
#undef C2
  return RPC_ERR_UNSUPPORTED;
}

static bool wgrad_narrow(int CI, int CO, int K) { return (CI == 4 || CI == 5) && CO == 16 && K <= MAXK; }

static int wgrad_narrow_chunks(int n) {   // 256-row chunks: ~1.5 blocks per CU at 100k rows
  const int c = (n + 255) / 256;
  return c < 1 ? 1 : (c > 2048 ? 2048 : c);
}

static int launch_wgrad(int CI, int CO, int at, const WgradArgs& a, dim3 grid, hipStream_t st) {
#define C2(ci, co)                                                                               \
  if (CI == ci && CO == co) {                                                                    \
    if (at == A_BNRELU) hipLaunchKernelGGL((k_wgrad<ci, co, A_BNRELU>), grid, dim3(BLK), 0, st, a); \
    else hipLaunchKernelGGL((k_wgrad<ci, co, A_RAW>), grid, dim3(BLK), 0, st, a);                 \
    return RPC_OK;                                                                               \
  }
  C2(4, 16) C2(5, 16) C2(16, 16) C2(16, 32) C2(32, 32) C2(32, 64) C2(64, 64) C2(64, 128) C2(64, 16)
  C2(128, 128)
#undef C2
  return RPC_ERR_UNSUPPORTED;
}

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
static inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace sp
}  // namespace rpc

using namespace rpc;
using namespace rpc::sp;

static KGeom geom(const int* ks, const int* st, const int* pd) {
  KGeom g;
  for (int a = 0; a < 3; ++a) {
    g.k[a] = ks[a];
    g.s[a] = st ? st[a] : 1;
    g.p[a] = pd ? pd[a] : 0;
  }
  g.K = ks[0] * ks[1] * ks[2];
  return g;
}

extern "C" int rpc_subm_rulebook(const int* coors, int N, const int* shape /* host B,D,H,W */,
                                 const int* ksize /* host [3] */, int* grid, int* nbr, void* stream) {
  if (N < 0 || !shape || !ksize) return RPC_ERR_ARG;
  if (N == 0) return RPC_OK;
  if (!coors || !grid || !nbr) return RPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  Shape s{shape[0], shape[1], shape[2], shape[3]};
  KGeom g = geom(ksize, nullptr, nullptr);
  if (g.K > MAXK) return RPC_ERR_UNSUPPORTED;
  if ((long long)N * g.K >= (1LL << 31) - BLK) return RPC_ERR_ARG;   // 32-bit (row, offset) index
  hipLaunchKernelGGL(k_grid_set, dim3(cdiv(N, BLK)), dim3(BLK), 0, st, coors, N, s, grid, 0);
  hipLaunchKernelGGL(k_subm_nbr, dim3(cdiv((long long)N * g.K, BLK)), dim3(BLK), 0, st, coors, N, s, g,
                     grid, nbr);
  hipLaunchKernelGGL(k_grid_set, dim3(cdiv(N, BLK)), dim3(BLK), 0, st, coors, N, s, grid, 1);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" size_t rpc_spconv_rulebook_workspace_size(int N, int K) {
  size_t n = (size_t)N * K + 1, scan_b = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (int*)nullptr, (int*)nullptr, (int)n, (hipStream_t)0) !=
      hipSuccess)
    return 0;
  return al(n * sizeof(int)) * 2 + al(scan_b);
}

extern "C" int rpc_spconv_rulebook_count(const int* coors, int N, const int* out_shape /* B,D,H,W */,
                                         const int* ksize, const int* stride, const int* pad, int* grid_out,
                                         int* n_out /* device int */, void* ws, size_t ws_bytes, void* stream) {
  if (N < 1 || !coors || !grid_out || !n_out || !ws) return RPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  Shape so{out_shape[0], out_shape[1], out_shape[2], out_shape[3]};
  KGeom g = geom(ksize, stride, pad);
  if (g.K > MAXK) return RPC_ERR_UNSUPPORTED;
  if ((long long)N * g.K >= (1LL << 31) - BLK) return RPC_ERR_ARG;   // 32-bit (row, offset) index
  size_t n = (size_t)N * g.K + 1;
  if (ws_bytes < rpc_spconv_rulebook_workspace_size(N, g.K)) return RPC_ERR_WORKSPACE;
  // per-row head counts [N + 1] and their exclusive scan (the row positions of rpc_spconv_rulebook_build)
  int* cnt = (int*)ws;
  unsigned* hmask = (unsigned*)ws + (N + 1);   // the first region holds N*K + 1 >= 2N + 2 ints
  int* pos = (int*)((char*)ws + al(n * sizeof(int)));
  void* tmp = (char*)ws + 2 * al(n * sizeof(int));
  size_t tb = 0;
  RPC_CHECK(hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, pos, N + 1, st));
  if (g.K < 2 || tb > ws_bytes - 2 * al(n * sizeof(int))) return RPC_ERR_WORKSPACE;
  int nb = cdiv((long long)N * g.K, BLK);
  hipLaunchKernelGGL(k_cand_min, dim3(nb), dim3(BLK), 0, st, coors, N, g, so, (unsigned*)grid_out);
  hipLaunchKernelGGL(k_row_heads, dim3(cdiv(32LL * (N + 1), BLK)), dim3(BLK), 0, st, coors, N, g, so,
                     (const unsigned*)grid_out, cnt, hmask);
  RPC_LAUNCH_CHECK();
  RPC_CHECK(hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, pos, N + 1, st));
  RPC_CHECK(hipMemcpyAsync(n_out, pos + N, sizeof(int), hipMemcpyDeviceToDevice, st));
  return RPC_OK;
}

extern "C" int rpc_spconv_rulebook_build(const int* coors, int N, const int* out_shape, const int* ksize,
                                         const int* stride, const int* pad, int* grid_out, int n_out,
                                         int* coors_out, int* nbr_out, int* nbr_in, void* ws, void* stream) {
  if (N < 1 || !coors || !grid_out || !coors_out || !nbr_out || !nbr_in || !ws) return RPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  Shape so{out_shape[0], out_shape[1], out_shape[2], out_shape[3]};
  KGeom g = geom(ksize, stride, pad);
  if (g.K > MAXK || (long long)N * g.K >= (1LL << 31) - BLK) return RPC_ERR_ARG;
  size_t n = (size_t)N * g.K + 1;
  const unsigned* hmask = (const unsigned*)ws + (N + 1);
  int* pos = (int*)((char*)ws + al(n * sizeof(int)));
  int nb = cdiv((long long)N * g.K, BLK);
  RPC_CHECK(hipMemsetAsync(nbr_out, 0xFF, sizeof(int) * (size_t)n_out * g.K, st));
  hipLaunchKernelGGL(k_row_assign, dim3(cdiv(N, BLK)), dim3(BLK), 0, st, coors, N, g, so, pos, hmask, grid_out,
                     coors_out);
  hipLaunchKernelGGL(k_nbr_fill, dim3(nb), dim3(BLK), 0, st, coors, N, g, so, grid_out, nbr_out, nbr_in);
  if (n_out > 0)
    hipLaunchKernelGGL(k_grid_set, dim3(cdiv(n_out, BLK)), dim3(BLK), 0, st, coors_out, n_out, so, grid_out, 1);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

// forward conv: z_out = conv(A(in)) ; writes BatchNorm partial sums [nblk][2*CO] if part != NULL
extern "C" int rpc_spconv_gemm_blocks(int n_out) { return cdiv(n_out, BM); }

extern "C" int rpc_spconv_forward(const float* in, const float* in_bn /* scale,shift or NULL: raw */,
                                  int CI, const int* nbr, int K, int n_out, const float* W, int CO,
                                  float* z_out, float* part, void* stream) {
  if (n_out < 0 || K > MAXK) return RPC_ERR_ARG;
  if (n_out == 0) return RPC_OK;
  if (in_bn == nullptr && CO == 16 && (CI == 4 || CI == 5)) {   // the narrow input layer
    const dim3 grid(cdiv(n_out, L0R));
    if (CI == 4) hipLaunchKernelGGL(k_l0_fwd<4>, grid, dim3(L0T), 0, (hipStream_t)stream, in, nbr, K, W, n_out, z_out, part);
    else hipLaunchKernelGGL(k_l0_fwd<5>, grid, dim3(L0T), 0, (hipStream_t)stream, in, nbr, K, W, n_out, z_out, part);
    RPC_LAUNCH_CHECK();
    return RPC_OK;
  }
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.a = in;
  a.abn = in_bn;
  a.nbr = nbr;
  a.K = K;
  a.W = W;
  a.CIw = CI;
  a.COw = CO;
  a.Nout = n_out;
  a.out = z_out;
  a.CO_real = CO;
  a.part = part;
  int rc = launch_gemm(CI, CO, in_bn ? A_BNRELU : A_RAW, E_FWD, a, cdiv(n_out, BM), (hipStream_t)stream);
  if (rc) return rc;
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

// dgrad: din = sum_k dz_out[map[:, k]] W[k]^T, with dz computed on load from (dy, z, bnb);
// if prev_z != NULL, the ReLU mask and BatchNorm-backward partial sums of the previous
// layer (prev_bn = its forward scale/shift/mean/invstd) are applied/written.
extern "C" int rpc_spconv_dgrad(const float* dy_out, const float* z_out, const float* bnb /* 5*CO */,
                                int CO, const int* map, int K, int rev, int n_in, const float* W, int CI,
                                const float* prev_z, const float* prev_bn, float* din, float* part,
                                void* stream) {
  if (n_in < 0 || K > MAXK) return RPC_ERR_ARG;
  if (n_in == 0) return RPC_OK;
  if (prev_z == nullptr && CO == 16 && (CI == 4 || CI == 5)) {   // into the narrow input layer's rows
    const dim3 grid(cdiv(n_in, L0R));
    if (CI == 4)
      hipLaunchKernelGGL(k_l0_dgrad<4>, grid, dim3(L0T), 0, (hipStream_t)stream, dy_out, z_out, bnb, map, K, rev, W, n_in, din);
    else
      hipLaunchKernelGGL(k_l0_dgrad<5>, grid, dim3(L0T), 0, (hipStream_t)stream, dy_out, z_out, bnb, map, K, rev, W, n_in, din);
    RPC_LAUNCH_CHECK();
    return RPC_OK;
  }
  GemmArgs a;
  memset(&a, 0, sizeof(a));
  a.a = dy_out;
  a.a2 = z_out;
  a.abn = bnb;
  a.nbr = map;
  a.K = K;
  a.rev = rev;
  a.W = W;
  a.transW = 1;
  a.CIw = CI;
  a.COw = CO;
  a.Nout = n_in;
  a.out = din;
  a.CO_real = CI;
  a.ez = prev_z;
  a.ebn = prev_bn;
  a.part = part;
  int CIg = CO, COg = CI < 16 ? 16 : CI;
  int rc = launch_gemm(CIg, COg, A_BNBWD, prev_z ? E_DGRAD : E_PLAIN, a, cdiv(n_in, BM), (hipStream_t)stream);
  if (rc) return rc;
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" size_t rpc_spconv_wgrad_workspace_size(int n_out, int K, int CI, int CO) {
  if (wgrad_narrow(CI, CO, K)) return (size_t)wgrad_narrow_chunks(n_out) * K * CI * CO * sizeof(float);
  int chunks = cdiv(n_out > 0 ? n_out : 1, 2048);
  if (chunks > 64) chunks = 64;
  return (size_t)chunks * K * CI * CO * sizeof(float);
}

extern "C" int rpc_spconv_wgrad(const float* in, const float* in_bn, int CI, const int* nbr, int K, int n_out,
                                const float* dy_out, const float* z_out, const float* bnb, int CO, float* dW,
                                void* ws, size_t ws_bytes, void* stream) {
  if (n_out < 0 || K > MAXK) return RPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n_out == 0) {
    RPC_CHECK(hipMemsetAsync(dW, 0, sizeof(float) * (size_t)K * CI * CO, st));
    return RPC_OK;
  }
  const bool narrow = wgrad_narrow(CI, CO, K);
  int chunks = narrow ? wgrad_narrow_chunks(n_out) : cdiv(n_out, 2048);
  if (!narrow && chunks > 64) chunks = 64;
  if (ws_bytes < (size_t)chunks * K * CI * CO * sizeof(float)) return RPC_ERR_WORKSPACE;
  WgradArgs a;
  a.a = in;
  a.abn = in_bn;
  a.nbr = nbr;
  a.K = K;
  a.Nout = n_out;
  a.rows_per = ((cdiv(n_out, chunks) + 63) / 64) * 64;
  a.dy = dy_out;
  a.z = z_out;
  a.dbn = bnb;
  a.part = (float*)ws;
  int rc = RPC_OK;
  if (narrow) {
    a.rows_per = ((cdiv(n_out, chunks) + 63) / 64) * 64;
#define NW(ci)                                                                                              \
    if (CI == ci) {                                                                                         \
      if (in_bn) hipLaunchKernelGGL((k_wgrad_narrow<ci, 16, A_BNRELU>), dim3(chunks),                       \
                                    dim3(wn_threads<ci, 16, A_BNRELU>()), 0, st, a);                        \
      else hipLaunchKernelGGL((k_wgrad_narrow<ci, 16, A_RAW>), dim3(chunks), dim3(wn_threads<ci, 16, A_RAW>()), \
                              0, st, a);                                                                    \
    }
    NW(4) NW(5)
#undef NW
  } else {
    rc = launch_wgrad(CI, CO, in_bn ? A_BNRELU : A_RAW, a, dim3(chunks, K), st);
  }
  if (rc) return rc;
  long long total = (long long)K * CI * CO;
  slab_reduce((const float*)ws, chunks, total, dW, st);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" size_t rpc_bn_finalize_workspace_size(int C) { return 0; }

extern "C" int rpc_bn_finalize(const void* part, int nblk, int C, int N, int mode, const float* gamma,
                               const float* beta, float eps, float momentum, float* running_mean,
                               float* running_var, const float* fwd_bn, float* bn_out, float* dgamma, float* dbeta,
                               void* ws, void* stream) {
  (void)ws;   // single pass since r01 v11: no workspace (kept in the signature; may be NULL)
  if (C < 1 || nblk < 1 || !part || !bn_out || (mode & ~(1 | RPC_BN_PART_F64))) return RPC_ERR_ARG;
  if (mode & RPC_BN_PART_F64)
    hipLaunchKernelGGL(k_bn_finalize<double>, dim3(C), dim3(BLK), 0, (hipStream_t)stream, (const double*)part, nblk,
                       C, N, mode & 1, gamma, beta, eps, momentum, running_mean, running_var, fwd_bn, bn_out, dgamma,
                       dbeta);
  else
    hipLaunchKernelGGL(k_bn_finalize<float>, dim3(C), dim3(BLK), 0, (hipStream_t)stream, (const float*)part, nblk,
                       C, N, mode, gamma, beta, eps, momentum, running_mean, running_var, fwd_bn, bn_out, dgamma,
                       dbeta);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_sparse_to_dense(const float* z, const float* bn, const int* coors, int N, int C,
                                   const int* shape /* B,D,H,W */, int flags, void* dense, void* stream) {
  if (N < 0 || C < 1 || !shape || (flags & ~3)) return RPC_ERR_ARG;
  if (N == 0) return RPC_OK;
  Shape s{shape[0], shape[1], shape[2], shape[3]};
  hipStream_t st = (hipStream_t)stream;
  if (C % 4 == 0 && (long long)N * (C / 4) < (1LL << 31)) {
    dim3 g4(cdiv((long long)N * (C / 4), BLK));
    switch (flags) {
      case 0: hipLaunchKernelGGL((k_to_dense_v4<float, false>), g4, dim3(BLK), 0, st, z, bn, coors, N, C, s, (float*)dense); break;
      case 1: hipLaunchKernelGGL((k_to_dense_v4<float, true>), g4, dim3(BLK), 0, st, z, bn, coors, N, C, s, (float*)dense); break;
      case 2: hipLaunchKernelGGL((k_to_dense_v4<__hip_bfloat16, false>), g4, dim3(BLK), 0, st, z, bn, coors, N, C, s,
                                 (__hip_bfloat16*)dense); break;
      default: hipLaunchKernelGGL((k_to_dense_v4<__hip_bfloat16, true>), g4, dim3(BLK), 0, st, z, bn, coors, N, C, s,
                                  (__hip_bfloat16*)dense);
    }
    RPC_LAUNCH_CHECK();
    return RPC_OK;
  }
  dim3 g(cdiv((long long)N * C, BLK));
  switch (flags) {
    case 0: hipLaunchKernelGGL((k_to_dense<float, false>), g, dim3(BLK), 0, st, z, bn, coors, N, C, s, (float*)dense); break;
    case 1: hipLaunchKernelGGL((k_to_dense<float, true>), g, dim3(BLK), 0, st, z, bn, coors, N, C, s, (float*)dense); break;
    case 2: hipLaunchKernelGGL((k_to_dense<__hip_bfloat16, false>), g, dim3(BLK), 0, st, z, bn, coors, N, C, s,
                               (__hip_bfloat16*)dense); break;
    default: hipLaunchKernelGGL((k_to_dense<__hip_bfloat16, true>), g, dim3(BLK), 0, st, z, bn, coors, N, C, s,
                                (__hip_bfloat16*)dense);
  }
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_sparse_dense_clear(const int* coors, int N, int C, const int* shape /* B,D,H,W */, int flags,
                                      void* dense, void* stream) {
  if (N < 0 || C < 1 || !shape || (flags & ~3)) return RPC_ERR_ARG;
  if (N == 0) return RPC_OK;
  Shape s{shape[0], shape[1], shape[2], shape[3]};
  hipStream_t st = (hipStream_t)stream;
  if ((C & 3) || (long long)N * (C / 4) >= (1LL << 31)) {   // scalar form (mirrors k_to_dense's fallback)
    dim3 g1(cdiv((long long)N * C, BLK));
    switch (flags) {
      case 0: hipLaunchKernelGGL((k_dense_clear<float, false>), g1, dim3(BLK), 0, st, coors, (long long)N, C, s,
                                 (float*)dense); break;
      case 1: hipLaunchKernelGGL((k_dense_clear<float, true>), g1, dim3(BLK), 0, st, coors, (long long)N, C, s,
                                 (float*)dense); break;
      case 2: hipLaunchKernelGGL((k_dense_clear<__hip_bfloat16, false>), g1, dim3(BLK), 0, st, coors, (long long)N,
                                 C, s, (__hip_bfloat16*)dense); break;
      default: hipLaunchKernelGGL((k_dense_clear<__hip_bfloat16, true>), g1, dim3(BLK), 0, st, coors, (long long)N,
                                  C, s, (__hip_bfloat16*)dense);
    }
    RPC_LAUNCH_CHECK();
    return RPC_OK;
  }
  dim3 g4(cdiv((long long)N * (C / 4), BLK));
  switch (flags) {
    case 0: hipLaunchKernelGGL((k_dense_clear_v4<float, false>), g4, dim3(BLK), 0, st, coors, N, C, s, (float*)dense); break;
    case 1: hipLaunchKernelGGL((k_dense_clear_v4<float, true>), g4, dim3(BLK), 0, st, coors, N, C, s, (float*)dense); break;
    case 2: hipLaunchKernelGGL((k_dense_clear_v4<__hip_bfloat16, false>), g4, dim3(BLK), 0, st, coors, N, C, s,
                               (__hip_bfloat16*)dense); break;
    default: hipLaunchKernelGGL((k_dense_clear_v4<__hip_bfloat16, true>), g4, dim3(BLK), 0, st, coors, N, C, s,
                                (__hip_bfloat16*)dense);
  }
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dense_to_sparse_grad(const void* grad_dense, const float* z, const float* bn, const int* coors,
                                        int N, int C, const int* shape, int flags, float* dy, float* part,
                                        void* stream) {
  if (N < 0 || C < 1 || C > 256 || !shape || (flags & ~3)) return RPC_ERR_ARG;
  if (N == 0) return RPC_OK;
  Shape s{shape[0], shape[1], shape[2], shape[3]};
  dim3 g(cdiv(N, BM));
  hipStream_t st = (hipStream_t)stream;
  switch (flags) {
    case 0: hipLaunchKernelGGL((k_from_dense<float, false>), g, dim3(FBLK), 0, st, (const float*)grad_dense, z, bn,
                               coors, N, C, s, dy, part); break;
    case 1: hipLaunchKernelGGL((k_from_dense<float, true>), g, dim3(FBLK), 0, st, (const float*)grad_dense, z, bn,
                               coors, N, C, s, dy, part); break;
    case 2: hipLaunchKernelGGL((k_from_dense<__hip_bfloat16, false>), g, dim3(FBLK), 0, st,
                               (const __hip_bfloat16*)grad_dense, z, bn, coors, N, C, s, dy, part); break;
    default: hipLaunchKernelGGL((k_from_dense<__hip_bfloat16, true>), g, dim3(FBLK), 0, st,
                                (const __hip_bfloat16*)grad_dense, z, bn, coors, N, C, s, dy, part);
  }
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_sparse_res_forward_h16(const float* z, const float* bn, const float* res, int n, int c, float* out,
                                          void* out_h16, int fmt, void* out_bf16, void* stream) {
  if (n < 0 || c < 1 || !z || !bn || !out || (fmt != 0 && fmt != 1) || (out_bf16 && !fmt)) return RPC_ERR_ARG;
  if (n == 0) return RPC_OK;
  const int cp = (c + 7) / 8 * 8;
  if (c % 8 == 0 && (long long)n * c < (1LL << 31)) {
    const dim3 grid(cdiv((long long)n * (c / 8), BLK));
    if (fmt)
      hipLaunchKernelGGL(k_res_fwd_v8<1>, grid, dim3(BLK), 0, (hipStream_t)stream, z, bn, res, n, c, out,
                         (unsigned short*)out_h16, (unsigned short*)out_bf16);
    else
      hipLaunchKernelGGL(k_res_fwd_v8<0>, grid, dim3(BLK), 0, (hipStream_t)stream, z, bn, res, n, c, out,
                         (unsigned short*)out_h16, (unsigned short*)nullptr);
    RPC_LAUNCH_CHECK();
    return RPC_OK;
  }
  if (fmt)
    hipLaunchKernelGGL(k_res_fwd<1>, dim3(cdiv((long long)n * cp, BLK)), dim3(BLK), 0, (hipStream_t)stream, z, bn, res,
                       n, c, cp, out, (unsigned short*)out_h16, (unsigned short*)out_bf16);
  else
    hipLaunchKernelGGL(k_res_fwd<0>, dim3(cdiv((long long)n * cp, BLK)), dim3(BLK), 0, (hipStream_t)stream, z, bn, res,
                       n, c, cp, out, (unsigned short*)out_h16, (unsigned short*)nullptr);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_sparse_res_forward(const float* z, const float* bn, const float* res, int n, int c, float* out,
                                      void* out_bf16, void* stream) {
  return rpc_sparse_res_forward_h16(z, bn, res, n, c, out, out_bf16, 0, nullptr, stream);
}

extern "C" int rpc_sparse_res_backward(const float* g1, const float* g2, const float* out, const float* z,
                                       const float* bn, int n, int c, float* m, float* part, void* stream) {
  if (n < 0 || c < 1 || c > 256 || !g1 || !out || !z || !bn || !m || !part) return RPC_ERR_ARG;
  if (n == 0) return RPC_OK;
  // k_res_bwd_v4 needs Q = c / 4 to be a power of two: its row lanes tile a wave (64 % Q == 0), its xor
  // shuffles run over the lane bits above log2(Q), and its blocks cover whole BM-row partial groups
  const int q4 = c / 4;
  if (c % 4 == 0 && c >= 16 && c <= 128 && (q4 & (q4 - 1)) == 0 && (long long)n * c < (1LL << 31))
    hipLaunchKernelGGL(k_res_bwd_v4, dim3(cdiv(n, 8 * (BLK / (c / 4)))), dim3(BLK), 0, (hipStream_t)stream, g1, g2,
                       out, z, bn, n, c, m, part);
  else
    hipLaunchKernelGGL(k_res_bwd, dim3(cdiv(n, BM)), dim3(BLK), 0, (hipStream_t)stream, g1, g2, out, z, bn, n, c, m,
                       part);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
