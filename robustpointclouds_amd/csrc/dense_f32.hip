// a7 parity mode: the dense BEV backbone / neck (SECOND + SECONDFPN, upstream mmdet3d
// backbones/second.py, necks/second_fpn.py as configured at
// configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:25-36) and the
// Anchor3DHead 1x1 convs with fp32 operands on fp32 MFMA (v_mfma_f32_16x16x4_f32: fp32 products,
// fp32 accumulation — the reference arithmetic, only the summation order differs from MIOpen's).
//
// Same GEMM formulation and pixel maps as the bf16 engine (dense_common.h): rows = image pixels,
// K = (tap, input channel), NHWC fp32 images.
//   k_igemm_f32: 64 pixels x 64 output channels per 256-thread block (4 waves of 32 x 32 = 2 x 2
//     16x16 MFMA tiles), K-steps of 16 channels of one tap through register-staged double-buffered
//     LDS tiles; A = weights (lane: output channel l&15, channel 4k + l>>4), B = activations, so
//     each lane ends up with 4 consecutive output channels of one pixel (one 16-byte store).
//     Epilogue: optional accumulate into the existing image, optional channel offset (FPN concat),
//     per-block BatchNorm partial sums of the stored fp32 values (reduced by rpc_bn_finalize).
//   k_wgrad_f32: dW[t][ci][co] = sum_rows x[src(row,t)][ci] * dz[row][co] with rows as the MFMA
//     K dimension, 64 x 64 (ci, co) tiles, fp32 split-K slabs per row chunk reduced in a fixed
//     order (k_wgrad_reduce) straight into the torch layout.
#include <hip/hip_runtime.h>
#include <string.h>

#include "common.h"
#include "dense_common.h"
#include "rpc_hip.h"

namespace rpc {
namespace dn {
namespace f32 {

constexpr int BLK = 256;
constexpr int TM = 64;       // GEMM rows (pixels) per block
constexpr int TN = 64;       // output channels per block
constexpr int BK = 16;       // K-step = 16 channels of one tap
constexpr int LP = BK + 4;   // LDS pitch (floats; 16-byte aligned rows)

typedef float f32x4 __attribute__((ext_vector_type(4)));

struct IG {
  const float* src;  // K-operand image rows [S pixels][SP]
  int SP;
  int CIN;           // multiple of 16
  const float* wt;   // [taps][COUT][CIN] (U2: [parity][COUT][CIN])
  int COUT;          // multiple of 64
  float* out;        // output rows [O pixels][OP] at channel offset OOFF
  int OP, OOFF;
  int accum;
  float* part;       // [gridDim.z * gridDim.x][2 * COUT] BatchNorm partial sums, or null
  Img R, S, O;
  int M;
};

template <int MAP>
__global__ __launch_bounds__(BLK) void k_igemm_f32(IG g) {
  constexpr int T = taps_of<MAP>();
  __shared__ __attribute__((aligned(16))) float sX[2][TM * LP];
  __shared__ __attribute__((aligned(16))) float sW[2][TN * LP];
  __shared__ int sRow[TM * T];
  __shared__ float sP[2][2][TN];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wc = w >> 1, wp = w & 1;   // wave: output channels wc*32.., pixels wp*32..
  const int a = lane & 15, q = lane >> 4;
  const int bx = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = bx * TM, n0 = blockIdx.y * TN, par = blockIdx.z;
  if (m0 >= g.M) return;
  const int KC = g.CIN / BK, NKS = T * KC;
  const float* wbase = g.wt + (MAP == M_U2 ? (size_t)par * g.COUT * g.CIN : 0);
  const int HW = g.R.H * g.R.W;
  for (int i = tid; i < TM * T; i += BLK) {
    const int r = i / T, t = i - r * T, m = m0 + r;
    int s = -1;
    if (m < g.M) {
      const int b = m / HW, rem = m - b * HW, y = rem / g.R.W, x = rem - y * g.R.W;
      s = src_row<MAP>(b, y, x, t, g.S);
    }
    sRow[i] = s;
  }
  __syncthreads();
  // staging: thread loads 4 channels of row srow (activations) and of output channel srow (weights)
  const int srow = tid >> 2, sseg = (tid & 3) * 4;
  float4 rx, rw;
  auto load = [&](int ks) {
    const int t = ks / KC, kc = ks - t * KC;
    const int sr = sRow[srow * T + t];
    rx = *(const float4*)(g.src + (size_t)max(sr, 0) * g.SP + kc * BK + sseg);
    if (sr < 0) rx = make_float4(0.f, 0.f, 0.f, 0.f);
    rw = *(const float4*)(wbase + ((size_t)(t * g.COUT + n0 + srow)) * g.CIN + kc * BK + sseg);
  };
  auto store = [&](int buf) {
    *(float4*)&sX[buf][srow * LP + sseg] = rx;
    *(float4*)&sW[buf][srow * LP + sseg] = rw;
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  for (int ks = 0; ks < NKS; ++ks) {
    const int buf = ks & 1;
    const bool more = ks + 1 < NKS;
    if (more) load(ks + 1);
#pragma unroll
    for (int k4 = 0; k4 < BK / 4; ++k4) {
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = sW[buf][(wc * 32 + 16 * i + a) * LP + 4 * k4 + q];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = sX[buf][(wp * 32 + 16 * j + a) * LP + 4 * k4 + q];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds channels co = n0 + wc*32 + 16i + 4q + r of pixel m0 + wp*32 + 16j + a
  float s1[2][4], s2[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + wp * 32 + 16 * j + a;
    if (m >= g.M) continue;
    int orow = m;
    if (MAP == M_U2) {
      const int b = m / HW, rem = m - b * HW, y = rem / g.R.W, x = rem - y * g.R.W;
      orow = out_row<MAP>(m, b, y, x, par, g.O);
    }
    float* op = g.out + (size_t)orow * g.OP + g.OOFF + n0 + wc * 32 + 4 * q;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 v = acc[i][j];
      float4* p4 = (float4*)(op + 16 * i);
      if (g.accum) {
        const float4 e = *p4;
        v[0] += e.x;
        v[1] += e.y;
        v[2] += e.z;
        v[3] += e.w;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s1[i][r] += v[r];
        s2[i][r] += v[r] * v[r];
      }
      *p4 = make_float4(v[0], v[1], v[2], v[3]);
    }
  }
  if (g.part == nullptr) return;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[i][r] += __shfl_xor(s1[i][r], o, 64);
        s2[i][r] += __shfl_xor(s2[i][r], o, 64);
      }
    }
  if (a == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = wc * 32 + 16 * i + 4 * q + r;
        sP[wp][0][c] = s1[i][r];
        sP[wp][1][c] = s2[i][r];
      }
  }
  __syncthreads();
  float* prow = g.part + ((size_t)blockIdx.z * gridDim.x + bx) * 2 * g.COUT;
  if (tid < TN) {
    prow[n0 + tid] = sP[0][0][tid] + sP[1][0][tid];
    prow[g.COUT + n0 + tid] = sP[0][1][tid] + sP[1][1][tid];
  }
}

// ------------------------------------------------------------------ weight gradient
struct WG {
  const float* x;   // forward input image rows [S pixels][XP]
  int XP;
  const float* dz;  // output-side gradient rows [O pixels][DP]
  int DP;
  int CI, CO;       // multiples of 64
  Img R, S, O;
  int M, rows_per;
  float* part;      // [chunks][T][CI][CO]
};

constexpr int WTC = 64;          // (ci, co) tile edge
constexpr int WRT = 32;          // rows per LDS sub-tile
constexpr int WP = WTC + 4;      // LDS pitch (floats)
constexpr int WNLD = WRT * (WTC / 4) / BLK;   // 16-B loads per thread per operand and sub-tile (2)

// 1-D grid of chunks * T * (CI/64)*(CO/64) blocks, XCD-aware (a chunk's taps and channel tiles
// adjacent, so its x / dz rows are fetched into one XCD's L2 and re-read there).
template <int MAP>
__global__ __launch_bounds__(BLK) void k_wgrad_f32(WG g) {
  constexpr int T = wtaps_of<MAP>();
  __shared__ __attribute__((aligned(16))) float sX[WRT * WP];
  __shared__ __attribute__((aligned(16))) float sD[WRT * WP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wci = w >> 1, wco = w & 1;
  const int a = lane & 15, q = lane >> 4;
  const int nco = g.CO / WTC, ntile = (g.CI / WTC) * nco;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = lid / (T * ntile), rest = lid - chunk * (T * ntile);
  const int t = rest / ntile, tile = rest - t * ntile;
  const int ci0 = (tile / nco) * WTC, co0 = (tile % nco) * WTC;
  const int rb0 = chunk * g.rows_per, rb1 = min(g.M, rb0 + g.rows_per);
  const int HW = g.R.H * g.R.W;

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float4 rx[WNLD], rd[WNLD];
  auto gload = [&](int rs) {
#pragma unroll
    for (int s = 0; s < WNLD; ++s) {
      const int e = tid + s * BLK, r = e >> 4, seg = (e & 15) * 4;
      const int m = rs + r;
      rx[s] = rd[s] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < rb1) {
        const int b = m / HW, rem = m - b * HW, y = rem / g.R.W, x = rem - y * g.R.W;
        int xs, ds;
        if (MAP == M_U2) {
          xs = m;
          ds = out_row<MAP>(m, b, y, x, t, g.O);
        } else {
          xs = src_row<MAP>(b, y, x, t, g.S);
          ds = m;
        }
        if (xs >= 0) {
          rx[s] = *(const float4*)(g.x + (size_t)xs * g.XP + ci0 + seg);
          rd[s] = *(const float4*)(g.dz + (size_t)ds * g.DP + co0 + seg);
        }
      }
    }
  };
  if (rb0 < rb1) gload(rb0);
  for (int rs = rb0; rs < rb1; rs += WRT) {
    __syncthreads();
#pragma unroll
    for (int s = 0; s < WNLD; ++s) {
      const int e = tid + s * BLK, r = e >> 4, seg = (e & 15) * 4;
      *(float4*)&sX[r * WP + seg] = rx[s];
      *(float4*)&sD[r * WP + seg] = rd[s];
    }
    __syncthreads();
    if (rs + WRT < rb1) gload(rs + WRT);
#pragma unroll
    for (int k4 = 0; k4 < WRT / 4; ++k4) {
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = sX[(4 * k4 + q) * WP + wci * 32 + 16 * i + a];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = sD[(4 * k4 + q) * WP + wco * 32 + 16 * j + a];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
  }
  // lane holds dW[ci = ci0 + wci*32 + 16i + 4q + r][co = co0 + wco*32 + 16j + a]
  float* out = g.part + ((size_t)chunk * T + t) * g.CI * g.CO;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ci = ci0 + wci * 32 + 16 * i + 4 * q + r, co = co0 + wco * 32 + 16 * j + a;
        out[(size_t)ci * g.CO + co] = acc[i][j][r];
      }
}

// ------------------------------------------------------------------ weight preparation (fp32 operands)
// torch layouts -> fwd [T][co][ci] and dgrad [T][ci][co] (S1: taps flipped), as the bf16 k_wprep
constexpr int WPREP_MAX = 16;
struct WprepBatch {
  RpcDenseWprep d[WPREP_MAX];
};
__global__ __launch_bounds__(BLK) void k_wprep_batch_f32(WprepBatch bt) {
  const RpcDenseWprep& d = bt.d[blockIdx.y];
  const long long e = (long long)blockIdx.x * BLK + threadIdx.x;
  const long long n = (long long)d.taps * d.ci * d.co;
  if (e >= n) return;
  const int CI = d.ci, CO = d.co, T = d.taps;
  const int t = (int)(e / ((long long)CI * CO));
  const int rem = (int)(e - (long long)t * CI * CO), ci = rem / CO, co = rem - ci * CO;
  const float v = d.kind == 0 ? (d.co_src > 0 && co >= d.co_src ? 0.0f : d.W[((size_t)co * CI + ci) * T + t])
                              : d.W[((size_t)ci * CO + co) * T + t];
  if (d.w_fwd) ((float*)d.w_fwd)[((size_t)t * CO + co) * CI + ci] = v;
  if (d.w_dgrad) {
    const int td = d.flip ? T - 1 - t : t;
    ((float*)d.w_dgrad)[((size_t)td * CI + ci) * CO + co] = v;
  }
}

template <int MAP>
static void launch_igemm(const IG& g, int par_count, hipStream_t st) {
  dim3 grid(cdivu(g.M, TM), g.COUT / TN, par_count);
  hipLaunchKernelGGL((k_igemm_f32<MAP>), grid, dim3(BLK), 0, st, g);
}

template <int MAP>
static void launch_wgrad(const WG& g, int chunks, hipStream_t st) {
  dim3 grid(chunks * wtaps_of<MAP>() * (g.CI / WTC) * (g.CO / WTC));
  hipLaunchKernelGGL((k_wgrad_f32<MAP>), grid, dim3(BLK), 0, st, g);
}

// row chunks: the grid fills ~4 resident blocks per CU in whole rounds, chunks <= 2048 rows
static int wgrad_chunks(int M, int T, int ci, int co) {
  const int per = T * (ci / WTC) * (co / WTC);
  const int slots = 4 * cu_count();
  const int step = slots / per > 0 ? slots / per : 1;
  int c = step;
  while ((M + c - 1) / c > 2048 && c < 2048) c += step;
  return c < 2048 ? c : 2048;
}

}  // namespace f32
}  // namespace dn
}  // namespace rpc

using namespace rpc;
using namespace rpc::dn;

static inline Img img3f(const int* d) { return Img{d[0], d[1], d[2]}; }

extern "C" int rpc_dense_conv_f32(int map, const float* src, int sp, int cin, const float* wt, int cout, float* out,
                                  int op, int ooff, int accum, float* part, const int* r_img, const int* s_img,
                                  const int* o_img, void* stream) {
  if (map < M_S1 || map > M_G2 || !src || !wt || !out || !r_img || !s_img || !o_img) return RPC_ERR_ARG;
  if (cin % f32::BK || cout % f32::TN || sp < cin || op < ooff + cout || (sp & 3) || (op & 3) || (ooff & 3))
    return RPC_ERR_ARG;
  f32::IG g{src, sp, cin, wt, cout, out, op, ooff, accum, part, img3f(r_img), img3f(s_img), img3f(o_img), 0};
  g.M = g.R.B * g.R.H * g.R.W;
  if (g.M == 0) return RPC_OK;
  hipStream_t st = (hipStream_t)stream;
  switch (map) {
    case M_S1: f32::launch_igemm<M_S1>(g, 1, st); break;
    case M_S2: f32::launch_igemm<M_S2>(g, 1, st); break;
    case M_D2: f32::launch_igemm<M_D2>(g, 1, st); break;
    case M_P1: f32::launch_igemm<M_P1>(g, 1, st); break;
    case M_U2: f32::launch_igemm<M_U2>(g, 4, st); break;
    default: f32::launch_igemm<M_G2>(g, 1, st); break;
  }
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dense_conv_blocks_f32(int map, const int* r_img) {
  const long long M = (long long)r_img[0] * r_img[1] * r_img[2];
  return (int)((M + f32::TM - 1) / f32::TM) * (map == M_U2 ? 4 : 1);
}

extern "C" size_t rpc_dense_wgrad_workspace_size_f32(int map, const int* r_img, int ci, int co) {
  if (ci % f32::WTC || co % f32::WTC) return 0;
  const int M = r_img[0] * r_img[1] * r_img[2];
  const int T = map_wtaps(map);
  return (size_t)f32::wgrad_chunks(M, T, ci, co) * T * ci * co * sizeof(float);
}

extern "C" int rpc_dense_wgrad_f32(int map, int kind, const float* x, int xp, int ci, const float* dz, int dp, int co,
                                   const int* r_img, const int* s_img, const int* o_img, float* dW, void* ws,
                                   size_t ws_bytes, void* stream) {
  if (map < M_S1 || map > M_G2 || map == M_D2 || map == M_G2 || !x || !dz || !dW) return RPC_ERR_ARG;
  if (ci % f32::WTC || co % f32::WTC || (xp & 3) || (dp & 3) || (kind != 0 && kind != 1)) return RPC_ERR_ARG;
  Img R = img3f(r_img), S = img3f(s_img), O = img3f(o_img);
  const int M = R.B * R.H * R.W, T = map_wtaps(map);
  const int chunks = f32::wgrad_chunks(M, T, ci, co);
  const size_t slab = (size_t)T * ci * co;
  hipStream_t st = (hipStream_t)stream;
  if (M == 0) {
    RPC_CHECK(hipMemsetAsync(dW, 0, slab * sizeof(float), st));
    return RPC_OK;
  }
  if (!ws || ws_bytes < chunks * slab * sizeof(float)) return RPC_ERR_WORKSPACE;
  float* part = (float*)ws;
  const int rows_per = ((M + chunks - 1) / chunks + f32::WRT - 1) / f32::WRT * f32::WRT;
  f32::WG g{x, xp, dz, dp, ci, co, R, S, O, M, rows_per, part};
  switch (map) {
    case M_S1: f32::launch_wgrad<M_S1>(g, chunks, st); break;
    case M_S2: f32::launch_wgrad<M_S2>(g, chunks, st); break;
    case M_P1: f32::launch_wgrad<M_P1>(g, chunks, st); break;
    default: f32::launch_wgrad<M_U2>(g, chunks, st); break;
  }
  RPC_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_wgrad_reduce<0>, dim3(cdivu(slab, 64)), dim3(256), 0, st, (const float*)part, chunks, kind, ci,
                     co, T, dW);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dense_wprep_batch_f32(const RpcDenseWprep* descs, int n, void* stream) {
  if (n < 0 || n > f32::WPREP_MAX || (n > 0 && !descs)) return RPC_ERR_ARG;
  if (n == 0) return RPC_OK;
  f32::WprepBatch b;
  memset(&b, 0, sizeof(b));
  long long most = 0;
  for (int i = 0; i < n; ++i) {
    const RpcDenseWprep& d = descs[i];
    if (!d.W || d.ci < 1 || d.co < 1 || d.taps < 1 || (d.kind != 0 && d.kind != 1) || d.co_src < 0 ||
        d.co_src > d.co || (d.co_src && d.kind != 0))
      return RPC_ERR_ARG;
    b.d[i] = d;
    const long long e = (long long)d.taps * d.ci * d.co;
    most = e > most ? e : most;
  }
  hipLaunchKernelGGL(f32::k_wprep_batch_f32, dim3(cdivu(most, f32::BLK), n), dim3(f32::BLK), 0, (hipStream_t)stream,
                     b);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
