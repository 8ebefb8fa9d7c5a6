// a7 perf mode: the dense BEV backbone / neck (SECOND + SECONDFPN, upstream mmdet3d
// backbones/second.py, necks/second_fpn.py as configured at
// configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-car.py via its base) as
// bf16-MFMA implicit GEMMs over NHWC images, for gfx950.
//
// Every convolution of the stack (and its data / weight gradients) is one GEMM whose rows are
// image pixels and whose K dimension is (tap, input channel); a "map" turns (row pixel, tap)
// into the source pixel arithmetically (zero padding = no source):
//   S1  3x3 stride-1 pad-1 conv (also its data gradient, with the taps flipped)
//   S2  3x3 stride-2 pad-1 conv (block 2's first layer)
//   D2  data gradient of S2 (a transposed conv: source = (y+1-dy)/2 when even)
//   P1  1x1 (FPN deblock 0: ConvTranspose2d kernel 1 stride 1) and its data gradient
//   U2  FPN deblock 1 (ConvTranspose2d kernel 2 stride 2): one GEMM per output parity,
//       rows = input pixels, output row = (2y+a, 2x+b)
//   G2  data gradient of U2 (4 taps gathering (2y+a, 2x+b))
// k_igemm: 128 pixels x 128 output channels per 256-thread block (4 waves, 64x64 each,
// v_mfma_f32_16x16x32_bf16 with the weights as the A operand so each lane ends up holding 4
// consecutive output channels of one pixel), K-steps of 64 channels of one tap, register-staged
// double-buffered LDS tiles (pitch 72 elements: conflict-free ds_read_b128), XCD-aware block
// order. Epilogue: bf16 output (optionally added into an existing image, optionally at a channel
// offset of a wider image = the FPN concat) + per-block BatchNorm partial sums (sum, sum of
// squares) of the stored values, reduced in a fixed order by rpc_bn_finalize.
// k_wgrad: dW[t][ci][co] = sum_rows x[src(row,t)][ci] * dz[row][co] with rows as the MFMA K
// dimension (row-major LDS tiles read back with ds_read_b64_tr_b16), split over row chunks into
// fp32 slabs reduced in a fixed order (k_slab_reduce). BatchNorm apply / backward are
// vectorised elementwise passes (8 channels per thread).
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "common.h"
#include "dense_common.h"
#include "rpc_hip.h"

namespace rpc {
namespace dn {

constexpr int BLK = 256;
constexpr int TM = 128;     // GEMM rows (pixels) per block
constexpr int TN = 128;     // output channels per block
constexpr int BK = 64;      // K-step = 64 channels of one tap
constexpr int LP = BK + 8;  // LDS pitch (elements)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef unsigned short u16;

// M_D2P (internal): the data gradient of S2 split by input-pixel parity (blockIdx.z = 2*py + px):
// a pixel of parity (py, px) receives only the taps ty in {1} (py = 0) or {0, 2} (py = 1), and
// likewise tx, so the four classes run 1, 2, 2 and 4 taps instead of 9 taps of mostly zero rows

// tap j < ntaps of parity (py, px) of M_D2P -> 3x3 tap index
__device__ __forceinline__ int d2p_tap(int j, int py, int px) {
  const int ntx = px ? 2 : 1;
  const int ty = py ? 2 * (j / ntx) : 1, tx = px ? 2 * (j % ntx) : 1;
  return ty * 3 + tx;
}

__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float((unsigned)h << 16); }

// ------------------------------------------------------------------ implicit GEMM (fwd / dgrad)
struct IG {
  const u16* src;  // K-operand image rows [S pixels][SP]
  int SP;
  int CIN;         // K channels per tap (multiple of 64)
  const u16* wt;   // [taps][COUT][CIN] bf16 (U2: [parity][COUT][CIN])
  int COUT;        // multiple of 128
  u16* out;        // output rows [O pixels][OP] at channel offset OOFF
  int OP, OOFF;
  int accum;       // add into the existing output
  float* part;     // [gridDim.z * gridDim.x][2 * COUT] BatchNorm partial sums, or null
  Img R, S, O;     // GEMM-row image, source image, output image
  int M;           // GEMM rows = R.B * R.H * R.W
  int flat;        // grid: 1 = row tiles x channel blocks flattened, a tile's channel blocks adjacent
};

// 1-tap maps (P1, U2: 2-4 K-steps per block, latency-bound prologue / epilogue) use ONE LDS tile
// pair (37 KB) so four blocks share a CU and hide each other's global round trips; the 9-tap maps
// keep the double-buffered pair (two blocks per CU).
template <int MAP>
__global__ __launch_bounds__(BLK, (taps_of<MAP>() == 1 ? 4 : 2)) void k_igemm(IG g) {
  constexpr int T = taps_of<MAP>();
  constexpr int NB = T == 1 ? 1 : 2;
  // the operand tiles, and after the K-loop the bf16 output tile [TM][TN] of the epilogue (32 KB)
  constexpr int TILEB = NB * (TM + TN) * LP * 2;
  static_assert(TILEB >= TM * TN * 2, "epilogue staging");
  __shared__ __attribute__((aligned(16))) unsigned char ldsb[TILEB];
  u16 (*sX)[TM * LP] = (u16 (*)[TM * LP])ldsb;
  u16 (*sW)[TN * LP] = (u16 (*)[TN * LP])(ldsb + NB * TM * LP * 2);
  __shared__ int sRow[TM * T];
  __shared__ float sP[2][2][TN];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wc = w >> 1, wp = w & 1;  // wave: output channels wc*64.., pixels wp*64..
  // flat grid: the COUT/TN channel blocks of one row tile are consecutive items on one XCD, so the
  // tile's activation rows are fetched from HBM once and re-read from that XCD's L2 (the 2-D grid
  // dispatched every tile of channel block 0 before any of block 1: each re-read went back to memory)
  const int ncob = g.COUT / TN, ntiles = g.flat ? gridDim.x / ncob : gridDim.x;
  int bx, cob;
  if (g.flat) {
    const int item = xcd_remap(blockIdx.x, gridDim.x);
    bx = item / ncob;
    cob = item - bx * ncob;
  } else {
    bx = xcd_remap(blockIdx.x, gridDim.x);
    cob = blockIdx.y;
  }
  // M_D2P: the 4-tap class (odd, odd) is dispatched first, the 1-tap class last (shorter tail)
  const int m0 = bx * TM, n0 = cob * TN, par = MAP == M_D2P ? 3 - (int)blockIdx.z : blockIdx.z;
  const int py = par >> 1, px = par & 1;
  // M_D2P: rows of parity class par, a (Hp x Wp) sub-grid of the row image
  const int Hp = MAP == M_D2P ? (g.R.H - py + 1) >> 1 : g.R.H, Wp = MAP == M_D2P ? (g.R.W - px + 1) >> 1 : g.R.W;
  const int Mrows = MAP == M_D2P ? g.R.B * Hp * Wp : g.M;
  if (m0 >= Mrows) return;
  const int KC = g.CIN / BK, NKS = (MAP == M_D2P ? (py + 1) * (px + 1) : T) * KC;
  const u16* wbase = g.wt + (MAP == M_U2 ? (size_t)par * g.COUT * g.CIN : 0);
  const int HW = g.R.H * g.R.W;

  for (int q = tid; q < TM * T; q += BLK) {
    const int r = q / T, t = q - r * T, m = m0 + r;
    int s = -1;
    if (MAP == M_D2P) {
      if (m < Mrows && t < (py + 1) * (px + 1)) {
        const int b = m / (Hp * Wp), rem = m - b * (Hp * Wp), yy = rem / Wp, xx = rem - yy * Wp;
        s = src_row<M_D2>(b, 2 * yy + py, 2 * xx + px, d2p_tap(t, py, px), g.S);
      }
    } else if (m < g.M) {
      const int b = m / HW, rem = m - b * HW, y = rem / g.R.W, x = rem - y * g.R.W;
      s = src_row<MAP>(b, y, x, t, g.S);
    }
    sRow[q] = s;
  }
  __syncthreads();

  // register staging: rx = activation chunks, rw = weight chunks of K-step ks (padding rows read
  // row 0 and are zeroed by a select, so the loads stay branch-free and in flight)
  uint4 rx0, rx1, rx2, rx3, rw0, rw1, rw2, rw3;
  const int srow = tid >> 3, sseg = (tid & 7) * 8;   // chunk s: row srow + 32*s, channels sseg..+8
#define IG_LOAD1(S, ks)                                                                             \
  {                                                                                                 \
    const int t_ = (ks) / KC, kc_ = (ks) - t_ * KC;                                                 \
    const int sr_ = sRow[(srow + 32 * S) * T + t_];                                                 \
    const unsigned keep_ = ~(unsigned)(sr_ >> 31);                                                  \
    uint4 v_ = *(const uint4*)(g.src + (size_t)max(sr_, 0) * g.SP + kc_ * BK + sseg);                \
    rx##S = make_uint4(v_.x & keep_, v_.y & keep_, v_.z & keep_, v_.w & keep_);                     \
    const int tw_ = MAP == M_D2P ? d2p_tap(t_, py, px) : t_;                                        \
    rw##S = *(const uint4*)(wbase + ((size_t)(tw_ * g.COUT + n0 + srow + 32 * S)) * g.CIN + kc_ * BK + sseg); \
  }
#define IG_LOAD(ks) { IG_LOAD1(0, ks) IG_LOAD1(1, ks) IG_LOAD1(2, ks) IG_LOAD1(3, ks) }
#define IG_STORE1(S, buf)                                          \
  *(uint4*)&sX[buf][(srow + 32 * S) * LP + sseg] = rx##S;          \
  *(uint4*)&sW[buf][(srow + 32 * S) * LP + sseg] = rw##S;
#define IG_STORE(buf) { IG_STORE1(0, buf) IG_STORE1(1, buf) IG_STORE1(2, buf) IG_STORE1(3, buf) }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  IG_LOAD(0)
  IG_STORE(0)
  __syncthreads();
  for (int ks = 0; ks < NKS; ++ks) {
    const int buf = NB == 2 ? (ks & 1) : 0;
    const bool more = ks + 1 < NKS;
    if (more) {
      IG_LOAD(ks + 1)
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the next tile's loads issued ahead of the MFMAs
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *(const bf16x8*)&sW[buf][(wc * 64 + i * 16 + (lane & 15)) * LP + kk * 32 + 8 * (lane >> 4)];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *(const bf16x8*)&sX[buf][(wp * 64 + j * 16 + (lane & 15)) * LP + kk * 32 + 8 * (lane >> 4)];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (NB == 1 && more) __syncthreads();   // one tile pair: every wave has read it before it is refilled
    if (more) {
      IG_STORE(NB == 2 ? (buf ^ 1) : 0)
    }
    __syncthreads();
  }
#undef IG_LOAD1
#undef IG_LOAD
#undef IG_STORE1
#undef IG_STORE

  // epilogue: lane holds channels co = n0 + wc*64 + i*16 + 4*(lane>>4) + r of pixel wp*64 + j*16 + (lane&15)
  if (!g.accum) {
    // staged through LDS as whole 256-byte pixel rows (granule gr of pixel p at slot gr ^ (p & 15)) and
    // written 16 bytes per lane: the 8-byte stores of the accumulator layout touch 16 rows per instruction
    // (store-issue bound, k_conv3x3x); BatchNorm sums from the stored bf16 values
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = wp * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q4 = lane >> 4, gr = (wc * 8 + i * 2 + (q4 >> 1)) ^ (p & 15);
        const unsigned lo = (unsigned)f2bf(acc[i][j][0]) | ((unsigned)f2bf(acc[i][j][1]) << 16);
        const unsigned hi = (unsigned)f2bf(acc[i][j][2]) | ((unsigned)f2bf(acc[i][j][3]) << 16);
        *(uint2*)(ldsb + p * 256 + gr * 16 + (q4 & 1) * 8) = make_uint2(lo, hi);
      }
    }
    __syncthreads();
    const int c = tid & 15, pq = tid >> 4;
    float t1[8], t2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t1[e] = t2[e] = 0.f;
#pragma unroll 4
    for (int k = 0; k < TM / 16; ++k) {
      const int p = pq + 16 * k, m = m0 + p;
      if (m >= Mrows) continue;
      int orow = m;
      if (MAP == M_U2) {
        const int b = m / HW, rem = m - b * HW, y = rem / g.R.W, x = rem - y * g.R.W;
        orow = out_row<MAP>(m, b, y, x, par, g.O);
      } else if (MAP == M_D2P) {
        const int b = m / (Hp * Wp), rem = m - b * (Hp * Wp), yy = rem / Wp, xx = rem - yy * Wp;
        orow = (b * g.R.H + 2 * yy + py) * g.R.W + 2 * xx + px;
      }
      const uint4 v = *(const uint4*)(ldsb + p * 256 + ((c ^ (p & 15)) * 16));
      *(uint4*)(g.out + (size_t)orow * g.OP + g.OOFF + n0 + c * 8) = v;
      const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float f0 = bf2f((u16)(u[e] & 0xffff)), f1 = bf2f((u16)(u[e] >> 16));
        t1[2 * e] += f0;
        t2[2 * e] += f0 * f0;
        t1[2 * e + 1] += f1;
        t2[2 * e + 1] += f1 * f1;
      }
    }
    if (g.part == nullptr) return;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      t1[e] += __shfl_xor(t1[e], 16, 64);
      t2[e] += __shfl_xor(t2[e], 16, 64);
      t1[e] += __shfl_xor(t1[e], 32, 64);
      t2[e] += __shfl_xor(t2[e], 32, 64);
    }
    __syncthreads();   // the tile reads are done: the sums go where it was
    float* sR = (float*)ldsb;   // [4 waves][2][TN]
    if (lane < 16) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sR[(w * 2 + 0) * TN + c * 8 + e] = t1[e];
        sR[(w * 2 + 1) * TN + c * 8 + e] = t2[e];
      }
    }
    __syncthreads();
    float* prow = g.part + ((size_t)blockIdx.z * ntiles + bx) * 2 * g.COUT;
    {
      const int k2 = tid >> 7, ch = tid & 127;
      prow[k2 * g.COUT + n0 + ch] = ((sR[(0 * 2 + k2) * TN + ch] + sR[(1 * 2 + k2) * TN + ch]) +
                                     sR[(2 * 2 + k2) * TN + ch]) + sR[(3 * 2 + k2) * TN + ch];
    }
    return;
  }
  float s1[4][4], s2[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int m = m0 + wp * 64 + j * 16 + (lane & 15);
    if (m >= Mrows) continue;
    int orow = m;
    if (MAP == M_U2) {
      const int b = m / HW, rem = m - b * HW, y = rem / g.R.W, x = rem - y * g.R.W;
      orow = out_row<MAP>(m, b, y, x, par, g.O);
    } else if (MAP == M_D2P) {
      const int b = m / (Hp * Wp), rem = m - b * (Hp * Wp), yy = rem / Wp, xx = rem - yy * Wp;
      orow = (b * g.R.H + 2 * yy + py) * g.R.W + 2 * xx + px;
    }
    u16* op = g.out + (size_t)orow * g.OP + g.OOFF + n0 + wc * 64 + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      uint2* p2 = (uint2*)(op + i * 16);
      if (g.accum) {
        uint2 e = *p2;
        v[0] += bf2f((u16)(e.x & 0xffff));
        v[1] += bf2f((u16)(e.x >> 16));
        v[2] += bf2f((u16)(e.y & 0xffff));
        v[3] += bf2f((u16)(e.y >> 16));
      }
      u16 hb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hb[r] = f2bf(v[r]);
        const float q = bf2f(hb[r]);
        s1[i][r] += q;
        s2[i][r] += q * q;
      }
      *p2 = make_uint2((unsigned)hb[0] | ((unsigned)hb[1] << 16), (unsigned)hb[2] | ((unsigned)hb[3] << 16));
    }
  }
  if (g.part == nullptr) return;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[i][r] += __shfl_xor(s1[i][r], o, 64);
        s2[i][r] += __shfl_xor(s2[i][r], o, 64);
      }
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = wc * 64 + i * 16 + 4 * (lane >> 4) + r;
        sP[wp][0][c] = s1[i][r];
        sP[wp][1][c] = s2[i][r];
      }
  }
  __syncthreads();
  float* prow = g.part + ((size_t)blockIdx.z * ntiles + bx) * 2 * g.COUT;
  if (tid < TN) {
    prow[n0 + tid] = sP[0][0][tid] + sP[1][0][tid];
    prow[g.COUT + n0 + tid] = sP[0][1][tid] + sP[1][1][tid];
  }
}

// ------------------------------------------------------------------ 3x3 stride-1 conv (S1) with halo tiles
// The 10 stride-1 layers of SECOND and their data gradients (and the 64-channel CenterHead convs).
// Block = 16x16 output pixels of one image x 64 output channels, 4 waves (pixel quarters, 64 px x
// 64 co each), 65 KB of LDS: two blocks share a CU, so one block's barriers and LDS stores overlap
// the other's MFMAs. Per 64-channel chunk the 18x18 input halo is staged ONCE in LDS and all 9
// taps read it at shifted rows (9x fewer activation loads than the generic implicit GEMM); the
// per-tap weight tiles (64 x 64, shared by every block through L2) stream through a 3-deep
// register ring into a double-buffered LDS tile; the next chunk's halo is prefetched into
// registers during taps 5-8.
constexpr int CT = 16;                  // spatial tile edge
constexpr int HT = CT + 2;              // halo edge
constexpr int HR = HT * HT;             // halo rows (324)
constexpr int CBLK = 256;               // threads
constexpr int HCH = (HR * 8 + CBLK - 1) / CBLK;   // halo 16-B chunks per thread (11)
constexpr int LP3 = 80;                 // LDS row pitch (elements): conflict-free ds_read_b128 fragments

struct C3 {
  const u16* src;  // input image rows [B*H*W][SP]
  int SP, CIN;
  const u16* wt;   // [9][COUT][CIN]
  int COUT;
  u16* out;        // [B*H*W][OP] at OOFF
  int OP, OOFF, accum;
  float* part;     // [tiles][2*COUT] or null
  int B, H, W, TY, TX;   // image, tiles per column / row
  // k_conv3x3x / y data gradients only (rpc_dense_conv_bnbwd): the output is dh of a BatchNorm + ReLU layer
  // with pre-activation image bnz [B*H*W][COUT] and forward parameters bnp (scale, beta, mean, invstd);
  // part then receives that layer's BatchNorm-backward partial sums (sum dm, sum dm * xhat), dm = dh * [pre > 0]
  const u16* bnz;
  const float* bnp;
  int ysplit;      // k_conv3x3y: the last ysplit items run as two 64-channel blocks each (launch_s1)
};

// TNB = 32 (half the output channels per block, twice the blocks): the grids of less than one round of two
// blocks per CU (CenterPoint's 64-channel head convs at 4 x 128 x 128: 256 tiles) — one wave per SIMD left every
// step's LDS-read / MFMA / barrier chain exposed
template <int DUMMY = 0, int TNB = 64>
__global__ __launch_bounds__(CBLK, 2) void k_conv3x3(C3 g) {
  static_assert(TNB == 64 || TNB == 32, "k_conv3x3: 32 or 64 output channels per block");
  constexpr int WCO = TNB;                // output channels per wave
  constexpr int NI = WCO / 16;            // 16-channel MFMA tiles per wave
  __shared__ __attribute__((aligned(16))) u16 sA[HR * LP3];
  __shared__ __attribute__((aligned(16))) u16 sW[2][TNB * LP3];
  __shared__ float sP[4][2][TNB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wp = w, wc = 0;
  const int ntiles = g.B * g.TY * g.TX;
  const int tile = xcd_remap(blockIdx.x, ntiles);
  const int b = tile / (g.TY * g.TX), trem = tile - b * g.TY * g.TX;
  const int ty0 = (trem / g.TX) * CT, tx0 = (trem % g.TX) * CT;
  const int n0 = blockIdx.y * TNB;
  const int NKC = g.CIN / BK, NS = 9 * NKC;

  // ---- halo staging (chunk q: halo row q>>3, 8 channels (q&7)*8). Out-of-image rows load row 0
  // and are zeroed when stored (the mask is applied at store time so the loads stay in flight).
  uint4 ra[HCH];
  unsigned hkeep = 0;
  auto halo_load = [&](int kc) {
    hkeep = 0;
#pragma unroll
    for (int i = 0; i < HCH; ++i) {
      const int q = tid + i * CBLK;
      const int hr = q >> 3, seg = (q & 7) * 8;
      const int hy = hr / HT, hx = hr - hy * HT;
      const int y = ty0 + hy - 1, x = tx0 + hx - 1;
      const bool ok = q < HR * 8 && y >= 0 && y < g.H && x >= 0 && x < g.W;
      hkeep |= (ok ? 1u : 0u) << i;
      const size_t row = ok ? ((size_t)(b * g.H + y) * g.W + x) : 0;
      ra[i] = *(const uint4*)(g.src + row * g.SP + kc * BK + seg);
    }
  };
  auto halo_store = [&]() {
#pragma unroll
    for (int i = 0; i < HCH; ++i) {
      const int q = tid + i * CBLK;
      const unsigned keep = ((hkeep >> i) & 1u) ? 0xffffffffu : 0u;
      if (q < HR * 8)
        *(uint4*)&sA[(q >> 3) * LP3 + (q & 7) * 8] =
            make_uint4(ra[i].x & keep, ra[i].y & keep, ra[i].z & keep, ra[i].w & keep);
    }
  };
  // ---- weight tiles: step s = kc*9 + t; chunk q = tid, tid+256: row q>>3, channels (q&7)*8
  const int wrow = tid >> 3, wseg = (tid & 7) * 8;
  const u16* wbase = g.wt + (size_t)(n0 + wrow) * g.CIN + wseg;
  const size_t wtap = (size_t)g.COUT * g.CIN, whalf = (size_t)32 * g.CIN;
#define C3_WLOAD(R, s)                                                          \
  {                                                                             \
    const int kc_ = (s) / 9, t_ = (s) - kc_ * 9;                                \
    const u16* p_ = wbase + t_ * wtap + kc_ * BK;                               \
    R##a = *(const uint4*)p_;                                                   \
    if constexpr (TNB == 64) R##b = *(const uint4*)(p_ + whalf);                \
  }
#define C3_WSTORE(R, buf)                                                     \
  {                                                                           \
    *(uint4*)&sW[buf][wrow * LP3 + wseg] = R##a;                               \
    if constexpr (TNB == 64) *(uint4*)&sW[buf][(wrow + 32) * LP3 + wseg] = R##b; \
  }
  uint4 r0a, r0b, r1a, r1b, r2a, r2b;

  f32x4 acc[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // pixel p = wp*64 + j*16 + (lane&15) -> tile row wp*4 + j, column lane&15
  const int pcol = lane & 15;
  const u16* aw = &sW[0][(wc * WCO + (lane & 15)) * LP3 + 8 * (lane >> 4)];
  const u16* ab = &sA[(wp * 4 * HT + pcol) * LP3 + 8 * (lane >> 4)];
#define C3_COMPUTE(buf, t)                                                                                  \
  {                                                                                                         \
    const int dy_ = (t) / 3, dx_ = (t) % 3;                                                                 \
    _Pragma("unroll") for (int kk = 0; kk < BK / 32; ++kk) {                                                \
      bf16x8 a[NI], bb[4];                                                                                  \
      _Pragma("unroll") for (int i = 0; i < NI; ++i)                                                        \
        a[i] = *(const bf16x8*)(aw + (buf) * (TNB * LP3) + i * 16 * LP3 + kk * 32);                           \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                         \
        bb[j] = *(const bf16x8*)(ab + ((j + dy_) * HT + dx_) * LP3 + kk * 32);                               \
      _Pragma("unroll") for (int i = 0; i < NI; ++i)                                                        \
        _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                       \
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[j], acc[i][j], 0, 0, 0);             \
    }                                                                                                       \
  }
  // one tap step: MFMAs on LDS tile s; tile s+1 (register slot RN) -> the other LDS buffer;
  // barrier; slot RN reloaded with tile s+4. All loads unconditional (clamped step index) so
  // the counted vmcnt waits see a straight-line stream.
#define C3_TAP(t, RN)                                      \
  {                                                        \
    const int s_ = kc * 9 + (t);                           \
    if ((t) == 5) halo_load(min(kc + 1, NKC - 1));         \
    C3_COMPUTE(s_ & 1, t)                                  \
    C3_WSTORE(RN, (s_ + 1) & 1)                            \
    __syncthreads();                                       \
    C3_WLOAD(RN, min(s_ + 4, NS - 1))                      \
  }

  // prologue: halo(0) and W tile 0 in LDS; tiles 1, 2, 3 in flight in slots r1, r2, r0
  halo_load(0);
  C3_WLOAD(r0, 0)
  halo_store();
  C3_WSTORE(r0, 0)
  C3_WLOAD(r1, min(1, NS - 1))
  C3_WLOAD(r2, min(2, NS - 1))
  C3_WLOAD(r0, min(3, NS - 1))
  __syncthreads();
  for (int kc = 0; kc < NKC; ++kc) {
    if (kc > 0) {
      halo_store();
      __syncthreads();
    }
    C3_TAP(0, r1)
    C3_TAP(1, r2)
    C3_TAP(2, r0)
    C3_TAP(3, r1)
    C3_TAP(4, r2)
    C3_TAP(5, r0)
    C3_TAP(6, r1)
    C3_TAP(7, r2)
    C3_TAP(8, r0)
  }
#undef C3_TAP
#undef C3_COMPUTE
#undef C3_WLOAD
#undef C3_WSTORE

  // ---- epilogue (as k_igemm): lane holds co = n0 + wc*64 + i*16 + 4*(lane>>4) + r of pixel (wp*4+j, lane&15)
  float s1[NI][4], s2[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int y = ty0 + wp * 4 + j, x = tx0 + pcol;
    if (y >= g.H || x >= g.W) continue;
    const size_t orow = (size_t)(b * g.H + y) * g.W + x;
    u16* op = g.out + orow * g.OP + g.OOFF + n0 + wc * WCO + 4 * (lane >> 4);
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      uint2* p2 = (uint2*)(op + i * 16);
      if (g.accum) {
        uint2 e = *p2;
        v[0] += bf2f((u16)(e.x & 0xffff));
        v[1] += bf2f((u16)(e.x >> 16));
        v[2] += bf2f((u16)(e.y & 0xffff));
        v[3] += bf2f((u16)(e.y >> 16));
      }
      u16 hb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hb[r] = f2bf(v[r]);
        const float q = bf2f(hb[r]);
        s1[i][r] += q;
        s2[i][r] += q * q;
      }
      *p2 = make_uint2((unsigned)hb[0] | ((unsigned)hb[1] << 16), (unsigned)hb[2] | ((unsigned)hb[3] << 16));
    }
  }
  if (g.part == nullptr) return;
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[i][r] += __shfl_xor(s1[i][r], o, 64);
        s2[i][r] += __shfl_xor(s2[i][r], o, 64);
      }
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = wc * WCO + i * 16 + 4 * (lane >> 4) + r;
        sP[wp][0][c] = s1[i][r];
        sP[wp][1][c] = s2[i][r];
      }
  }
  __syncthreads();
  float* prow = g.part + (size_t)tile * 2 * g.COUT;
  if (tid < TNB) {
    prow[n0 + tid] = ((sP[0][0][tid] + sP[1][0][tid]) + sP[2][0][tid]) + sP[3][0][tid];
    prow[g.COUT + n0 + tid] = ((sP[0][1][tid] + sP[1][1][tid]) + sP[2][1][tid]) + sP[3][1][tid];
  }
}

// ------------------------------------------------------------------ 3x3 stride-1 conv, 128-channel blocks, LDS-DMA pipeline
// k_conv3x3w: the S1 launches whose output channels are a multiple of 128 (SECOND's 128/256-channel
// layers and their data gradients). One 512-thread block (8 waves, one block per CU, 146 KB of LDS)
// computes a 16x16-pixel tile x 128 output channels; wave w owns 4 tile rows (64 px) x 64 channels,
// the same 4x4 MFMA accumulator tiles as k_conv3x3, and the waves sharing a SIMD (w, w + 4) hold
// the upper and the lower half of the tile (a half-filled bottom tile costs half the SIMD time).
// Staging is LDS-DMA only (global_load_lds_dwordx4, no VGPR round trip): per 64-channel chunk the
// 18x18 halo goes into one of two halo buffers during tap 1 of the previous chunk, and the 128 x 64
// weight tile of each tap goes into a 4-slot ring two taps ahead. Every buffer is an unpadded image
// of 128-byte rows with the 16-byte granules XOR-swizzled (weights by (row >> 1) & 7, halo by a
// column table) — applied on the DMA's per-lane SOURCE address, since the DMA writes lane-linearly —
// so each ds_read_b128 lane group of the MFMA operand reads hits 16 distinct bank slots. One raw barrier per tap, after a counted vmcnt that
// retires exactly that tap's tile (and the halo at a chunk start); DMAs stay in flight across it.
// Out-of-image halo pixels are DMA'd from a zero row. Epilogue as k_conv3x3 (bf16 store, optional
// accumulate / channel offset, per-tile BatchNorm partial sums of the stored values).
constexpr int WB = 512;                       // threads
constexpr int HROW = 128;                     // bytes per halo / weight LDS row (64 bf16 channels)
constexpr int HBUF = 41 * 1024;               // halo buffer: 324 rows (41.5 KB) rounded to whole DMA KBs
constexpr int WTILE = 128 * HROW;             // weight tile: 128 output channels x 64 channels
constexpr int WRING = 4;                      // weight ring slots
constexpr int WDIST = 2;                      // weight tiles in flight ahead of the one computed
constexpr int WLDS = 2 * HBUF + WRING * WTILE;   // 149504 B
constexpr int HTAP = 1;                       // tap of chunk c at which the halo of chunk c + 1 is issued

__device__ uint4 g_zero_row[256];             // 4 KB of zeros: source of out-of-image halo pixels (any chunk offset)

// halo granule swizzle by column hx (0..17): slot = granule ^ hswz(hx). Found by exhaustive search so
// that every ds_read_b128 lane group of the B-operand reads (16 consecutive columns from dx = 0, 1, 2;
// granule pairs kk*4 + {0,1} / {2,3} split over the groups as the hardware groups lanes) hits 16
// distinct 16-byte bank slots; the column parity picks the half of the 256-byte bank row.
__device__ __forceinline__ int hswz(int hx) { return (int)((0x062654210ull >> (4 * (hx >> 1))) & 7); }

__device__ __forceinline__ void glds16(const void* g, unsigned char* l) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

template <int DUMMY = 0>
__global__ __launch_bounds__(WB, 2) void k_conv3x3w(C3 g) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WLDS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wc = (w >> 1) & 1, wp = (w & 1) | ((w >> 2) << 1);   // SIMD partners w, w+4: rows 0-7 / 8-15
  const int ncob = g.COUT >> 7;
  const int ntiles = g.B * g.TY * g.TX;
  const int item = xcd_remap(blockIdx.x, ntiles * ncob);           // tile-major: a tile's co-blocks adjacent
  const int tile = item / ncob, cob = item - tile * ncob;
  const int b = tile / (g.TY * g.TX), trem = tile - b * g.TY * g.TX;
  const int ty0 = (trem / g.TX) * CT, tx0 = (trem % g.TX) * CT;
  const int n0 = cob * 128;
  const int NKC = g.CIN / BK, NS = 9 * NKC;
  unsigned char* const hbuf = lds;
  unsigned char* const wring = lds + 2 * HBUF;

  // ---- DMA sources, fixed per lane. Halo row r = hy*18 + hx holds the 8 granules of 8 channels with
  // granule g at slot g ^ hswz(hx) (a function of the column only, so every tap's operand address is
  // the lane's base + constants); weight row r (output channel n0 + r) at g ^ ((r >> 1) & 7).
  // Halo: 41 wave-instructions of 1 KB over the 8 waves, 6 per wave (surplus ones repeat instruction 40:
  // the same bytes to the same place). Weights: 16 instructions, 2 per wave.
  const u16* hsrc[6];
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const int k = min(w + 8 * m, 40);
    const int P = k * 64 + lane, r = P >> 3, pg = P & 7;
    const int hy = r / HT, hx = r - hy * HT;
    const int y = ty0 + hy - 1, x = tx0 + hx - 1;
    const int gl = pg ^ hswz(hx);
    hsrc[m] = (r < HR && y >= 0 && y < g.H && x >= 0 && x < g.W)
                  ? g.src + ((size_t)(b * g.H + y) * g.W + x) * g.SP + gl * 8
                  : (const u16*)g_zero_row;
  }
  const u16* wsrc[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int P = (2 * w + m) * 64 + lane, r = P >> 3, pg = P & 7;
    wsrc[m] = g.wt + (size_t)(n0 + r) * g.CIN + (pg ^ ((r >> 1) & 7)) * 8;
  }
  auto issue_halo = [&](int kc, int hb) {
#pragma unroll
    for (int m = 0; m < 6; ++m)
      glds16(hsrc[m] + kc * BK, hbuf + hb * HBUF + min(w + 8 * m, 40) * 1024);
  };
  auto issue_w = [&](int s) {
    s = min(s, NS - 1);
    const int kc = s / 9, t = s - kc * 9;
    const size_t off = (size_t)t * g.COUT * g.CIN + kc * BK;
#pragma unroll
    for (int m = 0; m < 2; ++m) glds16(wsrc[m] + off, wring + (s & (WRING - 1)) * WTILE + (2 * w + m) * 1024);
  };

  // ---- MFMA operand addresses: A (weights) rows wc*64 + i*16 + a15, B (halo) rows (wp*4 + j + dy)*18
  // + dx + a15; granule kk*4 + q swizzled as stored
  const int a15 = lane & 15, q = lane >> 4;
  int woff[2], hoff[3][2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    woff[kk] = (wc * 64 + a15) * HROW + (((kk * 4 + q) ^ ((a15 >> 1) & 7)) * 16);
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
      hoff[dx][kk] = (wp * 4 * HT + dx + a15) * HROW + (((kk * 4 + q) ^ hswz(dx + a15)) * 16);
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: halo(0), weight tiles 0 .. WDIST-1
  issue_halo(0, 0);
#pragma unroll
  for (int s = 0; s < WDIST; ++s) issue_w(s);

  // ---- main loop, staggered: every step s is a READ phase (issue the DMAs two taps ahead, load
  // this step's operand fragments) and a MATH phase (32 MFMAs from registers), each closed by a
  // barrier. Waves 4-7 (tile rows 8-15) run one phase behind waves 0-3 (rows 0-7) — one extra
  // barrier before their loop, one after waves 0-3's — so on every SIMD one wave's MFMAs overlap its
  // partner's LDS reads and DMA issue. RAW: tile s + 1 is retired (counted vmcnt: only younger DMAs
  // stay in flight) by each wave before the barrier that precedes the first read of it by either
  // group (waves 0-3 in MATH(s), waves 4-7 in READ(s)). WAR: ring slot (s + 2) & 3 last held tile
  // s - 2, whose last reads completed (lgkmcnt(0)) before an older barrier; the halo buffer of chunk
  // kc + 1 last held chunk kc - 1. A wave whose 4 rows are all below the image skips its reads and
  // MFMAs (the bottom tile row of a 200-row image is half full).
  const int grp = w >> 2;
  const bool live = ty0 + wp * 4 < g.H;
  asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // halo 0 + tile 0
  if (grp) asm volatile("s_barrier" ::: "memory");
#define C3W_STEP(t, LIVE)                                                                                     \
  {                                                                                                           \
    const int s_ = kc * 9 + (t);                                                                              \
    issue_w(s_ + WDIST);                                                                                      \
    if ((t) == HTAP) issue_halo(min(kc + 1, NKC - 1), (kc + 1) & 1);                                          \
    const unsigned char* hb_ = hbuf + (kc & 1) * HBUF;                                                        \
    const unsigned char* wt_ = wring + (s_ & (WRING - 1)) * WTILE;                                            \
    constexpr int dy_ = (t) / 3, dx_ = (t) % 3;                                                               \
    bf16x8 av[2][4], bv[2][4];                                                                                \
    if (LIVE) {                                                                                               \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) {                                                      \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                         \
          av[kk][i] = *(const bf16x8*)(wt_ + woff[kk] + i * 16 * HROW);                                       \
        _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                         \
          bv[kk][j] = *(const bf16x8*)(hb_ + hoff[dx_][kk] + (j + dy_) * HT * HROW);                          \
      }                                                                                                       \
    }                                                                                                         \
    if (grp) {                                                                                                \
      if ((t) == HTAP || (t) == HTAP + 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                    \
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");                                                   \
    }                                                                                                         \
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");                                           \
    if (LIVE) {                                                                                               \
      __builtin_amdgcn_s_setprio(1);                                                                          \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                                        \
        _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                         \
          _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                       \
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[kk][i], bv[kk][j], acc[i][j], 0, 0, 0);    \
      __builtin_amdgcn_s_setprio(0);                                                                          \
    }                                                                                                         \
    if (!grp) {                                                                                               \
      if ((t) == HTAP || (t) == HTAP + 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                    \
      else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");                                                   \
    }                                                                                                         \
    asm volatile("s_barrier" ::: "memory");                                                                   \
  }
  if (live) {
    for (int kc = 0; kc < NKC; ++kc) {
      C3W_STEP(0, true)
      C3W_STEP(1, true)
      C3W_STEP(2, true)
      C3W_STEP(3, true)
      C3W_STEP(4, true)
      C3W_STEP(5, true)
      C3W_STEP(6, true)
      C3W_STEP(7, true)
      C3W_STEP(8, true)
    }
  } else {   // DMA issue and barriers only
    for (int kc = 0; kc < NKC; ++kc) {
      C3W_STEP(0, false)
      C3W_STEP(1, false)
      C3W_STEP(2, false)
      C3W_STEP(3, false)
      C3W_STEP(4, false)
      C3W_STEP(5, false)
      C3W_STEP(6, false)
      C3W_STEP(7, false)
      C3W_STEP(8, false)
    }
  }
#undef C3W_STEP
  if (!grp) asm volatile("s_barrier" ::: "memory");
  // drain every DMA (the surplus re-issues too) before the LDS is reused or the block exits
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue: lane holds co = n0 + wc*64 + i*16 + 4q + r of pixel (wp*4 + j, a15)
  float s1[4][4], s2[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int y = ty0 + wp * 4 + j, x = tx0 + a15;
    if (y >= g.H || x >= g.W) continue;
    const size_t orow = (size_t)(b * g.H + y) * g.W + x;
    u16* op = g.out + orow * g.OP + g.OOFF + n0 + wc * 64 + 4 * q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      uint2* p2 = (uint2*)(op + i * 16);
      if (g.accum) {
        uint2 e = *p2;
        v[0] += bf2f((u16)(e.x & 0xffff));
        v[1] += bf2f((u16)(e.x >> 16));
        v[2] += bf2f((u16)(e.y & 0xffff));
        v[3] += bf2f((u16)(e.y >> 16));
      }
      u16 hb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hb[r] = f2bf(v[r]);
        const float qv = bf2f(hb[r]);
        s1[i][r] += qv;
        s2[i][r] += qv * qv;
      }
      *p2 = make_uint2((unsigned)hb[0] | ((unsigned)hb[1] << 16), (unsigned)hb[2] | ((unsigned)hb[3] << 16));
    }
  }
  if (g.part == nullptr) return;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[i][r] += __shfl_xor(s1[i][r], o, 64);
        s2[i][r] += __shfl_xor(s2[i][r], o, 64);
      }
    }
  float* sP = (float*)lds;   // [4 wp][2][128]
  if (a15 == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = wc * 64 + i * 16 + 4 * q + r;
        sP[(wp * 2 + 0) * 128 + c] = s1[i][r];
        sP[(wp * 2 + 1) * 128 + c] = s2[i][r];
      }
  }
  __syncthreads();
  float* prow = g.part + (size_t)tile * 2 * g.COUT;
  if (tid < 128) {
    prow[n0 + tid] = ((sP[0 * 128 + tid] + sP[2 * 128 + tid]) + sP[4 * 128 + tid]) + sP[6 * 128 + tid];
  } else if (tid < 256) {
    const int c = tid - 128;
    prow[g.COUT + n0 + c] = ((sP[1 * 128 + c] + sP[3 * 128 + c]) + sP[5 * 128 + c]) + sP[7 * 128 + c];
  }
}

// ------------------------------------------------------------------ 3x3 stride-1 conv, 16x32-pixel tiles x 128 channels
// k_conv3x3x: k_conv3x3w's 8-wave LDS-DMA pipeline with twice the pixels per wave. Each wave owns
// 4 tile rows x 32 columns (128 pixels) x 64 output channels = 8 x 4 MFMA accumulator tiles (128
// VGPRs), so one step's 32 MFMAs read 12 operand fragments (8 pixel + 4 weight) instead of 16
// (4 + 4 for 16 MFMAs, twice): 0.375 ds_read_b128 per MFMA instead of 0.5, and each staged weight
// tile feeds 512 pixels instead of 256 (half the weight bytes per FLOP through L2 and the DMA).
// K-steps are 32 channels of one tap (a step still has 32 MFMAs per wave), so a 32-channel chunk
// of the 18x34 halo (36-pixel LDS row pitch, 64-byte rows: 41 KB) and an 8-slot ring of 128 x 32
// weight tiles (8 KB each) (four in flight ahead of the one computed) fit twice the tile in 146 KB. 64-byte rows carry their four 16-byte
// granules XOR-swizzled by bit 2 of the pixel column / weight row (g ^ ((x >> 1) & 2)), found by
// exhaustive search so that every ds_read_b128 lane group of an MFMA operand read (16 consecutive
// columns from dx = 0..2 or 16..18; 16 aligned weight rows) hits 16 distinct bank slots; the row
// pitch of 36 pixels keeps the bank of a pixel a function of its column only, so every tap's
// operand address is the lane's base + constants. Staggered READ / MATH phases, counted vmcnt
// waits, one raw barrier per phase and the zero-row halo as in k_conv3x3w. SECOND's 200x176
// layers: 468 tiles = 1.83 rounds of the CUs (858 16x16 tiles = 3.35 rounds).
constexpr int XTW = 32;                        // tile columns
constexpr int XHW = XTW + 2;                   // halo columns (34)
constexpr int XHP = 36;                        // halo LDS row pitch in pixels (bank = f(column))
constexpr int XHR = HT * XHP;                  // halo LDS rows (648)
constexpr int XROW = 64;                       // bytes per LDS row (32 bf16 channels)
constexpr int XBK = 32;                        // channels per K-step
constexpr int XHBUF = 41 * 1024;               // halo buffer: 648 rows (40.5 KB) rounded to whole DMA KBs
constexpr int XWTILE = 128 * XROW;             // weight tile: 128 output channels x 32 channels (8 KB)
constexpr int XWR = 8;                         // weight ring slots
constexpr int XWD = 4;                         // weight tiles in flight ahead of the one computed
constexpr int XLDS = 2 * XHBUF + XWR * XWTILE;     // 149504 B
constexpr int XHI = 6;                         // halo DMA instructions per wave (41 over 8 waves)

__device__ __forceinline__ int xswz(int x) { return (x >> 1) & 2; }

// DBG (timing experiments only, rpc_dense_tune knob 4; outputs are garbage): bit 0 = no MFMAs, bit 1 =
// no operand reads, bit 2 = no weight DMAs, bit 3 = no halo DMAs, bit 4 = no barriers in the K-loop,
// bit 5 = the register-direct epilogue (8-byte stores from the accumulator layout)
template <int DBG = 0>
__global__ __launch_bounds__(WB, 2) void k_conv3x3x(C3 g) {
  // ONE LDS object: a second __shared__ array gives the accesses alias scopes, and the compiler then
  // waits for every LDS-DMA in flight (vmcnt(0)) before each step's operand reads
  __shared__ __attribute__((aligned(1024))) unsigned char lds[XLDS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wc = (w >> 1) & 1, wp = (w & 1) | ((w >> 2) << 1);   // SIMD partners w, w+4: rows 0-7 / 8-15
  const int ncob = g.COUT >> 7;
  const int ntiles = g.B * g.TY * g.TX;
  const int item = xcd_remap(blockIdx.x, ntiles * ncob);           // tile-major: a tile's co-blocks adjacent
  const int tile = item / ncob, cob = item - tile * ncob;
  const int b = tile / (g.TY * g.TX), trem = tile - b * g.TY * g.TX;
  const int ty0 = (trem / g.TX) * CT, tx0 = (trem % g.TX) * XTW;
  const int n0 = cob * 128;
  const int NKC = g.CIN / XBK, NS = 9 * NKC;
  unsigned char* const hbuf = lds;
  unsigned char* const wring = lds + 2 * XHBUF;

  // ---- DMA sources, fixed per lane. Instruction k of a halo chunk writes LDS granules k*64 + lane:
  // row r = hy*36 + hx, slot j holds channel granule j ^ xswz(hx) (pad columns 34, 35 and rows past
  // 648 read the zero row). Weights: instruction w writes rows w*16 + (lane >> 2) = output channel
  // n0 + r, slot j = granule j ^ xswz(r).
  // 32-bit byte offsets into buffer resources (rpc_dense_conv checks the image and weights fit in 2 GB);
  // out-of-image halo pixels get an offset past the range, which the buffer load returns as zeros
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)g.src, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwt = __builtin_amdgcn_make_buffer_rsrc((void*)g.wt, (short)0, 0x7fffffff, 0x00020000);
  unsigned hofs[XHI];
#pragma unroll
  for (int m = 0; m < XHI; ++m) {
    const int k = min(w + 8 * m, 40);
    const int P = k * 64 + lane, r = P >> 2, j = P & 3;
    const int hy = r / XHP, hx = r - hy * XHP;
    const int y = ty0 + hy - 1, x = tx0 + hx - 1;
    hofs[m] = (r < XHR && hx < XHW && y >= 0 && y < g.H && x >= 0 && x < g.W)
                  ? (unsigned)((((b * g.H + y) * g.W + x) * g.SP + (j ^ xswz(hx)) * 8) * 2)
                  : 0x80000000u;
  }
  unsigned wofs;
  {
    const int r = w * 16 + (lane >> 2), j = lane & 3;
    wofs = (unsigned)(((n0 + r) * g.CIN + (j ^ xswz(r)) * 8) * 2);
  }
  auto issue_halo = [&](int kc, int hb) {
    if (DBG & 8) return;
#pragma unroll
    for (int m = 0; m < XHI; ++m)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (__attribute__((address_space(3))) void*)(hbuf + hb * XHBUF + min(w + 8 * m, 40) * 1024), 16,
          hofs[m], kc * XBK * 2, 0, 0);
  };
  const int wtap = g.COUT * g.CIN * 2;
  auto issue_w = [&](int s) {
    if (DBG & 4) return;
    s = min(s, NS - 1);
    const int kc = s / 9, t = s - kc * 9;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(
        rwt, (__attribute__((address_space(3))) void*)(wring + (s & (XWR - 1)) * XWTILE + w * 1024), 16, wofs,
        t * wtap + kc * XBK * 2, 0, 0);
  };

  // ---- MFMA operand addresses: A (weights) rows wc*64 + i*16 + a15; B (halo) pixel (wp*4 + r + dy,
  // hh*16 + a15 + dx) — the swizzle of column hh*16 + a15 + dx equals that of a15 + dx
  const int a15 = lane & 15, q = lane >> 4;
  const int woff = (wc * 64 + a15) * XROW + ((q ^ xswz(a15)) * 16);
  int hoff[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) hoff[dx] = (wp * 4 * XHP + dx + a15) * XROW + ((q ^ xswz(dx + a15)) * 16);

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  issue_halo(0, 0);
#pragma unroll
  for (int s = 0; s < XWD; ++s) issue_w(s);

  // DBG bit 128: operand fragments read a quarter step ahead (C3X_PSTEP, one barrier per step) instead of
  // the partner groups staggered one phase (two barriers per step). Measured equal (100x88 256->256 63.8
  // vs 62.4 us, 200x176 128->128 69.7 vs 69.7, profiles/r03_conv_pipe.log): the stagger already hides
  // the reads here, unlike k_conv3x3y's, so the staggered loop stays the default
  constexpr bool PIPE = (DBG & 128) != 0;
  const int grp = PIPE ? 0 : w >> 2;
  const bool live = ty0 + wp * 4 < g.H;
  static_assert(XWD == 4 && XHI == 6 && HTAP + XWD <= 8, "vmcnt immediates below");
  // halo 0 + tile 0 (pipelined: + tile 1; tiles 2, 3 stay in flight)
  if (PIPE) asm volatile("s_waitcnt vmcnt(2)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(3)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (grp) asm volatile("s_barrier" ::: "memory");
  // per step: 1 weight DMA XWD tiles ahead (+ XHI halo DMAs at tap HTAP, after it); the tile of the next
  // step is retired by vmcnt(XWD - 1), or vmcnt(XWD - 1 + XHI) at taps HTAP .. HTAP + XWD - 1 while the
  // halo is younger than that tile (it is retired XWD steps after its issue)
// the step's wait: retire the next step's tile (vmcnt 3; 9 while the halo issued at HTAP is younger than it); LAST
// (the last K-chunk, which issues no weight DMA past the last real tile): the tiles still in flight at step t are
// those of steps t + 1 .. 8, so vmcnt(7 - t) from step 9 - XWD on (the halo is retired by then)
#define C3X_VMWAIT(t, LAST)                                                                                   \
  {                                                                                                           \
    if ((t) >= HTAP && (t) < HTAP + XWD) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");                     \
    else if ((LAST) && (t) == 5) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");                            \
    else if ((LAST) && (t) == 6) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");                            \
    else if ((LAST) && (t) >= 7) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                            \
    else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");                                                     \
  }
#define C3X_STEP(t, LIVE, LAST)                                                                               \
  {                                                                                                           \
    const int s_ = kc * 9 + (t);                                                                              \
    if (!(LAST) || (t) + XWD < 9) issue_w(s_ + XWD);                                                          \
    if ((t) == HTAP) issue_halo(min(kc + 1, NKC - 1), (kc + 1) & 1);                                          \
    const unsigned char* hb_ = hbuf + (kc & 1) * XHBUF;                                                       \
    const unsigned char* wt_ = wring + (s_ & (XWR - 1)) * XWTILE;                                             \
    constexpr int dy_ = (t) / 3, dx_ = (t) % 3;                                                               \
    bf16x8 av[4], bv[8];                                                                                      \
    if (DBG & 2) {                                                                                            \
      _Pragma("unroll") for (int i = 0; i < 4; ++i) av[i] = __builtin_bit_cast(bf16x8, make_uint4(lane, i, w, s_)); \
      _Pragma("unroll") for (int j = 0; j < 8; ++j) bv[j] = __builtin_bit_cast(bf16x8, make_uint4(j, lane, s_, w)); \
    }                                                                                                         \
    if (LIVE && !(DBG & 2)) {                                                                                 \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                           \
        av[i] = *(const bf16x8*)(wt_ + woff + i * 16 * XROW);                                                 \
      _Pragma("unroll") for (int j = 0; j < 8; ++j)                                                           \
        bv[j] = *(const bf16x8*)(hb_ + hoff[dx_] + ((j >> 1) + dy_) * XHP * XROW + (j & 1) * 16 * XROW);      \
    }                                                                                                         \
    if (grp) C3X_VMWAIT(t, LAST)                                                                              \
    if (DBG & 16) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); else asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");                                           \
    if (LIVE && !(DBG & 1)) {                                                                                 \
      __builtin_amdgcn_s_setprio(1);                                                                          \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                           \
        _Pragma("unroll") for (int j = 0; j < 8; ++j)                                                         \
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);              \
      __builtin_amdgcn_s_setprio(0);                                                                          \
    }                                                                                                         \
    if (!grp) C3X_VMWAIT(t, LAST)                                                                             \
    if (!(DBG & 16)) asm volatile("s_barrier" ::: "memory");                                                  \
  }
  // pipelined form: a step's 32 MFMAs run as four quarters (the 4 weight fragments x the 2 halo fragments
  // of one tile row); before quarter q's MFMAs the wave reads quarter q + 1's 2 halo fragments, before
  // quarter 3's the next step's 4 weight fragments and its quarter-0 halo fragments, so every LDS read
  // lies under the same wave's MFMAs (fragment registers: two 4-fragment weight buffers + a 2 x 2 halo
  // ring = the former loop's 48). The next step's tile must then be published one step earlier: step s
  // retires tile s + 2 (vmcnt(2), or vmcnt(8) while a halo chunk issued at step s - 2 .. s is younger),
  // so a halo chunk issued at tap HTAP is retired at tap HTAP + 2 <= 7, before tap 8 reads its first
  // fragments; its buffer was last read during step (kc - 1, 8). Tile s + 4 goes to ring slot
  // (s + 4) & 7, last read during step s - 4. At the last step the reads for "step NS" hit valid LDS
  // (clamped tile / halo) and are never used.
#define C3X_PREAD_B(FB, tn, kn, qq)                                                                         \
  {                                                                                                         \
    const unsigned char* hb_ = hbuf + ((kn) & 1) * XHBUF;                                                   \
    const int dy_ = (tn) / 3, dx_ = (tn) % 3;                                                               \
    FB[0] = *(const bf16x8*)(hb_ + hoff[dx_] + ((qq) + dy_) * XHP * XROW);                                  \
    FB[1] = *(const bf16x8*)(hb_ + hoff[dx_] + ((qq) + dy_) * XHP * XROW + 16 * XROW);                      \
  }
#define C3X_PREAD_A(FA, sn)                                                                                 \
  {                                                                                                         \
    const unsigned char* wt_ = wring + ((sn) & (XWR - 1)) * XWTILE;                                         \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) FA[i] = *(const bf16x8*)(wt_ + woff + i * 16 * XROW);     \
  }
#define C3X_PMMA(FA, FB, qq)                                                                                \
  __builtin_amdgcn_s_setprio(1);                                                                            \
  _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                             \
    _Pragma("unroll") for (int j = 0; j < 2; ++j)                                                           \
      acc[i][2 * (qq) + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA[i], FB[j], acc[i][2 * (qq) + j], 0, 0, 0); \
  __builtin_amdgcn_s_setprio(0);
#define C3X_PSTEP(t, FA, NA, LIVE)                                                                          \
  {                                                                                                         \
    const int s_ = kc * 9 + (t);                                                                            \
    issue_w(s_ + XWD);                                                                                      \
    if ((t) == HTAP) issue_halo(min(kc + 1, NKC - 1), (kc + 1) & 1);                                        \
    if (LIVE) {                                                                                             \
      C3X_PREAD_B(by, (t), kc, 1)                                                                           \
      asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");                                                    \
      C3X_PMMA(FA, bx, 0)                                                                                   \
      C3X_PREAD_B(bx, (t), kc, 2)                                                                           \
      asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");                                                    \
      C3X_PMMA(FA, by, 1)                                                                                   \
      C3X_PREAD_B(by, (t), kc, 3)                                                                           \
      asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");                                                    \
      C3X_PMMA(FA, bx, 2)                                                                                   \
      C3X_PREAD_A(NA, s_ + 1)                                                                               \
      C3X_PREAD_B(bx, ((t) + 1) % 9, kc + ((t) == 8), 0)                                                    \
      asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");                                                    \
      C3X_PMMA(FA, by, 3)                                                                                   \
    }                                                                                                       \
    if ((t) >= HTAP && (t) <= HTAP + 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                    \
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");                                                   \
    asm volatile("s_barrier" ::: "memory");                                                                 \
  }
#define C3X_PKC(LIVE)                                                                                       \
  C3X_PSTEP(0, a0, a1, LIVE) C3X_PSTEP(1, a1, a0, LIVE) C3X_PSTEP(2, a0, a1, LIVE)                          \
  C3X_PSTEP(3, a1, a0, LIVE) C3X_PSTEP(4, a0, a1, LIVE) C3X_PSTEP(5, a1, a0, LIVE)                          \
  C3X_PSTEP(6, a0, a1, LIVE) C3X_PSTEP(7, a1, a0, LIVE) C3X_PSTEP(8, a0, a1, LIVE)
  if constexpr (PIPE) {
    bf16x8 a0[4], a1[4], bx[2], by[2];
    if (live) {
      C3X_PREAD_A(a0, 0)
      C3X_PREAD_B(bx, 0, 0, 0)
      for (int kc = 0; kc < NKC; ++kc) {   // 9 steps (odd): the next chunk's weight fragments move back to a0
        C3X_PKC(true)
#pragma unroll
        for (int i = 0; i < 4; ++i) a0[i] = a1[i];
      }
    } else {
      for (int kc = 0; kc < NKC; ++kc) { C3X_PKC(false) }
    }
  } else if (live) {
#define C3X_KC(LIVE, LAST)                                                                                    \
  C3X_STEP(0, LIVE, LAST) C3X_STEP(1, LIVE, LAST) C3X_STEP(2, LIVE, LAST) C3X_STEP(3, LIVE, LAST)             \
  C3X_STEP(4, LIVE, LAST) C3X_STEP(5, LIVE, LAST) C3X_STEP(6, LIVE, LAST) C3X_STEP(7, LIVE, LAST)             \
  C3X_STEP(8, LIVE, LAST)
    for (int kc = 0; kc < NKC - 1; ++kc) { C3X_KC(true, false) }
    {
      const int kc = NKC - 1;
      C3X_KC(true, true)
    }
  } else {   // DMA issue and barriers only
    for (int kc = 0; kc < NKC - 1; ++kc) { C3X_KC(false, false) }
    {
      const int kc = NKC - 1;
      C3X_KC(false, true)
    }
  }
#undef C3X_STEP
#undef C3X_KC
#undef C3X_VMWAIT
#undef C3X_PKC
#undef C3X_PSTEP
#undef C3X_PMMA
#undef C3X_PREAD_A
#undef C3X_PREAD_B
  if (!PIPE && !grp) asm volatile("s_barrier" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue: lane holds co = n0 + wc*64 + i*16 + 4q + r of pixel (wp*4 + (j >> 1), (j & 1)*16 + a15)
  if (!g.accum && !(DBG & 32)) {
    // Staged through LDS (the pipeline buffers are drained): the bf16 tile [512 px][128 co] (256-byte
    // rows, 16-byte granule g of pixel p at slot g ^ (p & 15): the 16 pixels of one ds_write_b64 lane
    // group hit 16 slots), then written back as whole 256-byte pixel rows, 16 bytes per lane — a tile
    // row of 32 pixels is 8 KB contiguous. Direct 8-byte stores from the accumulator layout touched 16
    // rows per instruction (store-issue bound: 128 KB per block). BatchNorm sums from the same bf16
    // values: per thread 8 channels over its 16 pixels, then lane groups, then waves in fixed order.
    // fused BatchNorm-backward sums: the 16 pre-activation loads of this thread's store column are issued
    // before the accumulator tile is staged, so their latency lies under the staging and its barrier
    uint4 zpre[CT];
    if (g.bnz != nullptr) {
      const int zc_ = tid & 15, zx_ = min(tx0 + (tid >> 4), g.W - 1);
#pragma unroll
      for (int k = 0; k < CT; ++k)
        zpre[k] = *(const uint4*)(g.bnz + ((size_t)(b * g.H + min(ty0 + k, g.H - 1)) * g.W + zx_) * g.COUT + n0 +
                                  zc_ * 8);
    }
    unsigned char* tileb = lds;
    if (live) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = (wp * 4 + (j >> 1)) * XTW + (j & 1) * 16 + a15;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int gr = (wc * 8 + i * 2 + (q >> 1)) ^ (p & 15);
          const unsigned lo = (unsigned)f2bf(acc[i][j][0]) | ((unsigned)f2bf(acc[i][j][1]) << 16);
          const unsigned hi = (unsigned)f2bf(acc[i][j][2]) | ((unsigned)f2bf(acc[i][j][3]) << 16);
          *(uint2*)(tileb + p * 256 + gr * 16 + (q & 1) * 8) = make_uint2(lo, hi);
        }
      }
    }
    __syncthreads();
    const int c = tid & 15, px = tid >> 4;   // 16-byte chunk (8 channels) c of column px of every tile row
    float t1[8], t2[8], bsc[8], bbe[8], bmu[8], bis[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t1[e] = t2[e] = 0.f;
    if (g.bnz != nullptr) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = n0 + c * 8 + e;
        bsc[e] = g.bnp[ch];
        bbe[e] = g.bnp[g.COUT + ch];
        bmu[e] = g.bnp[2 * g.COUT + ch];
        bis[e] = g.bnp[3 * g.COUT + ch];
      }
    }
    const int x = tx0 + px;
    if (g.bnz != nullptr) {
      // BatchNorm-backward sums of the layer this gradient enters: all 16 pre-activation loads issued
      // before the first is used (clamped addresses; a load per pixel waited out one round trip each)
#pragma unroll
      for (int k = 0; k < CT; ++k) {
        const int y = ty0 + k, p = k * XTW + px;
        if (y >= g.H || x >= g.W) continue;
        const size_t pix = (size_t)(b * g.H + y) * g.W + x;
        const uint4 v = *(const uint4*)(tileb + p * 256 + ((c ^ (p & 15)) * 16));
  *(uint4*)(g.out + pix * g.OP + g.OOFF + n0 + c * 8) = v;
        const unsigned u[4] = {v.x, v.y, v.z, v.w};
        const unsigned zu[4] = {zpre[k].x, zpre[k].y, zpre[k].z, zpre[k].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float zz = bf2f((u16)(zu[e >> 1] >> (16 * (e & 1)))), d0 = bf2f((u16)(u[e >> 1] >> (16 * (e & 1))));
          const float pre = fmaf(zz - bmu[e], bsc[e], bbe[e]);
          const float d = pre > 0.f ? d0 : 0.f;
          t1[e] += d;
          t2[e] += d * ((zz - bmu[e]) * bis[e]);
        }
      }
    }
#pragma unroll 4
    for (int k = 0; k < (g.bnz != nullptr ? 0 : CT); ++k) {
      const int y = ty0 + k, p = k * XTW + px;
      if (y >= g.H || x >= g.W) continue;
      const size_t pix = (size_t)(b * g.H + y) * g.W + x;
      const uint4 v = *(const uint4*)(tileb + p * 256 + ((c ^ (p & 15)) * 16));
      *(uint4*)(g.out + pix * g.OP + g.OOFF + n0 + c * 8) = v;
      const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float f0 = bf2f((u16)(u[e] & 0xffff)), f1 = bf2f((u16)(u[e] >> 16));
        t1[2 * e] += f0;
        t2[2 * e] += f0 * f0;
        t1[2 * e + 1] += f1;
        t2[2 * e + 1] += f1 * f1;
      }
    }
    if (g.part == nullptr) return;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      t1[e] += __shfl_xor(t1[e], 16, 64);
      t2[e] += __shfl_xor(t2[e], 16, 64);
      t1[e] += __shfl_xor(t1[e], 32, 64);
      t2[e] += __shfl_xor(t2[e], 32, 64);
    }
    float* sR = (float*)(lds + 128 * 1024);   // [8 waves][2][128 channels]
    if (lane < 16) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sR[(w * 2 + 0) * 128 + c * 8 + e] = t1[e];
        sR[(w * 2 + 1) * 128 + c * 8 + e] = t2[e];
      }
    }
    __syncthreads();
    if (tid < 256) {
      const int k2 = tid >> 7, ch = tid & 127;
      float s = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) s += sR[(ww * 2 + k2) * 128 + ch];
      g.part[(size_t)tile * 2 * g.COUT + k2 * g.COUT + n0 + ch] = s;
    }
    return;
  }
  float s1[4][4], s2[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int y = ty0 + wp * 4 + (j >> 1), x = tx0 + (j & 1) * 16 + a15;
    if (y >= g.H || x >= g.W) continue;
    const size_t orow = (size_t)(b * g.H + y) * g.W + x;
    u16* op = g.out + orow * g.OP + g.OOFF + n0 + wc * 64 + 4 * q;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
      uint2* p2 = (uint2*)(op + i * 16);
      if (g.accum) {
        uint2 e = *p2;
        v[0] += bf2f((u16)(e.x & 0xffff));
        v[1] += bf2f((u16)(e.x >> 16));
        v[2] += bf2f((u16)(e.y & 0xffff));
        v[3] += bf2f((u16)(e.y >> 16));
      }
      u16 hb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        hb[r] = f2bf(v[r]);
        const float qv = bf2f(hb[r]);
        s1[i][r] += qv;
        s2[i][r] += qv * qv;
      }
      *p2 = make_uint2((unsigned)hb[0] | ((unsigned)hb[1] << 16), (unsigned)hb[2] | ((unsigned)hb[3] << 16));
    }
  }
  if (g.part == nullptr) return;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[i][r] += __shfl_xor(s1[i][r], o, 64);
        s2[i][r] += __shfl_xor(s2[i][r], o, 64);
      }
    }
  float* sP = (float*)lds;   // [4 wp][2][128]
  if (a15 == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = wc * 64 + i * 16 + 4 * q + r;
        sP[(wp * 2 + 0) * 128 + c] = s1[i][r];
        sP[(wp * 2 + 1) * 128 + c] = s2[i][r];
      }
  }
  __syncthreads();
  float* prow = g.part + (size_t)tile * 2 * g.COUT;
  if (tid < 128) {
    prow[n0 + tid] = ((sP[0 * 128 + tid] + sP[2 * 128 + tid]) + sP[4 * 128 + tid]) + sP[6 * 128 + tid];
  } else if (tid < 256) {
    const int c = tid - 128;
    prow[g.COUT + n0 + c] = ((sP[1 * 128 + c] + sP[3 * 128 + c]) + sP[5 * 128 + c]) + sP[7 * 128 + c];
  }
}

// ------------------------------------------------------------------ 3x3 stride-1 conv, two 4-wave blocks per CU
// k_conv3x3y: k_conv3x3x's per-wave work (128 accumulator VGPRs, 12 operand fragments per 32 MFMAs,
// 32-channel K-steps, 64-byte swizzled rows, buffer-load DMA, LDS-staged epilogue) in a 4-wave block
// of 16x16 pixels x 128 output channels (wave w: tile rows 4w..4w+3 = 64 pixels x 128 channels),
// 78 KB of LDS, so TWO blocks share a CU. k_conv3x3x's 8-wave blocks fill whole rounds of the CUs
// at once: every block stages its halo, computes, and stores its 128 KB output at the same time
// (measured: prologue + epilogue 17 us of a 71 us 200x176 launch, not overlapped). Two independent
// blocks per CU overlap one block's prologue / epilogue with the other's MFMAs, and the grid of
// 16x16 tiles (858 at 200x176) is drained by whichever slot frees first. One barrier per step
// (the other block on the SIMD plays the partner wave); halo: 18 rows of 20 pixels (row pitch
// 20 = 0 mod 4, so a pixel's bank is a function of its column), double-buffered 23 KB chunks; weights: 4-slot
// ring of 128 x 32 tiles two steps ahead.
constexpr int YB = 256;                        // threads
constexpr int YHP = 20;                        // halo LDS row pitch in pixels
constexpr int YHR = HT * YHP;                  // halo LDS rows (360)
constexpr int YHBUF = 23 * 1024;               // halo buffer: 360 rows (22.5 KB) rounded to whole DMA KBs
constexpr int YHI = 6;                         // halo DMA instructions per wave (23 over 4 waves)
constexpr int YLDS = 2 * YHBUF + WRING * XWTILE;   // 79872 B

// the DMA waits of k_conv3x3y's steps: retire all but the youngest weight tile (WI instructions per wave), or at
// taps HTAP, HTAP + 1 all but that tile and the next chunk's halo (YHI = 6 instructions)
template <int WI>
__device__ __forceinline__ void c3y_vm_tile() {
  if constexpr (WI == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
}
template <int WI>
__device__ __forceinline__ void c3y_vm_halo() {
  if constexpr (WI == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
}

// CH = 64 (the split tail, C3::ysplit): the same block over half the output channels of its tile — 16 MFMAs per
// step on a 64 x 32 weight tile (one DMA instruction per wave), the epilogue's stores / sums on its 64 channels
// ZPF (data gradients with fused BatchNorm-backward sums): the epilogue's first ZPN pre-activation rows are loaded during
// the last K-chunk — issued after its last real weight tile (step 5); the later steps issue no weight DMAs (in every
// launch: they were clamped repeats), so the loads stay in flight through steps 6-8 and the accumulator staging
template <int DBG, int CH, bool ZPF = false>
__device__ __forceinline__ void conv3x3y_body(const C3& g, unsigned char* lds, const int tile, const int n0) {
  static_assert(CH == 128 || CH == 64, "k_conv3x3y: 128 or 64 output channels per block");
  constexpr int NI = CH / 16, WI = CH / 64;   // accumulator fragments per wave; weight DMAs per wave and step
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = tile / (g.TY * g.TX), trem = tile - b * g.TY * g.TX;
  const int ty0 = (trem / g.TX) * CT, tx0 = (trem % g.TX) * CT;
  const int NKC = g.CIN / XBK, NS = 9 * NKC;
  unsigned char* const hbuf = lds;
  unsigned char* const wring = lds + 2 * YHBUF;

  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)g.src, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rwt = __builtin_amdgcn_make_buffer_rsrc((void*)g.wt, (short)0, 0x7fffffff, 0x00020000);
  // halo: instruction k writes LDS granules k*64 + lane (row r = hy*20 + hx, slot j = granule j ^ xswz(hx));
  // pad columns 18, 19 and rows past 360 read zeros (offset past the range)
  unsigned hofs[YHI];
#pragma unroll
  for (int m = 0; m < YHI; ++m) {
    const int k = min(w + 4 * m, 22);
    const int P = k * 64 + lane, r = P >> 2, j = P & 3;
    const int hy = r / YHP, hx = r - hy * YHP;
    const int y = ty0 + hy - 1, x = tx0 + hx - 1;
    hofs[m] = (r < YHR && hx < HT && y >= 0 && y < g.H && x >= 0 && x < g.W)
                  ? (unsigned)((((b * g.H + y) * g.W + x) * g.SP + (j ^ xswz(hx)) * 8) * 2)
                  : 0x80000000u;
  }
  // weights: instructions 2w, 2w + 1 write rows (2w + m)*16 + (lane >> 2) = output channel n0 + r
  unsigned wofs[WI];
#pragma unroll
  for (int m = 0; m < WI; ++m) {
    const int r = (WI * w + m) * 16 + (lane >> 2), j = lane & 3;
    wofs[m] = (unsigned)(((n0 + r) * g.CIN + (j ^ xswz(r)) * 8) * 2);
  }
  auto issue_halo = [&](int kc, int hb) {
#pragma unroll
    for (int m = 0; m < YHI; ++m)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsrc, (__attribute__((address_space(3))) void*)(hbuf + hb * YHBUF + min(w + 4 * m, 22) * 1024), 16,
          hofs[m], kc * XBK * 2, 0, 0);
  };
  const int wtap = g.COUT * g.CIN * 2;
  auto issue_w = [&](int s) {
    s = min(s, NS - 1);
    const int kc = s / 9, t = s - kc * 9;
#pragma unroll
    for (int m = 0; m < WI; ++m)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rwt, (__attribute__((address_space(3))) void*)(wring + (s & (WRING - 1)) * XWTILE + (WI * w + m) * 1024), 16,
          wofs[m], t * wtap + kc * XBK * 2, 0, 0);
  };

  // operands: A (weights) rows i*16 + a15 (i = 0..7); B (halo) pixel (4w + j + dy, a15 + dx)
  const int a15 = lane & 15, q = lane >> 4;
  const int woff = a15 * XROW + ((q ^ xswz(a15)) * 16);
  int hoff[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) hoff[dx] = (w * 4 * YHP + dx + a15) * XROW + ((q ^ xswz(dx + a15)) * 16);

  f32x4 acc[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // operand fragments read a quarter step ahead (C3Y_PSTEP); DBG bit 128 (and the timing arms 1 / 16):
  // the former loop, which reads a step's 12 fragments, waits for all of them, then runs its 32 MFMAs
  // (200x176 128->128 72.6 -> 66.9 us, 128->256 113.9 -> 109.8 us, profiles/r03_conv_pipe.log)
  // ZPF: the epilogue's first ZPN pre-activation rows of this thread's 16-byte column chunk (see C3Y_PKCZ)
  constexpr int ZPN = 4, ZQ = ZPF ? ZPN : 0;   // ZQ: the prefetch loads outstanding after the last weight tile
  uint4 zpa[ZPF ? ZPN : 1];
  const int zpx_ = min(tx0 + (tid >> 4), g.W - 1), zpch_ = min(n0 + (tid & 15) * 8, g.COUT - 8);
#define C3Y_ZISSUE                                                                                          \
  {                                                                                                         \
    _Pragma("unroll") for (int k_ = 0; k_ < ZPN; ++k_) zpa[k_] =                                            \
        *(const uint4*)(g.bnz + ((size_t)(b * g.H + min(ty0 + k_, g.H - 1)) * g.W + zpx_) * g.COUT + zpch_); \
  }
  constexpr bool PIPE = (DBG & (128 | 16 | 1)) == 0;
  issue_halo(0, 0);
#pragma unroll
  for (int s = 0; s < WDIST; ++s) issue_w(s);
  if constexpr (PIPE) issue_w(WDIST);
  const bool live = ty0 + w * 4 < g.H;
  // halo 0 + tile 0 (+ tile 1 when pipelined: the youngest tile stays in flight)
  c3y_vm_tile<WI>();
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  // per step: issue the DMAs two steps ahead, read this step's 12 fragments, 32 MFMAs, retire the next
  // step's tile (vmcnt(2); vmcnt(8) at taps HTAP, HTAP + 1 whose younger DMAs include the halo), barrier
#define C3Y_STEP(t, LIVE)                                                                                     \
  {                                                                                                           \
    const int s_ = kc * 9 + (t);                                                                              \
    issue_w(s_ + WDIST);                                                                                      \
    if ((t) == HTAP) issue_halo(min(kc + 1, NKC - 1), (kc + 1) & 1);                                          \
    if (LIVE && !(DBG & 1)) {                                                                                 \
      const unsigned char* hb_ = hbuf + (kc & 1) * YHBUF;                                                     \
      const unsigned char* wt_ = wring + (s_ & (WRING - 1)) * XWTILE;                                         \
      constexpr int dy_ = (t) / 3, dx_ = (t) % 3;                                                             \
      bf16x8 av[NI], bv[4];                                                                                    \
      _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                           \
        bv[j] = *(const bf16x8*)(hb_ + hoff[dx_] + (j + dy_) * YHP * XROW);                                   \
      _Pragma("unroll") for (int i = 0; i < NI; ++i)                                                          \
        av[i] = *(const bf16x8*)(wt_ + woff + i * 16 * XROW);                                                 \
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                      \
      __builtin_amdgcn_s_setprio(1);                                                                          \
      _Pragma("unroll") for (int i = 0; i < NI; ++i)                                                          \
        _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                         \
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);              \
      __builtin_amdgcn_s_setprio(0);                                                                          \
    }                                                                                                         \
    if ((t) == HTAP || (t) == HTAP + 1) c3y_vm_halo<WI>();                                                        \
    else c3y_vm_tile<WI>();                                                                                       \
    asm volatile("s_barrier" ::: "memory");                                                                   \
  }
  // pipelined form: the 32 MFMAs of a step run as four quarters of 2 weight fragments x 4 halo
  // fragments; before the MFMAs of quarter q the wave issues the reads of quarter q + 1 (2 weight
  // fragments), and before those of quarter 3 the reads of the next step's quarter 0 and its 4 halo
  // fragments (that tile was published by the previous step's barrier), so every LDS read lies under the
  // same wave's MFMAs and the fragment registers stay at k_conv3x3y's 48 (two 2-fragment weight buffers,
  // two 4-fragment halo buffers). Step s issues tile s + 3 and retires tile s + 2 before its barrier.
  // The slot that tile s + 3 overwrites, (s - 1) & 3, was last read during step s - 1; the halo buffer of
  // chunk kc + 1 (issued at tap HTAP of chunk kc) was last read during step (kc - 1, 7) and is retired by
  // the wait of step (kc, 7), before step (kc, 8) reads chunk kc + 1's first fragments. At the last step
  // the reads for "step NS" hit valid LDS (clamped tile / halo) and are never used.
#define C3Y_PREAD_B(FB, tn, kn)                                                                             \
  {                                                                                                         \
    const unsigned char* hb_ = hbuf + ((kn) & 1) * YHBUF;                                                   \
    const int dy_ = (tn) / 3, dx_ = (tn) % 3;                                                               \
    _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                           \
      FB[j] = *(const bf16x8*)(hb_ + hoff[dx_] + (j + dy_) * YHP * XROW);                                   \
  }
#define C3Y_PREAD_A(FA, sn, qq)                                                                             \
  {                                                                                                         \
    const unsigned char* wt_ = wring + ((sn) & (WRING - 1)) * XWTILE + (qq) * 2 * 16 * XROW;                \
    FA[0] = *(const bf16x8*)(wt_ + woff);                                                                   \
    FA[1] = *(const bf16x8*)(wt_ + woff + 16 * XROW);                                                       \
  }
#define C3Y_PMMA(FA, FB, qq)                                                                                \
  __builtin_amdgcn_s_setprio(1);                                                                            \
  _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_)                                                          \
    _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                           \
      acc[((qq) * 2 + i_) % NI][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(FA[i_], FB[j], acc[((qq) * 2 + i_) % NI][j], 0, 0, 0); \
  __builtin_amdgcn_s_setprio(0);
#define C3Y_PSTEP(i, FB, NB, LIVE, MODE)                                                                    \
  {                                                                                                         \
    constexpr int t_ = (i) % 9;                                                                             \
    const int kq_ = kc + (i) / 9, s_ = kq_ * 9 + t_;                                                        \
    if constexpr ((MODE) != 2) issue_w(s_ + WDIST + 1);                                                     \
    if (t_ == HTAP) issue_halo(min(kq_ + 1, NKC - 1), (kq_ + 1) & 1);                                       \
    if constexpr ((MODE) == 1) C3Y_ZISSUE                                                                   \
    if (LIVE && CH == 64) {                                                                                 \
      C3Y_PREAD_A(ay, s_, 1)                                                                                \
      asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");                                                    \
      C3Y_PMMA(ax, FB, 0)                                                                                   \
      C3Y_PREAD_A(ax, s_ + 1, 0)                                                                            \
      C3Y_PREAD_B(NB, (t_ + 1) % 9, kq_ + (t_ == 8))                                                        \
      asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");                                                    \
      C3Y_PMMA(ay, FB, 1)                                                                                   \
    } else if (LIVE) {                                                                                      \
      C3Y_PREAD_A(ay, s_, 1)                                                                                \
      asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");                                                    \
      C3Y_PMMA(ax, FB, 0)                                                                                   \
      C3Y_PREAD_A(ax, s_, 2)                                                                                \
      asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");                                                    \
      C3Y_PMMA(ay, FB, 1)                                                                                   \
      C3Y_PREAD_A(ay, s_, 3)                                                                                \
      asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");                                                    \
      C3Y_PMMA(ax, FB, 2)                                                                                   \
      C3Y_PREAD_A(ax, s_ + 1, 0)                                                                            \
      C3Y_PREAD_B(NB, (t_ + 1) % 9, kq_ + (t_ == 8))                                                        \
      asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");                                                    \
      C3Y_PMMA(ay, FB, 3)                                                                                   \
    }                                                                                                       \
    if constexpr ((MODE) == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(WI + ZPN) : "memory");           \
    else if constexpr ((MODE) == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ZQ) : "memory");             \
    else if (t_ == HTAP || t_ == HTAP + 1) c3y_vm_halo<WI>();                                              \
    else c3y_vm_tile<WI>();                                                                                 \
    asm volatile("s_barrier" ::: "memory");                                                                 \
  }
#define C3Y_PKC(LIVE)                                                                                       \
  C3Y_PSTEP(0, fb0, fb1, LIVE, 0) C3Y_PSTEP(1, fb1, fb0, LIVE, 0) C3Y_PSTEP(2, fb0, fb1, LIVE, 0)           \
  C3Y_PSTEP(3, fb1, fb0, LIVE, 0) C3Y_PSTEP(4, fb0, fb1, LIVE, 0) C3Y_PSTEP(5, fb1, fb0, LIVE, 0)           \
  C3Y_PSTEP(6, fb0, fb1, LIVE, 0) C3Y_PSTEP(7, fb1, fb0, LIVE, 0) C3Y_PSTEP(8, fb0, fb1, LIVE, 0)
// the last K-chunk: steps 6-8 issue no weight DMA (they were repeats of the last tile, clamped) and wait for
// vmcnt ZQ; ZPF: step 5 issues the last real weight tile and then the ZPN pre-activation loads (vmcnt WI + ZPN
// retires only the older tile), which stay in flight through steps 6-8 and the staging
#define C3Y_PKCZ(LIVE)                                                                                      \
  C3Y_PSTEP(0, fb0, fb1, LIVE, 0) C3Y_PSTEP(1, fb1, fb0, LIVE, 0) C3Y_PSTEP(2, fb0, fb1, LIVE, 0)           \
  C3Y_PSTEP(3, fb1, fb0, LIVE, 0) C3Y_PSTEP(4, fb0, fb1, LIVE, 0) C3Y_PSTEP(5, fb1, fb0, LIVE, ZPF ? 1 : 0)  \
  C3Y_PSTEP(6, fb0, fb1, LIVE, 2) C3Y_PSTEP(7, fb1, fb0, LIVE, 2) C3Y_PSTEP(8, fb0, fb1, LIVE, 2)
  if constexpr (PIPE) {
    bf16x8 ax[2], ay[2], fb0[4], fb1[4];
    if (live) {
      C3Y_PREAD_A(ax, 0, 0)
      C3Y_PREAD_B(fb0, 0, 0)
      for (int kc = 0; kc < NKC - 1; ++kc) {   // 9 steps (odd): the next chunk's halo fragments move back to fb0
        C3Y_PKC(true)
#pragma unroll
        for (int j = 0; j < 4; ++j) fb0[j] = fb1[j];
      }
      {
        const int kc = NKC - 1;
        C3Y_PKCZ(true)
      }
    } else {
      for (int kc = 0; kc < NKC - 1; ++kc) { C3Y_PKC(false) }
      {
        const int kc = NKC - 1;
        C3Y_PKCZ(false)
      }
    }
  } else if (DBG & 16) {
  } else if (live) {
    for (int kc = 0; kc < NKC; ++kc) {
      C3Y_STEP(0, true)
      C3Y_STEP(1, true)
      C3Y_STEP(2, true)
      C3Y_STEP(3, true)
      C3Y_STEP(4, true)
      C3Y_STEP(5, true)
      C3Y_STEP(6, true)
      C3Y_STEP(7, true)
      C3Y_STEP(8, true)
    }
  } else {
    for (int kc = 0; kc < NKC; ++kc) {
      C3Y_STEP(0, false)
      C3Y_STEP(1, false)
      C3Y_STEP(2, false)
      C3Y_STEP(3, false)
      C3Y_STEP(4, false)
      C3Y_STEP(5, false)
      C3Y_STEP(6, false)
      C3Y_STEP(7, false)
      C3Y_STEP(8, false)
    }
  }
#undef C3Y_STEP
#undef C3Y_PKC
#undef C3Y_PKCZ
#undef C3Y_ZISSUE
#undef C3Y_PSTEP
#undef C3Y_PMMA
#undef C3Y_PREAD_A
#undef C3Y_PREAD_B
  if constexpr (PIPE)   // every weight / halo DMA retired by the last steps' waits; ZPF: the pre-activation loads stay
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(ZQ) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- epilogue: lane holds co = n0 + i*16 + 4q + r of pixel (4w + j, a15)
  if (!g.accum) {
    // bf16 tile [256 px][128 co] in LDS (granule g of pixel p at slot g ^ (p & 15)), written back as
    // whole 256-byte pixel rows; BatchNorm sums from the same bf16 values (as k_conv3x3x)
    // fused BatchNorm-backward sums: the 16 pre-activation loads of this thread's store column are issued
    // before the accumulator tile is staged, so their latency lies under the staging and its barrier
    uint4 zpre[CT];
    const bool cact = CH == 128 || (tid & 15) < CH / 8;   // this thread's 16-byte chunk is one of the block's
    if (g.bnz != nullptr && cact) {
      const int zc_ = tid & 15, zx_ = min(tx0 + (tid >> 4), g.W - 1);
#pragma unroll
      for (int k = 0; k < CT; ++k) {
        if (ZPF && PIPE && k < ZPN) zpre[k] = zpa[k % (ZPF ? ZPN : 1)];
        else
          zpre[k] = *(const uint4*)(g.bnz + ((size_t)(b * g.H + min(ty0 + k, g.H - 1)) * g.W + zx_) * g.COUT + n0 +
                                    zc_ * 8);
      }
    }
    unsigned char* tileb = lds;
    if (live) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = (w * 4 + j) * CT + a15;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          const int gr = (i * 2 + (q >> 1)) ^ (p & 15);
          const unsigned lo = (unsigned)f2bf(acc[i][j][0]) | ((unsigned)f2bf(acc[i][j][1]) << 16);
          const unsigned hi = (unsigned)f2bf(acc[i][j][2]) | ((unsigned)f2bf(acc[i][j][3]) << 16);
          *(uint2*)(tileb + p * 256 + gr * 16 + (q & 1) * 8) = make_uint2(lo, hi);
        }
      }
    }
    __syncthreads();
    const int c = tid & 15, px = tid >> 4;   // 16-byte chunk c of column px of every tile row
    float t1[8], t2[8], bsc[8], bbe[8], bmu[8], bis[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t1[e] = t2[e] = 0.f;
    if (g.bnz != nullptr && cact) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = n0 + c * 8 + e;
        bsc[e] = g.bnp[ch];
        bbe[e] = g.bnp[g.COUT + ch];
        bmu[e] = g.bnp[2 * g.COUT + ch];
        bis[e] = g.bnp[3 * g.COUT + ch];
      }
    }
    const int x = tx0 + px;
    if (g.bnz != nullptr && cact) {
      // BatchNorm-backward sums of the layer this gradient enters: all 16 pre-activation loads issued
      // before the first is used (clamped addresses; a load per pixel waited out one round trip each)
#pragma unroll
      for (int k = 0; k < CT; ++k) {
        const int y = ty0 + k, p = k * CT + px;
        if (y >= g.H || x >= g.W) continue;
        const size_t pix = (size_t)(b * g.H + y) * g.W + x;
        const uint4 v = *(const uint4*)(tileb + p * 256 + ((c ^ (p & 15)) * 16));
  if (!(DBG & 64)) *(uint4*)(g.out + pix * g.OP + g.OOFF + n0 + c * 8) = v;
        const unsigned u[4] = {v.x, v.y, v.z, v.w};
        const unsigned zu[4] = {zpre[k].x, zpre[k].y, zpre[k].z, zpre[k].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float zz = bf2f((u16)(zu[e >> 1] >> (16 * (e & 1)))), d0 = bf2f((u16)(u[e >> 1] >> (16 * (e & 1))));
          const float pre = fmaf(zz - bmu[e], bsc[e], bbe[e]);
          const float d = pre > 0.f ? d0 : 0.f;
          t1[e] += d;
          t2[e] += d * ((zz - bmu[e]) * bis[e]);
        }
      }
    }
#pragma unroll 4
    for (int k = 0; k < (g.bnz != nullptr || !cact ? 0 : CT); ++k) {
      const int y = ty0 + k, p = k * CT + px;
      if (y >= g.H || x >= g.W) continue;
      const size_t pix = (size_t)(b * g.H + y) * g.W + x;
      const uint4 v = *(const uint4*)(tileb + p * 256 + ((c ^ (p & 15)) * 16));
      if (!(DBG & 64)) *(uint4*)(g.out + pix * g.OP + g.OOFF + n0 + c * 8) = v;
      const unsigned u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float f0 = bf2f((u16)(u[e] & 0xffff)), f1 = bf2f((u16)(u[e] >> 16));
        t1[2 * e] += f0;
        t2[2 * e] += f0 * f0;
        t1[2 * e + 1] += f1;
        t2[2 * e + 1] += f1 * f1;
      }
    }
    if (g.part == nullptr) return;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      t1[e] += __shfl_xor(t1[e], 16, 64);
      t2[e] += __shfl_xor(t2[e], 16, 64);
      t1[e] += __shfl_xor(t1[e], 32, 64);
      t2[e] += __shfl_xor(t2[e], 32, 64);
    }
    float* sR = (float*)(lds + 64 * 1024);   // [4 waves][2][128 channels]
    if (lane < 16) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sR[(w * 2 + 0) * 128 + c * 8 + e] = t1[e];
        sR[(w * 2 + 1) * 128 + c * 8 + e] = t2[e];
      }
    }
    __syncthreads();
    {
      const int k2 = tid >> 7, ch = tid & 127;
      const float s = ((sR[(0 * 2 + k2) * 128 + ch] + sR[(1 * 2 + k2) * 128 + ch]) + sR[(2 * 2 + k2) * 128 + ch]) +
                      sR[(3 * 2 + k2) * 128 + ch];
      if (ch < CH) g.part[(size_t)tile * 2 * g.COUT + k2 * g.COUT + n0 + ch] = s;
    }
    return;
  }
  // accumulate into the existing image: fp32 sum, one rounding (register-direct stores), in two halves
  // of 64 channels (BatchNorm sums of half the accumulator tiles live at a time)
  float* sP = (float*)lds;   // [4 waves][2][128]
#pragma unroll
  for (int ih = 0; ih < CH / 64; ++ih) {
    float s1[4][4], s2[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int y = ty0 + w * 4 + j, x = tx0 + a15;
      if (y >= g.H || x >= g.W) continue;
      u16* op = g.out + ((size_t)(b * g.H + y) * g.W + x) * g.OP + g.OOFF + n0 + ih * 64 + 4 * q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x4 a = acc[ih * 4 + i][j];
        float v[4] = {a[0], a[1], a[2], a[3]};
        uint2* p2 = (uint2*)(op + i * 16);
        uint2 e = *p2;
        v[0] += bf2f((u16)(e.x & 0xffff));
        v[1] += bf2f((u16)(e.x >> 16));
        v[2] += bf2f((u16)(e.y & 0xffff));
        v[3] += bf2f((u16)(e.y >> 16));
        u16 hb[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          hb[r] = f2bf(v[r]);
          const float qv = bf2f(hb[r]);
          s1[i][r] += qv;
          s2[i][r] += qv * qv;
        }
        *p2 = make_uint2((unsigned)hb[0] | ((unsigned)hb[1] << 16), (unsigned)hb[2] | ((unsigned)hb[3] << 16));
      }
    }
    if (g.part == nullptr) continue;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[i][r] += __shfl_xor(s1[i][r], o, 64);
          s2[i][r] += __shfl_xor(s2[i][r], o, 64);
        }
      }
    if (a15 == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cc = ih * 64 + i * 16 + 4 * q + r;
          sP[(w * 2 + 0) * 128 + cc] = s1[i][r];
          sP[(w * 2 + 1) * 128 + cc] = s2[i][r];
        }
    }
  }
  if (g.part == nullptr) return;
  __syncthreads();
  {
    const int k2 = tid >> 7, ch = tid & 127;
    const float s = ((sP[(0 * 2 + k2) * 128 + ch] + sP[(1 * 2 + k2) * 128 + ch]) + sP[(2 * 2 + k2) * 128 + ch]) +
                    sP[(3 * 2 + k2) * 128 + ch];
    if (ch < CH) g.part[(size_t)tile * 2 * g.COUT + k2 * g.COUT + n0 + ch] = s;
  }
}


// the grid: the first nitems - ysplit items (tile-major, a tile's co-blocks adjacent, XCD-aware) one 128-channel
// block each, then the last ysplit items as two 64-channel blocks each (dispatched last: the tail of the launch)
template <int DBG = 0, bool ZPF = false>
__global__ __launch_bounds__(YB, 2) void k_conv3x3y(C3 g) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[YLDS];   // ONE LDS object (see k_conv3x3x)
  const int ncob = g.COUT >> 7;
  const int nfull = g.B * g.TY * g.TX * ncob - g.ysplit;
  if ((int)blockIdx.x < nfull) {
    const int item = xcd_remap(blockIdx.x, nfull);
    const int tile = item / ncob;
    conv3x3y_body<DBG, 128, ZPF>(g, lds, tile, (item - tile * ncob) * 128);
  } else if constexpr (DBG == 0) {
    const int t = (int)blockIdx.x - nfull, item = nfull + (t >> 1);
    const int tile = item / ncob;
    conv3x3y_body<0, 64, ZPF>(g, lds, tile, (item - tile * ncob) * 128 + (t & 1) * 64);
  }
}

// ------------------------------------------------------------------ weight gradient
__device__ __forceinline__ s16x4 tr_read(const u16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

struct WG {
  const u16* x;   // forward input image rows [S pixels][XP]
  int XP;
  const u16* dz;  // output-side gradient rows [O pixels][DP] at channel offset 0
  int DP;
  int CI, CO;     // multiples of 128
  Img R, S, O;
  int M, rows_per;
  float* part;    // [chunks][T][CI][CO]
};

// 1-D grid of chunks * T * (CI/TC)*(CO/TC) blocks, XCD-aware: each XCD walks whole chunks with
// the taps and channel tiles of one chunk adjacent, so a chunk's x / dz rows are fetched into that
// XCD's L2 once and re-read by its T * tiles blocks. 4 waves as 2 (ci) x 2 (co).
// NARROW = 1: 64 x 64 (ci, co) tiles (waves 32 x 32) for the 64-channel CenterHead layers.
template <int MAP, int NARROW = 0>
__global__ __launch_bounds__(BLK, 2) void k_wgrad(WG g) {
  constexpr int T = wtaps_of<MAP>();
  constexpr int TC = NARROW ? 64 : 128;   // block tile edge (ci and co)
  constexpr int WT = TC / 2;              // wave tile edge
  constexpr int NW = WT / 16;             // 16 x 16 MFMA tiles per wave edge
  constexpr int SEGS = TC / 8;            // 16-B segments per row
  constexpr int NLD = 64 * SEGS / BLK;    // 16-B loads per thread per operand and sub-tile
  constexpr int RT = 64, P = TC + 16;     // rows per sub-tile, LDS pitch (conflict-free tr reads)
  __shared__ __attribute__((aligned(16))) u16 sX[RT * P];
  __shared__ __attribute__((aligned(16))) u16 sD[RT * P];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wci = w >> 1, wco = w & 1;
  const int nco = g.CO / TC, ntile = (g.CI / TC) * nco;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = lid / (T * ntile), rest = lid - chunk * (T * ntile);
  const int t = rest / ntile, tile = rest - t * ntile;
  const int ci0 = (tile / nco) * TC, co0 = (tile % nco) * TC;
  const int rb0 = chunk * g.rows_per, rb1 = min(g.M, rb0 + g.rows_per);
  const int HW = g.R.H * g.R.W;
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3, rowoff = 4 * g4 + qq;

  f32x4 acc[NW][NW];
#pragma unroll
  for (int i = 0; i < NW; ++i)
#pragma unroll
    for (int j = 0; j < NW; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  uint4 rx[NLD], rd[NLD];
  // Row decode without per-load divisions: thread rows are r0 + (BLK / SEGS) * s of each sub-tile,
  // so (b, y, x) of row rs + r0 is carried across sub-tiles and stepped by adding columns.
  constexpr int RSTEP = BLK / SEGS;
  const int r0 = tid / SEGS, seg = tid % SEGS;
  int cb, cy, cx;
  {
    const int m = rb0 + r0, rem = m % HW;
    cb = m / HW;
    cy = rem / g.R.W;
    cx = rem - cy * g.R.W;
  }
  auto step = [&](int& b, int& y, int& x, int k) {
    x += k;
    while (x >= g.R.W) {
      x -= g.R.W;
      if (++y == g.R.H) {
        y = 0;
        ++b;
      }
    }
  };
  auto gload = [&](int rs) {
    int b = cb, y = cy, x = cx;
#pragma unroll
    for (int s = 0; s < NLD; ++s) {
      if (s) step(b, y, x, RSTEP);
      const int m = rs + r0 + s * RSTEP;
      rx[s] = rd[s] = make_uint4(0u, 0u, 0u, 0u);
      if (m < rb1) {
        int xs, ds;
        if (MAP == M_U2) {
          xs = m;
          ds = out_row<MAP>(m, b, y, x, t, g.O);
        } else {
          xs = src_row<MAP>(b, y, x, t, g.S);
          ds = m;
        }
        if (xs >= 0) {
          rx[s] = *(const uint4*)(g.x + (size_t)xs * g.XP + ci0 + seg * 8);
          rd[s] = *(const uint4*)(g.dz + (size_t)ds * g.DP + co0 + seg * 8);
        }
      }
    }
    step(cb, cy, cx, RT);
  };
  gload(rb0);
  for (int rs = rb0; rs < rb1; rs += RT) {
    __syncthreads();
#pragma unroll
    for (int s = 0; s < NLD; ++s) {
      const int q = tid + s * BLK, r = q / SEGS, seg = q % SEGS;
      *(uint4*)&sX[r * P + seg * 8] = rx[s];
      *(uint4*)&sD[r * P + seg * 8] = rd[s];
    }
    __syncthreads();
    if (rs + RT < rb1) gload(rs + RT);
#pragma unroll
    for (int ks = 0; ks < RT / 32; ++ks) {
      const int r0 = 32 * ks + rowoff;
      bf16x8 a[NW], b[NW];
#pragma unroll
      for (int i = 0; i < NW; ++i) {
        const int c = wci * WT + i * 16 + 4 * pp;
        s16x4 v[2] = {tr_read(&sX[r0 * P + c]), tr_read(&sX[(r0 + 16) * P + c])};
        a[i] = *(bf16x8*)v;
      }
#pragma unroll
      for (int j = 0; j < NW; ++j) {
        const int c = wco * WT + j * 16 + 4 * pp;
        s16x4 v[2] = {tr_read(&sD[r0 * P + c]), tr_read(&sD[(r0 + 16) * P + c])};
        b[j] = *(bf16x8*)v;
      }
#pragma unroll
      for (int i = 0; i < NW; ++i)
#pragma unroll
        for (int j = 0; j < NW; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  float* out = g.part + ((size_t)chunk * T + t) * g.CI * g.CO;
#pragma unroll
  for (int i = 0; i < NW; ++i)
#pragma unroll
    for (int j = 0; j < NW; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ci = ci0 + wci * WT + i * 16 + 4 * g4 + r, co = co0 + wco * WT + j * 16 + (lane & 15);
        out[(size_t)ci * g.CO + co] = acc[i][j][r];
      }
}

// ------------------------------------------------------------------ 3x3 stride-1 weight gradient, taps sharing tiles
// k_wgrad_s1: dW[t][ci][co] = sum_m x[src(m, t)][ci] dz[m][co] for the S1 map, with the output pixels
// walked as SEG-pixel segments of one image row. A segment's dz tile (SEG rows) and its x tile of the
// input row y + dy - 1 (SEG + 2 rows: columns x0 - 1 .. x0 + SEG, zero outside the image) feed all three
// taps (dy, 0..2) of that row: tap dx reads x rows r + dx for output row r, so no per-tap masking is
// needed (a segment never crosses an image row) and every staged byte serves 3 taps (k_wgrad stages
// both operands once per tap). Block = (chunk of segments, dy, 128 x 128 (ci, co) tile), 8 waves as
// 4 (ci, 32 each) x 2 (co, 64 each), each with 3 taps x 2 x 4 MFMA accumulator tiles (96 AGPRs; two
// waves per SIMD, so one wave's LDS reads overlap the other's MFMAs).
// Staging is LDS-DMA only, into a ring of WS_ST segment stages issued WS_ST - 1 segments ahead (no
// VGPR round trip: the register-staged form of this kernel was bound by its one-segment-ahead
// prefetch). Rows are unpadded 256-byte images whose 16-byte granules are XOR-swizzled by
// ((row & 7) << 1) through the DMA's per-lane source address, which makes the transposed 8-byte
// operand reads (ds_read_b64_tr_b16) of any 8 consecutive rows conflict-free. Every wave issues the
// same number of DMA instructions per segment (surplus ones repeat the last: same bytes, same place),
// so one counted vmcnt per segment retires exactly that segment's tiles before the barrier. Segments
// whose source row y + dy - 1 lies outside the image are skipped (walked with counters, no
// divisions); pixels past the row end are zero rows. Partial sums go to part[chunk][t][ci][co] like
// k_wgrad (same k_wgrad_reduce).
constexpr int WS_ST = 4;    // ring stages
// ds_read_b64_tr_b16 at an LDS byte address, as inline asm (the caller waits on lgkmcnt)
__device__ __forceinline__ s16x4 tr_read_asm(unsigned addr) {
  s16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
constexpr int WSB = 512;    // threads
template <int SEG, int PIPE = 0>
__global__ __launch_bounds__(WSB, 1) void k_wgrad_s1(WG g, int nseg_x, int seg_per) {
  constexpr int TC = 128, RB = 256;                              // 256-byte rows (128 bf16 channels)
  constexpr int NWI = 2, NWJ = 4;                                // 16x16 tiles per wave (ci, co)
  constexpr int XR = SEG + 2, NX = (XR + 3) / 4, ND = SEG / 4;   // DMA instructions (4 rows each)
  constexpr int NI = NX + ND, PW = (NI + 7) / 8;                 // per segment, per wave
  constexpr int XB = NX * 4 * RB, STB = XB + SEG * RB;           // x tile bytes, stage bytes
  static_assert(SEG % 32 == 0 && WS_ST * STB <= 160 * 1024, "segment");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[WS_ST * STB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wci = w >> 1, wco = w & 1;
  const int nco = g.CO / TC, ntile = (g.CI / TC) * nco;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = lid / (3 * ntile), rest = lid - chunk * (3 * ntile);
  const int dy = rest / ntile, tile = rest - dy * ntile;
  const int ci0 = (tile / nco) * TC, co0 = (tile % nco) * TC;
  const int H = g.R.H, W = g.R.W;
  const int nseg = g.R.B * H * nseg_x;
  const int sg0 = min(nseg, chunk * seg_per), sg1 = min(nseg, sg0 + seg_per);
  const bool skip_top = dy == 0, skip_bot = dy == 2;   // source row outside the image at y = 0 / H - 1

  // ---- segment walk (uniform): position of segment sg0, count of valid segments
  int cx = sg0 % nseg_x, cby = sg0 / nseg_x;
  int cy = cby % H, cb = cby / H;
  int nvalid = 0;
  {
    int y = cy, left = sg1 - sg0, xs = cx;
    while (left > 0) {
      const int n = min(left, nseg_x - xs);
      if (!((skip_top && y == 0) || (skip_bot && y == H - 1))) nvalid += n;
      left -= n;
      xs = 0;
      if (++y == H) y = 0;
    }
  }
  int ileft = sg1 - sg0;   // segments not yet passed by the issue cursor
  auto skip_invalid = [&]() {
    while (ileft > 0 && ((skip_top && cy == 0) || (skip_bot && cy == H - 1))) {
      ileft -= nseg_x - cx;
      cx = 0;
      if (++cy == H) { cy = 0; ++cb; }
    }
  };
  auto advance = [&]() {
    --ileft;
    if (++cx == nseg_x) {
      cx = 0;
      if (++cy == H) { cy = 0; ++cb; }
    }
  };

  // ---- DMA: instruction k = w + 8m covers rows 4k' .. 4k' + 3 of the x (k < NX) or dz (k' = k - NX)
  // tile; lane L writes row 4k' + L / 16, slot L % 16 = granule ^ swz(row)
  // per-lane constants of each DMA instruction (g's fields copied to registers first: reading them
  // inside the loop went through memory and made the compiler wait for every DMA in flight)
  const u16* const gx = g.x;
  const u16* const gdz = g.dz;
  const int XP = g.XP, DP = g.DP;
  const u16* lbase[PW];
  int lrow[PW], lpitch[PW], ladj[PW], llim[PW], kslot[PW];
  bool isx[PW];
#pragma unroll
  for (int m = 0; m < PW; ++m) {
    const int k = min(w + 8 * m, NI - 1);
    isx[m] = k < NX;
    kslot[m] = k;
    lrow[m] = 4 * (isx[m] ? k : k - NX) + (lane >> 4);
    const int gsrc = ((lane & 15) ^ ((lrow[m] & 7) << 1)) * 8;   // source channel offset of the granule
    lbase[m] = isx[m] ? gx + ci0 + gsrc : gdz + co0 + gsrc;
    lpitch[m] = isx[m] ? XP : DP;
    ladj[m] = isx[m] ? -1 : 0;
    llim[m] = isx[m] ? XR : SEG;
  }
  int lastx = 0, lasty = 0, lastb = 0;
  auto issue = [&](int st) {
    // the cursor's segment, or (past the end) the last one again into a stage that is never read
    const bool have = ileft > 0;
    const int xs = have ? cx : lastx, y = have ? cy : lasty, b = have ? cb : lastb;
    lastx = xs; lasty = y; lastb = b;
    const int x0 = xs * SEG;
    const int xrow0 = (b * H + y + dy - 1) * W, drow0 = (b * H + y) * W;
    unsigned char* base = lds + st * STB;
#pragma unroll
    for (int m = 0; m < PW; ++m) {
      const int xc = x0 + lrow[m] + ladj[m];
      const bool ok = lrow[m] < llim[m] && xc >= 0 && xc < W;
      const int row = (isx[m] ? xrow0 : drow0) + xc;
      const u16* src = ok ? lbase[m] + (size_t)row * lpitch[m] : (const u16*)g_zero_row;
      glds16(src, base + kslot[m] * 1024);
    }
    if (have) {
      advance();
      skip_invalid();
    }
  };

  // ---- operand addresses: transposed reads of rows r0 (+16) (+dx), r0 = 32 ks + 4 (lane >> 4) + (lane & 15) / 4,
  // 4 channels 4 (lane & 3) of a 16-column block; granule ((c >> 3) ^ swz(row)), byte 8 (lane & 1) in it
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3, rowoff = 4 * g4 + qq;
  int aoff[3][NWI], boff[NWJ];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int sw = ((rowoff + dx) & 7) << 1;
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int gr = ((wci * 32 + i * 16) >> 3) + (pp >> 1);
      aoff[dx][i] = (rowoff + dx) * RB + ((gr ^ sw) << 4) + 8 * (pp & 1);
    }
  }
#pragma unroll
  for (int j = 0; j < NWJ; ++j) {
    const int gr = ((wco * 64 + j * 16) >> 3) + (pp >> 1);
    boff[j] = XB + rowoff * RB + ((gr ^ ((rowoff & 7) << 1)) << 4) + 8 * (pp & 1);
  }

  f32x4 acc[3][NWI][NWJ];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < NWI; ++i)
#pragma unroll
      for (int j = 0; j < NWJ; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (nvalid > 0) {
    skip_invalid();
#pragma unroll
    for (int st = 0; st < WS_ST - 1; ++st) issue(st);
    int st = 0;
    const unsigned lds0 = (unsigned)(size_t)((__attribute__((address_space(3))) unsigned char*)lds);
    if constexpr (PIPE) {
      // pipelined form: the 20 transposed reads of the next K sub-step (this segment's second, or the next
      // segment's first) are issued before the 24 MFMAs of this one, whose fragments were read before
      // the previous sub-step's MFMAs. The next segment's stage must then be published one segment
      // earlier: each segment retires its own AND the next stage (vmcnt(PW): only the stage issued last
      // segment stays in flight). The refill after the barrier overwrites the stage of segment k - 1,
      // last read during segment k - 1. At the last segment the reads of "segment nvalid" hit LDS that
      // is never used.
#define WS1_READ(AV, BV, sbase, ks)                                                                         \
      {                                                                                                     \
        _Pragma("unroll") for (int j = 0; j < NWJ; ++j) {                                                   \
          const unsigned pb = (sbase) + boff[j] + 32 * (ks) * RB;                                           \
          s16x4 v[2] = {tr_read_asm(pb), tr_read_asm(pb + 16 * RB)};                                        \
          BV[j] = *(bf16x8*)v;                                                                              \
        }                                                                                                   \
        _Pragma("unroll") for (int dx = 0; dx < 3; ++dx)                                                    \
          _Pragma("unroll") for (int i = 0; i < NWI; ++i) {                                                 \
            const unsigned pa = (sbase) + aoff[dx][i] + 32 * (ks) * RB;                                     \
            s16x4 v[2] = {tr_read_asm(pa), tr_read_asm(pa + 16 * RB)};                                      \
            AV[dx][i] = *(bf16x8*)v;                                                                        \
          }                                                                                                 \
      }
#define WS1_MMA(AV, BV, WAIT)                                                                               \
      {                                                                                                     \
        asm volatile(WAIT : "+v"(BV[0]), "+v"(BV[1]), "+v"(BV[2]), "+v"(BV[3]), "+v"(AV[0][0]),              \
                     "+v"(AV[0][1]), "+v"(AV[1][0]), "+v"(AV[1][1]), "+v"(AV[2][0]), "+v"(AV[2][1]));        \
        _Pragma("unroll") for (int dx = 0; dx < 3; ++dx)                                                    \
          _Pragma("unroll") for (int i = 0; i < NWI; ++i)                                                   \
            _Pragma("unroll") for (int j = 0; j < NWJ; ++j)                                                 \
              acc[dx][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(AV[dx][i], BV[j], acc[dx][i][j], 0, 0, 0); \
      }
      // one segment: publish, refill, then its SEG / 32 sub-steps (FC: this sub-step's fragments)
#define WS1_SEG(FCA, FCB, FNA, FNB)                                                                         \
      {                                                                                                     \
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PW) : "memory");                             \
        issue(st == 0 ? WS_ST - 1 : st - 1);                                                                \
        const unsigned base = lds0 + st * STB;                                                              \
        const unsigned nbase = lds0 + (st == WS_ST - 1 ? 0 : st + 1) * STB;                                 \
        if constexpr (SEG == 64) {                                                                          \
          WS1_READ(FNA, FNB, base, 1)                                                                       \
          WS1_MMA(FCA, FCB, "s_waitcnt lgkmcnt(15)")                                                        \
          WS1_READ(FCA, FCB, nbase, 0)                                                                      \
          WS1_MMA(FNA, FNB, "s_waitcnt lgkmcnt(15)")                                                        \
        } else {                                                                                            \
          WS1_READ(FNA, FNB, nbase, 0)                                                                      \
          WS1_MMA(FCA, FCB, "s_waitcnt lgkmcnt(15)")                                                        \
        }                                                                                                   \
        st = st == WS_ST - 1 ? 0 : st + 1;                                                                  \
      }
      static_assert(NWI == 2 && NWJ == 4 && (SEG == 64 || SEG == 32), "operand tie list");
      bf16x8 a0[3][NWI], b0[NWJ], a1[3][NWI], b1[NWJ];
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(PW) : "memory");   // stages 0 and 1
      WS1_READ(a0, b0, lds0, 0)
      int k = 0;
      if constexpr (SEG == 64) {
        for (; k < nvalid; ++k) WS1_SEG(a0, b0, a1, b1)
      } else {
        for (; k + 1 < nvalid; k += 2) {
          WS1_SEG(a0, b0, a1, b1)
          WS1_SEG(a1, b1, a0, b0)
        }
        if (k < nvalid) WS1_SEG(a0, b0, a1, b1)
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#undef WS1_SEG
#undef WS1_MMA
#undef WS1_READ
    } else {
    for (int k = 0; k < nvalid; ++k) {
        // retire this segment's DMAs (the WS_ST - 2 younger segments stay in flight), then publish
        asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((WS_ST - 2) * PW) : "memory");
        // refill the stage computed last iteration (every wave has passed this barrier after reading it)
        issue(st == 0 ? WS_ST - 1 : st - 1);
        const unsigned base = lds0 + st * STB;
  #pragma unroll
        for (int ks = 0; ks < SEG / 32; ++ks) {
          // operand reads as inline asm: the compiler cannot tell the transposed-read intrinsic apart
          // from the DMA-written stages in flight and put a vmcnt(0) (every DMA, the look-ahead too)
          // before it. The asm wait below ties the fragments, so no MFMA is scheduled above it.
          bf16x8 bv[NWJ], av[3][NWI];
  #pragma unroll
          for (int j = 0; j < NWJ; ++j) {
            const unsigned pb = base + boff[j] + 32 * ks * RB;
            s16x4 v[2] = {tr_read_asm(pb), tr_read_asm(pb + 16 * RB)};
            bv[j] = *(bf16x8*)v;
          }
  #pragma unroll
          for (int dx = 0; dx < 3; ++dx)
  #pragma unroll
            for (int i = 0; i < NWI; ++i) {
              const unsigned pa = base + aoff[dx][i] + 32 * ks * RB;
              s16x4 v[2] = {tr_read_asm(pa), tr_read_asm(pa + 16 * RB)};
              av[dx][i] = *(bf16x8*)v;
            }
          static_assert(NWI == 2 && NWJ == 4, "operand tie list");
          asm volatile("s_waitcnt lgkmcnt(0)"
                       : "+v"(bv[0]), "+v"(bv[1]), "+v"(bv[2]), "+v"(bv[3]), "+v"(av[0][0]), "+v"(av[0][1]),
                         "+v"(av[1][0]), "+v"(av[1][1]), "+v"(av[2][0]), "+v"(av[2][1]));
  #pragma unroll
          for (int dx = 0; dx < 3; ++dx)
  #pragma unroll
            for (int i = 0; i < NWI; ++i)
  #pragma unroll
              for (int j = 0; j < NWJ; ++j)
                acc[dx][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[dx][i], bv[j], acc[dx][i][j], 0, 0, 0);
        }
        st = st == WS_ST - 1 ? 0 : st + 1;
      }
    }
    // drain the look-ahead DMAs before the block exits
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    float* out = g.part + ((size_t)chunk * 9 + dy * 3 + dx) * g.CI * g.CO;
#pragma unroll
    for (int i = 0; i < NWI; ++i)
#pragma unroll
      for (int j = 0; j < NWJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ci = ci0 + wci * 32 + i * 16 + 4 * g4 + r, co = co0 + wco * 64 + j * 16 + (lane & 15);
          out[(size_t)ci * g.CO + co] = acc[dx][i][j][r];
        }
  }
}

// ------------------------------------------------------------------ 3x3 stride-1 weight gradient, column walk, 9 taps
// k_wgrad_s1c: the S1 weight gradient with ONE block per (SEG-pixel column strip, 64 ci x 128 co tile, run of
// image rows) accumulating all 9 taps, walking the strip DOWN the image. An x row r (pixels x0 - 1 .. x0 + SEG)
// is staged once and serves output rows r + 1, r, r - 1 (dy = 0, 1, 2) at its three column shifts (dx); the dz
// row y once for all 9 taps. Per output row the block stages one x row (SEG + 2 px x 128 B) and one dz row (SEG
// px x 256 B) for 9 x 64 x 128 MACs per pixel: 2.6 KB of LDS-DMA per MFLOP against k_wgrad_s1's 5.2 (3 taps of
// one kernel row per staged tile) — the S1 weight gradient is bound by its per-CU staging.
// Steps walk the x rows r = -1 .. H of each image (zero rows at -1 and H, so no row ever mixes two images); the
// step of x row r computes output row r - 1 (none for r < 1). A run of steps [s0, s1) is preceded by its two
// warm-up rows s0 - 2, s0 - 1 (staged, not computed). Ring: XS = L + 3 x-row slots (three read per step, L in
// flight), DS = L + 1 dz slots; every wave issues the same PW DMA instructions per step, so one counted vmcnt
// retires a step. Rows are unpadded: x rows of 128 B with granule g at slot g ^ (((p >> 1) & 3) << 1), dz rows
// of 256 B at g ^ ((p & 7) << 1) (pixel p): every transposed operand read (8 consecutive pixels x one granule
// pair per 32 lanes) hits 32 distinct 8-byte bank words. 8 waves = 4 (16 ci) x 2 (64 co), each 9 taps x 4
// accumulator tiles (144 VGPRs), two waves per SIMD. Partial sums go to part[run][strip][t][ci][co] (the
// k_wgrad_reduce slab layout: chunks = runs x strips).
constexpr int WC_L = 2;     // steps of DMA look-ahead
template <int SEG>
struct S1C {
  static constexpr int XR = SEG + 2, NXI = (XR + 7) / 8, NDI = SEG / 4, NI = NXI + NDI, PW = (NI + 7) / 8;
  static constexpr int XSB = NXI * 1024, DSB = NDI * 1024, XS = WC_L + 3, DS = WC_L + 1;
  static constexpr int LDSB = XS * XSB + DS * DSB;
  static_assert(LDSB <= 160 * 1024, "ring");
};
__device__ __forceinline__ int s1c_xswz(int p) { return ((p >> 1) & 3) << 1; }
__device__ __forceinline__ int s1c_dswz(int p) { return (p & 7) << 1; }
template <int SEG, int DBG = 0>   // DBG: timing arms (knob 7) — 1: no slab stores, 2: no MFMAs, 4: no LDS reads
__global__ __launch_bounds__(WSB, 1) void k_wgrad_s1c(WG g, int nstrip, int steps_per) {
  using K = S1C<SEG>;
  constexpr int PW = K::PW, NXI = K::NXI, NI = K::NI, XR = K::XR;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[K::LDSB];
  unsigned char* const xring = lds;
  unsigned char* const dring = lds + K::XS * K::XSB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: the DMA table below stays scalar
  const int wci = w >> 1, wco = w & 1;
  const int nco = g.CO / 128, ntile = (g.CI / 64) * nco;
  const int lid = xcd_remap(blockIdx.x, gridDim.x);        // a run's tiles and strips adjacent (one XCD's L2)
  const int tile = lid % ntile, rest = lid / ntile;
  const int strip = rest % nstrip, run = rest / nstrip;
  const int ci0 = (tile / nco) * 64, co0 = (tile % nco) * 128;
  const int H = g.R.H, W = g.R.W, HP = H + 2;
  const int nsteps = g.R.B * HP;
  const int s0 = min(nsteps, run * steps_per), s1 = min(nsteps, s0 + steps_per);
  const int x0 = strip * SEG;

  // ---- per-lane DMA constants: instruction k = w + 8m (surplus ones repeat the last: same bytes, same place);
  // k < NXI: x pixels 8k .. 8k + 7 (lane L: pixel 8k + L / 8, slot L % 8), else dz pixels 4k' .. 4k' + 3 (lane L:
  // pixel 4k' + L / 16, slot L % 16); the lane's source granule is its slot ^ swizzle(pixel)
  const u16* const gx = g.x;
  const u16* const gdz = g.dz;
  const int XP = g.XP, DP = g.DP;
  int loff[PW];   // per lane: element offset of its granule in the image row, -1: zero (outside the image)
#pragma unroll
  for (int m = 0; m < PW; ++m) {
    const int k = min(w + 8 * m, NI - 1);
    if (k < NXI) {
      const int p = 8 * k + (lane >> 3), sl = lane & 7, xc = x0 - 1 + p;
      loff[m] = (p < XR && xc >= 0 && xc < W) ? xc * XP + ci0 + (sl ^ s1c_xswz(p)) * 8 : -1;
    } else {
      const int kd = k - NXI, p = 4 * kd + (lane >> 4), sl = lane & 15, xc = x0 + p;
      loff[m] = xc < W ? xc * DP + co0 + (sl ^ s1c_dswz(p)) * 8 : -1;
    }
  }
  // step s: x row r = s % HP - 1 of image s / HP into x slot s % XS; for r >= 1 the dz row r - 1 into dz slot
  // s % DS; rows outside the image / steps outside [0, nsteps) read the zero row
  struct Iss {
    const u16* xsrc;   // image row base of the x row (nullptr: zero row)
    const u16* dsrc;   // of the dz row
    unsigned char* xdst;
    unsigned char* ddst;
  };
  auto issue_prep = [&](int s) {
    const int b = s >= 0 ? s / HP : 0, r = s >= 0 ? s - b * HP - 1 : -1;
    const bool live = s >= 0 && s < nsteps;
    const bool xrow = live && r >= 0 && r < H, drow = live && r >= 1;
    const int xs = ((s % K::XS) + K::XS) % K::XS, ds = ((s % K::DS) + K::DS) % K::DS;
    Iss q;
    q.xsrc = xrow ? gx + (size_t)(b * H + r) * W * XP : nullptr;
    q.dsrc = drow ? gdz + (size_t)(b * H + r - 1) * W * DP : nullptr;
    q.xdst = xring + xs * K::XSB;
    q.ddst = dring + ds * K::DSB;
    return q;
  };
  auto issue_one = [&](const Iss& q, int m) {
    const int k = min(w + 8 * m, NI - 1);   // (uniform)
    const bool isx = k < NXI;
    const u16* base = isx ? q.xsrc : q.dsrc;
    const u16* src = (loff[m] >= 0 && base != nullptr) ? base + loff[m] : (const u16*)g_zero_row;
    glds16(src, (isx ? q.xdst + k * 1024 : q.ddst + (k - NXI) * 1024));
  };
  auto issue = [&](int s) {
    const Iss q = issue_prep(s);
#pragma unroll
    for (int m = 0; m < PW; ++m) issue_one(q, m);
  };

  // ---- operand offsets (as k_wgrad_s1): lane reads pixel rowoff (+16) of a 32-pixel K-step, 4 channels 4 (lane & 3)
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3, rowoff = 4 * g4 + qq;
  unsigned aoff[3], boff[4];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) {
    const int p = rowoff + dx, gr = 2 * wci + (pp >> 1);
    aoff[dx] = p * 128 + ((gr ^ s1c_xswz(p)) << 4) + 8 * (pp & 1);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int gr = ((wco * 64 + j * 16) >> 3) + (pp >> 1);
    boff[j] = rowoff * 256 + ((gr ^ s1c_dswz(rowoff)) << 4) + 8 * (pp & 1);
  }
  f32x4 acc[9][4];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[t][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const unsigned xl0 = (unsigned)(size_t)((__attribute__((address_space(3))) unsigned char*)xring);
  const unsigned dl0 = (unsigned)(size_t)((__attribute__((address_space(3))) unsigned char*)dring);
  if (s0 < s1) {
#pragma unroll
    for (int k = 0; k < WC_L; ++k) issue(s0 - 2 + k);
    for (int s = s0 - 2; s < s1; ++s) {
      // retire step s (the L - 1 younger steps stay in flight), publish, then refill the slots step s - 1 read
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"((WC_L - 1) * PW) : "memory");
      const int r = s - (s / HP) * HP - 1;   // (s >= s0 - 2 >= -2; only s >= s0 computes)
      // a computing step spreads the DMA of step s + L over its MFMA groups (issued between them, each piece's
      // issue cost lies under the wave's MFMAs instead of delaying its first operand reads); DBG 8: all at once.
      // (Written as two ifs, not an early `continue`: with the continue the compiler kept the DMA state live
      // across both paths and spilled the accumulators.)
      const Iss iq = issue_prep(s + WC_L);
      const bool comp = s >= s0 && r >= 1;
      if (!comp || (DBG & 8)) {
#pragma unroll
        for (int m = 0; m < PW; ++m) issue_one(iq, m);
      }
      if (comp) {
      // x slots of steps s - 2, s - 1, s = x rows y - 1, y, y + 1 of output row y = r - 1 (dy = 0, 1, 2)
      unsigned xb[3];
#pragma unroll
      for (int dy = 0; dy < 3; ++dy) xb[dy] = xl0 + (unsigned)(((s - 2 + dy) % K::XS) * K::XSB);
      const unsigned db = dl0 + (unsigned)((s % K::DS) * K::DSB);
      // per K-step of 32 pixels: 4 dz fragments + 3 x fragments per kernel row dy; the reads of the next
      // kernel row (or the next K-step's dz and first row) are issued before this row's 12 MFMAs, so each
      // wave's LDS reads lie under its own MFMAs (two fragment buffers per operand)
#define S1C_RB(BV, ks)                                                                                      \
      if (!(DBG & 4)) _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                        \
        const unsigned pb = db + boff[j] + 32 * (ks) * 256;                                                 \
        s16x4 v[2] = {tr_read_asm(pb), tr_read_asm(pb + 16 * 256)};                                         \
        BV[j] = *(bf16x8*)v;                                                                                \
      }
#define S1C_RA(AV, ks, dy)                                                                                  \
      if (!(DBG & 4)) _Pragma("unroll") for (int dx = 0; dx < 3; ++dx) {                                     \
        const unsigned pa = xb[dy] + aoff[dx] + 32 * (ks) * 128;                                            \
        s16x4 v[2] = {tr_read_asm(pa), tr_read_asm(pa + 16 * 128)};                                         \
        AV[dx] = *(bf16x8*)v;                                                                               \
      }
#define S1C_WAIT_A(AV) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(AV[0]), "+v"(AV[1]), "+v"(AV[2]));
#define S1C_WAIT_AB(AV, BV)                                                                                 \
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(AV[0]), "+v"(AV[1]), "+v"(AV[2]), "+v"(BV[0]), "+v"(BV[1]), \
                   "+v"(BV[2]), "+v"(BV[3]));
#define S1C_MMA(AV, BV, dy)                                                                                 \
      if (!(DBG & 2)) _Pragma("unroll") for (int dx = 0; dx < 3; ++dx)                                       \
        _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                       \
          acc[(dy) * 3 + dx][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(AV[dx], BV[j], acc[(dy) * 3 + dx][j], 0, 0, 0);
      constexpr int NG = 3 * (SEG / 32);   // MFMA groups per step
#define S1C_ISSUE(gi)                                                                                       \
      if (!(DBG & 8)) _Pragma("unroll") for (int m = (gi) * PW / NG; m < ((gi) + 1) * PW / NG; ++m) issue_one(iq, m);
      // dz fragments double-buffered: the next K-step's dz and first x row are read before this K-step's last
      // MFMA group
      bf16x8 b0[4], b1[4], a0[3], a1[3];
      S1C_RB(b0, 0)
      S1C_RA(a0, 0, 0)
#pragma unroll
      for (int ks = 0; ks < SEG / 32; ++ks) {
        bf16x8* bc = (ks & 1) ? b1 : b0;   // (constant after unrolling)
        bf16x8* bn = (ks & 1) ? b0 : b1;
        S1C_WAIT_AB(a0, bc)
        S1C_RA(a1, ks, 1)
        S1C_MMA(a0, bc, 0)
        S1C_ISSUE(ks * 3 + 0)
        S1C_WAIT_A(a1)
        S1C_RA(a0, ks, 2)
        S1C_MMA(a1, bc, 1)
        S1C_ISSUE(ks * 3 + 1)
        S1C_WAIT_A(a0)
        if (ks + 1 < SEG / 32) {
          S1C_RB(bn, ks + 1)
          S1C_RA(a1, ks + 1, 0)
        }
        S1C_MMA(a0, bc, 2)
        S1C_ISSUE(ks * 3 + 2)
        if (ks + 1 < SEG / 32) {
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) a0[dx] = a1[dx];
        }
      }
#undef S1C_RB
#undef S1C_RA
#undef S1C_WAIT_A
#undef S1C_WAIT_AB
#undef S1C_MMA
#undef S1C_ISSUE
      }
    }
    // drain the look-ahead DMAs before the block exits
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // lane (a15 = lane & 15, g4) of tile (t, j) holds dW[t][ci0 + 16 wci + 4 g4 + r][co0 + 64 wco + 16 j + a15]
  const size_t slab = (size_t)g.CI * g.CO;
  float* out = g.part + (size_t)(run * nstrip + strip) * 9 * slab;
  if (DBG & 1) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) t += acc[k][j][0] + acc[k][j][1] + acc[k][j][2] + acc[k][j][3];
    if (t == 12345.f) out[tid] = t;
    return;
  }
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ci = ci0 + 16 * wci + 4 * g4 + r, co = co0 + 64 * wco + 16 * j + (lane & 15);
        out[t * slab + (size_t)ci * g.CO + co] = acc[t][j][r];
      }
}

// ------------------------------------------------------------------ BatchNorm passes (8 channels / thread)
// Every pass maps a 256-thread block to (256 / CG) row lanes x CG channel groups of 8 (CG = C / 8),
// so a thread keeps its 8 channels' BatchNorm parameters in registers for all of its rows, and
// walks rows strided over the grid with RU rows per iteration (RU 16-byte loads per stream in flight).
// The element type E is u16 (bf16 images, perf mode) or float (fp32 images, parity mode): 8 channels
// are one 16-byte load of bf16 or two of fp32.
constexpr int RU = 4;

template <typename E>
struct Raw8 {
  uint4 u[sizeof(E) / 2];
};
template <typename E>
__device__ __forceinline__ Raw8<E> ld8(const E* p) {
  Raw8<E> r;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(E) / 2); ++k) r.u[k] = ((const uint4*)p)[k];
  return r;
}
__device__ __forceinline__ float el(const Raw8<u16>& r, int j) { return bf2f(((const u16*)r.u)[j]); }
__device__ __forceinline__ float el(const Raw8<float>& r, int j) { return ((const float*)r.u)[j]; }
__device__ __forceinline__ void st8(u16* p, const float* v) {
  u16 o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
  *(uint4*)p = *(uint4*)o;
}
__device__ __forceinline__ void st8(float* p, const float* v) {
  ((float4*)p)[0] = make_float4(v[0], v[1], v[2], v[3]);
  ((float4*)p)[1] = make_float4(v[4], v[5], v[6], v[7]);
}

// h = relu((z - mean) * scale + beta) -> image rows at (OP, OOFF); bn = scale, beta, mean, invstd
// row mapping of the elementwise passes (knob 9): V = 0 grid-stride batches of RU rows (a thread's rows
// gridDim * RL apart); V = 1 / 2: each block one contiguous chunk of RL * 4 / RL * 8 rows, all in flight at once
template <int V>
__device__ __forceinline__ int ew_row(int m0, int u, int step, int RL) {
  return V == 0 ? m0 + u * step : m0 + u * RL;
}
template <int V>
constexpr int ew_ru() { return V == 2 ? 8 : RU; }

template <typename E, int V = 0>
__global__ __launch_bounds__(BLK) void k_bn_apply(const E* __restrict__ z, int M, int C, const float* __restrict__ bn,
                                                  E* __restrict__ out, int OP, int OOFF) {
  const int CG = C >> 3, RL = BLK / CG;
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  if (rl >= RL) return;
  float sc[8], sh[8], mu[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cg * 8 + j;
    sc[j] = bn[c];
    sh[j] = bn[C + c];
    mu[j] = bn[2 * C + c];
  }
  constexpr int R = ew_ru<V>();
  const int step = gridDim.x * RL;
  for (int m0 = V == 0 ? blockIdx.x * RL + rl : blockIdx.x * RL * R + rl; m0 < M; m0 += V == 0 ? R * step : R * step) {
    Raw8<E> v[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int m = ew_row<V>(m0, u, step, RL);
      if (m < M) v[u] = ld8(z + (size_t)m * C + cg * 8);
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int m = ew_row<V>(m0, u, step, RL);
      if (m >= M) continue;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaxf(fmaf(el(v[u], j) - mu[j], sc[j], sh[j]), 0.0f);
      st8(out + (size_t)m * OP + OOFF + cg * 8, o);
    }
  }
}

// BatchNorm-backward partial sums: dm = dh * [pre > 0]; part[blk] = (sum dm, sum dm * xhat).
// A: the accumulator and partial-row type — float for the bf16 engine; double for the fp32 (parity)
// engine, whose sums over sparse BEV images cancel (rpc_bn_finalize mode 1 | RPC_BN_PART_F64 reads them)
template <typename E, typename A>
__global__ __launch_bounds__(BLK) void k_bnbwd_stats(const E* __restrict__ dh, int DP, int DOFF,
                                                     const E* __restrict__ z, int M, int C,
                                                     const float* __restrict__ bn, A* __restrict__ part) {
  __shared__ A sh[2][BLK * 8];
  const int CG = C >> 3, RL = BLK / CG;
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  A s1[8], s2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s1[j] = s2[j] = A(0);
  if (rl < RL) {
    float sc[8], be[8], mu[8], is[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cg * 8 + j;
      sc[j] = bn[c];
      be[j] = bn[C + c];
      mu[j] = bn[2 * C + c];
      is[j] = bn[3 * C + c];
    }
    const int step = gridDim.x * RL;
    for (int m0 = blockIdx.x * RL + rl; m0 < M; m0 += RU * step) {
      Raw8<E> dv[RU], zv[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        const int m = m0 + u * step;
        if (m < M) {
          dv[u] = ld8(dh + (size_t)m * DP + DOFF + cg * 8);
          zv[u] = ld8(z + (size_t)m * C + cg * 8);
        }
      }
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        if (m0 + u * step >= M) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float zz = el(zv[u], j);
          const float pre = fmaf(zz - mu[j], sc[j], be[j]);
          const A d = pre > 0.f ? A(el(dv[u], j)) : A(0);
          s1[j] += d;
          s2[j] += d * ((A(zz) - A(mu[j])) * A(is[j]));
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sh[0][threadIdx.x * 8 + j] = s1[j];
    sh[1][threadIdx.x * 8 + j] = s2[j];
  }
  __syncthreads();
  // fixed-order combine over the row lanes: channel c = cg*8 + j
  for (int c = threadIdx.x; c < C; c += BLK) {
    const int g8 = c >> 3, j = c & 7;
    A a = A(0), b = A(0);
    for (int r = 0; r < RL; ++r) {
      a += sh[0][(r * CG + g8) * 8 + j];
      b += sh[1][(r * CG + g8) * 8 + j];
    }
    part[(size_t)blockIdx.x * 2 * C + c] = a;
    part[(size_t)blockIdx.x * 2 * C + C + c] = b;
  }
}

// dz = gi * (dm - m1 - xhat * m2) -> [M][C]; bnb = gi, m1, m2, mean, invstd; bn = forward
template <typename E, int V = 0>
__global__ __launch_bounds__(BLK) void k_bnbwd_apply(const E* __restrict__ dh, int DP, int DOFF,
                                                     const E* __restrict__ z, int M, int C,
                                                     const float* __restrict__ bn, const float* __restrict__ bnb,
                                                     E* __restrict__ dz) {
  const int CG = C >> 3, RL = BLK / CG;
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  if (rl >= RL) return;
  float sc[8], be[8], mu[8], gi[8], m1[8], m2[8], mb[8], ib[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = cg * 8 + j;
    sc[j] = bn[c];
    be[j] = bn[C + c];
    mu[j] = bn[2 * C + c];
    gi[j] = bnb[c];
    m1[j] = bnb[C + c];
    m2[j] = bnb[2 * C + c];
    mb[j] = bnb[3 * C + c];
    ib[j] = bnb[4 * C + c];
  }
  constexpr int R = ew_ru<V>();
  const int step = gridDim.x * RL;
  for (int m0 = V == 0 ? blockIdx.x * RL + rl : blockIdx.x * RL * R + rl; m0 < M; m0 += R * step) {
    Raw8<E> dv[R], zv[R];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int m = ew_row<V>(m0, u, step, RL);
      if (m < M) {
        dv[u] = ld8(dh + (size_t)m * DP + DOFF + cg * 8);
        zv[u] = ld8(z + (size_t)m * C + cg * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int m = ew_row<V>(m0, u, step, RL);
      if (m >= M) continue;
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float zz = el(zv[u], j);
        const float pre = fmaf(zz - mu[j], sc[j], be[j]);
        const float d = pre > 0.f ? el(dv[u], j) : 0.f;
        const float xh = (zz - mb[j]) * ib[j];
        o[j] = gi[j] * (d - m1[j] - xh * m2[j]);
      }
      st8(dz + (size_t)m * C + cg * 8, o);
    }
  }
}

// ------------------------------------------------------------------ weight preparation
// torch layouts -> bf16 GEMM operands. kind: 0 Conv2d 3x3 [co][ci][3][3]; 1 ConvTranspose2d
// [ci][co][k][k] (k = 1 or 2). fwd: [T][co][ci]; dgrad: [T][ci][co] with, for a stride-1 3x3
// conv, the taps flipped (S1 data gradient), otherwise the same tap order (D2 / P1 / G2).
__device__ __forceinline__ void wprep_elem(long long e, const float* __restrict__ W, int kind, int CI, int CO, int T,
                                           int flip, u16* __restrict__ wf, u16* __restrict__ wd) {
  const int t = (int)(e / ((long long)CI * CO));
  const int rem = (int)(e - (long long)t * CI * CO), ci = rem / CO, co = rem - ci * CO;
  const float v = kind == 0 ? W[((size_t)co * CI + ci) * T + t] : W[((size_t)ci * CO + co) * T + t];
  if (wf) wf[((size_t)t * CO + co) * CI + ci] = f2bf(v);
  if (wd) {
    const int td = flip ? T - 1 - t : t;
    wd[((size_t)td * CI + ci) * CO + co] = f2bf(v);
  }
}

__global__ __launch_bounds__(BLK) void k_wprep(const float* __restrict__ W, int kind, int CI, int CO, int T,
                                               int flip, u16* __restrict__ wf, u16* __restrict__ wd) {
  const long long e = (long long)blockIdx.x * BLK + threadIdx.x;
  if (e < (long long)T * CI * CO) wprep_elem(e, W, kind, CI, CO, T, flip, wf, wd);
}

// every layer of a module in one launch: blockIdx.y = layer
constexpr int WPREP_MAX = 16;
struct WprepBatch {
  RpcDenseWprep d[WPREP_MAX];
};
// LDS-tiled form: the torch weight of a layer is [A][Bd][T] (Conv2d: A = co, Bd = ci; ConvTranspose2d:
// A = ci, Bd = co) and both operands are a tap-major copy of it, one as [t][a][b], the other as [t][b][a].
// A block moves a 32 x 32 (a, b) tile with all its taps: source rows of 32*T contiguous floats read
// coalesced into LDS, then 64-byte bf16 rows written to both operands (the per-element form read with
// a stride of CI*T floats and wrote 2-byte scattered stores, behind 64-bit index divisions).
constexpr int WPT = 32;
constexpr int WPT_MAXT = 9;
__global__ __launch_bounds__(BLK) void k_wprep_batch(WprepBatch b) {
  // [t][a][b] at t*TP + a*(WPT+1) + b: the odd tap stride keeps the tap-fastest stores of the load
  // loop on distinct banks, the row pad the transposed reads of out2
  constexpr int TP = WPT * (WPT + 1) + 1;
  __shared__ float tile[WPT_MAXT * TP];
  const RpcDenseWprep& d = b.d[blockIdx.y];
  const int T = d.taps;
  const int A = d.kind == 0 ? d.co : d.ci, Bd = d.kind == 0 ? d.ci : d.co;
  const int nbt = (Bd + WPT - 1) / WPT;
  const int ntile = ((A + WPT - 1) / WPT) * nbt;
  if ((int)blockIdx.x >= ntile) return;
  const int a0 = (blockIdx.x / nbt) * WPT, b0 = (blockIdx.x % nbt) * WPT;
  const int an = min(WPT, A - a0), bn = min(WPT, Bd - b0);
  const int row = bn * T;   // contiguous source floats per a
  const int alim = (d.kind == 0 && d.co_src > 0) ? d.co_src : A;   // rows past co_src: zero (padded outputs)
  for (int q = threadIdx.x; q < an * row; q += BLK) {
    const int ar = q / row, k = q - ar * row, br = k / T, t = k - br * T;
    tile[t * TP + ar * (WPT + 1) + br] = a0 + ar < alim ? d.W[((size_t)(a0 + ar) * Bd + b0) * T + k] : 0.0f;
  }
  __syncthreads();
  // out1[t][a][b] (Conv2d: w_fwd [t][co][ci]; ConvTranspose2d: w_dgrad [t][ci][co])
  // out2[t][b][a] (Conv2d: w_dgrad [td][ci][co], td = flip ? T-1-t : t; ConvTranspose2d: w_fwd [t][co][ci])
  u16* out1 = (u16*)(d.kind == 0 ? d.w_fwd : d.w_dgrad);
  u16* out2 = (u16*)(d.kind == 0 ? d.w_dgrad : d.w_fwd);
  const int flip1 = d.kind == 0 ? 0 : d.flip, flip2 = d.kind == 0 ? d.flip : 0;
  for (int q = threadIdx.x; q < T * WPT * WPT; q += BLK) {
    const int t = q / (WPT * WPT), r = (q / WPT) % WPT, c = q % WPT;
    if (out1 && r < an && c < bn)
      out1[((size_t)(flip1 ? T - 1 - t : t) * A + a0 + r) * Bd + b0 + c] = f2bf(tile[t * TP + r * (WPT + 1) + c]);
    if (out2 && r < bn && c < an)
      out2[((size_t)(flip2 ? T - 1 - t : t) * Bd + b0 + r) * A + a0 + c] = f2bf(tile[t * TP + c * (WPT + 1) + r]);
  }
}

template <int MAP>
static void launch_igemm(const IG& g, int par_count, hipStream_t st) {
  // M_D2P: grid over the largest parity class (even rows, even columns)
  const int rows = MAP == M_D2P ? g.R.B * ((g.R.H + 1) / 2) * ((g.R.W + 1) / 2) : g.M;
  dim3 grid(cdivu(rows, TM), g.COUT / TN, par_count);
  if (g.flat) {
    grid.x *= grid.y;
    grid.y = 1;
  }
  hipLaunchKernelGGL((k_igemm<MAP>), grid, dim3(BLK), 0, st, g);
}

template <int MAP>
static void launch_wgrad(const WG& g, int chunks, hipStream_t st) {
  if (g.CI % 128 == 0 && g.CO % 128 == 0) {
    dim3 grid(chunks * wtaps_of<MAP>() * (g.CI / 128) * (g.CO / 128));
    hipLaunchKernelGGL((k_wgrad<MAP, 0>), grid, dim3(BLK), 0, st, g);
  } else {
    dim3 grid(chunks * wtaps_of<MAP>() * (g.CI / 64) * (g.CO / 64));
    hipLaunchKernelGGL((k_wgrad<MAP, 1>), grid, dim3(BLK), 0, st, g);
  }
}

static int wgrad_chunks(int M, int T, int ci, int co) {
  const int tc = (ci % 128 == 0 && co % 128 == 0) ? 128 : 64;
  const int per = T * (ci / tc) * (co / tc);
  const int slots = 3 * cu_count();
  const int step = slots / per > 0 ? slots / per : 1;
  int c = step;
  while ((M + c - 1) / c > 4096 && c < 1024) c += step;
  return c < 1024 ? c : 1024;
}

}  // namespace dn
}  // namespace rpc

using namespace rpc;
using namespace rpc::dn;

static inline Img img3(const int* d) { return Img{d[0], d[1], d[2]}; }

// elementwise BatchNorm passes: blocks of (256 / (C/8)) row lanes, ~2*RU rows per thread
// one contiguous chunk of RL * R rows per block (V = 1, 2)
static unsigned ew_chunks(long long m, int c, int R) {
  const long long rl = BLK / (c / 8 > 0 ? c / 8 : 1);
  const long long b = (m + rl * R - 1) / (rl * R);
  return (unsigned)(b < 1 ? 1 : (b > 2147483647LL ? 2147483647LL : b));
}
static unsigned ew_blocks(long long m, int c) {
  const long long rl = BLK / (c / 8 > 0 ? c / 8 : 1);
  long long b = (m + rl * 2 * RU - 1) / (rl * 2 * RU);
  return (unsigned)(b < 1 ? 1 : (b > 65535 ? 65535 : b));
}

// tuning knobs (rpc_dense_tune): 0 = S1 kernel for 128-multiple outputs (0: by shape, 1: k_conv3x3,
// 2: k_conv3x3w). By shape: k_conv3x3w (one 128-channel block per CU) when its blocks fill whole rounds
// of the CUs to >= 90 % (SECOND's 100x88 layers: 504 blocks = 0.98 of 2 rounds), else k_conv3x3 (two
// 64-channel blocks per CU overlap each other's prologue / epilogue; the 200x176 layers' 858 tiles are
// 0.84 of 4 rounds for either kernel, and there the register-staged kernel measured 3-8 % faster).
static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return v && *v ? atoi(v) : dflt;
}
// knob 9 / RPC_DENSE_EW: the row mapping of the BatchNorm elementwise passes — 0: each block one contiguous chunk
// of rows, all in flight at once (k_bn_apply 4 rows per thread, V = 1; k_bnbwd_apply 8, V = 2; default), 1: the
// former grid-stride batches (V = 0). Same bits either way (tools/ew_bench.py, profiles/r06_ew_rows_ab.txt:
// 200x176x6 x 128 bn_apply 17.9 -> 16.8 us, bnbwd_apply 27.2 -> 25.8 us)
static int g_ew_var = env_int("RPC_DENSE_EW", 0);
static int g_s1_variant = env_int("RPC_DENSE_S1", 0);   // A/B: RPC_DENSE_S1=<knob 0 value> for a whole run
// S1 weight gradient (knob 1 / RPC_DENSE_WGRAD): 0 = by shape (k_wgrad_s1c where ci % 64 == 0 and co % 128 == 0,
// else k_wgrad_s1 for 128-multiples, else k_wgrad), 1 = k_wgrad, 2 = k_wgrad_s1 without its read pipeline,
// 3 = k_wgrad_s1c, 4 = k_wgrad_s1 (r03-r05 default). r06: k_wgrad_s1c 0.88 vs k_wgrad_s1 1.00 ms per 3-class step
// (tools/s1wg_bench.py, profiles/r06_s1wg_ab.txt)
static int g_wgrad_variant = env_int("RPC_DENSE_WGRAD", 0);
static int g_s1x_dbg = 0;          // knob 4: k_conv3x3x timing experiments (0 = the real kernel)
static int g_y_split = env_int("RPC_DENSE_YSPLIT", 1);
static int g_y_zpf = env_int("RPC_DENSE_YZPF", 1);   // knob 10: k_conv3x3y<0, true> for fused BN-backward data gradients   // knob 8: k_conv3x3y split tail (C3::ysplit), 0 = off
static int g_ig_order = 0;        // implicit-GEMM grid: 0 = by shape (flat for 2 channel blocks), 1 = 2-D   // S1 weight gradient: 0 = k_wgrad_s1 (128-multiple channels), 1 = k_wgrad

// 128-multiple outputs, by shape: k_conv3x3y (two 4-wave 16x16 blocks per CU) when its grid is more than
// one round of the 2 x CUs block slots (SECOND's 200x176 layers: 858 / 1716 blocks; 128->128 73.6 -> 68.4,
// 128->256 130.0 -> 114.0 us vs k_conv3x3x), else k_conv3x3x (16x32 tiles, one 8-wave block per CU:
// 100x88 256->256, 504 16x16 blocks = 0.98 rounds: 59.8 -> 57.6 us) — profiles/r03_conv_bench_y1.log
static bool s1_ybig(const int* r_img, int cout) {
  const long long blocks = (long long)r_img[0] * ((r_img[1] + CT - 1) / CT) * ((r_img[2] + CT - 1) / CT) * (cout / 128);
  return blocks > 2LL * cu_count();
}
static bool s1_ytwo(const int* r_img, int cout) {
  return cout % 128 == 0 && (g_s1_variant == 4 || (g_s1_variant == 0 && s1_ybig(r_img, cout)));
}
// grids of at most half a round of the x kernel's one-block-per-CU slots (CenterPoint's 128x128 / 64x64 images at
// batch 4: 128 / 64 blocks) leave most CUs idle; there the 64-channel k_conv3x3 (two 4-wave blocks per CU, 4x
// the blocks) is used (CenterPoint 164.8 / 164.9 -> 166.5 / 166.4 frames/s with every S1 launch on it,
// profiles/r04_ab_centerpoint_s1.txt; the metric's SECOND shapes keep x / y: their smallest grid is 252 blocks)
static bool s1_small(const int* r_img, int cout) {
  const long long bx = (long long)r_img[0] * ((r_img[1] + CT - 1) / CT) * ((r_img[2] + XTW - 1) / XTW) * (cout / 128);
  return 2 * bx <= cu_count();
}
static bool s1_xwide(const int* r_img, int cout) {
  return cout % 128 == 0 && (g_s1_variant == 3 || (g_s1_variant == 0 && !s1_small(r_img, cout)));
}

// k_conv3x3 at 32 output channels per block when the 64-channel grid is less than one round of its two
// blocks per CU (knob 5 / RPC_DENSE_S1N32: 0 = by shape, 1 = never, 2 = always)
static int g_s1_n32 = env_int("RPC_DENSE_S1N32", 0);
// k_wgrad_s1c segment length (knob 6 / RPC_DENSE_S1C_SEG: 0 = by shape, else 32 / 64 / 96)
static int g_s1c_seg = env_int("RPC_DENSE_S1C_SEG", 0);
static int g_s1c_dbg = 0;   // knob 7: k_wgrad_s1c timing arms (0 = the real kernel)

// k_wgrad_s1c geometry: column strips of SEG pixels (the segment length with the least padding of an image row),
// tiles of 64 ci x 128 co, runs of steps sized so strips x tiles x runs fills one round of the CUs (one block per
// CU); the slabs it writes (runs x strips of [9][CI][CO]) are the workspace
struct S1cGeo {
  int seg, nstrip, nrun, steps_per;
};
static S1cGeo s1c_geometry(const Img& R, int ci, int co, int force_seg = 0) {
  S1cGeo q;
  // the segment (32 / 64 / 96 pixels) with the least padding of an image row, the longest on a tie (fewer
  // barriers per MFMA); knob 6 / RPC_DENSE_S1C_SEG forces one
  const int cand[3] = {96, 64, 32};
  q.seg = 96;
  int best = 1 << 30;
  for (int k = 0; k < 3; ++k) {
    const int pad = (R.W + cand[k] - 1) / cand[k] * cand[k] - R.W;
    if (pad < best) { best = pad; q.seg = cand[k]; }
  }
  if (g_s1c_seg == 32 || g_s1c_seg == 64 || g_s1c_seg == 96) q.seg = g_s1c_seg;
  if (force_seg) q.seg = force_seg;
  q.nstrip = (R.W + q.seg - 1) / q.seg;
  const int per = q.nstrip * (ci / 64) * (co / 128);
  const int nsteps = R.B * (R.H + 2);
  int nrun = cu_count() / per > 0 ? cu_count() / per : 1;
  nrun = nrun < nsteps ? nrun : nsteps;
  q.steps_per = (nsteps + nrun - 1) / nrun;
  q.nrun = (nsteps + q.steps_per - 1) / q.steps_per;
  return q;
}
static bool s1c_ok(int ci, int co) { return ci % 64 == 0 && co % 128 == 0; }

static bool s1_n32(int tiles, int cout) {
  if (g_s1_n32 == 1) return false;
  if (g_s1_n32 == 2) return true;
  return (long long)tiles * (cout / 64) < 2LL * cu_count();
}

static bool s1_wide(int tiles, int cout) {
  if (cout % 128 || g_s1_variant == 1) return false;
  if (g_s1_variant == 2) return true;
  const long long items = (long long)tiles * (cout / 128), cus = cu_count();
  const long long rounds = (items + cus - 1) / cus;
  return items * 10 >= rounds * cus * 9;
}

extern "C" int rpc_dense_tune(int knob, int value) {
  if (knob == 0) {
    const int old = g_s1_variant;
    if (value >= 0) g_s1_variant = value;
    return old;
  }
  if (knob == 1) {
    const int old = g_wgrad_variant;
    if (value >= 0) g_wgrad_variant = value;
    return old;
  }
  if (knob == 4) {
    const int old = g_s1x_dbg;
    if (value >= 0 && value <= 255) g_s1x_dbg = value;
    return old;
  }
  if (knob == 5) {
    const int old = g_s1_n32;
    if (value >= 0 && value <= 2) g_s1_n32 = value;
    return old;
  }
  if (knob == 7) {
    const int old = g_s1c_dbg;
    if (value >= 0) g_s1c_dbg = value;
    return old;
  }
  if (knob == 6) {
    const int old = g_s1c_seg;
    if (value >= 0) g_s1c_seg = value;
    return old;
  }
  if (knob == 10) {
    const int old = g_y_zpf;
    if (value == 0 || value == 1) g_y_zpf = value;
    return old;
  }
  if (knob == 8) {
    const int old = g_y_split;
    if (value == 0 || value == 1) g_y_split = value;
    return old;
  }
  if (knob == 9) {
    const int old = g_ew_var;
    if (value == 0 || value == 1) g_ew_var = value;
    return old;
  }
  if (knob == 2) {
    const int old = g_ig_order;
    if (value >= 0) g_ig_order = value;
    return old;
  }
  return RPC_ERR_ARG;
}

// the S1 kernels; bnz / bnp (k_conv3x3x / y only, checked by the caller): BatchNorm-backward partial sums
// of the layer the output gradient enters, instead of the output's own statistics
static int launch_s1(const IG& g, const u16* bnz, const float* bnp, hipStream_t st) {
  const int TY = (g.R.H + CT - 1) / CT, TX = (g.R.W + CT - 1) / CT;
  C3 c{g.src, g.SP, g.CIN, g.wt, g.COUT, g.out, g.OP, g.OOFF, g.accum, g.part, g.R.B, g.R.H, g.R.W, TY, TX,
       bnz, bnp, 0};
  const bool fits32 = (long long)g.M * g.SP * 2 < (1LL << 31) && 9LL * g.COUT * g.CIN * 2 < (1LL << 31);
  const int rimg[3] = {g.R.B, g.R.H, g.R.W};
  if (s1_ytwo(rimg, g.COUT) && fits32) {
    // the items past the last whole round of one block per CU (k_conv3x3y's time is a staircase in
    // ceil(items / CUs), profiles/r06_conv3x3y_tiles.txt) run as 64-channel halves when those fit one round
    const int items = g.R.B * TY * TX * (g.COUT / 128), tail = items % cu_count();
    c.ysplit = (g_y_split && g_s1x_dbg == 0 && items > cu_count() && 2 * tail <= cu_count()) ? tail : 0;
    const dim3 grid(items + c.ysplit);
    switch (g_s1x_dbg) {
      case 1: hipLaunchKernelGGL(k_conv3x3y<1>, grid, dim3(YB), 0, st, c); break;
      case 17: hipLaunchKernelGGL(k_conv3x3y<17>, grid, dim3(YB), 0, st, c); break;
      case 64: hipLaunchKernelGGL(k_conv3x3y<64>, grid, dim3(YB), 0, st, c); break;
      case 65: hipLaunchKernelGGL(k_conv3x3y<65>, grid, dim3(YB), 0, st, c); break;
      case 81: hipLaunchKernelGGL(k_conv3x3y<81>, grid, dim3(YB), 0, st, c); break;
      case 128: hipLaunchKernelGGL(k_conv3x3y<128>, grid, dim3(YB), 0, st, c); break;
      default:
        if (bnz != nullptr && g_y_zpf) hipLaunchKernelGGL((k_conv3x3y<0, true>), grid, dim3(YB), 0, st, c);
        else hipLaunchKernelGGL(k_conv3x3y<0>, grid, dim3(YB), 0, st, c);
    }
  } else if (s1_xwide(rimg, g.COUT)) {
    if (!fits32) return RPC_ERR_UNSUPPORTED;   // 32-bit buffer offsets (part rows are those of 16x32 tiles)
    c.TX = (g.R.W + XTW - 1) / XTW;
    const dim3 grid(g.R.B * TY * c.TX * (g.COUT / 128));
    switch (g_s1x_dbg) {
      case 1: hipLaunchKernelGGL(k_conv3x3x<1>, grid, dim3(WB), 0, st, c); break;
      case 3: hipLaunchKernelGGL(k_conv3x3x<3>, grid, dim3(WB), 0, st, c); break;
      case 12: hipLaunchKernelGGL(k_conv3x3x<12>, grid, dim3(WB), 0, st, c); break;
      case 13: hipLaunchKernelGGL(k_conv3x3x<13>, grid, dim3(WB), 0, st, c); break;
      case 30: hipLaunchKernelGGL(k_conv3x3x<30>, grid, dim3(WB), 0, st, c); break;
      case 31: hipLaunchKernelGGL(k_conv3x3x<31>, grid, dim3(WB), 0, st, c); break;
      case 32: hipLaunchKernelGGL(k_conv3x3x<32>, grid, dim3(WB), 0, st, c); break;
      case 128: hipLaunchKernelGGL(k_conv3x3x<128>, grid, dim3(WB), 0, st, c); break;
      default: hipLaunchKernelGGL(k_conv3x3x<0>, grid, dim3(WB), 0, st, c);
    }
  } else if (bnz != nullptr) {
    return RPC_ERR_UNSUPPORTED;
  } else if (s1_wide(g.R.B * TY * TX, g.COUT)) {
    hipLaunchKernelGGL(k_conv3x3w<0>, dim3(g.R.B * TY * TX * (g.COUT / 128)), dim3(WB), 0, st, c);
  } else if (s1_n32(g.R.B * TY * TX, g.COUT)) {
    hipLaunchKernelGGL((k_conv3x3<0, 32>), dim3(g.R.B * TY * TX, g.COUT / 32), dim3(CBLK), 0, st, c);
  } else {
    hipLaunchKernelGGL(k_conv3x3<0>, dim3(g.R.B * TY * TX, g.COUT / 64), dim3(CBLK), 0, st, c);
  }
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dense_conv(int map, const void* src, int sp, int cin, const void* wt, int cout, void* out, int op,
                              int ooff, int accum, float* part, const int* r_img, const int* s_img,
                              const int* o_img, void* stream) {
  if (map < M_S1 || map > M_G2 || !src || !wt || !out || !r_img || !s_img || !o_img) return RPC_ERR_ARG;
  // S1 takes any multiple of 64 output channels (64-channel blocks when not a multiple of 128)
  if (cin % BK || (map == M_S1 ? cout % 64 : cout % TN) || sp < cin || op < ooff + cout || (sp & 7) || (op & 7) ||
      (ooff & 7))
    return RPC_ERR_ARG;
  IG g{(const u16*)src, sp, cin, (const u16*)wt, cout, (u16*)out, op, ooff, accum, part,
       img3(r_img), img3(s_img), img3(o_img), 0};
  g.M = g.R.B * g.R.H * g.R.W;
  // flat grid for two channel blocks (P1 128->256, U2, G2, S2: 3-7 % faster); four adjacent blocks
  // of one tile (the head's 128->512 data gradient) measured 10 % slower than the 2-D order
  g.flat = g_ig_order == 0 && cout / TN == 2;
  if (g.M == 0) return RPC_OK;
  hipStream_t st = (hipStream_t)stream;
  if (map == M_S1) return launch_s1(g, nullptr, nullptr, st);
  switch (map) {
    case M_S1: launch_igemm<M_S1>(g, 1, st); break;
    case M_S2: launch_igemm<M_S2>(g, 1, st); break;
    case M_D2:   // BatchNorm partials need the row-tile layout of rpc_dense_conv_blocks: 9-tap form
      if (g.part) launch_igemm<M_D2>(g, 1, st);
      else launch_igemm<M_D2P>(g, 4, st);
      break;
    case M_P1: launch_igemm<M_P1>(g, 1, st); break;
    case M_U2: launch_igemm<M_U2>(g, 4, st); break;
    default: launch_igemm<M_G2>(g, 1, st); break;
  }
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

// S1 data gradient whose output dh enters a BatchNorm + ReLU layer: also that layer's BatchNorm-backward
// partial sums (replaces rpc_dense_bnbwd_stats for it; part: [rpc_dense_conv_part_rows][2*cout])
extern "C" int rpc_dense_conv_bnbwd(const void* src, int sp, int cin, const void* wt, int cout, void* out, int op,
                                    const void* bnz, const float* bnp, float* part, const int* r_img, void* stream) {
  if (!src || !wt || !out || !r_img || !bnz || !bnp || !part) return RPC_ERR_ARG;
  if (cin % BK || cout % 128 || sp < cin || op < cout || (sp & 7) || (op & 7)) return RPC_ERR_ARG;
  if (!s1_ytwo(r_img, cout) && !s1_xwide(r_img, cout)) return RPC_ERR_UNSUPPORTED;
  IG g{(const u16*)src, sp, cin, (const u16*)wt, cout, (u16*)out, op, 0, 0, part, img3(r_img), img3(r_img),
       img3(r_img), 0};
  g.M = g.R.B * g.R.H * g.R.W;
  if ((long long)g.M * g.SP * 2 >= (1LL << 31) || 9LL * g.COUT * g.CIN * 2 >= (1LL << 31)) return RPC_ERR_UNSUPPORTED;
  if (g.M == 0) return RPC_OK;
  return launch_s1(g, (const u16*)bnz, bnp, (hipStream_t)stream);
}

extern "C" int rpc_dense_conv_s1_kernel(int map, int cout, const int* r_img) {
  if (map != M_S1 || !r_img || cout % 64) return -1;
  const int TY = (r_img[1] + CT - 1) / CT, TX = (r_img[2] + CT - 1) / CT;
  if (s1_ytwo(r_img, cout)) return 3;
  if (s1_xwide(r_img, cout)) return 2;
  return s1_wide(r_img[0] * TY * TX, cout) ? 1 : 0;
}

extern "C" int rpc_dense_conv_part_rows(int map, int cout, const int* r_img) {
  if (!r_img || map < M_S1 || map > M_G2) return -1;
  if (map == M_S1 && !s1_ytwo(r_img, cout) && s1_xwide(r_img, cout))   // one row per 16x32 tile
    return r_img[0] * ((r_img[1] + CT - 1) / CT) * ((r_img[2] + XTW - 1) / XTW);
  return rpc_dense_conv_blocks(map, r_img);
}

extern "C" int rpc_dense_conv_blocks(int map, const int* r_img) {
  if (map == M_S1) return r_img[0] * ((r_img[1] + CT - 1) / CT) * ((r_img[2] + CT - 1) / CT);
  const long long M = (long long)r_img[0] * r_img[1] * r_img[2];
  return (int)((M + TM - 1) / TM) * (map == M_U2 ? 4 : 1);
}

extern "C" size_t rpc_dense_wgrad_workspace_size(int map, const int* r_img, int ci, int co) {
  const int M = r_img[0] * r_img[1] * r_img[2];
  const int T = map_wtaps(map);
  size_t n = (size_t)wgrad_chunks(M, T, ci, co);
  if (map == M_S1 && s1c_ok(ci, co)) {   // any S1 kernel and segment (knobs 1 / 6 may switch between launches)
    for (int seg = 32; seg <= 96; seg += 32) {
      const S1cGeo q = s1c_geometry(img3(r_img), ci, co, seg);
      const size_t c = (size_t)q.nrun * q.nstrip;
      n = c > n ? c : n;
    }
  }
  return n * T * ci * co * sizeof(float);
}

extern "C" int rpc_dense_wgrad(int map, int kind, const void* x, int xp, int ci, const void* dz, int dp, int co,
                               const int* r_img, const int* s_img, const int* o_img, float* dW, void* ws,
                               size_t ws_bytes, void* stream) {
  if (map < M_S1 || map > M_G2 || map == M_D2 || map == M_G2) return RPC_ERR_ARG;
  if (ci % 64 || co % 64 || (xp & 7) || (dp & 7)) return RPC_ERR_ARG;
  Img R = img3(r_img), S = img3(s_img), O = img3(o_img);
  const int M = R.B * R.H * R.W, T = map_wtaps(map);
  const int chunks = wgrad_chunks(M, T, ci, co);
  const size_t slab = (size_t)T * ci * co;
  if (ws_bytes < chunks * slab * sizeof(float)) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  float* part = (float*)ws;
  if (M == 0) {
    RPC_CHECK(hipMemsetAsync(dW, 0, slab * sizeof(float), st));
    return RPC_OK;
  }
  const int rows_per = ((M + chunks - 1) / chunks + 63) / 64 * 64;
  WG g{(const u16*)x, xp, (const u16*)dz, dp, ci, co, R, S, O, M, rows_per, part};
  int nred = chunks;
  if (map == M_S1 && s1c_ok(ci, co) && (g_wgrad_variant == 0 || g_wgrad_variant == 3)) {
    // column walk, all 9 taps per block
    const S1cGeo q = s1c_geometry(R, ci, co);
    nred = q.nrun * q.nstrip;
    if (ws_bytes < (size_t)nred * slab * sizeof(float)) return RPC_ERR_WORKSPACE;
    if ((size_t)M * (xp > dp ? xp : dp) >= (1ULL << 31)) return RPC_ERR_UNSUPPORTED;   // 32-bit lane offsets
    const dim3 grid(q.nrun * q.nstrip * (ci / 64) * (co / 128));
    if (q.seg == 96) {
      switch (g_s1c_dbg) {
        case 1: hipLaunchKernelGGL((k_wgrad_s1c<96, 1>), grid, dim3(WSB), 0, st, g, q.nstrip, q.steps_per); break;
        case 3: hipLaunchKernelGGL((k_wgrad_s1c<96, 3>), grid, dim3(WSB), 0, st, g, q.nstrip, q.steps_per); break;
        case 7: hipLaunchKernelGGL((k_wgrad_s1c<96, 7>), grid, dim3(WSB), 0, st, g, q.nstrip, q.steps_per); break;
        case 5: hipLaunchKernelGGL((k_wgrad_s1c<96, 5>), grid, dim3(WSB), 0, st, g, q.nstrip, q.steps_per); break;
        case 8: hipLaunchKernelGGL((k_wgrad_s1c<96, 8>), grid, dim3(WSB), 0, st, g, q.nstrip, q.steps_per); break;
        default: hipLaunchKernelGGL((k_wgrad_s1c<96>), grid, dim3(WSB), 0, st, g, q.nstrip, q.steps_per);
      }
    } else if (q.seg == 64) hipLaunchKernelGGL(k_wgrad_s1c<64>, grid, dim3(WSB), 0, st, g, q.nstrip, q.steps_per);
    else hipLaunchKernelGGL(k_wgrad_s1c<32>, grid, dim3(WSB), 0, st, g, q.nstrip, q.steps_per);
  } else if (map == M_S1 && ci % 128 == 0 && co % 128 == 0 &&
             (g_wgrad_variant == 0 || g_wgrad_variant == 2 || g_wgrad_variant == 4)) {
    // tap-sharing row-segment kernel: segment length with the least padding of the image row
    const int seg = (R.W + 63) / 64 * 64 <= (R.W + 31) / 32 * 32 ? 64 : 32;
    const int nsx = (R.W + seg - 1) / seg, nseg = R.B * R.H * nsx;
    const int seg_per = (nseg + chunks - 1) / chunks;
    const dim3 grid(chunks * 3 * (ci / 128) * (co / 128));
    // knob 1 = 2: the former loop (each sub-step's 20 transposed reads, then its 24 MFMAs); the default
    // issues the next sub-step's reads first (bit-identical; 200x176 128->128 91.3 -> 90.7 us, 100x88
    // 256->256 94.8 -> 90.9, 128->256 153.4 -> 150.2, profiles/r03_wgrad_pipe.log)
    const bool pipe = g_wgrad_variant != 2;
    if (seg == 64 && pipe) hipLaunchKernelGGL((k_wgrad_s1<64, 1>), grid, dim3(WSB), 0, st, g, nsx, seg_per);
    else if (seg == 64) hipLaunchKernelGGL((k_wgrad_s1<64, 0>), grid, dim3(WSB), 0, st, g, nsx, seg_per);
    else if (pipe) hipLaunchKernelGGL((k_wgrad_s1<32, 1>), grid, dim3(WSB), 0, st, g, nsx, seg_per);
    else hipLaunchKernelGGL((k_wgrad_s1<32, 0>), grid, dim3(WSB), 0, st, g, nsx, seg_per);
  } else switch (map) {
    case M_S1: launch_wgrad<M_S1>(g, chunks, st); break;
    case M_S2: launch_wgrad<M_S2>(g, chunks, st); break;
    case M_P1: launch_wgrad<M_P1>(g, chunks, st); break;
    default: launch_wgrad<M_U2>(g, chunks, st); break;
  }
  RPC_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_wgrad_reduce<0>, dim3(cdivu(slab, 64)), dim3(256), 0, st, (const float*)part, nred, kind, ci, co,
                     T, dW);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

template <typename E>
static int bn_apply(const void* z, int m, int c, const float* bn, void* out, int op, int ooff, void* stream) {
  if (m < 0 || c < 8 || c > 2048 || (c & 7) || (op & 7) || (ooff & 7) || op < ooff + c) return RPC_ERR_ARG;
  if (m == 0) return RPC_OK;
  const hipStream_t st = (hipStream_t)stream;
  if (g_ew_var == 1)
    hipLaunchKernelGGL((k_bn_apply<E, 0>), dim3(ew_blocks(m, c)), dim3(BLK), 0, st, (const E*)z, m, c, bn, (E*)out,
                       op, ooff);
  else
    hipLaunchKernelGGL((k_bn_apply<E, 1>), dim3(ew_chunks(m, c, RU)), dim3(BLK), 0, st, (const E*)z, m, c, bn, (E*)out,
                       op, ooff);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

template <typename E, typename A>
static int bnbwd_stats(const void* dh, int dp, int doff, const void* z, int m, int c, const float* bn, A* part,
                       void* stream) {
  if (m < 0 || c < 8 || c > 2048 || (c & 7) || (dp & 7) || (doff & 7)) return RPC_ERR_ARG;
  const int nb = rpc_dense_bnbwd_blocks(m);
  hipLaunchKernelGGL((k_bnbwd_stats<E, A>), dim3(nb), dim3(BLK), 0, (hipStream_t)stream, (const E*)dh, dp, doff,
                     (const E*)z, m, c, bn, part);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

template <typename E>
static int bnbwd_apply(const void* dh, int dp, int doff, const void* z, int m, int c, const float* bn,
                       const float* bnb, void* dz, void* stream) {
  if (m < 0 || c < 8 || c > 2048 || (c & 7) || (dp & 7) || (doff & 7)) return RPC_ERR_ARG;
  if (m == 0) return RPC_OK;
  const hipStream_t st = (hipStream_t)stream;
  if (g_ew_var == 1)
    hipLaunchKernelGGL((k_bnbwd_apply<E, 0>), dim3(ew_blocks(m, c)), dim3(BLK), 0, st, (const E*)dh, dp, doff,
                       (const E*)z, m, c, bn, bnb, (E*)dz);
  else
    hipLaunchKernelGGL((k_bnbwd_apply<E, 2>), dim3(ew_chunks(m, c, 8)), dim3(BLK), 0, st, (const E*)dh, dp, doff,
                       (const E*)z, m, c, bn, bnb, (E*)dz);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dense_bnbwd_blocks(int m) {
  int b = (m + 255) / 256;   // ~16-32 rows per thread: enough blocks to fill the chip
  return b < 1 ? 1 : (b > 2048 ? 2048 : b);
}

extern "C" int rpc_dense_bn_apply(const void* z, int m, int c, const float* bn, void* out, int op, int ooff,
                                  void* stream) {
  return bn_apply<u16>(z, m, c, bn, out, op, ooff, stream);
}
extern "C" int rpc_dense_bn_apply_f32(const float* z, int m, int c, const float* bn, float* out, int op, int ooff,
                                      void* stream) {
  return bn_apply<float>(z, m, c, bn, out, op, ooff, stream);
}
extern "C" int rpc_dense_bnbwd_stats(const void* dh, int dp, int doff, const void* z, int m, int c, const float* bn,
                                     float* part, void* stream) {
  return bnbwd_stats<u16, float>(dh, dp, doff, z, m, c, bn, part, stream);
}
extern "C" int rpc_dense_bnbwd_stats_f32(const float* dh, int dp, int doff, const float* z, int m, int c,
                                         const float* bn, double* part, void* stream) {
  return bnbwd_stats<float, double>(dh, dp, doff, z, m, c, bn, part, stream);
}
extern "C" int rpc_dense_bnbwd_apply(const void* dh, int dp, int doff, const void* z, int m, int c, const float* bn,
                                     const float* bnb, void* dz, void* stream) {
  return bnbwd_apply<u16>(dh, dp, doff, z, m, c, bn, bnb, dz, stream);
}
extern "C" int rpc_dense_bnbwd_apply_f32(const float* dh, int dp, int doff, const float* z, int m, int c,
                                         const float* bn, const float* bnb, float* dz, void* stream) {
  return bnbwd_apply<float>(dh, dp, doff, z, m, c, bn, bnb, dz, stream);
}

extern "C" int rpc_dense_wprep_batch(const RpcDenseWprep* descs, int n, void* stream) {
  if (n < 0 || n > WPREP_MAX || (n > 0 && !descs)) return RPC_ERR_ARG;
  if (n == 0) return RPC_OK;
  WprepBatch b;
  memset(&b, 0, sizeof(b));
  long long most = 0;
  for (int i = 0; i < n; ++i) {
    const RpcDenseWprep& d = descs[i];
    if (!d.W || d.ci < 1 || d.co < 1 || d.taps < 1 || d.taps > WPT_MAXT || (d.kind != 0 && d.kind != 1) ||
        d.co_src < 0 || d.co_src > d.co || (d.co_src && d.kind != 0))
      return RPC_ERR_ARG;
    b.d[i] = d;
    const long long e = (long long)((d.ci + WPT - 1) / WPT) * ((d.co + WPT - 1) / WPT);
    most = e > most ? e : most;
  }
  hipLaunchKernelGGL(k_wprep_batch, dim3((unsigned)most, n), dim3(BLK), 0, (hipStream_t)stream, b);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dense_wprep(const float* W, int kind, int ci, int co, int taps, int flip, void* wf, void* wd,
                               void* stream) {
  if (!W || ci < 1 || co < 1 || taps < 1 || (kind != 0 && kind != 1)) return RPC_ERR_ARG;
  const long long n = (long long)taps * ci * co;
  hipLaunchKernelGGL(k_wprep, dim3(cdivu(n, BLK)), dim3(BLK), 0, (hipStream_t)stream, W, kind, ci, co, taps, flip,
                     (u16*)wf, (u16*)wd);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
