// §8(f3): the deformable convolutions of the CenterPoint DCNSeparateHead, for gfx950.
//
// mmcv DeformConv2dPack as built by the CenterHead base of
// configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py:11-13 (separate_head = DCNSeparateHead,
// dcn_config = DCN(64 -> 64, kernel 3, padding 1, groups 4), deform_groups 1): for output pixel p and
// tap k = (i, j) the input is sampled bilinearly at (y - 1 + i + dy_k, x - 1 + j + dx_k), with the
// offsets (dy_k, dx_k) = channels (2k, 2k+1) of the offset convolution (its bias added here); a sample
// point outside (-1, H) x (-1, W) reads 0, corners outside the image read 0 (mmcv
// deformable_im2col_bilinear). Output channel co uses input channels of its group (16 each).
//
// Tiles are 8 x 8 output pixels. The 12 x 12 input window every |offset| < 1 sample of the tile can
// touch is staged in LDS once (bf16, 64 channels); corners outside it are read from global memory.
//   forward:  per tap, 256 threads sample the tile's 64 x 64 column block into LDS (thread = pixel x
//             group), 4 waves multiply it by the tap's block-diagonal 64 x 64 weight (bf16 MFMA
//             16x16x32, fp32 accumulate over the 9 taps), bf16 output image.
//   backward: per tap, the same sampling, dcol = dOut x W_k (MFMA), dW_k's four diagonal 16 x 16
//             blocks = dOut^T x col (one wave per group, MFMA over the 64 pixels), the offset
//             gradient per (pixel, group) thread (mmcv get_coordinate_weight), and the input
//             gradient as a GEMM: dx_window += S_k x dcol_k with S_k the [144 x 64] bilinear-weight
//             matrix of the in-window corners (corners outside: global atomics); the window goes to
//             a per-tile slab and k_gather_dx sums, per pixel, the (at most 4) covering slabs in a
//             fixed order.
#include <hip/hip_runtime.h>
#include <math.h>

#include "common.h"

namespace rpc {
namespace dcn {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
typedef unsigned short u16;

constexpr int BLK = 256;
constexpr int C = 64;          // channels in and out
constexpr int CG = 16;         // channels per group
constexpr int KT = 9;          // taps
constexpr int TE = 8;          // output tile edge
constexpr int WE = TE + 4;     // input window edge (covers floor(y - 1 + i + dy) .. +1 for |dy| < 1)
constexpr int WR = WE * WE;    // window pixels (144)
constexpr int PW = C + 8;      // window LDS pitch (elements)
constexpr int P = C + 16;      // tile LDS pitch (elements, conflict-free transposed reads)
// backward partial row per tile: dW diagonal blocks (KT * 1024), the offset-bias gradient (2 * KT), padded to 64 bytes
// (the rows, the reduced row and the window slabs after them stay 16-byte aligned for the vector stores)
constexpr int PWR = KT * 1024 + 32;
static_assert(2 * KT <= 32, "offset-bias gradient fits the row padding");

__device__ __forceinline__ u16 f2bf(float f) { return __builtin_bit_cast(u16, (__bf16)f); }
__device__ __forceinline__ float bf2f(u16 h) { return __uint_as_float((unsigned)h << 16); }
__device__ __forceinline__ s16x4 tr_read(const u16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

struct Geo {
  int B, H, W, TY, TX;
};

struct Tile {
  int b, y0, x0;
};

__device__ __forceinline__ Tile tile_of(const Geo& g, int t) {
  const int b = t / (g.TY * g.TX), r = t - b * g.TY * g.TX;
  return Tile{b, (r / g.TX) * TE, (r % g.TX) * TE};
}

// stage the 12 x 12 x 64 input window (zero outside the image)
__device__ __forceinline__ void stage_window(const Geo& g, const Tile& tl, const u16* __restrict__ x, int xp,
                                             u16* sXw) {
  for (int q = threadIdx.x; q < WR * 8; q += BLK) {
    const int wp = q >> 3, seg = q & 7;
    const int hy = tl.y0 - 2 + wp / WE, hx = tl.x0 - 2 + wp % WE;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (hy >= 0 && hy < g.H && hx >= 0 && hx < g.W)
      v = *(const uint4*)(x + ((size_t)(tl.b * g.H + hy) * g.W + hx) * xp + seg * 8);
    *(uint4*)&sXw[wp * PW + seg * 8] = v;
  }
}

// the 16 channels [16q, 16q+16) of input pixel (cy, cx) (caller checks the image bounds)
__device__ __forceinline__ void fetch16(const Geo& g, const Tile& tl, const u16* __restrict__ x, int xp,
                                        const u16* sXw, int cy, int cx, int q, float* v) {
  const int wy = cy - (tl.y0 - 2), wx = cx - (tl.x0 - 2);
  uint4 a, b;
  if (wy >= 0 && wy < WE && wx >= 0 && wx < WE) {
    const u16* p = sXw + (wy * WE + wx) * PW + q * CG;
    a = *(const uint4*)p;
    b = *(const uint4*)(p + 8);
  } else {
    const u16* p = x + ((size_t)(tl.b * g.H + cy) * g.W + cx) * xp + q * CG;
    a = *(const uint4*)p;
    b = *(const uint4*)(p + 8);
  }
  const unsigned w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// sample geometry of (pixel, tap): mmcv deformable_im2col_bilinear / get_coordinate_weight
struct Samp {
  int valid, hl, wl;
  float lh, lw, hh, hw;
  int c1, c2, c3, c4;
};

__device__ __forceinline__ Samp samp(const Geo& g, int y, int x, int k, float dy, float dx) {
  Samp s;
  const float ph = (float)(y - 1 + k / 3) + dy, pw = (float)(x - 1 + k % 3) + dx;
  s.valid = ph > -1.0f && pw > -1.0f && ph < (float)g.H && pw < (float)g.W;
  const float fh = floorf(ph), fw = floorf(pw);
  s.hl = (int)fh;
  s.wl = (int)fw;
  s.lh = ph - fh;
  s.lw = pw - fw;
  s.hh = 1.0f - s.lh;
  s.hw = 1.0f - s.lw;
  s.c1 = s.hl >= 0 && s.wl >= 0;
  s.c2 = s.hl >= 0 && s.wl + 1 <= g.W - 1;
  s.c3 = s.hl + 1 <= g.H - 1 && s.wl >= 0;
  s.c4 = s.hl + 1 <= g.H - 1 && s.wl + 1 <= g.W - 1;
  return s;
}

__device__ __forceinline__ void offsets(const u16* __restrict__ off, int offp, const float* __restrict__ ob,
                                        size_t pix, int k, float* dy, float* dx) {
  *dy = bf2f(off[pix * offp + 2 * k]) + ob[2 * k];
  *dx = bf2f(off[pix * offp + 2 * k + 1]) + ob[2 * k + 1];
}

// col values of one (pixel, tap, group): bilinear of the four corners
__device__ __forceinline__ void sample16(const Geo& g, const Tile& tl, const u16* __restrict__ x, int xp,
                                         const u16* sXw, const Samp& s, int q, float* col) {
#pragma unroll
  for (int c = 0; c < CG; ++c) col[c] = 0.0f;
  if (!s.valid) return;
  float v[CG];
  const float w1 = s.hh * s.hw, w2 = s.hh * s.lw, w3 = s.lh * s.hw, w4 = s.lh * s.lw;
  if (s.c1) {
    fetch16(g, tl, x, xp, sXw, s.hl, s.wl, q, v);
#pragma unroll
    for (int c = 0; c < CG; ++c) col[c] = w1 * v[c];
  }
  if (s.c2) {
    fetch16(g, tl, x, xp, sXw, s.hl, s.wl + 1, q, v);
#pragma unroll
    for (int c = 0; c < CG; ++c) col[c] += w2 * v[c];
  }
  if (s.c3) {
    fetch16(g, tl, x, xp, sXw, s.hl + 1, s.wl, q, v);
#pragma unroll
    for (int c = 0; c < CG; ++c) col[c] += w3 * v[c];
  }
  if (s.c4) {
    fetch16(g, tl, x, xp, sXw, s.hl + 1, s.wl + 1, q, v);
#pragma unroll
    for (int c = 0; c < CG; ++c) col[c] += w4 * v[c];
  }
}

__device__ __forceinline__ void store_col(u16* sC, int p, int q, const float* col) {
  uint4 a, b;
  a.x = f2bf(col[0]) | ((unsigned)f2bf(col[1]) << 16);
  a.y = f2bf(col[2]) | ((unsigned)f2bf(col[3]) << 16);
  a.z = f2bf(col[4]) | ((unsigned)f2bf(col[5]) << 16);
  a.w = f2bf(col[6]) | ((unsigned)f2bf(col[7]) << 16);
  b.x = f2bf(col[8]) | ((unsigned)f2bf(col[9]) << 16);
  b.y = f2bf(col[10]) | ((unsigned)f2bf(col[11]) << 16);
  b.z = f2bf(col[12]) | ((unsigned)f2bf(col[13]) << 16);
  b.w = f2bf(col[14]) | ((unsigned)f2bf(col[15]) << 16);
  *(uint4*)&sC[p * P + q * CG] = a;
  *(uint4*)&sC[p * P + q * CG + 8] = b;
}

// weights: W [64 co][16 ci_l][3][3] fp32 -> wf [9][64 co][64 ci] and wd [9][64 ci][64 co], bf16,
// zero outside the diagonal group blocks
__global__ __launch_bounds__(BLK) void k_prep(const float* __restrict__ W, u16* __restrict__ wf, u16* __restrict__ wd) {
  const int e = blockIdx.x * BLK + threadIdx.x;
  if (e >= KT * C * C) return;
  const int k = e / (C * C), r = e - k * C * C, a = r / C, bb = r - a * C;
  // wf[k][co=a][ci=bb]
  {
    const int co = a, ci = bb;
    const float v = (co / CG == ci / CG) ? W[(co * CG + (ci % CG)) * KT + k] : 0.0f;
    wf[e] = f2bf(v);
  }
  // wd[k][ci=a][co=bb]
  {
    const int ci = a, co = bb;
    const float v = (co / CG == ci / CG) ? W[(co * CG + (ci % CG)) * KT + k] : 0.0f;
    wd[e] = f2bf(v);
  }
}

__global__ __launch_bounds__(BLK) void k_fwd(Geo g, const u16* __restrict__ x, int xp, const u16* __restrict__ off,
                                             int offp, const float* __restrict__ ob, const u16* __restrict__ wf,
                                             u16* __restrict__ out, int op) {
  __shared__ __attribute__((aligned(16))) u16 sXw[WR * PW];
  __shared__ __attribute__((aligned(16))) u16 sC[64 * P];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const Tile tl = tile_of(g, blockIdx.x);
  stage_window(g, tl, x, xp, sXw);
  const int p = tid >> 2, q = tid & 3;
  const int y = tl.y0 + (p >> 3), xx = tl.x0 + (p & 7);
  const size_t pix = (size_t)(tl.b * g.H + y) * g.W + xx;
  f32x4 acc[4];
#pragma unroll
  for (int n = 0; n < 4; ++n) acc[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  for (int k = 0; k < KT; ++k) {
    float dy, dx, col[CG];
    offsets(off, offp, ob, pix, k, &dy, &dx);
    const Samp s = samp(g, y, xx, k, dy, dx);
    sample16(g, tl, x, xp, sXw, s, q, col);
    store_col(sC, p, q, col);
    __syncthreads();
    const u16* wk = wf + (size_t)k * C * C;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 a = *(const bf16x8*)&sC[(16 * w + (lane & 15)) * P + 32 * ks + 8 * (lane >> 4)];
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const bf16x8 bv = *(const bf16x8*)&wk[(n * 16 + (lane & 15)) * C + 32 * ks + 8 * (lane >> 4)];
        acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bv, acc[n], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // D[px = 16w + 4*(lane>>4) + r][co = 16n + (lane&15)] -> LDS -> 16-B stores
#pragma unroll
  for (int n = 0; n < 4; ++n)
#pragma unroll
    for (int r = 0; r < 4; ++r) sC[(16 * w + 4 * (lane >> 4) + r) * P + 16 * n + (lane & 15)] = f2bf(acc[n][r]);
  __syncthreads();
  for (int qd = tid; qd < 64 * 8; qd += BLK) {
    const int pp = qd >> 3, seg = qd & 7;
    const int yy = tl.y0 + (pp >> 3), xw = tl.x0 + (pp & 7);
    *(uint4*)(out + ((size_t)(tl.b * g.H + yy) * g.W + xw) * op + seg * 8) = *(const uint4*)&sC[pp * P + seg * 8];
  }
}

// Input-gradient scatter as a GEMM: per tap, S_k [144 window pixels][64 tile pixels] holds the
// bilinear weight of every in-window corner (4 per sampled pixel), and dx_window += S_k x dcol_k
// (bf16 MFMA, fp32 accumulators held in registers across the taps: 9 16x16 tiles per wave).
// LDS 76 KB, two blocks per CU (r04; was 118 KB, one 4-wave block per CU: 157 -> 101 us per CenterPoint
// launch, profiles/r04_step_kernels_centerpoint_v4.txt): one S buffer (a thread clears its tap k-1 entry
// in phase A and sets its tap k entry after the A/B barrier), the offset gradients stored to the image per
// tap (no [64][18] staging) with the bias partials reduced per wave by shuffles, and the offset gradient's
// dcol read from the bf16 dcol^T tile of phase D (the fp32 copy is gone)
constexpr int PS = 64 + 8;     // S row pitch (elements)

__global__ __launch_bounds__(BLK) void k_bwd(Geo g, const u16* __restrict__ x, int xp, const u16* __restrict__ off,
                                             int offp, const float* __restrict__ ob, const u16* __restrict__ wd,
                                             const u16* __restrict__ dout, int dop, float* __restrict__ dx,
                                             u16* __restrict__ doff, int doffp, int dch, float* __restrict__ pw_part,
                                             float* __restrict__ pb_part, float* __restrict__ win_part) {
  __shared__ __attribute__((aligned(16))) u16 sXw[WR * PW];
  __shared__ __attribute__((aligned(16))) u16 sDo[64 * P];
  __shared__ __attribute__((aligned(16))) u16 sC[64 * P];
  __shared__ __attribute__((aligned(16))) u16 sDcT[64 * PS];    // dcol^T [channel][pixel], bf16
  __shared__ __attribute__((aligned(16))) u16 sS[WR * PS];       // S_k (one buffer: cleared in A, set in B)
  __shared__ float sOin[64 * 2 * KT];     // offsets (+ bias) of the tile, all taps
  __shared__ float sPb[4 * 2 * KT];       // offset-bias gradient partials per wave
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const Tile tl = tile_of(g, blockIdx.x);
  stage_window(g, tl, x, xp, sXw);
  for (int qd = tid; qd < 64 * 8; qd += BLK) {
    const int pp = qd >> 3, seg = qd & 7;
    const int yy = tl.y0 + (pp >> 3), xw = tl.x0 + (pp & 7);
    const size_t pix = (size_t)(tl.b * g.H + yy) * g.W + xw;
    *(uint4*)&sDo[pp * P + seg * 8] = *(const uint4*)(dout + pix * dop + seg * 8);
  }
  for (int i = tid; i < 64 * 2 * KT; i += BLK) {
    const int pp = i / (2 * KT), c = i - pp * 2 * KT;
    const int yy = tl.y0 + (pp >> 3), xw = tl.x0 + (pp & 7);
    sOin[i] = bf2f(off[((size_t)(tl.b * g.H + yy) * g.W + xw) * offp + c]) + ob[c];
  }
  for (int i = tid; i < WR * PS / 8; i += BLK) ((uint4*)sS)[i] = make_uint4(0u, 0u, 0u, 0u);
  const size_t mypix = (size_t)(tl.b * g.H + tl.y0 + ((tid >> 2) >> 3)) * g.W + tl.x0 + ((tid >> 2) & 7);
  const int p = tid >> 2, q = tid & 3;
  const int y = tl.y0 + (p >> 3), xx = tl.x0 + (p & 7);
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp4 = lane & 3, rowoff = 4 * g4 + qq;
  // B fragments of dcol = dOut x W_k (W_k as [ci][co]) for the current tap, prefetched one tap ahead
  bf16x8 bw[2][4];
  auto load_b = [&](int k) {
    const u16* wk = wd + (size_t)k * C * C;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int n = 0; n < 4; ++n) bw[ks][n] = *(const bf16x8*)&wk[(n * 16 + (lane & 15)) * C + 32 * ks + 8 * (lane >> 4)];
  };
  load_b(0);
  // dx window accumulators: wave w owns window rows 16*(w + 4*i) .. (i < 3, 9 row tiles over 4 waves),
  // all 64 channels (4 column tiles)
  f32x4 acc[3][4];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[i][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int prev_u = -1;                        // this thread's S entry of the previous tap
  __syncthreads();
#pragma unroll 1
  for (int k = 0; k < KT; ++k) {
    u16* S = sS;
    // A: sample the column block of tap k (thread = pixel x group); thread q also owns corner q of
    // its pixel: it clears its S entry of tap k-1 here (read by tap k-1's phase D before the last
    // barrier) and writes the new bilinear weight in phase B (after every thread's clear)
    const Samp s = samp(g, y, xx, k, sOin[p * 2 * KT + 2 * k], sOin[p * 2 * KT + 2 * k + 1]);
    int new_u = -1;
    u16 new_w = 0;
    {
      float col[CG];
      sample16(g, tl, x, xp, sXw, s, q, col);
      store_col(sC, p, q, col);
      if (prev_u >= 0) S[prev_u * PS + p] = 0;
      prev_u = -1;
      const int cok = q == 0 ? s.c1 : (q == 1 ? s.c2 : (q == 2 ? s.c3 : s.c4));
      if (s.valid && cok) {
        const float wq = q == 0 ? s.hh * s.hw : (q == 1 ? s.hh * s.lw : (q == 2 ? s.lh * s.hw : s.lh * s.lw));
        const int cy = s.hl + (q >> 1), cx = s.wl + (q & 1);
        const int wy = cy - (tl.y0 - 2), wx = cx - (tl.x0 - 2);
        if (wy >= 0 && wy < WE && wx >= 0 && wx < WE) {
          new_u = wy * WE + wx;
          new_w = f2bf(wq);
        } else {
          prev_u = -2 - (cy * 65536 + cx);   // out-of-window corner: global atomics after dcol
        }
      }
    }
    __syncthreads();
    if (new_u >= 0) {
      S[new_u * PS + p] = new_w;
      prev_u = new_u;
    }
    // B: dW_k diagonal block of group w (dOut^T col over the tile) and dcol (wave w: pixels 16w..)
    {
      f32x4 aw = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int r0 = 32 * ks + rowoff, c = w * CG + 4 * pp4;
        s16x4 va[2] = {tr_read(&sDo[r0 * P + c]), tr_read(&sDo[(r0 + 16) * P + c])};
        s16x4 vb[2] = {tr_read(&sC[r0 * P + c]), tr_read(&sC[(r0 + 16) * P + c])};
        aw = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*(bf16x8*)va, *(bf16x8*)vb, aw, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pw_part[(size_t)blockIdx.x * PWR + (k * 4 + w) * 256 + (4 * g4 + r) * 16 + (lane & 15)] = aw[r];
      f32x4 d[4];
#pragma unroll
      for (int n = 0; n < 4; ++n) d[n] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 a = *(const bf16x8*)&sDo[(16 * w + (lane & 15)) * P + 32 * ks + 8 * (lane >> 4)];
#pragma unroll
        for (int n = 0; n < 4; ++n) d[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bw[ks][n], d[n], 0, 0, 0);
      }
      if (k + 1 < KT) load_b(k + 1);
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int pr = 16 * w + 4 * g4 + r, cc = 16 * n + (lane & 15);
          sDcT[cc * PS + pr] = f2bf(d[n][r]);
        }
    }
    __syncthreads();
    // C: offset gradient (mmcv get_coordinate_weight), thread = pixel x group, the four groups
    // combined by two xor shuffles; out-of-window corners scatter with global atomics
    {
      float gh = 0.0f, gw = 0.0f;
      if (s.valid) {
        float dc[CG], v[CG];
#pragma unroll
        for (int c = 0; c < CG; ++c) dc[c] = bf2f(sDcT[(q * CG + c) * PS + p]);   // the bf16 dcol of phase D
        const int cok[4] = {s.c1, s.c2, s.c3, s.c4};
        const float ch[4] = {-s.hw, -s.lw, s.hw, s.lw}, cwd[4] = {-s.hh, s.hh, -s.lh, s.lh};
#pragma unroll
        for (int cn = 0; cn < 4; ++cn) {
          if (!cok[cn]) continue;
          fetch16(g, tl, x, xp, sXw, s.hl + (cn >> 1), s.wl + (cn & 1), q, v);
          float sv = 0.0f;
#pragma unroll
          for (int c = 0; c < CG; ++c) sv += dc[c] * v[c];
          gh += ch[cn] * sv;
          gw += cwd[cn] * sv;
        }
      }
      gh += __shfl_xor(gh, 1, 64);
      gw += __shfl_xor(gw, 1, 64);
      gh += __shfl_xor(gh, 2, 64);
      gw += __shfl_xor(gw, 2, 64);
      // the offset-conv output gradient of (pixel, tap k) straight to the image (bf16 pair), and the bias
      // gradient partials: the wave's 16 pixels summed by xor shuffles (fixed order), one row per wave
      if (q == 0)
        *(unsigned*)(doff + mypix * doffp + 2 * k) = (unsigned)f2bf(gh) | ((unsigned)f2bf(gw) << 16);
      float sh = gh, sw = gw;
#pragma unroll
      for (int m = 4; m < 64; m <<= 1) {
        sh += __shfl_xor(sh, m, 64);
        sw += __shfl_xor(sw, m, 64);
      }
      if (lane == 0) {
        sPb[w * 2 * KT + 2 * k] = sh;
        sPb[w * 2 * KT + 2 * k + 1] = sw;
      }
      if (prev_u <= -2) {                  // rare: this thread's corner lies outside the window
        const int code = -2 - prev_u, cy = code >> 16, cx = code & 0xffff;
        const float wq = q == 0 ? s.hh * s.hw : (q == 1 ? s.hh * s.lw : (q == 2 ? s.lh * s.hw : s.lh * s.lw));
        float* dst = dx + ((size_t)(tl.b * g.H + cy) * g.W + cx) * C;
        for (int c = 0; c < C; ++c) atomicAdd(&dst[c], wq * bf2f(sDcT[c * PS + p]));
        prev_u = -1;
      }
    }
    // D: dx_window += S_k x dcol_k (M = window pixels, N = channels, K = tile pixels)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int rt = w + 4 * i;               // window row tile (16 window pixels), 9 in all
      if (rt >= WR / 16) break;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 a = *(const bf16x8*)&S[(16 * rt + (lane & 15)) * PS + 32 * ks + 8 * (lane >> 4)];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const bf16x8 bv = *(const bf16x8*)&sDcT[(16 * n + (lane & 15)) * PS + 32 * ks + 8 * (lane >> 4)];
          acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bv, acc[i][n], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // the padded offset-gradient image (dch = 64): channels 18..63 zero (channels 0..17 were written per tap;
  // dch = 18 writes exactly those, a slice of a shared image)
  if (dch == C) {
    for (int qd = tid; qd < 64 * 8; qd += BLK) {
      const int pp = qd >> 3, j = qd & 7;
      u16* row = doff + ((size_t)(tl.b * g.H + tl.y0 + (pp >> 3)) * g.W + tl.x0 + (pp & 7)) * doffp;
      if (j < 3) *(unsigned*)(row + 2 * KT + 2 * j) = 0u;          // channels 18..23
      else *(uint4*)(row + 24 + 8 * (j - 3)) = make_uint4(0u, 0u, 0u, 0u);   // 24..63
    }
  }
  __syncthreads();
  if (tid < 2 * KT)
    pb_part[(size_t)blockIdx.x * PWR + tid] = ((sPb[tid] + sPb[2 * KT + tid]) + sPb[4 * KT + tid]) + sPb[6 * KT + tid];
  else if (tid < 32)   // the row's 64-byte padding: zeros, so the slab reduce never sums uninitialised words
    pb_part[(size_t)blockIdx.x * PWR + tid] = 0.0f;
  // the window's input gradient -> this tile's slab [144][64] (k_gather_dx sums the <= 4 covering
  // slabs per pixel in a fixed order: no atomics, deterministic)
  float* wdst = win_part + (size_t)blockIdx.x * WR * C;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int rt = w + 4 * i;
    if (rt >= WR / 16) break;
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) wdst[(16 * rt + 4 * g4 + r) * C + 16 * n + (lane & 15)] = acc[i][n][r];
  }
}

__global__ __launch_bounds__(BLK) void k_gather_dx(Geo g, const float* __restrict__ win_part, float* __restrict__ dx) {
  const long long e = (long long)blockIdx.x * BLK + threadIdx.x;
  if (e >= (long long)g.B * g.H * g.W * C) return;
  const long long pix = e / C;
  const int c = (int)(e - pix * C);
  const int b = (int)(pix / ((long long)g.H * g.W)), r = (int)(pix - (long long)b * g.H * g.W);
  const int y = r / g.W, x = r - (r / g.W) * g.W;
  // tiles whose window rows [8t - 2, 8t + 10) contain y
  const int ty0 = max(0, (y + 6) / TE - 1), ty1 = min(g.TY - 1, (y + 2) / TE);
  const int tx0 = max(0, (x + 6) / TE - 1), tx1 = min(g.TX - 1, (x + 2) / TE);
  float s = 0.0f;
  for (int ty = ty0; ty <= ty1; ++ty) {
    const int wy = y - (ty * TE - 2);
    if (wy < 0 || wy >= WE) continue;
    for (int tx = tx0; tx <= tx1; ++tx) {
      const int wx = x - (tx * TE - 2);
      if (wx < 0 || wx >= WE) continue;
      const size_t t = ((size_t)b * g.TY + ty) * g.TX + tx;
      s += win_part[(t * WR + wy * WE + wx) * C + c];
    }
  }
  dx[e] += s;
}

// dWdiag [9][4][16 co][16 ci] -> module layout [64 co][16 ci][3][3]; the reduced row's last 2 * KT values (the offset
// bias gradient) -> db
__global__ __launch_bounds__(BLK) void k_wstore(const float* __restrict__ d, float* __restrict__ dW,
                                                float* __restrict__ db) {
  const int e = blockIdx.x * BLK + threadIdx.x;
  if (e < 2 * KT) db[e] = d[KT * 1024 + e];
  if (e >= KT * 4 * 256) return;
  const int k = e / 1024, r = e - k * 1024, gq = r / 256, m = (r / 16) % 16, n = r % 16;
  dW[((gq * CG + m) * CG + n) * KT + k] = d[e];
}

// ------------------------------------------------------------------ fp32 (parity mode)
// The same semantics on fp32 images with fp32 VALU arithmetic (the 1e-4 loss parity of north_star):
//   forward:  thread = (pixel, group) of an 8 x 8 tile; per tap the 16 sampled channels of its group
//             (corners from global memory: the 12 x 12 window of a tile stays in L1/L2) times the
//             group's 16 x 16 block of W_k (LDS) -> 16 fp32 outputs.
//   backward: per tap, thread-local dcol = W_k^T dOut (its group), the offset gradient (four groups
//             combined by xor shuffles, as in k_bwd), the input gradient added with LDS float atomics
//             into the tile's window (-> the same per-tile slab + k_gather_dx; corners outside the
//             window: global atomics), and dW_k's diagonal blocks from the staged col / dOut tiles.
constexpr int PF = C + 4;        // fp32 tile pitch (floats)

__device__ __forceinline__ void fetch16f(const Geo& g, int b, const float* __restrict__ x, int xp, int cy, int cx,
                                         int q, float* v) {
  const float4* p = (const float4*)(x + ((size_t)(b * g.H + cy) * g.W + cx) * xp + q * CG);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float4 t = p[i];
    v[4 * i] = t.x;
    v[4 * i + 1] = t.y;
    v[4 * i + 2] = t.z;
    v[4 * i + 3] = t.w;
  }
}

__device__ __forceinline__ void sample16f(const Geo& g, int b, const float* __restrict__ x, int xp, const Samp& s,
                                          int q, float* col) {
#pragma unroll
  for (int c = 0; c < CG; ++c) col[c] = 0.0f;
  if (!s.valid) return;
  const int cok[4] = {s.c1, s.c2, s.c3, s.c4};
  const float wq[4] = {s.hh * s.hw, s.hh * s.lw, s.lh * s.hw, s.lh * s.lw};
  float v[CG];
#pragma unroll
  for (int cn = 0; cn < 4; ++cn) {
    if (!cok[cn]) continue;
    fetch16f(g, b, x, xp, s.hl + (cn >> 1), s.wl + (cn & 1), q, v);
#pragma unroll
    for (int c = 0; c < CG; ++c) col[c] = fmaf(wq[cn], v[c], col[c]);
  }
}

// W [64 co][16 ci][3][3] -> sW[k][group][a][b]: forward (a = ci, b = co) or backward (a = co, b = ci)
template <bool FWD>
__device__ __forceinline__ void stage_w(const float* __restrict__ W, float* sW) {
  for (int e = threadIdx.x; e < C * CG * KT; e += BLK) {
    const int co = e / (CG * KT), r = e - co * CG * KT, ci = r / KT, k = r - ci * KT;
    const int gq = co / CG, col = co % CG;
    sW[((k * 4 + gq) * CG + (FWD ? ci : col)) * CG + (FWD ? col : ci)] = W[e];
  }
}

__global__ __launch_bounds__(BLK) void k_fwd_f32(Geo g, const float* __restrict__ x, int xp,
                                                 const float* __restrict__ off, int offp,
                                                 const float* __restrict__ ob, const float* __restrict__ W,
                                                 float* __restrict__ out, int op) {
  __shared__ __attribute__((aligned(16))) float sW[KT * C * CG];
  stage_w<true>(W, sW);
  __syncthreads();
  const Tile tl = tile_of(g, blockIdx.x);
  const int p = threadIdx.x >> 2, q = threadIdx.x & 3;
  const int y = tl.y0 + (p >> 3), xx = tl.x0 + (p & 7);
  const size_t pix = (size_t)(tl.b * g.H + y) * g.W + xx;
  float acc[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) acc[c] = 0.0f;
#pragma unroll 1
  for (int k = 0; k < KT; ++k) {
    const Samp s = samp(g, y, xx, k, off[pix * offp + 2 * k] + ob[2 * k], off[pix * offp + 2 * k + 1] + ob[2 * k + 1]);
    if (!s.valid) continue;
    float col[CG];
    sample16f(g, tl.b, x, xp, s, q, col);
    const float4* wk = (const float4*)&sW[(k * 4 + q) * CG * CG];
#pragma unroll
    for (int ci = 0; ci < CG; ++ci)
#pragma unroll
      for (int c4 = 0; c4 < CG / 4; ++c4) {
        const float4 w = wk[ci * (CG / 4) + c4];
        acc[4 * c4] = fmaf(w.x, col[ci], acc[4 * c4]);
        acc[4 * c4 + 1] = fmaf(w.y, col[ci], acc[4 * c4 + 1]);
        acc[4 * c4 + 2] = fmaf(w.z, col[ci], acc[4 * c4 + 2]);
        acc[4 * c4 + 3] = fmaf(w.w, col[ci], acc[4 * c4 + 3]);
      }
  }
  float4* o = (float4*)(out + pix * op + q * CG);
#pragma unroll
  for (int c4 = 0; c4 < CG / 4; ++c4) o[c4] = make_float4(acc[4 * c4], acc[4 * c4 + 1], acc[4 * c4 + 2], acc[4 * c4 + 3]);
}

__global__ __launch_bounds__(BLK) void k_bwd_f32(Geo g, const float* __restrict__ x, int xp,
                                                 const float* __restrict__ off, int offp,
                                                 const float* __restrict__ ob, const float* __restrict__ W,
                                                 const float* __restrict__ dout, int dop, float* __restrict__ dx,
                                                 float* __restrict__ doff, int doffp, int dch, float* __restrict__ pw_part,
                                                 float* __restrict__ pb_part, float* __restrict__ win_part) {
  __shared__ __attribute__((aligned(16))) float sW[KT * C * CG];     // [k][group][co][ci]
  __shared__ __attribute__((aligned(16))) float sWin[WR * C];        // window input gradient
  __shared__ __attribute__((aligned(16))) float sC[64 * PF];         // col of the current tap
  __shared__ __attribute__((aligned(16))) float sDo[64 * PF];        // dOut of the tile
  __shared__ float sOff[64 * 2 * KT];
  const int tid = threadIdx.x;
  const Tile tl = tile_of(g, blockIdx.x);
  stage_w<false>(W, sW);
  for (int i = tid; i < WR * C / 4; i += BLK) ((float4*)sWin)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int qd = tid; qd < 64 * 16; qd += BLK) {
    const int pp = qd >> 4, seg = qd & 15;
    const size_t pix = (size_t)(tl.b * g.H + tl.y0 + (pp >> 3)) * g.W + tl.x0 + (pp & 7);
    *(float4*)&sDo[pp * PF + seg * 4] = *(const float4*)(dout + pix * dop + seg * 4);
  }
  __syncthreads();
  const int p = tid >> 2, q = tid & 3;
  const int y = tl.y0 + (p >> 3), xx = tl.x0 + (p & 7);
  const size_t pix = (size_t)(tl.b * g.H + y) * g.W + xx;
  float go[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) go[c] = sDo[p * PF + q * CG + c];
  // dW phase: 64 threads per group, thread = (co, 4 consecutive ci)
  const int wq_ = tid >> 6, wr = tid & 63, wco = wr >> 2, wci = (wr & 3) * 4;
#pragma unroll 1
  for (int k = 0; k < KT; ++k) {
    const Samp s = samp(g, y, xx, k, off[pix * offp + 2 * k] + ob[2 * k], off[pix * offp + 2 * k + 1] + ob[2 * k + 1]);
    float col[CG], dc[CG];
    sample16f(g, tl.b, x, xp, s, q, col);
#pragma unroll
    for (int c4 = 0; c4 < CG / 4; ++c4)
      *(float4*)&sC[p * PF + q * CG + 4 * c4] = make_float4(col[4 * c4], col[4 * c4 + 1], col[4 * c4 + 2], col[4 * c4 + 3]);
#pragma unroll
    for (int c = 0; c < CG; ++c) dc[c] = 0.0f;
    const float4* wk = (const float4*)&sW[(k * 4 + q) * CG * CG];
#pragma unroll
    for (int co = 0; co < CG; ++co)
#pragma unroll
      for (int c4 = 0; c4 < CG / 4; ++c4) {
        const float4 w = wk[co * (CG / 4) + c4];
        dc[4 * c4] = fmaf(w.x, go[co], dc[4 * c4]);
        dc[4 * c4 + 1] = fmaf(w.y, go[co], dc[4 * c4 + 1]);
        dc[4 * c4 + 2] = fmaf(w.z, go[co], dc[4 * c4 + 2]);
        dc[4 * c4 + 3] = fmaf(w.w, go[co], dc[4 * c4 + 3]);
      }
    // offset gradient (mmcv get_coordinate_weight) and the input-gradient scatter
    float gh = 0.0f, gw = 0.0f;
    if (s.valid) {
      const int cok[4] = {s.c1, s.c2, s.c3, s.c4};
      const float ch[4] = {-s.hw, -s.lw, s.hw, s.lw}, cwd[4] = {-s.hh, s.hh, -s.lh, s.lh};
      const float wq[4] = {s.hh * s.hw, s.hh * s.lw, s.lh * s.hw, s.lh * s.lw};
#pragma unroll
      for (int cn = 0; cn < 4; ++cn) {
        if (!cok[cn]) continue;
        const int cy = s.hl + (cn >> 1), cx = s.wl + (cn & 1);
        float v[CG];
        fetch16f(g, tl.b, x, xp, cy, cx, q, v);
        float sv = 0.0f;
#pragma unroll
        for (int c = 0; c < CG; ++c) sv = fmaf(dc[c], v[c], sv);
        gh = fmaf(ch[cn], sv, gh);
        gw = fmaf(cwd[cn], sv, gw);
        const int wy = cy - (tl.y0 - 2), wx = cx - (tl.x0 - 2);
        if (wy >= 0 && wy < WE && wx >= 0 && wx < WE) {
          float* dst = &sWin[(wy * WE + wx) * C + q * CG];
#pragma unroll
          for (int c = 0; c < CG; ++c) atomicAdd(&dst[c], wq[cn] * dc[c]);
        } else {
          float* dst = dx + ((size_t)(tl.b * g.H + cy) * g.W + cx) * C + q * CG;
#pragma unroll
          for (int c = 0; c < CG; ++c) atomicAdd(&dst[c], wq[cn] * dc[c]);
        }
      }
    }
    gh += __shfl_xor(gh, 1, 64);
    gw += __shfl_xor(gw, 1, 64);
    gh += __shfl_xor(gh, 2, 64);
    gw += __shfl_xor(gw, 2, 64);
    if (q == 0) {
      sOff[p * 2 * KT + 2 * k] = gh;
      sOff[p * 2 * KT + 2 * k + 1] = gw;
    }
    __syncthreads();
    // dW_k[co][ci] of group wq_ = sum over the tile's pixels of dOut[co] * col[ci]
    {
      float a4[4] = {0.f, 0.f, 0.f, 0.f};
      for (int pp = 0; pp < 64; ++pp) {
        const float d = sDo[pp * PF + wq_ * CG + wco];
        const float4 cv = *(const float4*)&sC[pp * PF + wq_ * CG + wci];
        a4[0] = fmaf(d, cv.x, a4[0]);
        a4[1] = fmaf(d, cv.y, a4[1]);
        a4[2] = fmaf(d, cv.z, a4[2]);
        a4[3] = fmaf(d, cv.w, a4[3]);
      }
      float* dst = pw_part + (size_t)blockIdx.x * PWR + (k * 4 + wq_) * 256 + wco * 16 + wci;
      *(float4*)dst = make_float4(a4[0], a4[1], a4[2], a4[3]);
    }
    __syncthreads();
  }
  const int nseg = dch == C ? doffp / 4 : 0;   // dch = 18: exactly the offset channels (float2 stores below)
  for (int qd = tid; dch != C && qd < 64 * KT; qd += BLK) {
    const int pp = qd / KT, h = qd - pp * KT;
    const size_t px = (size_t)(tl.b * g.H + tl.y0 + (pp >> 3)) * g.W + tl.x0 + (pp & 7);
    *(float2*)(doff + px * doffp + 2 * h) = make_float2(sOff[pp * 2 * KT + 2 * h], sOff[pp * 2 * KT + 2 * h + 1]);
  }
  for (int qd = tid; qd < 64 * nseg; qd += BLK) {
    const int pp = qd / nseg, seg = qd - pp * nseg;
    const size_t px = (size_t)(tl.b * g.H + tl.y0 + (pp >> 3)) * g.W + tl.x0 + (pp & 7);
    float v[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) v[h] = seg * 4 + h < 2 * KT ? sOff[pp * 2 * KT + seg * 4 + h] : 0.0f;
    *(float4*)(doff + px * doffp + seg * 4) = make_float4(v[0], v[1], v[2], v[3]);
  }
  if (tid < 2 * KT) {
    float sacc = 0.0f;
    for (int pp = 0; pp < 64; ++pp) sacc += sOff[pp * 2 * KT + tid];
    pb_part[(size_t)blockIdx.x * PWR + tid] = sacc;
  } else if (tid < 32) {
    pb_part[(size_t)blockIdx.x * PWR + tid] = 0.0f;
  }
  float* wdst = win_part + (size_t)blockIdx.x * WR * C;
  for (int i = tid; i < WR * C / 4; i += BLK) ((float4*)wdst)[i] = ((const float4*)sWin)[i];
}

static int check_geo(int B, int H, int W, Geo* g) {
  if (B < 1 || H < 1 || W < 1 || H % TE || W % TE) return 0;
  *g = Geo{B, H, W, H / TE, W / TE};
  return 1;
}

}  // namespace dcn
}  // namespace rpc

using namespace rpc;
using namespace rpc::dcn;

extern "C" int rpc_dcn_prep_weight(const float* W, void* w_fwd, void* w_bwd, void* stream) {
  if (!W || !w_fwd || !w_bwd) return RPC_ERR_ARG;
  hipLaunchKernelGGL(k_prep, dim3((KT * C * C + BLK - 1) / BLK), dim3(BLK), 0, (hipStream_t)stream, W, (u16*)w_fwd,
                     (u16*)w_bwd);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dcn_forward(const void* x, int xp, const void* off, int offp, const float* off_bias,
                               const void* w_fwd, void* out, int op, int B, int H, int W, void* stream) {
  Geo g;
  if (!check_geo(B, H, W, &g)) return RPC_ERR_UNSUPPORTED;
  if (!x || !off || !off_bias || !w_fwd || !out || xp < C || (xp & 7) || offp < 2 * KT || (offp & 7) || op < C ||
      (op & 7))
    return RPC_ERR_ARG;
  hipLaunchKernelGGL(k_fwd, dim3(B * g.TY * g.TX), dim3(BLK), 0, (hipStream_t)stream, g, (const u16*)x, xp,
                     (const u16*)off, offp, off_bias, (const u16*)w_fwd, (u16*)out, op);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" size_t rpc_dcn_backward_workspace_size(int B, int H, int W) {
  Geo g;
  if (!check_geo(B, H, W, &g)) return 0;
  const size_t tiles = (size_t)B * g.TY * g.TX;
  return (tiles * PWR + PWR + tiles * WR * C) * sizeof(float);
}

// dch: offset-gradient channels written per pixel. C (64): a padded image of its own (channels 18..doffp-1
// zero, 16-byte stores); 2 * KT (18): exactly the offset channels, e.g. one DCN's slice of a shared image
// written by several DCNs (the concatenated offset conv of a CenterPoint head: doff at channel 18 j, pitch 256)
static int dcn_backward_bf16(const void* x, int xp, const void* off, int offp, const float* off_bias,
                             const void* w_bwd, const void* dout, int dop, float* dx, void* doff, int doffp, int dch,
                             float* doff_bias, float* dW, int B, int H, int W, void* workspace, size_t ws_bytes,
                             void* stream) {
  Geo g;
  if (!check_geo(B, H, W, &g)) return RPC_ERR_UNSUPPORTED;
  if (!x || !off || !off_bias || !w_bwd || !dout || !dx || !doff || !doff_bias || !dW || !workspace) return RPC_ERR_ARG;
  if (xp < C || (xp & 7) || offp < 2 * KT || (offp & 7) || dop < C || (dop & 7)) return RPC_ERR_ARG;
  if (dch == C ? (doffp < C || (doffp & 7) || ((uintptr_t)doff & 15))
               : (dch != 2 * KT || doffp < 2 * KT || (doffp & 1) || ((uintptr_t)doff & 3)))
    return RPC_ERR_ARG;
  if (ws_bytes < rpc_dcn_backward_workspace_size(B, H, W)) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int tiles = B * g.TY * g.TX;
  // per-tile partial rows [tiles][PWR]: the weight-gradient diagonal blocks, then the offset-bias gradient (one
  // slab reduce for both)
  float* pw = (float*)workspace;
  float* pb = pw + KT * 1024;
  float* dwd = pw + (size_t)tiles * PWR;
  float* win = dwd + PWR;
  hipLaunchKernelGGL(k_bwd, dim3(tiles), dim3(BLK), 0, st, g, (const u16*)x, xp, (const u16*)off, offp, off_bias,
                     (const u16*)w_bwd, (const u16*)dout, dop, dx, (u16*)doff, doffp, dch, pw, pb, win);
  RPC_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_gather_dx, dim3((unsigned)(((long long)B * H * W * C + BLK - 1) / BLK)), dim3(BLK), 0, st, g,
                     (const float*)win, dx);
  slab_reduce(pw, tiles, PWR, dwd, st);
  hipLaunchKernelGGL(k_wstore, dim3((KT * 1024 + BLK - 1) / BLK), dim3(BLK), 0, st, dwd, dW, doff_bias);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dcn_backward(const void* x, int xp, const void* off, int offp, const float* off_bias,
                                const void* w_bwd, const void* dout, int dop, float* dx, void* doff, int doffp,
                                float* doff_bias, float* dW, int B, int H, int W, void* workspace, size_t ws_bytes,
                                void* stream) {
  return dcn_backward_bf16(x, xp, off, offp, off_bias, w_bwd, dout, dop, dx, doff, doffp, C, doff_bias, dW, B, H, W,
                           workspace, ws_bytes, stream);
}

extern "C" int rpc_dcn_backward_ex(const void* x, int xp, const void* off, int offp, const float* off_bias,
                                   const void* w_bwd, const void* dout, int dop, float* dx, void* doff, int doffp,
                                   int doff_channels, float* doff_bias, float* dW, int B, int H, int W,
                                   void* workspace, size_t ws_bytes, void* stream) {
  return dcn_backward_bf16(x, xp, off, offp, off_bias, w_bwd, dout, dop, dx, doff, doffp, doff_channels, doff_bias,
                           dW, B, H, W, workspace, ws_bytes, stream);
}

extern "C" int rpc_dcn_forward_f32(const float* x, int xp, const float* off, int offp, const float* off_bias,
                                   const float* W, float* out, int op, int B, int H, int Wd, void* stream) {
  Geo g;
  if (!check_geo(B, H, Wd, &g)) return RPC_ERR_UNSUPPORTED;
  if (!x || !off || !off_bias || !W || !out || xp < C || (xp & 3) || offp < 2 * KT || op < C || (op & 3))
    return RPC_ERR_ARG;
  hipLaunchKernelGGL(k_fwd_f32, dim3(B * g.TY * g.TX), dim3(BLK), 0, (hipStream_t)stream, g, x, xp, off, offp,
                     off_bias, W, out, op);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

static int dcn_backward_f32(const float* x, int xp, const float* off, int offp, const float* off_bias,
                            const float* W, const float* dout, int dop, float* dx, float* doff, int doffp, int dch,
                            float* doff_bias, float* dW, int B, int H, int Wd, void* workspace, size_t ws_bytes,
                            void* stream) {
  Geo g;
  if (!check_geo(B, H, Wd, &g)) return RPC_ERR_UNSUPPORTED;
  if (!x || !off || !off_bias || !W || !dout || !dx || !doff || !doff_bias || !dW || !workspace) return RPC_ERR_ARG;
  if (xp < C || (xp & 3) || offp < 2 * KT || dop < C || (dop & 3)) return RPC_ERR_ARG;
  if (dch == C ? (doffp < 2 * KT || (doffp & 3) || ((uintptr_t)doff & 15))
               : (dch != 2 * KT || doffp < 2 * KT || (doffp & 1) || ((uintptr_t)doff & 7)))
    return RPC_ERR_ARG;
  if (ws_bytes < rpc_dcn_backward_workspace_size(B, H, Wd)) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int tiles = B * g.TY * g.TX;
  // per-tile partial rows [tiles][PWR]: the weight-gradient diagonal blocks, then the offset-bias gradient (one
  // slab reduce for both)
  float* pw = (float*)workspace;
  float* pb = pw + KT * 1024;
  float* dwd = pw + (size_t)tiles * PWR;
  float* win = dwd + PWR;
  hipLaunchKernelGGL(k_bwd_f32, dim3(tiles), dim3(BLK), 0, st, g, x, xp, off, offp, off_bias, W, dout, dop, dx, doff,
                     doffp, dch, pw, pb, win);
  RPC_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_gather_dx, dim3((unsigned)(((long long)B * H * Wd * C + BLK - 1) / BLK)), dim3(BLK), 0, st, g,
                     (const float*)win, dx);
  slab_reduce(pw, tiles, PWR, dwd, st);
  hipLaunchKernelGGL(k_wstore, dim3((KT * 1024 + BLK - 1) / BLK), dim3(BLK), 0, st, dwd, dW, doff_bias);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_dcn_backward_f32(const float* x, int xp, const float* off, int offp, const float* off_bias,
                                    const float* W, const float* dout, int dop, float* dx, float* doff, int doffp,
                                    float* doff_bias, float* dW, int B, int H, int Wd, void* workspace,
                                    size_t ws_bytes, void* stream) {
  return dcn_backward_f32(x, xp, off, offp, off_bias, W, dout, dop, dx, doff, doffp, C, doff_bias, dW, B, H, Wd,
                          workspace, ws_bytes, stream);
}

extern "C" int rpc_dcn_backward_f32_ex(const float* x, int xp, const float* off, int offp, const float* off_bias,
                                       const float* W, const float* dout, int dop, float* dx, float* doff, int doffp,
                                       int doff_channels, float* doff_bias, float* dW, int B, int H, int Wd,
                                       void* workspace, size_t ws_bytes, void* stream) {
  return dcn_backward_f32(x, xp, off, offp, off_bias, W, dout, dop, dx, doff, doffp, doff_channels, doff_bias, dW, B,
                          H, Wd, workspace, ws_bytes, stream);
}
