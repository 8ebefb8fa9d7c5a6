// a6 perf mode: bf16-MFMA implicit-GEMM sparse conv (forward and dgrad) for gfx950.
//
// Same neighbour-map semantics as spconv.hip, different data path:
//   * activations are gathered as bf16 rows [N][CP] (CP = channels padded to 8) that an
//     elementwise pass produced once per layer (relu(bn(z)) forward, the BatchNorm-backward
//     dz in backward) — a gathered neighbour row is 16..256 B;
//   * each wave owns 16 output rows and loads its A fragments of v_mfma_f32_16x16x32_bf16
//     (8 channels of one gathered row per lane, 16 B) straight from global memory into
//     registers — no LDS round trip, one offset ahead;
//   * the weight tile B_k^T [N][K] of the next offset is prefetched into registers and
//     written to the other half of a double-buffered LDS ring while the MFMAs of the current
//     offset run; one barrier per offset;
//   * blocks of 8 waves (128 rows; 4 waves for 128 x 128 tiles) share each LDS weight tile;
//     offsets with no neighbour in the block's rows are skipped by the block, offsets with
//     none in a wave's 16 rows are skipped by that wave (no loads, no MFMA).
// Accumulation in fp32; epilogues identical to spconv.hip (z out + BatchNorm partial sums,
// or the previous layer's ReLU mask + BatchNorm-backward partial sums). No atomics on data.
#include <hip/hip_runtime.h>
#include <string.h>
#include <algorithm>

#include "common.h"
#include <stdlib.h>
#include <hipcub/hipcub.hpp>
#include "dense_common.h"
#include "rpc_hip.h"

namespace rpc {
namespace spb {

constexpr int BLK = 256;
constexpr int BM = 64;          // rows per BatchNorm partial row (rpc_spconv_gemm_blocks)
// GEMM waves per block (16 rows each; all share one LDS weight tile per offset): 8 — the tile is
// fetched once per 128 rows — unless the 128 x 128 tiles' LDS ring would leave one block per CU
__host__ __device__ constexpr int gw_of(int kgp, int nt) { return kgp * nt * 16 >= 128 * 128 ? 4 : 8; }
// 16-row MFMA tiles per wave: every weight fragment a wave reads from LDS feeds RT MFMAs. Two for the
// mid-size tiles (K x 16*NT of 32x32 .. 64x32), whose time went to LDS weight reads (every wave re-read
// the whole tile per offset for its 16 rows): r02v30 <32,2,0> 35.0 -> 30.0 us, <32,2,1> 38.5 -> 36.5,
// <64,2,1> 49 -> 42. Measured and kept at RT=1: the 64x64 tiles (88 VGPRs, 5 waves/SIMD: <64,4,1>
// 47 -> 54 us) and the 32x16 tiles (<32,1,0> 21.3 -> 23.4 us). The 128 x 128 tiles (CenterPoint) take two
// (128-row blocks, one per CU: 88 KB of LDS, 262 registers): forward 259 -> 262, data gradient 624 -> 606,
// plain 407 -> 370 us per launch (profiles/r04_step_kernels_centerpoint_rt2.txt) — the weight tile
// staging and its LDS reads were not the limit either; the data-gradient launches run beside the
// 128 x 128 weight gradient on the side stream
__host__ __device__ constexpr int rt_of(int kgp, int nt) {
  return ((kgp * nt >= 64 && kgp * nt <= 128 && nt <= 4) || (kgp == 128 && nt == 8)) ? 2 : 1;
}
__host__ __device__ constexpr int gemm_waves_per_simd(int kgp, int nt) {
  return kgp * nt >= 1024 ? 1 : rt_of(kgp, nt) == 2 ? 5 : ((kgp * nt <= 256 && nt <= 4 && kgp <= 64) ? 8 : 1);
}
constexpr int MAXK = 27;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

__device__ __forceinline__ u16 to_bf16(float f) {
  __bf16 b = (__bf16)f;   // round-to-nearest-even, NaN kept (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(u16, b);
}
__device__ __forceinline__ u16 to_f16(float f) {
  _Float16 h = (_Float16)f;   // round-to-nearest-even (v_cvt_f16_f32)
  return __builtin_bit_cast(u16, h);
}
// 16-bit GEMM operand format: 0 = bf16, 1 = fp16 (RPC_H16_*). fp16 (3 more mantissa bits, same MFMA rate) is
// used for the FORWARD operands of the perf mode — the normalised activations relu(bn(z)) and the weights,
// both far inside its range — where the operand rounding decides the ReLU masks every later gradient goes
// through (oracle/sparse_encoder.py bf16_from emulation: perturber-gradient error 0.237 with bf16 forward
// operands, 0.077 with fp16, the backward's bf16 dz rows alike); the backward's dz rows stay bf16 (no range
// to manage: no loss scaling).
template <int FMT>
__device__ __forceinline__ u16 to_h16(float f) { return FMT ? to_f16(f) : to_bf16(f); }
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
template <bool F16>
__device__ __forceinline__ f32x4 mfma16(uint4 a, uint4 b, f32x4 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
                                                   0);
}

// E_RES: the data gradient into a basicblock's output rows: m = (acc + g2) * [out > 0] with the BatchNorm-
// backward partial sums (sum m, sum m * xhat(z)) of that layer — rpc_sparse_res_backward fused into the GEMM
enum { E_FWD = 0, E_DGRAD = 1, E_PLAIN = 2, E_RES = 3 };

struct GB {
  const u16* a;       // gathered source rows [Nsrc][CP] bf16
  int CP;             // row pitch (elements, multiple of 8)
  const int* nbr;     // [Nout][K]
  int K, rev;
  const u16* bt;      // B^T per offset [K][NGP][KGP] bf16 (zero padded)
  int Nout;
  float* out;         // [Nout][CO_real]
  int CO_real;
  const float* ez;    // E_DGRAD: z of the layer whose grad this is [Nout][CO_real]
  const float* ebn;   // E_DGRAD: scale, beta, mean, invstd [4*CO_real]
  float* part;        // [blocks][2*NGP] or null
  RpcBnFin fin;       // BatchNorm finalize by the last-arriving blocks (fin.ticket null: off)
  int fmt;            // operand format of a and bt: 0 bf16, 1 fp16 (E_FWD only)
  const int* perm;    // row visiting order [Nout] (rpc_rulebook_mask_perm) or null; rows are written in place
  const float* eg2;   // E_RES: the other gradient contribution [Nout][CO_real] (identity path) or null
  const float* eout;  // E_RES: the block output rows [Nout][CO_real] (ReLU mask)
};

// ---- BatchNorm finalize fused into the GEMM (k_gemm_pipe, RpcBnFin): the partial rows every block writes
// are summed in two fixed-order levels by last-arriving blocks — each group of FGS consecutive blocks
// (logical index lb) by its last arriver, in row order, into a double row gpart[q]; the groups by the
// last group finisher, in group order — which then applies rpc_bn_finalize's arithmetic (mode 0 / 1) to
// the totals. Replaces the standalone k_bn_finalize launch after each GEMM (run-to-run deterministic; the
// totals are summed in another order than k_bn_finalize's, so they may differ from it in the last bits).
constexpr int FGS = 32;
__host__ __device__ inline int fin_groups(int nblk) { return (nblk + FGS - 1) / FGS; }

// hand-off data (partial rows, group totals) written with agent-scope atomic stores and read with agent-scope
// atomic loads: the blocks' arrivals need no L2 writeback (last_block_arrive_lite)
template <int NTHR>
__device__ void fused_bn_finalize(const GB& g, int lb, int PRB, double* sh, int* flag) {
  const RpcBnFin& f = g.fin;
  const int C = g.CO_real, C2 = 2 * C;
  const int nblk = (int)gridDim.x, ng = fin_groups(nblk), q = lb / FGS;
  const int nrow = (g.Nout + BM - 1) / BM;
  const int gb0 = q * FGS, gbn = min(FGS, nblk - gb0);
  if (!last_block_arrive_lite(f.ticket + 1 + q, flag, gbn)) return;
  {
    const int pr0 = gb0 * PRB, pr1 = min(nrow, (gb0 + gbn) * PRB);
    for (int j = threadIdx.x; j < C2; j += NTHR) {
      double t = 0.0;
      int r = pr0;
      for (; r + 8 <= pr1; r += 8) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = ld_agent(&g.part[(long long)(r + i) * C2 + j]);
#pragma unroll
        for (int i = 0; i < 8; ++i) t += (double)v[i];
      }
      for (; r < pr1; ++r) t += (double)ld_agent(&g.part[(long long)r * C2 + j]);
      st_agent(&f.gpart[(long long)q * C2 + j], t);
    }
  }
  if (!last_block_arrive_lite(f.ticket, flag, ng)) return;
  for (int j = threadIdx.x; j < C2; j += NTHR) {
    double t = 0.0;
    int r = 0;
    for (; r + 8 <= ng; r += 8) {
      double v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = ld_agent(&f.gpart[(long long)(r + i) * C2 + j]);
#pragma unroll
      for (int i = 0; i < 8; ++i) t += v[i];
    }
    for (; r < ng; ++r) t += ld_agent(&f.gpart[(long long)r * C2 + j]);
    sh[j] = t;
  }
  __syncthreads();
  const int N = g.Nout;
  for (int c = threadIdx.x; c < C; c += NTHR) {
    const double s1 = sh[c], s2 = sh[C + c];
    if (f.mode == 0) {   // k_bn_finalize mode 0
      const double mean = s1 / N;
      double var = s2 / N - mean * mean;
      if (var < 0) var = 0;
      const float invstd = 1.0f / sqrtf((float)var + f.eps);
      f.bn[c] = f.gamma[c] * invstd;
      f.bn[C + c] = f.beta[c];
      f.bn[2 * C + c] = (float)mean;
      f.bn[3 * C + c] = invstd;
      const double uvar = N > 1 ? var * N / (N - 1) : var;
      f.running_mean[c] = (1.0f - f.momentum) * f.running_mean[c] + f.momentum * (float)mean;
      f.running_var[c] = (1.0f - f.momentum) * f.running_var[c] + f.momentum * (float)uvar;
    } else {             // k_bn_finalize mode 1
      f.bn[c] = f.gamma[c] * f.fbn[3 * C + c];
      f.bn[C + c] = (float)(s1 / N);
      f.bn[2 * C + c] = (float)(s2 / N);
      f.bn[3 * C + c] = f.fbn[2 * C + c];
      f.bn[4 * C + c] = f.fbn[3 * C + c];
      if (f.dgamma) f.dgamma[c] = (float)s2;
      if (f.dbeta) f.dbeta[c] = (float)s1;
    }
  }
}

// Occupancy: the <= 64 x 64 tiles are held to 64 VGPRs (8 waves per SIMD, 4 blocks per CU) — at 72 the
// 106k-row 64-channel layers needed 1.08 rounds of 3 blocks per CU (k_gemm_bf16<64,4,1> 60.6 -> 51.5 us)
// DBG (timing attribution only, rpc_spconv_gemm_bf16_mode 4 + DBG for the 64 x 64 tiles; results are
// garbage): bit 0 = no MFMAs, bit 1 = every gather offset out of range (no memory traffic, same
// instructions), bit 2 = the same for the weight tiles, bit 3 = no gather instructions at all
template <int KGP, int NT, int EPI, int DBG = 0, bool F16 = false>
__global__ __launch_bounds__(64 * gw_of(KGP, NT), gemm_waves_per_simd(KGP, NT)) void k_gemm_bf16(GB g) {
  constexpr int GW = gw_of(KGP, NT), GBLK = 64 * GW, RT = rt_of(KGP, NT), WR = 16 * RT, GBM = WR * GW;
  constexpr int KS = KGP / 32;
  constexpr int NGP = NT * 16;
  // LDS row stride: 8 mod 16 dwords (conflict-free b128 reads), except the 128 x 128 tiles, whose
  // smaller 16-B pad keeps two blocks per CU (a 144-element pitch leaves one: 1.7x slower)
  constexpr int LS = (KGP >= 128 && NT >= 8) ? KGP + 8 : KGP + 16;
  constexpr int BV = NGP * KGP / 8;           // 16-B vectors per offset tile
  constexpr int BPT = (BV + GBLK - 1) / GBLK;
  __shared__ __attribute__((aligned(16))) u16 sB[2][NGP * LS];
  __shared__ int sN[GBM * MAXK];
  __shared__ unsigned wmask[GW];
  __shared__ int klist[MAXK];
  __shared__ int nk;
  __shared__ float sP[GW][2 * NGP];
  __shared__ int sRow[GBM];   // physical row of each logical row (the visiting order; -1 past Nout)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // XCD-aware row blocks: each XCD takes one contiguous eighth of the (spatially sorted) rows, so the
  // neighbour rows its blocks gather — mostly within a few thousand rows — stay in that XCD's L2
  // (round-robin placement made every XCD gather from the whole source table: L2 misses)
  const int lb = dn::xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = lb * GBM;
  const int K = g.K;
  {
    // each wave stages its own 16 rows: lane = (offset group k4, row lane&15), 4 offsets per pass;
    // the wave's offset mask comes from ballots (no LDS atomics)
    const int rr = lane & 15, k4 = lane >> 4;
    unsigned m = 0;
    // the wave's index loads are all in flight before the first is used (a load per pass, each
    // waited out before the next, cost 7 round trips at the start of every block)
    constexpr int NP = (MAXK + 3) / 4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int lr = w * WR + rt * 16 + rr, lrow = r0 + lr;
      const int row = lrow < g.Nout ? (g.perm ? g.perm[lrow] : lrow) : g.Nout;
      if (k4 == 0) sRow[lr] = row < g.Nout ? row : -1;
      int nv[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int k = 4 * i + k4;
        nv[i] = (k < K && row < g.Nout) ? g.nbr[(long long)row * K + (g.rev ? K - 1 - k : k)] : -1;
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int kb = 4 * i, k = kb + k4, v = nv[i];
        if (kb >= K) break;
        if (k < K) sN[lr * MAXK + k] = v;
        const unsigned long long b = __ballot(v >= 0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if ((b >> (16 * q)) & 0xffffull) m |= 1u << (kb + q);
      }
    }
    if (lane == 0) wmask[w] = m;
  }
  __syncthreads();
  if (tid == 0) {
    unsigned m = 0;
    for (int q = 0; q < GW; ++q) m |= wmask[q];
    int n = 0;
    for (int k = 0; k < K; ++k)
      if ((m >> k) & 1u) klist[n++] = k;
    nk = n;
  }
  __syncthreads();
  const int NK = nk;
  const unsigned my = wmask[w];
  f32x4 acc[RT][NT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int arow = w * WR + (lane & 15);
  const int ag = lane >> 4;
  // Every load of the main loop is issued unconditionally as a buffer load: a missing neighbour, a
  // padding column or an idle thread gets an offset past the descriptor's range, which the hardware
  // returns as zeros. With conditional loads the compiler could not count the loads in flight: the
  // weight-tile LDS store waited on vmcnt(0), i.e. for the next offset's gathers too, every offset.
  // Offsets are 32-bit: the host checks that the source table and the weight tiles fit below 2 GB.
  constexpr unsigned OOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)g.a, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)g.bt, (short)0, 0x7fffffff, 0x00020000);
  auto load_a = [&](int k, uint4 (&dst)[RT][KS]) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int src = sN[(arow + rt * 16) * MAXK + k];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int c0 = ks * 32 + ag * 8;
        if (DBG & 8) {
          dst[rt][ks] = make_uint4(0u, 0u, 0u, 0u);
          continue;
        }
        unsigned off = (src >= 0 && c0 < g.CP && !(DBG & 2)) ? ((unsigned)src * (unsigned)g.CP + (unsigned)c0) * 2u : OOB;
        asm volatile("" : "+v"(off));   // keeps the select a select (else: one load per branch of a diamond)
        dst[rt][ks] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsa, off, 0, 0));
      }
    }
  };
  auto load_b = [&](int k, uint4 (&dst)[BPT]) {
    const unsigned base = (unsigned)k * (unsigned)(NGP * KGP * 2);
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int v = tid + j * GBLK;
      unsigned off = ((BV % GBLK == 0 || v < BV) && !(DBG & 4)) ? base + (unsigned)v * 16u : OOB;
      asm volatile("" : "+v"(off));
      dst[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsb, off, 0, 0));
    }
  };
  auto store_b = [&](int buf, const uint4 (&src)[BPT]) {
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      int v = tid + j * GBLK;
      if (BV % GBLK == 0 || v < BV) {
        int e = v * 8, n = e / KGP, c = e - n * KGP;
        *(uint4*)&sB[buf][n * LS + c] = src[j];
      }
    }
  };

  if (NK > 0) {
    uint4 a0[RT][KS], a1[RT][KS], bw0[BPT], bw1[BPT];
    load_b(klist[0], bw0);
    store_b(0, bw0);
    load_b(klist[NK > 1 ? 1 : 0], bw0);
    load_a(klist[0], a0);
    __syncthreads();
    // one offset per step. Loads run ahead: the A fragments of offset t+1 and the weight tile of
    // offset t+2 are issued at the top of step t, so the LDS store of tile t+1 (loaded one step
    // earlier) and the MFMAs of offset t wait only on loads a whole step old. A fragments and weight
    // registers ping-pong (a0 / a1, bw0 / bw1: no register copy that would wait on the newest loads);
    // the steps near the end re-fetch the last offset so the load count per step is fixed.
    auto step = [&](int t, const uint4 (&ac)[RT][KS], uint4 (&an)[RT][KS], const uint4 (&bc)[BPT],
                    uint4 (&bn)[BPT]) {
      const int k = klist[t];
      load_b(klist[t + 2 < NK ? t + 2 : NK - 1], bn);
      load_a(klist[t + 1 < NK ? t + 1 : t], an);
      if (((my >> k) & 1u) && !(DBG & 1)) {
        const u16* bb = sB[t & 1] + (lane & 15) * LS + ag * 8;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
          for (int n = 0; n < NT; ++n) {
            const uint4 bv = *(const uint4*)(bb + n * 16 * LS + ks * 32);
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) acc[rt][n] = mfma16<F16>(ac[rt][ks], bv, acc[rt][n]);
          }
        }
      }
      store_b((t + 1) & 1, bc);
      __syncthreads();
    };
    // pairs in the loop, an odd last offset after it (a conditional second step inside the loop
    // gave the compiler a path step(t) -> step(t+2) on which a1's gathers were still in flight, and a
    // vmcnt(0) at the loop head for it)
    int t = 0;
    for (; t + 1 < NK; t += 2) {
      step(t, a0, a1, bw0, bw1);
      step(t + 1, a1, a0, bw1, bw0);
    }
    if (t < NK) step(t, a0, a1, bw0, bw1);
  }

  // epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + reg (16x16 shapes, gfx950)
  // E_DGRAD: per output tile n, the previous layer's z of the lane's 4 rows and the column's BatchNorm
  // parameters are loaded together before the tile's stores (out and ez are not known not to alias:
  // interleaved with the stores, every z load waited for its own round trip — 16 per lane)
  float s1[NT], s2[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) s1[n] = s2[n] = 0.0f;
  // (rows in visiting order: lane rows lr .. lr + 3 of the block, physical rows from sRow)
  int prow[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j) prow[rt][j] = sRow[w * WR + rt * 16 + (lane >> 4) * 4 + j];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      int col = n * 16 + (lane & 15);
      float zr[4], pb[4], orr[4], g2r[4];
      if (EPI == E_DGRAD || EPI == E_RES) {
        const int C = g.CO_real, cc = min(col, C - 1);
#pragma unroll
        for (int q = 0; q < 4; ++q) pb[q] = g.ebn[q * C + cc];   // scale, beta, mean, invstd
#pragma unroll
        for (int j = 0; j < 4; ++j) zr[j] = g.ez[(long long)max(prow[rt][j], 0) * C + cc];
      }
      if (EPI == E_RES) {
        const int C = g.CO_real, cc = min(col, C - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const long long e = (long long)max(prow[rt][j], 0) * C + cc;
          orr[j] = g.eout[e];
          g2r[j] = g.eg2 ? g.eg2[e] : 0.0f;
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int row = prow[rt][j];
        float v = acc[rt][n][j];
        if (row >= 0 && col < g.CO_real) {
          if (EPI == E_RES) {
            const float gg = v + g2r[j];
            v = orr[j] > 0.0f ? gg : 0.0f;
            s1[n] += v;
            s2[n] += v * ((zr[j] - pb[2]) * pb[3]);
          } else if (EPI == E_DGRAD) {
            const float zz = zr[j];
            float h = fmaxf(fmaf(zz - pb[2], pb[0], pb[1]), 0.0f);
            v = h > 0.0f ? v : 0.0f;
            float xh = (zz - pb[2]) * pb[3];
            s1[n] += v;
            s2[n] = fmaf(v, xh, s2[n]);   // explicit: contraction left to -ffp-contract differed between kernels
          } else {
            s1[n] += v;
            s2[n] = fmaf(v, v, s2[n]);
          }
          g.out[(long long)row * g.CO_real + col] = v;
        }
      }
    }
  }
  if (EPI == E_PLAIN || g.part == nullptr) return;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    s1[n] += __shfl_xor(s1[n], 16, 64);
    s1[n] += __shfl_xor(s1[n], 32, 64);
    s2[n] += __shfl_xor(s2[n], 16, 64);
    s2[n] += __shfl_xor(s2[n], 32, 64);
    if (lane < 16) {
      sP[w][n * 16 + lane] = s1[n];
      sP[w][NGP + n * 16 + lane] = s2[n];
    }
  }
  __syncthreads();
  // partial rows keep the CO_real-wide layout expected by rpc_bn_finalize: [blocks][2*CO_real]
  const int C = g.CO_real;
  // one partial row per 64 rows (the layout of rpc_spconv_gemm_blocks): waves WPR*h .. WPR*h + WPR-1
  constexpr int WPR = 64 / WR, PRB = GBM / 64;
  const int nrow = (g.Nout + BM - 1) / BM;
  for (int j = tid; j < PRB * 2 * C; j += GBLK) {
    const int h = j / (2 * C), jj = j - h * 2 * C, prow = lb * PRB + h;
    if (prow >= nrow) continue;
    int which = jj / C, c = jj - which * C;
    float s = 0.0f;
    for (int ww = 0; ww < WPR; ++ww) s += sP[WPR * h + ww][which * NGP + c];
    if (g.fin.ticket)
      st_agent(&g.part[(long long)prow * 2 * C + jj], s);
    else
      g.part[(long long)prow * 2 * C + jj] = s;
  }
  if (g.fin.ticket) {
    // the neighbour table is free: the totals (double [2C], C <= 256 -> 4 KB) and the arrival flag go there
    static_assert(GBM * MAXK * 4 >= 4096 + 4, "LDS for the fused finalize");
    fused_bn_finalize<GBLK>(g, lb, PRB, (double*)sN, sN + 1024);
  }
}

// ------------------------------------------------------------------ r04: deep LDS-DMA ring
// k_gemm_bf16 waits out one memory round trip per kernel offset: the A fragments of offset t+1 are the
// only loads in flight while offset t computes, and one offset of MFMAs (8 per wave at 64 x 64) is far
// shorter than a gather under load (~1.7 us per offset step at the 106k-row layers: 23 steps, 39 us).
// k_gemm_pipe issues S-1 offsets ahead instead, straight into LDS (`buffer_load ... lds`, no VGPR round
// trip): per offset and wave the wave's own 16 gathered rows (16 x KGP bf16, NA instructions) and its
// share of the weight tile (NGP x KGP bf16, WI instructions per block), into ring slot t % S. Per step:
// wait for this wave's loads of stage t (vmcnt of the stages issued after it), one barrier (every wave's
// stage-t loads have landed and every wave is done with stage t-1, whose slot the next issue reuses),
// issue stage t+S-1, then the MFMAs of stage t from LDS. LDS rows are KGP bf16 (G = KGP/8 granules of
// 16 B) with granule j of row r stored at j ^ pswz(r): every ds_read_b128 lane group of an A or B
// fragment read then hits 16 distinct bank slots (exhaustive check, tools/swz_check.py). Gathers of
// absent neighbours (and the padding granules of a 16-channel row) get an offset past the buffer range:
// the DMA writes zeros and touches no memory. Same MFMAs in the same order per accumulator as
// k_gemm_bf16 (offsets ascending, K-steps, output tiles), so the same bits; same epilogue.
__host__ __device__ constexpr int pswz(int G, int row) { return G == 16 ? (row & 15) : ((row >> 1) & (G - 1)); }

template <int NPS, int R>
__device__ __forceinline__ void vm_wait(int rem) {
  if constexpr (R > 0) {
    if (rem >= R) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(R * NPS) : "memory");
      return;
    }
    vm_wait<NPS, R - 1>(rem);
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

template <int KGP, int NT, int GW, int S>
struct PipeCfg {
  // RT: 16-row MFMA tiles per wave, as k_gemm_bf16 (rt_of): the same rows per wave and per partial row,
  // so the BatchNorm partial sums are added in the same order (same bits) — except 128 x 128, whose two-tile
  // waves would not fit the ring's LDS (one tile here)
  static constexpr int RT = (KGP == 128 && NT == 8) ? 1 : rt_of(KGP, NT);
  static constexpr int G = KGP / 8, KS = KGP / 32, NGP = NT * 16, WR = 16 * RT, GBM = WR * GW, GBLK = 64 * GW;
  static constexpr int ABYTES = WR * KGP * 2;            // one wave's gathered rows
  static constexpr int NA = WR * G / 64;                 // their DMA instructions (1 KB each)
  static constexpr int WBYTES = NGP * KGP * 2;           // one offset's weight tile
  static constexpr int WI = WBYTES / 1024;               // its DMA instructions (per block)
  static constexpr int NWH = (WI + GW - 1) / GW, NWL = WI / GW, WREM = WI % GW;
  static constexpr int STAGE = GW * ABYTES + WBYTES;
  static constexpr int SN = GBM * MAXK * 4;
  static constexpr int MISC = 256;                       // wmask[GW], klist[MAXK], nk
  static constexpr int LDS = S * STAGE + SN + MISC;
  static_assert(KGP % 32 == 0 && WBYTES % 1024 == 0 && ABYTES % 1024 == 0, "DMA tiles are whole KBs");
  static_assert(GW * 2 * NGP * 4 <= S * STAGE && GW <= 8, "epilogue partials alias the ring");
  static_assert(LDS <= 160 * 1024, "LDS");
};

template <int KGP, int NT, int EPI, int GW, int S>
__global__ __launch_bounds__(64 * GW, 1) void k_gemm_pipe(GB g) {
  using P = PipeCfg<KGP, NT, GW, S>;
  constexpr int G = P::G, KS = P::KS, NGP = P::NGP, GBM = P::GBM, GBLK = P::GBLK, NA = P::NA, RT = P::RT;
  constexpr int WR = P::WR;
  // ONE LDS object: separate __shared__ arrays get alias scopes, and the compiler then drains every
  // DMA in flight (vmcnt(0)) before the operand reads of each step (dense_conv.hip k_conv3x3x)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[P::LDS];
  int* const sN = (int*)(lds + S * P::STAGE);
  unsigned* const wmask = (unsigned*)(lds + S * P::STAGE + P::SN);
  int* const klist = (int*)(wmask + 8);
  int* const nkp = klist + 32;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lb = dn::xcd_remap(blockIdx.x, gridDim.x);
  const int r0 = lb * GBM;
  const int K = g.K;
  {
    // neighbour indices of the wave's rows into LDS, the wave's offset mask by ballots (k_gemm_bf16)
    const int rr = lane & 15, k4 = lane >> 4;
    unsigned m = 0;
    constexpr int NP = (MAXK + 3) / 4;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int lr = w * WR + rt * 16 + rr, row = r0 + lr;
      int nv[NP];
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int k = 4 * i + k4;
        nv[i] = (k < K && row < g.Nout) ? g.nbr[(long long)row * K + (g.rev ? K - 1 - k : k)] : -1;
      }
#pragma unroll
      for (int i = 0; i < NP; ++i) {
        const int kb = 4 * i, k = kb + k4, v = nv[i];
        if (kb >= K) break;
        if (k < K) sN[lr * MAXK + k] = v;
        const unsigned long long b = __ballot(v >= 0);
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if ((b >> (16 * q)) & 0xffffull) m |= 1u << (kb + q);
      }
    }
    if (lane == 0) wmask[w] = m;
  }
  __syncthreads();
  if (tid == 0) {
    unsigned m = 0;
    for (int q = 0; q < GW; ++q) m |= wmask[q];
    int n = 0;
    for (int k = 0; k < K; ++k)
      if ((m >> k) & 1u) klist[n++] = k;
    *nkp = n;
  }
  __syncthreads();
  const int NK = *nkp;
  const unsigned my = wmask[w];

  // ---- fixed per-lane DMA geometry. A instruction i writes LDS granule P = i*64 + lane of this wave's
  // slot: local row P / G, stored granule P % G, which holds source granule (P % G) ^ pswz(row)
  constexpr unsigned OOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)g.a, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)g.bt, (short)0, 0x7fffffff, 0x00020000);
  int ar[NA], ac[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int Pg = i * 64 + lane, r = Pg / G, j = (Pg % G) ^ pswz(G, r);
    ar[i] = (w * WR + r) * MAXK;
    ac[i] = j * 8 < g.CP ? j * 8 : -1;
  }
  constexpr int NWH = P::NWH;
  int wo[NWH > 0 ? NWH : 1];
#pragma unroll
  for (int m = 0; m < NWH; ++m) {
    const int q = w + m * GW, Pg = q * 64 + lane, n = Pg / G, j = (Pg % G) ^ pswz(G, n);
    wo[m] = q < P::WI ? (n * KGP + j * 8) * 2 : (int)OOB;
  }
  // (the DMA builtin's offsets as explicit int casts: passed as plain lvalues — or unsigned — hipcc dropped
  // the kernel from the host pass without a diagnostic: no launch stub, an undefined symbol at load time)
  auto issue = [&](int t) {
    unsigned char* st = lds + (t % S) * P::STAGE;
    const int k = __builtin_amdgcn_readfirstlane(klist[t]);   // the weight offset goes in an SGPR (soffset)
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int src = sN[ar[i] + k];
      const int off = (src >= 0 && ac[i] >= 0) ? (int)(((unsigned)src * (unsigned)g.CP + (unsigned)ac[i]) * 2u)
                                               : (int)OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (__attribute__((address_space(3))) void*)(st + w * P::ABYTES + i * 1024),
                                               16, (int)off, 0, 0, 0);
    }
    const int kb = k * P::WBYTES;
#pragma unroll
    for (int m = 0; m < NWH; ++m) {
      const int q = w + m * GW;
      if (m < P::NWL || w < P::WREM)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsb, (__attribute__((address_space(3))) void*)(st + GW * P::ABYTES + q * 1024), 16, (int)wo[m], (int)kb, 0, 0);
    }
  };

  f32x4 acc[RT][NT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[rt][n] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // operand byte offsets inside a slot: A rows rt*16 + lane&15 of this wave, B rows n*16 + lane&15;
  // granule ks*4 + (lane >> 4), swizzled by the row (pswz(n*16 + r) = pswz(r))
  const int a15 = lane & 15, q4 = lane >> 4;
  int aoff[RT][KS], boff[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      aoff[rt][ks] = w * P::ABYTES + ((rt * 16 + a15) * G + ((ks * 4 + q4) ^ pswz(G, a15))) * 16;
    boff[ks] = GW * P::ABYTES + (a15 * G + ((ks * 4 + q4) ^ pswz(G, a15))) * 16;
  }

#pragma unroll
  for (int t = 0; t < S - 1; ++t)
    if (t < NK) issue(t);
  constexpr int NPS_H = NA + P::NWH, NPS_L = NA + P::NWL;
  for (int t = 0; t < NK; ++t) {
    const int rem = min(S - 2, NK - 1 - t);   // stages issued after stage t
    if (P::WREM == 0 || w < P::WREM) vm_wait<NPS_H, S - 2>(rem);
    else vm_wait<NPS_L, S - 2>(rem);
    // a bare barrier: __syncthreads() is a workgroup fence and waits for every DMA in flight (vmcnt(0))
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + S - 1 < NK) issue(t + S - 1);
    const int k = __builtin_amdgcn_readfirstlane(klist[t]);
    if ((my >> k) & 1u) {
      const unsigned char* st = lds + (t % S) * P::STAGE;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        bf16x8 av[RT];
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) av[rt] = *(const bf16x8*)(st + aoff[rt][ks]);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const bf16x8 bv = *(const bf16x8*)(st + boff[ks] + n * 16 * G * 16);
#pragma unroll
          for (int rt = 0; rt < RT; ++rt)
            acc[rt][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[rt], bv, acc[rt][n], 0, 0, 0);
        }
      }
    }
  }

  // epilogue: k_gemm_bf16's, line for line
  float s1[NT], s2[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) s1[n] = s2[n] = 0.0f;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int rb = r0 + w * WR + rt * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      int col = n * 16 + (lane & 15);
      float zr[4], pb[4];
      if (EPI == E_DGRAD) {
        const int C = g.CO_real, cc = min(col, C - 1);
#pragma unroll
        for (int q = 0; q < 4; ++q) pb[q] = g.ebn[q * C + cc];
#pragma unroll
        for (int j = 0; j < 4; ++j) zr[j] = g.ez[(long long)min(rb + j, g.Nout - 1) * C + cc];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int row = rb + j;
        float v = acc[rt][n][j];
        if (row < g.Nout && col < g.CO_real) {
          if (EPI == E_DGRAD) {
            const float zz = zr[j];
            float h = fmaxf(fmaf(zz - pb[2], pb[0], pb[1]), 0.0f);
            v = h > 0.0f ? v : 0.0f;
            float xh = (zz - pb[2]) * pb[3];
            s1[n] += v;
            s2[n] = fmaf(v, xh, s2[n]);   // explicit: contraction left to -ffp-contract differed between kernels
          } else {
            s1[n] += v;
            s2[n] = fmaf(v, v, s2[n]);
          }
          g.out[(long long)row * g.CO_real + col] = v;
        }
      }
    }
  }
  if (EPI == E_PLAIN || g.part == nullptr) return;
  float* const sP = (float*)lds;   // aliases the ring: every wave is past its last step's reads
  __syncthreads();
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    s1[n] += __shfl_xor(s1[n], 16, 64);
    s1[n] += __shfl_xor(s1[n], 32, 64);
    s2[n] += __shfl_xor(s2[n], 16, 64);
    s2[n] += __shfl_xor(s2[n], 32, 64);
    if (lane < 16) {
      sP[w * 2 * NGP + n * 16 + lane] = s1[n];
      sP[w * 2 * NGP + NGP + n * 16 + lane] = s2[n];
    }
  }
  __syncthreads();
  const int C = g.CO_real;
  constexpr int WPR = 64 / WR, PRB = GBM / 64;
  const int nrow = (g.Nout + BM - 1) / BM;
  for (int j = tid; j < PRB * 2 * C; j += GBLK) {
    const int h = j / (2 * C), jj = j - h * 2 * C, prow = lb * PRB + h;
    if (prow >= nrow) continue;
    int which = jj / C, c = jj - which * C;
    float s = 0.0f;
    for (int ww = 0; ww < WPR; ++ww) s += sP[(WPR * h + ww) * 2 * NGP + which * NGP + c];
    if (g.fin.ticket)
      st_agent(&g.part[(long long)prow * 2 * C + jj], s);
    else
      g.part[(long long)prow * 2 * C + jj] = s;
  }
  if (g.fin.ticket) {
    // the ring is free: the totals (double [2C], C <= 256 -> 4 KB) and the arrival flag go there
    fused_bn_finalize<GBLK>(g, lb, PRB, (double*)(lds + 1024), (int*)(lds + 8192));
  }
}

// ------------------------------------------------------------------ elementwise producers
template <int FMT>
__global__ __launch_bounds__(BLK) void k_to_bf16(const float* __restrict__ z, const float* __restrict__ bn, int N,
                                                 int C, int CP, int relu, u16* __restrict__ h, u16* __restrict__ h2) {
  long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  if (t >= (long long)N * CP) return;
  int r = (int)(t / CP), c = (int)(t - (long long)r * CP);
  float v = 0.0f;
  if (c < C) {
    v = z[(long long)r * C + c];
    if (bn) v = fmaf(v - bn[2 * C + c], bn[c], bn[C + c]);   // (z - mean) * scale + beta
    if (relu) v = fmaxf(v, 0.0f);
  }
  h[t] = to_h16<FMT>(v);
  if (FMT && h2) h2[t] = to_bf16(v);
}

__global__ __launch_bounds__(BLK) void k_dz_bf16(const float* __restrict__ dy, const float* __restrict__ z,
                                                 const float* __restrict__ bnb, int N, int C, int CP,
                                                 u16* __restrict__ dz) {
  long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  if (t >= (long long)N * CP) return;
  int r = (int)(t / CP), c = (int)(t - (long long)r * CP);
  float v = 0.0f;
  if (c < C) {
    long long i = (long long)r * C + c;
    float xh = (z[i] - bnb[3 * C + c]) * bnb[4 * C + c];
    v = bnb[c] * (dy[i] - bnb[C + c] - xh * bnb[2 * C + c]);
  }
  dz[t] = to_bf16(v);
}

// 8-channel forms of the two producers for C % 8 == 0 (every bf16 layer): one thread per 8 channels of
// a row — two float4 loads per operand, BatchNorm parameters as float4, one 16-byte bf16 store, 32-bit
// index arithmetic (the scalar forms above spend their time in the 64-bit division t / CP). Same
// arithmetic per element, so the same bits.
__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <int FMT = 0>
__device__ __forceinline__ void st8h(u16* p, const float (&v)[8]) {
  u16 o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = to_h16<FMT>(v[j]);
  *(uint4*)p = *(const uint4*)o;
}

// Channel-group passes (C % 8 == 0, C / 8 divides BLK): thread = (row lane, 8-channel group), the group's
// BatchNorm parameters loaded once into registers, RV rows per thread in flight per iteration (one row per
// thread with the parameters re-read from L1 per row: the parameter loads were 2.5x the data bytes through
// the load path, k_dz_bf16_v8 ~3.7 TB/s)
constexpr int RV = 4;
__host__ __device__ inline int rowpass_blocks(long long n, int c) {
  const long long rl = BLK / (c / 8), per = rl * RV;
  const long long b = (n + per - 1) / per;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

template <int FMT>
__global__ __launch_bounds__(BLK) void k_to_bf16_v8(const float* __restrict__ z, const float* __restrict__ bn, int N,
                                                    int C, int relu, u16* __restrict__ h, u16* __restrict__ h2) {
  const int C8 = C >> 3, RL = BLK / C8;
  const int cg = threadIdx.x % C8, rl = threadIdx.x / C8, c = cg * 8;
  if (rl >= RL) return;
  float mu[8], sc[8], be[8];
  if (bn) {
    ld8f(bn + 2 * C + c, mu);
    ld8f(bn + c, sc);
    ld8f(bn + C + c, be);
  }
  const int step = gridDim.x * RL;
  for (int r0 = blockIdx.x * RL + rl; r0 < N; r0 += RV * step) {
    float v[RV][8];
#pragma unroll
    for (int u = 0; u < RV; ++u) ld8f(z + (size_t)min(r0 + u * step, N - 1) * C + c, v[u]);
#pragma unroll
    for (int u = 0; u < RV; ++u) {
      const int r = r0 + u * step;
      if (r >= N) break;
      if (bn) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[u][j] = fmaf(v[u][j] - mu[j], sc[j], be[j]);
      }
      if (relu) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[u][j] = fmaxf(v[u][j], 0.0f);
      }
      st8h<FMT>(h + (size_t)r * C + c, v[u]);
      if (FMT && h2) st8h<0>(h2 + (size_t)r * C + c, v[u]);   // + the bf16 rows the weight gradient gathers
    }
  }
}

__global__ __launch_bounds__(BLK) void k_dz_bf16_v8(const float* __restrict__ dy, const float* __restrict__ z,
                                                    const float* __restrict__ bnb, int N, int C,
                                                    u16* __restrict__ dz) {
  const int C8 = C >> 3, RL = BLK / C8;
  const int cg = threadIdx.x % C8, rl = threadIdx.x / C8, c = cg * 8;
  if (rl >= RL) return;
  float gi[8], m1[8], m2[8], mb[8], ib[8];
  ld8f(bnb + c, gi);
  ld8f(bnb + C + c, m1);
  ld8f(bnb + 2 * C + c, m2);
  ld8f(bnb + 3 * C + c, mb);
  ld8f(bnb + 4 * C + c, ib);
  const int step = gridDim.x * RL;
  for (int r0 = blockIdx.x * RL + rl; r0 < N; r0 += RV * step) {
    float d[RV][8], zz[RV][8];
#pragma unroll
    for (int u = 0; u < RV; ++u) {
      const size_t o = (size_t)min(r0 + u * step, N - 1) * C + c;
      ld8f(dy + o, d[u]);
      ld8f(z + o, zz[u]);
    }
#pragma unroll
    for (int u = 0; u < RV; ++u) {
      const int r = r0 + u * step;
      if (r >= N) break;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (zz[u][j] - mb[j]) * ib[j];
        v[j] = gi[j] * (d[u][j] - m1[j] - xh * m2[j]);
      }
      st8h(dz + (size_t)r * C + c, v);
    }
  }
}

// W fp32 [K][CI][CO] -> B^T bf16 [K][NGP][KGP]; fwd: n = co, kk = ci ; dgrad: n = ci, kk = co
__device__ __forceinline__ void wprep_elem(long long t, const float* __restrict__ W, int CI, int CO, int dgrad,
                                           int NGP, int KGP, u16* __restrict__ bt, int fmt = 0) {
  int kk = (int)(t % KGP);
  long long q = t / KGP;
  int n = (int)(q % NGP), k = (int)(q / NGP);
  float v = 0.0f;
  if (!dgrad) { if (n < CO && kk < CI) v = W[((long long)k * CI + kk) * CO + n]; }
  else { if (n < CI && kk < CO) v = W[((long long)k * CI + n) * CO + kk]; }
  bt[t] = fmt ? to_f16(v) : to_bf16(v);
}

__global__ __launch_bounds__(BLK) void k_wprep(const float* __restrict__ W, int K, int CI, int CO, int dgrad,
                                               int NGP, int KGP, u16* __restrict__ bt) {
  long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  if (t < (long long)K * NGP * KGP) wprep_elem(t, W, CI, CO, dgrad, NGP, KGP, bt);
}

// every layer (forward and data-gradient tiles) of an encoder in one launch: blockIdx.y = entry
constexpr int SWPREP_MAX = 32;
struct SWprepBatch {
  RpcSpconvWprep d[SWPREP_MAX];
};
__global__ __launch_bounds__(BLK) void k_wprep_batch(SWprepBatch b) {
  const RpcSpconvWprep& d = b.d[blockIdx.y];
  const int ng = d.dgrad ? d.ci : d.co, kg = d.dgrad ? d.co : d.ci;
  const int NGP = (ng + 15) / 16 * 16, KGP = (kg + 31) / 32 * 32;
  const long long t = (long long)blockIdx.x * BLK + threadIdx.x;
  if (t < (long long)d.kvol * NGP * KGP) wprep_elem(t, d.W, d.ci, d.co, d.dgrad, NGP, KGP, (u16*)d.bt, d.fmt);
}

// ------------------------------------------------------------------ weight gradient
// dW[k][ci][co] = sum_r h[nbr[r,k]][ci] * dz[r][co]. Block = (chunk of output rows, group of KG
// offsets). Rows are the K dimension of v_mfma_f32_16x16x32_bf16 (A = h^T, B = dz): per 64-row
// sub-tile the dz rows (shared by the KG offsets) and the gathered h rows are staged ROW-MAJOR
// in LDS (one ds_write_b128 per 16-B chunk) and read back column-wise with ds_read_b64_tr_b16.
// Row pitch = C + 16 elements and the (group, half, q) -> row map below make the transposed
// reads conflict-free for C = 32/64/128. The neighbour indices of 512 rows are preloaded into
// LDS so the gathers of sub-tile s+1 are issued (register staging) before the MFMAs of sub-tile s.
// Partial slabs [chunk][K][ci][co] are reduced in a fixed order by k_slab_reduce (common.h).
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ s16x4 tr_read(const u16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}

// 8 fp16 -> 8 bf16 (the fp16 forward rows of the perf mode, gathered by the bf16 weight gradient)
__device__ __forceinline__ uint4 f16x8_to_bf16x8(uint4 v) {
  const f16x8 h = __builtin_bit_cast(f16x8, v);
  u16 o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = to_bf16((float)h[j]);
  return *(const uint4*)o;
}

// weight-gradient block: 4 waves; 8 for the 128 x 128 tiles, whose 3 offsets per block (KG = 3) then fit
// 24 accumulator tiles per wave (192 VGPRs, no spill): each staged dz sub-tile serves 3 offsets instead
// of 1 — CenterPoint k_wgrad_bf16<128,128> 458 -> 403 us per launch (r04_step_kernels_centerpoint_wg3.txt;
// the step unchanged: these run on the side stream beside the data-gradient chain)
__host__ __device__ constexpr int wg_threads(int ci, int co) { return ci * co >= 128 * 128 ? 512 : 256; }
template <int CI, int CO, int KG, bool HF16 = false>
__global__ __launch_bounds__(wg_threads(CI, CO), (CI * CO <= 32 * 32) ? 4 : 1) void k_wgrad_bf16(const u16* __restrict__ h, int HP, const int* __restrict__ nbr,
                                                    int K, int N, int rows_per, const u16* __restrict__ dz, int DP,
                                                    float* __restrict__ part) {
  constexpr int TB = wg_threads(CI, CO), NWV = TB / 64;   // threads, waves
  constexpr int RT = 64;                                   // rows per sub-tile (2 MFMA k-steps)
  constexpr int SEG = 512;                                 // rows per neighbour preload
  constexpr int CIR = (CI + 15) / 16 * 16;
  constexpr int PA = CIR + 16, PD = CO + 16;               // LDS row pitch (elements)
  constexpr int MT = CIR / 16, NT = CO / 16;
  // NWV waves as WM x WN over the (ci, co) tiles: wave (wm, wn) owns m = wm + WM*a, n = wn + WN*b
  constexpr int WM = MT < 4 ? MT : 4, WN = NWV / WM;
  constexpr int WMT = MT / WM, WNT = (NT + WN - 1) / WN, TPW = WMT * WNT;
  constexpr int CA = (CI + 7) / 8, CD = CO / 8;            // 16-B chunks per row
  constexpr int NA = (RT * CA + TB - 1) / TB, ND = (RT * CD + TB - 1) / TB;
  __shared__ __attribute__((aligned(16))) u16 sA[KG][RT * PA];
  __shared__ __attribute__((aligned(16))) u16 sD[RT * PD];
  __shared__ int sN[SEG * KG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % WM, wn = w / WM;
  // 1-D grid over (chunk, offset group), XCD-aware: the groups of one row chunk are consecutive items on
  // one XCD, so its dz rows (read by every group) and its neighbours' h rows are fetched once into that
  // XCD's L2 (a 2-D grid dispatched a chunk's groups `chunks` blocks apart, after its rows were evicted)
  const int ngroups = (K + KG - 1) / KG;
  const int item = dn::xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = item / ngroups, k0 = (item - chunk * ngroups) * KG;
  const int rb0 = chunk * rows_per, rb1 = min(N, rb0 + rows_per);
  f32x4 acc[KG][TPW];
#pragma unroll
  for (int g = 0; g < KG; ++g)
#pragma unroll
    for (int i = 0; i < TPW; ++i) acc[g][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // zero the padded channels of the A tiles once (CI = 16 * MT always here, kept for safety)
  if (CIR != CI)
    for (int q = tid; q < KG * RT * PA; q += TB) (&sA[0][0])[q] = 0;
  // transposed-read lane geometry: group g4, lane i = 4q + p of the group
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int rowoff = 4 * g4 + qq;                          // + 16*half + 32*kstep
  uint4 ra[KG][NA], rd[ND];
  for (int seg = rb0; seg < rb1; seg += SEG) {
    const int se = min(rb1, seg + SEG);
    __syncthreads();
    {
      // all of a thread's index loads in flight at once, from clamped addresses (a guarded load per
      // pass compiled to a branch that waited for its load before the next pass: 2-6 round trips)
      // (32-bit buffer offsets; an index outside the map reads as -1 via the OOB-zero + select)
      constexpr int NQ = (SEG * KG + TB - 1) / TB;
      const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc((void*)nbr, (short)0, 0x7fffffff, 0x00020000);
      int v[NQ];
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        const int q = tid + i * TB, r = q / KG, g = q - r * KG, row = seg + r, k = k0 + g;
        unsigned off = (q < SEG * KG && row < se && k < K) ? (unsigned)(row * K + k) * 4u : 0x80000000u;
        asm volatile("" : "+v"(off));
        v[i] = off == 0x80000000u ? -1 : __builtin_amdgcn_raw_buffer_load_b32(rn, off, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < NQ; ++i)
        if (tid + i * TB < SEG * KG) sN[tid + i * TB] = v[i];
    }
    __syncthreads();
    auto load = [&](int rs) {   // global -> registers for the sub-tile starting at segment row rs
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        int q = tid + j * TB;
        rd[j] = make_uint4(0u, 0u, 0u, 0u);
        if (q < RT * CD) {
          int r = q / CD, c8 = q - r * CD, row = seg + rs + r;
          if (row < se) rd[j] = *(const uint4*)(dz + (long long)row * DP + c8 * 8);
        }
      }
#pragma unroll
      for (int g = 0; g < KG; ++g)
#pragma unroll
        for (int j = 0; j < NA; ++j) {
          int q = tid + j * TB;
          ra[g][j] = make_uint4(0u, 0u, 0u, 0u);
          if (q < RT * CA) {
            int r = q / CA, c8 = q - r * CA;
            int src = (rs + r < SEG) ? sN[(rs + r) * KG + g] : -1;
            if (src >= 0) ra[g][j] = *(const uint4*)(h + (long long)src * HP + c8 * 8);
          }
        }
    };
    load(0);
    for (int rs = 0; rs < se - seg; rs += RT) {
      __syncthreads();   // previous sub-tile's MFMAs are done with the LDS tiles
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        int q = tid + j * TB;
        if (q < RT * CD) {
          int r = q / CD, c8 = q - r * CD;
          *(uint4*)&sD[r * PD + c8 * 8] = rd[j];
        }
      }
#pragma unroll
      for (int g = 0; g < KG; ++g)
#pragma unroll
        for (int j = 0; j < NA; ++j) {
          int q = tid + j * TB;
          if (q < RT * CA) {
            int r = q / CA, c8 = q - r * CA;
            *(uint4*)&sA[g][r * PA + c8 * 8] = HF16 ? f16x8_to_bf16x8(ra[g][j]) : ra[g][j];
          }
        }
      // which offsets have any neighbour in this sub-tile (wave-uniform, from the LDS indices)
      bool any[KG];
#pragma unroll
      for (int g = 0; g < KG; ++g) any[g] = __ballot(sN[min(rs + lane, SEG - 1) * KG + g] >= 0 && rs + lane < SEG) != 0;
      __syncthreads();
      if (rs + RT < se - seg) load(rs + RT);               // in flight during the MFMAs below
#pragma unroll
      for (int ks = 0; ks < RT / 32; ++ks) {
        const int r0 = 32 * ks + rowoff;
        bf16x8 bv[WNT];                                    // dz fragments, shared by the KG offsets
#pragma unroll
        for (int b = 0; b < WNT; ++b) {
          const int n = wn + WN * b;
          s16x4 x[2] = {tr_read(&sD[r0 * PD + n * 16 + 4 * pp]), tr_read(&sD[(r0 + 16) * PD + n * 16 + 4 * pp])};
          bv[b] = *(bf16x8*)x;
        }
#pragma unroll
        for (int g = 0; g < KG; ++g) {
          if (!any[g]) continue;
#pragma unroll
          for (int a = 0; a < WMT; ++a) {
            const int m = wm + WM * a;
            s16x4 x[2] = {tr_read(&sA[g][r0 * PA + m * 16 + 4 * pp]),
                          tr_read(&sA[g][(r0 + 16) * PA + m * 16 + 4 * pp])};
            bf16x8 av = *(bf16x8*)x;
#pragma unroll
            for (int b = 0; b < WNT; ++b)
              acc[g][a * WNT + b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv[b], acc[g][a * WNT + b], 0, 0, 0);
          }
        }
      }
    }
  }
#pragma unroll
  for (int g = 0; g < KG; ++g) {
    int k = k0 + g;
    if (k >= K) break;
    float* out = part + ((long long)chunk * K + k) * CI * CO;
#pragma unroll
    for (int a = 0; a < WMT; ++a)
#pragma unroll
      for (int b = 0; b < WNT; ++b) {
        const int m = wm + WM * a, n = wn + WN * b;
        if (n >= NT) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int ci = m * 16 + (lane >> 4) * 4 + j, co = n * 16 + (lane & 15);
          if (ci < CI) out[ci * CO + co] = acc[g][a * WNT + b][j];
        }
      }
  }
}

// ------------------------------------------------------------------ r04: weight gradient over pair lists
// k_wgrad_bf16 walks every (row chunk, offset group) over ALL rows of the chunk: a row with no neighbour at
// offset k still costs its dz / h loads, staging and MFMA rows (sub-tiles are skipped only when none of
// their 64 rows has one). Here the neighbour map is first compacted into per-offset pair lists
// (k_pair_count -> one hipcub exclusive scan over the offset-major count table -> k_pair_scatter: pairs of
// offset k in ascending output-row order, deterministic), and the weight gradient runs over the pairs
// only: block b of S + K takes a slice of ONE offset's pairs, the offsets getting ceil(count_k * S / P)
// blocks each (balanced: ~P / S pairs per block whatever the offsets' counts), with dz rows gathered by the
// pair's output row and h rows by its input row, the same LDS staging / transposed reads / MFMA tiling as
// k_wgrad_bf16<., ., 1>. One fp32 partial per block (S + K partials instead of chunks x K), reduced per
// offset over its blocks in block order (k_pair_reduce).
constexpr int PRB = 256;   // rows per count / scatter block

// the block's PRB x K slice of nbr, staged into LDS with coalesced loads (each thread reading its own row's K
// entries straight from global memory strided the wave's 64 accesses over 64 rows: 103 us per 360k-row map)
__device__ __forceinline__ void stage_nbr(const int* __restrict__ nbr, int n, int K, int* snb) {
  const long long r0 = (long long)blockIdx.x * PRB;
  const int tot = (int)(min((long long)PRB, (long long)n - r0) * K);
  const int* src = nbr + r0 * K;
  int v[MAXK];   // all of the thread's loads in flight before the first LDS store
#pragma unroll
  for (int i = 0; i < MAXK; ++i) {
    const int q = threadIdx.x + i * PRB;
    v[i] = (i < K && q < tot) ? src[q] : -1;
  }
#pragma unroll
  for (int i = 0; i < MAXK; ++i)
    if (i < K) snb[threadIdx.x + i * PRB] = v[i];
}

__global__ __launch_bounds__(PRB) void k_pair_count(const int* __restrict__ nbr, int n, int K, int nb,
                                                    int* __restrict__ cnt) {
  __shared__ int snb[PRB * MAXK];
  __shared__ int sc[PRB / 64][MAXK];
  stage_nbr(nbr, n, K, snb);
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < K; ++k) {
    const unsigned long long m = __ballot(snb[threadIdx.x * K + k] >= 0);
    if (lane == 0) sc[w][k] = __popcll(m);
  }
  __syncthreads();
  if (threadIdx.x < K) {
    int c = 0;
    for (int ww = 0; ww < PRB / 64; ++ww) c += sc[ww][threadIdx.x];
    cnt[(long long)threadIdx.x * nb + blockIdx.x] = c;   // offset-major: the scan runs k by k
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) cnt[(long long)K * nb] = 0;   // the scan's total lands past it
}

__global__ __launch_bounds__(PRB) void k_pair_scatter(const int* __restrict__ nbr, int n, int K, int nb,
                                                      const int* __restrict__ base, int2* __restrict__ pairs) {
  __shared__ int snb[PRB * MAXK];
  __shared__ int sw[PRB / 64][MAXK];
  stage_nbr(nbr, n, K, snb);
  __syncthreads();
  const int r = blockIdx.x * PRB + threadIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int k = 0; k < K; ++k) {
    const unsigned long long m = __ballot(snb[threadIdx.x * K + k] >= 0);
    if (lane == 0) sw[w][k] = __popcll(m);
  }
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    const int src = snb[threadIdx.x * K + k];
    const unsigned long long m = __ballot(src >= 0);
    if (src < 0) continue;
    int pos = base[(long long)k * nb + blockIdx.x];
    for (int ww = 0; ww < w; ++ww) pos += sw[ww][k];
    pos += __popcll(m & below);
    pairs[pos] = make_int2(r, src);
  }
}

// the block -> (offset, slice) assignment every block and the reduce recompute from the K + 1 offsets
__device__ __forceinline__ void pair_blocks(const int* koff, int K, int S, int* kb) {
  const long long P = koff[K];
  kb[0] = 0;
  for (int k = 0; k < K; ++k) {
    const long long c = koff[k + 1] - koff[k];
    kb[k + 1] = kb[k] + (c > 0 ? (int)((c * S + P - 1) / P) : 0);
  }
}

template <int CI, int CO, bool HF16 = false>
__global__ __launch_bounds__(BLK, (CI * CO <= 32 * 32) ? 4 : 1) void k_wgrad_pairs(
    const u16* __restrict__ h, int HP, const int2* __restrict__ pairs, const int* __restrict__ base, int nb, int K,
    int S, const u16* __restrict__ dz, int DP, float* __restrict__ part) {
  constexpr int RT = 64, SEG = 512;
  constexpr int CIR = (CI + 15) / 16 * 16;
  constexpr int PA = CIR + 16, PD = CO + 16;
  constexpr int MT = CIR / 16, NT = CO / 16;
  constexpr int WM = MT < 4 ? MT : 4, WN = 4 / WM;
  constexpr int WMT = MT / WM, WNT = (NT + WN - 1) / WN, TPW = WMT * WNT;
  constexpr int CA = (CI + 7) / 8, CD = CO / 8;
  constexpr int NA = (RT * CA + BLK - 1) / BLK, ND = (RT * CD + BLK - 1) / BLK;
  __shared__ __attribute__((aligned(16))) u16 sA[RT * PA];
  __shared__ __attribute__((aligned(16))) u16 sD[RT * PD];
  __shared__ int2 sP[SEG];
  __shared__ int skoff[MAXK + 1], skb[MAXK + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % WM, wn = w / WM;
  if (tid <= K) skoff[tid] = base[(long long)tid * nb];
  __syncthreads();
  if (tid == 0) pair_blocks(skoff, K, S, skb);
  __syncthreads();
  const int b = blockIdx.x;
  if (b >= skb[K]) return;   // uniform: a spare block of the S + K grid
  int k = 0;
  while (skb[k + 1] <= b) ++k;
  const long long cnt = skoff[k + 1] - skoff[k];
  const int nbk = skb[k + 1] - skb[k], i = b - skb[k];
  const int p0 = skoff[k] + (int)(cnt * i / nbk), p1 = skoff[k] + (int)(cnt * (i + 1) / nbk);
  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (CIR != CI)
    for (int q = tid; q < RT * PA; q += BLK) sA[q] = 0;
  const int g4 = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  const int rowoff = 4 * g4 + qq;
  // register prefetch PF sub-tiles ahead: one. Two measured slower (64 x 64: 50.9 -> 57.6 us in the step,
  // CenterPoint 358 -> 409 us, profiles/r04_wgrad_pairs_ab.txt); kept as a compile-time choice
  constexpr int PF = 1;
  uint4 ra0[NA], rd0[ND], ra1[NA], rd1[ND];
  for (int seg = p0; seg < p1; seg += SEG) {
    const int se = min(p1, seg + SEG), len = se - seg;
    __syncthreads();
    for (int q = tid; q < SEG; q += BLK) sP[q] = q < len ? pairs[seg + q] : make_int2(-1, -1);
    __syncthreads();
    auto load = [&](int rs, uint4 (&ra)[NA], uint4 (&rd)[ND]) {
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const int q = tid + j * BLK;
        rd[j] = make_uint4(0u, 0u, 0u, 0u);
        if (q < RT * CD) {
          const int r = q / CD, c8 = q - r * CD;
          const int row = rs + r < SEG ? sP[rs + r].x : -1;
          if (row >= 0) rd[j] = *(const uint4*)(dz + (long long)row * DP + c8 * 8);
        }
      }
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int q = tid + j * BLK;
        ra[j] = make_uint4(0u, 0u, 0u, 0u);
        if (q < RT * CA) {
          const int r = q / CA, c8 = q - r * CA;
          const int src = rs + r < SEG ? sP[rs + r].y : -1;
          if (src >= 0) ra[j] = *(const uint4*)(h + (long long)src * HP + c8 * 8);
        }
      }
    };
    auto stage = [&](const uint4 (&ra)[NA], const uint4 (&rd)[ND]) {
      __syncthreads();   // the previous sub-tile's MFMAs are done with the LDS tiles
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        const int q = tid + j * BLK;
        if (q < RT * CD) {
          const int r = q / CD, c8 = q - r * CD;
          *(uint4*)&sD[r * PD + c8 * 8] = rd[j];
        }
      }
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int q = tid + j * BLK;
        if (q < RT * CA) {
          const int r = q / CA, c8 = q - r * CA;
          *(uint4*)&sA[r * PA + c8 * 8] = HF16 ? f16x8_to_bf16x8(ra[j]) : ra[j];
        }
      }
      __syncthreads();
    };
    auto mma = [&]() {
#pragma unroll
      for (int ks = 0; ks < RT / 32; ++ks) {
        const int r0 = 32 * ks + rowoff;
        bf16x8 bv[WNT];
#pragma unroll
        for (int bb = 0; bb < WNT; ++bb) {
          const int n = wn + WN * bb;
          s16x4 x[2] = {tr_read(&sD[r0 * PD + n * 16 + 4 * pp]), tr_read(&sD[(r0 + 16) * PD + n * 16 + 4 * pp])};
          bv[bb] = *(bf16x8*)x;
        }
#pragma unroll
        for (int a = 0; a < WMT; ++a) {
          const int m = wm + WM * a;
          s16x4 x[2] = {tr_read(&sA[r0 * PA + m * 16 + 4 * pp]), tr_read(&sA[(r0 + 16) * PA + m * 16 + 4 * pp])};
          const bf16x8 av = *(bf16x8*)x;
#pragma unroll
          for (int bb = 0; bb < WNT; ++bb)
            acc[a * WNT + bb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv[bb], acc[a * WNT + bb], 0, 0, 0);
        }
      }
    };
    load(0, ra0, rd0);
    if (PF == 2 && RT < len) load(RT, ra1, rd1);
    for (int rs = 0; rs < len; rs += RT * PF) {
      stage(ra0, rd0);
      if (rs + PF * RT < len) load(rs + PF * RT, ra0, rd0);   // in flight during the MFMAs below
      mma();
      if constexpr (PF == 2) {
        if (rs + RT >= len) break;
        stage(ra1, rd1);
        if (rs + 3 * RT < len) load(rs + 3 * RT, ra1, rd1);
        mma();
      }
    }
  }
  float* out = part + (long long)b * CI * CO;
#pragma unroll
  for (int a = 0; a < WMT; ++a)
#pragma unroll
    for (int bb = 0; bb < WNT; ++bb) {
      const int m = wm + WM * a, n = wn + WN * bb;
      if (n >= NT) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ci = m * 16 + (lane >> 4) * 4 + j, co = n * 16 + (lane & 15);
        if (ci < CI) out[ci * CO + co] = acc[a * WNT + bb][j];
      }
    }
}

// dW[k][e] = sum of the partials of offset k's blocks, in block order (8 interleaved sums, fixed combine)
__global__ __launch_bounds__(BLK) void k_pair_reduce(const float* __restrict__ part, const int* __restrict__ base,
                                                     int nb, int K, int S, long long per, float* __restrict__ dW) {
  __shared__ int skoff[MAXK + 1], skb[MAXK + 1];
  if (threadIdx.x <= K) skoff[threadIdx.x] = base[(long long)threadIdx.x * nb];
  __syncthreads();
  if (threadIdx.x == 0) pair_blocks(skoff, K, S, skb);
  __syncthreads();
  const long long e = (long long)blockIdx.x * BLK + threadIdx.x;
  if (e >= per * K) return;
  const int k = (int)(e / per);
  const long long j = e - (long long)k * per;
  const int b0 = skb[k], b1 = skb[k + 1];
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int bb = b0;
  for (; bb + 8 <= b1; bb += 8) {   // 8 loads in flight
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(long long)(bb + u) * per + j];
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += v[u];
  }
  for (int u = 0; bb < b1; ++bb, ++u) s[u] += part[(long long)bb * per + j];
  dW[e] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

template <int CI, int CO>
static int pairs_slots() {   // resident k_wgrad_pairs blocks on the device
  static int r = 0;
  if (r == 0) {
    int per = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_wgrad_pairs<CI, CO>, BLK, 0) != hipSuccess || per <= 0)
      per = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    r = per * cus;
  }
  return r;
}

template <int KGP, int NT>
static void launch_t(int epi, const GB& a, int n_rows, hipStream_t st) {
  constexpr int GW = gw_of(KGP, NT), GBM = 16 * rt_of(KGP, NT) * GW;
  const int nblk = (n_rows + GBM - 1) / GBM;
  if (a.fmt == 1)   // fp16 operands: forward GEMMs only (checked by gemm_bf16_launch)
    hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_FWD, 0, true>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else if (epi == E_FWD) hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_FWD>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else if (epi == E_DGRAD) hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_DGRAD>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else if (epi == E_RES) hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_RES>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_PLAIN>), dim3(nblk), dim3(64 * GW), 0, st, a);
}

template <int KGP, int NT, int GW, int S>
static void launch_pipe_t(int epi, const GB& a, int n_rows, hipStream_t st) {
  constexpr int GBM = PipeCfg<KGP, NT, GW, S>::GBM;
  const int nblk = (n_rows + GBM - 1) / GBM;
  if (epi == E_FWD) hipLaunchKernelGGL((k_gemm_pipe<KGP, NT, E_FWD, GW, S>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else if (epi == E_DGRAD) hipLaunchKernelGGL((k_gemm_pipe<KGP, NT, E_DGRAD, GW, S>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else hipLaunchKernelGGL((k_gemm_pipe<KGP, NT, E_PLAIN, GW, S>), dim3(nblk), dim3(64 * GW), 0, st, a);
}

// RPC_SPGEMM (A/B): 0 (default) = k_gemm_bf16 (one offset of look-ahead in registers, 4 blocks per CU);
// 1 = k_gemm_pipe, 8-wave blocks with a 4-stage ring; 2 = 4-wave blocks, 4 stages; 3 = 8-wave blocks,
// 3 stages (the 128-wide GEMM K always takes 4-wave blocks: 4 stages, 3 at 128 x 128). Measured on the
// metric's rulebooks (profiles/r04_spgemm_pipe_ab.txt): the ring is 2-2.6x SLOWER (<64,4,0> 87 vs 41 us,
// <64,4,1> 138 vs 53 us) — one block per CU keeps fewer bytes in flight than four blocks with one offset of
// register look-ahead each; kept for A/B. 4 + DBG: timing arms of k_gemm_bf16<64, 4, ·>.
static int g_gemm_mode = -1;
static int gemm_mode() {
  if (g_gemm_mode < 0) {
    const char* e = getenv("RPC_SPGEMM");
    int m = e ? atoi(e) : 0;
    g_gemm_mode = (m < 0 || m > 19) ? 0 : m;
  }
  return g_gemm_mode;
}

static int launch(int KGP, int NT, int epi, const GB& a, int n_rows, hipStream_t st) {
  int mode = gemm_mode();
#define C2(kg, nt)                                                  \
  if (KGP == kg && NT == nt) {                                      \
    if (mode == 0) launch_t<kg, nt>(epi, a, n_rows, st);            \
    else if (mode == 2) launch_pipe_t<kg, nt, 4, 4>(epi, a, n_rows, st); \
    else if (mode == 3) launch_pipe_t<kg, nt, 8, 3>(epi, a, n_rows, st); \
    else launch_pipe_t<kg, nt, 8, 4>(epi, a, n_rows, st);           \
    return RPC_OK;                                                  \
  }
#define C2W(kg, nt, s)                                              \
  if (KGP == kg && NT == nt) {                                      \
    if (mode == 0) launch_t<kg, nt>(epi, a, n_rows, st);            \
    else launch_pipe_t<kg, nt, 4, s>(epi, a, n_rows, st);           \
    return RPC_OK;                                                  \
  }
  // 128-wide GEMM K: 4-wave blocks (a 32 KB weight tile per stage at 128 x 128)
#define C2H(kg, nt)                                                 \
  if (KGP == kg && NT == nt) {                                      \
    if (mode == 0) launch_t<kg, nt>(epi, a, n_rows, st);            \
    else if (mode == 3) launch_pipe_t<kg, nt, 8, 3>(epi, a, n_rows, st); \
    else launch_pipe_t<kg, nt, 4, 4>(epi, a, n_rows, st);           \
    return RPC_OK;                                                  \
  }
  // 64-wide GEMM K with two row tiles per wave (rt_of): 4-wave blocks by default (8 x 4 KB of gathered rows
  // per stage would not fit 4 stages); 128-wide: 4-wave blocks (a 32 KB weight tile per stage at 128 x 128)
  if (epi == E_RES) mode = 0;   // the regular kernel only
  if (mode >= 4 && KGP == 64 && NT == 4) {   // timing arms of k_gemm_bf16 (DBG = mode - 4)
    const int nblk = (n_rows + 127) / 128;
#define DB(d)                                                                                              \
  if (mode - 4 == d) {                                                                                     \
    if (epi == E_FWD) hipLaunchKernelGGL((k_gemm_bf16<64, 4, E_FWD, d>), dim3(nblk), dim3(512), 0, st, a);   \
    else if (epi == E_DGRAD) hipLaunchKernelGGL((k_gemm_bf16<64, 4, E_DGRAD, d>), dim3(nblk), dim3(512), 0, st, a); \
    else hipLaunchKernelGGL((k_gemm_bf16<64, 4, E_PLAIN, d>), dim3(nblk), dim3(512), 0, st, a);              \
    return RPC_OK;                                                                                         \
  }
    DB(0) DB(1) DB(2) DB(3) DB(4) DB(5) DB(6) DB(7) DB(8) DB(9) DB(12) DB(13)
#undef DB
    return RPC_ERR_ARG;
  }
  if (mode >= 4 || a.fmt || a.perm) mode = 0;   // (the ring variants: bf16, natural row order only)
  C2(32, 1) C2(32, 2) C2(32, 4) C2H(64, 2) C2(64, 4) C2(64, 8) C2W(128, 4, 4) C2(32, 8) C2H(64, 1) C2W(128, 2, 4)
  C2W(128, 8, 3)
#undef C2H
#undef C2
#undef C2W
  return RPC_ERR_UNSUPPORTED;
}

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
static inline int r8(int c) { return (c + 7) / 8 * 8; }
static inline int r16(int c) { return (c + 15) / 16 * 16; }
static inline int r32(int c) { return (c + 31) / 32 * 32; }

}  // namespace spb
}  // namespace rpc

using namespace rpc;
using namespace rpc::spb;

// A/B and tests: select the sparse bf16 GEMM kernel (see gemm_mode); returns the previous mode
extern "C" int rpc_spconv_gemm_bf16_mode(int mode) {
  const int prev = gemm_mode();
  if (mode >= 0 && mode <= 19) g_gemm_mode = mode;
  return prev;
}

extern "C" int rpc_to_h16_rows(const float* z, const float* bn, int n, int c, int relu, int fmt, void* h,
                               void* h_bf16, void* stream) {
  if (n < 0 || c < 1 || (fmt != 0 && fmt != 1) || (h_bf16 && !fmt)) return RPC_ERR_ARG;
  if (n == 0) return RPC_OK;
  int cp = r8(c);
  hipStream_t st = (hipStream_t)stream;
  u16 *o = (u16*)h, *o2 = (u16*)h_bf16;
  if (c % 8 == 0 && BLK % (c / 8) == 0 && (long long)n * c < (1LL << 31)) {
    if (fmt) hipLaunchKernelGGL(k_to_bf16_v8<1>, dim3(rowpass_blocks(n, c)), dim3(BLK), 0, st, z, bn, n, c, relu, o, o2);
    else hipLaunchKernelGGL(k_to_bf16_v8<0>, dim3(rowpass_blocks(n, c)), dim3(BLK), 0, st, z, bn, n, c, relu, o, o2);
  } else {
    if (fmt)
      hipLaunchKernelGGL(k_to_bf16<1>, dim3(cdiv((long long)n * cp, BLK)), dim3(BLK), 0, st, z, bn, n, c, cp, relu, o, o2);
    else
      hipLaunchKernelGGL(k_to_bf16<0>, dim3(cdiv((long long)n * cp, BLK)), dim3(BLK), 0, st, z, bn, n, c, cp, relu, o, o2);
  }
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_to_bf16_rows(const float* z, const float* bn, int n, int c, int relu, void* h, void* stream) {
  return rpc_to_h16_rows(z, bn, n, c, relu, 0, h, nullptr, stream);
}

extern "C" int rpc_bnbwd_to_bf16_rows(const float* dy, const float* z, const float* bnb, int n, int c, void* dz,
                                      void* stream) {
  if (n < 0 || c < 1) return RPC_ERR_ARG;
  if (n == 0) return RPC_OK;
  int cp = r8(c);
  if (c % 8 == 0 && BLK % (c / 8) == 0 && (long long)n * c < (1LL << 31))
    hipLaunchKernelGGL(k_dz_bf16_v8, dim3(rowpass_blocks(n, c)), dim3(BLK), 0, (hipStream_t)stream, dy, z, bnb, n, c,
                       (u16*)dz);
  else
    hipLaunchKernelGGL(k_dz_bf16, dim3(cdiv((long long)n * cp, BLK)), dim3(BLK), 0, (hipStream_t)stream, dy, z, bnb,
                       n, c, cp, (u16*)dz);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" size_t rpc_spconv_bf16_weight_elems(int kvol, int ci, int co, int dgrad) {
  int ng = dgrad ? ci : co, kg = dgrad ? co : ci;
  return (size_t)kvol * r16(ng) * r32(kg);
}

extern "C" int rpc_spconv_prep_weight_bf16_batch(const RpcSpconvWprep* descs, int n, void* stream) {
  if (n < 0 || n > SWPREP_MAX || (n > 0 && !descs)) return RPC_ERR_ARG;
  if (n == 0) return RPC_OK;
  SWprepBatch b;
  memset(&b, 0, sizeof(b));
  long long most = 0;
  for (int i = 0; i < n; ++i) {
    const RpcSpconvWprep& d = descs[i];
    if (!d.W || !d.bt || d.kvol < 1 || d.kvol > MAXK || d.ci < 1 || d.co < 1) return RPC_ERR_ARG;
    b.d[i] = d;
    const long long e = (long long)rpc_spconv_bf16_weight_elems(d.kvol, d.ci, d.co, d.dgrad);
    most = e > most ? e : most;
  }
  hipLaunchKernelGGL(k_wprep_batch, dim3(cdiv(most, BLK), n), dim3(BLK), 0, (hipStream_t)stream, b);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_spconv_prep_weight_bf16(const float* W, int kvol, int ci, int co, int dgrad, void* bt,
                                           void* stream) {
  int ng = dgrad ? ci : co, kg = dgrad ? co : ci;
  long long n = (long long)kvol * r16(ng) * r32(kg);
  hipLaunchKernelGGL(k_wprep, dim3(cdiv(n, BLK)), dim3(BLK), 0, (hipStream_t)stream, W, kvol, ci, co, dgrad, r16(ng),
                     r32(kg), (u16*)bt);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

// out[r] = sum_k a[map[r, k']] . B_k  with a: bf16 rows of width round8(kg) (kg = GEMM K),
// B^T from rpc_spconv_prep_weight_bf16; epi 0 = forward (z + BN partial sums), 1 = dgrad with the
// previous layer's ReLU mask + BN-backward partial sums (prev_z, prev_bn), 2 = plain store.
static int gemm_bf16_launch(GB& g, const void* a, int n_src, int kg, const int* map, int kvol, int rev, int n_out,
                            const void* bt, int ng, float* out, const float* prev_z, const float* prev_bn, float* part,
                            int epi, void* stream) {
  if (n_out < 0 || kvol > MAXK || kg < 1 || ng < 1) return RPC_ERR_ARG;
  // 32-bit buffer offsets (src * CP + c) * 2 into the gathered source table of n_src rows
  if (n_src >= 0 && (long long)n_src * r8(kg) * 2 >= (1LL << 31)) return RPC_ERR_UNSUPPORTED;
  if (n_out == 0) return RPC_OK;
  if (g.fmt != 0 && (g.fmt != 1 || epi != E_FWD)) return RPC_ERR_UNSUPPORTED;
  g.a = (const u16*)a;
  g.CP = r8(kg);
  g.nbr = map;
  g.K = kvol;
  g.rev = rev;
  g.bt = (const u16*)bt;
  g.Nout = n_out;
  g.out = out;
  g.CO_real = ng;
  g.ez = prev_z;
  g.ebn = prev_bn;
  g.part = part;
  // 32-bit buffer offsets in k_gemm_bf16: the output rows (epilogue) and weight tiles; the source table's
  // rows are checked above when the caller passes them (n_src < 0: the legacy entry point, which bounds
  // the source by n_out rows — exact for submanifold layers only)
  if ((long long)(n_src >= 0 ? std::max(n_src, n_out) : n_out) * g.CP * 2 >= (1LL << 31) ||
      (long long)kvol * r16(ng) * r32(kg) * 2 >= (1LL << 31))
    return RPC_ERR_UNSUPPORTED;
  int rc = launch(r32(kg), r16(ng) / 16, epi, g, n_out, (hipStream_t)stream);
  if (rc) return rc;
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_spconv_gemm_bf16_n(const void* a, int n_src, int kg, const int* map, int kvol, int rev,
                                      int n_out, const void* bt, int ng, float* out, const float* prev_z,
                                      const float* prev_bn, float* part, int epi, void* stream) {
  GB g;
  memset(&g, 0, sizeof(g));
  return gemm_bf16_launch(g, a, n_src, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part, epi, stream);
}

// the forward GEMM on 16-bit operands of either format (fmt RPC_H16_BF16 / RPC_H16_F16); other epilogues bf16
extern "C" int rpc_spconv_gemm_h16(const void* a, int fmt, int n_src, int kg, const int* map, int kvol, int rev,
                                   int n_out, const void* bt, int ng, float* out, const float* prev_z,
                                   const float* prev_bn, float* part, int epi, void* stream) {
  GB g;
  memset(&g, 0, sizeof(g));
  g.fmt = fmt;
  return gemm_bf16_launch(g, a, n_src, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part, epi, stream);
}

// the general form: operand format fmt (fp16: forward only) and rows visited in the order perm (may be NULL)
extern "C" int rpc_spconv_gemm_perm(const void* a, int fmt, int n_src, int kg, const int* map, int kvol, int rev,
                                    const int* perm, int n_out, const void* bt, int ng, float* out,
                                    const float* prev_z, const float* prev_bn, float* part, int epi, void* stream) {
  GB g;
  memset(&g, 0, sizeof(g));
  g.fmt = fmt;
  g.perm = perm;
  return gemm_bf16_launch(g, a, n_src, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part, epi, stream);
}

// the data gradient into a basicblock's output rows with rpc_sparse_res_backward fused into its epilogue:
// m = (dgrad + g2) * [out > 0] -> m [n_out][ng] fp32, and the BatchNorm-backward partial rows (sum m,
// sum m * (z - mean) * invstd) of that layer (bn: scale, beta, mean, invstd) -> part [gemm blocks][2 * ng]
extern "C" int rpc_spconv_gemm_res(const void* a, int n_src, int kg, const int* map, int kvol, int rev,
                                   const int* perm, int n_out, const void* bt, int ng, float* m, const float* g2,
                                   const float* out, const float* z, const float* bn, float* part,
                                   const RpcBnFin* fin, void* stream) {
  if (!m || !out || !z || !bn || !part) return RPC_ERR_ARG;
  if (fin && (fin->mode != 1 || !fin->ticket || !fin->gpart || !fin->gamma || !fin->fbn || !fin->bn || ng > 256 ||
              n_out <= 0))
    return RPC_ERR_ARG;
  GB g;
  memset(&g, 0, sizeof(g));
  if (fin) g.fin = *fin;   // + that layer's BatchNorm-backward finalize (mode 1) in the last-arriving blocks
  g.perm = perm;
  g.eg2 = g2;
  g.eout = out;
  return gemm_bf16_launch(g, a, n_src, kg, map, kvol, rev, n_out, bt, ng, m, z, bn, part, E_RES, stream);
}

// largest block of the k_gemm_pipe launches (rows): fin_groups of n_out at the smallest block (64 rows)
extern "C" int rpc_bn_fin_groups(int n_out) { return fin_groups(cdiv(n_out > 0 ? n_out : 1, 64)); }
extern "C" int rpc_bn_fin_tickets(int n_out) { return 1 + rpc_bn_fin_groups(n_out); }

// the fused-finalize GEMM on 16-bit operands of either format (fp16: the forward, epi 0, only)
extern "C" int rpc_spconv_gemm_h16_fin(const void* a, int fmt, int n_src, int kg, const int* map, int kvol, int rev,
                                       int n_out, const void* bt, int ng, float* out, const float* prev_z,
                                       const float* prev_bn, float* part, int epi, const RpcBnFin* fin, void* stream) {
  if (fmt != 0 && (fmt != 1 || epi != 0)) return RPC_ERR_ARG;
  if (!fin) return rpc_spconv_gemm_h16(a, fmt, n_src, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part,
                                       epi, stream);
  if ((epi != 0 && epi != 1) || !part || !fin->ticket || !fin->gpart || !fin->gamma || !fin->bn ||
      (epi == 0 && (!fin->beta || !fin->running_mean || !fin->running_var)) || (epi == 1 && !fin->fbn) ||
      fin->mode != epi || ng > 256)
    return RPC_ERR_ARG;
  if (n_out <= 0) return RPC_ERR_ARG;   // the finalize divides by the row count
  if (gemm_mode() >= 4) {   // the timing arms of k_gemm_bf16: no fused finalize
    int rc = rpc_spconv_gemm_h16(a, fmt, n_src, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part, epi,
                                 stream);
    if (rc) return rc;
    return rpc_bn_finalize(part, cdiv(n_out, BM), ng, n_out, epi, fin->gamma, fin->beta, fin->eps, fin->momentum,
                           fin->running_mean, fin->running_var, fin->fbn, fin->bn, fin->dgamma, fin->dbeta, nullptr,
                           stream);
  }
  GB g;
  memset(&g, 0, sizeof(g));
  g.fmt = fmt;
  g.fin = *fin;
  return gemm_bf16_launch(g, a, n_src, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part, epi, stream);
}

extern "C" int rpc_spconv_gemm_bf16_fin(const void* a, int n_src, int kg, const int* map, int kvol, int rev,
                                        int n_out, const void* bt, int ng, float* out, const float* prev_z,
                                        const float* prev_bn, float* part, int epi, const RpcBnFin* fin,
                                        void* stream) {
  return rpc_spconv_gemm_h16_fin(a, 0, n_src, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part, epi, fin,
                                 stream);
}

extern "C" int rpc_spconv_gemm_bf16(const void* a, int kg, const int* map, int kvol, int rev, int n_out,
                                    const void* bt, int ng, float* out, const float* prev_z, const float* prev_bn,
                                    float* part, int epi, void* stream) {
  return rpc_spconv_gemm_bf16_n(a, -1, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part, epi, stream);
}

template <int CI, int CO, int KG>
static int wgrad_resident() {   // resident blocks per CU of one k_wgrad_bf16 instantiation
  static int r = 0;
  if (r == 0 && (hipOccupancyMaxActiveBlocksPerMultiprocessor(&r, k_wgrad_bf16<CI, CO, KG>, wg_threads(CI, CO), 0) != hipSuccess ||
                 r <= 0))
    r = 1;
  return r;
}

static int wgrad_slots(int ci, int co) {   // resident blocks on the whole device
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  int per = 1;
#define WR(a, b, kg) if (ci == a && co == b) per = wgrad_resident<a, b, kg>(); else
  WR(16, 16, 3) WR(16, 32, 3) WR(32, 32, 3) WR(32, 64, 3) WR(64, 64, 3) WR(64, 128, 3) WR(128, 128, 3) {}
#undef WR
  return per * cus;
}

static int wgrad_kg(int ci, int co) { (void)ci; (void)co; return 3; }

static int wgrad_fill() {   // RPC_SPWG_FILL (A/B): percent of one round of resident blocks, 0 = 512-row chunks
  static int r = -1;
  if (r < 0) {
    const char* e = getenv("RPC_SPWG_FILL");
    r = e ? atoi(e) : 100;
    if (r < 0) r = 100;
  }
  return r;
}

// row chunks: as many as one round of the resident blocks holds (chunks x offset groups <= slots), at
// least 256 rows each. Every chunk writes a [K][ci][co] fp32 partial slab that k_slab_reduce reads back:
// with ~512-row chunks over 3 rounds the 106k-row 64 x 64 layers wrote and re-read 75 MB of slabs per
// launch on the side stream, which slowed the data-gradient chain beside it (step 827 -> 833 frames/s
// with one round, profiles/r03_spwg_ab.log; 60 % / 35 % of a round measured equal / slower).
// RPC_SPWG_FILL=0: the former ~512-row chunks trimmed to whole rounds.
static int wgrad_chunks(int n, int kvol, int ci, int co) {
  const int groups = (kvol + wgrad_kg(ci, co) - 1) / wgrad_kg(ci, co);
  const long long slots = wgrad_slots(ci, co);
  const int R = wgrad_fill();
  if (R > 0) {
    long long c = (long long)R * slots / (100 * groups);
    const long long cmax = (n + 255) / 256;
    if (c > cmax) c = cmax;
    if (c > 512) c = 512;
    return c < 1 ? 1 : (int)c;
  }
  int c = (n + 511) / 512;
  c = c < 1 ? 1 : (c > 512 ? 512 : c);
  const long long total = (long long)c * groups;
  if (total > slots) {
    const long long rounds = total / slots;
    const int c2 = (int)(rounds * slots / groups);
    if (c2 >= 1 && c2 < c) c = c2;
  }
  return c;
}

static int pairs_slots_dyn(int ci, int co) {
#define PS(a, b) if (ci == a && co == b) return pairs_slots<a, b>();
  PS(16, 16) PS(16, 32) PS(32, 32) PS(32, 64) PS(64, 64) PS(64, 128) PS(128, 128)
#undef PS
  return 0;
}

struct PairWs {
  int* cnt;
  int* base;
  void* scan_tmp;
  size_t scan_bytes;
  int2* pairs;
  float* part;
  size_t total;
};

static int pair_ws(int n_out, int kvol, int ci, int co, char* w, PairWs* o) {
  const int S = pairs_slots_dyn(ci, co);
  if (S <= 0) return RPC_ERR_UNSUPPORTED;
  const int nb = cdiv(n_out > 0 ? n_out : 1, PRB);
  const long long nc = (long long)kvol * nb + 1;
  size_t scan_b = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (const int*)nullptr, (int*)nullptr, (int)nc, (hipStream_t)0) !=
      hipSuccess)
    return RPC_ERR_HIP;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  size_t off = 0;
  o->cnt = (int*)(w + off);
  off += al(sizeof(int) * nc);
  o->base = (int*)(w + off);
  off += al(sizeof(int) * nc);
  o->scan_tmp = w + off;
  o->scan_bytes = scan_b;
  off += al(scan_b);
  o->pairs = (int2*)(w + off);
  off += al(sizeof(int2) * (size_t)(n_out > 0 ? n_out : 1) * kvol);
  o->part = (float*)(w + off);
  off += al(sizeof(float) * (size_t)(S + kvol) * ci * co);
  o->total = off;
  return RPC_OK;
}

extern "C" size_t rpc_spconv_wgrad_pairs_workspace_size(int n_out, int kvol, int ci, int co) {
  PairWs o;
  if (n_out < 0 || kvol < 1 || kvol > MAXK || pair_ws(n_out, kvol, ci, co, nullptr, &o)) return 0;
  return o.total;
}

// the same weight gradient as rpc_spconv_wgrad_h16 over per-offset pair lists built from nbr here
extern "C" int rpc_spconv_wgrad_pairs(const void* h, int hfmt, int ci, const int* nbr, int kvol, int n_out,
                                      const void* dz, int co, float* dW, void* ws, size_t ws_bytes, void* stream) {
  if (hfmt != 0 && hfmt != 1) return RPC_ERR_ARG;
  if (n_out < 0 || kvol < 1 || kvol > MAXK || !h || !nbr || !dz || !dW || !ws) return RPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (n_out == 0) {
    RPC_CHECK(hipMemsetAsync(dW, 0, sizeof(float) * (size_t)kvol * ci * co, st));
    return RPC_OK;
  }
  if ((long long)n_out * kvol >= (1LL << 31)) return RPC_ERR_UNSUPPORTED;
  PairWs o;
  int rc = pair_ws(n_out, kvol, ci, co, (char*)ws, &o);
  if (rc) return rc;
  if (ws_bytes < o.total) return RPC_ERR_WORKSPACE;
  const int S = pairs_slots_dyn(ci, co), nb = cdiv(n_out, PRB);
  const int nc = kvol * nb + 1;
  hipLaunchKernelGGL(k_pair_count, dim3(nb), dim3(PRB), 0, st, nbr, n_out, kvol, nb, o.cnt);
  RPC_LAUNCH_CHECK();
  size_t sb = o.scan_bytes;
  if (hipcub::DeviceScan::ExclusiveSum(o.scan_tmp, sb, o.cnt, o.base, nc, st) != hipSuccess) return RPC_ERR_HIP;
  hipLaunchKernelGGL(k_pair_scatter, dim3(nb), dim3(PRB), 0, st, nbr, n_out, kvol, nb, (const int*)o.base, o.pairs);
  RPC_LAUNCH_CHECK();
  const u16* hp = (const u16*)h;
  const u16* dp = (const u16*)dz;
  const int HP = r8(ci), DP = r8(co);
  const dim3 grid(S + kvol);
#define W2(a, b)                                                                                              \
  if (ci == a && co == b) {                                                                                  \
    if (hfmt)                                                                                                \
      hipLaunchKernelGGL((k_wgrad_pairs<a, b, true>), grid, dim3(BLK), 0, st, hp, HP, (const int2*)o.pairs,    \
                         (const int*)o.base, nb, kvol, S, dp, DP, o.part);                                    \
    else                                                                                                     \
      hipLaunchKernelGGL((k_wgrad_pairs<a, b>), grid, dim3(BLK), 0, st, hp, HP, (const int2*)o.pairs,          \
                         (const int*)o.base, nb, kvol, S, dp, DP, o.part);                                    \
  } else
  W2(16, 16) W2(16, 32) W2(32, 32) W2(32, 64) W2(64, 64) W2(64, 128) W2(128, 128)
  { return RPC_ERR_UNSUPPORTED; }
#undef W2
  RPC_LAUNCH_CHECK();
  const long long per = (long long)ci * co;
  hipLaunchKernelGGL(k_pair_reduce, dim3((unsigned)((per * kvol + BLK - 1) / BLK)), dim3(BLK), 0, st,
                     (const float*)o.part, (const int*)o.base, nb, kvol, S, per, dW);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_spconv_wgrad_pairs(const void* h, int hfmt, int ci, const int* nbr, int kvol, int n_out,
                                      const void* dz, int co, float* dW, void* ws, size_t ws_bytes, void* stream);
// RPC_SPWG_PAIRS=1 (A/B): the pair-list weight gradient behind rpc_spconv_wgrad_h16. Off by default: measured
// on the step (profiles/r04_wgrad_pairs_ab.txt) the weight-gradient kernel gets only 10-25 % faster
// (k_wgrad_bf16<64,64,3> 69.6 -> 50.9 us; CenterPoint <128,128> 449 -> 354 us) — rows without a neighbour
// at an offset were cheap already (contiguous dz rows, no h gather, zero MFMA rows) and the time is the
// per-sub-tile gather round trip, which the pairs keep — while the compaction (count + scan + scatter per
// layer: 10-50 us) and the per-offset reduce eat the gain: SECOND 7.16 -> 7.65 ms/step, CenterPoint
// 150.0 -> 147.1 frames/s
static bool wgrad_pairs_mode() {
  static int m = -1;
  if (m < 0) {
    const char* e = getenv("RPC_SPWG_PAIRS");
    m = (e && atoi(e) != 0) ? 1 : 0;
  }
  return m == 1;
}

extern "C" size_t rpc_spconv_wgrad_bf16_workspace_size(int n_out, int kvol, int ci, int co) {
  if (wgrad_pairs_mode() && pairs_slots_dyn(ci, co) > 0) return rpc_spconv_wgrad_pairs_workspace_size(n_out, kvol, ci, co);
  return (size_t)wgrad_chunks(n_out, kvol, ci, co) * kvol * ci * co * sizeof(float);
}

// dW[k] = sum_r h[nbr[r,k]]^T dz[r] with 16-bit rows h [.][round8(ci)] (hfmt: bf16, or fp16 forward rows,
// rounded to bf16 as they are staged) and bf16 dz [n_out][round8(co)]
extern "C" int rpc_spconv_wgrad_h16(const void* h, int hfmt, int ci, const int* nbr, int kvol, int n_out,
                                    const void* dz, int co, float* dW, void* ws, size_t ws_bytes, void* stream);
extern "C" int rpc_spconv_wgrad_bf16(const void* h, int ci, const int* nbr, int kvol, int n_out, const void* dz,
                                     int co, float* dW, void* ws, size_t ws_bytes, void* stream) {
  return rpc_spconv_wgrad_h16(h, 0, ci, nbr, kvol, n_out, dz, co, dW, ws, ws_bytes, stream);
}

extern "C" int rpc_spconv_wgrad_h16(const void* h, int hfmt, int ci, const int* nbr, int kvol, int n_out,
                                    const void* dz, int co, float* dW, void* ws, size_t ws_bytes, void* stream) {
  if (hfmt != 0 && hfmt != 1) return RPC_ERR_ARG;
  if (n_out < 0 || kvol < 1 || kvol > MAXK) return RPC_ERR_ARG;
  if (wgrad_pairs_mode() && pairs_slots_dyn(ci, co) > 0)
    return rpc_spconv_wgrad_pairs(h, hfmt, ci, nbr, kvol, n_out, dz, co, dW, ws, ws_bytes, stream);
  bool ok = (ci == 16 && (co == 16 || co == 32)) || (ci == 32 && (co == 32 || co == 64)) ||
            (ci == 64 && (co == 64 || co == 128)) || (ci == 128 && co == 128);
  if (!ok) return RPC_ERR_UNSUPPORTED;
  hipStream_t st = (hipStream_t)stream;
  if (n_out == 0) {
    RPC_CHECK(hipMemsetAsync(dW, 0, sizeof(float) * (size_t)kvol * ci * co, st));
    return RPC_OK;
  }
  // 32-bit buffer offsets: the index staging reads nbr[(row * kvol + k)] as bytes (row * K + k) * 4
  if ((long long)n_out * kvol * 4 >= (1LL << 31)) return RPC_ERR_UNSUPPORTED;
  int chunks = wgrad_chunks(n_out, kvol, ci, co);
  if (ws_bytes < (size_t)chunks * kvol * ci * co * sizeof(float)) return RPC_ERR_WORKSPACE;
  int rows_per = ((n_out + chunks - 1) / chunks + 31) / 32 * 32;
  // 3 kernel offsets per block share each staged dz sub-tile (the 128 x 128 tiles with 8 waves: 24
  // accumulator tiles per wave)
  const int KG = wgrad_kg(ci, co);
  dim3 grid(chunks * ((kvol + KG - 1) / KG));
  float* part = (float*)ws;
  const u16* hp = (const u16*)h;
  const u16* dp = (const u16*)dz;
  int HP = r8(ci), DP = r8(co);
#define W2(a, b, kg)                                                                                   \
  if (ci == a && co == b) {                                                                           \
    if (hfmt)                                                                                         \
      hipLaunchKernelGGL((k_wgrad_bf16<a, b, kg, true>), grid, dim3(wg_threads(a, b)), 0, st, hp, HP, nbr, kvol, n_out, \
                         rows_per, dp, DP, part);                                                     \
    else                                                                                              \
      hipLaunchKernelGGL((k_wgrad_bf16<a, b, kg>), grid, dim3(wg_threads(a, b)), 0, st, hp, HP, nbr, kvol, n_out, rows_per, dp, \
                         DP, part);                                                                   \
  } else
  W2(16, 16, 3) W2(16, 32, 3) W2(32, 32, 3) W2(32, 64, 3) W2(64, 64, 3) W2(64, 128, 3) W2(128, 128, 3)
  { return RPC_ERR_UNSUPPORTED; }
#undef W2
  RPC_LAUNCH_CHECK();
  long long total = (long long)kvol * ci * co;
  slab_reduce(part, chunks, total, dW, st);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
