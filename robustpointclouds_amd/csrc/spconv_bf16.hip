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
#include <type_traits>

#include "common.h"
#include <stdlib.h>
#include <hipcub/hipcub.hpp>
#include "dense_common.h"
#include "rpc_hip.h"

namespace rpc {
namespace spb {

constexpr int BLK = 256;
constexpr int BM = 64;          // rows per BatchNorm partial row (rpc_spconv_gemm_blocks)
// GEMM waves per block (16 x RT rows each; all share one LDS weight tile per step): 8 — the tile is
// fetched once per 128 rows — except the 128 x 128 tiles: 4 waves of 32 rows
__host__ __device__ constexpr int gw_of(int kgp, int nt) { return kgp * nt * 16 >= 128 * 128 ? 4 : 8; }
// 16-row MFMA tiles per wave: every weight fragment a wave reads from LDS feeds RT MFMAs. Two for the
// mid-size tiles (K x 16*NT of 32x32 .. 64x32), whose time went to LDS weight reads (every wave re-read
// the whole tile per offset for its 16 rows): r02v30 <32,2,0> 35.0 -> 30.0 us, <32,2,1> 38.5 -> 36.5,
// <64,2,1> 49 -> 42. Measured and kept at RT=1: the 64x64 tiles (88 VGPRs, 5 waves/SIMD: <64,4,1>
// 47 -> 54 us) and the 32x16 tiles (<32,1,0> 21.3 -> 23.4 us). The 128 x 128 tiles (CenterPoint) take two
// (r04, then one 128-row block per CU: forward 259 -> 262, data gradient 624 -> 606, plain 407 -> 370 us per
// launch, profiles/r04_step_kernels_centerpoint_rt2.txt; since r05 two blocks per CU, see ksplit_of)
__host__ __device__ constexpr int rt_of(int kgp, int nt) {
  return ((kgp * nt >= 64 && kgp * nt <= 128 && nt <= 4) || (kgp == 128 && nt == 8)) ? 2 : 1;
}
// K halves per offset step: the 128 x 128 tiles stage their weight tile half a K at a time (2 x 20 KB of LDS
// instead of 2 x 34 KB), so two 128-row blocks share a CU (r05: one, with 88 KB of LDS and 262 VGPRs — the
// launch was bound by the rows one block keeps in flight: 4 x 32-row and 8 x 16-row wave layouts timed the same).
// Standalone 279 -> 190 us per launch, CenterPoint 179-180 -> 188-189 frames/s (profiles/r05_gemm128_ksplit_ab.txt)
__host__ __device__ constexpr int ksplit_of(int kgp, int nt) { return (kgp == 128 && nt == 8) ? 2 : 1; }
__host__ __device__ constexpr int gemm_waves_per_simd(int kgp, int nt) {
  return kgp * nt >= 1024 ? 2 : rt_of(kgp, nt) == 2 ? 5 : ((kgp * nt <= 256 && nt <= 4 && kgp <= 64) ? 8 : 1);
}
constexpr int MAXK = 27;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16;

__device__ __forceinline__ u16 to_bf16(float f) {
  __bf16 b = (__bf16)f;   // round-to-nearest-even, NaN kept (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(u16, b);
}
// finite values beyond the fp16 range saturate to +-65504 instead of becoming inf (which the MFMA and the
// BatchNorm sums would turn into NaN); inf / NaN pass through as they would in bf16
__device__ __forceinline__ float sat_f16(float f) {
  return (fabsf(f) > 65504.0f && fabsf(f) < __builtin_inff()) ? copysignf(65504.0f, f) : f;
}
__device__ __forceinline__ u16 to_f16(float f) {
  _Float16 h = (_Float16)sat_f16(f);   // round-to-nearest-even (v_cvt_f16_f32)
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
  const float* eg2;   // E_RES: the other gradient contribution [Nout][CO_real] (identity path) or null
  const float* eout;  // E_RES: the block output rows [Nout][CO_real] (ReLU mask)
};

// ---- BatchNorm finalize fused into the GEMM (RpcBnFin, data gradients): the partial rows every block writes
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
  for (int c = threadIdx.x; c < C; c += NTHR) {   // rpc_bn_finalize mode 1
    const double s1 = sh[c], s2 = sh[C + c];
    f.bn[c] = f.gamma[c] * f.fbn[3 * C + c];
    f.bn[C + c] = (float)(s1 / N);
    f.bn[2 * C + c] = (float)(s2 / N);
    f.bn[3 * C + c] = f.fbn[2 * C + c];
    f.bn[4 * C + c] = f.fbn[3 * C + c];
    if (f.dgamma) f.dgamma[c] = (float)s2;
    if (f.dbeta) f.dbeta[c] = (float)s1;
  }
}

// Occupancy: the <= 64 x 64 tiles are held to 64 VGPRs (8 waves per SIMD, 4 blocks per CU) — at 72 the
// 106k-row 64-channel layers needed 1.08 rounds of 3 blocks per CU (k_gemm_bf16<64,4,1> 60.6 -> 51.5 us)
template <int KGP, int NT, int EPI, bool F16 = false>
__global__ __launch_bounds__(64 * gw_of(KGP, NT), gemm_waves_per_simd(KGP, NT)) void k_gemm_bf16(GB g) {
  constexpr int RT = rt_of(KGP, NT), GW = gw_of(KGP, NT), GBLK = 64 * GW, WR = 16 * RT, GBM = WR * GW;
  constexpr int KS = KGP / 32;
  constexpr int NGP = NT * 16;
  constexpr int KSP = ksplit_of(KGP, NT), KGH = KGP / KSP, KSH = KS / KSP;   // K halves per offset step
  // LDS row stride: 8 mod 16 dwords (conflict-free b128 reads)
  constexpr int LS = KGH + 16;
  constexpr int BV = NGP * KGH / 8;           // 16-B vectors per step's weight tile
  constexpr int BPT = (BV + GBLK - 1) / GBLK;
  __shared__ __attribute__((aligned(16))) u16 sB[2][NGP * LS];
  __shared__ int sN[GBM * MAXK];
  __shared__ unsigned wmask[GW];
  __shared__ int klist[MAXK];
  __shared__ int nk;
  __shared__ float sP[GW][2 * NGP];
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
  constexpr unsigned OOB = 0x80000000u;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)g.a, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)g.bt, (short)0, 0x7fffffff, 0x00020000);
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
  auto load_b = [&](int k, int kh, uint4 (&dst)[BPT]) {
    const unsigned base = (unsigned)k * (unsigned)(NGP * KGP * 2) + (unsigned)(kh * KGH * 2);
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      const int v = tid + j * GBLK, e = v * 8, n = e / KGH, c = e - n * KGH;
      unsigned off = (BV % GBLK == 0 || v < BV) ? base + (unsigned)(n * KGP + c) * 2u : OOB;
      asm volatile("" : "+v"(off));
      dst[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsb, off, 0, 0));
    }
  };
  auto store_b = [&](int buf, const uint4 (&src)[BPT]) {
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      int v = tid + j * GBLK;
      if (BV % GBLK == 0 || v < BV) {
        int e = v * 8, n = e / KGH, c = e - n * KGH;
        *(uint4*)&sB[buf][n * LS + c] = src[j];
      }
    }
  };
  // The offset loop.
  auto mainloop = [&]() {
    // Every global load of the loop is issued unconditionally as a buffer load: a missing neighbour, a
    // padding column or an idle thread gets an offset past the descriptor's range, which the hardware
    // returns as zeros. With conditional loads the compiler could not count the loads in flight: the
    // weight-tile LDS store waited on vmcnt(0), i.e. for the next offset's gathers too, every offset.
    // Offsets are 32-bit: the host checks that the source table and the weight tiles fit below 2 GB.
    auto load_a = [&](int k, int kh, uint4 (&dst)[RT][KSH]) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int src = sN[(arow + rt * 16) * MAXK + k];
#pragma unroll
        for (int ks = 0; ks < KSH; ++ks) {
          const int c0 = (kh * KSH + ks) * 32 + ag * 8;
          unsigned off = (src >= 0 && c0 < g.CP) ? ((unsigned)src * (unsigned)g.CP + (unsigned)c0) * 2u : OOB;
          asm volatile("" : "+v"(off));   // keeps the select a select (else: one load per branch of a diamond)
          dst[rt][ks] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rsa, off, 0, 0));
        }
      }
    };
    // steps t = offset index * KSP + K half
    const int NS = NK * KSP;
    uint4 a0[RT][KSH], a1[RT][KSH], bw0[BPT], bw1[BPT];
    load_b(klist[0], 0, bw0);
    store_b(0, bw0);
    load_b(klist[(NS > 1 ? 1 : 0) / KSP], (NS > 1 ? 1 : 0) % KSP, bw0);
    load_a(klist[0], 0, a0);
    __syncthreads();
    // one offset per step. Loads run ahead: the A fragments of offset t+1 and the weight tile of
    // offset t+2 are issued at the top of step t, so the LDS store of tile t+1 (loaded one step
    // earlier) and the MFMAs of offset t wait only on loads a whole step old. A fragments and weight
    // registers ping-pong (a0 / a1, bw0 / bw1: no register copy that would wait on the newest loads);
    // the steps near the end re-fetch the last offset so the load count per step is fixed.
    auto step = [&](int t, const uint4 (&ac)[RT][KSH], uint4 (&an)[RT][KSH], const uint4 (&bc)[BPT],
                    uint4 (&bn)[BPT]) {
      const int k = klist[t / KSP];
      const int t2 = t + 2 < NS ? t + 2 : NS - 1, t1 = t + 1 < NS ? t + 1 : t;
      load_b(klist[t2 / KSP], t2 % KSP, bn);
      load_a(klist[t1 / KSP], t1 % KSP, an);
      if ((my >> k) & 1u) {
        const u16* bb = sB[t & 1] + (lane & 15) * LS + ag * 8;
#pragma unroll
        for (int ks = 0; ks < KSH; ++ks) {
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
    for (; t + 1 < NS; t += 2) {
      step(t, a0, a1, bw0, bw1);
      step(t + 1, a1, a0, bw1, bw0);
    }
    if (t < NS) step(t, a0, a1, bw0, bw1);
  };
  if (NK > 0) mainloop();

  // epilogue: C/D layout col = lane&15, row = (lane>>4)*4 + reg (16x16 shapes, gfx950)
  // E_DGRAD: per output tile n, the previous layer's z of the lane's 4 rows and the column's BatchNorm
  // parameters are loaded together before the tile's stores (out and ez are not known not to alias:
  // interleaved with the stores, every z load waited for its own round trip — 16 per lane)
  float s1[NT], s2[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) s1[n] = s2[n] = 0.0f;
  int prow[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + w * WR + rt * 16 + (lane >> 4) * 4 + j;
      prow[rt][j] = r < g.Nout ? r : -1;
    }
  // E_DGRAD / E_RES: the BatchNorm parameters of the block's columns are staged in LDS (the weight tiles' space, free
  // after the loop's last barrier), and with few output tiles every tile's z rows are loaded before the first store
  // (one round trip for the epilogue instead of one per tile: the stores of tile n may alias the loads of tile n + 1
  // as far as the compiler knows; 4 * RT * NT registers, only where RT * NT <= 4)
  float* const sEbn = (float*)&sB[0][0];   // [4][NGP]: scale, beta, mean, invstd
  if constexpr (EPI == E_DGRAD || EPI == E_RES) {
    static_assert(4 * NGP * 4 <= (int)sizeof(sB), "sEbn");
    const int C = g.CO_real;
    for (int j = tid; j < 4 * NGP; j += GBLK) {
      const int q = j / NGP, c = j - q * NGP;
      sEbn[j] = g.ebn[q * C + min(c, C - 1)];
    }
    __syncthreads();
  }
  constexpr bool PRE = EPI == E_DGRAD && RT * NT <= 4;
  float zpre[PRE ? RT : 1][PRE ? NT : 1][4];
  if constexpr (PRE) {
    const int C = g.CO_real;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int cc = min(n * 16 + (lane & 15), C - 1);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int j = 0; j < 4; ++j) zpre[rt][n][j] = g.ez[(long long)max(prow[rt][j], 0) * C + cc];
    }
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      int col = n * 16 + (lane & 15);
      float zr[4], pb[4], orr[4], g2r[4];
      if (EPI == E_DGRAD || EPI == E_RES) {
        const int C = g.CO_real, cc = min(col, C - 1);
#pragma unroll
        for (int q = 0; q < 4; ++q) pb[q] = sEbn[q * NGP + col];   // scale, beta, mean, invstd (of column cc)
        if constexpr (PRE) {
#pragma unroll
          for (int j = 0; j < 4; ++j) zr[j] = zpre[PRE ? rt : 0][PRE ? n : 0][j];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) zr[j] = g.ez[(long long)max(prow[rt][j], 0) * C + cc];
        }
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
            s2[n] = fmaf(v, (zr[j] - pb[2]) * pb[3], s2[n]);   // explicit (see E_DGRAD)
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

// The same pass with one float4 (4 channels) of the flattened [N][C] rows per thread: every load instruction reads
// 1 KB of consecutive bytes (the 8-channel form's lanes read 32 B each at a 32-B stride of the other lanes' rows: two
// half-used 2 KB spans per operand and row — 2.6 TB/s on CenterPoint's 16-channel layers). The grid stride is a
// multiple of C / 4 (C / 4 divides BLK), so a thread's channels and BatchNorm parameters never change. Same
// arithmetic per element, so the same bits.
constexpr int RV4 = 4;
__global__ __launch_bounds__(BLK) void k_dz_bf16_v4(const float* __restrict__ dy, const float* __restrict__ z,
                                                    const float* __restrict__ bnb, int N, int C,
                                                    u16* __restrict__ dz) {
  const int C4 = C >> 2;
  const long long total = (long long)N * C4;
  const long long t0 = (long long)blockIdx.x * BLK + threadIdx.x;
  const int c = (int)(t0 % C4) * 4;
  const float4 g4 = *(const float4*)(bnb + c), a4 = *(const float4*)(bnb + C + c), b4 = *(const float4*)(bnb + 2 * C + c);
  const float4 u4 = *(const float4*)(bnb + 3 * C + c), i4 = *(const float4*)(bnb + 4 * C + c);
  const float gi[4] = {g4.x, g4.y, g4.z, g4.w}, m1[4] = {a4.x, a4.y, a4.z, a4.w}, m2[4] = {b4.x, b4.y, b4.z, b4.w};
  const float mb[4] = {u4.x, u4.y, u4.z, u4.w}, ib[4] = {i4.x, i4.y, i4.z, i4.w};
  const long long step = (long long)gridDim.x * BLK;
  for (long long i0 = t0; i0 < total; i0 += RV4 * step) {
    float4 d[RV4], zz[RV4];
#pragma unroll
    for (int u = 0; u < RV4; ++u) {
      const long long i = min(i0 + u * step, total - 1);
      d[u] = ((const float4*)dy)[i];
      zz[u] = ((const float4*)z)[i];
    }
#pragma unroll
    for (int u = 0; u < RV4; ++u) {
      const long long i = i0 + u * step;
      if (i >= total) break;
      const float dv[4] = {d[u].x, d[u].y, d[u].z, d[u].w}, zv[4] = {zz[u].x, zz[u].y, zz[u].z, zz[u].w};
      u16 o[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float xh = (zv[j] - mb[j]) * ib[j];
        o[j] = to_h16<0>(gi[j] * (dv[j] - m1[j] - xh * m2[j]));
      }
      *(uint2*)(dz + i * 4) = *(const uint2*)o;
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
// reads conflict-free for C = 32/64/128.
// Loads run as a three-stage register pipeline over the sub-tiles t of the chunk: the neighbour
// indices of t + 3 and the row gathers of t + 2 are issued while the MFMAs of t run (two sub-tiles
// of gathers in flight; r05: one, behind an LDS index stage whose every read was waited out before
// its gather was issued). Every load is issued unconditionally — a missing neighbour, a row past
// the chunk or an idle lane reads a zero row (indices: an offset past the buffer range) — so the
// compiler counts the loads in flight and each wait retires exactly one stage.
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

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));   // first-class 16-B value (HIP's uint4 is a
// struct: its copies were memcpys that kept the load registers in scratch)
__device__ __attribute__((aligned(16))) u32x4 g_wg_zero[1];
template <int P, class T>
__device__ __forceinline__ T& pick(T& a, T& b) {
  if constexpr (P == 0) return a; else return b;
}   // the row a masked gather reads (zeros)

// weight-gradient block: 4 waves; 8 from 64 x 64 up. With 3 offsets per block (KG = 3) each staged dz
// sub-tile serves 3 offsets (CenterPoint k_wgrad_bf16<128,128> 458 -> 403 us per launch at r04,
// r04_step_kernels_centerpoint_wg3.txt); 8 waves halve each thread's share of the two gather stages in
// flight (64 x 64: 100 VGPRs, two blocks per CU). HIP's second launch bound is the minimum number of waves
// per SIMD: capping 64 x 128 at 128 VGPRs (4) spilled and measured slower than 154 VGPRs at one block per CU
// (159.7 vs 147.4 us standalone, gpurun_out r05wg4)
__host__ __device__ constexpr int wg_threads(int ci, int co) { return ci * co >= 64 * 64 ? 512 : 256; }
__host__ __device__ constexpr int wg_min_waves(int ci, int co) {
  return ci * co >= 128 * 128 ? 1 : (ci * co >= 64 * 64 ? 2 : 4);
}
template <int CI, int CO, int KG, bool HF16 = false>
__global__ __launch_bounds__(wg_threads(CI, CO), wg_min_waves(CI, CO)) void k_wgrad_bf16(const u16* __restrict__ h, int HP, const int* __restrict__ nbr,
                                                    int K, int N, int rows_per, const u16* __restrict__ dz, int DP,
                                                    float* __restrict__ part) {
  constexpr int TB = wg_threads(CI, CO), NWV = TB / 64;   // threads, waves
  constexpr int RT = 64;                                   // rows per sub-tile (2 MFMA k-steps)
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
  __shared__ unsigned sAny[4][NWV];                        // per sub-tile (ring of 4): offsets with a neighbour
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w % WM, wn = w / WM;
  // 1-D grid over (chunk, offset group), XCD-aware: the groups of one row chunk are consecutive items on
  // one XCD, so its dz rows (read by every group) and its neighbours' h rows are fetched once into that
  // XCD's L2 (a 2-D grid dispatched a chunk's groups `chunks` blocks apart, after its rows were evicted)
  const int ngroups = (K + KG - 1) / KG;
  const int item = dn::xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = item / ngroups, k0 = (item - chunk * ngroups) * KG;
  const int rb0 = chunk * rows_per, rb1 = min(N, rb0 + rows_per);
  const int nsub = rb1 > rb0 ? (rb1 - rb0 + RT - 1) / RT : 0;
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
  const u32x4* const zrow = g_wg_zero;
  constexpr unsigned OOB = 0x80000000u;
  // (32-bit buffer offsets for the indices: the host checks n_out * K * 4 < 2^31)
  const __amdgpu_buffer_rsrc_t rn = __builtin_amdgcn_make_buffer_rsrc((void*)nbr, (short)0, 0x7fffffff, 0x00020000);
  // the neighbour index of (row slot j, offset g) of sub-tile t: raw value (0 when masked: see a_ok)
  auto load_idx = [&](int t, int (&I)[KG][NA]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int q = tid + j * TB, row = rb0 + t * RT + q / CA;
#pragma unroll
      for (int g = 0; g < KG; ++g) {
        unsigned off = ((RT * CA) % TB == 0 || q < RT * CA) && row < rb1 && k0 + g < K
                           ? (unsigned)(row * K + k0 + g) * 4u : OOB;
        asm volatile("" : "+v"(off));
        I[g][j] = __builtin_amdgcn_raw_buffer_load_b32(rn, off, 0, 0);
      }
    }
  };
  // the gathers of sub-tile t (h rows by the indices I, dz rows), and its per-wave offset mask -> sAny
  auto load_rows = [&](int t, const int (&I)[KG][NA], u32x4 (&GA)[KG][NA], u32x4 (&GD)[ND]) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int q = tid + j * TB, r = q / CD, c8 = q - r * CD, row = rb0 + t * RT + r;
      const u32x4* p = ((RT * CD) % TB == 0 || q < RT * CD) && row < rb1
                           ? (const u32x4*)(dz + (long long)row * DP + c8 * 8) : zrow;
      GD[j] = *p;
    }
    unsigned m = 0;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int q = tid + j * TB, r = q / CA, c8 = q - r * CA, row = rb0 + t * RT + r;
#pragma unroll
      for (int g = 0; g < KG; ++g) {
        const bool ok = ((RT * CA) % TB == 0 || q < RT * CA) && row < rb1 && k0 + g < K && I[g][j] >= 0;
        const u32x4* p = ok ? (const u32x4*)(h + (long long)I[g][j] * HP + c8 * 8) : zrow;
        GA[g][j] = *p;
        m |= ok ? 1u << g : 0u;
      }
    }
    unsigned wmask = 0;
#pragma unroll
    for (int g = 0; g < KG; ++g) wmask |= __ballot((m >> g) & 1u) != 0 ? 1u << g : 0u;
    if (lane == 0) sAny[t & 3][w] = wmask;
  };
  auto mfma_tile = [&](unsigned any) __attribute__((always_inline)) {
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
        if (!((any >> g) & 1u)) continue;
#pragma unroll
        for (int a = 0; a < WMT; ++a) {
          const int m = wm + WM * a;
          s16x4 x[2] = {tr_read(&sA[g][r0 * PA + m * 16 + 4 * pp]), tr_read(&sA[g][(r0 + 16) * PA + m * 16 + 4 * pp])};
          bf16x8 av = *(bf16x8*)x;
#pragma unroll
          for (int b = 0; b < WNT; ++b)
            acc[g][a * WNT + b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv[b], acc[g][a * WNT + b], 0, 0, 0);
        }
      }
    }
  };
  // step t: stage t's rows (gathered two steps ago) into LDS, issue indices t + 3 and gathers t + 2 (into
  // the registers just freed), then the MFMAs of t. Register sets ping-pong by the parity P of t, chosen at
  // compile time (a run-time choice between two register arrays put them in scratch).
  int I0[KG][NA], I1[KG][NA];
  u32x4 A0[KG][NA], D0[ND], A1[KG][NA], D1[ND];
  auto step = [&](auto par, int t) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value;
    auto& GA = pick<P>(A0, A1);
    auto& GD = pick<P>(D0, D1);
    auto& In = pick<P>(I0, I1);
    auto& If = pick<P>(I1, I0);
    __syncthreads();   // the MFMAs of t - 1 are done with the LDS tiles
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const int q = tid + j * TB;
      if ((RT * CD) % TB == 0 || q < RT * CD) {
        const int r = q / CD, c8 = q - r * CD;
        *(u32x4*)&sD[r * PD + c8 * 8] = GD[j];
      }
    }
#pragma unroll
    for (int g = 0; g < KG; ++g)
#pragma unroll
      for (int j = 0; j < NA; ++j) {
        const int q = tid + j * TB;
        if ((RT * CA) % TB == 0 || q < RT * CA) {
          const int r = q / CA, c8 = q - r * CA;
          *(u32x4*)&sA[g][r * PA + c8 * 8] =
              HF16 ? __builtin_bit_cast(u32x4, f16x8_to_bf16x8(__builtin_bit_cast(uint4, GA[g][j]))) : GA[g][j];
        }
      }
    __syncthreads();
    unsigned any = 0;
#pragma unroll
    for (int v = 0; v < NWV; ++v) any |= sAny[t & 3][v];
    load_idx(t + 3, If);
    load_rows(t + 2, In, GA, GD);
    mfma_tile(any);
  };
  if (nsub > 0) {
    load_idx(0, I0);
    load_idx(1, I1);
    load_rows(0, I0, A0, D0);
    load_idx(2, I0);
    load_rows(1, I1, A1, D1);
    int t = 0;
    for (; t + 1 < nsub; t += 2) {
      step(std::integral_constant<int, 0>{}, t);
      step(std::integral_constant<int, 1>{}, t + 1);
    }
    if (t < nsub) step(std::integral_constant<int, 0>{}, t);
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

template <int KGP, int NT>
static void launch_k(int epi, const GB& a, int n_rows, hipStream_t st) {
  constexpr int RT = rt_of(KGP, NT), GW = gw_of(KGP, NT), GBM = 16 * RT * GW;
  const int nblk = (n_rows + GBM - 1) / GBM;
  if (a.fmt == 1)   // fp16 operands: forward GEMMs only (checked by gemm_bf16_launch)
    hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_FWD, true>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else if (epi == E_FWD) hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_FWD>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else if (epi == E_DGRAD) hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_DGRAD>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else if (epi == E_RES) hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_RES>), dim3(nblk), dim3(64 * GW), 0, st, a);
  else hipLaunchKernelGGL((k_gemm_bf16<KGP, NT, E_PLAIN>), dim3(nblk), dim3(64 * GW), 0, st, a);
}

static int launch(int KGP, int NT, int epi, const GB& a, int n_rows, hipStream_t st) {
#define C2(kg, nt)                                          \
  if (KGP == kg && NT == nt) {                              \
    launch_k<kg, nt>(epi, a, n_rows, st);                   \
    return RPC_OK;                                          \
  }
  C2(32, 1) C2(32, 2) C2(32, 4) C2(64, 2) C2(64, 4) C2(64, 8) C2(128, 4) C2(32, 8) C2(64, 1) C2(128, 2) C2(128, 8)
#undef C2
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
  if (c % 8 == 0 && BLK % (c / 4) == 0 && (long long)n * c < (1LL << 31)) {
    const long long per = (long long)BLK * RV4;
    const long long nb = ((long long)n * (c / 4) + per - 1) / per;
    hipLaunchKernelGGL(k_dz_bf16_v4, dim3((unsigned)(nb < 1 ? 1 : (nb > 8192 ? 8192 : nb))), dim3(BLK), 0,
                       (hipStream_t)stream, dy, z, bnb, n, c, (u16*)dz);
  } else if (c % 8 == 0 && BLK % (c / 8) == 0 && (long long)n * c < (1LL << 31))
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

// the data gradient into a basicblock's output rows with rpc_sparse_res_backward fused into its epilogue:
// m = (dgrad + g2) * [out > 0] -> m [n_out][ng] fp32, and the BatchNorm-backward partial rows (sum m,
// sum m * (z - mean) * invstd) of that layer (bn: scale, beta, mean, invstd) -> part [gemm blocks][2 * ng]
extern "C" int rpc_spconv_gemm_res(const void* a, int n_src, int kg, const int* map, int kvol, int rev,
                                   int n_out, const void* bt, int ng, float* m, const float* g2, const float* out,
                                   const float* z, const float* bn, float* part, const RpcBnFin* fin, void* stream) {
  if (!m || !out || !z || !bn || !part) return RPC_ERR_ARG;
  if (fin && (fin->mode != 1 || !fin->ticket || !fin->gpart || !fin->gamma || !fin->fbn || !fin->bn || ng > 256 ||
              n_out <= 0))
    return RPC_ERR_ARG;
  GB g;
  memset(&g, 0, sizeof(g));
  if (fin) g.fin = *fin;   // + that layer's BatchNorm-backward finalize (mode 1) in the last-arriving blocks
  g.eg2 = g2;
  g.eout = out;
  return gemm_bf16_launch(g, a, n_src, kg, map, kvol, rev, n_out, bt, ng, m, z, bn, part, E_RES, stream);
}

// largest block of the GEMM launches (rows): fin_groups of n_out at the smallest block (64 rows)
extern "C" int rpc_bn_fin_groups(int n_out) { return fin_groups(cdiv(n_out > 0 ? n_out : 1, 64)); }
extern "C" int rpc_bn_fin_tickets(int n_out) { return 1 + rpc_bn_fin_groups(n_out); }

// the data gradient (epi 1) with the BatchNorm-backward finalize of the layer whose ReLU mask it applies fused in
extern "C" int rpc_spconv_gemm_bf16_fin(const void* a, int n_src, int kg, const int* map, int kvol, int rev,
                                        int n_out, const void* bt, int ng, float* out, const float* prev_z,
                                        const float* prev_bn, float* part, int epi, const RpcBnFin* fin,
                                        void* stream) {
  GB g;
  memset(&g, 0, sizeof(g));
  if (fin) {
    if (epi != 1 || !part || !fin->ticket || !fin->gpart || !fin->gamma || !fin->bn || !fin->fbn || fin->mode != 1 ||
        ng > 256 || n_out <= 0)
      return RPC_ERR_ARG;
    g.fin = *fin;
  }
  return gemm_bf16_launch(g, a, n_src, kg, map, kvol, rev, n_out, bt, ng, out, prev_z, prev_bn, part, epi, stream);
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

extern "C" size_t rpc_spconv_wgrad_bf16_workspace_size(int n_out, int kvol, int ci, int co) {
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
