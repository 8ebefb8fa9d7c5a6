// a2/a3/a4: VoxelPerturber forward + backward on gfx950, fused with the valid-point
// compaction / masked scatter of AdversarialVoxelNet.extract_feat and the HardSimpleVFE
// that follows it.
//
// Reference semantics (models/adversarial/voxel_perturber.py):
//   s     = std(x, dim=0, unbiased) + 1e-6 ; NaN/Inf -> 1                 (:158-163)
//   xn    = clamp(x / s, -10, 10)                                         (:165-168)
//   raw   = Tanh(L5(ReLU(BN4(L4(... ReLU(BN0(L0(xn))) ...)))))            (:82-103, :176)
//   raw  *= sigmoid(La1(ReLU(La0(xn))))                                   (:107-112, :203-205)
//   pert  = clamp(raw * bound, -cbound, cbound), nan_to_num               (:209-256, :323-365)
//   out   = x + pert ; l2 = mean ||pert||_2 ; intensity = mean |pert_3| ;
//   bias  = mean_f |mean_n pert| ; imbalance = std_f(std_n pert)          (:268-299)
// BatchNorm1d in train mode uses batch statistics (biased var) and updates the running
// stats with momentum 0.1 and the unbiased var; eval mode uses the running stats.
//
// Structure: one launch per layer over the valid points (grid-stride, 256 blocks of 256
// threads); per-channel batch statistics are reduced per wave with shuffles, per block in
// LDS and across blocks by the last-arriving block (agent-scope release/acquire ticket),
// in a fixed order, so results are run-to-run deterministic. Activations z_l are kept in
// HBM for the backward pass. The weight gradients dW = dZ^T H are split-K reductions over
// the points (one batched launch for all layers), summed in double in a fixed order and
// passed through the reference's grad hook clamp(nan_to_num(g), -0.1, 0.1).
#include <hipcub/hipcub.hpp>
#include <type_traits>
#include <math.h>
#include <string.h>

#include "common.h"

namespace rpc {
namespace pert {

constexpr int BLK = 256;
constexpr int NWAVE = BLK / 64;
constexpr int GRID = 256;        // blocks of every per-point VALU pass (= partial rows)
constexpr int MFW = 8;           // waves per block of the MFMA hidden-layer passes: 256 blocks x 8
constexpr int MFBLK = MFW * 64;  // waves = 2 waves per SIMD on 256 CUs (256 VGPRs), GRID partial rows
constexpr int MAXF = 8;
constexpr int MAXC = 128;         // widest layer of the MFMA hidden-layer kernels (their LDS sums)
constexpr int MAXW = 256;         // widest hidden layer: wider ones run on the per-point VALU kernels
constexpr int PSTR = 2 * MAXW;    // row stride of the partial-sum rows part / gpart
constexpr int NTICKET = 16;       // hand-off points per pass (each TSTRIDE counters, see grid_col_totals)
constexpr int GS = 16;            // blocks per first-level reduction group
constexpr int NGRP = GRID / GS;   // groups
constexpr int TSTRIDE = 1 + NGRP;

struct Dev {
  int F, A, C[7];
  int a16;         // effective rpc_perturber_cfg.act16 (0 unless every hidden shape has a 16-bit instantiation)
  int S;           // channel stride of the SoA activation buffers (>= N)
  int rows, slots, fused, training, use_att, vfe_f;
  float eps, mom;
  float bscale[MAXF], bclamp[MAXF];
  const float* x;
  const int* npts;
  const float* W[6];
  const float* b[6];
  const float* g[5];
  const float* be[5];
  float* rm[5];
  float* rv[5];
  const float* Wa0;
  const float* ba0;
  const float* Wa1;
  const float* ba1;
  float* out;
  float* vfe;
  float* losses;
  // workspace
  int* off;        // fused: [rows+1] exclusive scan of valid-slot counts
  int* list;       // fused: [rows*slots] slot index of each valid point
  int* meta;       // [8]: 0 N, 1 fallback flag (NaN / empty)
  float* xs;       // [MAXF] s_f
  float* z[5];     // [C_{l+1}][S] channel-major
  float* bn[5];    // [4*C]: scale (gamma*invstd), beta, mean, invstd
  double* bnsum[5];  // backward: [2*C] sum dy, sum dy*xhat
  double* part;    // [GRID][PSTR]
  double* gpart;   // [NGRP][PSTR] group sums of part
  float* pstat;    // [4*MAXF]: mean_f, s_f, cimb_f, S
  unsigned* ticket;
  float* dz[6];    // dz_0..dz_4 [C_{l+1}][S], dz_5 [F][S]
  float* dh[2];    // [MAXW][S] post-ReLU grads, ping-pong
  float* dsig;     // [S]
  float* da;       // [A][S]
  float* aact;     // [A][S]
  float* wpart;    // [KS][total elements] split-K partial weight grads
  const float* dout;
  const float* dl;  // [4]
};

__device__ __forceinline__ int point_slot(const Dev& d, int i) { return d.fused ? d.list[i] : i; }

// per-lane double accumulators for per-channel sums; channel c lives in lane c&63, slot c>>6
template <int C>
struct ChanAcc {
  static constexpr int K = (C + 63) / 64;
  double s[2][K];
  __device__ void zero() {
#pragma unroll
    for (int k = 0; k < K; ++k) s[0][k] = s[1][k] = 0.0;
  }
  // wave-reduce this thread's (v, w) for channel c; lane c&63 keeps the running sums.
  // c must be a compile-time constant after unrolling (static register index).
  __device__ __forceinline__ void add1(int c, float v, float w) {
    const int lane = threadIdx.x & 63;
    float a = wave_sum(v);
    float q = wave_sum(w);
    if (lane == (c & 63)) {
      s[0][c >> 6] += (double)a;
      s[1][c >> 6] += (double)q;
    }
  }
  // block-combine into part[blockIdx.x][0..2C)
  __device__ void flush(double* part, double* lds) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      int c = k * 64 + lane;
      if (c < C) {
        lds[(w * 2 + 0) * MAXW + c] = s[0][k];
        lds[(w * 2 + 1) * MAXW + c] = s[1][k];
      }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 2 * C; j += BLK) {
      int which = j / C, c = j - which * C;
      double t = 0.0;
      for (int ww = 0; ww < NWAVE; ++ww) t += lds[(ww * 2 + which) * MAXW + c];
      part[(size_t)blockIdx.x * PSTR + j] = t;
    }
  }
};

// Column totals of the GRID partial rows part[r][0..ncol) (ncol <= PSTR), handed off in two
// levels: the last-arriving block of each group of GS consecutive blocks sums its group's rows in row
// order into gpart[q]; the last group finisher sums gpart[0..NGRP) in group order into lds[0..ncol)
// and returns true (every other block returns false). Each level issues all of its GS resp. NGRP
// loads per column at once: a single block sweeping 256 rows 4 at a time spent ~64 back-to-back
// memory latencies (~40-50 us) at the end of every BatchNorm pass. Fixed groups and fixed order:
// run-to-run deterministic. ticket k owns counters d.ticket[k * TSTRIDE + 0 .. TSTRIDE).
__device__ bool grid_col_totals(Dev& d, int k, int ncol, double* lds, int* flag) {
  unsigned* tk = d.ticket + k * TSTRIDE;
  const int q = blockIdx.x / GS;
  if (!last_block_arrive_2d(tk + 1 + q, flag, GS)) return false;
  for (int j = threadIdx.x; j < ncol; j += blockDim.x) {
    double v[GS];
#pragma unroll
    for (int i = 0; i < GS; ++i) v[i] = d.part[(size_t)(q * GS + i) * PSTR + j];
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < GS; ++i) t += v[i];
    d.gpart[(size_t)q * PSTR + j] = t;
  }
  if (!last_block_arrive_2d(tk, flag, NGRP)) return false;
  for (int j = threadIdx.x; j < ncol; j += blockDim.x) {
    double v[NGRP];
#pragma unroll
    for (int i = 0; i < NGRP; ++i) v[i] = d.gpart[(size_t)i * PSTR + j];
    double t = 0.0;
#pragma unroll
    for (int i = 0; i < NGRP; ++i) t += v[i];
    lds[j] = t;
  }
  __syncthreads();
  return true;
}

// finalize a BatchNorm layer from its batch sums (train) — run by the last block
template <int C>
__device__ void bn_finalize(Dev& d, int l, double* lds) {
  const int N = d.meta[0];
  for (int c = threadIdx.x; c < C; c += BLK) {
    double mean = lds[c] / N;
    double var = lds[C + c] / N - mean * mean;
    if (var < 0) var = 0;
    float invstd = 1.0f / sqrtf((float)var + d.eps);
    // applied as (z - mean) * scale + beta (no cancellation)
    float* bn = d.bn[l];
    bn[c] = d.g[l][c] * invstd;
    bn[C + c] = d.be[l][c];
    bn[2 * C + c] = (float)mean;
    bn[3 * C + c] = invstd;
    double uvar = N > 1 ? var * N / (N - 1) : var;
    d.rm[l][c] = (1.0f - d.mom) * d.rm[l][c] + d.mom * (float)mean;
    d.rv[l][c] = (1.0f - d.mom) * d.rv[l][c] + d.mom * (float)uvar;
  }
}

// ------------------------------------------------------------------ forward kernels
// stats of x over the valid points + compaction list + copy of the voxel slots to out
template <int F>
__global__ __launch_bounds__(BLK) void k_xstats(Dev d) {
  __shared__ double lds[NWAVE * 2 * MAXC];
  __shared__ int lastf;
  double s1[F], s2[F];
#pragma unroll
  for (int f = 0; f < F; ++f) s1[f] = s2[f] = 0.0;
  int nan = 0;
  const int stride = GRID * BLK;
  for (int r = blockIdx.x * BLK + threadIdx.x; r < d.rows; r += stride) {
    if (d.fused) {
      int base = d.off[r], j = 0;
      // eight slots' loads in flight before their copies are stored (d.out may alias d.x as far as the
      // compiler knows: interleaved, every slot's loads waited behind the previous slot's stores)
      for (int s0 = 0; s0 < d.slots; s0 += 8) {
        float vv[8][F];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const size_t slot = (size_t)r * d.slots + s0 + u;
#pragma unroll
          for (int f = 0; f < F; ++f) vv[u][f] = s0 + u < d.slots ? d.x[slot * F + f] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (s0 + u >= d.slots) break;
          const size_t slot = (size_t)r * d.slots + s0 + u;
          float sum = 0.0f;
#pragma unroll
          for (int f = 0; f < F; ++f) {
            sum = f == 0 ? vv[u][0] : sum + vv[u][f];
            d.out[slot * F + f] = vv[u][f];
          }
          if (sum != 0.0f) {
            d.list[base + j++] = (int)slot;
#pragma unroll
            for (int f = 0; f < F; ++f) {
              s1[f] += vv[u][f];
              s2[f] += (double)vv[u][f] * vv[u][f];
              nan |= isnan(vv[u][f]);
            }
          }
        }
      }
    } else {
      const float* p = d.x + (size_t)r * F;
#pragma unroll
      for (int f = 0; f < F; ++f) {
        float v = p[f];
        s1[f] += v;
        s2[f] += (double)v * v;
        nan |= isnan(v);
      }
    }
  }
  // block reduce 2F doubles + nan flag
#pragma unroll
  for (int f = 0; f < F; ++f) {
    s1[f] = wave_sum(s1[f]);
    s2[f] = wave_sum(s2[f]);
  }
  nan = __any(nan);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int f = 0; f < F; ++f) {
      lds[w * 2 * MAXC + f] = s1[f];
      lds[w * 2 * MAXC + F + f] = s2[f];
    }
    lds[w * 2 * MAXC + 2 * F] = nan;
  }
  __syncthreads();
  if (threadIdx.x < 2 * F + 1) {
    double t = 0.0;
    for (int ww = 0; ww < NWAVE; ++ww) t += lds[ww * 2 * MAXC + threadIdx.x];
    d.part[(size_t)blockIdx.x * PSTR + threadIdx.x] = t;
  }
  if (!grid_col_totals(d, 0, 2 * F + 1, lds, &lastf)) return;
  if (threadIdx.x == 0) {
    int N = d.fused ? d.off[d.rows] : d.rows;
    d.meta[0] = N;
    int flag = (lds[2 * F] != 0.0) || N == 0;
    d.meta[1] = flag;
    // s = std(x, unbiased) + 1e-6; any NaN/Inf entry resets the whole vector (:158-163)
    int bad = 0;
    for (int f = 0; f < F; ++f) {
      double mean = lds[f] / N;
      double var = N > 1 ? (lds[F + f] - N * mean * mean) / (N - 1) : NAN;
      if (var < 0) var = 0;
      float s = sqrtf((float)var) + 1e-6f;
      bad |= (isnan(s) || isinf(s));
      d.xs[f] = s;
    }
    if (bad)
      for (int f = 0; f < F; ++f) d.xs[f] = 1.0f;
  }
}

template <int F>
__device__ __forceinline__ void load_xn(const Dev& d, int slot, float (&xv)[F], float (&xn)[F]) {
  const float* p = d.x + (size_t)slot * F;
#pragma unroll
  for (int f = 0; f < F; ++f) {
    xv[f] = p[f];
    float t = xv[f] / d.xs[f];
    xn[f] = fminf(fmaxf(t, -10.0f), 10.0f);
  }
}

// VALU hidden layers whose weights exceed 64 KB read them from global memory (wave-uniform loads)
__host__ __device__ constexpr bool wide_w(int CI, int CO) { return CI * CO > 16384; }

// layer 0: xn -> z0 (+ batch stats / finalize BN0)
template <int F, int CO>
__global__ __launch_bounds__(BLK) void k_fwd_first(Dev d) {
  __shared__ float sW[CO * F + CO];
  __shared__ double lds[NWAVE * 2 * MAXW];
  __shared__ int lastf;
  for (int j = threadIdx.x; j < CO * F; j += BLK) sW[j] = d.W[0][j];
  for (int j = threadIdx.x; j < CO; j += BLK) sW[CO * F + j] = d.b[0][j];
  __syncthreads();
  const int N = d.meta[0];
  ChanAcc<CO> acc;
  acc.zero();
  for (int t = blockIdx.x; t * BLK < N; t += GRID) {
    int i = t * BLK + threadIdx.x;
    bool act = i < N;
    float xv[F], xn[F];
#pragma unroll
    for (int f = 0; f < F; ++f) xn[f] = 0.0f;
    if (act) load_xn<F>(d, point_slot(d, i), xv, xn);
#pragma unroll
    for (int o = 0; o < CO; ++o) {
      float a = sW[CO * F + o];
#pragma unroll
      for (int f = 0; f < F; ++f) a = fmaf(sW[o * F + f], xn[f], a);
      float z = act ? a : 0.0f;
      if (act) d.z[0][(size_t)o * d.S + i] = z;
      if (d.training) acc.add1(o, z, z * z);
    }
  }
  if (!d.training) return;
  acc.flush(d.part, lds);
  if (!grid_col_totals(d, 1, 2 * CO, lds, &lastf)) return;
  bn_finalize<CO>(d, 0, lds);
}

// layer l (1..4): relu(bn_{l-1}(z_{l-1})) -> z_l
template <int CI, int CO>
__global__ __launch_bounds__(BLK) void k_fwd_mid(Dev d, int l) {
  constexpr int WN = wide_w(CI, CO) ? 0 : CO * CI;  // weights staged in LDS (else read from global)
  __shared__ float sW[WN + CO + 3 * CI];
  __shared__ double lds[NWAVE * 2 * MAXW];
  __shared__ int lastf;
  for (int j = threadIdx.x; j < WN; j += BLK) sW[j] = d.W[l][j];
  for (int j = threadIdx.x; j < CO; j += BLK) sW[WN + j] = d.b[l][j];
  for (int j = threadIdx.x; j < 3 * CI; j += BLK) sW[WN + CO + j] = d.bn[l - 1][j];
  __syncthreads();
  const float* Wl = WN ? sW : d.W[l];
  const float* sc = sW + WN + CO;
  const float* sh = sc + CI;
  const float* mu = sh + CI;
  const int N = d.meta[0];
  ChanAcc<CO> acc;
  acc.zero();
  for (int t = blockIdx.x; t * BLK < N; t += GRID) {
    int i = t * BLK + threadIdx.x;
    bool act = i < N;
    float h[CI];
    const float* zi = d.z[l - 1] + (act ? i : 0);
#pragma unroll
    for (int c = 0; c < CI; ++c)
      h[c] = act ? fmaxf(fmaf(zi[(size_t)c * d.S] - mu[c], sc[c], sh[c]), 0.0f) : 0.0f;
#pragma unroll
    for (int o = 0; o < CO; ++o) {
      float a = sW[WN + o];
#pragma unroll
      for (int c = 0; c < CI; ++c) a = fmaf(Wl[o * CI + c], h[c], a);
      float z = act ? a : 0.0f;
      if (act) d.z[l][(size_t)o * d.S + i] = z;
      if (d.training) acc.add1(o, z, z * z);
    }
  }
  if (!d.training) return;
  acc.flush(d.part, lds);
  if (!grid_col_totals(d, 1 + l, 2 * CO, lds, &lastf)) return;
  bn_finalize<CO>(d, l, lds);
}

// recompute the attention gate for one point
template <int F>
__device__ __forceinline__ float attention(const Dev& d, const float (&xn)[F], float (&a)[MAXF]) {
  const int A = d.A;
  float t = d.ba1[0];
  for (int j = 0; j < A; ++j) {
    float s = d.ba0[j];
#pragma unroll
    for (int f = 0; f < F; ++f) s = fmaf(d.Wa0[j * F + f], xn[f], s);
    a[j] = fmaxf(s, 0.0f);
    t = fmaf(d.Wa1[j], a[j], t);
  }
  return 1.0f / (1.0f + expf(-t));
}

// output layer: relu(bn4(z4)) -> tanh -> *att -> bounds -> clamp -> out, loss sums
template <int CI, int F>
__global__ __launch_bounds__(BLK) void k_fwd_last(Dev d) {
  __shared__ float sW[F * CI + F + 3 * CI];
  __shared__ double lds[NWAVE * 2 * MAXC];
  __shared__ int lastf;
  for (int j = threadIdx.x; j < F * CI; j += BLK) sW[j] = d.W[5][j];
  for (int j = threadIdx.x; j < F; j += BLK) sW[F * CI + j] = d.b[5][j];
  for (int j = threadIdx.x; j < 3 * CI; j += BLK) sW[F * CI + F + j] = d.bn[4][j];
  __syncthreads();
  const float* sc = sW + F * CI + F;
  const float* sh = sc + CI;
  const float* mu = sh + CI;
  const int N = d.meta[0];
  // sums: [0] sum ||pert||, [1] sum |pert_3|, [2..2+F) sum pert_f, [2+F..2+2F) sum pert_f^2, [2+2F] nan
  constexpr int NS = 3 + 2 * F;
  double acc[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) acc[k] = 0.0;
  for (int t = blockIdx.x; t * BLK < N; t += GRID) {
    int i = t * BLK + threadIdx.x;
    bool act = i < N;
    float v[NS];
#pragma unroll
    for (int k = 0; k < NS; ++k) v[k] = 0.0f;
    if (act) {
      int slot = point_slot(d, i);
      float xv[F], xn[F], h[CI];
      load_xn<F>(d, slot, xv, xn);
      const float* zi = d.z[4] + i;
#pragma unroll
      for (int c = 0; c < CI; ++c) h[c] = fmaxf(fmaf(zi[(size_t)c * d.S] - mu[c], sc[c], sh[c]), 0.0f);
      float am[MAXF];
      float att = d.use_att ? attention<F>(d, xn, am) : 1.0f;
      float nrm2 = 0.0f;
      int bad = 0;
#pragma unroll
      for (int f = 0; f < F; ++f) {
        float u = sW[F * CI + f];
#pragma unroll
        for (int c = 0; c < CI; ++c) u = fmaf(sW[f * CI + c], h[c], u);
        float raw = tanhf(u);
        float pp = (raw * att) * d.bscale[f];
        bad |= isnan(pp);
        float p = fminf(fmaxf(pp, -d.bclamp[f]), d.bclamp[f]);
        d.out[(size_t)slot * F + f] = xv[f] + p;
        nrm2 = fmaf(p, p, nrm2);
        v[2 + f] = p;
        v[2 + F + f] = p * p;
        if (f == 3) v[1] = fabsf(p);
      }
      v[0] = sqrtf(nrm2);
      v[2 + 2 * F] = (float)bad;
    }
#pragma unroll
    for (int k = 0; k < NS; ++k) acc[k] += (double)wave_sum(v[k]);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NS; ++k) lds[w * 2 * MAXC + k] = acc[k];
  __syncthreads();
  if (threadIdx.x < NS) {
    double t = 0.0;
    for (int ww = 0; ww < NWAVE; ++ww) t += lds[ww * 2 * MAXC + threadIdx.x];
    d.part[(size_t)blockIdx.x * PSTR + threadIdx.x] = t;
  }
  if (!grid_col_totals(d, 6, NS, lds, &lastf)) return;
  if (threadIdx.x == 0) {
    const int n = N;
    int flag = d.meta[1] || lds[2 + 2 * F] != 0.0;
    d.meta[1] = flag;
    float l2 = (float)(lds[0] / n);
    float inten = F >= 4 ? (float)(lds[1] / n) : 0.0f;
    float bias = 0.0f, S = 0.0f;
    float sf[F], mf[F];
    for (int f = 0; f < F; ++f) {
      double m = lds[2 + f] / n;
      double var = n > 1 ? (lds[2 + F + f] - n * m * m) / (n - 1) : NAN;
      if (var < 0) var = 0;
      mf[f] = (float)m;
      sf[f] = sqrtf((float)var);
      bias += fabsf(mf[f]);
      S += sf[f];
    }
    bias /= F;
    S /= F;
    float q = 0.0f;
    for (int f = 0; f < F; ++f) q += (sf[f] - S) * (sf[f] - S);
    float imb = sqrtf(q / (F - 1));
    for (int f = 0; f < F; ++f) {
      d.pstat[f] = mf[f];
      d.pstat[MAXF + f] = sf[f];
      // d imb / d pert[n,f] = cimb_f * (pert[n,f] - mean_f)
      float ci = (imb > 0.0f && sf[f] > 0.0f && n > 1)
                     ? (sf[f] - S) / ((F - 1) * imb) / ((n - 1) * sf[f])
                     : 0.0f;
      d.pstat[2 * MAXF + f] = ci;
    }
    if (flag) l2 = inten = bias = imb = 0.0f;
    d.losses[0] = l2;
    d.losses[1] = inten;
    d.losses[2] = bias;
    d.losses[3] = imb;
    d.losses[4] = (float)n;
    d.losses[5] = (float)flag;
    d.losses[6] = 0.0f;
    d.losses[7] = 0.0f;
  }
}

// fused VFE: mean over the slots of the (perturbed) voxel; the unperturbed voxels when the
// NaN / empty fallback fired (adversarial_voxelnet.py:123-132).
__global__ __launch_bounds__(BLK) void k_vfe(Dev d, int F) {
  int t = blockIdx.x * BLK + threadIdx.x;
  if (t >= d.rows * d.vfe_f) return;
  int v = t / d.vfe_f, f = t - v * d.vfe_f;
  const float* src = d.meta[1] ? d.x : d.out;
  const float* p = src + (size_t)v * d.slots * F + f;
  float s = p[0];
  for (int j = 1; j < d.slots; ++j) s += p[(size_t)j * F];
  d.vfe[t] = s / (float)d.npts[v];
}

// fallback: out = x (unperturbed) when the flag is set
__global__ __launch_bounds__(BLK) void k_restore(Dev d, int F) {
  if (!d.meta[1]) return;
  long long n = (long long)d.rows * d.slots * F;
  for (long long t = (long long)blockIdx.x * BLK + threadIdx.x; t < n; t += (long long)gridDim.x * BLK)
    d.out[t] = d.x[t];
}

// eval mode: BN scale/shift from the running stats
__global__ void k_bn_eval(Dev d) {
  for (int l = 0; l < 5; ++l) {
    int C = d.C[l + 1];
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float invstd = 1.0f / sqrtf(d.rv[l][c] + d.eps);
      d.bn[l][c] = d.g[l][c] * invstd;
      d.bn[l][C + c] = d.be[l][c];
      d.bn[l][2 * C + c] = d.rm[l][c];
      d.bn[l][3 * C + c] = invstd;
    }
  }
}

// ------------------------------------------------------------------ backward kernels
template <int C>
__device__ void bnb_finalize(Dev& d, int l, double* lds) {
  for (int j = threadIdx.x; j < 2 * C; j += blockDim.x) d.bnsum[l][j] = lds[j];
}

// output layer + attention: dz5 = d u, dsig, da, a, dh4' and BN4 backward sums
template <int CI, int F>
__global__ __launch_bounds__(BLK) void k_bwd_last(Dev d) {
  __shared__ float sW[F * CI + F + 4 * CI];
  __shared__ double lds[NWAVE * 2 * MAXW];
  __shared__ int lastf;
  for (int j = threadIdx.x; j < F * CI; j += BLK) sW[j] = d.W[5][j];
  for (int j = threadIdx.x; j < F; j += BLK) sW[F * CI + j] = d.b[5][j];
  for (int j = threadIdx.x; j < 4 * CI; j += BLK) sW[F * CI + F + j] = d.bn[4][j];
  __syncthreads();
  const float* sc = sW + F * CI + F;
  const float* sh = sc + CI;
  const float* mean4 = sh + CI;
  const float* inv4 = mean4 + CI;
  const int N = d.meta[0];
  const float gl2 = d.dl[0], gint = d.dl[1], gbias = d.dl[2], gimb = d.dl[3];
  const float invN = 1.0f / (float)N;
  ChanAcc<CI> acc;
  acc.zero();
  for (int t = blockIdx.x; t * BLK < N; t += GRID) {
    int i = t * BLK + threadIdx.x;
    bool act = i < N;
    float du[F];
#pragma unroll
    for (int f = 0; f < F; ++f) du[f] = 0.0f;
    const float* zi = d.z[4] + (act ? i : 0);
    if (act) {
      int slot = point_slot(d, i);
      float xv[F], xn[F], h[CI];
      load_xn<F>(d, slot, xv, xn);
#pragma unroll
      for (int c = 0; c < CI; ++c) h[c] = fmaxf(fmaf(zi[(size_t)c * d.S] - mean4[c], sc[c], sh[c]), 0.0f);
      float am[MAXF];
      float att = d.use_att ? attention<F>(d, xn, am) : 1.0f;
      float raw[F], pp[F], p[F], dout[F];
      float nrm2 = 0.0f;
#pragma unroll
      for (int f = 0; f < F; ++f) {
        float u = sW[F * CI + f];
#pragma unroll
        for (int c = 0; c < CI; ++c) u = fmaf(sW[f * CI + c], h[c], u);
        raw[f] = tanhf(u);
        pp[f] = (raw[f] * att) * d.bscale[f];
        p[f] = fminf(fmaxf(pp[f], -d.bclamp[f]), d.bclamp[f]);
        nrm2 = fmaf(p[f], p[f], nrm2);
      }
      if (d.fused) {
        int v = slot / d.slots;
        float rn = 1.0f / (float)d.npts[v];
#pragma unroll
        for (int f = 0; f < F; ++f) dout[f] = f < d.vfe_f ? d.dout[(size_t)v * d.vfe_f + f] * rn : 0.0f;
      } else {
#pragma unroll
        for (int f = 0; f < F; ++f) dout[f] = d.dout[(size_t)i * F + f];
      }
      float nrm = sqrtf(nrm2);
      float datt = 0.0f;
#pragma unroll
      for (int f = 0; f < F; ++f) {
        float g = dout[f];
        if (nrm > 0.0f) g += gl2 * invN * (p[f] / nrm);
        if (f == 3) g += gint * invN * (float)((p[3] > 0.0f) - (p[3] < 0.0f));
        float m = d.pstat[f];
        g += gbias * invN / (float)F * (float)((m > 0.0f) - (m < 0.0f));
        g += gimb * d.pstat[2 * MAXF + f] * (p[f] - m);
        float dpp = (pp[f] >= -d.bclamp[f] && pp[f] <= d.bclamp[f]) ? g : 0.0f;
        float draw = dpp * att * d.bscale[f];
        datt = fmaf(dpp * raw[f], d.bscale[f], datt);
        du[f] = draw * (1.0f - raw[f] * raw[f]);
        d.dz[5][(size_t)f * d.S + i] = du[f];
      }
      if (d.use_att) {
        float dt = datt * att * (1.0f - att);
        d.dsig[i] = dt;
        for (int j = 0; j < d.A; ++j) {
          d.aact[(size_t)j * d.S + i] = am[j];
          d.da[(size_t)j * d.S + i] = am[j] > 0.0f ? d.Wa1[j] * dt : 0.0f;
        }
      }
    }
    // dh4' = relu'(h4) * W5^T du, and the BN4 backward sums
#pragma unroll
    for (int c = 0; c < CI; ++c) {
      float s = 0.0f, sx = 0.0f;
      if (act) {
#pragma unroll
        for (int f = 0; f < F; ++f) s = fmaf(sW[f * CI + c], du[f], s);
        float zc = zi[(size_t)c * d.S];
        float hv = fmaxf(fmaf(zc - mean4[c], sc[c], sh[c]), 0.0f);
        s = hv > 0.0f ? s : 0.0f;
        d.dh[0][(size_t)c * d.S + i] = s;
        sx = s * ((zc - mean4[c]) * inv4[c]);
      }
      acc.add1(c, s, sx);
    }
  }
  acc.flush(d.part, lds);
  if (!grid_col_totals(d, 7, 2 * CI, lds, &lastf)) return;
  bnb_finalize<CI>(d, 4, lds);
}

// BN layer l backward (l = 4..1): dz_l from dh_l'; dh_{l-1}' = relu'(.) * W_l^T dz_l
template <int CI, int CO>
__global__ __launch_bounds__(BLK) void k_bwd_mid(Dev d, int l, int src) {
  constexpr int WN = wide_w(CI, CO) ? 0 : CO * CI;  // weights staged in LDS (else read from global)
  __shared__ float sW[WN + 7 * CO + 4 * CI];
  __shared__ double lds[NWAVE * 2 * MAXW];
  __shared__ int lastf;
  const int N = d.meta[0];
  const double invN = 1.0 / N;
  for (int j = threadIdx.x; j < WN; j += BLK) sW[j] = d.W[l][j];
  for (int j = threadIdx.x; j < 4 * CO; j += BLK) sW[WN + j] = d.bn[l][j];
  for (int j = threadIdx.x; j < 4 * CI; j += BLK) sW[WN + 4 * CO + j] = d.bn[l - 1][j];
  for (int j = threadIdx.x; j < CO; j += BLK) {
    float* m = sW + WN + 4 * CO + 4 * CI;
    m[j] = (float)(d.bnsum[l][j] * invN);
    m[CO + j] = (float)(d.bnsum[l][CO + j] * invN);
    m[2 * CO + j] = d.g[l][j] * d.bn[l][3 * CO + j];
  }
  __syncthreads();
  const float* Wl = WN ? sW : d.W[l];
  const float* bo = sW + WN;           // scale, beta, mean, invstd of layer l
  const float* bi = bo + 4 * CO;       // of layer l-1
  const float* m1 = bi + 4 * CI;
  const float* m2 = m1 + CO;
  const float* gi = m2 + CO;
  ChanAcc<CI> acc;
  acc.zero();
  for (int t = blockIdx.x; t * BLK < N; t += GRID) {
    int i = t * BLK + threadIdx.x;
    bool act = i < N;
    int ii = act ? i : 0;
    const float* dhi = d.dh[src] + ii;
    const float* zl = d.z[l] + ii;
    float dz[CO];
#pragma unroll
    for (int o = 0; o < CO; ++o) {
      float xh = (zl[(size_t)o * d.S] - bo[2 * CO + o]) * bo[3 * CO + o];
      dz[o] = act ? gi[o] * (dhi[(size_t)o * d.S] - m1[o] - xh * m2[o]) : 0.0f;
      if (act) d.dz[l][(size_t)o * d.S + i] = dz[o];
    }
    const float* zp = d.z[l - 1] + ii;
#pragma unroll
    for (int c = 0; c < CI; ++c) {
      float s = 0.0f;
#pragma unroll
      for (int o = 0; o < CO; ++o) s = fmaf(Wl[o * CI + c], dz[o], s);
      float zc = zp[(size_t)c * d.S];
      float hv = fmaxf(fmaf(zc - bi[2 * CI + c], bi[c], bi[CI + c]), 0.0f);
      s = (act && hv > 0.0f) ? s : 0.0f;
      if (act) d.dh[src ^ 1][(size_t)c * d.S + i] = s;
      acc.add1(c, s, s * ((zc - bi[2 * CI + c]) * bi[3 * CI + c]));
    }
  }
  acc.flush(d.part, lds);
  if (!grid_col_totals(d, 7 + (5 - l), 2 * CI, lds, &lastf)) return;
  bnb_finalize<CI>(d, l - 1, lds);
}

// layer 0: dz_0 from dh_0'
template <int CO>
__global__ __launch_bounds__(BLK) void k_bwd_first(Dev d, int src) {
  const int N = d.meta[0];
  const double invN = 1.0 / N;
  const float* bo = d.bn[0];
  for (int i = blockIdx.x * BLK + threadIdx.x; i < N; i += GRID * BLK) {
#pragma unroll
    for (int o = 0; o < CO; ++o) {
      float m1 = (float)(d.bnsum[0][o] * invN), m2 = (float)(d.bnsum[0][CO + o] * invN);
      float xh = (d.z[0][(size_t)o * d.S + i] - bo[2 * CO + o]) * bo[3 * CO + o];
      d.dz[0][(size_t)o * d.S + i] =
          d.g[0][o] * bo[3 * CO + o] * (d.dh[src][(size_t)o * d.S + i] - m1 - xh * m2);
    }
  }
}

// ------------------------------------------------------------------ per-point boundary layers
// The VALU boundary layers (F -> C0 forward, C4 -> F backward, and the layer-0 BatchNorm backward) as
// per-point passes over ceil(S / BLK) blocks (the point count N lives on the device: blocks past it
// exit) with no reductions in the loop; their BatchNorm sums run as a separate column pass
// (k_colstats). The grid-stride versions above reduced every channel of every point with two wave
// shuffles chains on one wave per SIMD (k_bwd_last 96 us, k_fwd_first 55 us for 112k points).
template <int F, int CO>
__global__ __launch_bounds__(BLK) void k_fwd_first_pp(Dev d) {
  __shared__ float sW[CO * F + CO];
  for (int j = threadIdx.x; j < CO * F; j += BLK) sW[j] = d.W[0][j];
  for (int j = threadIdx.x; j < CO; j += BLK) sW[CO * F + j] = d.b[0][j];
  __syncthreads();
  const int i = blockIdx.x * BLK + threadIdx.x;
  if (i >= d.meta[0]) return;
  float xv[F], xn[F];
  load_xn<F>(d, point_slot(d, i), xv, xn);
#pragma unroll
  for (int o = 0; o < CO; ++o) {
    float a = sW[CO * F + o];
#pragma unroll
    for (int f = 0; f < F; ++f) a = fmaf(sW[o * F + f], xn[f], a);
    d.z[0][(size_t)o * d.S + i] = a;
  }
}

// per-channel sums over the N points of channel-major [C][S] rows: MODE 0 (forward BatchNorm of
// layer l): sum z, sum z^2 of z_l, then bn_finalize; MODE 1 (backward of layer l): sum g, sum g*xhat_l
// with g = the masked post-ReLU gradient, then bnb_finalize. GRID blocks of contiguous point ranges,
// 1024 threads = 64 channels x 16 lanes of float4 (the whole range in flight at once: 256-thread blocks
// ran these at 1.4 TB/s), double accumulation, fixed-order combine (deterministic).
constexpr int CSB = 1024;
template <int C, int MODE>
__global__ __launch_bounds__(CSB) void k_colstats(Dev d, int l, const float* __restrict__ gsrc, int tk) {
  __shared__ double lds[PSTR];
  __shared__ int lastf;
  const int N = d.meta[0];
  const int rows_per = ((N + GRID - 1) / GRID + 15) & ~15;
  const int p0 = blockIdx.x * rows_per, p1 = min(N, p0 + rows_per);
  const int q = threadIdx.x & 15;
  for (int c0 = 0; c0 < C; c0 += CSB / 16) {
    const int c = c0 + (threadIdx.x >> 4);
    double s1 = 0.0, s2 = 0.0;
    if (c < C) {
      const float* zr = d.z[l] + (size_t)c * d.S;
      const float* ar = MODE == 0 ? zr : gsrc + (size_t)c * d.S;
      const float mu = MODE == 1 ? d.bn[l][2 * C + c] : 0.0f;
      const float is = MODE == 1 ? d.bn[l][3 * C + c] : 0.0f;
      for (int pb = p0 + 4 * q; pb < p1; pb += 64 * 8) {
        float4 a[8], z[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int p = pb + 64 * u;
          a[u] = p < p1 ? *(const float4*)(ar + p) : make_float4(0.f, 0.f, 0.f, 0.f);
          z[u] = a[u];
          if (MODE == 1 && p < p1) z[u] = *(const float4*)(zr + p);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int p = pb + 64 * u;
          const float av[4] = {a[u].x, a[u].y, a[u].z, a[u].w}, zv[4] = {z[u].x, z[u].y, z[u].z, z[u].w};
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (p + j < p1) {
              s1 += (double)av[j];
              s2 += MODE == 0 ? (double)av[j] * av[j] : (double)(av[j] * ((zv[j] - mu) * is));
            }
        }
      }
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (q == 0 && c < C) {
      d.part[(size_t)blockIdx.x * PSTR + c] = s1;
      d.part[(size_t)blockIdx.x * PSTR + C + c] = s2;
    }
  }
  if (!grid_col_totals(d, tk, 2 * C, lds, &lastf)) return;
  if (MODE == 0) bn_finalize<C>(d, l, lds);
  else bnb_finalize<C>(d, l, lds);
}

// output layer + attention backward, per point: dz5 = d u, dsig, da, a, and dh4' (BN4 sums: k_colstats).
// Block = 64 points x 4 waves; wave w owns a quarter of the CI channels (their z4 rows are loaded once
// per wave, coalesced over the 64 points), the partial products u = W5 h4 are combined through LDS in
// wave order, and every wave then finishes the per-point output-layer math for its own channels.
template <int CI, int F>
__global__ __launch_bounds__(BLK) void k_bwd_last_pp(Dev d) {
  __shared__ float sW[F * CI + F + 4 * CI];
  __shared__ float su[NWAVE][F][64];
  const int N = d.meta[0];
  if (blockIdx.x * 64 >= N) return;
  for (int j = threadIdx.x; j < F * CI; j += BLK) sW[j] = d.W[5][j];
  for (int j = threadIdx.x; j < F; j += BLK) sW[F * CI + j] = d.b[5][j];
  for (int j = threadIdx.x; j < 4 * CI; j += BLK) sW[F * CI + F + j] = d.bn[4][j];
  __syncthreads();
  const float* sc = sW + F * CI + F;
  const float* sh = sc + CI;
  const float* mean4 = sh + CI;
  const int pl = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + pl;
  const bool act = i < N;
  constexpr int CQ = (CI + NWAVE - 1) / NWAVE;
  const int cb = w * CQ, ce = min(CI, cb + CQ);
  const float* zi = d.z[4] + (act ? i : 0);
  float up[F];
#pragma unroll
  for (int f = 0; f < F; ++f) up[f] = 0.0f;
  if (act) {
#pragma unroll 8
    for (int c = cb; c < ce; ++c) {
      const float hc = fmaxf(fmaf(zi[(size_t)c * d.S] - mean4[c], sc[c], sh[c]), 0.0f);
#pragma unroll
      for (int f = 0; f < F; ++f) up[f] = fmaf(sW[f * CI + c], hc, up[f]);
    }
  }
#pragma unroll
  for (int f = 0; f < F; ++f) su[w][f][pl] = up[f];
  __syncthreads();
  if (!act) return;
  const float gl2 = d.dl[0], gint = d.dl[1], gbias = d.dl[2], gimb = d.dl[3];
  const float invN = 1.0f / (float)N;
  const int slot = point_slot(d, i);
  float xv[F], xn[F], du[F];
  load_xn<F>(d, slot, xv, xn);
  float am[MAXF];
  const float att = d.use_att ? attention<F>(d, xn, am) : 1.0f;
  float raw[F], pp[F], p[F], dout[F];
  float nrm2 = 0.0f;
#pragma unroll
  for (int f = 0; f < F; ++f) {
    float u = sW[F * CI + f];
#pragma unroll
    for (int ww = 0; ww < NWAVE; ++ww) u += su[ww][f][pl];
    raw[f] = tanhf(u);
    pp[f] = (raw[f] * att) * d.bscale[f];
    p[f] = fminf(fmaxf(pp[f], -d.bclamp[f]), d.bclamp[f]);
    nrm2 = fmaf(p[f], p[f], nrm2);
  }
  if (d.fused) {
    const int v = slot / d.slots;
    const float rn = 1.0f / (float)d.npts[v];
#pragma unroll
    for (int f = 0; f < F; ++f) dout[f] = f < d.vfe_f ? d.dout[(size_t)v * d.vfe_f + f] * rn : 0.0f;
  } else {
#pragma unroll
    for (int f = 0; f < F; ++f) dout[f] = d.dout[(size_t)i * F + f];
  }
  const float nrm = sqrtf(nrm2);
  float datt = 0.0f;
#pragma unroll
  for (int f = 0; f < F; ++f) {
    float g = dout[f];
    if (nrm > 0.0f) g += gl2 * invN * (p[f] / nrm);
    if (f == 3) g += gint * invN * (float)((p[3] > 0.0f) - (p[3] < 0.0f));
    const float m = d.pstat[f];
    g += gbias * invN / (float)F * (float)((m > 0.0f) - (m < 0.0f));
    g += gimb * d.pstat[2 * MAXF + f] * (p[f] - m);
    const float dpp = (pp[f] >= -d.bclamp[f] && pp[f] <= d.bclamp[f]) ? g : 0.0f;
    const float draw = dpp * att * d.bscale[f];
    datt = fmaf(dpp * raw[f], d.bscale[f], datt);
    du[f] = draw * (1.0f - raw[f] * raw[f]);
    if (w == 0) d.dz[5][(size_t)f * d.S + i] = du[f];
  }
  if (d.use_att && w == 0) {
    const float dt = datt * att * (1.0f - att);
    d.dsig[i] = dt;
    for (int j = 0; j < d.A; ++j) {
      d.aact[(size_t)j * d.S + i] = am[j];
      d.da[(size_t)j * d.S + i] = am[j] > 0.0f ? d.Wa1[j] * dt : 0.0f;
    }
  }
#pragma unroll 8
  for (int c = cb; c < ce; ++c) {
    float s = 0.0f;
#pragma unroll
    for (int f = 0; f < F; ++f) s = fmaf(sW[f * CI + c], du[f], s);
    const float hc = fmaxf(fmaf(zi[(size_t)c * d.S] - mean4[c], sc[c], sh[c]), 0.0f);
    d.dh[0][(size_t)c * d.S + i] = hc > 0.0f ? s : 0.0f;
  }
}

// layer 0 BatchNorm backward, 4 points of one channel per thread (grid: point quads x CO)
__global__ __launch_bounds__(BLK) void k_bwd_first_pp(Dev d, int src, int CO) {
  const int o = blockIdx.y;
  const int i = (blockIdx.x * BLK + threadIdx.x) * 4;
  const int N = d.meta[0];
  if (i >= N) return;
  const double invN = 1.0 / N;
  const float* bo = d.bn[0];
  const float m1 = (float)(d.bnsum[0][o] * invN), m2 = (float)(d.bnsum[0][CO + o] * invN);
  const float mu = bo[2 * CO + o], is = bo[3 * CO + o], gi = d.g[0][o] * is;
  const size_t base = (size_t)o * d.S + i;
  const float4 z = *(const float4*)(d.z[0] + base);
  const float4 g = *(const float4*)(d.dh[src] + base);
  float4 r;
  r.x = gi * (g.x - m1 - ((z.x - mu) * is) * m2);
  r.y = gi * (g.y - m1 - ((z.y - mu) * is) * m2);
  r.z = gi * (g.z - m1 - ((z.z - mu) * is) * m2);
  r.w = gi * (g.w - m1 - ((z.w - mu) * is) * m2);
  *(float4*)(d.dz[0] + base) = r;
}

// ------------------------------------------------------------------ weight gradients
// job: dW[o][i] = sum_n dz[n][o] * h[n][i] ; i == CI is the bias column (h = 1)
enum HSrc { H_XN = 0, H_BNRELU = 1, H_RAW = 2 };
struct Job {
  const float* dz;  // [CO][S]
  int CO, CI;
  int hsrc;         // HSrc
  const float* h;   // H_BNRELU: z_{l-1} ; H_RAW: activations, both [CI][S]
  const float* bn;  // H_BNRELU: scale, beta, mean of layer l-1
  int eoff;         // element offset in wpart rows
  int nelem;        // CO * (CI + 1)
};
constexpr int MAXJOB = 8;
struct Jobs {
  Job j[MAXJOB];
  int njob;
  int echunks[MAXJOB];  // element chunks per job
  int cbase[MAXJOB];    // first chunk id of each job
  int KS;               // row splits
  int total;            // total elements over jobs
};
constexpr int EPT = 8;
constexpr int TR = 64;

// LDS rows are [r][CO + 1] dz and [r][CI + 2] h values; the row tile tr shrinks so that layers up to MAXW
// channels wide fit the same 66 KB as the 64-row tile of MAXC-wide ones.
constexpr int WG_LDS = 2 * TR * (MAXC + 1);
template <int F>
__global__ __launch_bounds__(BLK) void k_wgrad(Dev d, Jobs J) {
  __shared__ float sbuf[WG_LDS];
  int chunk = blockIdx.x / J.KS, ks = blockIdx.x - chunk * J.KS;
  int jb = 0;
  while (jb + 1 < J.njob && chunk >= J.cbase[jb + 1]) ++jb;
  const Job& job = J.j[jb];
  const int e0 = (chunk - J.cbase[jb]) * BLK * EPT;
  const int CO = job.CO, CI = job.CI, CI1 = CI + 1;
  const int SZ = CO + 1, SH = CI1 + 1;
  const int tr = min(TR, WG_LDS / (SZ + SH));
  float* sdz = sbuf;
  float* shh = sbuf + tr * SZ;
  const int N = d.meta[0];
  const int rows_per = (N + J.KS - 1) / J.KS;
  const int r0 = ks * rows_per, r1 = min(N, r0 + rows_per);
  float acc[EPT];
  int eo[EPT], ei[EPT];
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    acc[k] = 0.0f;
    int e = e0 + k * BLK + threadIdx.x;
    eo[k] = e < job.nelem ? e / CI1 : -1;
    ei[k] = e < job.nelem ? e - (e / CI1) * CI1 : 0;
  }
  for (int rb = r0; rb < r1; rb += tr) {
    int nr = min(tr, r1 - rb);
    __syncthreads();
    for (int q = threadIdx.x; q < tr * CO; q += BLK) {
      int o = q / tr, r = q - o * tr;
      sdz[r * SZ + o] = r < nr ? job.dz[(size_t)o * d.S + rb + r] : 0.0f;
    }
    for (int q = threadIdx.x; q < tr * CI1; q += BLK) {
      int c = q / tr, r = q - c * tr;
      float v = 0.0f;
      if (r < nr) {
        int n = rb + r;
        if (c == CI) v = 1.0f;
        else if (job.hsrc == H_XN) {
          int slot = point_slot(d, n);
          float t = d.x[(size_t)slot * F + c] / d.xs[c];
          v = fminf(fmaxf(t, -10.0f), 10.0f);
        } else if (job.hsrc == H_BNRELU) {
          v = fmaxf(fmaf(job.h[(size_t)c * d.S + n] - job.bn[2 * CI + c], job.bn[c], job.bn[CI + c]), 0.0f);
        } else {
          v = job.h[(size_t)c * d.S + n];
        }
      }
      shh[r * SH + c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
      if (eo[k] < 0) continue;
      float a = acc[k];
      const float* pz = sdz + eo[k];
      const float* ph = shh + ei[k];
      for (int r = 0; r < tr; ++r) a = fmaf(pz[r * SZ], ph[r * SH], a);
      acc[k] = a;
    }
  }
#pragma unroll
  for (int k = 0; k < EPT; ++k) {
    int e = e0 + k * BLK + threadIdx.x;
    if (e < job.nelem) d.wpart[(size_t)ks * J.total + job.eoff + e] = acc[k];
  }
}

// All VALU weight-gradient jobs of one point range per block (grid = KS ranges): per 64-point tile
// every job's dz rows and h rows are staged channel-major in LDS (dynamic: the host sizes it), then
// each thread accumulates up to EPT (job, o, i) elements in fixed row order. The staging is one flat
// sweep over a per-block table of source rows (raw / BatchNorm+ReLU / normalised-x gather), double
// buffered: the next tile's loads are in flight while the current one is summed.
// (One block grid per job — 4 jobs x 256 ranges of 7 serial tiles — took 97 us.)
// 1024 threads (16 waves per CU keep the staging loads in flight); WPRE float4 per thread: nrow * TR / 4 <= 12288.
// TR = points per tile, the largest of 256 / 128 / 64 whose two tile buffers fit the LDS (host): a block's range is
// a chain of tiles (fetch one ahead, two barriers per tile), so fewer, larger tiles shorten it (r06: 64-point tiles
// made nuScenes' 10-sweep batch ~60 tiles per block)
constexpr int WPB = 1024, WPRE = 12, WEPT = 2;
struct RowSrc {
  const float* p;   // channel row base ([S] floats); XN: nullptr
  float mu, sc, be; // BNRELU: relu((v - mu) * sc + be)
  int kind;         // HSrc, or 3 = dz row (raw)
  int c;            // XN: feature index
};
template <int F>
__device__ __forceinline__ float row_value(const Dev& d, const RowSrc& rs, int n) {
  if (rs.kind == H_XN) {
    const float t = d.x[(size_t)point_slot(d, n) * F + rs.c] / d.xs[rs.c];
    return fminf(fmaxf(t, -10.0f), 10.0f);
  }
  const float v = rs.p[n];
  return rs.kind == H_BNRELU ? fmaxf(fmaf(v - rs.mu, rs.sc, rs.be), 0.0f) : v;
}
template <int F, int TRP>
__global__ __launch_bounds__(WPB) void k_wgrad_pp(Dev d, Jobs J, int nrow) {
  constexpr int TPP = TRP + 1;
  extern __shared__ float sbuf[];
  RowSrc* rows = (RowSrc*)(sbuf + 2 * ((nrow * TPP + 3) & ~3));
  const int N = d.meta[0];
  const int rows_per = ((N + J.KS - 1) / J.KS + TRP - 1) / TRP * TRP;
  const int r0 = blockIdx.x * rows_per, r1 = min(N, r0 + rows_per);
  int joff[MAXJOB + 1];
  joff[0] = 0;
  for (int k = 0; k < J.njob; ++k) joff[k + 1] = joff[k] + J.j[k].CO + J.j[k].CI;
  // source table: job k's dz rows at joff[k] .., then its h rows
  for (int k = 0; k < J.njob; ++k) {
    const Job& job = J.j[k];
    for (int q = threadIdx.x; q < job.CO + job.CI; q += WPB) {
      RowSrc rs{};
      if (q < job.CO) {
        rs.p = job.dz + (size_t)q * d.S;
        rs.kind = 3;
      } else {
        const int c = q - job.CO;
        rs.kind = job.hsrc;
        rs.c = c;
        if (job.hsrc != H_XN) rs.p = job.h + (size_t)c * d.S;
        if (job.hsrc == H_BNRELU) {
          rs.mu = job.bn[2 * job.CI + c];
          rs.sc = job.bn[c];
          rs.be = job.bn[job.CI + c];
        }
      }
      rows[joff[k] + q] = rs;
    }
  }
  // this thread's elements
  int ej[WEPT];
  int pz[WEPT], ph[WEPT];
  float acc[WEPT];
  int nE = 0;
  for (int k = 0; k < J.njob; ++k) nE += J.j[k].nelem;
#pragma unroll
  for (int k = 0; k < WEPT; ++k) {
    acc[k] = 0.0f;
    ej[k] = -1;
    pz[k] = ph[k] = -1;
    int e = threadIdx.x + k * WPB;
    if (e < nE) {
      int jb = 0;
      while (e >= J.j[jb].nelem) { e -= J.j[jb].nelem; ++jb; }
      const int CI1 = J.j[jb].CI + 1, o = e / CI1, ii = e - o * CI1;
      ej[k] = J.j[jb].eoff + e;
      pz[k] = (joff[jb] + o) * TPP;
      ph[k] = ii < J.j[jb].CI ? (joff[jb] + J.j[jb].CO + ii) * TPP : -1;
    }
  }
  __syncthreads();
  // staging sweep: float4 of 4 consecutive points per lane (rows_per is a multiple of 64, so every
  // tile starts 16-byte aligned); tile t + 1 is fetched into registers while tile t is summed
  const int nq = nrow * (TRP / 4);
  float4 pre[WPRE];
  auto fetch = [&](int rb) {
#pragma unroll
    for (int u = 0; u < WPRE; ++u) {
      const int q = threadIdx.x + u * WPB;
      float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (q < nq) {
        const int row = q / (TRP / 4), n0 = rb + (q - row * (TRP / 4)) * 4;
        const RowSrc rs = rows[row];
        if (rs.kind == H_XN) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (n0 + j < r1) {
              const float t = d.x[(size_t)point_slot(d, n0 + j) * F + rs.c] / d.xs[rs.c];
              v[j] = fminf(fmaxf(t, -10.0f), 10.0f);
            }
        } else if (n0 < r1) {
          const float4 x = *(const float4*)(rs.p + n0);
          v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (rs.kind == H_BNRELU) v[j] = fmaxf(fmaf(v[j] - rs.mu, rs.sc, rs.be), 0.0f);
            if (n0 + j >= r1) v[j] = 0.0f;
          }
        }
      }
      pre[u] = make_float4(v[0], v[1], v[2], v[3]);
    }
  };
  const int tsz = (nrow * TPP + 3) & ~3;
  int cur = 0;
  if (r0 < r1) fetch(r0);
  for (int rb = r0; rb < r1; rb += TRP) {
    float* buf = sbuf + cur * tsz;
#pragma unroll
    for (int u = 0; u < WPRE; ++u) {
      const int q = threadIdx.x + u * WPB;
      if (q < nq) {
        const int row = q / (TRP / 4), r4 = (q - row * (TRP / 4)) * 4;
        float* dst = buf + row * TPP + r4;
        dst[0] = pre[u].x;
        dst[1] = pre[u].y;
        dst[2] = pre[u].z;
        dst[3] = pre[u].w;
      }
    }
    __syncthreads();
    if (rb + TRP < r1) fetch(rb + TRP);
#pragma unroll
    for (int k = 0; k < WEPT; ++k) {
      if (ej[k] < 0) continue;
      float a = acc[k];
      const float* z = buf + pz[k];
      if (ph[k] >= 0) {
        const float* hh = buf + ph[k];
        for (int r = 0; r < TRP; ++r) a = fmaf(z[r], hh[r], a);
      } else {
        for (int r = 0; r < TRP; ++r) a += z[r];
      }
      acc[k] = a;
    }
    cur ^= 1;
  }
#pragma unroll
  for (int k = 0; k < WEPT; ++k)
    if (ej[k] >= 0) d.wpart[(size_t)blockIdx.x * J.total + ej[k]] = acc[k];
}

__device__ __forceinline__ float grad_hook(float g) {
  // clamp(nan_to_num(g, nan=0, posinf=0, neginf=0), -0.1, 0.1)  (voxel_perturber.py:465-470)
  if (isnan(g) || isinf(g)) g = 0.0f;
  return fminf(fmaxf(g, -0.1f), 0.1f);
}

struct GradOut {
  float* W[MAXJOB];
  float* b[MAXJOB];
  float* gg[5];
  float* gb[5];
};

// Fixed-order reduction of the KS partial rows + the reference's grad hook. Block = 64 elements x 4
// row quarters (each quarter 8 interleaved sums, 8 loads in flight), quarters combined in order through
// LDS; elements past J.total are the BatchNorm affine gradients (no rows).
__global__ __launch_bounds__(BLK) void k_wgrad_reduce(Dev d, Jobs J, GradOut G) {
  __shared__ double sq[4][64];
  const int el = threadIdx.x & 63, qt = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el;
  const int flag = d.meta[1];
  if (e < J.total) {
    const int k0 = qt * J.KS / 4, k1 = (qt + 1) * J.KS / 4;
    double q[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    int k = k0;
    for (; k + 8 <= k1; k += 8)
#pragma unroll
      for (int u = 0; u < 8; ++u) q[u] += d.wpart[(size_t)(k + u) * J.total + e];
    for (; k < k1; ++k) q[0] += d.wpart[(size_t)k * J.total + e];
    sq[qt][el] = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  }
  __syncthreads();
  if (qt != 0) return;
  if (e < J.total) {
    int jb = 0;
    while (jb + 1 < J.njob && e >= J.j[jb + 1].eoff) ++jb;
    const Job& job = J.j[jb];
    const int le = e - job.eoff;
    const double s = (sq[0][el] + sq[1][el]) + (sq[2][el] + sq[3][el]);
    const float g = flag ? 0.0f : grad_hook((float)s);
    const int CI1 = job.CI + 1, o = le / CI1, i = le - o * CI1;
    if (i < job.CI) { if (G.W[jb]) G.W[jb][o * job.CI + i] = g; }
    else if (G.b[jb]) G.b[jb][o] = g;
  }
  // BatchNorm gamma / beta: sum dy*xhat, sum dy
  const int t = e - J.total;
  if (t >= 0) {
    int l = 0, base = 0;
    while (l < 5 && t >= base + d.C[l + 1]) { base += d.C[l + 1]; ++l; }
    if (l < 5) {
      const int c = t - base, C = d.C[l + 1];
      const float gg = flag ? 0.0f : grad_hook((float)d.bnsum[l][C + c]);
      const float gb = flag ? 0.0f : grad_hook((float)d.bnsum[l][c]);
      if (G.gg[l]) G.gg[l][c] = gg;
      if (G.gb[l]) G.gb[l][c] = gb;
    }
  }
}


// ------------------------------------------------------------------ fp32 MFMA hidden layers
// The hidden Linear layers as 16-point x 16-channel v_mfma_f32_16x16x4_f32 tiles (fp32 operands,
// fp32 accumulation — the reference arithmetic, only the summation order differs). One wave owns a
// 64-point group = 4 interleaved tiles: A = activations (lane: 4 consecutive points 4(l&15).., channel
// 4s + l>>4, one 16-byte load from the channel-major [C][S] buffers feeds the 4 tiles), B = weights
// from LDS (pitch chosen so the 64 lanes hit 64 distinct banks), D = 4 consecutive points x 1
// channel per lane across the 4 tiles, stored as one 16-byte vector per channel row. BatchNorm batch
// sums are reduced across the 4 lane groups with two shuffles per group and kept in double, then
// combined in fixed order like the VALU kernels.
typedef float f32x4 __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int pitch_mod(int ci, int m) { return ci + ((m - ci % 64) + 64) % 64; }

__device__ __forceinline__ float grp_sum(float v) {  // sum over the 4 lanes sharing l&15
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// BatchNorm batch sums of the MFMA passes: each wave accumulates its channel sums in its own LDS rows
// lds[w][2][MAXC] (double, lanes l < 16 own channel 16j + l of tile column j), then the block
// combines the waves in fixed order into its partial row (keeps 2 * C / 16 doubles out of VGPRs).
__device__ __forceinline__ void wave_sums_zero(double* lds) {
  for (int j = threadIdx.x; j < MFW * 2 * MAXC; j += MFBLK) lds[j] = 0.0;
}
__device__ __forceinline__ void wave_sums_add(double* lds, int j, float t1, float t2) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  t1 = grp_sum(t1);
  t2 = grp_sum(t2);
  if (lane < 16) {
    lds[(w * 2 + 0) * MAXC + 16 * j + lane] += (double)t1;
    lds[(w * 2 + 1) * MAXC + 16 * j + lane] += (double)t2;
  }
}
template <int C>
__device__ __forceinline__ void tile_flush(double* part, const double* lds) {
  __syncthreads();
  for (int j = threadIdx.x; j < 2 * C; j += MFBLK) {
    int which = j / C, c = j - which * C;
    double t = 0.0;
    for (int ww = 0; ww < MFW; ++ww) t += lds[(ww * 2 + which) * MAXC + c];
    part[(size_t)blockIdx.x * PSTR + j] = t;
  }
}

// 4 consecutive points n..n+3 of one channel row (n % 4 == 0). Rows are S >= 64-rounded N floats
// long and n lies in a 64-point group (16-point block) that starts below N, so the 16-byte access never leaves the row:
// branch-free (a tail branch per access made the compiler wait for every outstanding load at each
// join); points >= N read as 0 and are written with whatever the caller put there (0: masked).
__device__ __forceinline__ f32x4 ld4(const float* p, int n, int N) {
  f32x4 v = *(const f32x4*)(p + n);
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = n + i < N ? v[i] : 0.0f;
  return v;
}
__device__ __forceinline__ void st4(float* p, int n, int N, f32x4 v) {
  (void)N;
  *(f32x4*)(p + n) = v;
}
// Q = 2 or 4 consecutive points of one channel row (same contract as ld4 / st4, n % Q == 0)
template <int Q>
using fvec = float __attribute__((ext_vector_type(Q)));
template <int Q>
__device__ __forceinline__ fvec<Q> ldq(const float* p, int n, int N) {
  fvec<Q> v = *(const fvec<Q>*)(p + n);
#pragma unroll
  for (int i = 0; i < Q; ++i) v[i] = n + i < N ? v[i] : 0.0f;
  return v;
}
template <int Q>
__device__ __forceinline__ void stq(float* p, int n, fvec<Q> v) { *(fvec<Q>*)(p + n) = v; }

// 16-bit activation rows (perf mode, rpc_perturber_cfg.act16): the same channel-major [C][S] rows with 2-byte
// elements — fp16 for the hidden pre-activations z_1..z_3 (the reference AMP's Linear outputs, train.py:91-103;
// finite values saturate at +-65504 like the fp16 sparse rows), bf16 for the gradient rows dh / dz_1..dz_4
// (unscaled gradients ~1e-7 need bf16's range; the AMP's loss scaling has no counterpart here). Values that
// are stored are also what the producer's BatchNorm sums see (rnd), so the statistics describe the rows.
typedef _Float16 f16;
typedef __bf16 b16;
__device__ __forceinline__ float rnd(float v, float*) { return v; }
__device__ __forceinline__ float rnd(float v, f16*) { return (float)(f16)fminf(fmaxf(v, -65504.0f), 65504.0f); }
__device__ __forceinline__ float rnd(float v, b16*) { return (float)(b16)v; }
template <typename T>
__device__ __forceinline__ float rnd_as(float v) { return rnd(v, (T*)nullptr); }
template <int Q, typename T>
__device__ __forceinline__ fvec<Q> ldq(const T* p, int n, int N) {
  if constexpr (sizeof(T) == 4) {
    return ldq<Q>((const float*)p, n, N);
  } else {
    typedef T tv __attribute__((ext_vector_type(Q)));
    const tv h = *(const tv*)(p + n);
    fvec<Q> v;
#pragma unroll
    for (int i = 0; i < Q; ++i) v[i] = n + i < N ? (float)h[i] : 0.0f;
    return v;
  }
}
// the values must already be representable (rnd_as<T>): the conversion is then exact
template <int Q, typename T>
__device__ __forceinline__ void stq(T* p, int n, fvec<Q> v) {
  if constexpr (sizeof(T) == 4) {
    stq<Q>((float*)p, n, v);
  } else {
    typedef T tv __attribute__((ext_vector_type(Q)));
    tv h;
#pragma unroll
    for (int i = 0; i < Q; ++i) h[i] = (T)v[i];
    *(tv*)(p + n) = h;
  }
}
// element types of one hidden-layer launch (host-chosen per layer, see row_types)
template <class ZI, class ZO>
struct FwdT {
  using zi = ZI;   // z_{l-1} rows read
  using zo = ZO;   // z_l rows written
};
template <class ZL, class ZP, class GI, class GO, class DZ>
struct BwdT {
  using zl = ZL;   // z_l rows read
  using zp = ZP;   // z_{l-1} rows read (ReLU mask of h_{l-1})
  using gi = GI;   // dh_l rows read
  using go = GO;   // dh_{l-1} rows written
  using dz = DZ;   // dz_l rows written (read by the weight gradient)
};
using FwdF32 = FwdT<float, float>;
using BwdF32 = BwdT<float, float, float, float, float>;
// 16-bit activation rows (act16) are instantiated for the encoder-decoder shapes of the configs in scope (each
// hidden width twice or half the previous: [64, 128, 64] 3-class, [16, 32, 64] nuScenes); any other hidden shape
// keeps fp32 rows for the whole perturber (fill_dev)
__host__ __device__ constexpr bool a16_shape(int CI, int CO) {
  return CI >= 16 && CO >= 16 && CI % 16 == 0 && CO % 16 == 0 && CI * CO <= 8192 && (CI == 2 * CO || CO == 2 * CI);
}
// W_l [R][CI] row-major -> LDS rows of pitch P: all of a thread's loads in flight before its first LDS
// store (a load -> store loop waited out one L2 round trip per pass: 16 at the start of every block)
template <int NTOT, int CI, int P>
__device__ __forceinline__ void stage_w(float* sW, const float* __restrict__ W) {
  constexpr int NQ = (NTOT + MFBLK - 1) / MFBLK;
  float v[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) v[i] = W[min((int)threadIdx.x + i * MFBLK, NTOT - 1)];
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int j = threadIdx.x + i * MFBLK;
    if (j < NTOT) sW[(j / CI) * P + j % CI] = v[i];
  }
}
// interleaved tiles per wave group: 4 (64 points, 16-byte accesses) while the group's activation
// operand fits 64 VGPRs, else 2 (32 points, 8-byte accesses) — 2 waves per SIMD, no spills
__host__ __device__ constexpr int tiles_per_group(int ks) { return ks * 4 <= 64 ? 4 : 2; }

// layer l (1..4) forward: z_l = W_l relu(bn_{l-1}(z_{l-1})) + b_l, BN_l batch statistics.
// A wave owns a 64-point group as 4 interleaved MFMA tiles: tile q holds points n0 + 4m + q (m = row),
// so the A operand of all 4 tiles for channel 4s + g is ONE 16-byte load of points n0 + 4a .. +3, and
// the 4 tiles' D values for output row 4g + i are 4 consecutive points (one 16-byte store). Every
// weight read from LDS feeds 4 MFMAs. Groups go to waves block-fastest (t = wave * GRID + block) so
// each CU gets an equal share when N / 64 is not much larger than the wave count.
template <int CI, int CO, class RT>
__global__ __launch_bounds__(MFBLK) void k_fwd_mid_mf(Dev d, int l) {
  using ZI = typename RT::zi;
  using ZO = typename RT::zo;
  constexpr int P = pitch_mod(CI, 4), NT = CO / 16, KS = CI / 4, TQ = tiles_per_group(KS), GP = 16 * TQ;
  __shared__ float sW[CO * P];
  __shared__ float sp[3 * CI + CO];
  __shared__ double lds[MFW * 2 * MAXC];
  __shared__ int lastf;
  stage_w<CO * CI, CI, P>(sW, d.W[l]);
  for (int j = threadIdx.x; j < 3 * CI; j += MFBLK) sp[j] = d.bn[l - 1][j];
  for (int j = threadIdx.x; j < CO; j += MFBLK) sp[3 * CI + j] = d.b[l][j];
  wave_sums_zero(lds);
  __syncthreads();
  const float* sc = sp;
  const float* sh = sp + CI;
  const float* mu = sp + 2 * CI;
  const float* bias = sp + 3 * CI;
  const int N = d.meta[0];
  const int lane = threadIdx.x & 63, a = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const ZI* zin = (const ZI*)d.z[l - 1];
  ZO* zout = (ZO*)d.z[l];
  for (int t = wv * GRID + blockIdx.x; t * GP < N; t += GRID * MFW) {
    const int n0 = t * GP, na = n0 + TQ * a;
    fvec<TQ> hv[KS];
    // all KS activation loads in flight before the first BN / ReLU (load + transform per s waited out
    // one round trip per s)
#pragma unroll
    for (int s = 0; s < KS; ++s) hv[s] = ldq<TQ>(zin + (size_t)(4 * s + g) * d.S, na, N);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int c = 4 * s + g;
#pragma unroll
      for (int q = 0; q < TQ; ++q) hv[s][q] = na + q < N ? fmaxf(fmaf(hv[s][q] - mu[c], sc[c], sh[c]), 0.0f) : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float b = bias[16 * j + a];
      f32x4 v[TQ];
#pragma unroll
      for (int q = 0; q < TQ; ++q) v[q] = (f32x4){b, b, b, b};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float w = sW[(16 * j + a) * P + 4 * s + g];
#pragma unroll
        for (int q = 0; q < TQ; ++q) v[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(hv[s][q], w, v[q], 0, 0, 0);
      }
      float t1 = 0.0f, t2 = 0.0f;
      ZO* row = zout + (size_t)(16 * j + a) * d.S;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int nb = n0 + TQ * (4 * g + i);
        fvec<TQ> o;
#pragma unroll
        for (int q = 0; q < TQ; ++q) {
          o[q] = nb + q < N ? rnd_as<ZO>(v[q][i]) : 0.0f;
          t1 += o[q];
          t2 = fmaf(o[q], o[q], t2);
        }
        stq<TQ>(row, nb, o);
      }
      if (d.training) wave_sums_add(lds, j, t1, t2);
      asm volatile("" ::: "memory");  // keep the next tile's B reads here (register pressure)
    }
  }
  if (!d.training) return;
  tile_flush<CO>(d.part, lds);
  if (!grid_col_totals(d, 1 + l, 2 * CO, lds, &lastf)) return;
  bn_finalize<CO>(d, l, lds);
}

// layer l (4..1) backward: dz_l = BN_l backward of dh_l (stored), dh_{l-1} = relu'(h_{l-1}) W_l^T dz_l,
// BN_{l-1} backward sums (sum dh, sum dh * xhat). Same interleaved point groups as the forward.
template <int CI, int CO, class RT>
__global__ __launch_bounds__(MFBLK) void k_bwd_mid_mf(Dev d, int l, int src) {
  using ZL = typename RT::zl;
  using ZP = typename RT::zp;
  using GI = typename RT::gi;
  using GO = typename RT::go;
  using DZ = typename RT::dz;
  constexpr int P = pitch_mod(CI, 16), NT = CI / 16, KS = CO / 4, TQ = tiles_per_group(KS), GP = 16 * TQ;
  __shared__ float sW[CO * P];
  __shared__ float sp[7 * CO + 4 * CI];
  __shared__ double lds[MFW * 2 * MAXC];
  __shared__ int lastf;
  const int N = d.meta[0];
  const double invN = 1.0 / N;
  stage_w<CO * CI, CI, P>(sW, d.W[l]);
  for (int j = threadIdx.x; j < 4 * CO; j += MFBLK) sp[j] = d.bn[l][j];
  for (int j = threadIdx.x; j < 4 * CI; j += MFBLK) sp[4 * CO + j] = d.bn[l - 1][j];
  for (int j = threadIdx.x; j < CO; j += MFBLK) {
    float* m = sp + 4 * CO + 4 * CI;
    m[j] = (float)(d.bnsum[l][j] * invN);
    m[CO + j] = (float)(d.bnsum[l][CO + j] * invN);
    m[2 * CO + j] = d.g[l][j] * d.bn[l][3 * CO + j];
  }
  wave_sums_zero(lds);
  __syncthreads();
  const float* bo = sp;            // scale, beta, mean, invstd of layer l
  const float* bi = sp + 4 * CO;   // of layer l-1
  const float* m1 = bi + 4 * CI;
  const float* m2 = m1 + CO;
  const float* gi = m2 + CO;
  const int lane = threadIdx.x & 63, a = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const GI* dhin = (const GI*)d.dh[src];
  GO* dhout = (GO*)d.dh[src ^ 1];
  const ZL* zl = (const ZL*)d.z[l];
  const ZP* zp = (const ZP*)d.z[l - 1];
  DZ* dzl = (DZ*)d.dz[l];
  for (int t = wv * GRID + blockIdx.x; t * GP < N; t += GRID * MFW) {
    const int n0 = t * GP, na = n0 + TQ * a;
    fvec<TQ> dzv[KS];
    // 8 channel rows per batch: their z / dh loads all in flight before the batch's dz stores (the
    // stores may alias the next rows' loads, so a load -> store per row waited one round trip per row)
    constexpr int SB = KS < 8 ? KS : 8;
#pragma unroll
    for (int s0 = 0; s0 < KS; s0 += SB) {
      fvec<TQ> zv[SB], dv[SB];
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int o = 4 * (s0 + u) + g;
        zv[u] = ldq<TQ>(zl + (size_t)o * d.S, na, N);
        dv[u] = ldq<TQ>(dhin + (size_t)o * d.S, na, N);
      }
#pragma unroll
      for (int u = 0; u < SB; ++u) {
        const int s = s0 + u, o = 4 * s + g;
#pragma unroll
        for (int q = 0; q < TQ; ++q) {
          const float xh = (zv[u][q] - bo[2 * CO + o]) * bo[3 * CO + o];
          dzv[s][q] = na + q < N ? gi[o] * (dv[u][q] - m1[o] - xh * m2[o]) : 0.0f;
        }
        if constexpr (sizeof(DZ) == 4) {
          stq<TQ>(dzl + (size_t)o * d.S, na, dzv[s]);
        } else {   // the weight gradient's rows (bf16); this kernel's data gradient keeps the fp32 values
          fvec<TQ> r;
#pragma unroll
          for (int q = 0; q < TQ; ++q) r[q] = rnd_as<DZ>(dzv[s][q]);
          stq<TQ>(dzl + (size_t)o * d.S, na, r);
        }
      }
      asm volatile("" ::: "memory");  // bound the loads in flight (register pressure)
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int c = 16 * j + a;
      fvec<TQ> zc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) zc[i] = ldq<TQ>(zp + (size_t)c * d.S, n0 + TQ * (4 * g + i), N);
      f32x4 v[TQ];
#pragma unroll
      for (int q = 0; q < TQ; ++q) v[q] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float w = sW[(4 * s + g) * P + c];
#pragma unroll
        for (int q = 0; q < TQ; ++q) v[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(dzv[s][q], w, v[q], 0, 0, 0);
      }
      float t1 = 0.0f, t2 = 0.0f;
      GO* row = dhout + (size_t)c * d.S;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int nb = n0 + TQ * (4 * g + i);
        fvec<TQ> o;
#pragma unroll
        for (int q = 0; q < TQ; ++q) {
          const float hv = fmaxf(fmaf(zc[i][q] - bi[2 * CI + c], bi[c], bi[CI + c]), 0.0f);
          o[q] = (nb + q < N && hv > 0.0f) ? rnd_as<GO>(v[q][i]) : 0.0f;
          t1 += o[q];
          t2 += o[q] * ((zc[i][q] - bi[2 * CI + c]) * bi[3 * CI + c]);
        }
        stq<TQ>(row, nb, o);
      }
      wave_sums_add(lds, j, t1, t2);
      asm volatile("" ::: "memory");  // keep the next tile's B reads here (register pressure)
    }
  }
  tile_flush<CI>(d.part, lds);
  if (!grid_col_totals(d, 7 + (5 - l), 2 * CI, lds, &lastf)) return;
  bnb_finalize<CI>(d, l - 1, lds);
}

// weight gradient of a hidden layer: dW[o][c] = sum_n dz_l[o][n] h_{l-1}[c][n], db[o] = sum_n dz_l[o][n],
// h = relu(bn_{l-1}(z_{l-1})). K = points: lane k-slot j of a 16-point block holds point 4(l>>4) + j,
// one 16-byte load per channel row for A and B alike. grid (KS row chunks, jobs): the 4 waves take
// interleaved 16-point blocks of the chunk and are combined in LDS in wave order; one slab row of
// the job's CO*(CI+1) elements per block (reduced with the VALU jobs by k_wgrad_reduce).
struct MfJob {
  const float* dz;  // [CO][S]
  const float* z;   // z_{l-1} [CI][S]
  const float* bn;  // scale, beta, mean of layer l-1
  int eoff;
};
struct MfJobs {
  MfJob j[4];
  int total, KS;
};

template <int CO, int CI>
__global__ __launch_bounds__(BLK, 2) void k_wgrad_mf(Dev d, MfJobs J) {
  // every block covers ALL output tiles of its point chunk (h_{l-1} and dz_l are read once per chunk;
  // splitting the outputs over blocks re-read h CO/16 times): wave wv accumulates the 16-point
  // blocks r0 + 16 wv, + 64, ... into CO/16 x CI/16 tiles (<= 32: 128 accumulator VGPRs), the 4 waves
  // are summed in wave order through one LDS image
  constexpr int TO = CO / 16, TC = CI / 16;
  static_assert(TO * TC <= 32, "accumulator tiles");
  __shared__ float red[CO * CI];
  __shared__ float bred[NWAVE][CO];
  const MfJob& job = J.j[blockIdx.y];
  const int N = d.meta[0];
  const int rows_per = ((N + J.KS - 1) / J.KS + 15) & ~15;
  const int r0 = blockIdx.x * rows_per, r1 = min(N, r0 + rows_per);
  const int lane = threadIdx.x & 63, a = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  float sc[TC], sh[TC], mu[TC];
#pragma unroll
  for (int jc = 0; jc < TC; ++jc) {
    const int c = 16 * jc + a;
    sc[jc] = job.bn[c];
    sh[jc] = job.bn[CI + c];
    mu[jc] = job.bn[2 * CI + c];
  }
  f32x4 acc[TO][TC];
  float bsum[TO];
#pragma unroll
  for (int i = 0; i < TO; ++i) {
    bsum[i] = 0.0f;
#pragma unroll
    for (int jc = 0; jc < TC; ++jc) acc[i][jc] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  }
  for (int n0 = r0 + 16 * wv; n0 < r1; n0 += 16 * NWAVE) {
    const int nb = n0 + 4 * g;
    f32x4 av[TO], bv[TC];
#pragma unroll
    for (int i = 0; i < TO; ++i) av[i] = ld4(job.dz + (size_t)(16 * i + a) * d.S, nb, r1);
#pragma unroll
    for (int jc = 0; jc < TC; ++jc) {
      const f32x4 zc = ld4(job.z + (size_t)(16 * jc + a) * d.S, nb, r1);
#pragma unroll
      for (int k = 0; k < 4; ++k) bv[jc][k] = nb + k < r1 ? fmaxf(fmaf(zc[k] - mu[jc], sc[jc], sh[jc]), 0.0f) : 0.0f;
    }
#pragma unroll
    for (int i = 0; i < TO; ++i) bsum[i] += (av[i][0] + av[i][1]) + (av[i][2] + av[i][3]);
    // k outermost: consecutive MFMAs update different accumulators (the 4 k-steps of one tile back to
    // back waited out the 16x16x4 f32 dependent latency, 40 of every 32-cycle issue slot); each tile
    // still sums k = 0..3 in order
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < TO; ++i)
#pragma unroll
        for (int jc = 0; jc < TC; ++jc)
          acc[i][jc] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][k], bv[jc][k], acc[i][jc], 0, 0, 0);
  }
  // lane (a, g) of tile (i, jc) holds dW[16i + 4g + r][16jc + a]; waves summed in order 0, 1, 2, 3
  for (int ww = 0; ww < NWAVE; ++ww) {
    if (wv == ww) {
#pragma unroll
      for (int i = 0; i < TO; ++i)
#pragma unroll
        for (int jc = 0; jc < TC; ++jc)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* e = &red[(16 * i + 4 * g + r) * CI + 16 * jc + a];
            *e = ww == 0 ? acc[i][jc][r] : *e + acc[i][jc][r];
          }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < TO; ++i) {
    const float bt = grp_sum(bsum[i]);
    if (g == 0) bred[wv][16 * i + a] = bt;
  }
  __syncthreads();
  float* out = d.wpart + (size_t)blockIdx.x * J.total + job.eoff;
  for (int e = threadIdx.x; e < CO * (CI + 1); e += BLK) {
    const int o = e / (CI + 1), c = e - o * (CI + 1);
    out[e] = c < CI ? red[o * CI + c] : ((bred[0][o] + bred[1][o]) + bred[2][o]) + bred[3][o];
  }
}

// Perf mode (cfg->wgrad_split_bf16): the same weight gradient on bf16 MFMA with each fp32 operand split
// into hi = bf16(v) and lo = bf16(v - hi) and dW += lo_a hi_b + hi_a lo_b + hi_a hi_b (fp32 accumulate):
// ~16 significant bits per product (relative error ~2^-16, the lo*lo term dropped) at 3 x 16-cycle
// v_mfma_f32_16x16x32_bf16 per 32 points where the fp32 path issues 8 x 32-cycle 16x16x4 MFMAs (5.3x
// fewer MFMA cycles). Lane (a, g) holds 8 consecutive points n0 + 8g .. of channel row 16i + a (A = dz_l
// rows, B = h_{l-1} rows), so one k-step covers 32 points; the tile / wave / bias bookkeeping is
// k_wgrad_mf's (same slab row, reduced by k_wgrad_reduce).
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void split_bf16x8(const float* v, bf16x8_t& hi, bf16x8_t& lo) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const __bf16 h = (__bf16)v[k];
    hi[k] = h;
    lo[k] = (__bf16)(v[k] - (float)h);
  }
}

template <int CO, int CI, class DZ, class ZP>
__global__ __launch_bounds__(BLK, 2) void k_wgrad_bx3(Dev d, MfJobs J) {
  // DZ / ZP: element types of the dz_l / z_{l-1} rows (float, or the 16-bit rows of act16); bf16 dz rows are
  // their own hi part (lo = 0 exactly), so their lo * hi product is skipped
  // above 8 accumulator tiles the output tiles are split in two halves (along the wider of CO / CI): waves
  // (2p + h) take half h of the tiles over the point stream p (32-point blocks, the 2 streams interleaved),
  // so a wave holds at most 16 tiles plus its hi / lo operand splits without spilling; the operand rows of
  // the other dimension are loaded by both halves (the second read hits L2)
  constexpr int TO = CO / 16, TC = CI / 16;
  static_assert(TO * TC <= 32, "accumulator tiles");
  constexpr bool SPLIT = TO * TC > 8, SPLIT_C = SPLIT && TC >= TO, SPLIT_O = SPLIT && !SPLIT_C;
  constexpr int TOW = SPLIT_O ? TO / 2 : TO, TCW = SPLIT_C ? TC / 2 : TC;
  constexpr int NSTREAM = SPLIT ? NWAVE / 2 : NWAVE;
  __shared__ float red[CO * CI];
  __shared__ float bred[NWAVE][CO];
  const MfJob& job = J.j[blockIdx.y];
  const int N = d.meta[0];
  const int rows_per = ((N + J.KS - 1) / J.KS + 31) & ~31;
  const int r0 = blockIdx.x * rows_per, r1 = min(N, r0 + rows_per);
  const int lane = threadIdx.x & 63, a = lane & 15, g = lane >> 4, wv = threadIdx.x >> 6;
  const int half = SPLIT ? (wv & 1) : 0, stream = SPLIT ? (wv >> 1) : wv;
  const int o0 = SPLIT_O ? half * TOW : 0, c0 = SPLIT_C ? half * TCW : 0;   // first tile row / column
  float sc[TCW], sh[TCW], mu[TCW];
#pragma unroll
  for (int jc = 0; jc < TCW; ++jc) {
    const int c = 16 * (c0 + jc) + a;
    sc[jc] = job.bn[c];
    sh[jc] = job.bn[CI + c];
    mu[jc] = job.bn[2 * CI + c];
  }
  f32x4 acc[TOW][TCW];
  float bsum[TOW];
#pragma unroll
  for (int i = 0; i < TOW; ++i) {
    bsum[i] = 0.0f;
#pragma unroll
    for (int jc = 0; jc < TCW; ++jc) acc[i][jc] = (f32x4){0.0f, 0.0f, 0.0f, 0.0f};
  }
  for (int n0 = r0 + 32 * stream; n0 < r1; n0 += 32 * NSTREAM) {
    const int nb = n0 + 8 * g;
    f32x4 dv[TOW][2], zv[TCW][2];
#pragma unroll
    for (int i = 0; i < TOW; ++i) {
      const DZ* row = (const DZ*)job.dz + (size_t)(16 * (o0 + i) + a) * d.S;
      dv[i][0] = ldq<4>(row, nb, r1);
      dv[i][1] = ldq<4>(row, nb + 4, r1);
    }
#pragma unroll
    for (int jc = 0; jc < TCW; ++jc) {
      const ZP* row = (const ZP*)job.z + (size_t)(16 * (c0 + jc) + a) * d.S;
      zv[jc][0] = ldq<4>(row, nb, r1);
      zv[jc][1] = ldq<4>(row, nb + 4, r1);
    }
    bf16x8_t ah[TOW], al[TOW];
#pragma unroll
    for (int i = 0; i < TOW; ++i) {
      float t[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        t[k] = dv[i][0][k];
        t[4 + k] = dv[i][1][k];
      }
      bsum[i] += ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
      split_bf16x8(t, ah[i], al[i]);
    }
#pragma unroll
    for (int jc = 0; jc < TCW; ++jc) {
      float t[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float z = k < 4 ? zv[jc][0][k] : zv[jc][1][k - 4];
        t[k] = nb + k < r1 ? fmaxf(fmaf(z - mu[jc], sc[jc], sh[jc]), 0.0f) : 0.0f;
      }
      bf16x8_t bh, bl;
      split_bf16x8(t, bh, bl);
#pragma unroll
      for (int i = 0; i < TOW; ++i) {
        if constexpr (!std::is_same<DZ, b16>::value)
          acc[i][jc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh, acc[i][jc], 0, 0, 0);
        acc[i][jc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl, acc[i][jc], 0, 0, 0);
        acc[i][jc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh, acc[i][jc], 0, 0, 0);
      }
    }
  }
  // streams summed in order per tile (the two halves own disjoint tiles)
  for (int s = 0; s < NSTREAM; ++s) {
    if (stream == s) {
#pragma unroll
      for (int i = 0; i < TOW; ++i)
#pragma unroll
        for (int jc = 0; jc < TCW; ++jc)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float* e = &red[(16 * (o0 + i) + 4 * g + r) * CI + 16 * (c0 + jc) + a];
            *e = s == 0 ? acc[i][jc][r] : *e + acc[i][jc][r];
          }
    }
    __syncthreads();
  }
  // bias sums: every stream's own rows (with the CI split both halves summed the same rows: half 0 only)
#pragma unroll
  for (int i = 0; i < TOW; ++i) {
    const float bt = grp_sum(bsum[i]);
    if (g == 0 && !(SPLIT_C && half == 1)) bred[stream][16 * (o0 + i) + a] = bt;
  }
  __syncthreads();
  float* out = d.wpart + (size_t)blockIdx.x * J.total + job.eoff;
  for (int e = threadIdx.x; e < CO * (CI + 1); e += BLK) {
    const int o = e / (CI + 1), c = e - o * (CI + 1);
    float b = 0.0f;
    if (c == CI)
      for (int s2 = 0; s2 < NSTREAM; ++s2) b += bred[s2][o];
    out[e] = c < CI ? red[o * CI + c] : b;
  }
}

// ------------------------------------------------------------------ host side
static inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }
// channel stride of the SoA activation buffers: whole 64-point MFMA groups, 16-byte aligned rows
static inline size_t chan_stride(int rows, int slots) {
  size_t n = (size_t)rows * slots;
  return n < 64 ? 64 : (n + 63) & ~(size_t)63;
}

struct Layout {
  size_t off, list, meta, xs, z[5], bn[5], bnsum[5], part, gpart, pstat, ticket, dz[6], dh[2], dsig, da,
      aact, wpart, scan_tmp, scan_bytes, cnt, total;
};

struct ValidCount {
  const float* x;
  int slots, F, rows;
  __host__ __device__ int operator()(int v) const {
    if (v >= rows) return 0;
    int c = 0;
    for (int s = 0; s < slots; ++s) {
      const float* p = x + ((size_t)v * slots + s) * F;
      float sum = p[0];
      for (int f = 1; f < F; ++f) sum += p[f];
      c += (sum != 0.0f);
    }
    return c;
  }
};
// per-row valid-slot counts as a plain pass (the scan then runs over ints: with the counting done inside
// the scan's transform iterator the strided slot reads ran at the scan's low parallelism, 38 us)
// per-row valid-slot counts with one thread per point slot (adjacent lanes read adjacent slots: the per-row form read
// each row's slots x F floats serially, 202 us on CenterPoint's 10-sweep voxels): a wave's lanes of one row
// add their valid bits by one popcount of the wave's ballot and one integer atomic (cnt zeroed first; integer
// sums, so the counts do not depend on the order). Validity as ValidCount: the F features summed in order
__global__ __launch_bounds__(BLK) void k_valid_count_pts(ValidCount vc, int* __restrict__ cnt) {
  const long long n = (long long)vc.rows * vc.slots;
  const long long p = (long long)blockIdx.x * BLK + threadIdx.x;
  const int lane = threadIdx.x & 63;
  bool valid = false;
  if (p < n) {
    const float* q = vc.x + p * vc.F;
    float sum = q[0];
    for (int f = 1; f < vc.F; ++f) sum += q[f];
    valid = sum != 0.0f;
  }
  const unsigned long long vb = __ballot(valid);
  if (p < n) {
    const int s = (int)(p % vc.slots);
    if (s == 0 || lane == 0) {   // first lane of this row's segment in the wave
      const int len = min(vc.slots - s, 64 - lane);
      const unsigned long long seg = (len >= 64 ? ~0ull : ((1ull << len) - 1ull)) << lane;
      const int c = __popcll(vb & seg);
      if (c) atomicAdd(&cnt[p / vc.slots], c);
    }
  }
}

constexpr int KS_MAX = 256;

static int widths(const rpc_perturber_cfg* cfg, int C[7]) {
  C[0] = cfg->F;
  C[1] = cfg->hidden[0];
  C[2] = cfg->hidden[1];
  C[3] = cfg->hidden[2];
  C[4] = cfg->hidden[1];
  C[5] = cfg->hidden[0];
  C[6] = cfg->F;
  if (cfg->F < 4 || cfg->F > 5) return RPC_ERR_UNSUPPORTED;
  for (int k = 1; k < 6; ++k)
    if (C[k] != 8 && C[k] != 16 && C[k] != 32 && C[k] != 64 && C[k] != 128 && C[k] != MAXW) return RPC_ERR_UNSUPPORTED;
  return RPC_OK;
}

static int make_layout(const rpc_perturber_cfg* cfg, int rows, int slots, Layout* L) {
  int C[7];
  int rc = widths(cfg, C);
  if (rc) return rc;
  size_t Nmax = chan_stride(rows, slots);
  size_t scan_b = 0;
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, scan_b, (const int*)nullptr, (int*)nullptr, rows + 1,
                                       (hipStream_t)0) != hipSuccess)
    return RPC_ERR_HIP;
  int A = cfg->F / 2 > 1 ? cfg->F / 2 : 1;
  size_t welems = 0;
  for (int l = 0; l < 6; ++l) welems += (size_t)C[l + 1] * (C[l] + 1);
  welems += (size_t)A * (cfg->F + 1) + (size_t)(A + 1);
  size_t o = 0;
  L->off = o; o += al(sizeof(int) * (rows + 2));
  L->cnt = o; o += al(sizeof(int) * (rows + 1));
  L->list = o; o += al(sizeof(int) * Nmax);
  L->meta = o; o += al(sizeof(int) * 8);
  L->xs = o; o += al(sizeof(float) * MAXF);
  for (int l = 0; l < 5; ++l) { L->z[l] = o; o += al(sizeof(float) * Nmax * C[l + 1]); }
  for (int l = 0; l < 5; ++l) { L->bn[l] = o; o += al(sizeof(float) * 4 * C[l + 1]); }
  for (int l = 0; l < 5; ++l) { L->bnsum[l] = o; o += al(sizeof(double) * 2 * C[l + 1]); }
  L->part = o; o += al(sizeof(double) * GRID * PSTR);
  L->pstat = o; o += al(sizeof(float) * 4 * MAXF);
  L->ticket = o; o += al(sizeof(unsigned) * NTICKET * TSTRIDE);
  L->gpart = o; o += al(sizeof(double) * NGRP * PSTR);
  for (int l = 0; l < 5; ++l) { L->dz[l] = o; o += al(sizeof(float) * Nmax * C[l + 1]); }
  L->dz[5] = o; o += al(sizeof(float) * Nmax * cfg->F);
  int cmax = 0;
  for (int k = 1; k < 6; ++k) cmax = C[k] > cmax ? C[k] : cmax;
  for (int k = 0; k < 2; ++k) { L->dh[k] = o; o += al(sizeof(float) * Nmax * cmax); }
  L->dsig = o; o += al(sizeof(float) * Nmax);
  L->da = o; o += al(sizeof(float) * Nmax * A);
  L->aact = o; o += al(sizeof(float) * Nmax * A);
  L->wpart = o; o += al(sizeof(float) * KS_MAX * welems);
  L->scan_tmp = o; o += al(scan_b);
  L->scan_bytes = scan_b;
  L->total = o;
  return RPC_OK;
}

static void float_bounds(const rpc_perturber_cfg* cfg, Dev& d) {
  // exact float32 op order of voxel_perturber.py:209-256 and :333-359
  const int F = cfg->F;
  const float e = cfg->sensor_error_bound;
  for (int f = 0; f < MAXF; ++f) d.bscale[f] = d.bclamp[f] = 0.0f;
  if (F == 4) {
    if (!cfg->training) {
      float eb = e;
      volatile float mult = (float)(2.5 * ((2.0 + 1.5 + 1.2) / 3.0));
      eb = eb * mult;
      for (int f = 0; f < 3; ++f) d.bscale[f] = eb * 2.0f;
      d.bscale[3] = 1.5f;
      volatile float fb = e * 5.0f;
      for (int f = 0; f < 3; ++f) d.bclamp[f] = fb * 5.0f;
      d.bclamp[3] = 2.0f;
    } else {
      volatile float eb = e * 0.8f;
      for (int f = 0; f < 3; ++f) d.bscale[f] = eb * 1.3f;
      d.bscale[3] = 0.2f;
      volatile float fb = e * 0.9f;
      for (int f = 0; f < 3; ++f) d.bclamp[f] = fb * 1.2f;
      d.bclamp[3] = 0.1f;
    }
  } else {
    for (int f = 0; f < 4; ++f) d.bscale[f] = d.bclamp[f] = e;
  }
}

static int fill_dev(const rpc_perturber_cfg* cfg, const float* const* P, const float* x, int rows,
                    int slots, const int* npts, void* ws, size_t wsb, Dev& d, Layout& L) {
  int rc = make_layout(cfg, rows, slots, &L);
  if (rc) return rc;
  if (wsb < L.total) return RPC_ERR_WORKSPACE;
  memset(&d, 0, sizeof(d));
  d.F = cfg->F;
  d.A = cfg->F / 2 > 1 ? cfg->F / 2 : 1;
  widths(cfg, d.C);
  // 16-bit rows only where every hidden layer has them, and the bf16 dz rows only with the split-bf16 weight
  // gradient (the fp32-MFMA k_wgrad_mf reads fp32 rows)
  d.a16 = cfg->act16 & 3;
  for (int l = 1; l < 5; ++l)
    if (!a16_shape(d.C[l], d.C[l + 1])) d.a16 = 0;
  if (!cfg->wgrad_split_bf16) d.a16 &= ~2;
  d.rows = rows;
  d.slots = slots;
  d.S = (int)chan_stride(rows, slots);
  d.fused = npts != nullptr;
  d.training = cfg->training;
  d.use_att = cfg->use_attention;
  d.vfe_f = cfg->vfe_features;
  d.eps = cfg->bn_eps;
  d.mom = cfg->bn_momentum;
  float_bounds(cfg, d);
  d.x = x;
  d.npts = npts;
  for (int l = 0; l < 5; ++l) {
    d.W[l] = P[6 * l + 0];
    d.b[l] = P[6 * l + 1];
    d.g[l] = P[6 * l + 2];
    d.be[l] = P[6 * l + 3];
    d.rm[l] = (float*)P[6 * l + 4];
    d.rv[l] = (float*)P[6 * l + 5];
  }
  d.W[5] = P[30];
  d.b[5] = P[31];
  d.Wa0 = P[32];
  d.ba0 = P[33];
  d.Wa1 = P[34];
  d.ba1 = P[35];
  char* w = (char*)ws;
  d.off = (int*)(w + L.off);
  d.list = (int*)(w + L.list);
  d.meta = (int*)(w + L.meta);
  d.xs = (float*)(w + L.xs);
  for (int l = 0; l < 5; ++l) {
    d.z[l] = (float*)(w + L.z[l]);
    d.bn[l] = (float*)(w + L.bn[l]);
    d.bnsum[l] = (double*)(w + L.bnsum[l]);
  }
  d.part = (double*)(w + L.part);
  d.gpart = (double*)(w + L.gpart);
  d.pstat = (float*)(w + L.pstat);
  d.ticket = (unsigned*)(w + L.ticket);
  for (int l = 0; l < 6; ++l) d.dz[l] = (float*)(w + L.dz[l]);
  d.dh[0] = (float*)(w + L.dh[0]);
  d.dh[1] = (float*)(w + L.dh[1]);
  d.dsig = (float*)(w + L.dsig);
  d.da = (float*)(w + L.da);
  d.aact = (float*)(w + L.aact);
  d.wpart = (float*)(w + L.wpart);
  return RPC_OK;
}

// ---- width dispatch
#define RPC_HID(X) X(8) X(16) X(32) X(64) X(128) X(256)

// per-point passes cover every slot the batch can have (S >= N); blocks past N exit at once
static inline dim3 pp_grid(const Dev& d) { return dim3((unsigned)((d.S + BLK - 1) / BLK)); }

static int launch_colstats(int C, int mode, Dev& d, int l, const float* g, int tk, hipStream_t st) {
  switch (C) {
#define CASE(c)                                                                                      \
  case c:                                                                                            \
    if (mode == 0) hipLaunchKernelGGL((k_colstats<c, 0>), dim3(GRID), dim3(CSB), 0, st, d, l, g, tk); \
    else hipLaunchKernelGGL((k_colstats<c, 1>), dim3(GRID), dim3(CSB), 0, st, d, l, g, tk);           \
    break;
    RPC_HID(CASE)
#undef CASE
    default: return RPC_ERR_UNSUPPORTED;
  }
  return RPC_OK;
}

template <int F>
static int launch_first(int C0, Dev& d, hipStream_t st) {
  switch (C0) {
#define CASE(c) case c: hipLaunchKernelGGL((k_fwd_first_pp<F, c>), pp_grid(d), dim3(BLK), 0, st, d); break;
    RPC_HID(CASE)
#undef CASE
    default: return RPC_ERR_UNSUPPORTED;
  }
  return RPC_OK;
}
template <int F>
static int launch_last(int CI, Dev& d, hipStream_t st, bool bwd) {
  switch (CI) {
#define CASE(c)                                                                          \
  case c:                                                                                \
    if (bwd) hipLaunchKernelGGL((k_bwd_last_pp<c, F>), dim3((d.S + 63) / 64), dim3(BLK), 0, st, d); \
    else hipLaunchKernelGGL((k_fwd_last<c, F>), dim3(GRID), dim3(BLK), 0, st, d);        \
    break;
    RPC_HID(CASE)
#undef CASE
    default: return RPC_ERR_UNSUPPORTED;
  }
  return RPC_OK;
}
template <bool H>
using Z16 = typename std::conditional<H, f16, float>::type;
template <bool H>
using G16 = typename std::conditional<H, b16, float>::type;
// row types of layer l: z_1..z_3 16-bit (z_0 / z_4 stay fp32: the per-point boundary passes read them), dh_l
// 16-bit between hidden layers (dh_4 comes from the fp32 output-layer pass, dh_0 feeds the fp32 layer-0 pass)
template <int CI, int CO, bool ZH, bool GH>
static void launch_mid16(Dev& d, int l, hipStream_t st, bool bwd, int src) {
  if (bwd) {
    if (l == 4)
      hipLaunchKernelGGL((k_bwd_mid_mf<CI, CO, BwdT<float, Z16<ZH>, float, G16<GH>, G16<GH>>>), dim3(GRID), dim3(MFBLK),
                         0, st, d, l, src);
    else if (l == 1)
      hipLaunchKernelGGL((k_bwd_mid_mf<CI, CO, BwdT<Z16<ZH>, float, G16<GH>, float, G16<GH>>>), dim3(GRID), dim3(MFBLK),
                         0, st, d, l, src);
    else
      hipLaunchKernelGGL((k_bwd_mid_mf<CI, CO, BwdT<Z16<ZH>, Z16<ZH>, G16<GH>, G16<GH>, G16<GH>>>), dim3(GRID),
                         dim3(MFBLK), 0, st, d, l, src);
  } else {
    if (l == 1)
      hipLaunchKernelGGL((k_fwd_mid_mf<CI, CO, FwdT<float, Z16<ZH>>>), dim3(GRID), dim3(MFBLK), 0, st, d, l);
    else if (l == 4)
      hipLaunchKernelGGL((k_fwd_mid_mf<CI, CO, FwdT<Z16<ZH>, float>>), dim3(GRID), dim3(MFBLK), 0, st, d, l);
    else
      hipLaunchKernelGGL((k_fwd_mid_mf<CI, CO, FwdT<Z16<ZH>, Z16<ZH>>>), dim3(GRID), dim3(MFBLK), 0, st, d, l);
  }
}
// hidden layer l: fp32-MFMA kernels where the tile shape fits (forward: CO % 16, backward: CI % 16),
// the per-point VALU kernels otherwise (8-channel layers of the small configs, and layers wider than MAXC)
template <int CI, int CO>
static void launch_mid_t(Dev& d, int l, hipStream_t st, bool bwd, int src) {
  if constexpr (a16_shape(CI, CO)) {
    switch (d.a16) {
      case 1: launch_mid16<CI, CO, true, false>(d, l, st, bwd, src); return;
      case 2: launch_mid16<CI, CO, false, true>(d, l, st, bwd, src); return;
      case 3: launch_mid16<CI, CO, true, true>(d, l, st, bwd, src); return;
      default: break;
    }
  }
  constexpr bool mf = CI <= MAXC && CO <= MAXC;
  if (bwd) {
    if constexpr (mf && CI % 16 == 0) hipLaunchKernelGGL((k_bwd_mid_mf<CI, CO, BwdF32>), dim3(GRID), dim3(MFBLK), 0, st, d, l, src);
    else hipLaunchKernelGGL((k_bwd_mid<CI, CO>), dim3(GRID), dim3(BLK), 0, st, d, l, src);
  } else {
    if constexpr (mf && CO % 16 == 0) hipLaunchKernelGGL((k_fwd_mid_mf<CI, CO, FwdF32>), dim3(GRID), dim3(MFBLK), 0, st, d, l);
    else hipLaunchKernelGGL((k_fwd_mid<CI, CO>), dim3(GRID), dim3(BLK), 0, st, d, l);
  }
}
template <int CI>
static int launch_mid_co(int CO, Dev& d, int l, hipStream_t st, bool bwd, int src) {
  switch (CO) {
#define CASE(c) case c: launch_mid_t<CI, c>(d, l, st, bwd, src); break;
    RPC_HID(CASE)
#undef CASE
    default: return RPC_ERR_UNSUPPORTED;
  }
  return RPC_OK;
}
static int launch_mid(int CI, int CO, Dev& d, int l, hipStream_t st, bool bwd, int src = 0) {
  switch (CI) {
#define CASE(c) case c: return launch_mid_co<c>(CO, d, l, st, bwd, src);
    RPC_HID(CASE)
#undef CASE
    default: return RPC_ERR_UNSUPPORTED;
  }
}
static bool wgrad_mf_ok(int CO, int CI) {
  return CO % 16 == 0 && CI % 16 == 0 && CO <= MAXC && CI <= MAXC && CO * CI <= 8192;
}
// zh16: the jobs' z_{l-1} rows are fp16 (act16 bit 0, layers 2..4); dz rows are bf16 under act16 bit 1 (the
// split-bf16 kernel only: act16 is a perf-mode option like wgrad_split_bf16)
template <int CO, int CI>
static void launch_wgrad_mf_t(Dev& d, const MfJobs& M, int njob, bool split, bool zh16, hipStream_t st) {
  if constexpr (CO % 16 == 0 && CI % 16 == 0 && CO <= MAXC && CI <= MAXC && CO * CI <= 8192) {
    if (split) {
      const bool gh = d.a16 & 2;
      if constexpr (a16_shape(CI, CO)) {
        if (zh16 && gh) { hipLaunchKernelGGL((k_wgrad_bx3<CO, CI, b16, f16>), dim3(M.KS, njob), dim3(BLK), 0, st, d, M); return; }
        if (zh16) { hipLaunchKernelGGL((k_wgrad_bx3<CO, CI, float, f16>), dim3(M.KS, njob), dim3(BLK), 0, st, d, M); return; }
        if (gh) { hipLaunchKernelGGL((k_wgrad_bx3<CO, CI, b16, float>), dim3(M.KS, njob), dim3(BLK), 0, st, d, M); return; }
      }
      hipLaunchKernelGGL((k_wgrad_bx3<CO, CI, float, float>), dim3(M.KS, njob), dim3(BLK), 0, st, d, M);
    } else {
      hipLaunchKernelGGL((k_wgrad_mf<CO, CI>), dim3(M.KS, njob), dim3(BLK), 0, st, d, M);
    }
  }
}
template <int CO>
static void launch_wgrad_mf_ci(int CI, Dev& d, const MfJobs& M, int njob, bool split, bool zh16, hipStream_t st) {
  switch (CI) {
#define CASE(c) case c: launch_wgrad_mf_t<CO, c>(d, M, njob, split, zh16, st); break;
    RPC_HID(CASE)
#undef CASE
  }
}
static void launch_wgrad_mf(int CO, int CI, Dev& d, const MfJobs& M, int njob, bool split, bool zh16, hipStream_t st) {
  switch (CO) {
#define CASE(c) case c: launch_wgrad_mf_ci<c>(CI, d, M, njob, split, zh16, st); break;
    RPC_HID(CASE)
#undef CASE
  }
}
static int launch_bwd_first(int CO, Dev& d, hipStream_t st, int src) {
  const unsigned nq = (unsigned)((d.S / 4 + BLK - 1) / BLK);
  hipLaunchKernelGGL(k_bwd_first_pp, dim3(nq, CO), dim3(BLK), 0, st, d, src, CO);
  return RPC_OK;
}

}  // namespace pert
}  // namespace rpc

using namespace rpc;
using namespace rpc::pert;

extern "C" size_t rpc_perturber_workspace_size(const rpc_perturber_cfg* cfg, int rows, int slots) {
  Layout L;
  if (!cfg || make_layout(cfg, rows, slots, &L) != RPC_OK) return 0;
  return L.total;
}

extern "C" int rpc_perturber_forward(const rpc_perturber_cfg* cfg, const float* const* params,
                                     const float* x, int rows, int slots, const int* num_points,
                                     float* out, float* vfe_out, float* losses, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  if (!cfg || !params || !x || !out || !losses || rows < 1 || slots < 1) return RPC_ERR_ARG;
  if (num_points && (!vfe_out || cfg->vfe_features < 1 || cfg->vfe_features > cfg->F)) return RPC_ERR_ARG;
  if (!num_points && slots != 1) return RPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  Dev d;
  Layout L;
  int rc = fill_dev(cfg, params, x, rows, slots, num_points, workspace, workspace_bytes, d, L);
  if (rc) return rc;
  d.out = out;
  d.vfe = vfe_out;
  d.losses = losses;
  RPC_CHECK(hipMemsetAsync(d.ticket, 0, sizeof(unsigned) * NTICKET * TSTRIDE, st));
  if (d.fused) {
    ValidCount vc{x, slots, cfg->F, rows};
    int* cnt = (int*)((char*)workspace + L.cnt);
    RPC_CHECK(hipMemsetAsync(cnt, 0, sizeof(int) * ((size_t)rows + 1), st));
    const long long npts = (long long)rows * slots;
    if (npts > 0)
      hipLaunchKernelGGL(k_valid_count_pts, dim3((unsigned)((npts + BLK - 1) / BLK)), dim3(BLK), 0, st, vc, cnt);
    RPC_LAUNCH_CHECK();
    size_t sb = L.scan_bytes;
    RPC_CHECK(hipcub::DeviceScan::ExclusiveSum((char*)workspace + L.scan_tmp, sb, cnt, d.off, rows + 1, st));
  }
  const int F = cfg->F;
  if (F == 4) hipLaunchKernelGGL((k_xstats<4>), dim3(GRID), dim3(BLK), 0, st, d);
  else hipLaunchKernelGGL((k_xstats<5>), dim3(GRID), dim3(BLK), 0, st, d);
  RPC_LAUNCH_CHECK();
  if (!cfg->training) {
    hipLaunchKernelGGL(k_bn_eval, dim3(1), dim3(BLK), 0, st, d);
    RPC_LAUNCH_CHECK();
  }
  rc = F == 4 ? launch_first<4>(d.C[1], d, st) : launch_first<5>(d.C[1], d, st);
  if (rc) return rc;
  RPC_LAUNCH_CHECK();
  if (cfg->training) {
    rc = launch_colstats(d.C[1], 0, d, 0, nullptr, 1, st);
    if (rc) return rc;
    RPC_LAUNCH_CHECK();
  }
  for (int l = 1; l < 5; ++l) {
    rc = launch_mid(d.C[l], d.C[l + 1], d, l, st, false);
    if (rc) return rc;
    RPC_LAUNCH_CHECK();
  }
  rc = F == 4 ? launch_last<4>(d.C[5], d, st, false) : launch_last<5>(d.C[5], d, st, false);
  if (rc) return rc;
  RPC_LAUNCH_CHECK();
  int ng = grid_for((long long)rows * slots * F, BLK, 1024);
  hipLaunchKernelGGL(k_restore, dim3(ng), dim3(BLK), 0, st, d, F);
  RPC_LAUNCH_CHECK();
  if (d.fused) {
    int nv = (rows * d.vfe_f + BLK - 1) / BLK;
    hipLaunchKernelGGL(k_vfe, dim3(nv), dim3(BLK), 0, st, d, F);
    RPC_LAUNCH_CHECK();
  }
  return RPC_OK;
}

extern "C" int rpc_perturber_backward(const rpc_perturber_cfg* cfg, const float* const* params,
                                      const float* x, int rows, int slots, const int* num_points,
                                      const float* dout, const float* dlosses, float* const* grads,
                                      void* workspace, size_t workspace_bytes, void* stream) {
  if (!cfg || !params || !x || !dout || !dlosses || !grads || rows < 1 || slots < 1) return RPC_ERR_ARG;
  if (!cfg->training) return RPC_ERR_ARG;
  hipStream_t st = (hipStream_t)stream;
  Dev d;
  Layout L;
  int rc = fill_dev(cfg, params, x, rows, slots, num_points, workspace, workspace_bytes, d, L);
  if (rc) return rc;
  d.dout = dout;
  d.dl = dlosses;
  RPC_CHECK(hipMemsetAsync(d.ticket, 0, sizeof(unsigned) * NTICKET * TSTRIDE, st));
  const int F = cfg->F;
  rc = F == 4 ? launch_last<4>(d.C[5], d, st, true) : launch_last<5>(d.C[5], d, st, true);
  if (rc) return rc;
  RPC_LAUNCH_CHECK();
  rc = launch_colstats(d.C[5], 1, d, 4, d.dh[0], 7, st);
  if (rc) return rc;
  RPC_LAUNCH_CHECK();
  int src = 0;
  for (int l = 4; l >= 1; --l) {
    rc = launch_mid(d.C[l], d.C[l + 1], d, l, st, true, src);
    if (rc) return rc;
    RPC_LAUNCH_CHECK();
    src ^= 1;
  }
  rc = launch_bwd_first(d.C[1], d, st, src);
  if (rc) return rc;
  RPC_LAUNCH_CHECK();
  // weight-gradient jobs
  Jobs J;
  memset(&J, 0, sizeof(J));
  GradOut G;
  memset(&G, 0, sizeof(G));
  int nj = 0, eoff = 0;
  auto add = [&](const float* dz, int CO, int CI, int hsrc, const float* h, const float* bn,
                 float* gW, float* gb) {
    Job& j = J.j[nj];
    j.dz = dz; j.CO = CO; j.CI = CI; j.hsrc = hsrc; j.h = h; j.bn = bn;
    j.eoff = eoff; j.nelem = CO * (CI + 1);
    G.W[nj] = gW; G.b[nj] = gb;
    eoff += j.nelem;
    ++nj;
  };
  for (int l = 0; l < 6; ++l) {
    int CO = d.C[l + 1], CI = d.C[l];
    if (l == 0) add(d.dz[0], CO, CI, H_XN, nullptr, nullptr, grads[0], grads[1]);
    else add(d.dz[l], CO, CI, H_BNRELU, d.z[l - 1], d.bn[l - 1],
             grads[l < 5 ? 6 * l : 30], grads[l < 5 ? 6 * l + 1 : 31]);
  }
  if (cfg->use_attention) {
    add(d.da, d.A, F, H_XN, nullptr, nullptr, grads[32], grads[33]);
    add(d.dsig, 1, d.A, H_RAW, d.aact, nullptr, grads[34], grads[35]);
  }
  J.njob = nj;
  J.total = eoff;
  // MFMA jobs: hidden layers 1..4 whose (CO, CI) tile; grouped by shape (one launch per shape)
  bool is_mf[MAXJOB] = {false};
  for (int l = 1; l < 5; ++l) is_mf[l] = wgrad_mf_ok(d.C[l + 1], d.C[l]);
  Jobs JV;
  memset(&JV, 0, sizeof(JV));
  int nv = 0;
  for (int k = 0; k < nj; ++k)
    if (!is_mf[k]) JV.j[nv++] = J.j[k];
  JV.njob = nv;
  JV.total = J.total;
  int chunks = 0;
  for (int k = 0; k < nv; ++k) {
    JV.cbase[k] = chunks;
    JV.echunks[k] = (JV.j[k].nelem + BLK * EPT - 1) / (BLK * EPT);
    chunks += JV.echunks[k];
  }
  const int ks = KS_MAX;   // point ranges of the weight-gradient passes (= partial rows reduced)
  J.KS = JV.KS = ks;
  if (nv) {
    // one launch over KS point ranges covering every VALU job (LDS sized to the jobs' tile rows)
    int nrow = 0, nel = 0;
    for (int k = 0; k < nv; ++k) { nrow += JV.j[k].CO + JV.j[k].CI; nel += JV.j[k].nelem; }
    auto lds_of = [&](int tr) {
      return (size_t)2 * ((nrow * (tr + 1) + 3) & ~3) * sizeof(float) + (size_t)nrow * sizeof(RowSrc);
    };
    int tr = 0;
    for (int t = 256; t >= 64 && !tr; t >>= 1)
      if (lds_of(t) <= 160 * 1024 && nrow * (t / 4) <= WPB * WPRE) tr = t;
    if (nel > WPB * WEPT || !tr) {
      // wide VALU hidden layers (CO * CI > 8192): the per-job chunked kernel
      if (F == 4) hipLaunchKernelGGL((k_wgrad<4>), dim3(chunks * ks), dim3(BLK), 0, st, d, JV);
      else hipLaunchKernelGGL((k_wgrad<5>), dim3(chunks * ks), dim3(BLK), 0, st, d, JV);
    } else {
      const size_t lds = lds_of(tr);
#define WPP_CASE(FF, TT)                                                                                      \
  if (F == FF && tr == TT) {                                                                                  \
    if (lds > 64 * 1024)                                                                                      \
      (void)hipFuncSetAttribute((const void*)k_wgrad_pp<FF, TT>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    hipLaunchKernelGGL((k_wgrad_pp<FF, TT>), dim3(ks), dim3(WPB), lds, st, d, JV, nrow);                     \
  }
      WPP_CASE(4, 256) WPP_CASE(4, 128) WPP_CASE(4, 64) WPP_CASE(5, 256) WPP_CASE(5, 128) WPP_CASE(5, 64)
#undef WPP_CASE
    }
    RPC_LAUNCH_CHECK();
  }
  // one launch per distinct (shape, z_{l-1} row type), covering every layer of that kind
  auto zh16 = [&](int k) { return (d.a16 & 1) && k - 1 >= 1 && k - 1 <= 3; };
  for (int l = 1; l < 5; ++l) {
    if (!is_mf[l]) continue;
    auto same = [&](int k) { return is_mf[k] && d.C[k + 1] == d.C[l + 1] && d.C[k] == d.C[l] && zh16(k) == zh16(l); };
    bool first = true;
    for (int k = 1; k < l; ++k)
      if (same(k)) first = false;
    if (!first) continue;
    MfJobs M;
    memset(&M, 0, sizeof(M));
    int nm = 0;
    for (int k = l; k < 5; ++k)
      if (same(k)) M.j[nm++] = MfJob{d.dz[k], d.z[k - 1], d.bn[k - 1], J.j[k].eoff};
    M.total = J.total;
    M.KS = ks;
    launch_wgrad_mf(d.C[l + 1], d.C[l], d, M, nm, cfg->wgrad_split_bf16 != 0, zh16(l), st);
    RPC_LAUNCH_CHECK();
  }
  for (int l = 0; l < 5; ++l) {
    G.gg[l] = grads[6 * l + 2];
    G.gb[l] = grads[6 * l + 3];
  }
  int nbn = d.C[1] + d.C[2] + d.C[3] + d.C[4] + d.C[5];
  int nr = (J.total + nbn + 63) / 64;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(nr), dim3(BLK), 0, st, d, J, G);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}
