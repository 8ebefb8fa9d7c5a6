// ★ HardVFE: the "VFE per-voxel PointNet MLP + max" of BASELINE.json's north_star.
// Restates upstream mmdet3d HardVFE / VFELayer (mmdet3d/models/voxel_encoders/voxel_encoder.py, not
// vendored) — semantics in oracle/hard_vfe.py; called where the reference calls its voxel encoder
// (models/detectors/adversarial_voxelnet.py:135-137, adversarial_centerpoint.py:100).
//
// Layout and kernels (VALU + LDS; the layers are 16-128 wide, far below where MFMA pays, and the
// whole encoder is a few GFLOP):
// * rows r = v*T + t (one row per voxel slot); per-layer pre-BN activations y_l [V*T][CP_l] fp32,
//   CP_l = the layer width rounded up to a power of two in 16..128 (padded channels stay zero);
// * a block walks voxel-aligned tiles of VB = ROWS / T voxels, so each voxel's slots ("point group")
//   sit in LDS together and the slot max is a segmented max over T consecutive LDS rows;
// * layer l > 0 consumes [p, max(p)] of layer l-1 as W_p p + W_m max(p): the max half is one
//   product per voxel instead of one per slot;
// * BatchNorm statistics are per-block partial sums reduced in fixed order by rpc_bn_finalize
//   (deterministic), weight gradients per-block register tiles reduced by k_slab_reduce;
// * forward: k_prep (weights -> padded / transposed tiles, all layers in one launch), per layer
//   k_fwd (+ finalize), k_out (last layer max + argmax); backward: k_top (last layer BN-backward
//   sums from the argmax slots only) then per layer k_bwd (dy, dW tile, input gradient, and the
//   previous layer's BN-backward sums in the same pass) + slab reduce + finalize.
#include <algorithm>

#include "common.h"

namespace rpc {
namespace hvfe {

constexpr int BLK = 256;
constexpr int MAXL = 4;
constexpr int K0P = 16;      // decorated input width, padded
constexpr int MAXG = 512;    // blocks per launch (fixed for a given V: deterministic reductions)

struct Geo {
  int V, T, F, L, C0, ROWS, VB, ntiles, G;
  int cl, ce, di;
  int C[MAXL], CP[MAXL], KP[MAXL];
  float vs[3], off[3];
};

struct Bufs {
  float* y[MAXL];
  float* dp[MAXL];
  unsigned char* idx[MAXL];
  float* bn[MAXL];
  float* bnb[MAXL];
  float* wf[MAXL];   // [KP][CP]   forward, input part (transposed)
  float* wm[MAXL];   // [KP][CP]   forward, max part (l > 0)
  float* wd[MAXL];   // [CP][KP]   data gradient, input part
  float* wdm[MAXL];  // [CP][KP]   data gradient, max part (l > 0)
  float* part;       // [G][2*Cmax]
  float* slab;       // [G][Cmax*Kmax]
};

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ void st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ float f4(const float4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

// ---------------------------------------------------------------- weight prep (all layers)
struct PrepArgs {
  const float* W[MAXL];
  float* wf[MAXL];
  float* wm[MAXL];
  float* wd[MAXL];
  float* wdm[MAXL];
  int C[MAXL], CP[MAXL], KP[MAXL], Kin[MAXL];  // Kin = real width of the input part
};

__global__ __launch_bounds__(BLK) void k_prep(PrepArgs a) {
  const int l = blockIdx.y;
  const int CP = a.CP[l], KP = a.KP[l], C = a.C[l], Kin = a.Kin[l];
  const int Ktot = l == 0 ? Kin : 2 * Kin;
  const int e = blockIdx.x * BLK + threadIdx.x;
  if (e >= KP * CP) return;
  const int k = e / CP, c = e - k * CP;
  const bool ok = k < Kin && c < C;
  const float w = ok ? a.W[l][(size_t)c * Ktot + k] : 0.0f;
  a.wf[l][(size_t)k * CP + c] = w;
  a.wd[l][(size_t)c * KP + k] = w;
  if (l > 0) {
    const float m = ok ? a.W[l][(size_t)c * Ktot + Kin + k] : 0.0f;
    a.wm[l][(size_t)k * CP + c] = m;
    a.wdm[l][(size_t)c * KP + k] = m;
  }
}

// eval mode: BN from the running statistics, in rpc_bn_finalize's mode-0 layout (scale, beta, mean, invstd)
__global__ void k_bn_eval(const float* gamma, const float* beta, const float* rm, const float* rv, float eps, int C,
                          float* bn) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = 1.0f / sqrtf(rv[c] + eps);
  bn[c] = gamma[c] * invstd;
  bn[C + c] = beta[c];
  bn[2 * C + c] = rm[c];
  bn[3 * C + c] = invstd;
}

// ---------------------------------------------------------------- input tile (shared by fwd / bwd)
struct TileIn {
  const float* feat;   // [V][T][F]
  const int* np;
  const int* coors;    // [V][4] (b, z, y, x)
  const float* yprev;  // y_{l-1}
  const float* bnprev; // forward BN of l-1 (scale, beta, mean, invstd)
  int Cprev;           // real width of l-1
};

// sX[r][k] (pitch KP+4) for the rows of voxels [v0, v0+VBt); rows >= VBt*T zero. FIRST: the masked
// decorated features (sMean must hold room for VB*3); else relu(bn(y_{l-1})).
template <bool FIRST>
__device__ void load_tile(const Geo& g, const TileIn& in, int v0, int VBt, int KP, float* sX, float* sMean) {
  const int R = VBt * g.T, px = KP + 4;
  if (FIRST) {
    if (g.cl) {
      for (int e = threadIdx.x; e < VBt * 3; e += BLK) {
        const int vv = e / 3, d = e - vv * 3, v = v0 + vv;
        const float* f = in.feat + (size_t)v * g.T * g.F + d;
        float s = 0.0f;
        for (int t = 0; t < g.T; ++t) s += f[(size_t)t * g.F];
        sMean[e] = s / (float)in.np[v];
      }
      __syncthreads();
    }
    for (int e = threadIdx.x; e < g.ROWS * K0P; e += BLK) {
      const int r = e / K0P, k = e - r * K0P;
      float val = 0.0f;
      if (r < R) {
        const int vv = r / g.T, t = r - vv * g.T, v = v0 + vv;
        if (t < in.np[v]) {
          const float* f = in.feat + ((size_t)v * g.T + t) * g.F;
          int kk = k;
          if (kk < g.F) {
            val = f[kk];
          } else {
            kk -= g.F;
            bool done = false;
            if (g.cl) {
              if (kk < 3) { val = f[kk] - sMean[vv * 3 + kk]; done = true; }
              kk -= 3;
            }
            if (!done && g.ce) {
              if (kk >= 0 && kk < 3) {
                const int* co = in.coors + (size_t)v * 4;
                val = f[kk] - ((float)co[3 - kk] * g.vs[kk] + g.off[kk]);
                done = true;
              }
              kk -= 3;
            }
            if (!done && g.di && kk == 0) val = sqrtf(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
          }
        }
      }
      sX[r * px + k] = val;
    }
  } else {
    const int C = in.Cprev;
    const float* bn = in.bnprev;
    for (int e = threadIdx.x; e < g.ROWS * (KP / 4); e += BLK) {
      const int r = e / (KP / 4), k0 = (e - r * (KP / 4)) * 4;
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < R) {
        const float4 y = ld4(in.yprev + ((size_t)v0 * g.T + r) * KP + k0);
        float ov[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int k = k0 + j;
          ov[j] = k < C ? fmaxf((f4(y, j) - bn[2 * C + k]) * bn[k] + bn[C + k], 0.0f) : 0.0f;
        }
        o = make_float4(ov[0], ov[1], ov[2], ov[3]);
      }
      st4(sX + r * px + k0, o);
    }
  }
}

// ---------------------------------------------------------------- forward, one layer
// y_l = x W_p^T (+ max(p_{l-1}) W_m^T); BN partial sums of y_l; (l > 0) argmax of layer l-1.
template <bool FIRST, int CP>
__global__ __launch_bounds__(BLK) void k_fwd(Geo g, TileIn in, int l, const float* __restrict__ wf,
                                             const float* __restrict__ wm, float* __restrict__ y,
                                             unsigned char* __restrict__ idxprev, float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NCT = CP / 4;
  const int KP = FIRST ? K0P : g.CP[l - 1];
  const int px = KP + 4;
  float* sW = smem;                       // [KP][CP]
  float* sX = sW + KP * CP;               // [ROWS][KP+4]
  float* sM = sX + g.ROWS * px;           // [VB][KP]  (FIRST: point means [VB][3])
  float* sQ = sM + g.VB * KP;             // [VB][CP]
  for (int e = threadIdx.x; e < KP * CP / 4; e += BLK) st4(sW + 4 * e, ld4(wf + 4 * e));
  const int C = g.C[l];
  const int ct = threadIdx.x % NCT, c0 = ct * 4;
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  for (int tile = blockIdx.x; tile < g.ntiles; tile += gridDim.x) {
    const int v0 = tile * g.VB, VBt = min(g.VB, g.V - v0), R = VBt * g.T;
    __syncthreads();
    load_tile<FIRST>(g, in, v0, VBt, KP, sX, sM);
    __syncthreads();
    if (!FIRST) {
      // segmented max over each voxel's T slots (first index of the maximum), then the per-voxel
      // max-half product q[v][c] = sum_k max[v][k] W_m[c][k]
      for (int e = threadIdx.x; e < VBt * KP; e += BLK) {
        const int vv = e / KP, k = e - vv * KP;
        const float* col = sX + vv * g.T * px + k;
        float m = col[0];
        int am = 0;
        for (int t = 1; t < g.T; ++t) {
          const float x = col[t * px];
          if (x > m) { m = x; am = t; }
        }
        sM[e] = m;
        idxprev[(size_t)(v0 + vv) * KP + k] = (unsigned char)am;
      }
      __syncthreads();
      for (int e = threadIdx.x; e < VBt * CP; e += BLK) {
        const int vv = e / CP, c = e - vv * CP;
        const float* mv = sM + vv * KP;
        float q = 0.0f;
        for (int k = 0; k < in.Cprev; ++k) q = fmaf(mv[k], wm[(size_t)k * CP + c], q);
        sQ[e] = q;
      }
      __syncthreads();
    }
    // y tile: thread micro-tiles of 4 rows x 4 channels, fixed channel tile per thread
    for (int rt = threadIdx.x / NCT; rt * 4 < R; rt += BLK / NCT) {
      const int r0 = rt * 4;
      float acc[4][4] = {};
      for (int k = 0; k < KP; k += 4) {
        float4 a[4], b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = ld4(sX + (r0 + i) * px + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = ld4(sW + (k + j) * CP + c0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            float s = acc[i][jj];
            s = fmaf(a[i].x, f4(b[0], jj), s);
            s = fmaf(a[i].y, f4(b[1], jj), s);
            s = fmaf(a[i].z, f4(b[2], jj), s);
            s = fmaf(a[i].w, f4(b[3], jj), s);
            acc[i][jj] = s;
          }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + i;
        if (r >= R) break;
        float o[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          o[jj] = acc[i][jj] + (FIRST ? 0.0f : sQ[(r / g.T) * CP + c0 + jj]);
          s1[jj] += (double)o[jj];
          s2[jj] += (double)o[jj] * (double)o[jj];
        }
        st4(y + ((size_t)v0 * g.T + r) * CP + c0, make_float4(o[0], o[1], o[2], o[3]));
      }
    }
  }
  if (!part) return;
  // fixed-order combine of the row groups sharing a channel tile
  __syncthreads();
  double* red = reinterpret_cast<double*>(smem);   // [BLK][8]
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[threadIdx.x * 8 + j] = s1[j];
    red[threadIdx.x * 8 + 4 + j] = s2[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += BLK) {
    const int t0 = c / 4, j = c % 4;
    double a = 0.0, b = 0.0;
    for (int t = t0; t < BLK; t += NCT) {
      a += red[t * 8 + j];
      b += red[t * 8 + 4 + j];
    }
    part[(size_t)blockIdx.x * 2 * C + c] = (float)a;
    part[(size_t)blockIdx.x * 2 * C + C + c] = (float)b;
  }
}

// last layer: out[v][c] = max_t relu(bn(y[v,t][c])), argmax kept for the backward
__global__ __launch_bounds__(BLK) void k_out(const float* __restrict__ y, const float* __restrict__ bn, int V, int T,
                                             int C, int CP, float* __restrict__ out, unsigned char* __restrict__ idx) {
  const long long e = (long long)blockIdx.x * BLK + threadIdx.x;
  if (e >= (long long)V * CP) return;
  const int v = (int)(e / CP), c = (int)(e - (long long)v * CP);
  if (c >= C) { idx[e] = 0; return; }
  const float sc = bn[c], be = bn[C + c], mu = bn[2 * C + c];
  const float* p = y + (size_t)v * T * CP + c;
  float m = fmaxf((p[0] - mu) * sc + be, 0.0f);
  int am = 0;
  for (int t = 1; t < T; ++t) {
    const float x = fmaxf((p[(size_t)t * CP] - mu) * sc + be, 0.0f);
    if (x > m) { m = x; am = t; }
  }
  out[(size_t)v * C + c] = m;
  idx[e] = (unsigned char)am;
}

// ---------------------------------------------------------------- backward
// last layer BN-backward sums: only the argmax slot of each (voxel, channel) carries a gradient
template <int CP>
__global__ __launch_bounds__(BLK) void k_top(Geo g, const float* __restrict__ y, const float* __restrict__ bn,
                                             const unsigned char* __restrict__ idx, const float* __restrict__ dout,
                                             float* __restrict__ part) {
  __shared__ double red[BLK][2];
  const int L = g.L - 1, C = g.C[L];
  const int c = threadIdx.x % CP, vl = threadIdx.x / CP;
  const int vpb = (g.V + gridDim.x - 1) / gridDim.x;
  const int va = blockIdx.x * vpb, vb = min(g.V, va + vpb);
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const float sc = bn[c], be = bn[C + c], mu = bn[2 * C + c], is = bn[3 * C + c];
    for (int v = va + vl; v < vb; v += BLK / CP) {
      const int t = idx[(size_t)v * CP + c];
      const float yy = y[((size_t)v * g.T + t) * CP + c];
      if ((yy - mu) * sc + be > 0.0f) {
        const float d = dout[(size_t)v * C + c];
        s1 += (double)d;
        s2 += (double)(d * ((yy - mu) * is));
      }
    }
  }
  red[threadIdx.x][0] = s1;
  red[threadIdx.x][1] = s2;
  __syncthreads();
  if (threadIdx.x < C) {
    double a = 0.0, b = 0.0;
    for (int t = threadIdx.x; t < BLK; t += CP) {
      a += red[t][0];
      b += red[t][1];
    }
    part[(size_t)blockIdx.x * 2 * C + threadIdx.x] = (float)a;
    part[(size_t)blockIdx.x * 2 * C + C + threadIdx.x] = (float)b;
  }
}

struct BwdArgs {
  const float* y;        // y_l
  const float* bn;       // forward BN of l
  const float* bnb;      // backward BN of l (gi, m1, m2, mean, invstd)
  const float* dp;       // gradient wrt p_l (l < L-1)
  const float* dout;     // [V][C] (l == L-1)
  const unsigned char* idx;      // argmax of l (l == L-1)
  const unsigned char* idxprev;  // argmax of l-1
  const float* wd;
  const float* wdm;
  float* dy;             // dy_l rows out (may alias dp: each row is read, then written, by one thread)
  float* dpprev;         // gradient wrt p_{l-1}
  float* part;           // BN-backward sums of l-1
  float* dfeat;          // FIRST: [V][T][F]
  int top;
};

// dy_l = BN-backward(dz_l) (kept for k_wgrad); input gradient -> dp_{l-1} (+ BN-backward sums of
// l-1) or, for layer 0, the gradient of the raw features through the decoration.
template <bool FIRST, int CP>
__global__ __launch_bounds__(BLK) void k_bwd(Geo g, TileIn in, int l, BwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NCT = CP / 4;
  const int KP = FIRST ? K0P : g.CP[l - 1];
  const int px = KP + 4, pd = CP + 4;
  const int C = g.C[l];
  float* sWd = smem;                      // [CP][KP]
  float* sX = sWd + CP * KP;              // [ROWS][KP+4]
  float* sDY = sX + g.ROWS * px;          // [ROWS][CP+4]
  float* sM = sDY + g.ROWS * pd;          // [VB][KP]   (FIRST: point means, then cluster sums)
  float* sDYs = sM + g.VB * KP;           // [VB][CP]
  float* sQd = sDYs + g.VB * CP;          // [VB][KP]
  for (int e = threadIdx.x; e < CP * KP / 4; e += BLK) st4(sWd + 4 * e, ld4(a.wd + 4 * e));
  (void)NCT;
  const float* bn = a.bn;
  const float* bnb = a.bnb;
  // input-gradient micro-tiles: fixed k tile per thread (KP/4 divides BLK)
  const int nkt_dx = KP / 4;
  const int kt_dx = threadIdx.x % nkt_dx, k0_dx = kt_dx * 4;
  double s1[4] = {0, 0, 0, 0}, s2[4] = {0, 0, 0, 0};
  const int Cprev = in.Cprev;
  const float* bnp = in.bnprev;
  for (int tile = blockIdx.x; tile < g.ntiles; tile += gridDim.x) {
    const int v0 = tile * g.VB, VBt = min(g.VB, g.V - v0), R = VBt * g.T;
    __syncthreads();
    load_tile<FIRST>(g, in, v0, VBt, KP, sX, sM);
    // dy rows
    for (int e = threadIdx.x; e < g.ROWS * NCT; e += BLK) {
      const int r = e / NCT, cq = (e - r * NCT) * 4;
      float o[4] = {0.f, 0.f, 0.f, 0.f};
      if (r < R) {
        const size_t row = (size_t)v0 * g.T + r;
        const float4 y4 = ld4(a.y + row * CP + cq);
        float4 d4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (!a.top) d4 = ld4(a.dp + row * CP + cq);
        const int vv = r / g.T, t = r - vv * g.T;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = cq + j;
          if (c < C) {
            const float yy = f4(y4, j);
            float dz;
            if (a.top) {
              dz = (a.idx[(size_t)(v0 + vv) * CP + c] == t) ? a.dout[(size_t)(v0 + vv) * C + c] : 0.0f;
            } else {
              dz = f4(d4, j);
            }
            if (!((yy - bn[2 * C + c]) * bn[c] + bn[C + c] > 0.0f)) dz = 0.0f;
            const float xh = (yy - bnb[3 * C + c]) * bnb[4 * C + c];
            o[j] = bnb[c] * (dz - bnb[C + c] - xh * bnb[2 * C + c]);
          }
        }
      }
      const float4 o4 = make_float4(o[0], o[1], o[2], o[3]);
      st4(sDY + r * pd + cq, o4);
      if (r < R) st4(a.dy + ((size_t)v0 * g.T + r) * CP + cq, o4);
    }
    __syncthreads();
    if (!FIRST) {
      // per-voxel sums of dy
      for (int e = threadIdx.x; e < VBt * CP; e += BLK) {
        const int vv = e / CP, c = e - vv * CP;
        float s = 0.0f;
        for (int t = 0; t < g.T; ++t) s += sDY[(vv * g.T + t) * pd + c];
        sDYs[e] = s;
      }
      __syncthreads();
      // max-half input gradient per voxel: qd[v][k] = sum_c dys[v][c] W_m[c][k]
      for (int e = threadIdx.x; e < VBt * KP; e += BLK) {
        const int vv = e / KP, k = e - vv * KP;
        const float* dv = sDYs + vv * CP;
        float q = 0.0f;
        for (int c = 0; c < C; ++c) q = fmaf(dv[c], a.wdm[(size_t)c * KP + k], q);
        sQd[e] = q;
      }
    }
    __syncthreads();
    // input gradient: dx[r][k] = sum_c dy[r][c] Wd[c][k]  (rows x 4 k per thread; sX overwritten)
    for (int rt = threadIdx.x / nkt_dx; rt * 4 < R; rt += BLK / nkt_dx) {
      const int r0 = rt * 4;
      float dx[4][4] = {};
#pragma unroll 2
      for (int c = 0; c < CP; c += 4) {
        float4 d[4], w[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) d[i] = ld4(sDY + (r0 + i) * pd + c);
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = ld4(sWd + (c + j) * KP + k0_dx);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            float s = dx[i][kk];
            s = fmaf(d[i].x, f4(w[0], kk), s);
            s = fmaf(d[i].y, f4(w[1], kk), s);
            s = fmaf(d[i].z, f4(w[2], kk), s);
            s = fmaf(d[i].w, f4(w[3], kk), s);
            dx[i][kk] = s;
          }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = r0 + i;
        if (r >= R) break;
        const int vv = r / g.T, t = r - vv * g.T, v = v0 + vv;
        float* xr = sX + r * px + k0_dx;
        if (FIRST) {
          const bool live = t < in.np[v];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) xr[kk] = live ? dx[i][kk] : 0.0f;
        } else {
          const size_t row = (size_t)v * g.T + t;
          const float4 yp = ld4(in.yprev + row * KP + k0_dx);
          float o[4];
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) {
            const int k = k0_dx + kk;
            float d = dx[i][kk];
            if (a.idxprev[(size_t)v * KP + k] == t) d += sQd[vv * KP + k];
            o[kk] = d;
            if (k < Cprev && xr[kk] > 0.0f) {   // ReLU of l-1 active <=> p > 0
              const float xh = (f4(yp, kk) - bnp[2 * Cprev + k]) * bnp[3 * Cprev + k];
              s1[kk] += (double)d;
              s2[kk] += (double)(d * xh);
            }
          }
          st4(a.dpprev + row * KP + k0_dx, make_float4(o[0], o[1], o[2], o[3]));
        }
      }
    }
    if (FIRST) {
      __syncthreads();
      // raw-feature gradient through the decoration (mask already applied to sX)
      if (g.cl) {
        for (int e = threadIdx.x; e < VBt * 3; e += BLK) {
          const int vv = e / 3, d = e - vv * 3;
          float s = 0.0f;
          for (int t = 0; t < g.T; ++t) s += sX[(vv * g.T + t) * px + g.F + d];
          sM[e] = s / (float)in.np[v0 + vv];
        }
        __syncthreads();
      }
      for (int e = threadIdx.x; e < R * g.F; e += BLK) {
        const int r = e / g.F, f = e - r * g.F;
        const int vv = r / g.T, t = r - vv * g.T, v = v0 + vv;
        const float* xr = sX + r * px;
        float d = xr[f];
        if (f < 3) {
          int off = g.F;
          if (g.cl) { d += xr[off + f] - sM[vv * 3 + f]; off += 3; }
          if (g.ce) { d += xr[off + f]; off += 3; }
          if (g.di) {
            const float* p = in.feat + ((size_t)v * g.T + t) * g.F;
            const float n = sqrtf(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
            if (n > 0.0f) d += xr[off] * (p[f] / n);
          }
        }
        a.dfeat[((size_t)v * g.T + t) * g.F + f] = d;
      }
    }
  }
  if (FIRST) return;
  __syncthreads();
  double* red = reinterpret_cast<double*>(smem);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    red[threadIdx.x * 8 + j] = s1[j];
    red[threadIdx.x * 8 + 4 + j] = s2[j];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < Cprev; k += BLK) {
    const int t0 = k / 4, j = k % 4;
    double x = 0.0, y2 = 0.0;
    for (int t = t0; t < BLK; t += nkt_dx) {
      x += red[t * 8 + j];
      y2 += red[t * 8 + 4 + j];
    }
    a.part[(size_t)blockIdx.x * 2 * Cprev + k] = (float)x;
    a.part[(size_t)blockIdx.x * 2 * Cprev + Cprev + k] = (float)y2;
  }
}

// dW_l = sum_rows x^T dy (x recomputed, dy from k_bwd); the max half sums per voxel. Each thread owns
// MT fixed 4x4 (k, c) tiles -> fixed summation order; one slab per block, reduced by k_slab_reduce.
template <bool FIRST, int CP, int MT>
__global__ __launch_bounds__(BLK) void k_wgrad(Geo g, TileIn in, int l, const float* __restrict__ dy,
                                               const unsigned char* __restrict__ idxprev, float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int NCT = CP / 4;
  const int KP = FIRST ? K0P : g.CP[l - 1];
  const int px = KP + 4, pd = CP + 4;
  const int C = g.C[l];
  float* sX = smem;                       // [ROWS][KP+4]
  float* sDY = sX + g.ROWS * px;          // [ROWS][CP+4]
  float* sM = sDY + g.ROWS * pd;          // [VB][KP]
  float* sDYs = sM + g.VB * KP;           // [VB][CP]
  const int Ktot = FIRST ? KP : 2 * KP;
  const int nmt = (Ktot / 4) * NCT;
  float acc[MT][4][4] = {};
  for (int tile = blockIdx.x; tile < g.ntiles; tile += gridDim.x) {
    const int v0 = tile * g.VB, VBt = min(g.VB, g.V - v0), R = VBt * g.T;
    __syncthreads();
    load_tile<FIRST>(g, in, v0, VBt, KP, sX, sM);
    for (int e = threadIdx.x; e < R * NCT; e += BLK) {
      const int r = e / NCT, cq = (e - r * NCT) * 4;
      st4(sDY + r * pd + cq, ld4(dy + ((size_t)v0 * g.T + r) * CP + cq));
    }
    __syncthreads();
    if (!FIRST) {
      for (int e = threadIdx.x; e < VBt * KP; e += BLK) {
        const int vv = e / KP, k = e - vv * KP;
        sM[e] = sX[(vv * g.T + idxprev[(size_t)(v0 + vv) * KP + k]) * px + k];
      }
      for (int e = threadIdx.x; e < VBt * CP; e += BLK) {
        const int vv = e / CP, c = e - vv * CP;
        float s = 0.0f;
        for (int t = 0; t < g.T; ++t) s += sDY[(vv * g.T + t) * pd + c];
        sDYs[e] = s;
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int mt = threadIdx.x + i * BLK;
      if (mt < nmt) {
        const int kt = mt / NCT, c0 = (mt - kt * NCT) * 4, k0 = kt * 4;
        const bool mx = !FIRST && k0 >= KP;
        const float* xb = mx ? sM + (k0 - KP) : sX + k0;
        const float* db = mx ? sDYs + c0 : sDY + c0;
        const int xs = mx ? KP : px, ds = mx ? CP : pd, n = mx ? VBt : R;
        for (int r = 0; r < n; ++r) {
          const float4 x = ld4(xb + r * xs), d = ld4(db + r * ds);
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int w = 0; w < 4; ++w) acc[i][u][w] = fmaf(f4(x, u), f4(d, w), acc[i][u][w]);
        }
      }
    }
  }
  // slab of this block, torch layout [C][K] (K = C0, or 2*C_{l-1}: input half, then max half)
  const int Cprev = in.Cprev;
  const int Kin = FIRST ? g.C0 : Cprev;
  const int Kl = FIRST ? g.C0 : 2 * Cprev;
  float* sl = slab + (size_t)blockIdx.x * C * Kl;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int mt = threadIdx.x + i * BLK;
    if (mt < nmt) {
      const int kt = mt / NCT, c0 = (mt - kt * NCT) * 4, k0 = kt * 4;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int kk = k0 + u;
        const int col = kk < KP ? (kk < Kin ? kk : -1) : (kk - KP < Cprev ? Cprev + kk - KP : -1);
        if (col < 0) continue;
#pragma unroll
        for (int w = 0; w < 4; ++w)
          if (c0 + w < C) sl[(size_t)(c0 + w) * Kl + col] = acc[i][u][w];
      }
    }
  }
}

// ---------------------------------------------------------------- host side
static inline size_t al(size_t x) { return (x + 255) & ~(size_t)255; }

static int pow2w(int c) {
  int p = 16;
  while (p < c) p <<= 1;
  return p;
}

static size_t fwd_lds(int KP, int CP, int ROWS, int VB) {
  size_t f = (size_t)KP * CP + (size_t)ROWS * (KP + 4) + (size_t)VB * KP + (size_t)VB * CP;
  return std::max(f * 4, (size_t)BLK * 8 * 8);
}
static size_t bwd_lds(int KP, int CP, int ROWS, int VB) {
  size_t f = (size_t)CP * KP + (size_t)ROWS * (KP + 4) + (size_t)ROWS * (CP + 4) + (size_t)VB * KP * 2 +
             (size_t)VB * CP;
  return std::max(f * 4, (size_t)BLK * 8 * 8);
}
static size_t wgrad_lds(int KP, int CP, int ROWS, int VB) {
  return ((size_t)ROWS * (KP + 4) + (size_t)ROWS * (CP + 4) + (size_t)VB * KP + (size_t)VB * CP) * 4;
}

static int make_geo(const RpcHardVfeCfg* c, int V, Geo& g) {
  if (!c || V < 0 || c->F < 3 || c->T < 1 || c->T > 64 || c->nlayers < 1 || c->nlayers > MAXL) return RPC_ERR_ARG;
  g = Geo{};
  g.V = V;
  g.T = c->T;
  g.F = c->F;
  g.L = c->nlayers;
  g.cl = c->with_cluster_center != 0;
  g.ce = c->with_voxel_center != 0;
  g.di = c->with_distance != 0;
  g.C0 = g.F + 3 * g.cl + 3 * g.ce + g.di;
  if (g.C0 > K0P) return RPC_ERR_UNSUPPORTED;
  for (int l = 0; l < g.L; ++l) {
    if (c->channels[l] < 1 || c->channels[l] > 128) return RPC_ERR_UNSUPPORTED;
    g.C[l] = c->channels[l];
    g.CP[l] = pow2w(g.C[l]);
    g.KP[l] = l == 0 ? K0P : g.CP[l - 1];
  }
  for (int d = 0; d < 3; ++d) {
    g.vs[d] = c->voxel_size[d];
    g.off[d] = (float)((double)c->voxel_size[d] / 2 + (double)c->pc_range_min[d]);
  }
  // rows per tile: 64 when every layer's LDS fits the CU, else 32 (T must fit a tile)
  for (int rows = 64; rows >= 32; rows >>= 1) {
    if (g.T > rows) break;
    const int vb = rows / g.T;
    size_t mx = 0;
    for (int l = 0; l < g.L; ++l) {
      mx = std::max(mx, fwd_lds(g.KP[l], g.CP[l], rows, vb));
      mx = std::max(mx, bwd_lds(g.KP[l], g.CP[l], rows, vb));
    }
    if (mx <= 160 * 1024) {
      g.ROWS = rows;
      g.VB = vb;
      break;
    }
  }
  if (!g.ROWS) return RPC_ERR_UNSUPPORTED;
  g.ntiles = V > 0 ? (V + g.VB - 1) / g.VB : 0;
  g.G = g.ntiles < MAXG ? g.ntiles : MAXG;
  return RPC_OK;
}

static size_t carve(const Geo& g, char* base, Bufs* b) {
  size_t o = 0;
  const size_t rows = (size_t)g.V * g.T;
  int cmax = 0, kmax = 0;
  auto take = [&](size_t bytes) -> char* { char* p = base ? base + o : nullptr; o += al(bytes); return p; };
  for (int l = 0; l < g.L; ++l) {
    const int K = l == 0 ? g.C0 : 2 * g.C[l - 1];
    cmax = std::max(cmax, g.C[l]);
    kmax = std::max(kmax, K);
    float* y = (float*)take(rows * g.CP[l] * 4);
    float* dp = (float*)take(rows * g.CP[l] * 4);   // gradient wrt p_l, then dy_l in place
    unsigned char* ix = (unsigned char*)take((size_t)g.V * g.CP[l]);
    float* bn = (float*)take((size_t)4 * g.C[l] * 4);
    float* bnb = (float*)take((size_t)5 * g.C[l] * 4);
    float* wf = (float*)take((size_t)g.KP[l] * g.CP[l] * 4);
    float* wm = (float*)take((size_t)g.KP[l] * g.CP[l] * 4);
    float* wd = (float*)take((size_t)g.KP[l] * g.CP[l] * 4);
    float* wdm = (float*)take((size_t)g.KP[l] * g.CP[l] * 4);
    if (b) {
      b->y[l] = y; b->dp[l] = dp; b->idx[l] = ix; b->bn[l] = bn; b->bnb[l] = bnb;
      b->wf[l] = wf; b->wm[l] = wm; b->wd[l] = wd; b->wdm[l] = wdm;
    }
  }
  const int G = g.G > 0 ? g.G : 1;
  float* part = (float*)take((size_t)G * 2 * cmax * 4);
  float* slab = (float*)take((size_t)G * cmax * kmax * 4);
  if (b) { b->part = part; b->slab = slab; }
  return o;
}

template <typename K>
static void set_lds(K kern, size_t bytes) {
  if (bytes > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <bool FIRST, int CP>
static void launch_fwd_t(const Geo& g, const TileIn& in, int l, const Bufs& b, float* part, hipStream_t st) {
  const size_t lds = fwd_lds(g.KP[l], CP, g.ROWS, g.VB);
  set_lds(k_fwd<FIRST, CP>, lds);
  hipLaunchKernelGGL((k_fwd<FIRST, CP>), dim3(g.G), dim3(BLK), lds, st, g, in, l, b.wf[l], b.wm[l], b.y[l],
                     l > 0 ? b.idx[l - 1] : nullptr, part);
}

static int launch_fwd(const Geo& g, const TileIn& in, int l, const Bufs& b, float* part, hipStream_t st) {
  const bool first = l == 0;
#define F1(cp) if (g.CP[l] == cp) { if (first) launch_fwd_t<true, cp>(g, in, l, b, part, st); \
                                    else launch_fwd_t<false, cp>(g, in, l, b, part, st); return RPC_OK; }
  F1(16) F1(32) F1(64) F1(128)
#undef F1
  return RPC_ERR_UNSUPPORTED;
}

template <bool FIRST, int CP>
static void launch_bwd_t(const Geo& g, const TileIn& in, int l, const BwdArgs& a, hipStream_t st) {
  const size_t lds = bwd_lds(g.KP[l], CP, g.ROWS, g.VB);
  set_lds(k_bwd<FIRST, CP>, lds);
  hipLaunchKernelGGL((k_bwd<FIRST, CP>), dim3(g.G), dim3(BLK), lds, st, g, in, l, a);
}

static int launch_bwd(const Geo& g, const TileIn& in, int l, const BwdArgs& a, hipStream_t st) {
#define B0(cp) if (g.CP[l] == cp) { if (l == 0) launch_bwd_t<true, cp>(g, in, l, a, st); \
                                    else launch_bwd_t<false, cp>(g, in, l, a, st); return RPC_OK; }
  B0(16) B0(32) B0(64) B0(128)
#undef B0
  return RPC_ERR_UNSUPPORTED;
}

template <bool FIRST, int CP, int MT>
static void launch_wgrad_t(const Geo& g, const TileIn& in, int l, const float* dy, const unsigned char* idxprev,
                           float* slab, hipStream_t st) {
  const size_t lds = wgrad_lds(g.KP[l], CP, g.ROWS, g.VB);
  set_lds(k_wgrad<FIRST, CP, MT>, lds);
  hipLaunchKernelGGL((k_wgrad<FIRST, CP, MT>), dim3(g.G), dim3(BLK), lds, st, g, in, l, dy, idxprev, slab);
}

static int launch_wgrad(const Geo& g, const TileIn& in, int l, const float* dy, const unsigned char* idxprev,
                        float* slab, hipStream_t st) {
  const int CP = g.CP[l], KP = g.KP[l];
  if (l == 0) {
#define W0(cp) if (CP == cp) { launch_wgrad_t<true, cp, 1>(g, in, l, dy, idxprev, slab, st); return RPC_OK; }
    W0(16) W0(32) W0(64) W0(128)
#undef W0
    return RPC_ERR_UNSUPPORTED;
  }
  const int nmt = (2 * KP / 4) * (CP / 4);
  const int mt = (nmt + BLK - 1) / BLK;
#define W1(cp, m) if (CP == cp && mt <= m) { launch_wgrad_t<false, cp, m>(g, in, l, dy, idxprev, slab, st); return RPC_OK; }
  W1(16, 1) W1(32, 1) W1(32, 2) W1(64, 1) W1(64, 2) W1(64, 4) W1(128, 2) W1(128, 4) W1(128, 8)
#undef W1
  return RPC_ERR_UNSUPPORTED;
}

template <int CP>
static void launch_top_t(const Geo& g, const Bufs& b, const float* dout, hipStream_t st) {
  const int L = g.L - 1;
  hipLaunchKernelGGL((k_top<CP>), dim3(g.G), dim3(BLK), 0, st, g, b.y[L], b.bn[L], b.idx[L], dout, b.part);
}

static TileIn tile_in(const Geo& g, const Bufs& b, int l, const float* feat, const int* np, const int* coors) {
  TileIn in{};
  in.feat = feat;
  in.np = np;
  in.coors = coors;
  if (l > 0) {
    in.yprev = b.y[l - 1];
    in.bnprev = b.bn[l - 1];
    in.Cprev = g.C[l - 1];
  }
  return in;
}

}  // namespace hvfe
}  // namespace rpc

using namespace rpc;
using namespace rpc::hvfe;

extern "C" size_t rpc_hard_vfe_workspace_size(const RpcHardVfeCfg* cfg, int V) {
  Geo g;
  if (make_geo(cfg, V, g) != RPC_OK) return 0;
  return carve(g, nullptr, nullptr);
}

extern "C" int rpc_hard_vfe_forward(const RpcHardVfeCfg* cfg, float* const* params, const float* feat,
                                    const int* np, const int* coors, int V, float* out, void* ws, size_t wsb,
                                    void* stream) {
  Geo g;
  int rc = make_geo(cfg, V, g);
  if (rc != RPC_OK) return rc;
  if (V == 0) return RPC_OK;
  if (!params || !feat || !np || !coors || !out || !ws) return RPC_ERR_ARG;
  for (int l = 0; l < g.L; ++l)
    for (int j = 0; j < 5; ++j)
      if (!params[5 * l + j]) return RPC_ERR_ARG;
  Bufs b;
  if (carve(g, (char*)ws, &b) > wsb) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  PrepArgs pa{};
  int mx = 0;
  for (int l = 0; l < g.L; ++l) {
    pa.W[l] = params[5 * l];
    pa.wf[l] = b.wf[l]; pa.wm[l] = b.wm[l]; pa.wd[l] = b.wd[l]; pa.wdm[l] = b.wdm[l];
    pa.C[l] = g.C[l]; pa.CP[l] = g.CP[l]; pa.KP[l] = g.KP[l];
    pa.Kin[l] = l == 0 ? g.C0 : g.C[l - 1];
    mx = std::max(mx, g.KP[l] * g.CP[l]);
  }
  hipLaunchKernelGGL(k_prep, dim3((mx + BLK - 1) / BLK, g.L), dim3(BLK), 0, st, pa);
  RPC_LAUNCH_CHECK();
  const int N = V * g.T;
  const bool train = cfg->training != 0;
  for (int l = 0; l < g.L; ++l) {
    float* const* p = params + 5 * l;
    if (!train)
      hipLaunchKernelGGL(k_bn_eval, dim3((g.C[l] + 127) / 128), dim3(128), 0, st, p[1], p[2], p[3], p[4],
                         cfg->bn_eps, g.C[l], b.bn[l]);
    rc = launch_fwd(g, tile_in(g, b, l, feat, np, coors), l, b, train ? b.part : nullptr, st);
    if (rc != RPC_OK) return rc;
    RPC_LAUNCH_CHECK();
    if (train) {
      rc = rpc_bn_finalize(b.part, g.G, g.C[l], N, 0, p[1], p[2], cfg->bn_eps, cfg->bn_momentum, p[3], p[4],
                           nullptr, b.bn[l], nullptr, nullptr, nullptr, stream);
      if (rc != RPC_OK) return rc;
    }
  }
  const int L = g.L - 1;
  const long long n = (long long)V * g.CP[L];
  hipLaunchKernelGGL(k_out, dim3((unsigned)((n + BLK - 1) / BLK)), dim3(BLK), 0, st, b.y[L], b.bn[L], V, g.T, g.C[L],
                     g.CP[L], out, b.idx[L]);
  RPC_LAUNCH_CHECK();
  return RPC_OK;
}

extern "C" int rpc_hard_vfe_backward(const RpcHardVfeCfg* cfg, float* const* params, const float* feat,
                                     const int* np, const int* coors, int V, const float* dout, float* dfeat,
                                     float* const* grads, void* ws, size_t wsb, void* stream) {
  Geo g;
  int rc = make_geo(cfg, V, g);
  if (rc != RPC_OK) return rc;
  if (!cfg->training) return RPC_ERR_UNSUPPORTED;
  if (!params || !grads) return RPC_ERR_ARG;
  if (V == 0) return RPC_OK;
  if (!feat || !np || !coors || !dout || !dfeat || !ws) return RPC_ERR_ARG;
  Bufs b;
  if (carve(g, (char*)ws, &b) > wsb) return RPC_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int N = V * g.T, L = g.L - 1;
  switch (g.CP[L]) {
    case 16: launch_top_t<16>(g, b, dout, st); break;
    case 32: launch_top_t<32>(g, b, dout, st); break;
    case 64: launch_top_t<64>(g, b, dout, st); break;
    default: launch_top_t<128>(g, b, dout, st);
  }
  RPC_LAUNCH_CHECK();
  for (int l = L; l >= 0; --l) {
    float* const* p = params + 5 * l;
    float* const* gr = grads + 3 * l;
    if (!gr[0] || !gr[1] || !gr[2]) return RPC_ERR_ARG;
    rc = rpc_bn_finalize(b.part, g.G, g.C[l], N, 1, p[1], p[2], cfg->bn_eps, cfg->bn_momentum, nullptr, nullptr,
                         b.bn[l], b.bnb[l], gr[1], gr[2], nullptr, stream);
    if (rc != RPC_OK) return rc;
    BwdArgs a{};
    a.y = b.y[l];
    a.bn = b.bn[l];
    a.bnb = b.bnb[l];
    a.top = l == L;
    a.dp = b.dp[l];
    a.dy = b.dp[l];
    a.dout = dout;
    a.idx = b.idx[l];
    a.idxprev = l > 0 ? b.idx[l - 1] : nullptr;
    a.wd = b.wd[l];
    a.wdm = b.wdm[l];
    a.dpprev = l > 0 ? b.dp[l - 1] : nullptr;
    a.part = b.part;
    a.dfeat = dfeat;
    const TileIn in = tile_in(g, b, l, feat, np, coors);
    rc = launch_bwd(g, in, l, a, st);
    if (rc != RPC_OK) return rc;
    RPC_LAUNCH_CHECK();
    rc = launch_wgrad(g, in, l, b.dp[l], a.idxprev, b.slab, st);
    if (rc != RPC_OK) return rc;
    RPC_LAUNCH_CHECK();
    const int K = l == 0 ? g.C0 : 2 * g.C[l - 1];
    slab_reduce(b.slab, g.G, (long long)g.C[l] * K, gr[0], st);
    RPC_LAUNCH_CHECK();
  }
  return RPC_OK;
}
