// a6 runtime: the SparseEncoder backward as ONE host call (rpc_sparse_backward).
//
// The backward of upstream mmdet3d SparseEncoder (12 sparse convs, SubMConv3d / SparseConv3d +
// BatchNorm1d + ReLU, and the SparseBasicBlock residuals of the basicblock variant) walks the layers
// in reverse: dense-BEV gradient gather, per layer the BatchNorm-backward finalize, the weight gradient
// and the data gradient into the layer below (its ReLU mask and BatchNorm-backward partial sums fused
// into the data-gradient epilogue). Issued from Python that is ~10 allocations, ~6 C-ABI calls, two
// stream switches and their events per layer — about 1.2 ms of host time per step, more than the GPU
// time of the kernels it issues, so the GPU waited on the host. Here the same launches, with the same
// arguments in the same order, come from one C++ loop over a layer table: temporaries are carved out of
// one caller-owned workspace (a bump arena, nothing freed during the call, so the side stream never
// races an allocator), and the weight gradients go to the caller's second stream behind one event per
// layer, joined back into the main stream before returning. Same kernels, same order, same bits as the
// Python loop in sparse_encoder.py (which remains the path for per-kernel timing / debugging).
#include <hip/hip_runtime.h>
#include <string.h>

#include <map>
#include <mutex>
#include <cstdlib>
#include <vector>

#include "common.h"
#include "rpc_hip.h"

namespace {

constexpr int BM = 64;   // rows per BatchNorm partial row (rpc_spconv_gemm_blocks)

inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }
inline int r8(int c) { return (c + 7) / 8 * 8; }

struct Arena {
  char* base;
  size_t cap, off;
  bool dry;
  void* take(size_t bytes) {
    off = (off + 255) & ~(size_t)255;
    void* p = dry ? nullptr : base + off;
    off += bytes;
    return p;
  }
  bool ok() const { return dry || off <= cap; }
};

// events of the main -> weight-gradient stream hand-offs, reused across calls (re-recording an event
// after a stream has been told to wait on it is safe: the wait captured the earlier record). One set per
// device (an event belongs to the device current at its creation), used under that device's lock: the
// whole issue of one rpc_sparse_backward holds it, so two host threads never interleave records and waits
// on the same events.
struct DevEvents {
  std::mutex mu;
  std::vector<hipEvent_t> ev;
};
std::mutex g_dev_mu;
std::map<int, DevEvents*> g_dev_events;   // never freed: the process's devices

DevEvents* device_events(int dev) {
  std::lock_guard<std::mutex> lk(g_dev_mu);
  DevEvents*& d = g_dev_events[dev];
  if (!d) d = new DevEvents();
  return d;
}

hipEvent_t event_at(DevEvents* d, size_t i) {
  while (d->ev.size() <= i) {
    hipEvent_t e;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    d->ev.push_back(e);
  }
  return d->ev[i];
}

// RPC_SPARSE_RES_FUSE=0 (A/B): the basicblock residual backward as its own pass (rpc_sparse_res_backward) instead
// of in the epilogue of the bf16 data-gradient GEMM that produces the block output's gradient (rpc_spconv_gemm_res)
int g_res_fuse = -1;
bool res_fuse() {
  if (g_res_fuse < 0) {
    const char* e = getenv("RPC_SPARSE_RES_FUSE");
    g_res_fuse = (e && atoi(e) == 0) ? 0 : 1;
  }
  return g_res_fuse == 1;
}

int run(const RpcSparseLayer* L, int nl, const void* grad_dense, const int* coors_last, const int* shape, int flags,
        float* dfeat, Arena& A, hipStream_t st, hipStream_t wg, DevEvents* evs) {
#define CHK(x)                 \
  do {                         \
    if (!A.dry) {              \
      int rc__ = (x);          \
      if (rc__) return rc__;   \
    }                          \
  } while (0)
  const RpcSparseLayer& last = L[nl - 1];
  int n = last.n_out, C = last.co;
  float* dy = (float*)A.take(sizeof(float) * (size_t)n * C);
  int nblk = cdiv(n, BM) > 0 ? cdiv(n, BM) : 1;
  float* part = (float*)A.take(sizeof(float) * (size_t)nblk * 2 * C);
  CHK(rpc_dense_to_sparse_grad(grad_dense, last.z, last.bn, coors_last, n, C, shape, flags, dy, part, st));
  // gradient contributions to materialised outputs (block outputs and their identities)
  std::vector<std::vector<const float*>> G(nl);
  const bool split = wg != nullptr && wg != st;
  float* bnb_fused = nullptr;   // bnb of layer li, already finalized by layer li+1's data-gradient launch
  // block outputs whose residual backward (m rows + partial sums) the layer above's data gradient produced
  std::vector<char> res_done(nl, 0);
  std::vector<float*> res_m(nl, nullptr), res_part(nl, nullptr);
  for (int li = nl - 1; li >= 0; --li) {
    const RpcSparseLayer& l = L[li];
    const int n_out = l.n_out;
    if (l.mat) {
      nblk = cdiv(n_out, BM) > 0 ? cdiv(n_out, BM) : 1;
      if (res_done[li]) {
        dy = res_m[li];
        part = res_part[li];
      } else {
        if (G[li].empty()) return RPC_ERR_ARG;
        dy = (float*)A.take(sizeof(float) * (size_t)n_out * l.co);
        part = (float*)A.take(sizeof(float) * (size_t)nblk * 2 * l.co);
        CHK(rpc_sparse_res_backward(G[li][0], G[li].size() > 1 ? G[li][1] : nullptr, l.out, l.z, l.bn, n_out, l.co,
                                    dy, part, st));
      }
      if (l.res >= 0) G[l.res].push_back(dy);
    }
    // BatchNorm backward statistics -> bnb, dgamma, dbeta (unless the data gradient that produced the partial
    // sums already finalized them)
    float* bnb = bnb_fused;
    bnb_fused = nullptr;
    if (!bnb) {
      bnb = (float*)A.take(sizeof(float) * 5 * (size_t)l.co);
      CHK(rpc_bn_finalize(part, nblk, l.co, n_out, 1, l.gamma, l.beta, 0.0f, 0.0f, nullptr, nullptr, l.bn, bnb,
                          l.dgamma, l.dbeta, nullptr, st));
    }
    // weight gradient, on the second stream (it reads only this layer's dz / input rows)
    void* dzb = nullptr;
    if (l.bf16) {
      dzb = A.take(2 * (size_t)n_out * r8(l.co));
      CHK(rpc_bnbwd_to_bf16_rows(dy, l.z, bnb, n_out, l.co, dzb, st));
    }
    hipStream_t sw = split ? wg : st;
    if (split && !A.dry) {
      hipEvent_t e = event_at(evs, (size_t)li);
      if (!e) return RPC_ERR_HIP;
      RPC_CHECK(hipEventRecord(e, st));
      RPC_CHECK(hipStreamWaitEvent(wg, e, 0));
    }
    const size_t wsz = l.bf16 ? rpc_spconv_wgrad_bf16_workspace_size(n_out, l.kvol, l.ci, l.co)
                              : rpc_spconv_wgrad_workspace_size(n_out, l.kvol, l.ci, l.co);
    void* wsw = A.take(wsz);
    if (l.bf16)
      CHK(rpc_spconv_wgrad_h16(l.h_in, l.h_fmt, l.ci, l.nbr, l.kvol, n_out, dzb, l.co, l.dW, wsw, wsz, sw));
    else
      CHK(rpc_spconv_wgrad(l.src, l.src_bn, l.ci, l.nbr, l.kvol, n_out, dy, l.z, bnb, l.co, l.dW, wsw, wsz, sw));
    // data gradient into the layer below (its ReLU mask + BatchNorm-backward partial sums)
    const int* mp = l.kind == 0 ? l.nbr : l.nbr_in;
    const int rev = l.kind == 0 ? 1 : 0;
    const int n_in = l.n_in;
    if (li > 0 && L[li - 1].mat && l.bf16 && res_fuse() && G[li - 1].size() <= 1) {
      // the layer below is a block output: its residual backward in this GEMM's epilogue
      const RpcSparseLayer& prev = L[li - 1];
      const int nb = cdiv(n_in, BM) > 0 ? cdiv(n_in, BM) : 1;
      float* m = (float*)A.take(sizeof(float) * (size_t)n_in * l.ci);
      float* pp = (float*)A.take(sizeof(float) * (size_t)nb * 2 * l.ci);
      RpcBnFin fin;
      const RpcBnFin* fp = nullptr;
      if (l.fin_ticket && n_in > 0) {   // + that layer's BatchNorm-backward finalize (bnb, dgamma, dbeta)
        memset(&fin, 0, sizeof(fin));
        fin.ticket = l.fin_ticket;
        fin.gpart = (double*)A.take(sizeof(double) * 2 * (size_t)rpc_bn_fin_groups(n_in) * l.ci);
        fin.mode = 1;
        fin.gamma = prev.gamma;
        fin.beta = prev.beta;
        fin.fbn = prev.bn;
        fin.bn = bnb_fused = (float*)A.take(sizeof(float) * 5 * (size_t)l.ci);
        fin.dgamma = prev.dgamma;
        fin.dbeta = prev.dbeta;
        fp = &fin;
      }
      CHK(rpc_spconv_gemm_res(dzb, n_out, l.co, mp, l.kvol, rev, n_in, l.btd, l.ci, m,
                              G[li - 1].empty() ? nullptr : G[li - 1][0], prev.out, prev.z, prev.bn, pp, fp, st));
      res_done[li - 1] = 1;
      res_m[li - 1] = m;
      res_part[li - 1] = pp;
    } else if (li > 0 && L[li - 1].mat) {
      float* din = (float*)A.take(sizeof(float) * (size_t)n_in * l.ci);
      if (l.bf16)
        CHK(rpc_spconv_gemm_h16(dzb, 0, n_out, l.co, mp, l.kvol, rev, n_in, l.btd, l.ci, din, nullptr, nullptr,
                                 nullptr, 2, st));
      else
        CHK(rpc_spconv_dgrad(dy, l.z, bnb, l.co, mp, l.kvol, rev, n_in, l.W, l.ci, nullptr, nullptr, din, nullptr, st));
      G[li - 1].push_back(din);
    } else if (li > 0) {
      const RpcSparseLayer& prev = L[li - 1];
      float* din = (float*)A.take(sizeof(float) * (size_t)n_in * l.ci);
      nblk = cdiv(n_in, BM) > 0 ? cdiv(n_in, BM) : 1;
      part = (float*)A.take(sizeof(float) * (size_t)nblk * 2 * l.ci);
      if (l.bf16 && l.fin_ticket && n_in > 0) {
        // + the layer below's BatchNorm-backward finalize (its bnb, dgamma, dbeta) in the same launch
        RpcBnFin fin;
        memset(&fin, 0, sizeof(fin));
        fin.ticket = l.fin_ticket;
        fin.gpart = (double*)A.take(sizeof(double) * 2 * (size_t)rpc_bn_fin_groups(n_in) * l.ci);
        fin.mode = 1;
        fin.gamma = prev.gamma;
        fin.beta = prev.beta;
        fin.fbn = prev.bn;
        fin.bn = bnb_fused = (float*)A.take(sizeof(float) * 5 * (size_t)l.ci);
        fin.dgamma = prev.dgamma;
        fin.dbeta = prev.dbeta;
        CHK(rpc_spconv_gemm_bf16_fin(dzb, n_out, l.co, mp, l.kvol, rev, n_in, l.btd, l.ci, din, prev.z, prev.bn, part,
                                     1, &fin, st));
      } else if (l.bf16)
        CHK(rpc_spconv_gemm_h16(dzb, 0, n_out, l.co, mp, l.kvol, rev, n_in, l.btd, l.ci, din, prev.z, prev.bn,
                                 part, 1, st));
      else
        CHK(rpc_spconv_dgrad(dy, l.z, bnb, l.co, mp, l.kvol, rev, n_in, l.W, l.ci, prev.z, prev.bn, din, part, st));
      dy = din;
    } else if (dfeat) {
      if (l.bf16)
        CHK(rpc_spconv_gemm_h16(dzb, 0, n_out, l.co, mp, l.kvol, rev, n_in, l.btd, l.ci, dfeat, nullptr, nullptr,
                                 nullptr, 2, st));
      else
        CHK(rpc_spconv_dgrad(dy, l.z, bnb, l.co, mp, l.kvol, rev, n_in, l.W, l.ci, nullptr, nullptr, dfeat, nullptr,
                             st));
    }
  }
  if (split && !A.dry) {   // the weight gradients are complete before the main stream goes on
    hipEvent_t e = event_at(evs, (size_t)nl);
    if (!e) return RPC_ERR_HIP;
    RPC_CHECK(hipEventRecord(e, wg));
    RPC_CHECK(hipStreamWaitEvent(st, e, 0));
  }
  return A.ok() ? RPC_OK : RPC_ERR_WORKSPACE;
#undef CHK
}

int check_layers(const RpcSparseLayer* L, int nl) {
  if (!L || nl < 1) return RPC_ERR_ARG;
  for (int i = 0; i < nl; ++i) {
    const RpcSparseLayer& l = L[i];
    if (l.n_in < 0 || l.n_out < 0 || l.ci < 1 || l.co < 1 || l.kvol < 1 || l.res >= i || !l.nbr || !l.z || !l.bn ||
        !l.W || !l.gamma || !l.beta || !l.dW || !l.dgamma || !l.dbeta || (l.kind != 0 && !l.nbr_in) ||
        (l.mat && !l.out) || (l.bf16 && (!l.h_in || !l.btd)) || (!l.bf16 && !l.src))
      return RPC_ERR_ARG;
    if (i > 0 && L[i - 1].n_out != l.n_in) return RPC_ERR_ARG;
  }
  return RPC_OK;
}

}  // namespace

extern "C" size_t rpc_sparse_backward_workspace_size(const RpcSparseLayer* layers, int nlayers) {
  if (check_layers(layers, nlayers)) return 0;
  Arena A{nullptr, 0, 0, true};
  int shape[4] = {1, 1, 1, 1};
  if (run(layers, nlayers, nullptr, nullptr, shape, 0, nullptr, A, nullptr, nullptr, nullptr)) return 0;
  return A.off + 256;
}

extern "C" int rpc_sparse_backward(const RpcSparseLayer* layers, int nlayers, const void* grad_dense,
                                   const int* coors_last, const int* shape, int flags, float* dfeat, void* workspace,
                                   size_t workspace_bytes, void* stream, void* wgrad_stream) {
  int rc = check_layers(layers, nlayers);
  if (rc) return rc;
  if (!grad_dense || !coors_last || !shape || !workspace) return RPC_ERR_ARG;
  Arena A{(char*)workspace, workspace_bytes, 0, false};
  // dry pass first: a workspace that is too small fails before anything is launched
  {
    Arena D{nullptr, 0, 0, true};
    if (run(layers, nlayers, grad_dense, coors_last, shape, flags, dfeat, D, nullptr, nullptr, nullptr))
      return RPC_ERR_ARG;
    if (D.off > workspace_bytes) return RPC_ERR_WORKSPACE;
  }
  int dev = 0;
  RPC_CHECK(hipGetDevice(&dev));
  DevEvents* evs = device_events(dev);
  std::lock_guard<std::mutex> lk(evs->mu);
  return run(layers, nlayers, grad_dense, coors_last, shape, flags, dfeat, A, (hipStream_t)stream,
             (hipStream_t)wgrad_stream, evs);
}

// Side-work streams at the device's least priority (the trainer's batch prefetch, the sparse rulebooks
// and weight gradients): the training stream's kernels are dispatched first when both have work queued.
// which > 0: least priority, which < 0: greatest, 0: default. Returns RPC_OK and the stream in *out.
extern "C" int rpc_stream_create(int which, void** out) {
  if (!out) return RPC_ERR_ARG;
  int least = 0, greatest = 0;
  RPC_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  const int prio = which > 0 ? least : (which < 0 ? greatest : 0);
  hipStream_t s = nullptr;
  RPC_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio));
  *out = (void*)s;
  return RPC_OK;
}

extern "C" int rpc_stream_priority_range(int* least, int* greatest) {
  if (!least || !greatest) return RPC_ERR_ARG;
  RPC_CHECK(hipDeviceGetStreamPriorityRange(least, greatest));
  return RPC_OK;
}

// knob 0: the fused residual backward (1 on, 0 off; the default follows RPC_SPARSE_RES_FUSE). Returns the
// previous value; value < 0 only reads it.
extern "C" int rpc_sparse_tune(int knob, int value) {
  if (knob != 0) return RPC_ERR_ARG;
  const int old = res_fuse() ? 1 : 0;
  if (value >= 0) g_res_fuse = value ? 1 : 0;
  return old;
}
