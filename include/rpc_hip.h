/*
 * rpc_hip.h — C ABI of librpc_hip.so, the gfx950 (MI355X) kernels of the
 * adversarial voxel-detector training step (SURVEY.md §8(a) rows a1–a6).
 *
 * Conventions (SURVEY.md §8(b) "C-ABI"):
 *   - every buffer is device memory owned by the caller (PyTorch caching allocator);
 *     the library never allocates: scratch comes in through `workspace`;
 *   - `stream` is a hipStream_t passed as void* (the launcher's current stream);
 *   - return value 0 = success, otherwise an RPC_ERR_* code (the Python side raises);
 *     nothing in the library aborts or synchronises the device;
 *
 * Each entry point names the reference interface it replaces (file:line in
 * /root/reference, or the un-vendored upstream call site that file reaches).
 */
#ifndef RPC_HIP_H
#define RPC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  RPC_OK = 0,
  RPC_ERR_ARG = 1,        /* bad sizes / null pointers */
  RPC_ERR_WORKSPACE = 2,  /* workspace too small */
  RPC_ERR_UNSUPPORTED = 3,/* width combination without a compiled kernel */
  RPC_ERR_HIP = 4         /* a HIP runtime call failed */
};

/* Library identity: returns a static string "rpc_hip <git-describe> gfx950". */
const char* rpc_version(void);

/* ------------------------------------------------------------------ a1 voxelize
 * Replaces mmcv.ops `hard_voxelize_forward` (upstream mmcv/ops/csrc/pytorch/cuda/
 * voxelization_cuda.cu, deterministic path) as called per frame by upstream
 * mmdet3d `Det3DDataPreprocessor.voxelize` for the voxel_layer of
 * configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-car.py:48-53,
 * batched over B frames and followed by the `F.pad(coors,(1,0),value=i)` + `torch.cat`
 * of that preprocessor.
 *
 * points         [total_points, num_features] float32, frames concatenated
 * frame_offsets  device int32 [batch+1]: frame b owns rows [off[b], off[b+1])
 * voxels         [batch*max_voxels, max_points, num_features] — rows >= total V are untouched
 * coors          [batch*max_voxels, 4] int32 (b, z, y, x)
 * num_points     [batch*max_voxels] int32
 * voxel_num      device int32 [batch+1]: per-frame voxel counts, then the total V
 * Semantics (bit-exact with the mmcv CPU/CUDA kernels): c = floor((p-min)/vs) per axis in
 * float32, point rejected if c<0 || c>=round((max-min)/vs); voxel ids in order of the
 * first point that lands in them; new voxels beyond max_voxels dropped; at most
 * max_points points per voxel, kept in point order; unused slots zero.
 */
size_t rpc_hard_voxelize_workspace_size(int total_points, int batch);
int rpc_hard_voxelize(const float* points, int num_features, int total_points,
                      const int* frame_offsets, int batch,
                      const float* voxel_size /* host [3] */, const float* coors_range /* host [6] */,
                      int max_points, int max_voxels,
                      float* voxels, int* coors, int* num_points, int* voxel_num,
                      void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ a5 HardSimpleVFE
 * Replaces upstream mmdet3d `HardSimpleVFE.forward` (voxel_encoders/voxel_encoder.py),
 * used at models/detectors/adversarial_voxelnet.py:135-137:
 *   out[v, f] = (sum_s voxels[v, s, f]) / num_points[v],  f < vfe_features
 * backward: dvoxels[v, s, f] = dout[v, f] / num_points[v] for every slot s.
 */
int rpc_vfe_mean_forward(const float* voxels, const int* num_points, int num_voxels,
                         int max_points, int num_features, int vfe_features,
                         float* out, void* stream);
int rpc_vfe_mean_backward(const float* dout, const int* num_points, int num_voxels,
                          int max_points, int num_features, int vfe_features,
                          float* dvoxels, void* stream);

/* ------------------------------------------------------------------ ★ HardVFE (PointNet MLP + max)
 * Replaces upstream mmdet3d `HardVFE.forward` + `VFELayer.forward`
 * (mmdet3d/models/voxel_encoders/voxel_encoder.py; not vendored: /root/reference/mmdetection3d is
 * empty), the "VFE per-voxel PointNet MLP+max" of BASELINE.json's north_star, called where
 * models/detectors/adversarial_voxelnet.py:135-137 and adversarial_centerpoint.py:100 call the voxel
 * encoder. Per voxel [T, F] slots: decoration (raw features, xyz - point mean, xyz - voxel centre,
 * |xyz|) masked to the first num_points slots, then per layer Linear(no bias) -> BatchNorm1d over
 * all V*T rows -> ReLU -> max over the T slots, [pointwise, max] concatenated into the next layer.
 * params: 5 pointers per layer (W [C][K] torch layout, gamma, beta, running_mean, running_var);
 * grads: 3 per layer (dW, dgamma, dbeta). The workspace carries the forward state to the backward
 * (keep it alive and unmodified in between). F <= 9 (decorated width <= 16), T <= 64, channels <= 128,
 * 1-4 layers; backward in training mode only. */
typedef struct {
  int F;                 /* raw features per point slot */
  int T;                 /* slots per voxel (max_num_points) */
  int nlayers;           /* 1..4 */
  int channels[4];       /* feat_channels */
  int with_cluster_center, with_voxel_center, with_distance;
  int training;
  float voxel_size[3];
  float pc_range_min[3];
  float bn_eps, bn_momentum;
} RpcHardVfeCfg;
size_t rpc_hard_vfe_workspace_size(const RpcHardVfeCfg* cfg, int num_voxels);
int rpc_hard_vfe_forward(const RpcHardVfeCfg* cfg, float* const* params, const float* features,
                         const int* num_points, const int* coors, int num_voxels, float* out /* [V][C_last] */,
                         void* workspace, size_t workspace_bytes, void* stream);
int rpc_hard_vfe_backward(const RpcHardVfeCfg* cfg, float* const* params, const float* features,
                          const int* num_points, const int* coors, int num_voxels, const float* dout,
                          float* dfeatures /* [V][T][F] */, float* const* grads, void* workspace,
                          size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ a2/a3/a4 VoxelPerturber
 * Replaces `VoxelPerturber.forward` + `_apply_physical_constraints`
 * (models/adversarial/voxel_perturber.py:120-321, 323-386), the compaction /
 * masked scatter of `AdversarialVoxelNet.extract_feat`
 * (models/detectors/adversarial_voxelnet.py:85-117) and, in fused mode, the
 * HardSimpleVFE that follows it (:135-137). The per-parameter grad hook
 * `clamp(nan_to_num(g), -0.1, 0.1)` (voxel_perturber.py:465-475) is applied to the
 * parameter gradients written by rpc_perturber_backward.
 *
 * params / grads: host arrays of RPC_PERTURBER_NPARAMS device pointers, order:
 *   for l in 0..4: W_l [C_{l+1}, C_l], b_l, gamma_l, beta_l, running_mean_l, running_var_l
 *   W_5 [F, h0], b_5, Wa0 [A, F], ba0 [A], Wa1 [1, A], ba1 [1]
 * with widths C = (F, h0, h1, h2, h1, h0, F) and A = max(F/2, 1) — the
 * nn.Sequential layout of voxel_perturber.py:82-112. grads[] entries for running
 * stats are ignored (may be NULL).
 *
 * Modes:
 *   standalone: num_points == NULL, x = [rows, F] (every row perturbed), out = [rows, F]
 *   fused:      num_points != NULL, x = voxels [rows, slots, F]; a slot is perturbed
 *               iff its F features sum to non-zero (adversarial_voxelnet.py:89);
 *               out = perturbed voxels; vfe_out = [rows, vfe_features] mean of out.
 * losses: device float[8] = l2_norm, intensity_loss, bias_loss, imbalance_loss,
 *   n_valid, nan_fallback flag, reserved x2 (voxel_perturber.py:268-299, 312-317).
 * Train mode updates running_mean/var in place (momentum, unbiased var) like BatchNorm1d.
 */
#define RPC_PERTURBER_NPARAMS 36

typedef struct {
  int F;                  /* point features (4 KITTI, 5 NuScenes) */
  int hidden[3];          /* hidden_channels, each 8, 16, 32, 64, 128 or 256 (the plugin zero-pads others;
                             256-wide layers run on the per-point VALU kernels); else RPC_ERR_UNSUPPORTED */
  int use_attention;      /* use_spatial_attention */
  int training;           /* 1 = batch-stat BN + train bounds, 0 = running stats + eval bounds */
  float sensor_error_bound;
  float bn_eps;           /* 1e-3 (voxel_perturber.py:462) */
  float bn_momentum;      /* 0.1  (voxel_perturber.py:461) */
  int vfe_features;       /* fused mode: HardSimpleVFE num_features (4 KITTI) */
  int wgrad_split_bf16;   /* perf mode: hidden-layer weight gradients on bf16 MFMA with hi/lo-split fp32
                             operands (~2^-16 relative per product); 0 = fp32 MFMA (parity mode) */
  int act16;              /* perf mode: 16-bit activation rows of the hidden layers in the workspace — bit 0:
                             pre-activations z_1..z_3 fp16 (the reference AMP's Linear outputs, train.py:91-103);
                             bit 1 (with wgrad_split_bf16): gradient rows dh_1..dh_3, dz_1..dz_4 bf16. Applied
                             when every hidden shape is an encoder-decoder step (width x2 or /2, >= 16), else
                             fp32 rows; fp32 arithmetic and fp32/double BatchNorm sums either way. 0 = parity */
} rpc_perturber_cfg;

size_t rpc_perturber_workspace_size(const rpc_perturber_cfg* cfg, int rows, int slots);
int rpc_perturber_forward(const rpc_perturber_cfg* cfg, const float* const* params,
                          const float* x, int rows, int slots, const int* num_points,
                          float* out, float* vfe_out, float* losses,
                          void* workspace, size_t workspace_bytes, void* stream);
/* dout: standalone [rows, F] = dL/dout; fused [rows, vfe_features] = dL/dvfe_out.
 * dlosses: device float[4] = dL/d(l2_norm, intensity_loss, bias_loss, imbalance_loss).
 * The workspace must be the one the matching forward filled. */
int rpc_perturber_backward(const rpc_perturber_cfg* cfg, const float* const* params,
                           const float* x, int rows, int slots, const int* num_points,
                           const float* dout, const float* dlosses, float* const* grads,
                           void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------ a6 SparseEncoder
 * Replaces the spconv (spconv-cu113>=2.3.0, requirements.txt:18) SubMConv3d /
 * SparseConv3d + BatchNorm1d + ReLU modules that upstream mmdet3d `SparseEncoder`
 * (config: adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:19-23) runs at
 * models/detectors/adversarial_voxelnet.py:141, and its `.dense()` BEV output.
 * Features are row-major [N, C] float32; coors [N, 4] int32 (b, z, y, x); weights
 * W[k][CI][CO] with k = (kz * kh + ky) * kw + kx. Rulebook builders need a dense int32
 * index grid [B, D, H, W] that is all -1 on entry and is left all -1 on exit.
 */
/* SubM neighbour map: nbr[r, k] = row at coors[r] + (k - centre), or -1. */
int rpc_subm_rulebook(const int* coors, int n, const int* shape /* host B,D,H,W */,
                      const int* ksize /* host [3] */, int* grid, int* nbr, void* stream);
/* Strided SparseConv3d rulebook, two phases around one host read of n_out. */
size_t rpc_spconv_rulebook_workspace_size(int n_in, int kvol);
int rpc_spconv_rulebook_count(const int* coors, int n_in, const int* out_shape, const int* ksize,
                              const int* stride, const int* pad, int* grid_out, int* n_out /* device */,
                              void* workspace, size_t workspace_bytes, void* stream);
int rpc_spconv_rulebook_build(const int* coors, int n_in, const int* out_shape, const int* ksize,
                              const int* stride, const int* pad, int* grid_out, int n_out,
                              int* coors_out, int* nbr_out /* [n_out, K] */, int* nbr_in /* [n_in, K] */,
                              void* workspace, void* stream);
/* number of 64-row tiles (= BatchNorm partial rows) of a conv over n_out output rows */
int rpc_spconv_gemm_blocks(int n_out);
/* z_out[r] = sum_k A(in[nbr[r,k]]) W[k], A = relu(in*scale+shift) if in_bn else identity;
 * part (nullable) = per-tile BatchNorm partial sums [blocks][2*CO]. */
int rpc_spconv_forward(const float* in, const float* in_bn, int ci, const int* nbr, int kvol, int n_out,
                       const float* W, int co, float* z_out, float* part, void* stream);
/* din[i] = sum_k dz(map[i,k']) W[k]^T with dz = bnb-normalised (dy_out, z_out), k' = rev ? K-1-k : k.
 * With prev_z/prev_bn the previous layer's ReLU mask is applied and its BatchNorm-backward
 * partial sums are written to part. */
int rpc_spconv_dgrad(const float* dy_out, const float* z_out, const float* bnb, int co, const int* map,
                     int kvol, int rev, int n_in, const float* W, int ci, const float* prev_z,
                     const float* prev_bn, float* din, float* part, void* stream);
size_t rpc_spconv_wgrad_workspace_size(int n_out, int kvol, int ci, int co);
int rpc_spconv_wgrad(const float* in, const float* in_bn, int ci, const int* nbr, int kvol, int n_out,
                     const float* dy_out, const float* z_out, const float* bnb, int co, float* dW,
                     void* workspace, size_t workspace_bytes, void* stream);
/* BatchNorm1d finalize from partial sums. mode 0: bn_out = scale, shift, mean, invstd and the
 * running stats update (train). mode 1: bn_out = gi, m1, m2, mean, invstd for the backward and
 * dgamma = sum dy*xhat, dbeta = sum dy. mode | RPC_BN_PART_F64: part holds double rows (the fp32
 * parity engine's rpc_dense_bnbwd_stats_f32), else float rows. One block per channel, no cross-block
 * step: the workspace is unused (size 0; may be NULL) and kept for signature stability. */
#define RPC_BN_PART_F64 4
size_t rpc_bn_finalize_workspace_size(int c);
int rpc_bn_finalize(const void* part, int nblk, int c, int n, int mode, const float* gamma,
                    const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                    const float* fwd_bn, float* bn_out, float* dgamma, float* dbeta, void* workspace,
                    void* stream);
/* SparseBasicBlock residual (upstream mmdet3d SparseBasicBlock.forward, the block_type='basicblock'
 * SparseEncoder of the CenterPoint nuScenes base, adversarial-centerpoint_voxel-nuscenes.py:11-13):
 * forward out = relu(bn(z) + res) (res may be NULL: a materialised relu(bn(z))), fp32 rows [n][c]
 * and optionally bf16 rows [n][round8(c)]; backward m = (g1 + g2) * (out > 0) (g2 may be NULL) with
 * the BatchNorm-backward partial sums (sum m, sum m*xhat) of z per rpc_spconv_gemm_blocks(n) rows,
 * for rpc_bn_finalize mode 1. c <= 256. */
int rpc_sparse_res_forward(const float* z, const float* bn, const float* res, int n, int c, float* out,
                           void* out_bf16, void* stream);
/* the same with the 16-bit rows in format fmt (RPC_H16_BF16 / RPC_H16_F16), and with fmt RPC_H16_F16 optionally a
 * bf16 copy (out_bf16) */
int rpc_sparse_res_forward_h16(const float* z, const float* bn, const float* res, int n, int c, float* out,
                               void* out_h16, int fmt, void* out_bf16, void* stream);
int rpc_sparse_res_backward(const float* g1, const float* g2, const float* out, const float* z, const float* bn,
                            int n, int c, float* m, float* part, void* stream);
/* SparseConvTensor.dense() of relu(bn(z)) viewed as [B, C*D, H, W] (channel c*D + z); backward
 * gathers, applies the ReLU mask and writes the BatchNorm-backward partial sums.
 * flags: RPC_DENSE_NHWC = channels_last image [B][H][W][C*D]; RPC_DENSE_BF16 = bf16 elements
 * (the caller zero-fills the dense buffer; only occupied cells are written). */
#define RPC_DENSE_NHWC 1
#define RPC_DENSE_BF16 2
int rpc_sparse_to_dense(const float* z, const float* bn, const int* coors, int n, int c,
                        const int* shape /* B,D,H,W */, int flags, void* dense, void* stream);
/* the cells rpc_sparse_to_dense writes for coors (c % 4 == 0) set back to 0: a persistent dense buffer
 * is cleared where the previous step scattered instead of zero-filled whole (same flags). */
int rpc_sparse_dense_clear(const int* coors, int n, int c, const int* shape /* B,D,H,W */, int flags, void* dense,
                           void* stream);
int rpc_dense_to_sparse_grad(const void* grad_dense, const float* z, const float* bn, const int* coors,
                             int n, int c, const int* shape, int flags, float* dy, float* part, void* stream);

/* ---- a6 perf mode (16-bit MFMA operands, fp32 accumulate and BatchNorm statistics). Forward GEMM operands
 * (the gathered rows relu(bn(z)) and the forward weight tiles) may be fp16 (RPC_H16_F16: 3 more mantissa bits
 * than bf16 at the same MFMA rate; the perf mode's default — see SparseEncoder.h16_fwd); the backward's dz rows
 * and data-gradient tiles are bf16. */
#define RPC_H16_BF16 0
#define RPC_H16_F16 1
/* h[r, c] = bf16(relu?(z*scale+shift)) (bn NULL: identity), rows padded to round8(c) */
int rpc_to_bf16_rows(const float* z, const float* bn, int n, int c, int relu, void* h, void* stream);
/* the same rows in format fmt; with fmt RPC_H16_F16, h_bf16 (optional) receives the same rows in bf16 too (the
 * weight gradient's operand) */
int rpc_to_h16_rows(const float* z, const float* bn, int n, int c, int relu, int fmt, void* h, void* h_bf16,
                    void* stream);
/* dz[r, c] = bf16(gi*(dy - m1 - xhat*m2)) with bnb = gi, m1, m2, mean, invstd (rpc_bn_finalize mode 1) */
int rpc_bnbwd_to_bf16_rows(const float* dy, const float* z, const float* bnb, int n, int c, void* dz, void* stream);
/* W [K][ci][co] fp32 -> per-offset B^T tiles bf16 (forward: [K][co][ci]; dgrad: [K][ci][co]), zero padded */
size_t rpc_spconv_bf16_weight_elems(int kvol, int ci, int co, int dgrad);
int rpc_spconv_prep_weight_bf16(const float* W, int kvol, int ci, int co, int dgrad, void* bt, void* stream);
/* up to 32 rpc_spconv_prep_weight_bf16 calls (forward and data-gradient tiles of every layer) in one launch */
typedef struct {
  const float* W;
  void* bt;
  int kvol, ci, co, dgrad;
  int fmt;               /* tile format: RPC_H16_BF16, or RPC_H16_F16 (forward tiles, dgrad 0) */
} RpcSpconvWprep;
int rpc_spconv_prep_weight_bf16_batch(const RpcSpconvWprep* descs, int n, void* stream);
/* out[r] = sum_k a[map[r, k']] . B_k ; epi 0 forward (+BN partial sums), 1 dgrad (prev ReLU mask +
 * BN-backward partial sums), 2 plain. The source rows a and the tiles bt are read through 32-bit
 * buffer offsets: both must stay below 2 GiB (RPC_ERR_UNSUPPORTED when n_out rows of a already
 * exceed it). */
int rpc_spconv_gemm_bf16(const void* a, int kg, const int* map, int kvol, int rev, int n_out, const void* bt,
                         int ng, float* out, const float* prev_z, const float* prev_bn, float* part, int epi,
                         void* stream);
/* the same with the gathered source table's row count n_src (rows of `a`), which bounds the kernel's 32-bit
 * source offsets: RPC_ERR_UNSUPPORTED when n_src * round8(kg) * 2 >= 2^31. rpc_spconv_gemm_bf16 = n_src -1
 * (bounded by n_out rows, exact for submanifold layers only). */
int rpc_spconv_gemm_bf16_n(const void* a, int n_src, int kg, const int* map, int kvol, int rev, int n_out,
                           const void* bt, int ng, float* out, const float* prev_z, const float* prev_bn,
                           float* part, int epi, void* stream);
/* the same with the operand format of a and bt: RPC_H16_BF16, or RPC_H16_F16 for the forward (epi 0) only
 * (RPC_ERR_UNSUPPORTED otherwise) */
int rpc_spconv_gemm_h16(const void* a, int fmt, int n_src, int kg, const int* map, int kvol, int rev, int n_out,
                        const void* bt, int ng, float* out, const float* prev_z, const float* prev_bn, float* part,
                        int epi, void* stream);
/* the same GEMM with the BatchNorm finalize of its partial sums fused in (the last
 * arriving blocks sum the partial rows in two fixed-order levels and apply rpc_bn_finalize's arithmetic),
 * replacing the rpc_bn_finalize launch that followed it: epi 0 -> mode 0 (this layer's bn + running stats),
 * epi 1 -> mode 1 (bnb, dgamma, dbeta of the layer whose ReLU mask the epilogue applies; fbn = its
 * forward bn). `part` is still written (the fused sums read it). fin NULL = rpc_spconv_gemm_bf16_n.
 * fin->ticket: rpc_bn_fin_tickets(n_out) counters, zero before first use (every launch leaves them zero);
 * fin->gpart: rpc_bn_fin_groups(n_out) * 2 * ng doubles. ng <= 256. */
typedef struct {
  unsigned* ticket;
  double* gpart;
  int mode;
  const float* gamma;
  const float* beta;
  float eps, momentum;
  float* running_mean;
  float* running_var;
  const float* fbn;
  float* bn;
  float* dgamma;
  float* dbeta;
} RpcBnFin;
int rpc_bn_fin_groups(int n_out);
int rpc_bn_fin_tickets(int n_out);
/* data gradient (epi 1) only (r05: the forward's fused finalize measured slower and was removed) */
int rpc_spconv_gemm_bf16_fin(const void* a, int n_src, int kg, const int* map, int kvol, int rev, int n_out,
                             const void* bt, int ng, float* out, const float* prev_z, const float* prev_bn,
                             float* part, int epi, const RpcBnFin* fin, void* stream);
/* the data gradient into a basicblock's output rows with rpc_sparse_res_backward in its epilogue (r04):
 * m = (dgrad + g2) * [out > 0] -> m [n_out][ng] fp32 (g2: the identity path's contribution or NULL; out: the
 * block output rows), and that layer's BatchNorm-backward partial rows (sum m, sum m * (z - mean) * invstd;
 * bn = scale, beta, mean, invstd) -> part [rpc_spconv_gemm_blocks(n_out)][2 * ng];
 * fin (mode 1, or NULL): that layer's BatchNorm-backward finalize in the last-arriving blocks. */
/* knob 0: rpc_sparse_backward's fused residual backward (1 on, 0 off); returns the previous value */
int rpc_sparse_tune(int knob, int value);
int rpc_spconv_gemm_res(const void* a, int n_src, int kg, const int* map, int kvol, int rev, int n_out, const void* bt,
                        int ng, float* m, const float* g2, const float* out, const float* z, const float* bn,
                        float* part, const RpcBnFin* fin, void* stream);
/* dW[k] = sum_r h[nbr[r,k]]^T dz[r] (bf16 rows, fp32 accumulate, fixed-order reduction) */
size_t rpc_spconv_wgrad_bf16_workspace_size(int n_out, int kvol, int ci, int co);
int rpc_spconv_wgrad_bf16(const void* h, int ci, const int* nbr, int kvol, int n_out, const void* dz, int co,
                          float* dW, void* workspace, size_t workspace_bytes, void* stream);
/* the same with h in format hfmt (fp16 forward rows are rounded to bf16 as they are staged) */
int rpc_spconv_wgrad_h16(const void* h, int hfmt, int ci, const int* nbr, int kvol, int n_out, const void* dz,
                         int co, float* dW, void* workspace, size_t workspace_bytes, void* stream);

/* ---- a6 runtime: the whole SparseEncoder backward in one call (csrc/sparse_exec.hip).
 * Replaces the per-layer backward of upstream mmdet3d SparseEncoder (adversarial_voxelnet.py:141;
 * configs/adversarial/…-3class.py:19-23) over spconv: one entry per sparse conv in forward order, with
 * the forward's saved tensors; the weight / BatchNorm-affine gradients are written to dW / dgamma / dbeta.
 * The launches are those of the per-layer entry points above, in the same order; weight gradients go to
 * wgrad_stream (NULL or == stream: the main stream) behind one event per layer and are joined back into
 * `stream` before the call returns. Temporaries come from `workspace` (no allocation). */
typedef struct {
  int kind;              /* 0 = submanifold (SubMConv3d), 1 = strided (SparseConv3d) */
  int ci, co, kvol;
  int n_in, n_out;
  int bf16;              /* bf16 MFMA path (perf mode, layers >= 1); 0 = fp32 */
  int mat;               /* output materialised as rows (basicblock output / identity) */
  int res;               /* layer whose output is this block's identity, or -1 */
  const int* nbr;        /* [n_out][kvol] */
  const int* nbr_in;     /* strided: [n_in][kvol] */
  const float* z;        /* [n_out][co] pre-BatchNorm output */
  const float* bn;       /* [4*co] forward scale, beta, mean, invstd */
  const float* out;      /* mat: [n_out][co] */
  const void* h_in;      /* bf16 layers: bf16 input rows [n_in][round8(ci)] */
  const float* src;      /* fp32 layers: input rows [n_in][ci] */
  const float* src_bn;   /* fp32 layers: BatchNorm params of src (folded into its gather) or NULL */
  const float* W;        /* [kvol][ci][co] */
  const float* gamma;
  const float* beta;
  const void* btd;       /* bf16 layers: data-gradient weight tiles (rpc_spconv_prep_weight_bf16, dgrad 1) */
  float* dW;
  float* dgamma;
  float* dbeta;
  int h_fmt;             /* bf16 layers: format of h_in (RPC_H16_BF16 / RPC_H16_F16) */
  unsigned* fin_ticket;  /* bf16 layers: rpc_bn_fin_tickets(n_in) zeroed counters — the data gradient into the
                            layer below then finalizes that layer's BatchNorm backward in its own launch
                            (rpc_spconv_gemm_bf16_fin); NULL: a separate rpc_bn_finalize */
} RpcSparseLayer;
/* Side-work stream (no reference counterpart: the reference runs one stream). which > 0: the device's
 * least stream priority, < 0: greatest, 0: default; hipStreamNonBlocking. */
int rpc_stream_create(int which, void** out);
int rpc_stream_priority_range(int* least, int* greatest);

size_t rpc_sparse_backward_workspace_size(const RpcSparseLayer* layers, int nlayers);
int rpc_sparse_backward(const RpcSparseLayer* layers, int nlayers, const void* grad_dense, const int* coors_last,
                        const int* shape /* B,D,H,W */, int flags, float* dfeat /* [n_in of layer 0][ci] or NULL */,
                        void* workspace, size_t workspace_bytes, void* stream, void* wgrad_stream);


/* ---- a7 perf mode: dense BEV backbone / neck (SECOND + SECONDFPN) on bf16 MFMA, NHWC images.
 * Replaces the Conv2d/ConvTranspose2d + BatchNorm2d + ReLU stacks of upstream mmdet3d
 * backbones/second.py and necks/second_fpn.py (called at models/detectors/adversarial_voxelnet.py:142-145,
 * configured at configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-car.py / -3class.py:25-36).
 * Images are given as {B, H, W}; rows are pixels ((b*H + y)*W + x), pitch in elements. */
#define RPC_DMAP_S1 0 /* 3x3 stride 1 pad 1 (and its data gradient with flipped taps) */
#define RPC_DMAP_S2 1 /* 3x3 stride 2 pad 1 */
#define RPC_DMAP_D2 2 /* data gradient of S2 */
#define RPC_DMAP_P1 3 /* 1x1 (ConvTranspose2d k1 s1) */
#define RPC_DMAP_U2 4 /* ConvTranspose2d k2 s2 (4 parities) */
#define RPC_DMAP_G2 5 /* data gradient of U2 */
/* out[orow][ooff + n] (+)= sum_{t,k} src[src_row(row,t)][k] * wt[t][n][k]; cin % 64 == 0, cout % 128 == 0;
 * part (optional): [rpc_dense_conv_part_rows][2*cout] BatchNorm partial sums of the stored bf16 values */
int rpc_dense_conv(int map, const void* src, int src_pitch, int cin, const void* wt, int cout, void* out,
                   int out_pitch, int out_offset, int accumulate, float* part, const int* row_img,
                   const int* src_img, const int* out_img, void* stream);
int rpc_dense_conv_blocks(int map, const int* row_img);
/* exact number of BatchNorm partial-sum rows rpc_dense_conv writes for (map, cout, row_img): one per
 * 16x32-pixel tile for the S1 kernel k_conv3x3x, else rpc_dense_conv_blocks (the rows rpc_bn_finalize
 * reduces; never more than rpc_dense_conv_blocks) */
int rpc_dense_conv_part_rows(int map, int cout, const int* row_img);
/* RPC_DMAP_S1 data gradient (no accumulate, channel offset 0) whose output out = dh is the gradient of a
 * BatchNorm2d + ReLU layer with pre-activation image bnz [B*H*W][cout] and forward parameters bnp[4*cout]
 * (scale, beta, mean, invstd): also writes that layer's BatchNorm-backward partial sums (sum dm, sum dm*xhat;
 * dm = dh * [pre > 0]) to part [rpc_dense_conv_part_rows][2*cout] (rpc_bn_finalize mode 1 reduces them).
 * Replaces rpc_dense_bnbwd_stats for that layer; RPC_ERR_UNSUPPORTED when the shape takes an S1 kernel
 * without it (cout not a multiple of 128, images >= 2 GB) */
int rpc_dense_conv_bnbwd(const void* src, int src_pitch, int cin, const void* wt, int cout, void* out,
                         int out_pitch, const void* bnz, const float* bnp, float* part, const int* row_img,
                         void* stream);
/* which kernel rpc_dense_conv launches for an RPC_DMAP_S1 call with `cout` outputs over row_img:
 * 0 = rpc::dn::k_conv3x3<0> (64-channel blocks), 1 = rpc::dn::k_conv3x3w<0> (128-channel LDS-DMA
 * blocks), 2 = rpc::dn::k_conv3x3x<0> (16x32-pixel x 128-channel LDS-DMA blocks), -1 = not an S1 call (per-kernel roofline attribution in bench.py) */
int rpc_dense_conv_s1_kernel(int map, int cout, const int* row_img);
/* kernel-selection knob for A/B measurement (returns the previous value; value < 0 only reads it):
 * knob 0 = the S1 kernel for output channels that are a multiple of 128 (0: chosen by shape, default;
 * 1: the 64-channel register-staged kernel; 2: the 128-channel LDS-DMA kernel; 3: the 16x32-pixel
 * tile kernel; 4: the 16x16-pixel two-blocks-per-CU kernel); knob 1 = the S1 weight gradient for
 * 128-multiple channels (0: tap-sharing row-segment kernel with the next sub-step's operand reads issued
 * before this one's MFMAs, default; 1: per-tap kernel; 2: the row-segment kernel's former read-then-MFMA
 * loop); knob 4 = k_conv3x3x / k_conv3x3y loop variants and timing arms (128: x with operand reads a
 * quarter step ahead / y's former read-then-MFMA loop; bit-identical to the defaults); knob 5 = the
 * 64-channel-multiple k_conv3x3's output channels per block (0: 32 when the 64-channel grid is under one
 * round of two blocks per CU, default; 1: always 64; 2: always 32; bit-identical results); knob 8 = the
 * 16x16-pixel kernel's split tail (1: the items past the last whole round of one block per CU run as two
 * 64-channel blocks each when they fit one round, default; 0: off; bit-identical results); knob 9 = the row
 * mapping of rpc_dense_bn_apply / rpc_dense_bnbwd_apply (0: one contiguous chunk of rows per block, default;
 * 1: grid-stride batches; bit-identical results); knob 10 = the 16x16-pixel kernel's pre-activation prefetch for
 * rpc_dense_conv_bnbwd (1: the epilogue's first rows loaded during the last K-chunk, default; 0: all in the
 * epilogue; bit-identical results) */
int rpc_dense_tune(int knob, int value);
/* dW (torch layout; kind 0 = Conv2d [co][ci][kh][kw], 1 = ConvTranspose2d [ci][co][kh][kw]) of the
 * forward map (S1/S2/P1/U2): sum over rows of x[src_row(row,t)][ci] * dz[row][co]; ci, co % 128 == 0 */
size_t rpc_dense_wgrad_workspace_size(int map, const int* row_img, int ci, int co);
int rpc_dense_wgrad(int map, int kind, const void* x, int x_pitch, int ci, const void* dz, int dz_pitch, int co,
                    const int* row_img, const int* src_img, const int* out_img, float* dW, void* workspace,
                    size_t workspace_bytes, void* stream);
/* h = relu((z - mean) * scale + beta) -> out[row][offset + c] (bn = scale, beta, mean, invstd) */
int rpc_dense_bn_apply(const void* z, int m, int c, const float* bn, void* out, int out_pitch, int out_offset,
                       void* stream);
/* BatchNorm2d + ReLU backward: partial sums (sum dm, sum dm*xhat) per block, then
 * dz = gi * (dm - m1 - xhat * m2) with bnb from rpc_bn_finalize(mode 1) */
int rpc_dense_bnbwd_blocks(int m);
int rpc_dense_bnbwd_stats(const void* dh, int dh_pitch, int dh_offset, const void* z, int m, int c,
                          const float* bn, float* part, void* stream);
int rpc_dense_bnbwd_apply(const void* dh, int dh_pitch, int dh_offset, const void* z, int m, int c,
                          const float* bn, const float* bnb, void* dz, void* stream);
/* torch fp32 weights -> bf16 GEMM operands: fwd [taps][co][ci] and/or dgrad [taps][ci][co] (flip: taps reversed) */
int rpc_dense_wprep(const float* W, int kind, int ci, int co, int taps, int flip, void* w_fwd, void* w_dgrad,
                    void* stream);
/* up to 16 rpc_dense_wprep calls (every layer of a module) in one launch */
typedef struct {
  const float* W;
  void* w_fwd;
  void* w_dgrad;
  int kind, ci, co, taps, flip;
  int co_src;   /* kind 0: rows of W present (co_src <= co; rows co_src .. co-1 are written as zero, the
                   outputs of a conv padded to co channels); 0 = co */
} RpcDenseWprep;
int rpc_dense_wprep_batch(const RpcDenseWprep* descs, int n, void* stream);

/* ---- a7 parity mode: the same dense engine with fp32 operands on fp32 MFMA (v_mfma_f32_16x16x4_f32),
 * fp32 NHWC images; replaces the same upstream Conv2d / ConvTranspose2d + BatchNorm2d + ReLU stacks
 * (mmdet3d backbones/second.py, necks/second_fpn.py; …-3class.py:25-36) and the Anchor3DHead 1x1 convs
 * (dense_heads/anchor3d_head.py, …-3class.py:38-45) in fp32, for the 1e-4 detection-loss parity of
 * north_star. cin % 16 == 0, cout % 64 == 0 (conv); ci, co % 64 == 0 (wgrad); weights from
 * rpc_dense_wprep_batch_f32 (fp32 [taps][co][ci] / [taps][ci][co]). */
int rpc_dense_conv_f32(int map, const float* src, int src_pitch, int cin, const float* wt, int cout, float* out,
                       int out_pitch, int out_offset, int accumulate, float* part, const int* row_img,
                       const int* src_img, const int* out_img, void* stream);
int rpc_dense_conv_blocks_f32(int map, const int* row_img);
size_t rpc_dense_wgrad_workspace_size_f32(int map, const int* row_img, int ci, int co);
int rpc_dense_wgrad_f32(int map, int kind, const float* x, int x_pitch, int ci, const float* dz, int dz_pitch, int co,
                        const int* row_img, const int* src_img, const int* out_img, float* dW, void* workspace,
                        size_t workspace_bytes, void* stream);
int rpc_dense_bn_apply_f32(const float* z, int m, int c, const float* bn, float* out, int out_pitch, int out_offset,
                           void* stream);
int rpc_dense_bnbwd_stats_f32(const float* dh, int dh_pitch, int dh_offset, const float* z, int m, int c,
                              const float* bn, double* part, void* stream);
int rpc_dense_bnbwd_apply_f32(const float* dh, int dh_pitch, int dh_offset, const float* z, int m, int c,
                              const float* bn, const float* bnb, float* dz, void* stream);
int rpc_dense_wprep_batch_f32(const RpcDenseWprep* descs, int n, void* stream);


/* ------------------------------------------------------------------ a8 / §8(f1) Anchor3DHead targets + losses
 * Replaces upstream mmdet3d `Anchor3DHead.loss_by_feat` (dense_heads/anchor3d_head.py) with
 * `AnchorTrainMixin.anchor_target_3d` (Max3DIoUAssigner over BboxOverlapsNearest3D, no sampler),
 * mmcv `sigmoid_focal_loss`, mmdet `SmoothL1Loss` (+ add_sin_difference), `get_direction_target`
 * + `CrossEntropyLoss`, as configured at
 * configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:38-69,86-112 and
 * …-kitti-3d-car.py:18-39; called at models/detectors/adversarial_voxelnet.py:168 (`bbox_head.loss`).
 *
 * Head outputs z (the 1x1 conv WITHOUT bias; `bias` [N] is added here) hold N = A*(C+7+2) channels
 * ordered cls [A*C] | reg [A*7] | dir [A*2], anchor a = s*R + r; element (frame b, BEV cell
 * loc = h*W + w, channel n) lives at z[b*z_sb + loc*z_shw + n*z_sn] (fp32, or bf16 if z_bf16):
 * NCHW fp32 = (N*H*W, 1, H*W), the NHWC bf16 GEMM image with pitch P = (H*W*P, P, 1).
 * anchor_tab (device fp32): xc[S][W], yc[S][H], zc[S], sizes[S][3], rotations[R] — the
 * Anchor3DRangeGenerator centres (torch.linspace of each range).
 * gt_boxes [B][max_gts][7] fp32, gt_labels [B][max_gts] int64 (-1 = padding).
 * assigned [B][H*W*A] int32 out: -1 ignored, 0 negative, j+1 positive for gt j (kept for backward).
 * losses (device fp32 [4]) out: loss_cls, loss_bbox, loss_dir, num_total_pos (= sum_b max(pos_b, 1)).
 * The workspace must be kept between forward and backward. */
#define RPC_HEAD_MAX_SIZES 4
typedef struct {
  int B, H, W;
  int S, R, C;              /* anchor sizes (ranges), rotations, classes */
  int NA;                   /* assigners: S (list-valued train_cfg.assigner) or 1 */
  int assigner_per_size, assign_per_class, use_dir, diff_rad_by_sin;
  float pos_iou_thr[RPC_HEAD_MAX_SIZES], neg_iou_thr[RPC_HEAD_MAX_SIZES], min_pos_iou[RPC_HEAD_MAX_SIZES];
  float dir_offset, dir_limit_offset, pos_weight;
  float beta, gamma, alpha;           /* SmoothL1 beta, focal gamma / alpha */
  float lw_cls, lw_bbox, lw_dir;      /* loss weights */
  int z_bf16;
  long long z_sb, z_shw, z_sn;
  int dz_bf16;
  long long dz_sb, dz_shw, dz_sn;
  int dz_nwrite;                      /* channels written per cell in dz (>= N; extra ones zeroed) */
} RpcHeadCfg;

size_t rpc_anchor_head_workspace_size(const RpcHeadCfg* cfg, int max_gts);
int rpc_anchor_head_loss_forward(const RpcHeadCfg* cfg, const float* anchor_tab, const float* gt_boxes,
                                 const long long* gt_labels, int max_gts, const void* z, const float* bias,
                                 int* assigned, float* losses, void* workspace, size_t ws_bytes, void* stream);
/* d(losses)/dz scaled by grad_losses[3] (device fp32: upstream grads of loss_cls/bbox/dir), written
 * through the dz_* strides; dbias [N] (optional) = sum over cells of dz (fixed-order reduction). */
int rpc_anchor_head_loss_backward(const RpcHeadCfg* cfg, const float* anchor_tab, const float* gt_boxes,
                                  int max_gts, const void* z, const float* bias, const int* assigned,
                                  const float* grad_losses, const float* losses, void* dz, float* dbias,
                                  void* workspace, size_t ws_bytes, void* stream);


/* ------------------------------------------------------------------ a9 / a10 step tail
 * Loss combination of AdversarialVoxelNet.loss for upstream's list-valued head losses
 * (models/detectors/adversarial_voxelnet.py:187-421: det_loss_total = 0, so
 * loss_adversarial = 0.01*(loss_intensity+loss_bias+loss_imbalance), :378-413) followed by mmengine
 * parse_losses. head_losses (device fp32 [3]) = loss_cls, loss_bbox, loss_dir; pert_losses [4] =
 * VoxelPerturber (l2_norm, intensity_loss, bias_loss, imbalance_loss); reg_coef =
 * regularization_weight * max(0.1, 1-(epoch+1)/30). out [10] = loss_cls, loss_bbox, loss_dir,
 * loss_adversarial, loss_intensity, loss_bias, loss_imbalance, loss_l2_regularization,
 * perturbation_l2_norm, total. Backward: grad_out [10] -> grad_head [3], grad_pert [4]. */
int rpc_loss_tail_forward(const float* head_losses, const float* pert_losses, float reg_coef, float* out,
                          void* stream);
int rpc_loss_tail_backward(const float* pert_losses, float reg_coef, const float* grad_out, float* grad_head,
                           float* grad_pert, void* stream);
/* Loss combination of AdversarialCenterPoint.loss_by_feat_single (models/detectors/adversarial_centerpoint.py:
 * 203-257; the perturber's l2_norm scalar as the documented fix of :81) + parse_losses over the CenterHead's packed task
 * losses (device fp32 [n]: task t heatmap 2t, bbox 2t+1) and l2 (device fp32 scalar); negw = -min(w*epoch/10, w),
 * rw = regularization_weight. out [n + 4] = task losses, loss_adversarial (det > 0 ? negw*det : 0, det = sum of the
 * finite clamp(v, 0, 100)), loss_l2_regularization = rw*l2, perturbation_l2_norm = l2, total (dict order).
 * Backward: grad_out [n + 4] -> grad_losses [n], grad_l2 [1]. Values bit-identical to the torch composition. */
int rpc_center_tail_forward(const float* task_losses, int n, const float* l2, float negw, float rw, float* out,
                            void* stream);
int rpc_center_tail_backward(const float* task_losses, int n, float negw, float rw, const float* grad_out,
                             float* grad_losses, float* grad_l2, void* stream);

/* torch.nn.utils.clip_grad_norm_(max_norm) + torch.optim.AdamW step as mmengine's OptimWrapper runs
 * them (configs/adversarial/adversarial-second_hv_secfpn_8xb6-80e_kitti-3d-3class.py:130-140),
 * over a table of fp32 tensors (device int64 arrays of addresses; grad address 0 = no gradient:
 * the tensor is skipped like torch does). Tensors are processed in chunks of RPC_OPTIM_CHUNK
 * elements: chunk c covers elements [chunk_start[c], +RPC_OPTIM_CHUNK) of tensor chunk_tensor[c].
 * norm_out (device fp32 [2]) = total grad norm, clip coefficient. The clipped gradients are used
 * in the update and not written back. lr[group[t]] is tensor t's learning rate; steps (device fp32
 * [ntensors], torch's state['step']) advance by one for every tensor that has a gradient, and the
 * bias corrections 1 - beta^step are formed per tensor. */
#define RPC_OPTIM_CHUNK 16384
typedef struct {
  float lr[4];
  float beta1, beta2, eps, weight_decay;
} RpcAdamWHyper;
size_t rpc_clip_adamw_workspace_size(int nchunks);
int rpc_clip_adamw(const long long* param_ptrs, const long long* grad_ptrs, const long long* exp_avg_ptrs,
                   const long long* exp_avg_sq_ptrs, const int* numel, const int* group, const int* chunk_tensor,
                   const int* chunk_start, int nchunks, int ntensors, float* steps, const RpcAdamWHyper* hyper,
                   float max_norm, float* norm_out, void* workspace, size_t ws_bytes, void* stream);


/* ------------------------------------------------------------------ §8(f4) strong variant
 * StrongAdversarialVoxelNet.apply_enhanced_perturbations + update_adversarial_strength
 * (models/detectors/strong_adversarial_voxelnet.py:109-192) on the HardSimpleVFE output x [n]
 * (= V*F floats) and the adversary's output adv_out [n]:
 *   scaling = min(epoch_scaling * boost * complexity, max_scaling) (boost from the mean |l2| of the
 *   last 50 entries of the device ring `history` once history_count > 50; dynamic = 0 -> 1.0),
 *   scaled = (adv_out - x) * scaling [+ momentum_alpha * last_scaled], perturbed = x + scaled,
 *   l2 = ||scaled||_2, written to state[1] and history[history_count % RPC_STRONG_RING];
 *   state[0] = scaling, state[2] = adversarial_loss_weight * scaling (both rounded once). Host values are the reference's Python-side numbers (epoch_scaling =
 *   min(1 + 0.1 epoch, max_scaling), complexity = min(1 + iteration/1e4, 2)). */
#define RPC_STRONG_RING 64
typedef struct {
  double epoch_scaling, complexity, max_scaling, adversarial_loss_weight;
  float momentum_alpha;
  int dynamic, curriculum;
  long long history_count;   /* entries recorded before this step */
} RpcStrongCfg;
size_t rpc_strong_perturb_workspace_size(void);
int rpc_strong_perturb_forward(const RpcStrongCfg* cfg, const float* x, const float* adv_out,
                               const float* last_scaled, long long n, float* perturbed, float* scaled,
                               float* history, float* state, void* workspace, size_t ws_bytes, void* stream);
/* grad_x = g_p - g_s * scaling, grad_adv_out = g_s * scaling, g_s = g_p + grad_l2 * scaled / l2 */
int rpc_strong_perturb_backward(const float* scaled, long long n, const float* state, const float* grad_perturbed,
                                const float* grad_l2, float* grad_x, float* grad_adv_out, void* stream);


/* ------------------------------------------------------------------ §8(f2) train-pipeline augmentation
 * The per-frame point / box transforms of configs/_base_/kitti-3d-car.py:42-68 (upstream mmdet3d
 * RandomFlip3D, GlobalRotScaleTrans, PointsRangeFilter, ObjectRangeFilter, PointShuffle) for B
 * frames concatenated in `points` [P][F] with device offsets [B+1]. frames (device [B]): the random
 * draws of each frame (made on the host in the reference's RNG order) with cos/sin of the rotation.
 * out_points [P][F]: each frame's surviving points, compacted in order (or shuffled, shuffle != 0,
 * a seeded uniform permutation per frame), out_offsets (device [B+1]); rows beyond the survivors
 * are NaN (hard_voxelize drops them, so no host read of the count is needed).
 * rpc_augment_boxes transforms boxes [B][M][7] / labels [B][M] (int64, -1 = padding) in place;
 * boxes outside the BEV range become padding; yaw wrapped by limit_yaw(0.5, 2 pi). */
typedef struct {
  int flip_h, flip_v;
  float rot, cosr, sinr, scale, tx, ty, tz;
} RpcAugFrame;
size_t rpc_augment_points_workspace_size(int num_features, int total_points);
int rpc_augment_points(const float* points, int num_features, int total_points, const int* frame_offsets, int batch,
                       const RpcAugFrame* frames, const float* pc_range /* host [6] */, int shuffle,
                       unsigned long long seed, float* out_points, int* out_offsets, void* workspace,
                       size_t ws_bytes, void* stream);
int rpc_augment_boxes(float* boxes, long long* labels, int batch, int max_gts, const RpcAugFrame* frames,
                      const float* pc_range /* host [6] */, void* stream);


/* ------------------------------------------------------------------ §8(f3) CenterHead targets + losses
 * Replaces upstream mmdet3d `CenterHead.get_targets` / `loss_by_feat` (dense_heads/centerpoint_head.py;
 * draw_heatmap_gaussian, gaussian_radius, mmdet GaussianFocalLoss + L1Loss) as configured by
 * configs/adversarial/adversarial-centerpoint_voxel-nuscenes.py:11-13 (the upstream
 * centerpoint_voxel01_second_secfpn_head-dcn base) and called at
 * models/detectors/adversarial_centerpoint.py:224 (`pts_bbox_head.loss_by_feat`).
 * Feature map H x W (= grid_size[1] / osf, grid_size[0] / osf). Head outputs (fp32) per cell
 * p = (b*H + y)*W + x: heatmap logits hm[p*hm_pitch + g] for the global class g (classes in task
 * order, task t owning task_ncls[t] consecutive classes), boxes box[p*box_pitch + t*10 + c] with
 * c = reg(2) | height(1) | dim(3) | rot(2) | vel(2).
 * gt_boxes [B][max_gts][9] fp32 (LiDAR bottom centre x, y, z, dx, dy, dz, yaw, vx, vy), gt_labels
 * [B][max_gts] int64 (-1 = padding). losses (device fp32 [2*ntasks]) out: task t loss_heatmap at 2t,
 * loss_bbox at 2t+1. The workspace (targets, normalisers) must be kept between forward and backward. */
#define RPC_CENTER_MAX_TASKS 8
typedef struct {
  int B, H, W;
  int ntasks, ncls_total;
  int task_ncls[RPC_CENTER_MAX_TASKS];
  int max_objs, min_radius, out_size_factor, norm_bbox;
  float voxel_x, voxel_y, pc_x, pc_y;
  double gaussian_overlap;            /* python float: the radius constants are formed from it */
  float code_weights[10];
  float loss_cls_weight, loss_bbox_weight;
  int hm_pitch, box_pitch;
} RpcCenterCfg;

size_t rpc_center_head_workspace_size(const RpcCenterCfg* cfg, int max_gts);
int rpc_center_head_loss_forward(const RpcCenterCfg* cfg, const float* gt_boxes, const long long* gt_labels,
                                 int max_gts, const float* hm, const float* box, float* losses, void* workspace,
                                 size_t ws_bytes, void* stream);
/* grad_losses [2*ntasks] (device) -> dhm (cells x hm_pitch, every heatmap channel written) and dbox
 * (cells x box_pitch, zero except at the gathered cells). */
int rpc_center_head_loss_backward(const RpcCenterCfg* cfg, const float* hm, const float* box,
                                  const float* grad_losses, float* dhm, float* dbox, void* workspace,
                                  size_t ws_bytes, void* stream);
/* The training targets themselves (for tests / inspection): heatmap [B][H][W][ncls_total],
 * ind [B][ntasks][max_objs] int32, mask [B][ntasks][max_objs] int32, anno [B][ntasks][max_objs][10]
 * — views into a workspace filled by rpc_center_head_loss_forward. */
/* Task-head final conv outputs: out[p*op + ooff + c] = z[p*zp + c] (bf16) + bias[c], c < n <= 16;
 * backward: dz[p*zp + c] = bf16(dout[p*dp + doff + c]) (c < n, else 0) and dbias = sum_p dout. */
int rpc_head_pack(const void* z, int zp, int n, const float* bias, float* out, int op, int ooff, long long cells,
                  void* stream);
size_t rpc_head_unpack_workspace_size(void);
int rpc_head_unpack_grad(const float* dout, int dp, int doff, int n, void* dz, int zp, long long cells, float* dbias,
                         void* workspace, size_t ws_bytes, void* stream);
/* parity mode: the same with fp32 z / dz images */
int rpc_head_pack_f32(const float* z, int zp, int n, const float* bias, float* out, int op, int ooff, long long cells,
                      void* stream);
int rpc_head_unpack_grad_f32(const float* dout, int dp, int doff, int n, float* dz, int zp, long long cells,
                             float* dbias, void* workspace, size_t ws_bytes, void* stream);
int rpc_center_head_targets(const RpcCenterCfg* cfg, int max_gts, const void* workspace, const float** heatmap,
                            const int** ind, const int** mask, const float** anno);

/* ------------------------------------------------------------------ §8(f3) DCNSeparateHead deformable conv
 * mmcv DeformConv2dPack(64, 64, kernel 3, padding 1, groups 4, deform_groups 1) of the CenterHead base
 * (adversarial-centerpoint_voxel-nuscenes.py:11-13, DCNSeparateHead.feature_adapt_cls / _reg):
 * x, out: bf16 NHWC images (64 channels at pitch xp / op); off: the offset conv's bf16 output image
 * (pitch offp, channels 0..17 = (dy, dx) per tap k = 3i + j) to which off_bias [18] is added here.
 * W [64][16][3][3] fp32 -> rpc_dcn_prep_weight -> w_fwd / w_bwd (bf16 [9][64][64] each).
 * Backward: dx fp32 [B*H*W][64] is ACCUMULATED (atomics; zero it first), doff = the offset conv's
 * output gradient (bf16 image, pitch doffp >= 64, channels >= 18 written as zero), doff_bias [18] and
 * dW [64][16][3][3] are written. H and W must be multiples of 8. */
int rpc_dcn_prep_weight(const float* W, void* w_fwd, void* w_bwd, void* stream);
int rpc_dcn_forward(const void* x, int xp, const void* off, int offp, const float* off_bias, const void* w_fwd,
                    void* out, int op, int B, int H, int W, void* stream);
size_t rpc_dcn_backward_workspace_size(int B, int H, int W);
int rpc_dcn_backward(const void* x, int xp, const void* off, int offp, const float* off_bias, const void* w_bwd,
                     const void* dout, int dop, float* dx, void* doff, int doffp, float* doff_bias, float* dW,
                     int B, int H, int W, void* workspace, size_t ws_bytes, void* stream);
/* parity mode: the same deformable convolution on fp32 images (x, off, out, dout, doff; pitches
 * multiples of 4) in fp32 arithmetic, W [64][16][3][3] fp32 read directly (no prep); the backward
 * workspace is rpc_dcn_backward_workspace_size's. */
int rpc_dcn_forward_f32(const float* x, int xp, const float* off, int offp, const float* off_bias, const float* W,
                        float* out, int op, int B, int H, int W_, void* stream);
int rpc_dcn_backward_f32(const float* x, int xp, const float* off, int offp, const float* off_bias, const float* W,
                         const float* dout, int dop, float* dx, float* doff, int doffp, float* doff_bias, float* dW,
                         int B, int H, int W_, void* workspace, size_t ws_bytes, void* stream);
/* rpc_dcn_backward / _f32 with the offset-gradient channel count: doff_channels = 64 is the calls above
 * (a padded image of its own), 18 writes exactly the 18 offset channels at doff (4-byte aligned bf16 /
 * 8-byte aligned fp32, doffp >= 18 and even), so several DCNs can write their slices of ONE image: the
 * output gradient of the head's concatenated offset conv (12 offset convs of a CenterPoint head as one
 * 64 -> 216 (+40 zero) conv, DCN j at channel 18 j, pitch 256; center_head.py). */
int rpc_dcn_backward_ex(const void* x, int xp, const void* off, int offp, const float* off_bias, const void* w_bwd,
                        const void* dout, int dop, float* dx, void* doff, int doffp, int doff_channels,
                        float* doff_bias, float* dW, int B, int H, int W, void* workspace, size_t ws_bytes,
                        void* stream);
int rpc_dcn_backward_f32_ex(const float* x, int xp, const float* off, int offp, const float* off_bias,
                            const float* W, const float* dout, int dop, float* dx, float* doff, int doffp,
                            int doff_channels, float* doff_bias, float* dW, int B, int H, int W_, void* workspace,
                            size_t ws_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* RPC_HIP_H */
