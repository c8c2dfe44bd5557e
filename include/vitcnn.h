/*
 * vitcnn.h — C ABI of the MI355X (gfx950) ViT-CNN training hot path.
 *
 * libvitcnn_hip.so exports one entry point per fused device op of the reference's
 * "ViT-CNN (ours)" model (Multimodality_Mamba, /root/reference/model/Multimodality_Mamba/
 * Mutimodality_Mamba7.py:1141-1181) and of its training iteration (model_utils.py:918-936).
 * The reference has no native layer of its own: each entry
 * point below replaces a PyTorch op sequence of the reference, cited per function, and is
 * what the reference's plugin (get_model -> nn.Module.forward / loss.backward /
 * optimizer.step) binds through the Python mirror in vit-cnn_amd/vitcnn_amd (ctypes).
 *
 * Conventions (all functions):
 *   - plain device pointers (fp32 unless stated; int32 index tables), sizes and leading
 *     dimensions in elements; activations are channels-last [rows, C] row-major;
 *   - the caller owns every buffer, including the fp32 workspace `ws` (ws_floats elements)
 *     that reductions use for fixed-order partial sums; nothing is allocated, nothing
 *     synchronises, so every call is capturable into a hipGraph;
 *   - work is enqueued on `stream`; return 0 on success, a hipError_t code on a launch
 *     failure, 1 (hipErrorInvalidValue) on an invalid shape — the Python mirror raises
 *     RuntimeError, like the reference's shape errors;
 *   - `beta_*` arguments select overwrite (0) or accumulate (1) for outputs that several
 *     backward branches feed.
 */
#ifndef VITCNN_H
#define VITCNN_H

#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
#define VC_API extern "C" __attribute__((visibility("default")))
#else
#define VC_API __attribute__((visibility("default")))
#endif

/* ---------------------------------------------------------------- dense contractions
 * C[b] = alpha * op(A[b]) op(B[b]) + beta*C[b] (+ bias[n]) (+ addend[(m % add_mod)*add_ld + n]) (ReLU if flags&1)
 * op(A)(m,k) = transA ? A[k*lda+m] : A[m*lda+k];  op(B)(k,n) = transB ? B[n*ldb+k] : B[k*ldb+n].
 * fp32 in / fp32 accumulate on v_mfma_f32_16x16x4_f32, or, with flags&2, bf16 operands (rounded
 * RNE as they are staged) with fp32 accumulation on v_mfma_f32_16x16x32_bf16 (the config-2 mode);
 * flags&4 / flags&8 force the k-major / K-contiguous fp32 kernel, flags&16 / flags&32 take / skip the
 * pipelined LDS-DMA fp32 kernel (default: chosen by shape).  flags&64 turns the addend into a mask:
 * the result (after alpha, beta, bias) is kept where addend[(m % add_mod)*add_ld + n] > 0 and zeroed
 * elsewhere -- a ReLU backward through that layer output, fused into the GEMM producing the gradient.
 * Split-K (fixed-order, deterministic) when the output grid is small and ws is given.  bias_grad (batch 1 only, may be null) additionally receives
 * alpha * sum_k op(A)(m,k) (+ beta * bias_grad[m]) through an implicit ones column of op(B): the
 * bias gradient of a layer rides along its weight-gradient GEMM.  Replaces nn.Conv2d 1x1 /
 * 3x3-after-im2col / nn.Linear / torch.matmul forward and backward (Mutimodality_Mamba7.py:258,
 * :1040, :1068, :1071, :101-134, :147, :152, :1098, :1124, :1160; transformers
 * modeling_mamba.py:372, :433, :438, :481). */
VC_API int vc_gemm(int transA, int transB, int M, int N, int K, float alpha,
                   const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                   float beta, float* C, long ldc, long strideC, int batch,
                   const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                   float* bias_grad, float* ws, long ws_floats, hipStream_t stream);
/* vc_gemm with an in-launch split-K combine: tile_counters (n_counters >= the output tile count) is
 * a caller-owned unsigned array that is zero on entry and left zero; when split-K is chosen the
 * last-arriving slice of each tile sums the slices (same fixed order as vc_gemm's separate reduce
 * kernel: bit-identical results) instead of a second launch.  Counters must not be shared by
 * concurrently running calls (one array per stream).  NULL counters = vc_gemm. */
VC_API int vc_gemm_ex(int transA, int transB, int M, int N, int K, float alpha, const float* A, long lda,
                      long strideA, const float* B, long ldb, long strideB, float beta, float* C, long ldc,
                      long strideC, int batch, const float* bias, const float* addend, long add_ld, int add_mod,
                      int flags, float* bias_grad, float* ws, long ws_floats, unsigned int* tile_counters,
                      int n_counters, hipStream_t stream);

/* Measurement hook: force the tile (bm, bn in {64, 128}), split-K slice count, prefetch depth
 * (pf in {1, 2}) and combine path (combine: 1 in-launch, 0 separate reduce kernel) of the following
 * vc_gemm / vc_gemm_ex calls; 0 (-1 for combine) restores the automatic choice.  Only the probe
 * library (libvitcnn_probe.so, `make probe`; tools/gemm_sweep.py) keeps this state; the product
 * library keeps none and accepts only the automatic configuration (0, 0, 0, 0, -1). */
VC_API int vc_gemm_tune(int bm, int bn, int nsplit, int pf, int combine);

/* C [M, N] = A [M, K] W [N, K]^T + bias on the pipelined kernel (no split-K; flags & 2: bf16 operands) with the
 * BatchNorm statistics partials of C computed in the epilogue: colstats [ceil(M/64)][2][N] fp64 sums of (C - bias)
 * and (C - bias)^2 per 64-row tile -- the conv1x1 + BN forward's statistics pass folded into its GEMM
 * (vc_bn_apply_partials finishes the BatchNorm).  A, W 16-B aligned, K, lda, ldw multiples of 4. */
VC_API int vc_gemm_colstats(int M, int N, int K, const float* A, long lda, const float* W, long ldw, const float* bias,
                            float* C, long ldc, int flags, double* colstats, hipStream_t stream);
/* Grouped launches: a horizontal fusion of independent products (a layer's weight and data
 * gradients, parallel branches).  `group` is caller-owned host memory of VC_GEMM_GROUP_BYTES bytes
 * (8-byte aligned) holding the group's state -- the library keeps none, so distinct groups (one per
 * stream / thread) are independent and every entry point stays reentrant.  vc_gemm_group_begin
 * opens it for `stream`; vc_gemm_group_add takes vc_gemm_ex's arguments (minus the stream): fp32
 * problems of the k-major kernel and fp32 / bf16 problems of the pipelined 64x64 kernel are recorded;
 * anything else (bf16 problems on the legacy tiles, long K) launches at once on the group's stream;
 * vc_gemm_group_end launches the recorded problems as
 * one grid per kernel (up to 8 problems each) plus one grouped split-K reduce.  A problem's plan
 * depends on its shape and the workspace / counters passed to it only, so its result is bit-identical
 * grouped or alone.  The problems must not depend on each other; each takes its own
 * slice of the workspace and arrival counters passed to it.  Misuse (add / end on a group that is
 * not open) returns 1. */
#define VC_GEMM_GROUP_BYTES 16384
VC_API int vc_gemm_group_begin(void* group, hipStream_t stream);
VC_API int vc_gemm_group_add(void* group, int transA, int transB, int M, int N, int K, float alpha,
                             const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                             float beta, float* C, long ldc, long strideC, int batch, const float* bias,
                             const float* addend, long add_ld, int add_mod, int flags, float* bias_grad,
                             float* ws, long ws_floats, unsigned int* tile_counters, int n_counters);
VC_API int vc_gemm_group_end(void* group);

/* out[c] = beta*out[c] + sum_r X[r*ldx + c]  (bias gradients; fixed-order two-stage) */
VC_API int vc_colsum(int R, int C, const float* X, long ldx, float* out, float beta,
                     float* ws, long ws_floats, hipStream_t stream);
/* The same with >= ceil(C/64) zeroed arrival counters (left zero; per stream): the partials are
 * reduced in the last-arriving block of each column group, no second launch. */
VC_API int vc_colsum_ex(int R, int C, const float* X, long ldx, float* out, float beta,
                        float* ws, long ws_floats, unsigned int* counters, int n_counters, hipStream_t stream);

/* ---------------------------------------------------------------- normalisation
 * LayerNorm over the last dim (nn.LayerNorm eps=1e-6 via build_norm_layer,
 * mmpretrain/models/utils/norm.py:119-123; used at Mutimodality_Mamba7.py:656, :985,
 * :1083, :1085).  Saves per-row mean / rstd for the backward. */
VC_API int vc_layernorm_fwd(int R, int C, const float* x, long ldx, const float* w, const float* b, float eps,
                            float* y, long ldy, float* mean, float* rstd, hipStream_t stream);
VC_API int vc_layernorm_bwd(int R, int C, const float* dy, long lddy, const float* x, long ldx, const float* w,
                            const float* mean, const float* rstd, float* dx, long lddx, float beta_dx,
                            float* dw, float* db, float beta_w, float* ws, long ws_floats, hipStream_t stream);
/* The same with dx = res + LNgrad: the residual gradient is read from res (left untouched). */
VC_API int vc_layernorm_bwd_res(int R, int C, const float* dy, long lddy, const float* x, long ldx, const float* w,
                                const float* mean, const float* rstd, const float* res, long ldr, float* dx,
                                long lddx, float* dw, float* db, float beta_w, float* ws, long ws_floats,
                                hipStream_t stream);
/* Split form: dx now (res + LN grad, or beta_dx * dx + LN grad when res is null) with the dw / db
 * partials left in `part`; the parameter reduction later (same R, C, part_floats), e.g. on another
 * stream off the critical path.  Together bit-identical to vc_layernorm_bwd. */
VC_API int vc_layernorm_bwd_dx(int R, int C, const float* dy, long lddy, const float* x, long ldx, const float* w,
                               const float* mean, const float* rstd, const float* res, long ldr, float* dx,
                               long lddx, float beta_dx, float* part, long part_floats, hipStream_t stream);
VC_API int vc_layernorm_bwd_params(int R, int C, const float* part, long part_floats, float* dw, float* db,
                                   float beta_w, hipStream_t stream);

/* BatchNorm2d over channels-last rows (torch train/eval semantics, eps, momentum):
 * ms_conv_bn_relu.bn (Mutimodality_Mamba7.py:1039), FusionLayer BN (:1103, :1129),
 * NonLocal W[1] (:113).  train=1: batch stats (biased var) -> save_mean/save_invstd and the
 * running stats (unbiased var) are updated in place; train=0: save_* from running stats. */
VC_API int vc_bn_stats(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                       float* save_mean, float* save_invstd, float* run_mean, float* run_var,
                       float* ws, long ws_floats, hipStream_t stream);
/* stats + apply in one call (train: the partials kernel + a channel-tiled apply that reduces them itself,
 * two launches; eval: from the running statistics); bit-identical to vc_bn_stats + vc_bn_apply */
VC_API int vc_bn_forward(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                         float* save_mean, float* save_invstd, float* run_mean, float* run_var, const float* w,
                         const float* b, int relu, float* y, long ldy, float* ws, long ws_floats, hipStream_t stream);
VC_API int vc_bn_apply(long M, int C, const float* x, long ldx, const float* mean, const float* invstd,
                       const float* w, const float* b, int relu, float* y, long ldy, hipStream_t stream);
VC_API int vc_bn_bwd(int train, long M, int C, const float* dy, long lddy, const float* x, long ldx,
                     const float* relu_out, long ldo, const float* mean, const float* invstd, const float* w,
                     float* dx, long lddx, float beta_dx, float* dw, float* db, float beta_w,
                     float* ws, long ws_floats, hipStream_t stream);
/* The same with zeroed arrival counters (left zero; per stream, as vc_gemm_ex's).  vc_bn_stats_ex and
 * vc_bn_bwd_ex without dx (>= ceil(C/64) counters) reduce per channel in the last-arriving partial block,
 * one launch fewer than without counters; vc_bn_forward_ex and vc_bn_bwd_ex with dx ignore them (the
 * channel-tiled apply reduces the partials itself: two launches).  Results are bit-identical with and
 * without counters. */
VC_API int vc_bn_forward_ex(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                            float* save_mean, float* save_invstd, float* run_mean, float* run_var, const float* w,
                            const float* b, int relu, float* y, long ldy, float* ws, long ws_floats,
                            unsigned int* counters, int n_counters, hipStream_t stream);
VC_API int vc_bn_stats_ex(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                          float* save_mean, float* save_invstd, float* run_mean, float* run_var,
                          float* ws, long ws_floats, unsigned int* counters, int n_counters, hipStream_t stream);
VC_API int vc_bn_bwd_ex(int train, long M, int C, const float* dy, long lddy, const float* x, long ldx,
                        const float* relu_out, long ldo, const float* mean, const float* invstd, const float* w,
                        float* dx, long lddx, float beta_dx, float* dw, float* db, float beta_w,
                        float* ws, long ws_floats, unsigned int* counters, int n_counters, hipStream_t stream);
/* train-mode BatchNorm forward from fp64 partials another kernel produced ([P][2][C]: per partial p, sum (x - shift[c])
 * and sum (x - shift[c])^2 over its rows; vc_gemm_colstats writes them with P = ceil(M / 64), shift = its bias):
 * save_* and the running statistics as vc_bn_forward, y = relu?(BN(x)); one launch */
VC_API int vc_bn_apply_partials(long M, int C, const float* x, long ldx, int P, const double* part, const float* shift,
                                float eps, float momentum, float* save_mean, float* save_invstd, float* run_mean,
                                float* run_var, const float* w, const float* b, int relu, float* y, long ldy,
                                hipStream_t stream);
/* vc_bn_bwd_ex through the ReLU that follows the BatchNorm, its decisions recomputed from x, the saved
 * statistics and the affine (w, b) with the forward's own arithmetic instead of read from the forward's
 * output: bit-identical to vc_bn_bwd_ex with relu_out = that output, one [M, C] read less per pass. */
VC_API int vc_bn_bwd_relu_ex(int train, long M, int C, const float* dy, long lddy, const float* x, long ldx,
                             const float* mean, const float* invstd, const float* w, const float* b, float* dx,
                             long lddx, float beta_dx, float* dw, float* db, float beta_w, float* ws, long ws_floats,
                             unsigned int* counters, int n_counters, hipStream_t stream);

/* ---------------------------------------------------------------- layout / spatial
 * NCHW input patches (the reference's batch layout, datasets.py:571-572) -> channels-last. */
VC_API int vc_nchw_to_nhwc(int B, int C, int HW, const float* x, float* y, hipStream_t stream);
/* the same into rows of ldy >= C floats with columns C .. ldy - 1 written 0 (FusAtNet's 1-band LiDAR input padded
 * to 4 channels: 16-B rows for the pipelined conv) */
VC_API int vc_nchw_to_nhwc_pad(int B, int C, int HW, const float* x, float* y, int ldy, hipStream_t stream);

/* 3x3 valid im2col of a channels-last [B,H,W,C] map with the preceding BatchNorm's affine
 * (bn_* may be null) fused in: col[(b,oh,ow), c*9+kh*3+kw] — ms_conv_bn_relu
 * (Mutimodality_Mamba7.py:1035-1048), column order matching the [Co, Ci, 3, 3] weight. */
VC_API int vc_im2col3x3(int B, int H, int W, int C, const float* x, const float* bn_mean, const float* bn_invstd,
                        const float* bn_w, const float* bn_b, float* col, hipStream_t stream);
/* Implicit-GEMM 3x3 convolution (no im2col matrix) over channels-last maps, k = c*9 + kh*3 + kw over
 * the torch weight [O][C][3][3] = [O][9C] (ms_conv_bn_relu, Mutimodality_Mamba7.py:1035-1048; FusAtNet
 * ConvUnit / ConvUnit_NP / Residual units, FusAtNet.py:9-60).  x [B,H,W,C] (row stride ldx); pad 0
 * (valid) or 1; output map [B,OH,OW,O], OH = H + 2 pad - 2.  bn_* (all or none): the preceding
 * BatchNorm's affine (x - mean) * invstd * w + b applied to in-range pixels as the operand is gathered.
 *   fwd:   y (ld ldy) = conv(x) + bias (ReLU if relu)
 *   wgrad: dweight [O][9C] = beta*dweight + dY^T im2col(x); dbias [O] (may be null) = beta*dbias + colsum(dY)
 *   dgrad: dx (ld lddx) = beta*dx + the conv's input gradient for dY [B,OH,OW,O] (ld lddy)
 * ws: split-K slabs (fixed-order sums); may be null (no split). */
VC_API int vc_conv3x3_fwd(int B, int H, int W, int C, int O, int pad, const float* x, long ldx, const float* bn_mean,
                          const float* bn_invstd, const float* bn_w, const float* bn_b, const float* weight,
                          const float* bias, int relu, float* y, long ldy, float* ws, long ws_floats,
                          hipStream_t stream);
VC_API int vc_conv3x3_wgrad(int B, int H, int W, int C, int O, int pad, const float* x, long ldx, const float* bn_mean,
                            const float* bn_invstd, const float* bn_w, const float* bn_b, const float* dy, long lddy,
                            float beta, float* dweight, float* dbias, float* ws, long ws_floats, hipStream_t stream);
VC_API int vc_conv3x3_dgrad(int B, int H, int W, int C, int O, int pad, const float* dy, long lddy, const float* weight,
                            float beta, float* dx, long lddx, float* ws, long ws_floats, hipStream_t stream);
/* FusAtNet's 3x3 convs (FusAtNet.py:10-62, :168-186; stride 1, pad 0 or 1, channels-last rows) as
 * implicit GEMMs over a TAP-MAJOR contraction index k = tap * C + c (conv_tap.hip): operand tiles are
 * row gathers (one input row per output pixel and tap), no im2col matrix, no col2im.  Weights in
 * tap-major layouts made by vc_conv3x3_pack from the torch layout w [O][C][3][3]:
 *   mode 0: Wt [O][9][Cw] (fwd and dgrad), Cw = C rounded up to a multiple of 4, padding written 0
 *           (16-B aligned rows: float4 operand loads at any C)                mode 1: W2 [9][O][C]
 *   mode 2: w = beta w + dWt unpacked (wgrad's tap-major [O][9][C] gradient back to the torch layout)
 *   fwd:   y [B*OH*OW] (ld ldy) = conv(x) + bias (bias may be null); with C % 4 != 0 and ldx % 4 == 0 the
 *          row padding x[.][C .. C rounded to 4) is read (against zero weights) and must hold finite values
 *   wgrad: dWt [O][9][C] = sum over output pixels of dy x (overwritten; the bias gradient is colsum(dy))
 *   dgrad: dx (ld lddx) = beta dx + the conv's input gradient for dy
 * ws: split-K slabs when the tile grid is small (fixed-order sums; may be null: no split). */
VC_API int vc_conv3x3_pack(int O, int C, int mode, const float* src, float* dst, float beta, hipStream_t stream);
/* mode-0 packs of n convs in one launch per 48: shapes = host array {O0, C0, O1, C1, ...}, src / dst = host
 * arrays of n device pointers (torch-layout weights / Wt buffers); bit-identical to n vc_conv3x3_pack calls */
VC_API int vc_conv3x3_pack_many(int n, const int* shapes, const float* const* src, float* const* dst,
                                hipStream_t stream);
VC_API int vc_conv3x3_tap_fwd(int B, int H, int W, int C, int O, int pad, const float* x, long ldx, const float* wt,
                              const float* bias, float* y, long ldy, float* ws, long ws_floats, hipStream_t stream);
VC_API int vc_conv3x3_tap_wgrad(int B, int H, int W, int C, int O, int pad, const float* x, long ldx, const float* dy,
                                long lddy, float* dwt, float* ws, long ws_floats, hipStream_t stream);
VC_API int vc_conv3x3_tap_dgrad(int B, int H, int W, int C, int O, int pad, const float* dy, long lddy,
                                const float* wt, float beta, float* dx, long lddx, float* ws, long ws_floats,
                                hipStream_t stream);
/* wgrad written straight into the torch layout dw [O][C][3][3] (overwritten): vc_conv3x3_tap_wgrad +
 * vc_conv3x3_pack mode 2 with beta 0 in one call, bit-identical (the same sums, stored transposed); db
 * (nullable, overwritten) also receives the bias gradient sum over output pixels of dy (the blocks of the
 * first output tile column sum their staged dy tiles: no separate column-sum launches). */
VC_API int vc_conv3x3_tap_wgrad_oihw(int B, int H, int W, int C, int O, int pad, const float* x, long ldx,
                                     const float* dy, long lddy, float* dw, float* db, float* ws, long ws_floats,
                                     hipStream_t stream);
/* train-mode BatchNorm(x) (statistics as vc_bn_stats_ex: save_* and running stats written) followed by
 * vc_im2col3x3 of the normalised x, the statistics' final reduction done inside the im2col launch
 * (ms_conv_bn_relu's BN -> conv3x3, Mutimodality_Mamba7.py:1035-1048); bit-identical to the two calls. */
VC_API int vc_bn_im2col3x3(int B, int H, int W, int C, const float* x, float eps, float momentum, float* save_mean,
                           float* save_invstd, float* run_mean, float* run_var, const float* bn_w, const float* bn_b,
                           float* col, float* ws, long ws_floats, hipStream_t stream);
/* gradient of vc_im2col3x3 w.r.t. its (post-BN) input, gather form: dx [B,H,W,C] overwritten */
VC_API int vc_col2im3x3(int B, int H, int W, int C, const float* dcol, float* dx, hipStream_t stream);

/* vc_maxpool2_fwd of the phi | g map pg [B,Hs,Hs,2Ci] (row stride ldpg) followed by vc_nonlocal_attn_fwd, in
 * one launch where the wave-per-row forward runs (training batch sizes): pooled [B,P,2Ci] and arg are still
 * written for the backward. */
VC_API int vc_nonlocal_attn_pool_fwd(int B, int S, int P, int Ci, int Hs, const float* theta, const float* pg,
                                     long ldpg, float* pooled, unsigned char* arg, float* att, float* o,
                                     hipStream_t stream);
/* vc_nonlocal_attn_bwd followed by vc_maxpool2_bwd of the pooled phi | g map (Hs x Hs, P = (Hs/2)^2 keys), in
 * one launch where the MFMA backward applies: dpg [B,Hs,Hs,2Ci] overwritten (dpooled is then untouched;
 * it is the intermediate of the two-launch fallback). */
VC_API int vc_nonlocal_attn_pool_bwd(int B, int S, int P, int Ci, int Hs, const float* theta, const float* pooled,
                                     const float* att, const float* dout, const unsigned char* arg, float* dtheta,
                                     float* dpooled, float* dpg, hipStream_t stream);
/* nn.MaxPool2d(2) of the NonLocal phi/g branches (Mutimodality_Mamba7.py:94, :136-138):
 * x channels-last [B,H,W,C] with row stride ldx -> y [B,H/2,W/2,C] + winning tap (uint8). */
VC_API int vc_maxpool2_fwd(int B, int H, int W, int C, const float* x, long ldx, float* y, unsigned char* arg,
                           hipStream_t stream);
VC_API int vc_maxpool2_bwd(int B, int H, int W, int C, const float* dy, const unsigned char* arg, float* dx,
                           long lddx, hipStream_t stream);

/* ---------------------------------------------------------------- Mamba mixer (10 scan orders)
 * hsiMamba '81_2+8' / '49_2+8' (Mutimodality_Mamba7.py:608-701, :787-867) over transformers
 * MambaMixer (modeling_mamba.py:359-481).  order/inv_order: int32 [ndir, L] token order per
 * direction and its inverse; xz = in_proj(LN(tokens)) computed ONCE per token [B*L, 2D];
 * per-direction sequences are gathered through `order`, never materialised.
 * u [ndir*B*L, D] = SiLU(causal dwconv1d_k4(x-part) + bias). */
VC_API int vc_mamba_dirconv_fwd(int B, int L, int D, int ndir, const int* order, const float* xz,
                                const float* conv_w, const float* conv_b, float* u, hipStream_t stream);
/* selective scan of every direction's sequence (modeling_mamba.py:175-283), ungated:
 * yp[k,b,t,d] = sum_n C_t[n] h_t[d,n] + D_d u_t[d]; h_t = exp(dt A) h_{t-1} + dt B_t u_t,
 * dt = softplus(W_dt dtr_t + b_dt).  u/xdbl/yp are [ndir*B*L, D] / [.., R+32] / [.., D]. */
/* ckpt (nullable): [ndir*B][ceil(L/4)][16][D] fp32 states entering every 4-token segment, saved
 * for vc_mamba_scan_bwd; vc_mamba_scan_ckpt_floats gives its size (-1 on bad arguments) */
VC_API int vc_mamba_scan_ckpt_floats(int B, int L, int D, int ndir);
VC_API int vc_mamba_scan_fwd(int B, int L, int D, int R, int ndir, const float* u, const float* xdbl,
                             const int* order, const float* dt_w, const float* dt_b, const float* A_log,
                             const float* Dskip, float* yp, float* ckpt, hipStream_t stream);
/* ypsum[b,l,:] = sum_k softmax(gate_logits)_k yp[k, b, inv_k(l), :]  (un-permute + gate, :694-701);
 * ysum = ypsum * SiLU(z[b,l,:]) — the token-wise SiLU(z) gate of modeling_mamba.py:274 applied
 * once after the combine (it commutes with the permutation and the gated sum) */
VC_API int vc_mamba_combine_fwd(int B, int L, int D, int ndir, const int* inv_order, const float* gate_logits,
                                const float* yp, const float* xz, float* ypsum, float* ysum, hipStream_t stream);
/* backward of the SiLU(z) gate: dyp = dysum * SiLU(z); the z half of dxz (ld 2D) = dysum * ypsum * SiLU'(z) */
VC_API int vc_mamba_gate_bwd(int B, int L, int D, const float* xz, const float* ypsum, const float* dysum,
                             float* dyp, float* dxz, hipStream_t stream);
/* backward of scan + gated combine given dyp: du, ddt_lin (pre-softplus) per sequence position;
 * the B/C columns of dxdbl (ld R+32); dA_log [D,16], dDskip [D], dgate_logits [ndir] (all overwritten;
 * each may be NULL, its cross-sequence reduction is then skipped).
 * ckpt: the states vc_mamba_scan_fwd saved (nullable: recomputed into ws) */
VC_API int vc_mamba_scan_bwd(int B, int L, int D, int R, int ndir, const float* u, const float* xdbl,
                             const int* order, const float* dt_w, const float* dt_b, const float* A_log,
                             const float* Dskip, const float* gate_logits, const float* yp, const float* dyp,
                             const float* ckpt, float* du, float* ddt_lin, float* dxdbl, float* dA_log,
                             float* dDskip, float* dgate_logits, float* ws, long ws_floats, hipStream_t stream);
/* The parameter reductions of vc_mamba_scan_bwd (dA_log, D, gate logits) from the per-sequence partials a
 * call with null parameter outputs left at the head of its ws; run later / elsewhere, bit-identical. */
VC_API int vc_mamba_scan_bwd_params(int B, int D, int ndir, const float* gate_logits, const float* ws,
                                    float* dA_log, float* dDskip, float* dgate_logits, float* scratch,
                                    long scratch_floats, hipStream_t stream);
/* backward of gather + conv1d + SiLU: du is turned into dpre in place; the x half of dxz [B*L, 2D]
 * is overwritten (summed over the directions); conv weight [D,1,4] / bias [D] grads overwritten */
VC_API int vc_mamba_dirconv_bwd(int B, int L, int D, int ndir, const int* order, const int* inv_order,
                                const float* xz, const float* conv_w, const float* conv_b, float* du, float* dxz,
                                float* dconv_w, float* dconv_b, float* ws, long ws_floats, hipStream_t stream);
/* Fused forms (one launch each way per block on the critical chain; needs D % 4 == 0 and R <= 16 --
 * true for the model's (D, R) = (72, 9) and (128, 16)):
 * vc_mamba_scan_fwd_fused = vc_mamba_dirconv_fwd + xdbl = u x_proj_w^T (modeling_mamba.py:441-456) +
 * vc_mamba_scan_fwd in one kernel; u [ndir*B*L, D] (bit-identical to vc_mamba_dirconv_fwd) and xdbl
 * [.., R+32] are written for the backward. */
VC_API int vc_mamba_scan_fwd_fused(int B, int L, int D, int R, int ndir, const float* xz, const int* order,
                                   const float* conv_w, const float* conv_b, const float* x_proj_w,
                                   const float* dt_w, const float* dt_b, const float* A_log, const float* Dskip,
                                   float* u, float* xdbl, float* yp, float* ckpt, hipStream_t stream);
/* vc_mamba_scan_bwd followed, per sequence, by the dt_proj / x_proj data gradients and the conv1d + SiLU
 * backward (modeling_mamba.py:433-456 backward): dxdbl complete (all R+32 columns), dpre = d(conv
 * pre-activation) [ndir*B*L, D], ddt_lin and the scan parameter outputs as vc_mamba_scan_bwd, conv_part
 * [ndir*B][5D] the per-sequence conv weight / bias partials (reduce with vc_mamba_conv_params).  ckpt
 * required.  The x half of dxz then comes from vc_mamba_dirconv_bwd_gather. */
VC_API int vc_mamba_scan_bwd_fused(int B, int L, int D, int R, int ndir, const float* u, const float* xdbl,
                                   const int* order, const float* xz, const float* conv_w, const float* conv_b,
                                   const float* x_proj_w, const float* dt_w, const float* dt_b, const float* A_log,
                                   const float* Dskip, const float* gate_logits, const float* yp, const float* dyp,
                                   const float* ckpt, float* dpre, float* ddt_lin, float* dxdbl, float* conv_part,
                                   float* dA_log, float* dDskip, float* dgate_logits, float* ws, long ws_floats,
                                   hipStream_t stream);
VC_API int vc_mamba_dirconv_bwd_gather(int B, int L, int D, int ndir, const int* inv_order, const float* conv_w,
                                       const float* dpre, float* dxz, hipStream_t stream);
/* conv1d weight [D,1,4] / bias [D] gradients (overwritten) from vc_mamba_scan_bwd_fused's partials */
VC_API int vc_mamba_conv_params(int B, int D, int ndir, const float* conv_part, float* dconv_w, float* dconv_b,
                                hipStream_t stream);
/* vc_mamba_scan_bwd_params and vc_mamba_conv_params in ONE launch (round 6): dA_log, D, the gate logits and the
 * conv1d weight / bias gradients (all overwritten) from a deferred vc_mamba_scan_bwd_fused's partials (ws) and
 * conv_part; ndir <= 64 */
VC_API int vc_mamba_bwd_params(int B, int D, int ndir, const float* gate_logits, const float* ws, const float* conv_part,
                               float* dA_log, float* dDskip, float* dgate_logits, float* dconv_w, float* dconv_b,
                               hipStream_t stream);

/* ---------------------------------------------------------------- hsiMamba row chains
 * Two projections with a LayerNorm between them for 32-row blocks in one launch (rowchain.hip), fp32:
 * front (Mutimodality_Mamba7.py:651-656, modeling_mamba.py:433): t = x w_embed^T + pos[row % L],
 *   xn = LN(t) (ln_w, ln_b, eps; mean / rstd saved), out = xn w_proj^T   (K0, E, N2 <= 256, % 4 == 0);
 * back (:694-701, modeling_mamba.py:274, :481, Mutimodality_Mamba7.py:985, :1068): ypsum / ysum as
 *   vc_mamba_combine_fwd (bit-identical, ndir <= 10), t2 = ysum w_out^T + residual, g = LN(t2),
 *   out = g w_proj^T + b_proj.  Each replaces 3 / 4 launches of the separate path. */
VC_API int vc_rowchain_front(int rows, int K0, int E, int N2, const float* x, const float* w_embed, const float* pos,
                             int L, float* t, const float* ln_w, const float* ln_b, float eps, float* xn, float* mean,
                             float* rstd, const float* w_proj, float* out, hipStream_t stream);
VC_API int vc_rowchain_back(int B, int L, int D, int ndir, const int* inv_order, const float* gate_logits,
                            const float* yp, const float* xz, float* ypsum, float* ysum, int E, const float* w_out,
                            const float* residual, float* t2, const float* ln_w, const float* ln_b, float eps,
                            float* g, float* mean, float* rstd, int N2, const float* w_proj, const float* b_proj,
                            float* out, hipStream_t stream);

/* Backward chains (same blocking): back_bwd = change_dim's data gradient (dcd w_cd), the ln1 backward
 * (dt = LN grad; per-block dw / db partials into ln_part), out_proj's data gradient and the SiLU(z) gate
 * backward (dyp, the z half of dxz) -- the separate path's vc_gemm + vc_layernorm_bwd_dx + vc_gemm +
 * vc_mamba_gate_bwd; front_bwd = in_proj's data gradient (dxz w_in), the pre_norm backward with the
 * residual gradient (dtt = res + LN grad; partials) and dx = beta dx + dtt w_embed (+ dx_add) (dx and dx_add
 * nullable; dx_add: another branch's share of dx, e.g. computed concurrently on another stream).
 * vc_rowchain_ln_params reduces the partials (size: vc_rowchain_ln_part_floats).  Weight gradients of
 * the projections are separate vc_gemm calls. */
VC_API int vc_rowchain_back_bwd(int rows, int Cout, int E, int D, const float* dcd, const float* w_cd, const float* t2,
                                const float* mean, const float* rstd, const float* ln_w, float* dt, float* ln_part,
                                const float* w_out, const float* xz, const float* ypsum, float* dyp, float* dxz,
                                hipStream_t stream);
VC_API int vc_rowchain_front_bwd(int rows, int K0, int E, int Cin, const float* dxz, const float* w_in, const float* t,
                                 const float* mean, const float* rstd, const float* ln_w, const float* res, float* dtt,
                                 float* ln_part, const float* w_embed, float* dx, float beta, const float* dx_add,
                                 hipStream_t stream);
VC_API int vc_rowchain_ln_params(int rows, int E, const float* ln_part, float* dw, float* db, float beta,
                                 hipStream_t stream);
VC_API int vc_rowchain_ln_part_floats(int rows, int E);

/* ---------------------------------------------------------------- TokenLearner
 * TokenLearner(S) of SpatialAttention (Mutimodality_Mamba7.py:26-64) over x [B*HW, C] channels-last
 * (C % 4 == 0, ldx % 4 == 0, x / dZ 16-B aligned; HW, S within the LDS plans: vc_tl_check).  params: S x 5
 * floats [conv.0.weight(2),
 * conv.0.bias, conv.1.weight, conv.1.bias]; bn_buffers: S x 2 [running_mean, running_var]; stats: 2 S + 8
 * fp64 -- per token [mean, invstd] of its BN(1) input, then the shared moments of the pooled (max, mean)
 * pair [n, mbar, vbar, Cmm, Cmv, Cvv, Km, Kv] -- kept for the backward (statistics and gradient sums in
 * fp64, as torch's CPU BatchNorm accumulates); ws: vc_tl_ws_floats(B, HW, S) floats of per-call-site
 * scratch (8-B aligned).  vc_tl_pixel_stats leaves the moment partials in ws for vc_tl_fwd. */
VC_API int vc_tl_ws_floats(int B, int HW, int S);
/* 0 when vc_tl_pixel_stats / vc_tl_fwd / vc_tl_bwd support the shape (C <= 512; the tokens of the forward and the
 * pixels of the backward are chunked so their LDS fits: up to 20 x 20 pixel grids with S = 18 x 18 tokens),
 * 1 otherwise.  Host-only (no HIP call). */
VC_API int vc_tl_check(int HW, int C, int S);
/* per pixel row of x [M, C] (C <= 512): channel max, its first argmax, channel mean; + moment partials */
VC_API int vc_tl_pixel_stats(long M, int C, const float* x, long ldx, float* mx, int* amx, float* avg, double* ws,
                             hipStream_t stream);
/* stats (train: batch statistics from the moments, running statistics updated; eval: the running ones),
 * the attention maps a [B, S, HW] (may be null when no backward follows) and the pooled tokens Z [B, S, C] =
 * (1/HW) a x, in one launch */
VC_API int vc_tl_fwd(int train, int B, int HW, int C, int S, const float* x, long ldx, const float* mx,
                     const float* avg, const float* params, float* bn_buffers, float eps, float momentum,
                     const double* ws, double* stats, float* a, float* Z, hipStream_t stream);
/* backward from dZ [B, S, C]: dx [B*HW, C] (ld lddx, overwritten) = (1/HW) a^T dZ + the pooled-path gradient
 * (argmax channel and mean), dparams (S x 5, overwritten); a = the attention maps vc_tl_fwd wrote (round 6: the
 * backward reads them instead of recomputing them; the round-5 `da` scratch argument is gone).  Two launches. */
VC_API int vc_tl_bwd(int train, int B, int HW, int C, int S, const float* x, long ldx, const float* mx,
                     const float* avg, const int* amx, const float* params, const double* stats, const float* a,
                     const float* dZ, double* ws, float* dx, long lddx, float* dparams, hipStream_t stream);
/* mask [B, S, HW] uint8 = the ReLU decisions (BN(1) output > 0) vc_tl_fwd / vc_tl_bwd take, from the
 * same stats (test instrumentation: the float64 parity yardstick follows the HIP path's fp32 ties) */
VC_API int vc_tl_relu_mask(int B, int HW, int S, const float* mx, const float* avg, const float* params,
                           const double* stats, unsigned char* mask, hipStream_t stream);

/* ---------------------------------------------------------------- non-local cross attention
 * NONLocalBlock2D core (Mutimodality_Mamba7.py:143-152): softmax(theta phi^T) g, no scaling.
 * theta [B*S, Ci]; pooled [B*P, 2Ci] = maxpooled phi | g; att [B,S,P] saved; o [B*S, Ci]. */
VC_API int vc_nonlocal_attn_fwd(int B, int S, int P, int Ci, const float* theta, const float* pooled, float* att,
                                float* o, hipStream_t stream);
VC_API int vc_nonlocal_attn_bwd(int B, int S, int P, int Ci, const float* theta, const float* pooled,
                                const float* att, const float* dout, float* dtheta, float* dpooled,
                                hipStream_t stream);

/* ---------------------------------------------------------------- fusion glue, head, loss, optimiser */
/* torch.concat((x1, x2), 1) with ChannelExchange (even channels swapped) when exchange=1
 * (fusionBlock, Mutimodality_Mamba7.py:1133-1136; exchange semantics inferred) */
VC_API int vc_cat2_fwd(long M, int C1, int C2, const float* x1, long ld1, const float* x2, long ld2, int exchange,
                       float* out, hipStream_t stream);
VC_API int vc_cat2_bwd(long M, int C1, int C2, const float* dout, int exchange, float* dx1, long ld1, float beta1,
                       float* dx2, long ld2, float beta2, hipStream_t stream);
/* GLfusionBlock (:1112-1115 with NonLocal's W_y + z, :155-156): out [M, 2C] =
 * [ (BN(w_pre) + fc) + fl | fl + fc ] */
VC_API int vc_glf_combine_fwd(long M, int C, const float* w_pre, const float* bn_mean, const float* bn_invstd,
                              const float* bn_w, const float* bn_b, const float* fc, const float* fl, float* out,
                              hipStream_t stream);
/* train-mode BatchNorm statistics of w_pre (as vc_bn_stats_ex: save_* and running stats written) +
 * vc_glf_combine_fwd, the statistics' final reduction inside the combine launch */
VC_API int vc_bn_glf_combine(long M, int C, const float* w_pre, float eps, float momentum, float* save_mean,
                             float* save_invstd, float* run_mean, float* run_var, const float* bn_w, const float* bn_b,
                             const float* fc, const float* fl, float* out, float* ws, long ws_floats,
                             hipStream_t stream);
/* out = beta*out + a (+ b) over [M, C] strided rows */
VC_API int vc_add2_2d(long M, int C, const float* a, long lda, const float* b, long ldb, float* out, long ldo,
                      float beta, hipStream_t stream);
/* out = out2 = a + b, both overwritten (GLfusionBlock :1112-1115: the concat gradient summed into the
 * local- and channel-feature accumulators in one launch) */
VC_API int vc_add2_2d_dup(long M, int C, const float* a, long lda, const float* b, long ldb, float* out, long ldo,
                          float* out2, long ldo2, hipStream_t stream);
/* avgpool(f1) + avgpool(f2) -> feat [B,C]; logits = feat W^T + bias (Mutimodality_Mamba7.py:1174-1178) */
VC_API int vc_head_fwd(int B, int S1, int S2, int C, int ncls, const float* f1, const float* f2, const float* W,
                       const float* bias, float* feat, float* logits, hipStream_t stream);
VC_API int vc_head_bwd(int B, int S1, int S2, int C, int ncls, const float* dlogits, const float* W,
                       const float* feat, float* df1, float* df2, float* dW, float* db, hipStream_t stream);
/* nn.CrossEntropyLoss(weight) mean (model_utils.py:311): target int64, weight may be null */
VC_API int vc_ce_fwd(int B, int ncls, const float* logits, const long long* target, const float* weight,
                     long long ignore_index, float* loss, hipStream_t stream);
VC_API int vc_ce_bwd(int B, int ncls, const float* logits, const long long* target, const float* weight,
                     long long ignore_index, const float* grad_out, float* dlogits, hipStream_t stream);
/* vc_ce_fwd then vc_ce_bwd with grad_out = 1 in ONE launch (bit-identical to the two): the training step's
 * loss and dlogits */
VC_API int vc_ce_fwd_bwd(int B, int ncls, const float* logits, const long long* target, const float* weight,
                         long long ignore_index, float* loss, float* dlogits, hipStream_t stream);
/* torch.optim.AdamW step (model_utils.py:309-310) over a flat buffer; hyper = device
 * [lr, beta1, beta2, eps, weight_decay, grad_scale]; step = device float[3] state: step[0] = t is
 * incremented first, step[1..2] receive the bias corrections (1 - beta1^t, sqrt(1 - beta2^t)) */
VC_API int vc_adamw(long n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq,
                    const float* hyper, float* step, hipStream_t stream);
/* ptr[idx[i]] += val  (BatchNorm num_batches_tracked counters) */
VC_API int vc_index_add_i64(int n, const int* idx, long long* ptr, long long val, hipStream_t stream);
/* dx = dy * (y > 0)  (nn.ReLU backward from the saved output) */
VC_API int vc_relu_bwd(long n, const float* dy, const float* y, float* dx, hipStream_t stream);
VC_API int vc_fill(long n, float* ptr, float value, hipStream_t stream);
/* ptr[m * ld + c] = value over [M, C] strided rows (e.g. the padding columns of a channel concat) */
VC_API int vc_fill_2d(long M, int C, float* ptr, long ld, float value, hipStream_t stream);
/* ptr[idx[i]] = value  (the alignment gaps of the flat gradient: parameters start 16-B aligned) */
VC_API int vc_fill_index(int n, const int* idx, float* ptr, float value, hipStream_t stream);

/* ---------------------------------------------------------------- patch windows (callers of the step)
 * The reference cuts patches on the host: MultiModalX.__getitem__ (datasets.py:550-593) for
 * training batches and sliding_window/grouper + np.copy for whole-image inference
 * (utils.py:357-415, :567-582; model_utils.py:1067-1132).  Here the image cube stays resident in
 * HBM in its source layout, img[x][y][c] ([W][H][C], band-contiguous, fp32), and windows are
 * gathered on the device straight into the model's [n][C][P][P] input layout.
 *
 * Window i's top-left corner: corners != NULL -> (corners[2i], corners[2i+1]);
 * corners == NULL -> the (k0+i)-th window of sliding_window(step, (P,P)), row-major over
 * (x outer, y inner) with the reference's clamping of the last window to W-P / H-P.
 * xform (optional, training augmentation of datasets.py:511-526): bit0 = np.fliplr, bit1 = np.flipud
 * (applied in that order), bits 2-3 = k of np.rot90(patch, k) (applied when no flip bit is set). */
VC_API int vc_window_count(int W, int H, int P, int step, long* count);
VC_API int vc_patch_gather(int W, int H, int C, int P, const float* cube, const int* corners, long k0, int step,
                           int n, const unsigned char* xform, float* out, hipStream_t stream);
/* probs[(x + P/2) * H + (y + P/2)][c] += (double)logits[i][c] for each window i (center_pixel
 * mode of model_utils.py:1126-1128; windows are distinct, so no two i share a centre) */
VC_API int vc_center_accumulate(int W, int H, int P, int ncls, const int* corners, long k0, int step, int n,
                                const float* logits, double* probs, hipStream_t stream);
/* MultiModalX radiation / mixture noise (datasets.py:529-545, applied at :565-568 to the HSI patch
 * after flip / rot90), in place on gathered patches x [n][C][P][P]:
 *   rad[i] != 0:  x = rad[i] * x + N/25                                   (radiation_noise)
 *   mix[2i] > 0:  x = (a1 * x + a2 * d2) / (a1 + a2) + N/25, (a1, a2) = mix[2i..2i+1]  (mixture_noise)
 * d2[c][p] = cube[pix[off[v] + r]][c], v = (int)lab[i][p] the (transformed) label window, r uniform in
 * [0, off[v+1] - off[v]) per (sample, pixel) -- the reference's np.random.choice over the samples of
 * class v; an empty class (ignored labels) leaves d2 = 0.  pix: x * H + y pixel indices of the cube.
 * N: standard normals and r from a counter-based hash of (seed, gid0 + i, stream, element) -- the
 * host draws the per-sample decisions and alphas in the reference's RNG order; the per-element fields
 * are drawn on the device. */
VC_API int vc_patch_noise(int n, int C, int P, int H, float* x, const float* lab, const float* rad,
                          const float* mix, const int* off, const int* pix, int nlab, const float* cube,
                          unsigned long long seed, long long gid0, hipStream_t stream);

/* ---------------------------------------------------------------- classification metrics
 * Confusion matrix of a prediction map (utils.py:585-663 metrics(), counting step :596-611):
 * cm[t * n_classes + p] += number of pixels with target t, prediction p, both in
 * [0, n_classes), target not flagged in ignored[n_classes] (uint8).  cm (uint64) is
 * accumulated into: zero it first.  n_classes <= 64. */
VC_API int vc_confusion_matrix(long n, const long long* target, const long long* pred, int n_classes,
                               const unsigned char* ignored, unsigned long long* cm, hipStream_t stream);

/* ---------------------------------------------------------------- S2EFT (config 5)
 * model/compare_method/S2EFT.py.  Token rows are [B, T, D] row-major, T = N + 1 (cls first).
 * vc_s2eft_gate_fwd: spectral gate :134-143 (x [B,N,C]; w = conv1d weight [1,2,7] (mean, max),
 *   bias [1]): mask[b,t] = sigmoid(conv1d_k7_pad3([mean_c x, max_c x]))[t] >= beta; xg = x * mask
 *   (the reference thresholds `.data`: no gradient reaches the gate).
 * vc_s2eft_cls_rows: X[b,0,:] = cls + pos[0] (:150-152); vc_s2eft_strip_cls: dE = dX[:,1:,:].
 * vc_s2eft_attn_fwd/bwd: Attention :45-74 core, dim_head 16, softmax(q k^T * scale) v over
 *   qkv [B*T, 3*H*16] (to_qkv output, q|k|v blocks); out [B*T, H*16]; lse [B,H,T] saved; T <= 256.
 * vc_gelu_fwd/bwd: nn.GELU (erf form, FeedForward :25).
 * vc_s2eft_skip_pack/unpack/bias_grad: CAF skipcat Conv2d(T, T, [1,2]) (:88-106) as a GEMM with the
 *   weight viewed [T, 2T] over Z[b] = interleave(x, last) [2T, D]; biasmat [T, D] = bias broadcast. */
VC_API int vc_s2eft_gate_fwd(int B, int N, int C, const float* x, const float* w, const float* bias, float beta,
                             float* xg, float* mask, hipStream_t stream);
VC_API int vc_s2eft_cls_rows(int B, int T, int D, const float* cls, const float* pos, float* X, hipStream_t stream);
VC_API int vc_s2eft_strip_cls(int B, int N, int D, const float* dX, float* dE, hipStream_t stream);
VC_API int vc_s2eft_attn_fwd(int B, int T, int H, const float* qkv, float scale, float* out, float* lse,
                             hipStream_t stream);
VC_API int vc_s2eft_attn_bwd(int B, int T, int H, const float* qkv, const float* out, const float* dout,
                             const float* lse, float scale, float* dqkv, hipStream_t stream);
VC_API int vc_gelu_fwd(long n, const float* x, float* y, hipStream_t stream);
VC_API int vc_gelu_bwd(long n, const float* dy, const float* x, float* dx, hipStream_t stream);
VC_API int vc_s2eft_skip_pack(int B, int T, int D, const float* x, const float* last, const float* bias, float* Z,
                              float* biasmat, hipStream_t stream);
/* the skipcat backward's split of dZ [B, T, 2, D]: dx = (acc_x ? dx : 0) + dZ[:, :, 0] (+ addx, may be null: a
 * residual gradient folded in), dlast = dZ[:, :, 1] (overwritten, round 6: each layer's is written once) */
VC_API int vc_s2eft_skip_unpack(int B, int T, int D, const float* dZ, float* dx, int acc_x, const float* addx,
                                float* dlast, hipStream_t stream);
VC_API int vc_s2eft_skip_bias_grad(int B, int T, int D, const float* dY, float* db, hipStream_t stream);
/* nn.Dropout(p) in training (S2EFT emb_dropout :120, to_out :43, FeedForward :26, :28):
 * keep = hash(seed, i) >= p (counter-based), y = add + keep * x / (1 - p) (add may be null, y may
 * alias x), mask[i] = keep; backward dx = mask * dy / (1 - p) (dx may alias dy). */
VC_API int vc_dropout_fwd(long n, const float* x, const float* add, float* y, unsigned char* mask, float p,
                          unsigned long long seed, hipStream_t stream);
VC_API int vc_dropout_bwd(long n, const float* dy, const unsigned char* mask, float p, float* dx, hipStream_t stream);

/* ---------------------------------------------------------------- FusAtNet forward (config 5)
 * model/compare_method/FusAtNet.py over channels-last [B,H,W,C] rows.
 * vc_im2col3x3_pad: col[(b,oh,ow), c*9+kh*3+kw] of a 3x3 conv with padding pad (0: ConvUnit_NP :19-27,
 *   1: ConvUnit / Residual units :9-17, :29-62); OH = H + 2 pad - 2; GEMM against weight [O, C*9].
 * vc_mul2_2d: out = a * b elementwise (Mt = spatial_am(x2) * Fhs, Fss = Fm * Am, :178-183).
 * vc_pool_scale: out[b,hw,c] = mean_p pooled[b,p,c] * F[b,hw,c] (AdaptiveAvgPool2d(1) of the spectral
 *   attention map times Fhs, :100-101, :178). */
VC_API int vc_im2col3x3_pad(int B, int H, int W, int C, int pad, const float* x, long ldx, float* col,
                            hipStream_t stream);
VC_API int vc_mul2_2d(long M, int C, const float* a, long lda, const float* b, long ldb, float* out, long ldo,
                      hipStream_t stream);
VC_API int vc_pool_scale(int B, int HW, int HWp, int C, const float* pooled, const float* F, long ldf, float* out,
                         long ldo, hipStream_t stream);
/* backward (out-of-place residual semantics): gradient of vc_im2col3x3_pad
 * (gather form; dx rows of ld lddx, overwritten or accumulated), and of vc_pool_scale
 * (dF += mean_p(pooled) * dout; dpooled[b,p,c] = sum_hw dout*F / HWp). */
VC_API int vc_col2im3x3_pad(int B, int H, int W, int C, int pad, const float* dcol, float* dx, long lddx,
                            int accumulate, hipStream_t stream);
VC_API int vc_pool_scale_bwd(int B, int HW, int HWp, int C, const float* pooled, const float* F, long ldf,
                             const float* dout, long lddo, float* dF, long lddf, float* dpooled, hipStream_t stream);

#endif /* VITCNN_H */
