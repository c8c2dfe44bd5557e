// Fusion glue, classifier head, weighted cross-entropy, fused AdamW and small utilities.
//
//   vc_cat2_*            torch.concat((x1, x2), 1) of fusionBlock with the (inferred)
//                        ChannelExchange folded into the copy (Mutimodality_Mamba7.py:1133-1136)
//   vc_glf_combine_*     GLfusionBlock: localf = (BN(W o) + z) + x2, globalf = x2 + x1,
//                        cat(localf, globalf) (:154-156, :1112-1115)
//   vc_head_*            AdaptiveAvgPool2d(1) of both fusion maps, add, Linear(128 -> ncls) (:1174-1178)
//   vc_ce_*              nn.CrossEntropyLoss(weight) mean reduction (model_utils.py:311, :922)
//   vc_adamw             torch.optim.AdamW step over the flat parameter buffer (model_utils.py:309-310)
#include "common.h"

namespace {

__global__ void cat2_fwd(int total, FastDiv fCt, int C1, const float* __restrict__ x1, long ld1,
                         const float* __restrict__ x2, long ld2, int exchange, float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c;
  const long m = fdivmod(idx, fCt, c);
  float v;
  if (c < C1) v = (exchange && (c & 1) == 0) ? x2[m * ld2 + c] : x1[m * ld1 + c];
  else {
    const int c2 = c - C1;
    v = (exchange && (c2 & 1) == 0) ? x1[m * ld1 + c2] : x2[m * ld2 + c2];
  }
  out[idx] = v;
}

__global__ void cat2_bwd(int total, FastDiv fCm, int C1, int C2, const float* __restrict__ dout, int exchange,
                         float* __restrict__ dx1, long ld1, float beta1, float* __restrict__ dx2, long ld2, float beta2) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c;
  const long m = fdivmod(idx, fCm, c);
  const float* dr = dout + m * (C1 + C2);
  const bool sw = exchange && (c & 1) == 0;
  if (dx1 && c < C1) {
    const float g = sw ? dr[C1 + c] : dr[c];
    float* p = dx1 + m * ld1 + c;
    *p = (beta1 != 0.f ? beta1 * *p : 0.f) + g;
  }
  if (dx2 && c < C2) {
    const float g = sw ? dr[c] : dr[C1 + c];
    float* p = dx2 + m * ld2 + c;
    *p = (beta2 != 0.f ? beta2 * *p : 0.f) + g;
  }
}

__global__ void glf_combine_fwd(int total, FastDiv fC, const float* __restrict__ wpre, const float* __restrict__ mean,
                                const float* __restrict__ invstd, const float* __restrict__ gam,
                                const float* __restrict__ bet, const float* __restrict__ fc,
                                const float* __restrict__ fl, float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int C = fC.div;
  int c;
  const long m = fdivmod(idx, fC, c);
  const float wy = (wpre[idx] - mean[c]) * invstd[c] * gam[c] + bet[c];
  const float z = fc[idx], x2 = fl[idx];
  out[m * 2 * C + c] = (wy + z) + x2;
  out[m * 2 * C + C + c] = x2 + z;
}

__global__ void add2_2d(int total, FastDiv fC, const float* __restrict__ a, long lda, const float* __restrict__ b,
                        long ldb, float* __restrict__ out, long ldo, float beta, float* __restrict__ out2 = nullptr,
                        long ldo2 = 0) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c;
  const long m = fdivmod(idx, fC, c);
  float v = a[m * lda + c];
  if (b) v += b[m * ldb + c];
  float* p = out + m * ldo + c;
  *p = (beta != 0.f ? beta * *p : 0.f) + v;
  if (out2) out2[m * ldo2 + c] = v;
}

// feat[b,c] = mean_p f1[b,p,c] + mean_q f2[b,q,c];  logits = feat W^T + bias   (block per b)
__global__ __launch_bounds__(256) void head_fwd(int S1, int S2, int C, int ncls, const float* __restrict__ f1,
                                                const float* __restrict__ f2, const float* __restrict__ W,
                                                const float* __restrict__ bias, float* __restrict__ feat,
                                                float* __restrict__ logits) {
  extern __shared__ float fs[];  // [C] feat, then [4][64] partials
  float* red = fs + C;
  const int b = blockIdx.x;
  const int cl = threadIdx.x & 63, rg = threadIdx.x >> 6;
  for (int c0 = 0; c0 < C; c0 += 64) {
    const int c = c0 + cl;
    float s1 = 0.f, s2 = 0.f;
    if (c < C) {
      // a thread's first HR rows of each map are loaded before any is summed (one round of dependent
      // HBM loads instead of one per 4 rows; the sums keep the row order), the rest (S > 4 HR) in a loop
      constexpr int HR = 24;
      float v1[HR], v2[HR];
#pragma unroll
      for (int i = 0; i < HR; ++i) {
        const int p = rg + 4 * i;
        v1[i] = p < S1 ? f1[((long)b * S1 + p) * C + c] : 0.f;
        v2[i] = p < S2 ? f2[((long)b * S2 + p) * C + c] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < HR; ++i) {
        if (rg + 4 * i < S1) s1 += v1[i];
        if (rg + 4 * i < S2) s2 += v2[i];
      }
      for (int p = rg + 4 * HR; p < S1; p += 4) s1 += f1[((long)b * S1 + p) * C + c];
      for (int q = rg + 4 * HR; q < S2; q += 4) s2 += f2[((long)b * S2 + q) * C + c];
    }
    red[rg * 64 + cl] = s1 / (float)S1 + s2 / (float)S2;
    __syncthreads();
    if (rg == 0 && c < C) {
      const float v = red[cl] + red[64 + cl] + red[128 + cl] + red[192 + cl];
      fs[c] = v;
      feat[(long)b * C + c] = v;
    }
    __syncthreads();
  }
  // logits: a 16-lane row per class (16 classes per pass), DPP row sums instead of LDS shuffles
  const int g = threadIdx.x >> 4, l = threadIdx.x & 15;
  for (int k0 = 0; k0 < ncls; k0 += 16) {
    const int k = k0 + g;
    float acc = 0.f;
    if (k < ncls)
      for (int c = l; c < C; c += 16) acc += fs[c] * W[(long)k * C + c];
    acc = row16_sum(acc);
    if (l == 0 && k < ncls) logits[(long)b * ncls + k] = acc + bias[k];
  }
}

__device__ __forceinline__ void head_bwd_x(int b, int S1, int S2, int C, int ncls, const float* __restrict__ dlog,
                                           const float* __restrict__ W, float* __restrict__ df1,
                                           float* __restrict__ df2) {
  for (int c = threadIdx.x; c < C; c += 256) {
    float g = 0.f;
    for (int k = 0; k < ncls; ++k) g += dlog[(long)b * ncls + k] * W[(long)k * C + c];
    const float g1 = g / (float)S1, g2 = g / (float)S2;
    for (int p = 0; p < S1; ++p) df1[((long)b * S1 + p) * C + c] = g1;
    for (int q = 0; q < S2; ++q) df2[((long)b * S2 + q) * C + c] = g2;
  }
}

// block (k, y) of the (ncls, ceil((C+1)/64)) weight-gradient tiles: 64 columns x 4 batch groups, fixed-order LDS
// combine; column C is the bias gradient (sum over b of dlogits)
__device__ __forceinline__ void head_bwd_w(int k, int y, int B, int C, int ncls, const float* __restrict__ dlog,
                                           const float* __restrict__ feat, float* __restrict__ dW,
                                           float* __restrict__ db) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, bg = threadIdx.x >> 6;
  const int c = y * 64 + cl;
  float acc = 0.f;
  if (c <= C)
    for (int b = bg; b < B; b += 4) acc += dlog[(long)b * ncls + k] * (c < C ? feat[(long)b * C + c] : 1.f);
  red[bg][cl] = acc;
  __syncthreads();
  if (bg == 0 && c <= C) {
    const float v = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    if (c < C) dW[(long)k * C + c] = v;
    else db[k] = v;
  }
}

// the head backward in one grid: blocks [0, B) the feature gradient of sample b, the rest the classifier's weight
// and bias gradient tiles (independent halves: one launch instead of two on the step's critical chain)
__global__ __launch_bounds__(256) void head_bwd(int B, int S1, int S2, int C, int ncls, const float* __restrict__ dlog,
                                                const float* __restrict__ W, const float* __restrict__ feat,
                                                float* __restrict__ df1, float* __restrict__ df2,
                                                float* __restrict__ dW, float* __restrict__ db) {
  const int bid = blockIdx.x;
  if (bid < B) {
    head_bwd_x(bid, S1, S2, C, ncls, dlog, W, df1, df2);
    return;
  }
  const int t = bid - B;
  head_bwd_w(t % ncls, t / ncls, B, C, ncls, dlog, feat, dW, db);
}

// Weighted cross entropy, every sample at once: one 1024-thread block, a 16-lane row per sample
// (lane l holds logits l, l+16, ...), row max / sum by DPP within the row, the target's logit
// picked from the row's own registers.  64 samples per pass: one global round trip for B <= 64.
// loss = sum_b w[y_b] * (lse_b - logit[b, y_b]) / sum_b w[y_b]   (targets == ignore_index contribute 0)
constexpr int CET = 1024;

__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  return v;
}

// per sample row: max, sum of exp(logit - max) and the target's logit, in every lane of the row
__device__ __forceinline__ void ce_row(const float* __restrict__ lr, int ncls, long long y, int l, float& mx, float& se,
                                       float& ly) {
  mx = -INFINITY;
  float t = 0.f;
  for (int k = l; k < ncls; k += 16) {
    const float v = lr[k];
    mx = fmaxf(mx, v);
    if (k == y) t = v;
  }
  mx = row16_max(mx);
  ly = row16_sum(t);
  se = 0.f;
  for (int k = l; k < ncls; k += 16) se += __expf(lr[k] - mx);
  se = row16_sum(se);
}

__device__ __forceinline__ float block_sum1024(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < CET / 64; ++i) r += red[i];
  __syncthreads();
  return r;
}

__device__ __forceinline__ void ce_fwd_body(int B, int ncls, const float* __restrict__ logits,
                                            const long long* __restrict__ target, const float* __restrict__ w,
                                            long long ignore_index, float* __restrict__ loss, float* red) {
  const int g = threadIdx.x >> 4, l = threadIdx.x & 15;
  float num = 0.f, den = 0.f;
  for (int b = g; b < B; b += CET / 16) {
    const long long y = target[b];
    float mx, se, ly;
    ce_row(logits + (long)b * ncls, ncls, y, l, mx, se, ly);
    if (l == 0 && y != ignore_index) {
      const float wy = w ? w[y] : 1.f;
      num += wy * (logf(se) + mx - ly);
      den += wy;
    }
  }
  num = block_sum1024(num, red);
  den = block_sum1024(den, red);
  if (threadIdx.x == 0) loss[0] = num / den;
}

__global__ __launch_bounds__(CET) void ce_fwd(int B, int ncls, const float* __restrict__ logits,
                                              const long long* __restrict__ target, const float* __restrict__ w,
                                              long long ignore_index, float* __restrict__ loss) {
  __shared__ float red[CET / 64];
  ce_fwd_body(B, ncls, logits, target, w, ignore_index, loss, red);
}

__device__ __forceinline__ void ce_bwd_body(int B, int ncls, const float* __restrict__ logits,
                                            const long long* __restrict__ target, const float* __restrict__ w,
                                            long long ignore_index, const float* __restrict__ gout,
                                            float* __restrict__ dlogits, float* red) {
  float den = 0.f;
  for (int b = threadIdx.x; b < B; b += CET) {
    const long long y = target[b];
    if (y != ignore_index) den += w ? w[y] : 1.f;
  }
  den = block_sum1024(den, red);
  const float gs = (gout ? gout[0] : 1.f) / den;
  const int g = threadIdx.x >> 4, l = threadIdx.x & 15;
  for (int b = g; b < B; b += CET / 16) {
    const long long y = target[b];
    float mx, se, ly;
    ce_row(logits + (long)b * ncls, ncls, y, l, mx, se, ly);
    const float wy = (y == ignore_index) ? 0.f : (w ? w[y] : 1.f);
    const float* lr = logits + (long)b * ncls;
    for (int k = l; k < ncls; k += 16) {
      const float p = __expf(lr[k] - mx) / se;
      dlogits[(long)b * ncls + k] = gs * wy * (p - (k == y ? 1.f : 0.f));
    }
  }
}

__global__ __launch_bounds__(CET) void ce_bwd(int B, int ncls, const float* __restrict__ logits,
                                              const long long* __restrict__ target, const float* __restrict__ w,
                                              long long ignore_index, const float* __restrict__ gout,
                                              float* __restrict__ dlogits) {
  __shared__ float red[CET / 64];
  ce_bwd_body(B, ncls, logits, target, w, ignore_index, gout, dlogits, red);
}

// the loss and its gradient for d(loss) = 1 in one block: ce_fwd's then ce_bwd's code (the same bits as the
// two launches), one dependent launch fewer at the head of the training step's backward
__global__ __launch_bounds__(CET) void ce_fwd_bwd(int B, int ncls, const float* __restrict__ logits,
                                                  const long long* __restrict__ target, const float* __restrict__ w,
                                                  long long ignore_index, float* __restrict__ loss,
                                                  float* __restrict__ dlogits) {
  __shared__ float red[CET / 64];
  ce_fwd_body(B, ncls, logits, target, w, ignore_index, loss, red);
  __syncthreads();   // red reused
  ce_bwd_body(B, ncls, logits, target, w, ignore_index, nullptr, dlogits, red);
}

// step[0] = t (incremented), step[1] = 1 - beta1^t, step[2] = sqrt(1 - beta2^t)
__global__ void step_inc(float* step, const float* __restrict__ hyper) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float t = step[0] + 1.f;
    step[0] = t;
    step[1] = 1.f - powf(hyper[1], t);
    step[2] = sqrtf(1.f - powf(hyper[2], t));
  }
}

struct AdamHyper {
  float lr, b1, b2, eps, wd, gs, bc1, sbc2;
};

__device__ __forceinline__ void adamw_elem(const AdamHyper& h, float& p, float g, float& m, float& v) {
  const float gi = g * h.gs;
  const float pi = p * (1.f - h.lr * h.wd);
  m = m + (gi - m) * (1.f - h.b1);
  v = v * h.b2 + (1.f - h.b2) * gi * gi;
  const float denom = sqrtf(v) / h.sbc2 + h.eps;
  p = pi - (h.lr / h.bc1) * (m / denom);
}

// hyper = [lr, beta1, beta2, eps, weight_decay, grad_scale]; torch.optim.AdamW (amsgrad=False);
// grad_scale folds the 1/world_size of a data-parallel gradient SUM into the update
// 4 elements per thread (16-B loads/stores) over [0, n4*4), scalar tail after
__global__ void adamw(long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                      float* __restrict__ v, const float* __restrict__ hyper, const float* __restrict__ step) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const AdamHyper h{hyper[0], hyper[1], hyper[2], hyper[3], hyper[4], hyper[5], step[1], step[2]};
  const long n4 = n >> 2;
  if (i < n4) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    adamw_elem(h, pv.x, gv.x, mv.x, vv.x);
    adamw_elem(h, pv.y, gv.y, mv.y, vv.y);
    adamw_elem(h, pv.z, gv.z, mv.z, vv.z);
    adamw_elem(h, pv.w, gv.w, mv.w, vv.w);
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
  } else {
    const long j = n4 * 4 + (i - n4);
    if (j < n) adamw_elem(h, p[j], g[j], m[j], v[j]);
  }
}

__global__ void index_add_i64(int n, const int* __restrict__ idx, long long* __restrict__ ptr, long long val) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ptr[idx[i]] += val;
}

__global__ void relu_bwd(long n, const float* __restrict__ dy, const float* __restrict__ y, float* __restrict__ dx) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dx[i] = y[i] > 0.f ? dy[i] : 0.f;
}

__global__ void fill_f32(long n, float* __restrict__ p, float v) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void fill2d_f32(long M, int C, float* __restrict__ p, long ld, float v) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < M * C) p[(i / C) * ld + i % C] = v;
}

__global__ void fill_index_f32(int n, const int* __restrict__ idx, float* __restrict__ p, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[idx[i]] = v;
}

}  // namespace

VC_API int vc_cat2_fwd(long M, int C1, int C2, const float* x1, long ld1, const float* x2, long ld2, int exchange,
                       float* out, hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C1 > 0 && C2 > 0 && (!exchange || C1 == C2));
  if (M == 0) return VC_OK;
  VC_REQUIRE_I32(M * (C1 + C2));
  hipLaunchKernelGGL(cat2_fwd, dim3(vc_cdiv(M * (C1 + C2), 256)), dim3(256), 0, stream, (int)(M * (C1 + C2)),
                     make_fastdiv(C1 + C2), C1, x1, ld1, x2, ld2, exchange, out);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_cat2_bwd(long M, int C1, int C2, const float* dout, int exchange, float* dx1, long ld1, float beta1,
                       float* dx2, long ld2, float beta2, hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C1 > 0 && C2 > 0 && (!exchange || C1 == C2));
  if (M == 0) return VC_OK;
  const int Cm = C1 > C2 ? C1 : C2;
  VC_REQUIRE_I32(M * (C1 + C2));
  hipLaunchKernelGGL(cat2_bwd, dim3(vc_cdiv(M * Cm, 256)), dim3(256), 0, stream, (int)(M * Cm), make_fastdiv(Cm), C1,
                     C2, dout, exchange, dx1, ld1, beta1, dx2, ld2, beta2);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_glf_combine_fwd(long M, int C, const float* w_pre, const float* bn_mean, const float* bn_invstd,
                              const float* bn_w, const float* bn_b, const float* fc, const float* fl, float* out,
                              hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C > 0);
  if (M == 0) return VC_OK;
  VC_REQUIRE_I32(M * 2 * C);
  hipLaunchKernelGGL(glf_combine_fwd, dim3(vc_cdiv(M * C, 256)), dim3(256), 0, stream, (int)(M * C), make_fastdiv(C),
                     w_pre, bn_mean, bn_invstd, bn_w, bn_b, fc, fl, out);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// out = beta*out + a (+ b)
VC_API int vc_add2_2d(long M, int C, const float* a, long lda, const float* b, long ldb, float* out, long ldo,
                      float beta, hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C > 0);
  if (M == 0) return VC_OK;
  VC_REQUIRE_I32(M * C);
  hipLaunchKernelGGL(add2_2d, dim3(vc_cdiv(M * C, 256)), dim3(256), 0, stream, (int)(M * C), make_fastdiv(C), a, lda,
                     b, ldb, out, ldo, beta);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// out = out2 = a + b (both overwritten): the GLfusion FusionLayer's concat gradient summed into the two
// accumulators its consumers add to (Mutimodality_Mamba7.py:1112-1115), one launch instead of add + copy
VC_API int vc_add2_2d_dup(long M, int C, const float* a, long lda, const float* b, long ldb, float* out, long ldo,
                          float* out2, long ldo2, hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C > 0 && out2 != nullptr);
  if (M == 0) return VC_OK;
  VC_REQUIRE_I32(M * C);
  hipLaunchKernelGGL(add2_2d, dim3(vc_cdiv(M * C, 256)), dim3(256), 0, stream, (int)(M * C), make_fastdiv(C), a, lda,
                     b, ldb, out, ldo, 0.f, out2, ldo2);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_head_fwd(int B, int S1, int S2, int C, int ncls, const float* f1, const float* f2, const float* W,
                       const float* bias, float* feat, float* logits, hipStream_t stream) {
  VC_REQUIRE(B > 0 && S1 > 0 && S2 > 0 && C > 0 && ncls > 0);
  hipLaunchKernelGGL(head_fwd, dim3(B), dim3(256), sizeof(float) * (C + 256), stream, S1, S2, C, ncls, f1, f2, W,
                     bias, feat, logits);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_head_bwd(int B, int S1, int S2, int C, int ncls, const float* dlogits, const float* W, const float* feat,
                       float* df1, float* df2, float* dW, float* db, hipStream_t stream) {
  VC_REQUIRE(B > 0 && S1 > 0 && S2 > 0 && C > 0 && ncls > 0);
  hipLaunchKernelGGL(head_bwd, dim3(B + ncls * vc_cdiv(C + 1, 64)), dim3(256), 0, stream, B, S1, S2, C, ncls, dlogits,
                     W, feat, df1, df2, dW, db);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_ce_fwd(int B, int ncls, const float* logits, const long long* target, const float* weight,
                     long long ignore_index, float* loss, hipStream_t stream) {
  VC_REQUIRE(B > 0 && ncls > 0);
  hipLaunchKernelGGL(ce_fwd, dim3(1), dim3(CET), 0, stream, B, ncls, logits, target, weight, ignore_index, loss);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_ce_bwd(int B, int ncls, const float* logits, const long long* target, const float* weight,
                     long long ignore_index, const float* grad_out, float* dlogits, hipStream_t stream) {
  VC_REQUIRE(B > 0 && ncls > 0);
  hipLaunchKernelGGL(ce_bwd, dim3(1), dim3(CET), 0, stream, B, ncls, logits, target, weight, ignore_index, grad_out,
                     dlogits);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_ce_fwd_bwd(int B, int ncls, const float* logits, const long long* target, const float* weight,
                         long long ignore_index, float* loss, float* dlogits, hipStream_t stream) {
  VC_REQUIRE(B > 0 && ncls > 0 && loss && dlogits);
  hipLaunchKernelGGL(ce_fwd_bwd, dim3(1), dim3(CET), 0, stream, B, ncls, logits, target, weight, ignore_index, loss,
                     dlogits);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// step += 1 on device, then one fused AdamW update over n elements (graph-replay safe: the
// step count and hyper-parameters live in device memory)
VC_API int vc_adamw(long n, float* params, const float* grads, float* exp_avg, float* exp_avg_sq, const float* hyper,
                    float* step, hipStream_t stream) {
  VC_REQUIRE(n >= 0);
  VC_REQUIRE(((uintptr_t)params | (uintptr_t)grads | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0);
  hipLaunchKernelGGL(step_inc, dim3(1), dim3(64), 0, stream, step, hyper);
  VC_CHECK_LAUNCH();
  if (n == 0) return VC_OK;
  const long threads = (n >> 2) + (n & 3);
  hipLaunchKernelGGL(adamw, dim3(vc_cdiv(threads, 256)), dim3(256), 0, stream, n, params, grads, exp_avg, exp_avg_sq,
                     hyper, step);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_index_add_i64(int n, const int* idx, long long* ptr, long long val, hipStream_t stream) {
  VC_REQUIRE(n >= 0);
  if (n == 0) return VC_OK;
  hipLaunchKernelGGL(index_add_i64, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, n, idx, ptr, val);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_relu_bwd(long n, const float* dy, const float* y, float* dx, hipStream_t stream) {
  VC_REQUIRE(n >= 0);
  if (n == 0) return VC_OK;
  hipLaunchKernelGGL(relu_bwd, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, n, dy, y, dx);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_fill_index(int n, const int* idx, float* ptr, float value, hipStream_t stream) {
  VC_REQUIRE(n >= 0);
  if (n == 0) return VC_OK;
  hipLaunchKernelGGL(fill_index_f32, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, n, idx, ptr, value);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_fill_2d(long M, int C, float* ptr, long ld, float value, hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C >= 0 && ld >= C && ptr);
  if (M == 0 || C == 0) return VC_OK;
  hipLaunchKernelGGL(fill2d_f32, dim3(vc_cdiv(M * C, 256)), dim3(256), 0, stream, M, C, ptr, ld, value);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_fill(long n, float* ptr, float value, hipStream_t stream) {
  VC_REQUIRE(n >= 0);
  if (n == 0) return VC_OK;
  hipLaunchKernelGGL(fill_f32, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, n, ptr, value);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
