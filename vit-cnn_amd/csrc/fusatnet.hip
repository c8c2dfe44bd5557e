// FusAtNet comparison model (config 5), forward: the ops the existing
// kernels (vc_gemm, vc_bn_*, vc_maxpool2_fwd, vc_add2_2d) do not cover.
// Reference: model/compare_method/FusAtNet.py (ConvUnit :9-17 3x3 pad 1, ConvUnit_NP :19-27 valid,
// Spectral_Attention_Module :85-101 maxpool + AdaptiveAvgPool2d(1), FusAtNet.forward :176-184 products).
// Activations are channels-last [B, H, W, C] rows.
#include "common.h"

namespace {

// col[(b, oh, ow), c*9 + kh*3 + kw] = x[b, oh + kh - pad, ow + kw - pad, c] (zero outside), OH = H + 2 pad - 2.
// One thread per col element, so a wave's stores are 64 consecutive floats (the col matrix is the
// dominant write: up to 611 MB for the 2193-channel concat at B = 64); the nine lanes that share a
// channel read neighbouring pixels of one x row (cache hits).
__global__ void im2col3x3_pad(int total, FastDiv f9C, FastDiv fOW, FastDiv fOH, int H, int W, int pad,
                              const float* __restrict__ x, long ldx, float* __restrict__ col) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int j;
  const int row = fdivmod(idx, f9C, j);
  const int c = j / 9, k = j - c * 9;
  const int kh = k / 3, kw = k - kh * 3;
  int ow, oh;
  const int r2 = fdivmod(row, fOW, ow);
  const int b = fdivmod(r2, fOH, oh);
  const int ih = oh + kh - pad, iw = ow + kw - pad;
  float v = 0.f;
  if (ih >= 0 && ih < H && iw >= 0 && iw < W) v = x[((long)(b * H + ih) * W + iw) * ldx + c];
  col[idx] = v;
}

// out[m, c] = a[m, c] * b[m, c]  (strided rows)
__global__ void mul2_2d(int total, FastDiv fC, const float* __restrict__ a, long lda, const float* __restrict__ b,
                        long ldb, float* __restrict__ out, long ldo) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c;
  const long m = fdivmod(idx, fC, c);
  out[m * ldo + c] = a[m * lda + c] * b[m * ldb + c];
}

// the same with 4 consecutive channels per thread (C, the leading dimensions and the bases 16-B aligned)
__global__ void mul2_2d_v4(int total4, FastDiv fC4, const float* __restrict__ a, long lda, const float* __restrict__ b,
                           long ldb, float* __restrict__ out, long ldo) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total4) return;
  int c4;
  const long m = fdivmod(idx, fC4, c4);
  const float4 x = *reinterpret_cast<const float4*>(a + m * lda + 4 * c4);
  const float4 y = *reinterpret_cast<const float4*>(b + m * ldb + 4 * c4);
  *reinterpret_cast<float4*>(out + m * ldo + 4 * c4) = make_float4(x.x * y.x, x.y * y.y, x.z * y.z, x.w * y.w);
}

// out[b, hw, c] = mean_{p < HWp} pooled[b, p, c] * F[b, hw, c]   (AdaptiveAvgPool2d(1) then broadcast product)
__global__ void pool_scale(int total, FastDiv fC, FastDiv fHW, int HWp, const float* __restrict__ pooled,
                           const float* __restrict__ F, long ldf, float* __restrict__ out, long ldo) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c, hw;
  const int m = fdivmod(idx, fC, c);
  const int b = fdivmod(m, fHW, hw);
  const int C = (int)fC.div;
  float s = 0.f;
  for (int p = 0; p < HWp; ++p) s += pooled[((long)b * HWp + p) * C + c];
  out[(long)m * ldo + c] = (s / (float)HWp) * F[(long)m * ldf + c];
}

// gradient of im2col3x3_pad, gather form: dx[b, ih, iw, c] (= or +=) sum over taps of dcol
__global__ void col2im3x3_pad(int total, FastDiv fC, FastDiv fW, FastDiv fH, int pad, const float* __restrict__ dcol,
                              float* __restrict__ dx, long lddx, int accumulate) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c, iw, ih;
  const int p = fdivmod(idx, fC, c);
  const int q = fdivmod(p, fW, iw);
  const int b = fdivmod(q, fH, ih);
  const int C = (int)fC.div, H = (int)fH.div, W = (int)fW.div;
  const int OH = H + 2 * pad - 2, OW = W + 2 * pad - 2;
  float v = 0.f;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int oh = ih - kh + pad;
    if (oh < 0 || oh >= OH) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int ow = iw - kw + pad;
      if (ow < 0 || ow >= OW) continue;
      v += dcol[((long)(b * OH + oh) * OW + ow) * C * 9 + c * 9 + kh * 3 + kw];
    }
  }
  float* o = dx + (long)p * lddx + c;
  *o = accumulate ? *o + v : v;
}

// backward of pool_scale: one thread per (b, c): s = mean_p pooled; dF (+)= s * dout; dpooled = sum_hw dout*F / HWp
// block = (64 channels, sample b) x PS_RL row lanes over the HW pixels (8 pixels' loads in flight per lane);
// the lanes' ds partials summed in lane order through LDS (fixed order)
constexpr int PS_RL = 8;
__global__ __launch_bounds__(64 * PS_RL) void pool_scale_bwd(int B, int HW, int HWp, int C,
                                                            const float* __restrict__ pooled,
                                                            const float* __restrict__ F, long ldf,
                                                            const float* __restrict__ dout, long lddo,
                                                            float* __restrict__ dF, long lddf,
                                                            float* __restrict__ dpooled) {
  __shared__ float sh[PS_RL][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, b = blockIdx.y;
  float ds = 0.f;
  if (c < C) {
    float s = 0.f;
    for (int p = 0; p < HWp; ++p) s += pooled[((long)b * HWp + p) * C + c];
    s /= (float)HWp;
    constexpr int NBH = 8;
    for (int h0 = rl; h0 < HW; h0 += PS_RL * NBH) {
      float g[NBH], f[NBH], d[NBH];
#pragma unroll
      for (int i = 0; i < NBH; ++i) {
        const int hw = h0 + PS_RL * i;
        const long m = (long)b * HW + (hw < HW ? hw : 0);
        const bool ok = hw < HW;
        g[i] = ok ? dout[m * lddo + c] : 0.f;
        f[i] = ok ? F[m * ldf + c] : 0.f;
        d[i] = ok ? dF[m * lddf + c] : 0.f;
      }
#pragma unroll
      for (int i = 0; i < NBH; ++i) {
        const int hw = h0 + PS_RL * i;
        if (hw < HW) {
          ds += g[i] * f[i];
          dF[((long)b * HW + hw) * lddf + c] = d[i] + s * g[i];
        }
      }
    }
  }
  sh[rl][cl] = ds;
  __syncthreads();
  if (rl == 0 && c < C) {
    float t = sh[0][cl];
#pragma unroll
    for (int l = 1; l < PS_RL; ++l) t += sh[l][cl];
    for (int p = 0; p < HWp; ++p) dpooled[((long)b * HWp + p) * C + c] = t / (float)HWp;
  }
}

}  // namespace

VC_API int vc_col2im3x3_pad(int B, int H, int W, int C, int pad, const float* dcol, float* dx, long lddx,
                            int accumulate, hipStream_t stream) {
  VC_REQUIRE(B > 0 && C > 0 && (pad == 0 || pad == 1) && lddx >= C && H + 2 * pad - 2 > 0 && W + 2 * pad - 2 > 0);
  const long total = (long)B * H * W * C;
  VC_REQUIRE_I32(total);
  hipLaunchKernelGGL(col2im3x3_pad, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total, make_fastdiv(C),
                     make_fastdiv(W), make_fastdiv(H), pad, dcol, dx, lddx, accumulate);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_pool_scale_bwd(int B, int HW, int HWp, int C, const float* pooled, const float* F, long ldf,
                             const float* dout, long lddo, float* dF, long lddf, float* dpooled, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && HWp > 0 && C > 0);
  VC_REQUIRE(B < 65536);
  hipLaunchKernelGGL(pool_scale_bwd, dim3(vc_cdiv(C, 64), B), dim3(64 * PS_RL), 0, stream, B, HW, HWp, C, pooled, F,
                     ldf, dout, lddo, dF, lddf, dpooled);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_im2col3x3_pad(int B, int H, int W, int C, int pad, const float* x, long ldx, float* col,
                            hipStream_t stream) {
  VC_REQUIRE(B > 0 && C > 0 && (pad == 0 || pad == 1) && ldx >= C);
  const int OH = H + 2 * pad - 2, OW = W + 2 * pad - 2;
  VC_REQUIRE(OH > 0 && OW > 0);
  const long total = (long)B * OH * OW * C * 9;
  VC_REQUIRE_I32(total);
  hipLaunchKernelGGL(im2col3x3_pad, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total, make_fastdiv(9 * C),
                     make_fastdiv(OW), make_fastdiv(OH), H, W, pad, x, ldx, col);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_mul2_2d(long M, int C, const float* a, long lda, const float* b, long ldb, float* out, long ldo,
                      hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C > 0);
  if (M == 0) return VC_OK;
  VC_REQUIRE_I32(M * C);
  const bool v4 = C % 4 == 0 && lda % 4 == 0 && ldb % 4 == 0 && ldo % 4 == 0 && ((uintptr_t)a % 16) == 0 &&
                  ((uintptr_t)b % 16) == 0 && ((uintptr_t)out % 16) == 0;
  if (v4)
    hipLaunchKernelGGL(mul2_2d_v4, dim3(vc_cdiv(M * C / 4, 256)), dim3(256), 0, stream, (int)(M * C / 4),
                       make_fastdiv(C / 4), a, lda, b, ldb, out, ldo);
  else
    hipLaunchKernelGGL(mul2_2d, dim3(vc_cdiv(M * C, 256)), dim3(256), 0, stream, (int)(M * C), make_fastdiv(C), a,
                       lda, b, ldb, out, ldo);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_pool_scale(int B, int HW, int HWp, int C, const float* pooled, const float* F, long ldf, float* out,
                         long ldo, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && HWp > 0 && C > 0);
  const long total = (long)B * HW * C;
  VC_REQUIRE_I32(total);
  hipLaunchKernelGGL(pool_scale, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total, make_fastdiv(C),
                     make_fastdiv(HW), HWp, pooled, F, ldf, out, ldo);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
