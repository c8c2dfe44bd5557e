// Layout and spatial helpers: NCHW -> channels-last, 3x3 valid im2col with a fused
// BatchNorm affine (ms_conv_bn_relu, Mutimodality_Mamba7.py:1035-1048: BN -> conv3x3 -> ReLU),
// its col2im gradient (gather form, deterministic), and the 2x2 max-pool of the NonLocal
// phi / g branches (nn.MaxPool2d(kernel_size=(2, 2)), :94, :136-138).
//
// im2col column order is (ci, kh, kw) so the reference's conv weight [Co, Ci, 3, 3] is used
// in place as the [Co, 9*Ci] GEMM operand (no repacking of parameters or gradients).
#include "common.h"

namespace {

// y[b][p][c] = x[b][c][p] via 32x32 LDS tiles
__global__ __launch_bounds__(256) void nchw_to_nhwc(int B, int C, int HW, const float* __restrict__ x,
                                                    float* __restrict__ y) {
  __shared__ float t[32][33];
  const int b = blockIdx.z;
  const int c0 = blockIdx.y * 32, p0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 8 rows per pass
  const float* xb = x + (long)b * C * HW;
  for (int i = ty; i < 32; i += 8) {
    int c = c0 + i, p = p0 + tx;
    t[i][tx] = (c < C && p < HW) ? xb[(long)c * HW + p] : 0.f;
  }
  __syncthreads();
  float* yb = y + (long)b * C * HW;
  for (int i = ty; i < 32; i += 8) {
    int p = p0 + i, c = c0 + tx;
    if (p < HW && c < C) yb[(long)p * C + c] = t[tx][i];
  }
}

__global__ void im2col3x3(int total, FastDiv fC, FastDiv fOW, FastDiv fOH, int H, int W,
                          const float* __restrict__ x, const float* __restrict__ mean,
                          const float* __restrict__ invstd, const float* __restrict__ w, const float* __restrict__ b,
                          float* __restrict__ col) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int C = fC.div;
  int c, ow, oh;
  const int m = fdivmod(idx, fC, c);
  const int q = fdivmod(m, fOW, ow);
  const int bb = fdivmod(q, fOH, oh);
  float sc = 1.f, sh = 0.f;
  if (mean) {
    sc = invstd[c] * w[c];
    sh = b[c] - mean[c] * sc;
  }
  float* out = col + (long)m * (9 * C) + 9 * c;
  const float* xb = x + (((long)bb * H + oh) * W + ow) * C + c;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh)
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) out[kh * 3 + kw] = xb[((long)kh * W + kw) * C] * sc + sh;
}

// dx[b,ih,iw,c] = sum_{kh,kw} dcol[(b, ih-kh, iw-kw), c*9 + kh*3 + kw]
__global__ void col2im3x3(int total, FastDiv fC, FastDiv fW, FastDiv fH, const float* __restrict__ dcol,
                          float* __restrict__ dx) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int C = fC.div, H = fH.div, W = fW.div;
  const int OH = H - 2, OW = W - 2;
  int c, iw, ih;
  const int p = fdivmod(idx, fC, c);
  const int q = fdivmod(p, fW, iw);
  const int bb = fdivmod(q, fH, ih);
  float s = 0.f;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const int oh = ih - kh;
    if (oh < 0 || oh >= OH) continue;
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int ow = iw - kw;
      if (ow < 0 || ow >= OW) continue;
      const int m = (bb * OH + oh) * OW + ow;
      s += dcol[(long)m * (9 * C) + 9 * c + kh * 3 + kw];
    }
  }
  dx[idx] = s;
}

// 2x2 / stride 2 floor max-pool over a channels-last [B, H, W, C] (row stride ldx);
// arg = which of the 4 taps won (first max in (kh, kw) scan order, as torch).
__global__ void maxpool2(int total, FastDiv fC, FastDiv fPW, FastDiv fPH, int H, int W, const float* __restrict__ x,
                         long ldx, float* __restrict__ y, unsigned char* __restrict__ arg) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c, pw, ph;
  const int q = fdivmod(idx, fC, c);
  const int r = fdivmod(q, fPW, pw);
  const int bb = fdivmod(r, fPH, ph);
  const float* xb = x + (((long)bb * H + 2 * ph) * W + 2 * pw) * ldx + c;
  float best = xb[0];
  int bi = 0;
#pragma unroll
  for (int t = 1; t < 4; ++t) {
    const float v = xb[((long)(t >> 1) * W + (t & 1)) * ldx];
    if (v > best || isnan(v)) {  // torch: first max in scan order, NaN propagates
      best = v;
      bi = t;
    }
  }
  y[idx] = best;
  arg[idx] = (unsigned char)bi;
}

__global__ void maxpool2_bwd(int total, FastDiv fC, FastDiv fW, FastDiv fH, const float* __restrict__ dy,
                             const unsigned char* __restrict__ arg, float* __restrict__ dx, long lddx) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int C = fC.div, H = fH.div, W = fW.div;
  const int PH = H / 2, PW = W / 2;
  int c, iw, ih;
  const int p = fdivmod(idx, fC, c);
  const int q = fdivmod(p, fW, iw);
  const int bb = fdivmod(q, fH, ih);
  const int ph = ih >> 1, pw = iw >> 1;
  float v = 0.f;
  if (ph < PH && pw < PW) {
    const int q = ((bb * PH + ph) * PW + pw) * C + c;
    if (arg[q] == ((ih & 1) << 1 | (iw & 1))) v = dy[q];
  }
  dx[(long)p * lddx + c] = v;
}

}  // namespace

VC_API int vc_nchw_to_nhwc(int B, int C, int HW, const float* x, float* y, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && C > 0 && HW > 0);
  if (B == 0) return VC_OK;
  hipLaunchKernelGGL(nchw_to_nhwc, dim3(vc_cdiv(HW, 32), vc_cdiv(C, 32), B), dim3(256), 0, stream, B, C, HW, x, y);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_im2col3x3(int B, int H, int W, int C, const float* x, const float* bn_mean, const float* bn_invstd,
                        const float* bn_w, const float* bn_b, float* col, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && H >= 3 && W >= 3 && C > 0);
  long total = (long)B * (H - 2) * (W - 2) * C;
  if (total == 0) return VC_OK;
  VC_REQUIRE_I32(total * 9);
  hipLaunchKernelGGL(im2col3x3, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total, make_fastdiv(C),
                     make_fastdiv(W - 2), make_fastdiv(H - 2), H, W, x, bn_mean, bn_invstd, bn_w, bn_b, col);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_col2im3x3(int B, int H, int W, int C, const float* dcol, float* dx, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && H >= 3 && W >= 3 && C > 0);
  long total = (long)B * H * W * C;
  if (total == 0) return VC_OK;
  VC_REQUIRE_I32(total * 9);
  hipLaunchKernelGGL(col2im3x3, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total, make_fastdiv(C),
                     make_fastdiv(W), make_fastdiv(H), dcol, dx);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_maxpool2_fwd(int B, int H, int W, int C, const float* x, long ldx, float* y, unsigned char* arg,
                           hipStream_t stream) {
  VC_REQUIRE(B >= 0 && H >= 2 && W >= 2 && C > 0 && ldx >= C);
  long total = (long)B * (H / 2) * (W / 2) * C;
  if (total == 0) return VC_OK;
  VC_REQUIRE_I32((long)B * H * W * ldx);
  hipLaunchKernelGGL(maxpool2, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total, make_fastdiv(C),
                     make_fastdiv(W / 2), make_fastdiv(H / 2), H, W, x, ldx, y, arg);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_maxpool2_bwd(int B, int H, int W, int C, const float* dy, const unsigned char* arg, float* dx,
                           long lddx, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && H >= 2 && W >= 2 && C > 0 && lddx >= C);
  long total = (long)B * H * W * C;
  if (total == 0) return VC_OK;
  VC_REQUIRE_I32((long)B * H * W * lddx);
  hipLaunchKernelGGL(maxpool2_bwd, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total, make_fastdiv(C),
                     make_fastdiv(W), make_fastdiv(H), dy, arg, dx, lddx);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
