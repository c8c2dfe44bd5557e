// Layout and spatial helpers: NCHW -> channels-last, 3x3 valid im2col with a fused
// BatchNorm affine (ms_conv_bn_relu, Mutimodality_Mamba7.py:1035-1048: BN -> conv3x3 -> ReLU),
// its col2im gradient (gather form, deterministic), and the 2x2 max-pool of the NonLocal
// phi / g branches (nn.MaxPool2d(kernel_size=(2, 2)), :94, :136-138).
//
// im2col column order is (ci, kh, kw) so the reference's conv weight [Co, Ci, 3, 3] is used
// in place as the [Co, 9*Ci] GEMM operand (no repacking of parameters or gradients).
#include "common.h"

namespace {

// y[b][p][c] = x[b][c][p] via 32x32 LDS tiles; rows of ldy floats, columns C .. ldy - 1 written 0
__global__ __launch_bounds__(256) void nchw_to_nhwc(int B, int C, int HW, const float* __restrict__ x,
                                                    float* __restrict__ y, int ldy) {
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
  float* yb = y + (long)b * ldy * HW;
  for (int i = ty; i < 32; i += 8) {
    int p = p0 + i, c = c0 + tx;
    if (p < HW && c < ldy) yb[(long)p * ldy + c] = t[tx][i];
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

// LDS-staged forms of im2col3x3 / col2im3x3 for one batch element and a chunk of CC channels per block.
// The per-thread forms above touch col rows with a 36-byte lane stride (9 taps per channel); here every
// global access is a run of consecutive floats -- the image chunk [H*W][CC] and the col segments
// [S][9*CC] (S = OH*OW) go through LDS, where the stride-9 channel reads are bank-conflict free (9 odd).
// Same arithmetic and summation order as the per-thread kernels (bit-identical).
constexpr int C2I_T = 512, C2I_W = C2I_T / 64, C2I_CC = 32, C2I_JK = (9 * C2I_CC + 63) / 64;
// LDS pitch of a staged pixel: 33 floats, so a wave's col-row reads (channel j / 9, tap j % 9: taps 32
// floats apart at pitch 32, i.e. 2 banks for 9 taps) spread over the banks
constexpr int C2I_CP = C2I_CC + 1;

__global__ __launch_bounds__(C2I_T) void im2col3x3_lds(int nchunk, int H, int W, int C,
                                                      const float* __restrict__ x, const float* __restrict__ mean,
                                                      const float* __restrict__ invstd, const float* __restrict__ w,
                                                      const float* __restrict__ b, float* __restrict__ col) {
  extern __shared__ float img[];   // [H*W][C2I_CP]
  const int bb = blockIdx.x / nchunk, c0 = (blockIdx.x - bb * nchunk) * C2I_CC, nc = min(C2I_CC, C - c0);
  const int OW = W - 2, S = (H - 2) * OW, HW = H * W;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  {   // stage the chunk: thread -> (pixel i >> 5, channel i & 31), every load of a pass issued together
    const int c = threadIdx.x & (C2I_CC - 1);
    float sc = 1.f, sh = 0.f;
    if (mean && c < nc) {
      sc = invstd[c0 + c] * w[c0 + c];
      sh = b[c0 + c] - mean[c0 + c] * sc;
    }
    const float* xb = x + (long)bb * HW * C + c0 + c;
    constexpr int PP = C2I_T / C2I_CC, NBP = 8;   // pixels per pass, passes batched
    for (int p0 = threadIdx.x / C2I_CC; p0 < HW; p0 += PP * NBP) {
      float v[NBP];
#pragma unroll
      for (int k = 0; k < NBP; ++k) {
        const int p = p0 + k * PP;
        v[k] = (p < HW && c < nc) ? xb[(long)p * C] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < NBP; ++k) {
        const int p = p0 + k * PP;
        if (p < HW) img[p * C2I_CP + c] = v[k] * sc + sh;
      }
    }
  }
  __syncthreads();
  // write: a wave per col row m, lane -> the row segment's floats j = lane + 64 k (fixed per lane, so
  // their (channel, tap) offsets into the staged image are computed once)
  const int seg = 9 * nc;
  int off[C2I_JK];
#pragma unroll
  for (int k = 0; k < C2I_JK; ++k) {
    const int j = lane + 64 * k, c = j / 9, t = j - 9 * c, kh = t / 3, kw = t - 3 * kh;
    off[k] = j < seg ? (kh * W + kw) * C2I_CP + c : -1;
  }
  float* cb = col + (long)bb * S * 9 * C + 9 * c0;
  for (int m = wave; m < S; m += C2I_W) {
    const int oh = m / OW, ow = m - oh * OW, base = (oh * W + ow) * C2I_CP;
    float* row = cb + (long)m * 9 * C;
#pragma unroll
    for (int k = 0; k < C2I_JK; ++k)
      if (off[k] >= 0) row[lane + 64 * k] = img[base + off[k]];
  }
}

__global__ __launch_bounds__(C2I_T) void col2im3x3_lds(int nchunk, int H, int W, int C,
                                                      const float* __restrict__ dcol, float* __restrict__ dx) {
  extern __shared__ float seg_lds[];   // [S][9*C2I_CC]
  constexpr int LD = 9 * C2I_CC, RB = 3;   // rows per wave whose loads are issued together
  const int bb = blockIdx.x / nchunk, c0 = (blockIdx.x - bb * nchunk) * C2I_CC, nc = min(C2I_CC, C - c0);
  const int OH = H - 2, OW = W - 2, S = OH * OW, HW = H * W, seg = 9 * nc;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* db = dcol + (long)bb * S * 9 * C + 9 * c0;
  for (int m0 = wave; m0 < S; m0 += C2I_W * RB) {
    float v[RB][C2I_JK];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int m = m0 + r * C2I_W;
#pragma unroll
      for (int k = 0; k < C2I_JK; ++k) {
        const int j = lane + 64 * k;
        v[r][k] = (m < S && j < seg) ? db[(long)m * 9 * C + j] : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int m = m0 + r * C2I_W;
#pragma unroll
      for (int k = 0; k < C2I_JK; ++k) {
        const int j = lane + 64 * k;
        if (m < S && j < seg) seg_lds[m * LD + j] = v[r][k];
      }
    }
  }
  __syncthreads();
  // gather: thread -> (pixel, channel lane & 31), two pixels per wave
  const int c = lane & (C2I_CC - 1);
  float* xo = dx + (long)bb * HW * C + c0 + c;
  if (c < nc)
    for (int p = wave * 2 + (lane >> 5); p < HW; p += 2 * C2I_W) {
      const int ih = p / W, iw = p - ih * W;
      float s = 0.f;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int oh = ih - kh;
        if (oh < 0 || oh >= OH) continue;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int ow = iw - kw;
          if (ow < 0 || ow >= OW) continue;
          s += seg_lds[(oh * OW + ow) * LD + 9 * c + kh * 3 + kw];
        }
      }
      xo[(long)p * C] = s;
    }
}

// channels per block of the LDS forms (0: the per-thread kernels): the col chunk S x 9 x 32 floats in at
// most 64 KB of LDS (patches up to 11 x 11); knob C2I_LDS=0 keeps the per-thread kernels (probe library:
// tests compare both forms in one process)
static int c2i_chunk(int H, int W, int C) {
  if (vc_knob("VITCNN_C2I_LDS", 1) == 0) return 0;
  const long S = (long)(H - 2) * (W - 2);
  return S * 9 * C2I_CC * 4 <= 65536 ? C2I_CC : 0;
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
  hipLaunchKernelGGL(nchw_to_nhwc, dim3(vc_cdiv(HW, 32), vc_cdiv(C, 32), B), dim3(256), 0, stream, B, C, HW, x, y, C);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_nchw_to_nhwc_pad(int B, int C, int HW, const float* x, float* y, int ldy, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && C > 0 && HW > 0 && ldy >= C);
  if (B == 0) return VC_OK;
  hipLaunchKernelGGL(nchw_to_nhwc, dim3(vc_cdiv(HW, 32), vc_cdiv(ldy, 32), B), dim3(256), 0, stream, B, C, HW, x, y,
                     ldy);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_im2col3x3(int B, int H, int W, int C, const float* x, const float* bn_mean, const float* bn_invstd,
                        const float* bn_w, const float* bn_b, float* col, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && H >= 3 && W >= 3 && C > 0);
  long total = (long)B * (H - 2) * (W - 2) * C;
  if (total == 0) return VC_OK;
  VC_REQUIRE_I32(total * 9);
  if (const int cc = c2i_chunk(H, W, C)) {
    const int nchunk = vc_cdiv(C, cc);
    VC_REQUIRE_I32((long)B * nchunk);
    hipLaunchKernelGGL(im2col3x3_lds, dim3(B * nchunk), dim3(C2I_T), sizeof(float) * H * W * (cc + 1), stream, nchunk, H, W,
                       C, x, bn_mean, bn_invstd, bn_w, bn_b, col);
    VC_CHECK_LAUNCH();
    return VC_OK;
  }
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
  if (const int cc = c2i_chunk(H, W, C)) {
    const int nchunk = vc_cdiv(C, cc);
    VC_REQUIRE_I32((long)B * nchunk);
    hipLaunchKernelGGL(col2im3x3_lds, dim3(B * nchunk), dim3(C2I_T), sizeof(float) * (H - 2) * (W - 2) * 9 * cc,
                       stream, nchunk, H, W, C, dcol, dx);
    VC_CHECK_LAUNCH();
    return VC_OK;
  }
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
