// Implicit-GEMM 3x3 convolution on CDNA4 matrix cores (v_mfma_f32_16x16x4_f32): forward, weight
// gradient and data gradient of a 3x3 conv over channels-last maps WITHOUT an im2col matrix in HBM.
//
// Reference convs: ms_conv_bn_relu (Mutimodality_Mamba7.py:1035-1048: BN -> conv3x3 valid -> ReLU,
// the BN affine is applied as the operand is gathered) and FusAtNet's ConvUnit / ConvUnit_NP /
// Residual units (model/compare_method/FusAtNet.py:9-60, padding 1 or 0).  The im2col column order is
// the torch weight's: k = c*9 + kh*3 + kw over weight [O][C][3][3] = [O][9C], so parameters and
// gradients are used in place.
//
//  * forward   y[m, o]   = sum_k im2col(x)[m, k] W[o, k] (+ bias[o]) (ReLU)         m = (b, oh, ow)
//  * wgrad     dW[o, k]  = beta dW + sum_m dY[m, o] im2col(x)[m, k];  dbias[o] = beta dbias + sum_m dY[m, o]
//  * dgrad     dx[p, c]  = beta dx + sum_{tap, o} dY[(b, ih - kh + pad, iw - kw + pad), o] W[o, c*9 + tap]
//                                                                                   p = (b, ih, iw)
// The gathered operand is read from the (L2-resident) activation map as the tile is staged, so the
// 9x-wide col matrix (up to 611 MB for FusAtNet's 2193-channel concat at B = 64) is never written or
// read back.  Tiles, LDS layout and split-K follow gemm.hip's k-major fp32 kernel: 64 x 64 output
// tile per 256-thread block (4 waves of 32 x 32), BK = 32, one-tile register prefetch; split K
// (weight gradients: K = B*OH*OW rows) into fixed-order slabs summed by a separate kernel.
#include "common.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 32, LDS_STRIDE = 81, NE = 8;

enum { CONV_FWD = 0, CONV_WGRAD = 1, CONV_DGRAD = 2 };

struct ConvArgs {
  int B, H, W, C, O, pad, OH, OW;
  FastDiv fOW, fOH, fW, fH, fO;
  const float* x;        // fwd / wgrad: input map [B,H,W,C] (ld ldx); dgrad: dY [B,OH,OW,O] (ld ldx)
  long ldx;
  const float *bn_mean, *bn_invstd, *bn_w, *bn_b;   // optional affine of the input (null: none)
  const float* other;    // fwd: W [O][9C]; wgrad: dY [M][O] (ld ldo); dgrad: W [O][9C]
  long ldo;
  int M, N, K, Ne;       // GEMM view (Ne = N + 1 with the bias-gradient ones column)
  int k_chunk, nsplit;
  float* out;            // fwd: y (ld ldout); wgrad: dW [O][9C]; dgrad: dx (ld ldout)
  long ldout;
  const float* bias;     // fwd bias
  float* bias_grad;      // wgrad: dbias
  float beta;
  int relu;
  float* part;           // split-K slabs [nsplit][M][Ne]
};

// im2col(x)[m, k] with m = (b, oh, ow) decoded by the caller (pixel base index of (b, oh - pad, ow - pad))
__device__ __forceinline__ float gather_col(const ConvArgs& a, int b, int oh, int ow, int k) {
  const int c = k / 9, t = k - 9 * c;
  const int kh = t / 3, kw = t - 3 * kh;
  const int ih = oh + kh - a.pad, iw = ow + kw - a.pad;
  if (ih < 0 || ih >= a.H || iw < 0 || iw >= a.W) return 0.f;
  float v = a.x[((long)(b * a.H + ih) * a.W + iw) * a.ldx + c];
  if (a.bn_mean) {
    const float sc = a.bn_invstd[c] * a.bn_w[c];
    v = (v - a.bn_mean[c]) * sc + a.bn_b[c];
  }
  return v;
}

template <int MODE, bool VO>
__global__ __launch_bounds__(256) void conv_gemm(ConvArgs a) {
  __shared__ float As[BK * LDS_STRIDE];
  __shared__ float Bs[BK * LDS_STRIDE];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int zs = blockIdx.z;
  const int kbeg = zs * a.k_chunk;
  const int kend = min(a.K, kbeg + a.k_chunk);

  // per-thread fixed coordinates (decoded once)
  // A side: FWD / DGRAD: row r = tid >> 2 (gathered rows), k = (tid & 3) * 8 + e
  //         WGRAD: A(o, m) = dY[m][o]: o = (tid & 15) * 4 + (e & 3), m = (tid >> 4) + 16 (e >> 2)
  // B side: FWD: B(k, n) = W[n][k]: n = tid >> 2, k = (tid & 3) * 8 + e
  //         WGRAD / DGRAD: n = (tid & 15) * 4 + (e & 3), k = (tid >> 4) + 16 (e >> 2)
  int pb = 0, ph = 0, pw = 0;   // decoded gathered row (FWD: output pixel; DGRAD: input pixel)
  const int ar = m0 + (tid >> 2);
  if (MODE == CONV_FWD && ar < a.M) {
    int q = fdivmod(ar, a.fOW, pw);
    pb = fdivmod(q, a.fOH, ph);
  }
  if (MODE == CONV_DGRAD && ar < a.M) {
    int q = fdivmod(ar, a.fW, pw);
    pb = fdivmod(q, a.fH, ph);
  }
  float ra[NE], rb[NE];

  auto load = [&](int k0) {
    if constexpr (MODE == CONV_FWD) {
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int k = k0 + (tid & 3) * 8 + e;
        ra[e] = (ar < a.M && k < kend) ? gather_col(a, pb, ph, pw, k) : 0.f;
      }
      const int n = n0 + (tid >> 2);
      const int kb = k0 + (tid & 3) * 8;
      if (VO && n < a.N && kb + 7 < kend) {
        const float4 x0 = *reinterpret_cast<const float4*>(a.other + (long)n * a.K + kb);
        const float4 x1 = *reinterpret_cast<const float4*>(a.other + (long)n * a.K + kb + 4);
        rb[0] = x0.x; rb[1] = x0.y; rb[2] = x0.z; rb[3] = x0.w;
        rb[4] = x1.x; rb[5] = x1.y; rb[6] = x1.z; rb[7] = x1.w;
      } else {
#pragma unroll
        for (int e = 0; e < NE; ++e) rb[e] = (n < a.N && kb + e < kend) ? a.other[(long)n * a.K + kb + e] : 0.f;
      }
    } else if constexpr (MODE == CONV_WGRAD) {
      // A(o, m) = dY[m * ldo + o]
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = k0 + (tid >> 4) + 16 * h;
        const int o = m0 + (tid & 15) * 4;
        if (VO && m < kend && o + 3 < a.M) {
          const float4 v = *reinterpret_cast<const float4*>(a.other + (long)m * a.ldo + o);
          ra[4 * h] = v.x; ra[4 * h + 1] = v.y; ra[4 * h + 2] = v.z; ra[4 * h + 3] = v.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) ra[4 * h + j] = (m < kend && o + j < a.M) ? a.other[(long)m * a.ldo + o + j] : 0.f;
        }
      }
      // B(m, n) = im2col(x)[m, n] (n = conv k index), column N = the ones column (bias gradient)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int m = k0 + (tid >> 4) + 16 * h;
        int b = 0, oh = 0, ow = 0;
        if (m < kend) {
          int q = fdivmod(m, a.fOW, ow);
          b = fdivmod(q, a.fOH, oh);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + (tid & 15) * 4 + j;
          float v = 0.f;
          if (m < kend) {
            if (n < a.N) v = gather_col(a, b, oh, ow, n);
            else if (n == a.N && a.Ne > a.N) v = 1.f;
          }
          rb[4 * h + j] = v;
        }
      }
    } else {   // CONV_DGRAD
      // A(p, k') = dY[(b, ih - kh + pad, iw - kw + pad), o],  k' = tap * O + o
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const int k = k0 + (tid & 3) * 8 + e;
        float v = 0.f;
        if (ar < a.M && k < kend) {
          int o;
          const int tap = fdivmod(k, a.fO, o);
          const int kh = tap / 3, kw = tap - 3 * kh;
          const int oh = ph - kh + a.pad, ow = pw - kw + a.pad;
          if (oh >= 0 && oh < a.OH && ow >= 0 && ow < a.OW) v = a.x[((long)(pb * a.OH + oh) * a.OW + ow) * a.ldx + o];
        }
        ra[e] = v;
      }
      // B(k', c) = W[o][c*9 + tap]
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = k0 + (tid >> 4) + 16 * h;
        int o = 0, tap = 0;
        if (k < kend) tap = fdivmod(k, a.fO, o);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = n0 + (tid & 15) * 4 + j;
          rb[4 * h + j] = (k < kend && c < a.N) ? a.other[(long)o * (9 * a.C) + c * 9 + tap] : 0.f;
        }
      }
    }
  };
  auto store = [&]() {
    if constexpr (MODE == CONV_WGRAD) {
#pragma unroll
      for (int e = 0; e < NE; ++e) As[((tid >> 4) + 16 * (e >> 2)) * LDS_STRIDE + (tid & 15) * 4 + (e & 3)] = ra[e];
    } else {
#pragma unroll
      for (int e = 0; e < NE; ++e) As[((tid & 3) * 8 + e) * LDS_STRIDE + (tid >> 2)] = ra[e];
    }
    if constexpr (MODE == CONV_FWD) {
#pragma unroll
      for (int e = 0; e < NE; ++e) Bs[((tid & 3) * 8 + e) * LDS_STRIDE + (tid >> 2)] = rb[e];
    } else {
#pragma unroll
      for (int e = 0; e < NE; ++e) Bs[((tid >> 4) + 16 * (e >> 2)) * LDS_STRIDE + (tid & 15) * 4 + (e & 3)] = rb[e];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fk = lane >> 4;
  if (kbeg < kend) {
    load(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      store();
      __syncthreads();
      if (k0 + BK < kend) load(k0 + BK);
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        const int kk = ks * 4 + fk;
        const float a0 = As[kk * LDS_STRIDE + wm * 32 + fr];
        const float a1 = As[kk * LDS_STRIDE + wm * 32 + 16 + fr];
        const float b0 = Bs[kk * LDS_STRIDE + wn * 32 + fr];
        const float b1 = Bs[kk * LDS_STRIDE + wn * 32 + 16 + fr];
        acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  // C/D map of 16x16x4: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + mi * 16 + fk * 4 + r;
        const int n = n0 + wn * 32 + ni * 16 + fr;
        if (m >= a.M || n >= a.Ne) continue;
        const float v = acc[mi][ni][r];
        if (a.nsplit > 1) {
          a.part[((long)zs * a.M + m) * a.Ne + n] = v;
        } else if (MODE == CONV_FWD) {
          float y = v + (a.bias ? a.bias[n] : 0.f);
          a.out[(long)m * a.ldout + n] = a.relu ? fmaxf(y, 0.f) : y;
        } else if (MODE == CONV_WGRAD && n == a.N) {
          a.bias_grad[m] = v + (a.beta != 0.f ? a.beta * a.bias_grad[m] : 0.f);
        } else {
          float* p = a.out + (long)m * a.ldout + n;
          *p = v + (a.beta != 0.f ? a.beta * *p : 0.f);
        }
      }
}

// fixed-order (z ascending) sum of the split-K slabs + the mode's epilogue; one thread per output
template <int MODE>
__global__ __launch_bounds__(256) void conv_splitk_reduce(ConvArgs a) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long tot = (long)a.M * a.Ne;
  if (idx >= tot) return;
  const int m = (int)(idx / a.Ne), n = (int)(idx - (long)m * a.Ne);
  float s = 0.f;
  for (int z = 0; z < a.nsplit; ++z) s += a.part[(long)z * tot + idx];
  if (MODE == CONV_FWD) {
    float y = s + (a.bias ? a.bias[n] : 0.f);
    a.out[(long)m * a.ldout + n] = a.relu ? fmaxf(y, 0.f) : y;
  } else if (MODE == CONV_WGRAD && n == a.N) {
    a.bias_grad[m] = s + (a.beta != 0.f ? a.beta * a.bias_grad[m] : 0.f);
  } else {
    float* p = a.out + (long)m * a.ldout + n;
    *p = s + (a.beta != 0.f ? a.beta * *p : 0.f);
  }
}

// split K while the output grid is short of ~3 blocks per CU: slices of >= 4 BK steps, slabs in ws
static void choose_split(ConvArgs& a, float* ws, long ws_floats) {
  const long tiles = (long)vc_cdiv(a.Ne, BN) * vc_cdiv(a.M, BM);
  int nsplit = 1;
  if (ws && a.K >= 8 * BK && tiles < 384) {
    const long want = (768 + tiles - 1) / tiles;
    nsplit = (int)std::min<long>(std::min<long>(want, a.K / (4 * BK)), 256);
    while (nsplit > 1 && (long)nsplit * a.M * a.Ne > ws_floats) --nsplit;
    nsplit = std::max(nsplit, 1);
  }
  a.k_chunk = a.K;
  if (nsplit > 1) {
    a.k_chunk = vc_cdiv(vc_cdiv(a.K, nsplit), BK) * BK;
    nsplit = vc_cdiv(a.K, a.k_chunk);
  }
  a.nsplit = nsplit;
  a.part = ws;
}

template <int MODE>
static int launch(ConvArgs& a, bool vo, float* ws, long ws_floats, hipStream_t stream) {
  choose_split(a, ws, ws_floats);
  dim3 grid(vc_cdiv(a.Ne, BN), vc_cdiv(a.M, BM), a.nsplit);
  if (vo) hipLaunchKernelGGL((conv_gemm<MODE, true>), grid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((conv_gemm<MODE, false>), grid, dim3(256), 0, stream, a);
  VC_CHECK_LAUNCH();
  if (a.nsplit > 1) {
    hipLaunchKernelGGL(conv_splitk_reduce<MODE>, dim3(vc_cdiv((long)a.M * a.Ne, 256)), dim3(256), 0, stream, a);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

static ConvArgs make_args(int B, int H, int W, int C, int O, int pad) {
  ConvArgs a{};
  a.B = B; a.H = H; a.W = W; a.C = C; a.O = O; a.pad = pad;
  a.OH = H + 2 * pad - 2;
  a.OW = W + 2 * pad - 2;
  a.fOW = make_fastdiv(a.OW);
  a.fOH = make_fastdiv(a.OH);
  a.fW = make_fastdiv(W);
  a.fH = make_fastdiv(H);
  a.fO = make_fastdiv(O);
  return a;
}

static bool aligned16(const void* p) { return ((uintptr_t)p % 16) == 0; }

}  // namespace

VC_API int vc_conv3x3_fwd(int B, int H, int W, int C, int O, int pad, const float* x, long ldx, const float* bn_mean,
                          const float* bn_invstd, const float* bn_w, const float* bn_b, const float* weight,
                          const float* bias, int relu, float* y, long ldy, float* ws, long ws_floats,
                          hipStream_t stream) {
  VC_REQUIRE(B > 0 && C > 0 && O > 0 && (pad == 0 || pad == 1) && ldx >= C && ldy >= O);
  VC_REQUIRE(H + 2 * pad - 2 > 0 && W + 2 * pad - 2 > 0);
  VC_REQUIRE(!bn_mean || (bn_invstd && bn_w && bn_b));
  ConvArgs a = make_args(B, H, W, C, O, pad);
  VC_REQUIRE_I32((long)B * H * W * ldx);
  VC_REQUIRE_I32((long)B * a.OH * a.OW * ldy);
  VC_REQUIRE_I32(9L * C * O);
  a.x = x; a.ldx = ldx;
  a.bn_mean = bn_mean; a.bn_invstd = bn_invstd; a.bn_w = bn_w; a.bn_b = bn_b;
  a.other = weight;
  a.M = B * a.OH * a.OW; a.N = O; a.K = 9 * C; a.Ne = O;
  a.out = y; a.ldout = ldy; a.bias = bias; a.relu = relu; a.beta = 0.f;
  return launch<CONV_FWD>(a, aligned16(weight) && (a.K % 4 == 0), ws, ws_floats, stream);
}

VC_API int vc_conv3x3_wgrad(int B, int H, int W, int C, int O, int pad, const float* x, long ldx, const float* bn_mean,
                            const float* bn_invstd, const float* bn_w, const float* bn_b, const float* dy, long lddy,
                            float beta, float* dweight, float* dbias, float* ws, long ws_floats, hipStream_t stream) {
  VC_REQUIRE(B > 0 && C > 0 && O > 0 && (pad == 0 || pad == 1) && ldx >= C && lddy >= O);
  VC_REQUIRE(H + 2 * pad - 2 > 0 && W + 2 * pad - 2 > 0);
  VC_REQUIRE(!bn_mean || (bn_invstd && bn_w && bn_b));
  ConvArgs a = make_args(B, H, W, C, O, pad);
  VC_REQUIRE_I32((long)B * H * W * ldx);
  VC_REQUIRE_I32((long)B * a.OH * a.OW * lddy);
  a.x = x; a.ldx = ldx;
  a.bn_mean = bn_mean; a.bn_invstd = bn_invstd; a.bn_w = bn_w; a.bn_b = bn_b;
  a.other = dy; a.ldo = lddy;
  a.M = O; a.N = 9 * C; a.K = B * a.OH * a.OW; a.Ne = a.N + (dbias ? 1 : 0);
  a.out = dweight; a.ldout = 9L * C; a.bias_grad = dbias; a.beta = beta;
  return launch<CONV_WGRAD>(a, aligned16(dy) && (lddy % 4 == 0), ws, ws_floats, stream);
}

VC_API int vc_conv3x3_dgrad(int B, int H, int W, int C, int O, int pad, const float* dy, long lddy, const float* weight,
                            float beta, float* dx, long lddx, float* ws, long ws_floats, hipStream_t stream) {
  VC_REQUIRE(B > 0 && C > 0 && O > 0 && (pad == 0 || pad == 1) && lddy >= O && lddx >= C);
  VC_REQUIRE(H + 2 * pad - 2 > 0 && W + 2 * pad - 2 > 0);
  ConvArgs a = make_args(B, H, W, C, O, pad);
  VC_REQUIRE_I32((long)B * H * W * lddx);
  VC_REQUIRE_I32((long)B * a.OH * a.OW * lddy);
  a.x = dy; a.ldx = lddy;
  a.other = weight;
  a.M = B * H * W; a.N = C; a.K = 9 * O; a.Ne = C;
  a.out = dx; a.ldout = lddx; a.beta = beta;
  return launch<CONV_DGRAD>(a, false, ws, ws_floats, stream);
}
