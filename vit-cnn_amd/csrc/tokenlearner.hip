// TokenLearner(S) = S independent SpatialAttention modules (Mutimodality_Mamba7.py:26-64),
// fused: the channel max / mean of the input are shared by all S tokens, so they are computed
// once per pixel; each token then only needs a 2->1 1x1 conv, a BatchNorm2d(1) over the whole
// batch (train: batch stats + running update), ReLU and sigmoid to produce its spatial weight
// map a[b, s, :] (one workgroup per token, two-pass block reductions).  The weighted spatial
// mean Z[b, s, :] = mean_p a[b, s, p] x[b, p, :] is a batched GEMM (vc_gemm).
//
// Parameter layout: the S SpatialAttention modules' parameters are contiguous in the flat
// parameter buffer in state_dict order, 5 floats per token
//   [conv.0.weight (2), conv.0.bias, conv.1.weight (gamma), conv.1.bias (beta)],
// and their BN buffers 2 floats per token [running_mean, running_var].
#include "common.h"

namespace {

constexpr int TPAR = 5, TBUF = 2;

// per pixel (row of C channels): max (+ first argmax) and mean; one wave per row
__global__ __launch_bounds__(256) void pixel_stats(long M, int C, const float* __restrict__ x, long ldx,
                                                   float* __restrict__ mx, int* __restrict__ amx,
                                                   float* __restrict__ avg) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  const float* xr = x + r * ldx;
  float best = -INFINITY, s = 0.f;
  int bi = 0x7fffffff;
  for (int c0 = lane; c0 < C; c0 += 64 * 8) {   // 8 of the lane's channels loaded, then scanned in order
    float xv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) xv[j] = c0 + 64 * j < C ? xr[c0 + 64 * j] : 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + 64 * j;
      if (c < C) {
        const float v = xv[j];
        s += v;
        if (v > best) {
          best = v;
          bi = c;
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob > best || (ob == best && oi < bi)) {
      best = ob;
      bi = oi;
    }
  }
  s = wave_sum(s);
  if (lane == 0) {
    mx[r] = best;
    amx[r] = bi;
    avg[r] = s / C;
  }
}

constexpr int TLT = 1024;  // threads per token block (16 waves): the token's B*HW elements are the long axis

// Reductions over a token's B*HW elements accumulate in fp64, like torch's CPU BatchNorm
// (acc_type<float> = double): these BN(1) inputs have a tiny spread around a large mean, so
// fp32 sums lose ~3 digits in the statistics and in the backward's dgamma / dbeta / dx terms.
__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double r = 0.0;
#pragma unroll
  for (int i = 0; i < TLT / 64; ++i) r += red[i];
  __syncthreads();
  return r;
}

// K independent block sums in one pass (one pair of barriers instead of K); each value is summed in
// block_sum's order, so the results are bit-identical to K block_sum calls
template <int K>
__device__ __forceinline__ void block_sums(double (&v)[K], double* red) {
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[k * (TLT / 64) + w] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double r = 0.0;
#pragma unroll
    for (int i = 0; i < TLT / 64; ++i) r += red[k * (TLT / 64) + i];
    v[k] = r;
  }
  __syncthreads();
}

// the token's 2->1 conv output for pixel i, in fp64: BN(1) normalises values with a tiny spread
// around a large mean, so the fp32 rounding of the conv would be amplified by 1/std
__device__ __forceinline__ double tl_fv(float m, float v, float w0, float w1, float bc) {
  return (double)w0 * m + (double)w1 * v + (double)bc;
}
__device__ __forceinline__ double tl_f(const float* __restrict__ mx, const float* __restrict__ avg, long i, float w0,
                                       float w1, float bc) {
  return tl_fv(mx[i], avg[i], w0, w1, bc);
}

// the token's BN(1) output for pixel i: forward, backward and vc_tl_relu_mask share this one
// expression, so they take identical ReLU decisions
__device__ __forceinline__ float tl_bnv(float m, float v, float w0, float w1, float bc, double mean, double invstd,
                                        float gam, float bet, double& xh) {
  xh = (tl_fv(m, v, w0, w1, bc) - mean) * invstd;
  return (float)xh * gam + bet;
}
__device__ __forceinline__ float tl_bn(const float* __restrict__ mx, const float* __restrict__ avg, long i, float w0,
                                       float w1, float bc, double mean, double invstd, float gam, float bet,
                                       double& xh) {
  return tl_bnv(mx[i], avg[i], w0, w1, bc, mean, invstd, gam, bet, xh);
}

// A token block's pass over its n elements i = threadIdx.x + TLT * k in increasing k: the (mx, avg)
// pairs of NBT consecutive k are loaded before any is used (one round of dependent loads per NBT
// elements instead of one per element), then fn(i, mx[i], avg[i]) runs in the same element order as
// a plain loop, so every accumulation is bit-identical to it.
constexpr int NBT = 8;
template <typename Fn>
__device__ __forceinline__ void tl_pass(long n, const float* __restrict__ mx, const float* __restrict__ avg, Fn fn) {
  for (long i0 = threadIdx.x; i0 < n; i0 += (long)TLT * NBT) {
    float m[NBT], v[NBT];
#pragma unroll
    for (int j = 0; j < NBT; ++j) {
      const long i = i0 + (long)TLT * j;
      m[j] = i < n ? mx[i] : 0.f;
      v[j] = i < n ? avg[i] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < NBT; ++j) {
      const long i = i0 + (long)TLT * j;
      if (i < n) fn(i, m[j], v[j]);
    }
  }
}

// one block per token s; a[(b*S + s)*HW + p]
__global__ __launch_bounds__(1024) void attn_fwd(int train, int B, int HW, FastDiv fHW, int S, const float* __restrict__ mx,
                                                const float* __restrict__ avg, const float* __restrict__ par,
                                                float* __restrict__ buf, float eps, float momentum,
                                                double* __restrict__ stats, float* __restrict__ a) {
  __shared__ double red[TLT / 64];
  const int s = blockIdx.x;
  const float* p = par + (long)s * TPAR;
  const float w0 = p[0], w1 = p[1], bc = p[2], gam = p[3], bet = p[4];
  const long n = (long)B * HW;
  double mean, invstd;
  if (train) {
    double acc = 0.0;
    tl_pass(n, mx, avg, [&](long, float m, float v) { acc += tl_fv(m, v, w0, w1, bc); });
    mean = block_sum(acc, red) / (double)n;
    double q = 0.0;
    tl_pass(n, mx, avg, [&](long, float m, float v) {
      const double d = tl_fv(m, v, w0, w1, bc) - mean;
      q += d * d;
    });
    const double m2 = block_sum(q, red);
    const double var = m2 / (double)n;
    invstd = 1.0 / sqrt(var + (double)eps);
    if (threadIdx.x == 0 && buf) {
      float* bb = buf + (long)s * TBUF;
      const double unb = n > 1 ? m2 / (double)(n - 1) : var;
      bb[0] = (float)((1.0 - momentum) * bb[0] + momentum * mean);
      bb[1] = (float)((1.0 - momentum) * bb[1] + momentum * unb);
    }
  } else {
    const float* bb = buf + (long)s * TBUF;
    mean = bb[0];
    invstd = 1.0 / sqrt((double)bb[1] + (double)eps);
  }
  if (threadIdx.x == 0) {  // saved as (mean, invstd) in fp64 for the backward
    stats[2 * s] = mean;
    stats[2 * s + 1] = invstd;
  }
  tl_pass(n, mx, avg, [&](long i, float m, float v) {
    double xh;
    const float bn = tl_bnv(m, v, w0, w1, bc, mean, invstd, gam, bet, xh);
    int q;
    const long b = fdivmod((int)i, fHW, q);   // n = B * HW < 2^31 (launcher): 32-bit magic division
    a[((long)b * S + s) * HW + q] = sigmoid_f(fmaxf(bn, 0.f));
  });
}

// one block per token: da -> df[s][i] (grad of the 2->1 conv output) + the token's 5 param grads
__global__ __launch_bounds__(1024) void attn_bwd(int train, int B, int HW, FastDiv fHW, int S, const float* __restrict__ mx,
                                                const float* __restrict__ avg, const float* __restrict__ par,
                                                const double* __restrict__ stats, const float* __restrict__ da,
                                                float* __restrict__ df, float* __restrict__ gpar) {
  __shared__ double red[3 * (TLT / 64)];
  const int s = blockIdx.x;
  const float* p = par + (long)s * TPAR;
  const float w0 = p[0], w1 = p[1], bc = p[2], gam = p[3], bet = p[4];
  const double mean = stats[2 * s], invstd = stats[2 * s + 1];
  const long n = (long)B * HW;
  // da[b, s, q] of element i = b * HW + q, loaded with the element's (mx, avg) (same batching and
  // element order as tl_pass)
  auto pass = [&](auto fn) {
    for (long i0 = threadIdx.x; i0 < n; i0 += (long)TLT * NBT) {
      float m[NBT], v[NBT], g[NBT];
#pragma unroll
      for (int j = 0; j < NBT; ++j) {
        const long i = i0 + (long)TLT * j;
        const bool ok = i < n;
        int q = 0;
        const long b = ok ? fdivmod((int)i, fHW, q) : 0;
        m[j] = ok ? mx[i] : 0.f;
        v[j] = ok ? avg[i] : 0.f;
        g[j] = ok ? da[((long)b * S + s) * HW + q] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < NBT; ++j) {
        const long i = i0 + (long)TLT * j;
        if (i < n) fn(i, m[j], v[j], g[j]);
      }
    }
  };
  double s1 = 0.0, s2 = 0.0;
  pass([&](long, float m, float v, float dav) {
    double xh;
    const float bn = tl_bnv(m, v, w0, w1, bc, mean, invstd, gam, bet, xh);
    float g1 = 0.f;
    if (bn > 0.f) {
      const float sg = sigmoid_f(bn);
      g1 = dav * sg * (1.f - sg);
    }
    s1 += g1;
    s2 += g1 * xh;
  });
  {
    double v2[2] = {s1, s2};
    block_sums(v2, red);
    s1 = v2[0];
    s2 = v2[1];
  }
  double gw0 = 0.0, gw1 = 0.0, gb = 0.0;
  pass([&](long i, float m, float v, float dav) {
    double xh;
    const float bn = tl_bnv(m, v, w0, w1, bc, mean, invstd, gam, bet, xh);
    float g1 = 0.f;
    if (bn > 0.f) {
      const float sg = sigmoid_f(bn);
      g1 = dav * sg * (1.f - sg);
    }
    const double d = train ? gam * invstd * (g1 - s1 / (double)n - xh * s2 / (double)n) : gam * invstd * g1;
    df[(long)s * n + i] = (float)d;
    gw0 += d * m;
    gw1 += d * v;
    gb += d;
  });
  {
    double v3[3] = {gw0, gw1, gb};
    block_sums(v3, red);
    gw0 = v3[0];
    gw1 = v3[1];
    gb = v3[2];
  }
  if (threadIdx.x == 0) {
    float* g = gpar + (long)s * TPAR;
    g[0] = (float)gw0;
    g[1] = (float)gw1;
    g[2] = (float)gb;
    g[3] = (float)s2;
    g[4] = (float)s1;
  }
}

// mask[(b*S + s)*HW + q] = (BN(1) output > 0): the ReLU decisions attn_fwd / attn_bwd took
__global__ __launch_bounds__(256) void attn_mask(int B, int HW, FastDiv fHW, int S, const float* __restrict__ mx,
                                                 const float* __restrict__ avg, const float* __restrict__ par,
                                                 const double* __restrict__ stats, unsigned char* __restrict__ mask) {
  const int s = blockIdx.y;
  const long n = (long)B * HW, i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float* p = par + (long)s * TPAR;
  double xh;
  const float bn = tl_bn(mx, avg, i, p[0], p[1], p[2], stats[2 * s], stats[2 * s + 1], p[3], p[4], xh);
  int q;
  const long bq = fdivmod((int)i, fHW, q);
  mask[(bq * S + s) * HW + q] = bn > 0.f ? 1 : 0;
}

// dx[i, c] += davg/C + (c == argmax ? dmx : 0),  dmx / davg summed over the S tokens
__global__ __launch_bounds__(256) void pixel_bwd(long M, int C, int S, const float* __restrict__ df,
                                                 const float* __restrict__ par, const int* __restrict__ amx,
                                                 float* __restrict__ dx, long lddx) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= M) return;
  float gm = 0.f, ga = 0.f;
  for (int s = lane; s < S; s += 64) {
    const float d = df[(long)s * M + r];
    gm += d * par[(long)s * TPAR];
    ga += d * par[(long)s * TPAR + 1];
  }
  gm = wave_sum(gm);
  ga = wave_sum(ga) / (float)C;
  const int am = amx[r];
  float* dr = dx + r * lddx;
  for (int c = lane; c < C; c += 64) dr[c] += ga + (c == am ? gm : 0.f);
}

}  // namespace

VC_API int vc_tl_pixel_stats(long M, int C, const float* x, long ldx, float* mx, int* amx, float* avg,
                             hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C > 0);
  if (M == 0) return VC_OK;
  hipLaunchKernelGGL(pixel_stats, dim3(vc_cdiv(M, 4)), dim3(256), 0, stream, M, C, x, ldx, mx, amx, avg);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_tl_attn_fwd(int train, int B, int HW, int S, const float* mx, const float* avg, const float* params,
                          float* bn_buffers, float eps, float momentum, double* stats, float* a, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && S > 0);
  VC_REQUIRE_I32((long)B * HW);
  hipLaunchKernelGGL(attn_fwd, dim3(S), dim3(TLT), 0, stream, train, B, HW, make_fastdiv(HW), S, mx, avg, params, bn_buffers, eps,
                     momentum, stats, a);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_tl_attn_bwd(int train, int B, int HW, int S, const float* mx, const float* avg, const float* params,
                          const double* stats, const float* da, float* df, float* dparams, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && S > 0);
  VC_REQUIRE_I32((long)B * HW);
  hipLaunchKernelGGL(attn_bwd, dim3(S), dim3(TLT), 0, stream, train, B, HW, make_fastdiv(HW), S, mx, avg, params, stats, da, df,
                     dparams);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_tl_relu_mask(int B, int HW, int S, const float* mx, const float* avg, const float* params,
                           const double* stats, unsigned char* mask, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && S > 0);
  VC_REQUIRE_I32((long)B * HW);
  hipLaunchKernelGGL(attn_mask, dim3(vc_cdiv((long)B * HW, 256), S), dim3(256), 0, stream, B, HW, make_fastdiv(HW), S, mx, avg, params,
                     stats, mask);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_tl_pixel_bwd(long M, int C, int S, const float* df, const float* params, const int* amx, float* dx,
                           long lddx, hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C > 0 && S > 0);
  if (M == 0) return VC_OK;
  hipLaunchKernelGGL(pixel_bwd, dim3(vc_cdiv(M, 4)), dim3(256), 0, stream, M, C, S, df, params, amx, dx, lddx);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
