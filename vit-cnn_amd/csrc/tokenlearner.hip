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
  for (int c = lane; c < C; c += 64) {
    const float v = xr[c];
    s += v;
    if (v > best) {
      best = v;
      bi = c;
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

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const float r = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return r;
}

// one block per token s; a[(b*S + s)*HW + p]
__global__ __launch_bounds__(256) void attn_fwd(int train, int B, int HW, int S, const float* __restrict__ mx,
                                                const float* __restrict__ avg, const float* __restrict__ par,
                                                float* __restrict__ buf, float eps, float momentum,
                                                float* __restrict__ stats, float* __restrict__ a) {
  __shared__ float red[4];
  const int s = blockIdx.x;
  const float* p = par + (long)s * TPAR;
  const float w0 = p[0], w1 = p[1], bc = p[2], gam = p[3], bet = p[4];
  const long n = (long)B * HW;
  float mean, invstd;
  if (train) {
    float acc = 0.f;
    for (long i = threadIdx.x; i < n; i += 256) acc += w0 * mx[i] + w1 * avg[i] + bc;
    mean = block_sum(acc, red) / (float)n;
    float q = 0.f;
    for (long i = threadIdx.x; i < n; i += 256) {
      const float d = w0 * mx[i] + w1 * avg[i] + bc - mean;
      q += d * d;
    }
    const float m2 = block_sum(q, red);
    const float var = m2 / (float)n;
    invstd = rsqrtf(var + eps);
    if (threadIdx.x == 0 && buf) {
      float* bb = buf + (long)s * TBUF;
      const float unb = n > 1 ? m2 / (float)(n - 1) : var;
      bb[0] = (1.f - momentum) * bb[0] + momentum * mean;
      bb[1] = (1.f - momentum) * bb[1] + momentum * unb;
    }
  } else {
    const float* bb = buf + (long)s * TBUF;
    mean = bb[0];
    invstd = rsqrtf(bb[1] + eps);
  }
  if (threadIdx.x == 0) {
    stats[2 * s] = mean;
    stats[2 * s + 1] = invstd;
  }
  for (long i = threadIdx.x; i < n; i += 256) {
    const float f = w0 * mx[i] + w1 * avg[i] + bc;
    const float bn = (f - mean) * invstd * gam + bet;
    const long b = i / HW, q = i % HW;
    a[((long)b * S + s) * HW + q] = sigmoid_f(fmaxf(bn, 0.f));
  }
}

// one block per token: da -> df[s][i] (grad of the 2->1 conv output) + the token's 5 param grads
__global__ __launch_bounds__(256) void attn_bwd(int train, int B, int HW, int S, const float* __restrict__ mx,
                                                const float* __restrict__ avg, const float* __restrict__ par,
                                                const float* __restrict__ stats, const float* __restrict__ da,
                                                float* __restrict__ df, float* __restrict__ gpar) {
  __shared__ float red[4];
  const int s = blockIdx.x;
  const float* p = par + (long)s * TPAR;
  const float w0 = p[0], w1 = p[1], bc = p[2], gam = p[3], bet = p[4];
  const float mean = stats[2 * s], invstd = stats[2 * s + 1];
  const long n = (long)B * HW;
  float s1 = 0.f, s2 = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) {
    const float xh = (w0 * mx[i] + w1 * avg[i] + bc - mean) * invstd;
    const float bn = xh * gam + bet;
    const long b = i / HW, q = i % HW;
    float g1 = 0.f;
    if (bn > 0.f) {
      const float sg = sigmoid_f(bn);
      g1 = da[((long)b * S + s) * HW + q] * sg * (1.f - sg);
    }
    s1 += g1;
    s2 += g1 * xh;
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red);
  float gw0 = 0.f, gw1 = 0.f, gb = 0.f;
  for (long i = threadIdx.x; i < n; i += 256) {
    const float xh = (w0 * mx[i] + w1 * avg[i] + bc - mean) * invstd;
    const float bn = xh * gam + bet;
    const long b = i / HW, q = i % HW;
    float g1 = 0.f;
    if (bn > 0.f) {
      const float sg = sigmoid_f(bn);
      g1 = da[((long)b * S + s) * HW + q] * sg * (1.f - sg);
    }
    const float d = train ? gam * invstd * (g1 - s1 / (float)n - xh * s2 / (float)n) : gam * invstd * g1;
    df[(long)s * n + i] = d;
    gw0 += d * mx[i];
    gw1 += d * avg[i];
    gb += d;
  }
  gw0 = block_sum(gw0, red);
  gw1 = block_sum(gw1, red);
  gb = block_sum(gb, red);
  if (threadIdx.x == 0) {
    float* g = gpar + (long)s * TPAR;
    g[0] = gw0;
    g[1] = gw1;
    g[2] = gb;
    g[3] = s2;
    g[4] = s1;
  }
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
                          float* bn_buffers, float eps, float momentum, float* stats, float* a, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && S > 0);
  hipLaunchKernelGGL(attn_fwd, dim3(S), dim3(256), 0, stream, train, B, HW, S, mx, avg, params, bn_buffers, eps,
                     momentum, stats, a);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_tl_attn_bwd(int train, int B, int HW, int S, const float* mx, const float* avg, const float* params,
                          const float* stats, const float* da, float* df, float* dparams, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && S > 0);
  hipLaunchKernelGGL(attn_bwd, dim3(S), dim3(256), 0, stream, train, B, HW, S, mx, avg, params, stats, da, df,
                     dparams);
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
