// Single-head non-local cross attention of GLfusionBlock (NONLocalBlock2D, sub_sample=True;
// Mutimodality_Mamba7.py:140-159): f = theta(x)^T phi(y) WITHOUT 1/sqrt(d) scaling,
// softmax over the max-pooled keys, o = f g(z).  Per batch element the problem is tiny
// (queries S = 49 / 25, keys P = 9 / 4, inter channels Ci = 128 / 72): keys and values live in
// LDS, one wave per query row, wave64 shuffle reductions for the dot products and the softmax.
// Forward: a workgroup of 16 waves owns 16 query rows of one batch element (grid B x S/16).
// Backward: a 16-wave workgroup owns a whole batch element, since d(phi|g) reduces over all
// of its query rows in LDS (fixed order, no atomics).
//
// Layouts: theta [B*S, Ci]; pooled phi|g [B*P, 2*Ci] (phi in columns [0,Ci), g in [Ci,2Ci));
// att (saved softmax) [B, S, P]; o [B*S, Ci].
#include "common.h"

namespace {

constexpr int MAXP = 16;  // 2x2-pooled 9x9 grid (the largest patch the build supports: 11x11 inputs)
constexpr int MAXCI = 256;

// PT = number of pooled keys (compile-time so the per-row score array stays in registers)
constexpr int NT = 1024, NW = NT / 64;

template <int PT>
__global__ __launch_bounds__(NT) void nl_fwd(int S, int Ci, const float* __restrict__ theta,
                                             const float* __restrict__ pooled, float* __restrict__ att,
                                             float* __restrict__ o) {
  constexpr int P = PT;
  extern __shared__ float kv[];  // [P][2*Ci]
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* src = pooled + (long)b * P * 2 * Ci;
  for (int i = threadIdx.x; i < P * 2 * Ci; i += NT) kv[i] = src[i];
  __syncthreads();
  {
    const int s = blockIdx.y * NW + wave;
    if (s >= S) return;
    const float* q = theta + ((long)b * S + s) * Ci;
    float sc[PT];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      float acc = 0.f;
      for (int c = lane; c < Ci; c += 64) acc += q[c] * kv[j * 2 * Ci + c];
      sc[j] = wave_sum(acc);
      mx = fmaxf(mx, sc[j]);
    }
    float den = 0.f;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      sc[j] = __expf(sc[j] - mx);
      den += sc[j];
    }
    const float inv = 1.f / den;
#pragma unroll
    for (int j = 0; j < P; ++j) sc[j] *= inv;
    if (lane < P) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < P; ++j)
        if (j == lane) v = sc[j];
      att[((long)b * S + s) * P + lane] = v;
    }
    float* orow = o + ((long)b * S + s) * Ci;
    for (int c = lane; c < Ci; c += 64) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < P; ++j) acc += sc[j] * kv[j * 2 * Ci + Ci + c];
      orow[c] = acc;
    }
  }
}

template <int PT>
__global__ __launch_bounds__(NT) void nl_bwd(int S, int Ci, const float* __restrict__ theta,
                                              const float* __restrict__ pooled, const float* __restrict__ att,
                                              const float* __restrict__ dout, float* __restrict__ dtheta,
                                              float* __restrict__ dpooled) {
  constexpr int P = PT;
  extern __shared__ float sm[];
  float* kv = sm;                   // [P][2Ci]
  float* ds = kv + P * 2 * Ci;      // [S][P] dscore
  float* at = ds + S * P;           // [S][P] att
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* src = pooled + (long)b * P * 2 * Ci;
  for (int i = threadIdx.x; i < P * 2 * Ci; i += NT) kv[i] = src[i];
  for (int i = threadIdx.x; i < S * P; i += NT) at[i] = att[(long)b * S * P + i];
  __syncthreads();
  for (int s = wave; s < S; s += NW) {
    const float* dr = dout + ((long)b * S + s) * Ci;
    float da[PT];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      float acc = 0.f;
      for (int c = lane; c < Ci; c += 64) acc += dr[c] * kv[j * 2 * Ci + Ci + c];
      da[j] = wave_sum(acc);
      dot += at[s * P + j] * da[j];
    }
#pragma unroll
    for (int j = 0; j < P; ++j) da[j] = at[s * P + j] * (da[j] - dot);
    if (lane < P) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < P; ++j)
        if (j == lane) v = da[j];
      ds[s * P + lane] = v;
    }
    float* dq = dtheta + ((long)b * S + s) * Ci;
    for (int c = lane; c < Ci; c += 64) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < P; ++j) acc += da[j] * kv[j * 2 * Ci + c];
      dq[c] = acc;
    }
  }
  __syncthreads();
  float* dp = dpooled + (long)b * P * 2 * Ci;
  for (int i = threadIdx.x; i < P * 2 * Ci; i += NT) {
    const int j = i / (2 * Ci), c = i - j * (2 * Ci);
    float acc = 0.f;
    if (c < Ci) {
      for (int s = 0; s < S; ++s) acc += ds[s * P + j] * theta[((long)b * S + s) * Ci + c];
    } else {
      for (int s = 0; s < S; ++s) acc += at[s * P + j] * dout[((long)b * S + s) * Ci + c - Ci];
    }
    dp[i] = acc;
  }
}

}  // namespace

VC_API int vc_nonlocal_attn_fwd(int B, int S, int P, int Ci, const float* theta, const float* pooled, float* att,
                                float* o, hipStream_t stream) {
  VC_REQUIRE(B > 0 && S > 0 && P > 0 && P <= MAXP && Ci > 0 && Ci <= MAXCI);
  const size_t sm = sizeof(float) * (size_t)P * 2 * Ci;
#define VC_NL_FWD(PT_) \
  hipLaunchKernelGGL((nl_fwd<PT_>), dim3(B, vc_cdiv(S, NW)), dim3(NT), sm, stream, S, Ci, theta, pooled, att, o)
  switch (P) {  // pooled key counts of 5x5 / 7x7 / 9x9 query grids, then generic buckets
    case 4: VC_NL_FWD(4); break;
    case 9: VC_NL_FWD(9); break;
    case 16: VC_NL_FWD(16); break;
    default: return VC_EINVAL;
  }
#undef VC_NL_FWD
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_nonlocal_attn_bwd(int B, int S, int P, int Ci, const float* theta, const float* pooled, const float* att,
                                const float* dout, float* dtheta, float* dpooled, hipStream_t stream) {
  VC_REQUIRE(B > 0 && S > 0 && P > 0 && P <= MAXP && Ci > 0 && Ci <= MAXCI);
  const size_t sm = sizeof(float) * ((size_t)P * 2 * Ci + 2 * (size_t)S * P);
  VC_REQUIRE(sm <= 160 * 1024);
#define VC_NL_BWD(PT_) \
  hipLaunchKernelGGL((nl_bwd<PT_>), dim3(B), dim3(NT), sm, stream, S, Ci, theta, pooled, att, dout, dtheta, dpooled)
  switch (P) {
    case 4: VC_NL_BWD(4); break;
    case 9: VC_NL_BWD(9); break;
    case 16: VC_NL_BWD(16); break;
    default: return VC_EINVAL;
  }
#undef VC_NL_BWD
  VC_CHECK_LAUNCH();
  return VC_OK;
}
