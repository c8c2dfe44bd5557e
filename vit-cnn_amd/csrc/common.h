// Shared device helpers for the ViT-CNN CDNA4 (gfx950) kernels.
// Wave = 64 lanes; every reduction below is written for wave64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "vitcnn.h"

#define VC_EXPORT extern "C" __attribute__((visibility("default")))

#define VC_OK 0
#define VC_EINVAL 1  // hipErrorInvalidValue

#define VC_CHECK_LAUNCH()                    \
  do {                                       \
    hipError_t e__ = hipGetLastError();      \
    if (e__ != hipSuccess) return (int)e__;  \
  } while (0)

#define VC_REQUIRE(cond)          \
  do {                            \
    if (!(cond)) return VC_EINVAL; \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

static inline int vc_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// sum over aligned groups of 16 lanes (all lanes of the group get the result)
__device__ __forceinline__ float group16_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}

__device__ __forceinline__ float silu_f(float x) { return x / (1.0f + __expf(-x)); }
__device__ __forceinline__ float sigmoid_f(float x) { return 1.0f / (1.0f + __expf(-x)); }

// torch.nn.functional.softplus(beta=1, threshold=20)
__device__ __forceinline__ float softplus_f(float x) { return x > 20.0f ? x : log1pf(__expf(x)); }

// block-wide sum for blockDim.x == 256 (4 waves); `sh` needs >= 4 floats
__device__ __forceinline__ float block256_sum(float v, float* sh) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = sh[0] + sh[1] + sh[2] + sh[3];
  return r;
}

// Chan's parallel combination of (count, mean, M2) triples.
__device__ __forceinline__ void welford_merge(float& n, float& mean, float& m2, float nb, float meanb, float m2b) {
  float nn = n + nb;
  if (nn <= 0.f) return;
  float d = meanb - mean;
  float fb = nb / nn;
  mean = mean + d * fb;
  m2 = m2 + m2b + d * d * n * fb;
  n = nn;
}
