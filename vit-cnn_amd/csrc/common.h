// Shared device helpers for the ViT-CNN CDNA4 (gfx950) kernels.
// Wave = 64 lanes; every reduction below is written for wave64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>

#include "vitcnn.h"

#define VC_EXPORT extern "C" __attribute__((visibility("default")))

// Measurement knobs: the A/B switches the tools/ probes flip (kernel variants, split policies, phase
// masks).  The product library (libvitcnn_hip.so, no VC_PROBE) reads no environment and keeps no
// state between calls: every knob is its compile-time default below, so an entry point's result
// depends on its arguments only.  `make probe` builds libvitcnn_probe.so with -DVC_PROBE, where
// vc_knob reads VITCNN_<name> on every call (tests that compare two bit-identical forms in one
// process, and the tools, load it explicitly).
#ifdef VC_PROBE
#include <cstdlib>
static inline long vc_knob(const char* env, long dflt) {
  const char* e = getenv(env);
  return e ? atol(e) : dflt;
}
#else
static inline long vc_knob(const char*, long dflt) { return dflt; }
#endif

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

// Division by a launch-time constant without the integer-divide sequence: q = (mulhi(n, mul) + n) >> shr,
// exact for 0 <= n < 2^31 and any divisor >= 1 (Granlund-Montgomery round-up multiplier).  Elementwise
// kernels index with 32-bit ints (every tensor of the step has < 2^31 elements; checked on the host).
struct FastDiv {
  uint32_t div, mul, shr;
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.div = d;
  uint32_t p = 0;
  while ((1ull << p) < d) ++p;
  f.shr = p;
  f.mul = (uint32_t)((((1ull << p) - d) << 32) / d + 1);
  return f;
}

__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)((__umulhi((uint32_t)n, f.mul) + (uint32_t)n) >> f.shr);
}

// n = q * div + r
__device__ __forceinline__ int fdivmod(int n, const FastDiv& f, int& r) {
  const int q = fdiv(n, f);
  r = n - q * (int)f.div;
  return q;
}

#define VC_REQUIRE_I32(n) VC_REQUIRE((long)(n) < (1L << 31))

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

// DPP (data-parallel primitives) lane moves within 16-lane rows: VALU ops, no LDS crossbar.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// sum over each aligned 16-lane row, result in every lane of the row:
// quad_perm[1,0,3,2] -> quad_perm[2,3,0,1] -> row_half_mirror -> row_mirror
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return v;
}

// sum over the 4 rows of a wave for every column (lane & 15): v + v^16 + v^32 + v^48, all lanes get
// the result.  gfx950 v_permlane16_swap / v_permlane32_swap are VALU half-exchanges, so this costs
// two VALU swaps + adds instead of two ds_bpermute round trips through the LDS crossbar.  Summation
// order equals __shfl_xor(16) then __shfl_xor(32) (bit-identical).
__device__ __forceinline__ float cross_row_sum(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto p = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
  const unsigned w = __builtin_bit_cast(unsigned, v);
  const auto q = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return __builtin_bit_cast(float, (unsigned)q[0]) + __builtin_bit_cast(float, (unsigned)q[1]);
}

// cross_row_sum of two values at once (both totals in every lane, each bit-identical to
// cross_row_sum): permlane16_swap(a, b) leaves rows [a0, b0, a2, b2] / [a1, b1, a3, b3], whose sum
// holds a's row-pair sums in rows 0 / 2 and b's in rows 1 / 3; a permlane32_swap of that with itself
// adds the halves ([A, B, A, B]), and a final permlane16_swap of the result with itself hands every
// lane A in the first register and B in the second: 3 swaps + 2 adds instead of 4 + 4.
__device__ __forceinline__ void cross_row_sum2(float& a, float& b) {
  const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                                                  false, false);
  const float x = __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
  const unsigned ux = __builtin_bit_cast(unsigned, x);
  const auto q = __builtin_amdgcn_permlane32_swap(ux, ux, false, false);
  const float y = __builtin_bit_cast(float, (unsigned)q[0]) + __builtin_bit_cast(float, (unsigned)q[1]);
  const unsigned uy = __builtin_bit_cast(unsigned, y);
  const auto r = __builtin_amdgcn_permlane16_swap(uy, uy, false, false);
  a = __builtin_bit_cast(float, (unsigned)r[0]);
  b = __builtin_bit_cast(float, (unsigned)r[1]);
}

// Reduce-scatter of 4 per-lane values over the 4 rows of a wave: lane (row r, column c) returns
// v_r summed over the 4 rows at column c, in cross_row_sum's order ((r0 + r1) + (r2 + r3)), so each
// total is bit-identical to cross_row_sum(v_r).  permlane16_swap(v0, v1) + add leaves v0's row-pair
// sums in the even rows and v1's in the odd rows (likewise v2 / v3); a permlane32_swap of the two
// results + add completes row r's value r: 3 swaps + 3 adds for four totals instead of 8 + 8.
__device__ __forceinline__ float row_scatter4(float v0, float v1, float v2, float v3) {
  const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v0), __builtin_bit_cast(unsigned, v1),
                                                  false, false);
  const float x01 = __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
  const auto q = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v2), __builtin_bit_cast(unsigned, v3),
                                                  false, false);
  const float x23 = __builtin_bit_cast(float, (unsigned)q[0]) + __builtin_bit_cast(float, (unsigned)q[1]);
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x01), __builtin_bit_cast(unsigned, x23),
                                                  false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

// max over the 4 rows of a wave for every column (lane & 15), all lanes get it: the permlane16 /
// permlane32 half swaps of cross_row_sum with fmaxf (exact, so identical to the __shfl_xor form)
__device__ __forceinline__ float cross_row_max(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto p = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  v = fmaxf(__builtin_bit_cast(float, (unsigned)p[0]), __builtin_bit_cast(float, (unsigned)p[1]));
  const unsigned w = __builtin_bit_cast(unsigned, v);
  const auto q = __builtin_amdgcn_permlane32_swap(w, w, false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)q[0]), __builtin_bit_cast(float, (unsigned)q[1]));
}

// a[r] for the lane's row r = lane >> 4 (register selects, no memory)
__device__ __forceinline__ float row_select4(const float (&a)[4], int r) {
  return r == 0 ? a[0] : (r == 1 ? a[1] : (r == 2 ? a[2] : a[3]));
}

// In-launch "last arriver" of a group of n blocks that each published a partial result (the split-K
// combine's protocol, cdna_hip_programming.md "In-launch split-K reduction"): the block's global
// stores are drained and released at agent scope, thread 0 takes a ticket from *cnt; the block that
// draws the last ticket re-zeroes *cnt (all n have arrived, so the next launch on this stream finds it
// zero), acquires the others' partials and returns true in every thread.  The partials are then
// reduced in a fixed order by the caller, so the result does not depend on which block came last.
// Call from all threads of the block (contains barriers).
__device__ __forceinline__ bool block_last_arriver(unsigned int* cnt, unsigned n) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == n - 1);
    if (last) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return last != 0;
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

// out[c] = beta*out[c] + sum_{p<P} part[p*stride + off + c]
// block = 16 columns x 16 partial lanes: coalesced 64-B row segments, 16 independent load streams
// per column, fixed-order LDS combine (deterministic).
static __global__ __launch_bounds__(256) void sum_rows_kernel(int P, int C, const float* __restrict__ part, long stride,
                                                              long off, float* __restrict__ out, float beta) {
  __shared__ float sh[16][17];
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int p = pl; p < P; p += 16) s += part[(long)p * stride + off + c];
  }
  sh[pl][cl] = s;
  __syncthreads();
  if (pl == 0 && c < C) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) v += sh[i][cl];
    out[c] = (beta != 0.f ? beta * out[c] : 0.f) + v;
  }
}

static inline int launch_sum_rows(int P, int C, const float* part, long stride, long off, float* out, float beta,
                                  hipStream_t stream) {
  if (C <= 0) return 0;
  hipLaunchKernelGGL(sum_rows_kernel, dim3((C + 15) / 16), dim3(256), 0, stream, P, C, part, stride, off, out, beta);
  return (int)hipGetLastError();
}
