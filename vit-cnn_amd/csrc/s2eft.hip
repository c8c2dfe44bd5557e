// S2EFT comparison model (config 5): the ops vc_gemm / vc_layernorm do
// not already cover.  Reference: model/compare_method/S2EFT.py
//   spectral gate            :134-143  sigmoid(conv1d_k7([mean_c, max_c])) >= 0.4 -> hard 0/1 mask
//   embedding + cls + pos    :146-153
//   4-head attention core    :45-74    softmax(q k^T * dim_head^-0.5) v, dim_head 16
//   GELU MLP                 :21-32    nn.GELU (erf form)
//   CAF skipcat              :88-106   Conv2d(T, T, [1, 2]) over cat(x, last_output[nl-2]) on a new axis
// Token rows are [B, T, D] row-major (token-major, the reference's [b, n, dim] layout); the qkv
// projection output is [B*T, 3*H*16] (q | k | v column blocks, head h at columns h*16.. of each).
#include "common.h"

namespace {

// ------------------------------------------------------------------ spectral gate
// Blocks (sample, 1/8 of its rows): each recomputes the sample's statistics (L2-resident).  Per token row: mean and max over C (one wave per row), then the k=7 conv over
// the token axis (zero padded), sigmoid, threshold; xg = x * mask (the mask is `.data`: no gradient).
__global__ __launch_bounds__(512) void gate_fwd(int N, int C, const float* __restrict__ x,
                                                const float* __restrict__ w, const float* __restrict__ bias,
                                                float beta, float* __restrict__ xg, float* __restrict__ mask) {
  extern __shared__ float sh[];
  float* avg = sh;
  float* mx = sh + N;
  float* msk = sh + 2 * N;
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* xb = x + (long)b * N * C;
  // GR rows per wave at a time (rows r, r + 8, ...): their loads are in flight together and their
  // reductions interleave; each row's sum / max keep the one-row order (bit-identical)
  constexpr int GR = 4, CV = 4;   // CV: a lane's channels per row held in registers (C <= 256)
  for (int r0 = wave; r0 < N; r0 += 8 * GR) {
    float v[GR][CV];
#pragma unroll
    for (int g = 0; g < GR; ++g)
#pragma unroll
      for (int j = 0; j < CV; ++j) {
        const int r = r0 + 8 * g, c = lane + 64 * j;
        v[g][j] = (r < N && c < C) ? xb[(long)r * C + c] : 0.f;
      }
    float s[GR], m[GR];
#pragma unroll
    for (int g = 0; g < GR; ++g) {
      s[g] = 0.f;
      m[g] = -INFINITY;
#pragma unroll
      for (int j = 0; j < CV; ++j)
        if (lane + 64 * j < C) {
          s[g] += v[g][j];
          m[g] = fmaxf(m[g], v[g][j]);
        }
      for (int c = lane + 64 * CV; c < C; c += 64) {   // channels beyond 64 * CV (not at config 5)
        const float vv = r0 + 8 * g < N ? xb[(long)(r0 + 8 * g) * C + c] : 0.f;
        s[g] += vv;
        m[g] = fmaxf(m[g], vv);
      }
    }
#pragma unroll
    for (int g = 0; g < GR; ++g) {
      s[g] = wave_sum(s[g]);
      m[g] = wave_max(m[g]);
    }
    if (lane == 0) {
#pragma unroll
      for (int g = 0; g < GR; ++g)
        if (r0 + 8 * g < N) {
          avg[r0 + 8 * g] = s[g] / (float)C;
          mx[r0 + 8 * g] = m[g];
        }
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < N; t += 512) {
    float v = bias[0];
    for (int k = 0; k < 7; ++k) {
      const int j = t + k - 3;
      if (j >= 0 && j < N) v += w[k] * avg[j] + w[7 + k] * mx[j];
    }
    const float s = 1.0f / (1.0f + expf(-v));
    const float m = s >= beta ? 1.0f : 0.0f;
    msk[t] = m;
    if (blockIdx.y == 0) mask[(long)b * N + t] = m;
  }
  __syncthreads();
  float* xgb = xg + (long)b * N * C;
  const int per = (N * C + gridDim.y - 1) / gridDim.y;
  const int end = min(N * C, per * ((int)blockIdx.y + 1));
  for (int i = per * blockIdx.y + threadIdx.x; i < end; i += 512) xgb[i] = xb[i] * msk[i / C];
}

// X[b, 0, :] = cls + pos[0]  (the other rows come from the embedding GEMM with pos fused as addend)
__global__ void cls_rows(int B, int T, int D, const float* __restrict__ cls, const float* __restrict__ pos,
                         float* __restrict__ X) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * D) return;
  const int b = i / D, d = i % D;
  X[(long)b * T * D + d] = cls[d] + pos[d];
}

// dE[b, t, :] = dX[b, 1 + t, :]
__global__ void strip_cls(int B, int N, int D, const float* __restrict__ dX, float* __restrict__ dE) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * N * D) return;
  const long b = i / ((long)N * D), r = i % ((long)N * D);
  dE[i] = dX[b * (N + 1) * D + D + r];
}

// ------------------------------------------------------------------ attention core (dim_head 16)
constexpr float ATT_LOG2E = 1.4426950408889634f;
constexpr float ATT_LN2 = 0.6931471805599453f;
// One block per (b, h) with ceil(T/16) waves (256 blocks x 10 waves at config 5), so the head's K/V (and
// for the backward Q, dO, lse, rowsum(dO*O)) are staged into LDS (sized to T) once per head.  P is never stored: the forward saves lse per row.
// Forward on the matrix cores (v_mfma_f32_16x16x4_f32).  A wave owns 16 queries of one (b, h) and walks
// the keys in 16-key tiles, computing S^T = K Q^T (so the scores of one query sit in the four
// registers of the four lanes l, l^16, l^32, l^48 that share l & 15) and O^T += V^T P^T, whose B
// operand is P^T straight from the S^T accumulator: the k order inside each MFMA is permuted so that
// step s of lane group g = l >> 4 pairs key (or head-dim) 4g + s on both operands.  Online softmax
// (running max / sum per query, rescaling the O^T accumulator) between tiles.
__global__ __launch_bounds__(1024) void attn_fwd(int T, int H, const float* __restrict__ qkv, float scale,
                                                float* __restrict__ out, float* __restrict__ lse, int wpb) {
  extern __shared__ f32x4 lds4[];  // 2 * T * 64 B
  f32x4* Ks = lds4;
  f32x4* Vs = lds4 + T * 4;
  const float* Vf = (const float*)Vs;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int ld = 3 * H * 16, ldo = H * 16;
  const float* base = qkv + (long)b * T * ld;
  for (int i = threadIdx.x; i < T * 4; i += blockDim.x) {
    const int t = i >> 2, q4 = i & 3;
    Ks[i] = *(const f32x4*)(base + (long)t * ld + H * 16 + h * 16 + q4 * 4);
    Vs[i] = *(const f32x4*)(base + (long)t * ld + 2 * H * 16 + h * 16 + q4 * 4);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q0 = (blockIdx.y * wpb + wave) * 16;   // blockIdx.y: chunk of wpb waves
  if (q0 >= T) return;                     // whole wave idle (no LDS barrier follows)
  const int c = lane & 15, g = lane >> 4;
  const int qi = min(q0 + c, T - 1);
  // B operand of S^T: Q^T[d = 4g + s][q = c]
  const f32x4 qv = *(const f32x4*)(base + (long)qi * ld + h * 16 + g * 4);
  // softmax in the base-2 domain: scores pre-scaled by log2(e), so every exponential is one v_exp_f32
  // (expf's range reduction would cost ~10 VALU per score); lse is stored in natural log as before
  const float scale2 = scale * ATT_LOG2E;
  float m = -INFINITY, l = 0.f;
  f32x4 o = {0.f, 0.f, 0.f, 0.f};          // O^T[d = 4g + r][q = c]
  for (int k0 = 0; k0 < T; k0 += 16) {
    const int key = min(k0 + c, T - 1);
    const f32x4 kv = Ks[key * 4 + g];      // A operand: K[key = k0 + c][d = 4g + s]
    f32x4 st = {0.f, 0.f, 0.f, 0.f};       // S^T[key = k0 + 4g + r][q = c]
    st = __builtin_amdgcn_mfma_f32_16x16x4f32(kv.x, qv.x, st, 0, 0, 0);
    st = __builtin_amdgcn_mfma_f32_16x16x4f32(kv.y, qv.y, st, 0, 0, 0);
    st = __builtin_amdgcn_mfma_f32_16x16x4f32(kv.z, qv.z, st, 0, 0, 0);
    st = __builtin_amdgcn_mfma_f32_16x16x4f32(kv.w, qv.w, st, 0, 0, 0);
    float sv[4];
    float tm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sv[r] = (k0 + 4 * g + r < T) ? st[r] * scale2 : -INFINITY;
      tm = fmaxf(tm, sv[r]);
    }
    tm = cross_row_max(tm);
    const float mn = fmaxf(m, tm);
    const float corr = (m == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(m - mn);
    m = mn;
    float pv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      pv[r] = (sv[r] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(sv[r] - mn);
      l = l * (r == 0 ? corr : 1.f) + pv[r];
    }
    o *= corr;
    // O^T += V^T P^T: step s, group g pairs key k0 + 4g + s; A = V[key][d = c], B = P^T (register s)
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int kk = min(k0 + 4 * g + s2, T - 1);
      o = __builtin_amdgcn_mfma_f32_16x16x4f32(Vf[kk * 16 + c], pv[s2], o, 0, 0, 0);
    }
  }
  l = cross_row_sum(l);   // same order as the xor-16 then xor-32 shuffles
  if (q0 + c >= T) return;
  const float rl = 1.0f / l;
  *(f32x4*)(out + ((long)b * T + q0 + c) * ldo + h * 16 + g * 4) = o * rl;
  if (g == 0) lse[((long)b * H + h) * T + q0 + c] = m * ATT_LN2 + logf(l);
}

// Backward on MFMA, same tile scheme as the forward.  dS = P * (dP - rowsum(dO*O)), P recomputed
// from lse.  Pass 1: a wave owns 16 queries and walks 16-key tiles: S^T = K Q^T, dP^T = V dO^T,
// dQ^T += K^T dS^T.  Pass 2: the wave owns 16 keys and walks 16-query tiles: S = Q K^T, dP = dO V^T,
// dV^T += dO^T P, dK^T += Q^T dS (P / dS taken from the accumulators as B operands).  The two passes run
// in two blocks per head (blockIdx.y), each staging the head: 2 x B*H blocks of T/16 waves keep twice
// the waves per SIMD of one block doing both passes; the accumulations alternate between two
// accumulators per output tile (even / odd tiles) so consecutive tiles' MFMA chains overlap.
__device__ __forceinline__ f32x4 mfma4(f32x4 a, f32x4 b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, c, 0, 0, 0);
  return c;
}

// Grid (B*H, 2, chunks): blockIdx.y = pass, blockIdx.z = chunk of wpb waves (rows (z wpb + wave) * 16).
__global__ __launch_bounds__(1024) void attn_bwd(int T, int H, const float* __restrict__ qkv,
                                                const float* __restrict__ out, const float* __restrict__ dout,
                                                const float* __restrict__ lse, float scale,
                                                float* __restrict__ dqkv, int wpb) {
  extern __shared__ f32x4 lds4[];  // 2 * T * 64 B + 2 * T * 4 B (19.8 KB at T = 146)
  f32x4* Ks = lds4;                // pass 1
  f32x4* Vs = lds4 + T * 4;
  f32x4* Qs = lds4;                // pass 2 (the same bytes)
  f32x4* dOs = lds4 + T * 4;
  float* Ls = (float*)(lds4 + 2 * T * 4);
  float* Ds = Ls + T;
  const float* Qf = (const float*)Qs;
  const float* Kf = (const float*)Ks;
  const float* dOf = (const float*)dOs;
  const int b = blockIdx.x / H, h = blockIdx.x % H;
  const int ld = 3 * H * 16, ldo = H * 16;
  const float* base = qkv + (long)b * T * ld;
  // the operands the pass walks staged (pass 1: K, V; pass 2: Q, dO; each pass reads its own 16 rows of
  // the other two straight from global memory) with (pass 2) rowsum(dO * O) in the same loop: 4 lanes per row (one
  // float4 of each array), every load of a lane issued before its first use; the row's four dot products
  // summed across the lanes (xor 1, xor 2)
  const bool p1 = blockIdx.y == 0;
  for (int i0 = 0; i0 < T * 4; i0 += blockDim.x) {   // uniform trip count: the shuffles see whole rows
    const int i = i0 + threadIdx.x;
    const bool ok = i < T * 4;
    const int t = ok ? i >> 2 : 0, q4 = i & 3;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    const f32x4 av = ok ? *(const f32x4*)(base + (long)t * ld + (p1 ? H * 16 : 0) + h * 16 + q4 * 4) : z;
    const f32x4 vv = (ok && p1) ? *(const f32x4*)(base + (long)t * ld + 2 * H * 16 + h * 16 + q4 * 4) : z;
    const f32x4 gv = (ok && !p1) ? *(const f32x4*)(dout + ((long)b * T + t) * ldo + h * 16 + q4 * 4) : z;
    const f32x4 ov = (ok && !p1) ? *(const f32x4*)(out + ((long)b * T + t) * ldo + h * 16 + q4 * 4) : z;
    const float lt = (ok && !p1 && q4 == 0) ? lse[((long)b * H + h) * T + t] : 0.f;
    if (ok) {
      if (p1) {
        Ks[i] = av;
        Vs[i] = vv;
      } else {
        Qs[i] = av;
        dOs[i] = gv;
      }
    }
    float v = fmaf(ov.w, gv.w, fmaf(ov.z, gv.z, fmaf(ov.y, gv.y, ov.x * gv.x)));   // explicit fmas: pass 1's bits
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    if (ok && !p1 && q4 == 0) {
      Ds[t] = v;
      Ls[t] = lt * ATT_LOG2E;   // base-2 lse
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = (blockIdx.z * wpb + wave) * 16;
  if (r0 >= T) return;
  const int c = lane & 15, g = lane >> 4;
  const int ri = min(r0 + c, T - 1);
  if (blockIdx.y == 0) {  // pass 1: dq of queries r0 .. r0 + 15 (query c of this lane)
    const f32x4 qv = *(const f32x4*)(base + (long)ri * ld + h * 16 + g * 4);
    const f32x4 gv = *(const f32x4*)(dout + ((long)b * T + ri) * ldo + h * 16 + g * 4);
    const f32x4 ov = *(const f32x4*)(out + ((long)b * T + ri) * ldo + h * 16 + g * 4);
    const float scale2 = scale * ATT_LOG2E;
    // this query's lse and rowsum(dO * O): pass 1 stages neither; the staging loop's operations and order
    // (explicit fmas, lane group g in the role of q4: xor 16, xor 32 for xor 1, xor 2), so the bits are pass 2's
    const float lq = lse[((long)b * H + h) * T + ri] * ATT_LOG2E;
    float dq_ = fmaf(ov.w, gv.w, fmaf(ov.z, gv.z, fmaf(ov.y, gv.y, ov.x * gv.x)));
    dq_ += __shfl_xor(dq_, 16, 64);
    dq_ += __shfl_xor(dq_, 32, 64);
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;  // dQ^T[d = 4g + r][q = c], even / odd tiles
    auto tile = [&](int k0, f32x4& acc) {
      const int key = min(k0 + c, T - 1);
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 st = mfma4(Ks[key * 4 + g], qv, z);   // S^T[key = k0 + 4g + r][q = c]
      const f32x4 dpt = mfma4(Vs[key * 4 + g], gv, z);  // dP^T
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const bool valid = k0 + 4 * g + r < T;
        const float p = valid ? __builtin_amdgcn_exp2f(fmaf(st[r], scale2, -lq)) : 0.f;
        ds[r] = p * (dpt[r] - dq_);
      }
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int kk = min(k0 + 4 * g + s2, T - 1);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Kf[kk * 16 + c], ds[s2], acc, 0, 0, 0);
      }
    };
    int k0 = 0;
    for (; k0 + 16 < T; k0 += 32) {
      tile(k0, acc0);
      tile(k0 + 16, acc1);
    }
    if (k0 < T) tile(k0, acc0);
    if (r0 + c < T) *(f32x4*)(dqkv + ((long)b * T + r0 + c) * ld + h * 16 + g * 4) = (acc0 + acc1) * scale;
  } else {  // pass 2: dk, dv of keys r0 .. r0 + 15 (key c of this lane)
    const f32x4 kv = *(const f32x4*)(base + (long)ri * ld + H * 16 + h * 16 + g * 4);
    const f32x4 vv = *(const f32x4*)(base + (long)ri * ld + 2 * H * 16 + h * 16 + g * 4);
    const float scale2 = scale * ATT_LOG2E;
    // dK^T / dV^T [d = 4g + r][key = c], even / odd query tiles
    f32x4 adk0 = {0.f, 0.f, 0.f, 0.f}, adk1 = adk0, adv0 = adk0, adv1 = adk0;
    auto tile = [&](int q0, f32x4& adk, f32x4& adv) {
      const int qq = min(q0 + c, T - 1);
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 sm = mfma4(Qs[qq * 4 + g], kv, z);    // S[q = q0 + 4g + r][key = c]
      const f32x4 dp = mfma4(dOs[qq * 4 + g], vv, z);   // dP
      float pr[4], ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int q = q0 + 4 * g + r;
        const bool valid = q < T;
        const int qc = valid ? q : T - 1;
        const float p = valid ? __builtin_amdgcn_exp2f(fmaf(sm[r], scale2, -Ls[qc])) : 0.f;
        pr[r] = p;
        ds[r] = p * (dp[r] - Ds[qc]);
      }
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int qk = min(q0 + 4 * g + s2, T - 1);
        adv = __builtin_amdgcn_mfma_f32_16x16x4f32(dOf[qk * 16 + c], pr[s2], adv, 0, 0, 0);
        adk = __builtin_amdgcn_mfma_f32_16x16x4f32(Qf[qk * 16 + c], ds[s2], adk, 0, 0, 0);
      }
    };
    int q0 = 0;
    for (; q0 + 16 < T; q0 += 32) {
      tile(q0, adk0, adv0);
      tile(q0 + 16, adk1, adv1);
    }
    if (q0 < T) tile(q0, adk0, adv0);
    if (r0 + c < T) {
      float* w = dqkv + ((long)b * T + r0 + c) * ld + h * 16 + g * 4;
      *(f32x4*)(w + H * 16) = (adk0 + adk1) * scale;
      *(f32x4*)(w + 2 * H * 16) = adv0 + adv1;
    }
  }
}

// ------------------------------------------------------------------ GELU (erf form, nn.GELU default)
__global__ void gelu_fwd(long n, const float* __restrict__ x, float* __restrict__ y) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  y[i] = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
}

__global__ void gelu_bwd(long n, const float* __restrict__ dy, const float* __restrict__ x, float* __restrict__ dx) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  const float cdf = 0.5f * (1.0f + erff(v * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * expf(-0.5f * v * v);
  dx[i] = dy[i] * (cdf + v * pdf);
}

// ------------------------------------------------------------------ CAF skipcat
// Z[b, i, k, :] = (k == 0 ? x : last)[b, i, :]  (the Conv2d(T, T, [1, 2]) input as a [2T, D] matrix
// whose row i*2+k meets weight column i*2+k); biasmat[o, :] = bias[o] (the GEMM's row addend).
__global__ void skip_pack(int B, int T, int D, const float* __restrict__ x, const float* __restrict__ last,
                          const float* __restrict__ bias, float* __restrict__ Z, float* __restrict__ biasmat) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = (long)B * T * D;
  if (i < (long)T * D) biasmat[i] = bias[i / D];
  if (i >= n) return;
  const long row = i / D, d = i % D;  // row = b*T + t
  Z[(row * 2) * D + d] = x[i];
  Z[(row * 2 + 1) * D + d] = last[i];
}

// dx (=/+=) dZ[:, :, 0, :] (+ addx); dlast = dZ[:, :, 1, :]
__global__ void skip_unpack(int B, int T, int D, const float* __restrict__ dZ, float* __restrict__ dx, int acc_x,
                            const float* __restrict__ addx, float* __restrict__ dlast) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long)B * T * D) return;
  const long row = i / D, d = i % D;
  float a = dZ[(row * 2) * D + d];
  if (addx) a = a + addx[i];
  dx[i] = acc_x ? dx[i] + a : a;
  dlast[i] = dZ[(row * 2 + 1) * D + d];
}

// dbias[o] = sum_{b, d} dY[b, o, d]  (one block per o)
__global__ __launch_bounds__(256) void skip_bias_grad(int B, int T, int D, const float* __restrict__ dY,
                                                      float* __restrict__ db) {
  __shared__ float sh[8];
  const int o = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < B * D; i += 256) {
    const int b = i / D, d = i % D;
    s += dY[((long)b * T + o) * D + d];
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) db[o] = sh[0] + sh[1] + sh[2] + sh[3];
}

// ------------------------------------------------------------------ dropout (nn.Dropout, train mode)
// keep_i = u_i >= p with u_i = hash(seed, i) / 2^32 (counter-based: no RNG state on the device);
// y = add + keep * x * (1 / (1 - p)); the keep mask is saved as bytes for the backward.
__device__ __forceinline__ uint32_t mix32(uint64_t seed, uint32_t i) {
  uint64_t z = seed ^ ((uint64_t)i * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}

__global__ void dropout_fwd(int n, const float* __restrict__ x, const float* __restrict__ add, float* __restrict__ y,
                            unsigned char* __restrict__ mask, float p, float scale, unsigned long long seed) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float u = (float)(mix32(seed, (uint32_t)i) >> 8) * (1.0f / 16777216.0f);
  const bool keep = u >= p;
  const float v = keep ? x[i] * scale : 0.f;
  y[i] = add ? add[i] + v : v;
  mask[i] = keep ? 1 : 0;
}

__global__ void dropout_bwd(int n, const float* __restrict__ dy, const unsigned char* __restrict__ mask, float scale,
                            float* __restrict__ dx) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dx[i] = mask[i] ? dy[i] * scale : 0.f;
}

}  // namespace

VC_API int vc_dropout_fwd(long n, const float* x, const float* add, float* y, unsigned char* mask, float p,
                          unsigned long long seed, hipStream_t stream) {
  VC_REQUIRE(n >= 0 && p >= 0.f && p < 1.f);
  VC_REQUIRE_I32(n);
  if (n == 0) return VC_OK;
  hipLaunchKernelGGL(dropout_fwd, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, (int)n, x, add, y, mask, p,
                     1.0f / (1.0f - p), seed);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_dropout_bwd(long n, const float* dy, const unsigned char* mask, float p, float* dx, hipStream_t stream) {
  VC_REQUIRE(n >= 0 && p >= 0.f && p < 1.f);
  VC_REQUIRE_I32(n);
  if (n == 0) return VC_OK;
  hipLaunchKernelGGL(dropout_bwd, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, (int)n, dy, mask, 1.0f / (1.0f - p), dx);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_s2eft_gate_fwd(int B, int N, int C, const float* x, const float* w, const float* bias, float beta,
                             float* xg, float* mask, hipStream_t stream) {
  VC_REQUIRE(B > 0 && N > 0 && C > 0 && N <= 4096);
  VC_REQUIRE_I32((long)N * C);
  hipLaunchKernelGGL(gate_fwd, dim3(B, 8), dim3(512), 3 * N * sizeof(float), stream, N, C, x, w, bias, beta, xg, mask);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_s2eft_cls_rows(int B, int T, int D, const float* cls, const float* pos, float* X, hipStream_t stream) {
  VC_REQUIRE(B > 0 && T > 0 && D > 0);
  hipLaunchKernelGGL(cls_rows, dim3(vc_cdiv((long)B * D, 256)), dim3(256), 0, stream, B, T, D, cls, pos, X);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_s2eft_strip_cls(int B, int N, int D, const float* dX, float* dE, hipStream_t stream) {
  VC_REQUIRE(B > 0 && N > 0 && D > 0);
  hipLaunchKernelGGL(strip_cls, dim3(vc_cdiv((long)B * N * D, 256)), dim3(256), 0, stream, B, N, D, dX, dE);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_s2eft_attn_fwd(int B, int T, int H, const float* qkv, float scale, float* out, float* lse,
                             hipStream_t stream) {
  VC_REQUIRE(B > 0 && H > 0 && T > 0 && T <= 256);
  const int waves = (T + 15) / 16;
  const int wpb = std::max(1, std::min(waves, (int)vc_knob("VITCNN_ATTN_FWD_WPB", waves)));   // knob: probe library
  hipLaunchKernelGGL(attn_fwd, dim3(B * H, vc_cdiv(waves, wpb)), dim3(64 * wpb), 2 * T * 64, stream, T, H, qkv, scale,
                     out, lse, wpb);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_s2eft_attn_bwd(int B, int T, int H, const float* qkv, const float* out, const float* dout,
                             const float* lse, float scale, float* dqkv, hipStream_t stream) {
  VC_REQUIRE(B > 0 && H > 0 && T > 0 && T <= 256);
  // waves per block: ceil(waves / 2) (config 5: 2 blocks of 5 waves per pass and head: 24.0 -> 22.2 us with
  // pass 1's lighter staging, tools/attn_probe.py, profiles/r05_attn_bwd.log); knob: probe library
  const int waves = (T + 15) / 16;
  const int wpb = std::max(1, std::min(waves, (int)vc_knob("VITCNN_ATTN_BWD_WPB", (waves + 1) / 2)));
  hipLaunchKernelGGL(attn_bwd, dim3(B * H, 2, vc_cdiv(waves, wpb)), dim3(64 * wpb), 2 * T * 64 + 2 * T * 4, stream, T,
                     H, qkv, out, dout, lse, scale, dqkv, wpb);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_gelu_fwd(long n, const float* x, float* y, hipStream_t stream) {
  VC_REQUIRE(n >= 0);
  if (n == 0) return VC_OK;
  hipLaunchKernelGGL(gelu_fwd, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, n, x, y);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_gelu_bwd(long n, const float* dy, const float* x, float* dx, hipStream_t stream) {
  VC_REQUIRE(n >= 0);
  if (n == 0) return VC_OK;
  hipLaunchKernelGGL(gelu_bwd, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, n, dy, x, dx);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_s2eft_skip_pack(int B, int T, int D, const float* x, const float* last, const float* bias, float* Z,
                              float* biasmat, hipStream_t stream) {
  VC_REQUIRE(B > 0 && T > 0 && D > 0);
  hipLaunchKernelGGL(skip_pack, dim3(vc_cdiv((long)B * T * D, 256)), dim3(256), 0, stream, B, T, D, x, last, bias,
                     Z, biasmat);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_s2eft_skip_unpack(int B, int T, int D, const float* dZ, float* dx, int acc_x, const float* addx,
                                float* dlast, hipStream_t stream) {
  VC_REQUIRE(B > 0 && T > 0 && D > 0);
  hipLaunchKernelGGL(skip_unpack, dim3(vc_cdiv((long)B * T * D, 256)), dim3(256), 0, stream, B, T, D, dZ, dx, acc_x,
                     addx, dlast);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_s2eft_skip_bias_grad(int B, int T, int D, const float* dY, float* db, hipStream_t stream) {
  VC_REQUIRE(B > 0 && T > 0 && D > 0);
  hipLaunchKernelGGL(skip_bias_grad, dim3(T), dim3(256), 0, stream, B, T, D, dY, db);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
