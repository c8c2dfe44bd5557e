// LayerNorm and BatchNorm (train + eval) for channels-last activations [rows, C].
//
// LayerNorm(eps=1e-6) rows: hsiMamba pre_norm / ln1 (Mutimodality_Mamba7.py:349, :353,
// applied at :656, :985), GlobalLocalBlock ln3 / ln4 (:1069, :1073).  One wave64 per row,
// shuffle reductions, two-pass variance.
// BatchNorm2d (eps 1e-5, momentum 0.1): ms_conv_bn_relu.bn (:1039), FusionLayer BN (:1103,
// :1129), NonLocal W[1] (:113).  Train mode normalises with the biased batch variance over
// all rows (B*H*W) and updates running_var with the unbiased one; eval mode uses the
// running statistics.  Reductions are deterministic (fixed-order partials + Chan merge).
#include "common.h"

namespace {

constexpr int LN_MAXV = 8;  // C <= 512
constexpr int NB = 8;       // rows (or partials) per lane whose loads a BatchNorm kernel issues together
// row lanes of the BatchNorm statistics / apply blocks (64 channels x BN_RL rows per block): 16 puts the
// ~80 rows of a B = 64 partial one batch of loads per lane (4 lanes: three dependent rounds of 8)
#ifndef VC_BN_RL
#define VC_BN_RL 16
#endif
constexpr int BN_RL = VC_BN_RL, BN_T = 64 * BN_RL;

__global__ __launch_bounds__(256) void ln_fwd(int R, int C, const float* __restrict__ x, long ldx,
                                              const float* __restrict__ w, const float* __restrict__ b, float eps,
                                              float* __restrict__ y, long ldy, float* __restrict__ mean_out,
                                              float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* xr = x + r * ldx;
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    int c = lane + 64 * j;
    v[j] = (c < C) ? xr[c] : 0.f;
    s += v[j];
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    int c = lane + 64 * j;
    float d = (c < C) ? v[j] - mean : 0.f;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
  float* yr = y + r * ldy;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    int c = lane + 64 * j;
    if (c < C) yr[c] = (v[j] - mean) * rstd * w[c] + b[c];
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w ; per-block partial dw / db.
// The result goes to dx as res + v (res given: a residual gradient read from another buffer) or
// beta_dx * dx + v.
__global__ __launch_bounds__(256) void ln_bwd(int R, int C, int rows_per_block, const float* __restrict__ dy,
                                              long lddy, const float* __restrict__ x, long ldx,
                                              const float* __restrict__ w, const float* __restrict__ mean,
                                              const float* __restrict__ rstd, float* __restrict__ dx, long lddx,
                                              float beta_dx, const float* __restrict__ res, long ldr,
                                              float* __restrict__ part) {
  __shared__ float sh[4][2][512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float pw[LN_MAXV], pb[LN_MAXV];
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) pw[j] = pb[j] = 0.f;
  const long rbeg = (long)blockIdx.x * rows_per_block;
  const long rend = min((long)R, rbeg + rows_per_block);
  // two rows (r, r + 4) per iteration: both rows' loads and both pairs of wave sums are independent,
  // so their latencies overlap; the partial dw / db take row r's terms before row r + 4's, as a
  // one-row loop would (bit-identical)
  for (long r = rbeg + wv; r < rend; r += 8) {
    const bool two = r + 4 < rend;
    const long r2 = two ? r + 4 : r;
    const float mu = mean[r], rs = rstd[r], mu2 = mean[r2], rs2 = rstd[r2];
    float xh[LN_MAXV], g[LN_MAXV], dd[LN_MAXV], xh2[LN_MAXV], g2[LN_MAXV], dd2[LN_MAXV];
    float sg = 0.f, sgx = 0.f, sg2 = 0.f, sgx2 = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAXV; ++j) {
      int c = lane + 64 * j;
      float d = 0.f, xv = 0.f, wc = 0.f, d2 = 0.f, xv2 = 0.f;
      if (c < C) {
        d = dy[r * lddy + c];
        xv = x[r * ldx + c];
        wc = w[c];
        d2 = dy[r2 * lddy + c];
        xv2 = x[r2 * ldx + c];
      }
      xh[j] = (xv - mu) * rs;
      g[j] = d * wc;
      dd[j] = d;
      sg += g[j];
      sgx += g[j] * xh[j];
      xh2[j] = (xv2 - mu2) * rs2;
      g2[j] = d2 * wc;
      dd2[j] = d2;
      sg2 += g2[j];
      sgx2 += g2[j] * xh2[j];
    }
    sg = wave_sum(sg) / C;
    sgx = wave_sum(sgx) / C;
    sg2 = wave_sum(sg2) / C;
    sgx2 = wave_sum(sgx2) / C;
#pragma unroll
    for (int j = 0; j < LN_MAXV; ++j) {
      pw[j] += dd[j] * xh[j];
      pb[j] += dd[j];
      if (two) {
        pw[j] += dd2[j] * xh2[j];
        pb[j] += dd2[j];
      }
    }
#pragma unroll
    for (int j = 0; j < LN_MAXV; ++j) {
      int c = lane + 64 * j;
      if (c < C) {
        float v = rs * (g[j] - sg - xh[j] * sgx);
        float* p = dx + r * lddx + c;
        *p = (res ? res[r * ldr + c] : (beta_dx != 0.f ? *p * beta_dx : 0.f)) + v;
        if (two) {
          float v2 = rs2 * (g2[j] - sg2 - xh2[j] * sgx2);
          float* p2 = dx + r2 * lddx + c;
          *p2 = (res ? res[r2 * ldr + c] : (beta_dx != 0.f ? *p2 * beta_dx : 0.f)) + v2;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    int c = lane + 64 * j;
    if (c < 512) {
      sh[wv][0][c] = pw[j];
      sh[wv][1][c] = pb[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = sh[0][0][c] + sh[1][0][c] + sh[2][0][c] + sh[3][0][c];
    float bb = sh[0][1][c] + sh[1][1][c] + sh[2][1][c] + sh[3][1][c];
    part[(long)blockIdx.x * 2 * C + c] = a;
    part[(long)blockIdx.x * 2 * C + C + c] = bb;
  }
}

// ---------------------------------------------------------------- BatchNorm (channels-last)
// Batch statistics as shifted sums in fp64 (torch's CPU kernels accumulate in double too): per
// channel s1 = sum (x - k), s2 = sum (x - k)^2 with the shift k = x[0, c] (the first row: keeps
// s2/M - (s1/M)^2 free of cancellation whatever the channel's offset), so mean = k + s1/M and the
// biased variance = s2/M - (s1/M)^2.  A partial block (64 channels x BN_RL row lanes) sums rows_per
// rows into part[p][2][C]; the reduction over the P partials runs in a fixed order (BN_RL partial lanes
// p = l, l+BN_RL, ..., then the lanes in order), either in the last-arriving partial block of each
// 64-channel group (tickets: no second launch) or in bn_stats_final (same code, same result).
// The elementwise BN arithmetic, spelled with explicit fmaf so that every kernel using it (separate or
// fused final + apply) rounds identically whatever the surrounding code lets the compiler contract.
__device__ __forceinline__ float bn_fwd_elem(float xv, float mean, float invstd, float w, float b) {
#pragma clang fp contract(off)
  return fmaf((xv - mean) * invstd, w, b);
}
// (fp contraction off inside: the caller's products a1 = s1 / M, a2 = s2 / M are never fused into the
// subtraction, whichever way the surrounding kernel hoists them): dx = w * invstd * (dyv - a1 - xhat * a2)
__device__ __forceinline__ float bn_bwd_elem(float d, float xv, float mean, float invstd, float w, float a1,
                                             float a2) {
#pragma clang fp contract(off)
  const float xh = (xv - mean) * invstd;
  return (w * invstd) * fmaf(-xh, a2, d - a1);
}
// dx = beta_dx * dx + v, the accumulation rounded once per element in every kernel
__device__ __forceinline__ void bn_dx_store(float* p, float beta_dx, float v) {
  *p = beta_dx != 0.f ? fmaf(beta_dx, *p, v) : v;
}

// The ReLU after a BatchNorm, for its backward: the decisions read from the forward's output (out, ld),
// or recomputed from x and the affine (w, b) with bn_fwd_elem -- the forward's own arithmetic on the same
// saved statistics, so the same decisions without reading the output; neither: no ReLU
struct ReluSrc {
  const float* out;
  long ld;
  const float* w;
  const float* b;
};

// The fixed-order reduction of the [P][2][C] fp64 partials of channel group cx (block = 64 channels x
// BN_RL partial lanes): on return (after a barrier) tot[0][cl] / tot[1][cl] hold channel cx*64+cl's two sums,
// visible to every thread of the block.  Every consumer (the separate final kernels and the fused
// apply kernels) sums in this one order, so their results agree bit for bit.
template <int T = BN_T>
__device__ __forceinline__ void bn_part_sums(int P, int C, const double* __restrict__ part, int cx,
                                             double (*tot)[64]) {
  // T threads = T / 64 real lanes, each computing BN_RL / (T / 64) of the BN_RL partial lanes in turn (the
  // same per-lane sums and combine order at any block size: bit-identical results)
  constexpr int RT = T / 64, VPT = BN_RL / RT;
  static_assert(RT * VPT == BN_RL, "block size");
  __shared__ double shr[2][BN_RL][64];
  const int cl = threadIdx.x & 63, pt = threadIdx.x >> 6;
  const int c = cx * 64 + cl;
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int pl = pt + RT * j;
    double s1 = 0.0, s2 = 0.0;
    if (c < C) {
      // NB partials per lane loaded before they are summed (one round of dependent loads per batch of
      // NB instead of one per 4); the sums keep the partial order
      for (int p0 = pl; p0 < P; p0 += BN_RL * NB) {
        double a[NB], bq[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int p = p0 + BN_RL * i;
          a[i] = p < P ? part[(long)p * 2 * C + c] : 0.0;
          bq[i] = p < P ? part[(long)p * 2 * C + C + c] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i)
          if (p0 + BN_RL * i < P) {
            s1 += a[i];
            s2 += bq[i];
          }
      }
    }
    shr[0][pl][cl] = s1;
    shr[1][pl][cl] = s2;
  }
  __syncthreads();
  if (pt == 0) {
    double t1 = shr[0][0][cl], t2 = shr[1][0][cl];
#pragma unroll
    for (int l = 1; l < BN_RL; ++l) {
      t1 += shr[0][l][cl];
      t2 += shr[1][l][cl];
    }
    tot[0][cl] = t1;
    tot[1][cl] = t2;
  }
  __syncthreads();
}

// mean / invstd of channel c from its sums (shift k = x[0, c]); writes save_* and the running stats
__device__ __forceinline__ void bn_stats_from_sums(double s1, double s2, int c, long M, const float* __restrict__ x,
                                                   float eps, float momentum, float& mean_f, float& invstd_f,
                                                   float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                                   float* __restrict__ run_mean, float* __restrict__ run_var,
                                                   bool write) {
  const double d = s1 / (double)M;
  const double var = fmax(s2 / (double)M - d * d, 0.0);
  const double mean = (double)x[c] + d;
  mean_f = (float)mean;
  invstd_f = (float)(1.0 / sqrt(var + (double)eps));
  if (!write) return;
  save_mean[c] = mean_f;
  save_invstd[c] = invstd_f;
  if (run_mean) {
    const double unb = M > 1 ? var * ((double)M / (double)(M - 1)) : var;
    run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mean);
    run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
  }
}

__device__ __forceinline__ void bn_stats_reduce(int P, int C, long M, const float* __restrict__ x,
                                                const double* __restrict__ part, int cx, float eps, float momentum,
                                                float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                                float* __restrict__ run_mean, float* __restrict__ run_var) {
  __shared__ double tot[2][64];
  bn_part_sums(P, C, part, cx, tot);
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int c = cx * 64 + cl;
  if (pl != 0 || c >= C) return;
  float mf, isf;
  bn_stats_from_sums(tot[0][cl], tot[1][cl], c, M, x, eps, momentum, mf, isf, save_mean, save_invstd, run_mean,
                     run_var, true);
}

// y = relu?((x - mean) * invstd * w + b) over rows [r0, r1) of channel c (row lane rl)
template <int NL = BN_RL>   // row lanes of the block (rl in [0, NL))
__device__ __forceinline__ void bn_apply_rows(const float* __restrict__ x, long ldx, float mf, float isf, float wc,
                                              float bc, int relu, float* __restrict__ y, long ldy, long r0, long r1,
                                              int c, int rl) {
  for (long rb = r0 + rl; rb < r1; rb += NL * NB) {   // NB rows' loads in flight
    float xv[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) xv[i] = rb + NL * i < r1 ? x[(rb + NL * i) * ldx + c] : 0.f;
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (rb + NL * i < r1) {
        float v = bn_fwd_elem(xv[i], mf, isf, wc, bc);
        if (relu) v = fmaxf(v, 0.f);
        y[(rb + NL * i) * ldy + c] = v;
      }
  }
}

// Fused final + apply (train mode): grid (ceil(C/64), ceil(M/rows_per_block)); every block reduces
// the channel group's partials itself (bn_part_sums), the blocks of row 0 write save_* and the running
// statistics, and all apply y = relu?((x - mean) * invstd * w + b) to their rows.
// shift: the per-channel shift of the partial sums (x itself, i.e. row 0, for bn_stats_sums' partials; the GEMM's
// bias for vc_gemm_colstats' epilogue partials)
__global__ __launch_bounds__(BN_T) void bn_apply_stats(int M, int C, const float* __restrict__ x, long ldx, int P,
                                                      const double* __restrict__ part, float eps, float momentum,
                                                      float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                                      float* __restrict__ run_mean, float* __restrict__ run_var,
                                                      const float* __restrict__ w, const float* __restrict__ b,
                                                      int relu, float* __restrict__ y, long ldy, int rows_per_block,
                                                      const float* __restrict__ shift) {
  __shared__ double tot[2][64];
  bn_part_sums(P, C, part, blockIdx.x, tot);
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  if (c >= C) return;
  float mf, isf;
  bn_stats_from_sums(tot[0][cl], tot[1][cl], c, M, shift, eps, momentum, mf, isf, save_mean, save_invstd, run_mean,
                     run_var, blockIdx.y == 0 && rl == 0);
  const long r0 = (long)blockIdx.y * rows_per_block;
  bn_apply_rows(x, ldx, mf, isf, w[c], b[c], relu, y, ldy, r0, min((long)M, r0 + rows_per_block), c, rl);
}

// partial block (channel group blockIdx.x, rows [blockIdx.y * rows_per, ...)) of the statistics:
// part[blockIdx.y][0 / 1][c] = its shifted sums
template <int T = BN_T>
__device__ __forceinline__ void bn_stats_partial(int M, int C, const float* __restrict__ x, long ldx, int rows_per,
                                                 double* __restrict__ part) {
  constexpr int RT = T / 64, VPT = BN_RL / RT;   // virtual row lanes per thread (see bn_part_sums)
  __shared__ double sh[2][BN_RL][64];
  const int cl = threadIdx.x & 63, rt = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = min((long)M, r0 + rows_per);
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int rl = rt + RT * j;
    double s1 = 0.0, s2 = 0.0;
    if (c < C) {
      const double k = x[c];
      for (long rb = r0 + rl; rb < r1; rb += BN_RL * NB) {   // NB rows' loads in flight, summed in row order
        float v[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) v[i] = rb + BN_RL * i < r1 ? x[(rb + BN_RL * i) * ldx + c] : 0.f;
#pragma unroll
        for (int i = 0; i < NB; ++i)
          if (rb + BN_RL * i < r1) {
            const double d = (double)v[i] - k;
            s1 += d;
            s2 = fma(d, d, s2);
          }
      }
    }
    sh[0][rl][cl] = s1;
    sh[1][rl][cl] = s2;
  }
  __syncthreads();
  if (rt == 0 && c < C) {
    double* p = part + (long)blockIdx.y * 2 * C + c;
    double t1 = sh[0][0][cl], t2 = sh[1][0][cl];
#pragma unroll
    for (int l = 1; l < BN_RL; ++l) {
      t1 += sh[0][l][cl];
      t2 += sh[1][l][cl];
    }
    p[0] = t1;
    p[C] = t2;
  }
}

// grid (ceil(C/64), P); cnt (optional) = one zeroed arrival counter per 64-channel group
__global__ __launch_bounds__(BN_T) void bn_stats_sums(int M, int C, const float* __restrict__ x, long ldx, int rows_per,
                                                     double* __restrict__ part, unsigned int* __restrict__ cnt,
                                                     float eps, float momentum, float* __restrict__ save_mean,
                                                     float* __restrict__ save_invstd, float* __restrict__ run_mean,
                                                     float* __restrict__ run_var) {
  bn_stats_partial(M, C, x, ldx, rows_per, part);
  if (!cnt || !block_last_arriver(cnt + blockIdx.x, gridDim.y)) return;
  bn_stats_reduce(gridDim.y, C, M, x, part, blockIdx.x, eps, momentum, save_mean, save_invstd, run_mean, run_var);
}

__global__ __launch_bounds__(BN_T) void bn_stats_final(int P, int C, long M, const float* __restrict__ x,
                                                      const double* __restrict__ part, float eps, float momentum,
                                                      float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                                      float* __restrict__ run_mean, float* __restrict__ run_var) {
  bn_stats_reduce(P, C, M, x, part, blockIdx.x, eps, momentum, save_mean, save_invstd, run_mean, run_var);
}

__global__ void bn_eval_prep(int C, const float* __restrict__ run_mean, const float* __restrict__ run_var, float eps,
                             float* __restrict__ save_mean, float* __restrict__ save_invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  save_mean[c] = run_mean[c];
  save_invstd[c] = rsqrtf(run_var[c] + eps);
}

__global__ void bn_apply(int total, FastDiv fC, const float* __restrict__ x, long ldx, const float* __restrict__ mean,
                         const float* __restrict__ invstd, const float* __restrict__ w, const float* __restrict__ b,
                         int relu, float* __restrict__ y, long ldy) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c;
  const long r = fdivmod(idx, fC, c);
  float v = bn_fwd_elem(x[r * ldx + c], mean[c], invstd[c], w[c], b[c]);
  if (relu) v = fmaxf(v, 0.f);
  y[r * ldy + c] = v;
}

// BN backward sums: s1 = sum dyv, s2 = sum dyv*xhat (dyv = dy * (relu_out > 0) if relu_out) in fp64.
// Partial blocks (64 channels x BN_RL row lanes) -> part[p][2][C]; the fixed-order reduction (as in
// bn_stats_reduce) writes sums[0:C] = s1, sums[C:2C] = s2 and dw = beta_w*dw + s2, db = beta_w*db + s1,
// in the last-arriving block of each 64-channel group (tickets) or in bn_bwd_final.
__device__ __forceinline__ void bn_bwd_reduce(int P, int C, const double* __restrict__ part, int cx,
                                              double* __restrict__ sums, float* __restrict__ dw,
                                              float* __restrict__ db, float beta_w) {
  __shared__ double tot[2][64];
  bn_part_sums(P, C, part, cx, tot);
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int c = cx * 64 + cl;
  if (pl != 0 || c >= C) return;
  const double s1 = tot[0][cl], s2 = tot[1][cl];
  sums[c] = s1;
  sums[C + c] = s2;
  if (dw) dw[c] = (beta_w != 0.f ? beta_w * dw[c] : 0.f) + (float)s2;
  if (db) db[c] = (beta_w != 0.f ? beta_w * db[c] : 0.f) + (float)s1;
}

// partial block of the backward sums: part[blockIdx.y][0 / 1][c] = sum dyv, sum dyv * xhat over its rows
template <int T = BN_T>
__device__ __forceinline__ void bn_bwd_partial(int M, int C, const float* __restrict__ dy, long lddy,
                                               const float* __restrict__ x, long ldx, ReluSrc rs,
                                               const float* __restrict__ mean, const float* __restrict__ invstd,
                                               int rows_per, double* __restrict__ part) {
  constexpr int RT = T / 64, VPT = BN_RL / RT;   // virtual row lanes per thread (see bn_part_sums)
  __shared__ double sh[2][BN_RL][64];
  const int cl = threadIdx.x & 63, rt = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = min((long)M, r0 + rows_per);
#pragma unroll
  for (int j = 0; j < VPT; ++j) {
    const int rl = rt + RT * j;
    double s1 = 0.0, s2 = 0.0;
    if (c < C) {
      const float mu = mean[c], is = invstd[c];
      const float rw = rs.b ? rs.w[c] : 0.f, rbc = rs.b ? rs.b[c] : 0.f;
      for (long rb = r0 + rl; rb < r1; rb += BN_RL * NB) {   // NB rows' loads in flight, summed in row order
        float dv[NB], xv[NB], ov[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const long r = rb + BN_RL * i;
          const bool ok = r < r1;
          dv[i] = ok ? dy[r * lddy + c] : 0.f;
          xv[i] = ok ? x[r * ldx + c] : 0.f;
          ov[i] = ok && rs.out ? rs.out[r * rs.ld + c] : 1.f;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i)
          if (rb + BN_RL * i < r1) {
            float d = dv[i];
            if (rs.out && !(ov[i] > 0.f)) d = 0.f;
            if (rs.b && !(bn_fwd_elem(xv[i], mu, is, rw, rbc) > 0.f)) d = 0.f;
            s1 += d;
            s2 += (double)d * ((xv[i] - mu) * is);
          }
      }
    }
    sh[0][rl][cl] = s1;
    sh[1][rl][cl] = s2;
  }
  __syncthreads();
  if (rt == 0 && c < C) {
    double* p = part + (long)blockIdx.y * 2 * C + c;
    double t1 = sh[0][0][cl], t2 = sh[1][0][cl];
#pragma unroll
    for (int l = 1; l < BN_RL; ++l) {
      t1 += sh[0][l][cl];
      t2 += sh[1][l][cl];
    }
    p[0] = t1;
    p[C] = t2;
  }
}

__global__ __launch_bounds__(BN_T) void bn_bwd_sums(int M, int C, const float* __restrict__ dy, long lddy,
                                                   const float* __restrict__ x, long ldx, ReluSrc rs,
                                                   const float* __restrict__ mean, const float* __restrict__ invstd,
                                                   int rows_per, double* __restrict__ part,
                                                   unsigned int* __restrict__ cnt, double* __restrict__ sums,
                                                   float* __restrict__ dw, float* __restrict__ db, float beta_w) {
  bn_bwd_partial(M, C, dy, lddy, x, ldx, rs, mean, invstd, rows_per, part);
  if (!cnt || !block_last_arriver(cnt + blockIdx.x, gridDim.y)) return;
  bn_bwd_reduce(gridDim.y, C, part, blockIdx.x, sums, dw, db, beta_w);
}

__global__ __launch_bounds__(BN_T) void bn_bwd_final(int P, int C, const double* __restrict__ part,
                                                    double* __restrict__ sums, float* __restrict__ dw,
                                                    float* __restrict__ db, float beta_w) {
  bn_bwd_reduce(P, C, part, blockIdx.x, sums, dw, db, beta_w);
}

// dx rows [r0, r1) of channel c (row lane rl) from the channel's sums s1, s2 (train) -- or w*invstd*dyv (eval)
template <int NL = BN_RL>   // row lanes of the block (rl in [0, NL))
__device__ __forceinline__ void bn_bwd_apply_rows(int train, int M, const float* __restrict__ dy, long lddy,
                                                  const float* __restrict__ x, long ldx, ReluSrc rs, float mu, float is,
                                                  float wc, double s1, double s2, float* __restrict__ dx, long lddx,
                                                  float beta_dx, long r0, long r1, int c, int rl) {
  const float invM = 1.f / (float)M;
  const float rw = rs.b ? rs.w[c] : 0.f, rbc = rs.b ? rs.b[c] : 0.f;
  const bool need_x = train || rs.b;
  for (long rb = r0 + rl; rb < r1; rb += NL * NB) {   // NB rows' loads in flight
    float dv[NB], xv[NB], ov[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const long r = rb + NL * i;
      const bool ok = r < r1;
      dv[i] = ok ? dy[r * lddy + c] : 0.f;
      xv[i] = ok && need_x ? x[r * ldx + c] : 0.f;
      ov[i] = ok && rs.out ? rs.out[r * rs.ld + c] : 1.f;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i)
      if (rb + NL * i < r1) {
        float d = dv[i];
        if (rs.out && !(ov[i] > 0.f)) d = 0.f;
        if (rs.b && !(bn_fwd_elem(xv[i], mu, is, rw, rbc) > 0.f)) d = 0.f;
        float v;
        if (train) v = bn_bwd_elem(d, xv[i], mu, is, wc, (float)s1 * invM, (float)s2 * invM);
        else v = (wc * is) * d;
        bn_dx_store(dx + (rb + NL * i) * lddx + c, beta_dx, v);
      }
  }
}

// Fused final + apply of the BN backward: grid (ceil(C/64), ceil(M/rows_per_block)); every block
// reduces the channel group's partials itself (bn_part_sums), the blocks of row 0 write dw / db, and
// all write dx = beta_dx*dx + w*invstd*(dyv - s1/M - xhat*s2/M) (train) or w*invstd*dyv (eval) for
// their rows -- the same arithmetic as bn_bwd_final + bn_bwd_apply.
__global__ __launch_bounds__(BN_T) void bn_bwd_apply_sums(int train, int M, int C, const float* __restrict__ dy,
                                                         long lddy, const float* __restrict__ x, long ldx, ReluSrc rs,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd,
                                                         const float* __restrict__ w, int P,
                                                         const double* __restrict__ part, float* __restrict__ dx,
                                                         long lddx, float beta_dx, float* __restrict__ dw,
                                                         float* __restrict__ db, float beta_w, int rows_per_block) {
  __shared__ double tot[2][64];
  bn_part_sums(P, C, part, blockIdx.x, tot);
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  if (c >= C) return;
  const double s1 = tot[0][cl], s2 = tot[1][cl];
  if (blockIdx.y == 0 && rl == 0) {
    if (dw) dw[c] = (beta_w != 0.f ? beta_w * dw[c] : 0.f) + (float)s2;
    if (db) db[c] = (beta_w != 0.f ? beta_w * db[c] : 0.f) + (float)s1;
  }
  const long r0 = (long)blockIdx.y * rows_per_block;
  bn_bwd_apply_rows(train, M, dy, lddy, x, ldx, rs, mean[c], invstd[c], w[c], s1, s2, dx, lddx, beta_dx, r0,
                    min((long)M, r0 + rows_per_block), c, rl);
}

// train: dx = w*invstd*(dyv - s1/M - xhat*s2/M);  eval (sums == null): dx = w*invstd*dyv
__global__ void bn_bwd_apply(int M, FastDiv fC, const float* __restrict__ dy, long lddy, const float* __restrict__ x,
                             long ldx, ReluSrc rs, const float* __restrict__ mean,
                             const float* __restrict__ invstd, const float* __restrict__ w,
                             const double* __restrict__ sums, float* __restrict__ dx, long lddx, float beta_dx) {
  const int C = fC.div;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * C) return;
  int c;
  const long r = fdivmod(idx, fC, c);
  float d = dy[r * lddy + c];
  const float is = invstd[c];
  if (rs.out && !(rs.out[r * rs.ld + c] > 0.f)) d = 0.f;
  if (rs.b && !(bn_fwd_elem(x[r * ldx + c], mean[c], is, rs.w[c], rs.b[c]) > 0.f)) d = 0.f;
  float v;
  if (sums) {
    const float invM = 1.f / (float)M;
    v = bn_bwd_elem(d, x[r * ldx + c], mean[c], is, w[c], (float)sums[c] * invM,
                    (float)sums[C + c] * invM);
  } else {
    v = (w[c] * is) * d;
  }
  bn_dx_store(dx + r * lddx + c, beta_dx, v);
}

// rows per partial block: at most 64 partials per 64-channel group (the fixed-order reduction reads
// P/4 of them per thread), at least 32 rows each, fewer partials if the fp64 workspace is short
constexpr int BN_APPLY_ROWS = 64;   // rows per block of the fused (partials-reducing) apply kernels
int bn_apply_rows() { return (int)std::max(16L, vc_knob("VITCNN_BN_APPLY_ROWS", BN_APPLY_ROWS)); }   // knob: probe

// The one-launch forms of round 4 (partial blocks meeting at a per-channel-group spin barrier) were
// measured slower than the two launches (ViT-CNN 1.82 -> 1.95 ms, FusAtNet 19.5 -> 20.7 ms,
// profiles/r04_ab_bn_fused.log) and a spin barrier without a co-residency guarantee can deadlock beside
// other streams' work, so they were removed; counters now only select the
// last-arriving-block reduction of a backward without dx.
int bn_rows_per(long M, int C, long ws_doubles, long reserve_doubles) {
  // most partials per channel (knob BN_PCAP, probe library)
  const int pcap = (int)std::max(16L, std::min(1024L, vc_knob("VITCNN_BN_PCAP", 64)));
  int rows_per = std::max<long>(32, (M + pcap - 1) / pcap);
  while ((long)vc_cdiv(M, rows_per) * 2 * C + reserve_doubles > ws_doubles && rows_per < (1 << 29)) rows_per *= 2;
  return rows_per;
}


// GLfusionBlock's NonLocal output BN(W y) combined with the two branches (vc_glf_combine_fwd's
// arithmetic, Mutimodality_Mamba7.py:154-156, :1112-1115), the BN statistics' final reduction inside the
// launch as in bn_apply_stats: out [M, 2C] = [ (BN(w_pre) + fc) + fl | fl + fc ].
__global__ __launch_bounds__(BN_T) void glf_combine_stats(int M, int C, const float* __restrict__ wpre, int P,
                                                         const double* __restrict__ part, float eps, float momentum,
                                                         float* __restrict__ save_mean,
                                                         float* __restrict__ save_invstd,
                                                         float* __restrict__ run_mean, float* __restrict__ run_var,
                                                         const float* __restrict__ gam, const float* __restrict__ bet,
                                                         const float* __restrict__ fc, const float* __restrict__ fl,
                                                         float* __restrict__ out, int rows_per_block) {
  __shared__ double tot[2][64];
  bn_part_sums(P, C, part, blockIdx.x, tot);
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  if (c >= C) return;
  float mf, isf;
  bn_stats_from_sums(tot[0][cl], tot[1][cl], c, M, wpre, eps, momentum, mf, isf, save_mean, save_invstd, run_mean,
                     run_var, blockIdx.y == 0 && rl == 0);
  const float g = gam[c], bt = bet[c];
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = min((long)M, r0 + rows_per_block);
  for (long rb = r0 + rl; rb < r1; rb += BN_RL * NB) {
    float wv[NB], zv[NB], xv[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const long r = rb + BN_RL * i;
      const bool ok = r < r1;
      wv[i] = ok ? wpre[r * C + c] : 0.f;
      zv[i] = ok ? fc[r * C + c] : 0.f;
      xv[i] = ok ? fl[r * C + c] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const long r = rb + BN_RL * i;
      if (r < r1) {
        const float wy = (wv[i] - mf) * isf * g + bt;
        out[r * 2 * C + c] = (wy + zv[i]) + xv[i];
        out[r * 2 * C + C + c] = xv[i] + zv[i];
      }
    }
  }
}

// Train-mode BatchNorm in front of a 3x3 valid conv, its statistics finished inside the im2col that
// applies it (the bn_stats_final launch folded in): block = (sample, 32-channel chunk) as im2col3x3_lds
// in conv.hip.  Each block reduces its channels' [P][2][C] partials in bn_part_sums' order (lane l sums
// p = l, l + BN_RL, ... in increasing p, then the lanes in order: the same fp64 operations, so mean /
// invstd are bit-identical to vc_bn_stats'), the sample-0 blocks write save_* and the running stats,
// and the chunk is staged BN-applied in LDS and written as col rows.
constexpr int IBS_CC = 32, IBS_T = 64 * BN_RL / 2, IBS_W = IBS_T / 64, IBS_JK = (9 * IBS_CC + 63) / 64;
constexpr int IBS_CP = IBS_CC + 1;   // LDS pitch of a staged pixel (conv.hip C2I_CP: bank spread of the tap reads)
static_assert(IBS_T == IBS_CC * BN_RL, "one thread per (channel, partial lane)");

__global__ __launch_bounds__(IBS_T) void im2col3x3_bnstats(int nchunk, int H, int W, int C, long M, int P,
                                                          const double* __restrict__ part, float eps,
                                                          float momentum, float* __restrict__ save_mean,
                                                          float* __restrict__ save_invstd,
                                                          float* __restrict__ run_mean, float* __restrict__ run_var,
                                                          const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, float* __restrict__ col) {
  extern __shared__ float img[];   // [H*W][IBS_CP]
  __shared__ double shr[2][BN_RL][IBS_CC];
  __shared__ float scs[IBS_CC], shs[IBS_CC];
  const int bb = blockIdx.x / nchunk, c0 = (blockIdx.x - bb * nchunk) * IBS_CC, nc = min(IBS_CC, C - c0);
  const int OW = W - 2, S = (H - 2) * OW, HW = H * W;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = threadIdx.x & (IBS_CC - 1), pl = threadIdx.x / IBS_CC;
  {
    double s1 = 0.0, s2 = 0.0;
    if (c < nc) {
      const int cg = c0 + c;
      for (int p0 = pl; p0 < P; p0 += BN_RL * NB) {
        double a[NB], bq[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
          const int p = p0 + BN_RL * i;
          a[i] = p < P ? part[(long)p * 2 * C + cg] : 0.0;
          bq[i] = p < P ? part[(long)p * 2 * C + C + cg] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < NB; ++i)
          if (p0 + BN_RL * i < P) {
            s1 += a[i];
            s2 += bq[i];
          }
      }
    }
    shr[0][pl][c] = s1;
    shr[1][pl][c] = s2;
  }
  __syncthreads();
  if (pl == 0 && c < nc) {
    double t1 = shr[0][0][c], t2 = shr[1][0][c];
#pragma unroll
    for (int l = 1; l < BN_RL; ++l) {
      t1 += shr[0][l][c];
      t2 += shr[1][l][c];
    }
    float mf, isf;
    bn_stats_from_sums(t1, t2, c0 + c, M, x, eps, momentum, mf, isf, save_mean, save_invstd, run_mean, run_var,
                       bb == 0);
    const float sc = isf * w[c0 + c];
    scs[c] = sc;
    shs[c] = b[c0 + c] - mf * sc;
  }
  __syncthreads();
  {   // stage the chunk BN-applied: thread -> (pixel, channel c)
    const float sc = c < nc ? scs[c] : 1.f, sh = c < nc ? shs[c] : 0.f;
    const float* xb = x + (long)bb * HW * C + c0 + c;
    constexpr int PP = IBS_T / IBS_CC, NBP = 8;
    for (int p0 = pl; p0 < HW; p0 += PP * NBP) {
      float v[NBP];
#pragma unroll
      for (int k = 0; k < NBP; ++k) {
        const int p = p0 + k * PP;
        v[k] = (p < HW && c < nc) ? xb[(long)p * C] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < NBP; ++k) {
        const int p = p0 + k * PP;
        if (p < HW) img[p * IBS_CP + c] = v[k] * sc + sh;
      }
    }
  }
  __syncthreads();
  const int seg = 9 * nc;
  int off[IBS_JK];
#pragma unroll
  for (int k = 0; k < IBS_JK; ++k) {
    const int j = lane + 64 * k, cc = j / 9, t = j - 9 * cc, kh = t / 3, kw = t - 3 * kh;
    off[k] = j < seg ? (kh * W + kw) * IBS_CP + cc : -1;
  }
  float* cb = col + (long)bb * S * 9 * C + 9 * c0;
  for (int m = wave; m < S; m += IBS_W) {
    const int oh = m / OW, ow = m - oh * OW, base = (oh * W + ow) * IBS_CP;
    float* row = cb + (long)m * 9 * C;
#pragma unroll
    for (int k = 0; k < IBS_JK; ++k)
      if (off[k] >= 0) row[lane + 64 * k] = img[base + off[k]];
  }
}

}  // namespace

VC_EXPORT int vc_layernorm_fwd(int R, int C, const float* x, long ldx, const float* w, const float* b, float eps,
                               float* y, long ldy, float* mean, float* rstd, hipStream_t stream) {
  VC_REQUIRE(C > 0 && C <= 64 * LN_MAXV && R >= 0);
  if (R == 0) return VC_OK;
  hipLaunchKernelGGL(ln_fwd, dim3(vc_cdiv(R, 4)), dim3(256), 0, stream, R, C, x, ldx, w, b, eps, y, ldy, mean, rstd);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// rows per ln_bwd block (P = ceil(R / rows_per) partial rows of 2C floats)
// (8 rows = one two-row iteration per wave: the B = 64 steps' 5184-row LayerNorms as 648 blocks)
static int ln_partial_rows(int R, int C, long part_floats) {
#ifndef VC_LN_MIN_ROWS
#define VC_LN_MIN_ROWS 8
#endif
  int rows_per = std::max(VC_LN_MIN_ROWS, vc_cdiv(R, 1024));
  while ((long)vc_cdiv(R, rows_per) * 2 * C > part_floats) rows_per *= 2;
  return rows_per;
}

static int layernorm_bwd(int R, int C, const float* dy, long lddy, const float* x, long ldx, const float* w,
                         const float* mean, const float* rstd, const float* res, long ldr, float* dx, long lddx,
                         float beta_dx, float* dw, float* db, float beta_w, float* ws, long ws_floats,
                         hipStream_t stream) {
  VC_REQUIRE(C > 0 && C <= 64 * LN_MAXV && R >= 0);
  if (R == 0) return VC_OK;
  const int rows_per = ln_partial_rows(R, C, ws_floats);
  const int P = vc_cdiv(R, rows_per);
  hipLaunchKernelGGL(ln_bwd, dim3(P), dim3(256), 0, stream, R, C, rows_per, dy, lddy, x, ldx, w, mean, rstd, dx,
                     lddx, beta_dx, res, ldr, ws);
  VC_CHECK_LAUNCH();
  // the [P][2C] partials: 16 columns x 16 partial lanes per block, in parallel over the columns
  if (dw && db == dw + C) return launch_sum_rows(P, 2 * C, ws, (long)2 * C, 0L, dw, beta_w, stream);  // adjacent
  if (dw) {
    int rc = launch_sum_rows(P, C, ws, (long)2 * C, 0L, dw, beta_w, stream);
    if (rc) return rc;
  }
  if (db) {
    int rc = launch_sum_rows(P, C, ws, (long)2 * C, (long)C, db, beta_w, stream);
    if (rc) return rc;
  }
  return VC_OK;
}

// Split form (the parameter reduction can run later, elsewhere): vc_layernorm_bwd_dx writes dx
// (= res + LN grad when res is given, else beta_dx * dx + LN grad) and leaves the per-block dw / db
// partials in `part`; vc_layernorm_bwd_params sums those partials (same R, C, part_floats) into
// dw = beta_w * dw + ..., db = beta_w * db + ...  Together they equal vc_layernorm_bwd bit for bit.
VC_EXPORT int vc_layernorm_bwd_dx(int R, int C, const float* dy, long lddy, const float* x, long ldx, const float* w,
                                  const float* mean, const float* rstd, const float* res, long ldr, float* dx,
                                  long lddx, float beta_dx, float* part, long part_floats, hipStream_t stream) {
  VC_REQUIRE(C > 0 && C <= 64 * LN_MAXV && R > 0 && part);
  const int rows_per = ln_partial_rows(R, C, part_floats);
  const int P = vc_cdiv(R, rows_per);
  VC_REQUIRE((long)P * 2 * C <= part_floats);
  hipLaunchKernelGGL(ln_bwd, dim3(P), dim3(256), 0, stream, R, C, rows_per, dy, lddy, x, ldx, w, mean, rstd, dx,
                     lddx, beta_dx, res, ldr, part);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_EXPORT int vc_layernorm_bwd_params(int R, int C, const float* part, long part_floats, float* dw, float* db,
                                      float beta_w, hipStream_t stream) {
  VC_REQUIRE(C > 0 && C <= 64 * LN_MAXV && R > 0 && part);
  const int P = vc_cdiv(R, ln_partial_rows(R, C, part_floats));
  if (dw && db == dw + C) return launch_sum_rows(P, 2 * C, part, (long)2 * C, 0L, dw, beta_w, stream);
  if (dw) {
    int rc = launch_sum_rows(P, C, part, (long)2 * C, 0L, dw, beta_w, stream);
    if (rc) return rc;
  }
  if (db) return launch_sum_rows(P, C, part, (long)2 * C, (long)C, db, beta_w, stream);
  return VC_OK;
}

// dx = beta_dx*dx + LNgrad;  dw = beta_w*dw + sum dy*xhat;  db = beta_w*db + sum dy
VC_EXPORT int vc_layernorm_bwd(int R, int C, const float* dy, long lddy, const float* x, long ldx, const float* w,
                               const float* mean, const float* rstd, float* dx, long lddx, float beta_dx, float* dw,
                               float* db, float beta_w, float* ws, long ws_floats, hipStream_t stream) {
  return layernorm_bwd(R, C, dy, lddy, x, ldx, w, mean, rstd, nullptr, 0, dx, lddx, beta_dx, dw, db, beta_w, ws,
                       ws_floats, stream);
}

// dx = res + LNgrad (a residual gradient from another buffer, which stays untouched)
VC_EXPORT int vc_layernorm_bwd_res(int R, int C, const float* dy, long lddy, const float* x, long ldx, const float* w,
                                   const float* mean, const float* rstd, const float* res, long ldr, float* dx,
                                   long lddx, float* dw, float* db, float beta_w, float* ws, long ws_floats,
                                   hipStream_t stream) {
  VC_REQUIRE(res != nullptr);
  return layernorm_bwd(R, C, dy, lddy, x, ldx, w, mean, rstd, res, ldr, dx, lddx, 0.f, dw, db, beta_w, ws, ws_floats,
                       stream);
}

// Train: batch statistics -> save_mean / save_invstd, running stats updated (if run_mean).
// Eval (train == 0): save_* filled from the running statistics.  counters (optional): >= ceil(C/64)
// zeroed arrival counters (left zero) — the reduction then runs in the partial launch itself.
VC_EXPORT int vc_bn_stats_ex(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                             float* save_mean, float* save_invstd, float* run_mean, float* run_var, float* ws,
                             long ws_floats, unsigned int* counters, int n_counters, hipStream_t stream) {
  VC_REQUIRE(C > 0 && M >= 0);
  if (!train) {
    hipLaunchKernelGGL(bn_eval_prep, dim3(vc_cdiv(C, 256)), dim3(256), 0, stream, C, run_mean, run_var, eps,
                       save_mean, save_invstd);
    VC_CHECK_LAUNCH();
    return VC_OK;
  }
  VC_REQUIRE(M > 0 && M < (1L << 31) && ((uintptr_t)ws & 7) == 0);
  // partial (s1, s2) pairs are fp64: the workspace holds ws_floats/2 doubles
  double* wsd = reinterpret_cast<double*>(ws);
  const long ws_doubles = ws_floats / 2;
  const int rows_per = bn_rows_per(M, C, ws_doubles, 0);
  const int P = vc_cdiv(M, rows_per);
  VC_REQUIRE((long)P * C * 2 <= ws_doubles && P <= 65535);
  unsigned int* cnt = (counters && n_counters >= vc_cdiv(C, 64)) ? counters : nullptr;
  hipLaunchKernelGGL(bn_stats_sums, dim3(vc_cdiv(C, 64), P), dim3(BN_T), 0, stream, (int)M, C, x, ldx, rows_per, wsd,
                     cnt, eps, momentum, save_mean, save_invstd, run_mean, run_var);
  VC_CHECK_LAUNCH();
  if (!cnt) {
    hipLaunchKernelGGL(bn_stats_final, dim3(vc_cdiv(C, 64)), dim3(BN_T), 0, stream, P, C, M, x, wsd, eps, momentum,
                       save_mean, save_invstd, run_mean, run_var);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

VC_EXPORT int vc_bn_stats(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                          float* save_mean, float* save_invstd, float* run_mean, float* run_var, float* ws,
                          long ws_floats, hipStream_t stream) {
  return vc_bn_stats_ex(train, M, C, x, ldx, eps, momentum, save_mean, save_invstd, run_mean, run_var, ws, ws_floats,
                        nullptr, 0, stream);
}

// BatchNorm forward in one call: train -> batch statistics (partials) + the fused final/apply kernel
// (save_* and running stats written as vc_bn_stats does, y as vc_bn_apply: two launches); eval ->
// save_* from the running statistics + apply.  Bit-identical to vc_bn_stats + vc_bn_apply.
VC_EXPORT int vc_bn_forward(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                            float* save_mean, float* save_invstd, float* run_mean, float* run_var, const float* w,
                            const float* b, int relu, float* y, long ldy, float* ws, long ws_floats,
                            hipStream_t stream) {
  return vc_bn_forward_ex(train, M, C, x, ldx, eps, momentum, save_mean, save_invstd, run_mean, run_var, w, b, relu, y,
                          ldy, ws, ws_floats, nullptr, 0, stream);
}

VC_EXPORT int vc_bn_forward_ex(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                               float* save_mean, float* save_invstd, float* run_mean, float* run_var, const float* w,
                               const float* b, int relu, float* y, long ldy, float* ws, long ws_floats,
                               unsigned int* counters, int n_counters, hipStream_t stream) {
  VC_REQUIRE(C > 0 && M >= 0);
  if (!train || M == 0) {
    int rc = vc_bn_stats(train, M, C, x, ldx, eps, momentum, save_mean, save_invstd, run_mean, run_var, ws, ws_floats,
                         stream);
    if (rc) return rc;
    return vc_bn_apply(M, C, x, ldx, save_mean, save_invstd, w, b, relu, y, ldy, stream);
  }
  VC_REQUIRE(M < (1L << 31) && ((uintptr_t)ws & 7) == 0);
  double* wsd = reinterpret_cast<double*>(ws);
  const long ws_doubles = ws_floats / 2;
  const int rows_per = bn_rows_per(M, C, ws_doubles, 0);
  const int P = vc_cdiv(M, rows_per);
  VC_REQUIRE((long)P * C * 2 <= ws_doubles && P <= 65535);
  (void)counters;
  (void)n_counters;
  hipLaunchKernelGGL(bn_stats_sums, dim3(vc_cdiv(C, 64), P), dim3(BN_T), 0, stream, (int)M, C, x, ldx, rows_per, wsd,
                     (unsigned int*)nullptr, eps, momentum, save_mean, save_invstd, run_mean, run_var);
  VC_CHECK_LAUNCH();
  const int rpb = bn_apply_rows();
  hipLaunchKernelGGL(bn_apply_stats, dim3(vc_cdiv(C, 64), vc_cdiv(M, rpb)), dim3(BN_T), 0, stream, (int)M, C, x, ldx,
                     P, wsd, eps, momentum, save_mean, save_invstd, run_mean, run_var, w, b, relu, y, ldy, rpb, x);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// train-mode BatchNorm forward from fp64 partials another kernel left (vc_gemm_colstats: P = ceil(M / 64) row tiles,
// [P][2][C] sums of (x - shift[c]) and (x - shift[c])^2): one launch, statistics + running stats + apply (+ ReLU)
VC_EXPORT int vc_bn_apply_partials(long M, int C, const float* x, long ldx, int P, const double* part,
                                   const float* shift, float eps, float momentum, float* save_mean, float* save_invstd,
                                   float* run_mean, float* run_var, const float* w, const float* b, int relu, float* y,
                                   long ldy, hipStream_t stream) {
  VC_REQUIRE(C > 0 && M > 0 && M < (1L << 31) && P > 0 && P <= 65535 && part && shift);
  const int rpb = bn_apply_rows();
  hipLaunchKernelGGL(bn_apply_stats, dim3(vc_cdiv(C, 64), vc_cdiv(M, rpb)), dim3(BN_T), 0, stream, (int)M, C, x, ldx,
                     P, part, eps, momentum, save_mean, save_invstd, run_mean, run_var, w, b, relu, y, ldy, rpb, shift);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_EXPORT int vc_bn_apply(long M, int C, const float* x, long ldx, const float* mean, const float* invstd,
                          const float* w, const float* b, int relu, float* y, long ldy, hipStream_t stream) {
  VC_REQUIRE(C > 0 && M >= 0);
  if (M == 0) return VC_OK;
  VC_REQUIRE_I32(M * C);
  hipLaunchKernelGGL(bn_apply, dim3(vc_cdiv(M * C, 256)), dim3(256), 0, stream, (int)(M * C), make_fastdiv(C), x, ldx,
                     mean, invstd, w, b,
                     relu, y, ldy);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// BN backward (optionally through a following ReLU whose output is relu_out).
// dx = beta_dx*dx + ...;  dw/db = beta_w*dw/db + ... (either may be null).  counters (optional):
// >= ceil(C/64) zeroed arrival counters (left zero): the sums are reduced inside the partial launch.
static int bn_bwd_impl(int train, long M, int C, const float* dy, long lddy, const float* x, long ldx, ReluSrc rs,
                       const float* mean, const float* invstd, const float* w, float* dx, long lddx, float beta_dx,
                       float* dw, float* db, float beta_w, float* ws, long ws_floats, unsigned int* counters,
                       int n_counters, hipStream_t stream) {
  VC_REQUIRE(C > 0 && M > 0 && M < (1L << 31) && ((uintptr_t)ws & 7) == 0);
  // per-row-block partial sums [P][2][C] and the final [2][C] sums are fp64
  double* wsd = reinterpret_cast<double*>(ws);
  const long ws_doubles = ws_floats / 2;
  const int rows_per = bn_rows_per(M, C, ws_doubles, 2L * C);
  const int P = vc_cdiv(M, rows_per);
  VC_REQUIRE((long)P * C * 2 + 2L * C <= ws_doubles && P <= 65535);
  double* sums = wsd + (long)P * C * 2;
  // tickets (the last-arriving partial block reduces) only without dx: with dx the channel-tiled apply
  // reduces the partials itself
  unsigned int* cnt = (!(train && dx) && counters && n_counters >= vc_cdiv(C, 64)) ? counters : nullptr;
  hipLaunchKernelGGL(bn_bwd_sums, dim3(vc_cdiv(C, 64), P), dim3(BN_T), 0, stream, (int)M, C, dy, lddy, x, ldx,
                     rs, mean, invstd, rows_per, wsd, cnt, sums, dw, db, beta_w);
  VC_CHECK_LAUNCH();
  if (!cnt && dx) {   // the channel-tiled apply reduces the partials itself: one launch fewer
    const int rpb = bn_apply_rows();
    hipLaunchKernelGGL(bn_bwd_apply_sums, dim3(vc_cdiv(C, 64), vc_cdiv(M, rpb)), dim3(BN_T), 0, stream, train,
                       (int)M, C, dy, lddy, x, ldx, rs, mean, invstd, w, P, wsd, dx, lddx, beta_dx, dw,
                       db, beta_w, rpb);
    VC_CHECK_LAUNCH();
    return VC_OK;
  }
  if (!cnt) {
    hipLaunchKernelGGL(bn_bwd_final, dim3(vc_cdiv(C, 64)), dim3(BN_T), 0, stream, P, C, wsd, sums, dw, db, beta_w);
    VC_CHECK_LAUNCH();
  }
  if (dx) {
    VC_REQUIRE_I32(M * C);
    hipLaunchKernelGGL(bn_bwd_apply, dim3(vc_cdiv(M * C, 256)), dim3(256), 0, stream, (int)M, make_fastdiv(C), dy,
                       lddy, x, ldx, rs, mean, invstd, w, train ? sums : (const double*)nullptr, dx, lddx,
                       beta_dx);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

VC_EXPORT int vc_bn_bwd_ex(int train, long M, int C, const float* dy, long lddy, const float* x, long ldx,
                           const float* relu_out, long ldo, const float* mean, const float* invstd, const float* w,
                           float* dx, long lddx, float beta_dx, float* dw, float* db, float beta_w, float* ws,
                           long ws_floats, unsigned int* counters, int n_counters, hipStream_t stream) {
  return bn_bwd_impl(train, M, C, dy, lddy, x, ldx, ReluSrc{relu_out, ldo, nullptr, nullptr}, mean, invstd, w, dx, lddx,
                     beta_dx, dw, db, beta_w, ws, ws_floats, counters, n_counters, stream);
}

// BN backward through the ReLU that follows it, the ReLU's decisions recomputed from x, the saved statistics
// and the affine (w, b) -- bit-identical to vc_bn_bwd_ex with relu_out = the forward's output, one read less
VC_EXPORT int vc_bn_bwd_relu_ex(int train, long M, int C, const float* dy, long lddy, const float* x, long ldx,
                                const float* mean, const float* invstd, const float* w, const float* b, float* dx,
                                long lddx, float beta_dx, float* dw, float* db, float beta_w, float* ws, long ws_floats,
                                unsigned int* counters, int n_counters, hipStream_t stream) {
  VC_REQUIRE(w && b);
  return bn_bwd_impl(train, M, C, dy, lddy, x, ldx, ReluSrc{nullptr, 0, w, b}, mean, invstd, w, dx, lddx, beta_dx,
                     dw, db, beta_w, ws, ws_floats, counters, n_counters, stream);
}

VC_EXPORT int vc_bn_bwd(int train, long M, int C, const float* dy, long lddy, const float* x, long ldx,
                        const float* relu_out, long ldo, const float* mean, const float* invstd, const float* w,
                        float* dx, long lddx, float beta_dx, float* dw, float* db, float beta_w, float* ws,
                        long ws_floats, hipStream_t stream) {
  return vc_bn_bwd_ex(train, M, C, dy, lddy, x, ldx, relu_out, ldo, mean, invstd, w, dx, lddx, beta_dx, dw, db,
                      beta_w, ws, ws_floats, nullptr, 0, stream);
}

// Train-mode BatchNorm(x) -> im2col for a 3x3 valid conv, the statistics' final reduction inside the
// im2col launch: vc_bn_stats_ex (train) + vc_im2col3x3 with the same save_* / running-stat / col
// results, bit for bit, in two launches instead of three.  Falls back to the three launches where the
// chunk does not fit the LDS budget.
VC_EXPORT int vc_bn_im2col3x3(int B, int H, int W, int C, const float* x, float eps, float momentum, float* save_mean,
                              float* save_invstd, float* run_mean, float* run_var, const float* bn_w,
                              const float* bn_b, float* col, float* ws, long ws_floats, hipStream_t stream) {
  VC_REQUIRE(B > 0 && H >= 3 && W >= 3 && C > 0 && ((uintptr_t)ws & 7) == 0);
  const long M = (long)B * H * W;
  VC_REQUIRE(M < (1L << 31));
  VC_REQUIRE_I32((long)B * (H - 2) * (W - 2) * C * 9);
  const long S = (long)(H - 2) * (W - 2);
  // knob BN_IM2COL=0 (probe library): the three launches
  if (S * 9 * IBS_CC * 4 > 65536 || vc_knob("VITCNN_BN_IM2COL", 1) == 0) {
    int rc = vc_bn_stats_ex(1, M, C, x, C, eps, momentum, save_mean, save_invstd, run_mean, run_var, ws, ws_floats,
                            nullptr, 0, stream);
    if (rc) return rc;
    return vc_im2col3x3(B, H, W, C, x, save_mean, save_invstd, bn_w, bn_b, col, stream);
  }
  double* wsd = reinterpret_cast<double*>(ws);
  const int rows_per = bn_rows_per(M, C, ws_floats / 2, 0);
  const int P = vc_cdiv(M, rows_per);
  VC_REQUIRE((long)P * C * 2 <= ws_floats / 2 && P <= 65535);
  hipLaunchKernelGGL(bn_stats_sums, dim3(vc_cdiv(C, 64), P), dim3(BN_T), 0, stream, (int)M, C, x, (long)C, rows_per,
                     wsd, (unsigned int*)nullptr, eps, momentum, save_mean, save_invstd, run_mean, run_var);
  VC_CHECK_LAUNCH();
  const int nchunk = vc_cdiv(C, IBS_CC);
  VC_REQUIRE_I32((long)B * nchunk);
  hipLaunchKernelGGL(im2col3x3_bnstats, dim3(B * nchunk), dim3(IBS_T), sizeof(float) * H * W * IBS_CP, stream, nchunk,
                     H, W, C, M, P, wsd, eps, momentum, save_mean, save_invstd, run_mean, run_var, x, bn_w, bn_b, col);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// train-mode vc_bn_stats_ex of w_pre + vc_glf_combine_fwd in two launches instead of three (the
// statistics' final reduction inside the combine); save_* / running stats as vc_bn_stats_ex writes them
VC_EXPORT int vc_bn_glf_combine(long M, int C, const float* w_pre, float eps, float momentum, float* save_mean,
                                float* save_invstd, float* run_mean, float* run_var, const float* bn_w,
                                const float* bn_b, const float* fc, const float* fl, float* out, float* ws,
                                long ws_floats, hipStream_t stream) {
  VC_REQUIRE(M > 0 && M < (1L << 31) && C > 0 && ((uintptr_t)ws & 7) == 0);
  VC_REQUIRE_I32(M * 2 * C);
  if (vc_knob("VITCNN_BN_GLF", 1) == 0) {   // knob BN_GLF=0 (probe library): the three launches
    int rc = vc_bn_stats_ex(1, M, C, w_pre, C, eps, momentum, save_mean, save_invstd, run_mean, run_var, ws,
                            ws_floats, nullptr, 0, stream);
    if (rc) return rc;
    return vc_glf_combine_fwd(M, C, w_pre, save_mean, save_invstd, bn_w, bn_b, fc, fl, out, stream);
  }
  double* wsd = reinterpret_cast<double*>(ws);
  const int rows_per = bn_rows_per(M, C, ws_floats / 2, 0);
  const int P = vc_cdiv(M, rows_per);
  VC_REQUIRE((long)P * C * 2 <= ws_floats / 2 && P <= 65535);
  hipLaunchKernelGGL(bn_stats_sums, dim3(vc_cdiv(C, 64), P), dim3(BN_T), 0, stream, (int)M, C, w_pre, (long)C, rows_per,
                     wsd, (unsigned int*)nullptr, eps, momentum, save_mean, save_invstd, run_mean, run_var);
  VC_CHECK_LAUNCH();
  const int rpb = BN_APPLY_ROWS;
  hipLaunchKernelGGL(glf_combine_stats, dim3(vc_cdiv(C, 64), vc_cdiv(M, rpb)), dim3(BN_T), 0, stream, (int)M, C, w_pre,
                     P, wsd, eps, momentum, save_mean, save_invstd, run_mean, run_var, bn_w, bn_b, fc, fl, out, rpb);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
