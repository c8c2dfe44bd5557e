// TokenLearner(S) = S independent SpatialAttention modules (Mutimodality_Mamba7.py:26-64), fused:
//   pooled[p] = (max_c x[p, c], mean_c x[p, c])                       shared by all S tokens
//   f_s[p]    = w0_s max + w1_s mean + b_s                             2->1 1x1 conv (:37)
//   a[b,s,p]  = sigmoid(ReLU(BN_s(f_s)[p]))                            BatchNorm2d(1) over B*HW (:38-48)
//   Z[b,s,:]  = mean_p a[b,s,p] x[b,p,:]                               (:61-63; a vc_gemm)
//
// Round 5 layout (the round-4 kernels ran one 1024-thread block per token, 25 / 49
// blocks walking all B*HW elements serially, 4 x 35 + 4 x 16 us per step).  f_s is LINEAR in the pooled
// pair, so every token's batch statistics follow from the moments of (max, mean) over the batch, which
// all tokens share:
//   mean_f = w0 mbar + w1 vbar + b,   n var_f = w0^2 Cmm + 2 w0 w1 Cmv + w1^2 Cvv
// with Cxy the centred second moments, accumulated in fp64 against a shift K = the pooled values of row 0
// (d = m - K is exact in fp64; |mbar - K| is within the data's range, so Cmm = sum d^2 - (sum d)^2 / n
// keeps ~15 digits -- these BN(1) inputs have a spread ~1e-3 of their mean).  The forward is then:
//   pixel_stats  (one wave per pixel row; 64 rows per block) + the block's shifted moment partials
//   attn_fwd     grid (sample chunks x token groups): every block combines the partials (fixed order),
//                derives its tokens' statistics, and writes a for its samples
// and the backward, with g1 = da sigmoid'(bn) [bn > 0], s1 = sum g1, s2 = sum g1 xh:
//   attn_bwd     grid (tokens x element chunks): per-token fp64 partials of s1, s2 and of the centred
//                sums sum g1 (m - mbar), sum g1 (v - vbar)
//   pixel_bwd    one wave per pixel row, a lane per token: df = gamma invstd (g1 - s1/n - xh s2/n)
//                recomputed in fp64, dmax / dmean summed over the tokens, the input gradient row updated;
//                block 0 also finishes the 5 parameter gradients per token from the partials:
//                  dw0 = gamma invstd (sum g1 (m - mbar) - s2/n invstd (w0 Cmm + w1 Cmv))   (and dw1 alike)
//                  db  = 0 in train mode (sum xh = 0), dgamma = s2, dbeta = s1
// Every sum is in a fixed order (no atomics): the results are run-to-run identical.
//
// Parameter layout: the S SpatialAttention modules' parameters are contiguous in the flat parameter
// buffer in state_dict order, 5 floats per token [conv.0.weight (2), conv.0.bias, conv.1.weight (gamma),
// conv.1.bias (beta)], their BN buffers 2 floats per token [running_mean, running_var].
// stats (fp64, [2 S + 8]): per token (mean_f, invstd), then the shared moments
//   [n, mbar, vbar, Cmm, Cmv, Cvv, Km, Kv].
#include "common.h"

namespace {

constexpr int TPAR = 5, TBUF = 2;
constexpr int PS_RW = 4;             // pixel rows per wave in pixel_stats (one batch of loads)
constexpr int PS_ROWS = 4 * PS_RW;   // rows per 256-thread block = one moment partial
constexpr int NMOM = 5;              // partial: sum dm, sum dv, sum dm^2, sum dm dv, sum dv^2
constexpr int NBS = 4;               // backward partial: s1, s2, sum g1 (m - mbar), sum g1 (v - vbar)

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// K independent fp64 sums over a 256-thread block (4 waves), fixed order; every thread gets the totals
template <int K>
__device__ __forceinline__ void block256_sums_d(double (&v)[K], double* red) {
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_sum_d(v[k]);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) red[k * 4 + w] = v[k];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = ((red[k * 4] + red[k * 4 + 1]) + red[k * 4 + 2]) + red[k * 4 + 3];
  __syncthreads();
}

// max (+ first argmax) and mean of RB pixel rows (row indices rows[k], valid when rows[k] >= 0), wave-wide (every
// lane gets the results): the rows' loads are issued together (one latency for RB rows), then each row is scanned
// in channel order -- per row the same arithmetic as a one-row pass, whatever RB.  C <= 512 (host check).
template <int RB>
__device__ __forceinline__ void rows_stats(const float* __restrict__ x, long ldx, const int (&rows)[RB], int C,
                                           int lane, float (&best)[RB], int (&bi)[RB], float (&mean)[RB]) {
  float xv[RB][8];
#pragma unroll
  for (int k = 0; k < RB; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = lane + 64 * j;
      xv[k][j] = (rows[k] >= 0 && c < C) ? x[(long)rows[k] * ldx + c] : 0.f;
    }
#pragma unroll
  for (int k = 0; k < RB; ++k) {
    float bk = -INFINITY, s = 0.f;
    int ik = 0x7fffffff;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = lane + 64 * j;
      if (c < C) {
        const float v = xv[k][j];
        s += v;
        if (v > bk) {
          bk = v;
          ik = c;
        }
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(bk, o, 64);
      const int oi = __shfl_xor(ik, o, 64);
      if (ob > bk || (ob == bk && oi < ik)) {
        bk = ob;
        ik = oi;
      }
    }
    best[k] = bk;
    bi[k] = ik;
    mean[k] = wave_sum(s) / C;
  }
}

// Block = PS_ROWS pixel rows, PS_RW per wave, loaded in one batch together with row 0 (the moments' shift K:
// the same code, so the same values as mx[0], avg[0]): mx / amx / avg per row, and the block's moment partial
// of (max, mean) -> part[blockIdx.x * NMOM + j] (part may be null)
__global__ __launch_bounds__(256) void pixel_stats(int M, int C, const float* __restrict__ x, long ldx,
                                                   float* __restrict__ mx, int* __restrict__ amx,
                                                   float* __restrict__ avg, double* __restrict__ part) {
  __shared__ float sm[PS_ROWS], sv[PS_ROWS];
  __shared__ double red[NMOM * 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = blockIdx.x * PS_ROWS + w * PS_RW;
  int rows[PS_RW + 1];
  rows[0] = part ? 0 : -1;
#pragma unroll
  for (int k = 0; k < PS_RW; ++k) rows[k + 1] = r0 + k < M ? r0 + k : -1;
  float best[PS_RW + 1], mean[PS_RW + 1];
  int bi[PS_RW + 1];
  rows_stats<PS_RW + 1>(x, ldx, rows, C, lane, best, bi, mean);
  if (lane < PS_RW && r0 + lane < M) {   // lane k stores row k
    float bk = best[1], mk = mean[1];
    int ik = bi[1];
#pragma unroll
    for (int k = 1; k < PS_RW; ++k)
      if (lane == k) {
        bk = best[k + 1];
        mk = mean[k + 1];
        ik = bi[k + 1];
      }
    mx[r0 + lane] = bk;
    amx[r0 + lane] = ik;
    avg[r0 + lane] = mk;
    sm[w * PS_RW + lane] = bk;
    sv[w * PS_RW + lane] = mk;
  }
  if (!part) return;
  const float km = best[0], kv = mean[0];
  __syncthreads();
  double v[NMOM] = {0.0, 0.0, 0.0, 0.0, 0.0};
  const int rb = blockIdx.x * PS_ROWS;
  if (threadIdx.x < PS_ROWS && rb + (int)threadIdx.x < M) {
    const double dm = (double)sm[threadIdx.x] - (double)km, dv = (double)sv[threadIdx.x] - (double)kv;
    v[0] = dm;
    v[1] = dv;
    v[2] = dm * dm;
    v[3] = dm * dv;
    v[4] = dv * dv;
  }
  block256_sums_d(v, red);
  if (threadIdx.x < NMOM) part[(long)blockIdx.x * NMOM + threadIdx.x] = v[threadIdx.x];
}

// the shared moments from the P pixel_stats partials, fixed order (every block computes them alike):
// out = [n, mbar, vbar, Cmm, Cmv, Cvv] (fp64)
__device__ __forceinline__ void combine_moments(int P, long n, const double* __restrict__ part, float km, float kv,
                                                double* red, double (&out)[6]) {
  double v[NMOM] = {0.0, 0.0, 0.0, 0.0, 0.0};
  // two of the thread's partials per round, both loaded before either is added (one latency per two; the
  // partials still added in p order)
  for (int p = threadIdx.x; p < P; p += 512) {
    double t[2][NMOM];
    const bool two = p + 256 < P;
#pragma unroll
    for (int j = 0; j < NMOM; ++j) {
      t[0][j] = part[(long)p * NMOM + j];
      t[1][j] = two ? part[(long)(p + 256) * NMOM + j] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < NMOM; ++j) v[j] += t[0][j];
    if (two)
#pragma unroll
      for (int j = 0; j < NMOM; ++j) v[j] += t[1][j];
  }
  block256_sums_d(v, red);
  const double nd = (double)n;
  out[0] = nd;
  out[1] = (double)km + v[0] / nd;
  out[2] = (double)kv + v[1] / nd;
  out[3] = v[2] - v[0] * v[0] / nd;
  out[4] = v[3] - v[0] * v[1] / nd;
  out[5] = v[4] - v[1] * v[1] / nd;
}

// the token's 2->1 conv output for pixel (m, v) in fp64 (exact products of fp32 values), and its BN(1)
// output: forward, backward and vc_tl_relu_mask share this one expression, so they take identical ReLU
// decisions
__device__ __forceinline__ double tl_fv(float m, float v, float w0, float w1, float bc) {
  return (double)w0 * m + (double)w1 * v + (double)bc;
}
__device__ __forceinline__ float tl_bnv(float m, float v, float w0, float w1, float bc, double mean, double invstd,
                                        float gam, float bet, double& xh) {
  xh = (tl_fv(m, v, w0, w1, bc) - mean) * invstd;
  return (float)xh * gam + bet;
}

// g1 = d(loss)/d(BN output) through sigmoid(ReLU(.)) for one element
__device__ __forceinline__ double tl_g1(float m, float v, const float* p, double mean, double invstd, float dav,
                                        double& xh) {
  const float bn = tl_bnv(m, v, p[0], p[1], p[2], mean, invstd, p[3], p[4], xh);
  if (!(bn > 0.f)) return 0.0;
  const float sg = sigmoid_f(bn);
  return (double)(dav * sg * (1.f - sg));
}

// v_mfma_f32_16x16x4_f32 over 16-wide k chunks with the k order permuted alike on both operands: in step j of
// a chunk, lane group g = lane / 16 supplies k = 16 kc + 4 g + j, so each lane feeds the four steps from ONE
// float4 of each operand (a[i] = A(row, 16 kc + 4 g + i), b[i] = B(16 kc + 4 g + i, col)).  The result is
// the chunk's sum over its 16 k in the MFMA's order; acc[r] = C(row 4 g + r, col lane % 16).
__device__ __forceinline__ void mfma_k16(const f32x4& a, const f32x4& b, f32x4& acc) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, b.x, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, b.y, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, b.z, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, b.w, acc, 0, 0, 0);
}

__device__ __forceinline__ f32x4 ld4_lds(const float* p) { return *reinterpret_cast<const f32x4*>(p); }

constexpr int TL_CT = 64;   // output columns (channels) per block of the pooling kernels

// the token statistics of the block into LDS: tok_mean / tok_inv [S] (train: from the shared moments, which
// every block combines alike; eval: the running statistics); block (0, 0) publishes stats (and the moments)
// and updates the running statistics
__device__ __forceinline__ void tl_token_stats(int train, long n, int S, const float* __restrict__ mx,
                                               const float* __restrict__ avg, const float* __restrict__ par,
                                               float* __restrict__ buf, float eps, float momentum,
                                               const double* __restrict__ part, int P, double* __restrict__ stats,
                                               double* red, double* tok_mean, double* tok_inv) {
  double mom[6];
  combine_moments(P, n, part, mx[0], avg[0], red, mom);
  const bool pub = blockIdx.x == 0 && blockIdx.y == 0;
  for (int s = threadIdx.x; s < S; s += 256) {
    const float* p = par + (long)s * TPAR;
    const double w0 = p[0], w1 = p[1], bc = p[2];
    double mean, invstd;
    if (train) {
      mean = w0 * mom[1] + w1 * mom[2] + bc;
      const double m2 = fmax(w0 * w0 * mom[3] + 2.0 * w0 * w1 * mom[4] + w1 * w1 * mom[5], 0.0);
      const double var = m2 / (double)n;
      invstd = 1.0 / sqrt(var + (double)eps);
      if (pub && buf) {
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
    tok_mean[s] = mean;
    tok_inv[s] = invstd;
    if (pub) {
      stats[2 * s] = mean;
      stats[2 * s + 1] = invstd;
    }
  }
  if (pub && threadIdx.x < 8) {
    double v = (double)avg[0];
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (threadIdx.x == j) v = mom[j];
    if (threadIdx.x == 6) v = (double)mx[0];
    stats[2 * S + threadIdx.x] = v;
  }
  __syncthreads();
}

// Forward: grid (B, ceil(C / 64)); block 256 (4 waves).  The block's sample b: its tokens' statistics, the
// attention map a[s][q] = sigmoid(ReLU(BN_s(f_s[q]))) of the tokens in LDS, and the pooled tokens of its 64
// channels Z[b, s, c] = (1/HW) sum_q a[s][q] x[b, q, c] on MFMA (A = a rows, B = x^T staged in LDS; the pixel
// axis padded to 16 with zeros).  a is also written to `a_out` (optional, [B, S, HW]) by the y = 0 blocks.
// The tokens go through the map in chunks of SC (a multiple of 16, chosen on the host so the LDS fits: all
// Sp tokens at once for the model's patches, fewer for large patches); a tile's sum over the pixels is the
// same whatever SC.
// LDS (dynamic): tok_mean / tok_inv [S] doubles, xt [64][Lp + 4], al [SC][Lp + 4], the sample's pooled max /
// mean [Lp] each and the tokens' parameters [S][TPAR] floats (Sp = S rounded up to 16, Lp = HW to 16).
__global__ __launch_bounds__(256) void tl_fwd_pool(int train, int B, int HW, int C, int S, int SC,
                                                   const float* __restrict__ x, long ldx, const float* __restrict__ mx,
                                                   const float* __restrict__ avg, const float* __restrict__ par,
                                                   float* __restrict__ buf, float eps, float momentum,
                                                   const double* __restrict__ part, int P, double* __restrict__ stats,
                                                   float* __restrict__ a_out, float* __restrict__ Z) {
  extern __shared__ __attribute__((aligned(16))) float sm_f[];
  __shared__ double red[NMOM * 4];
  const int b = blockIdx.x, c0 = blockIdx.y * TL_CT;
  const int Sp = (S + 15) & ~15, Lp = (HW + 15) & ~15, LS = Lp + 4;
  double* tok_mean = reinterpret_cast<double*>(sm_f);   // [S]
  double* tok_inv = tok_mean + S;                       // [S]
  float* xt = reinterpret_cast<float*>(tok_inv + S);    // [64][LS]  x^T of the block's channels (16-B aligned)
  float* al = xt + TL_CT * LS;                          // [SC][LS]
  float* mxl = al + SC * LS;                            // [Lp] the sample's pooled max / mean, [S][TPAR] params
  float* avl = mxl + Lp;
  float* parl = avl + Lp;
  const long n = (long)B * HW;
  // the sample's channel tile, transposed into LDS (coalesced rows of 64 channels; zero padding), 4 loads of a
  // thread in flight at a time
  for (int i0 = threadIdx.x; i0 < Lp * TL_CT; i0 += 4 * 256) {
    float xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 256 * u, q = i / TL_CT, c = c0 + (i - q * TL_CT);
      xv[u] = (i < Lp * TL_CT && q < HW && c < C) ? x[((long)b * HW + q) * ldx + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + 256 * u, q = i / TL_CT, cl = i - q * TL_CT;
      if (i < Lp * TL_CT) xt[cl * LS + q] = xv[u];
    }
  }
  for (int i = threadIdx.x; i < Lp; i += 256) {
    mxl[i] = i < HW ? mx[(long)b * HW + i] : 0.f;
    avl[i] = i < HW ? avg[(long)b * HW + i] : 0.f;
  }
  for (int i = threadIdx.x; i < S * TPAR; i += 256) parl[i] = par[i];
  tl_token_stats(train, n, S, mx, avg, par, buf, eps, momentum, part, P, stats, red, tok_mean, tok_inv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r16 = lane & 15, g = lane >> 4;
  const int nct = TL_CT / 16, nkc = Lp / 16;
  const float inv_l = 1.f / (float)HW;
  for (int sb = 0; sb < Sp; sb += SC) {
    const int nsc = min(SC, Sp - sb);   // a multiple of 16
    for (int i = threadIdx.x; i < nsc * Lp; i += 256) {
      const int sl = i / Lp, q = i - sl * Lp, s = sb + sl;
      float av = 0.f;
      if (s < S && q < HW) {
        const float* p = parl + s * TPAR;
        double xh;
        const float bn = tl_bnv(mxl[q], avl[q], p[0], p[1], p[2], tok_mean[s], tok_inv[s], p[3], p[4], xh);
        av = sigmoid_f(fmaxf(bn, 0.f));
        if (a_out && blockIdx.y == 0) a_out[((long)b * S + s) * HW + q] = av;
      }
      al[sl * LS + q] = av;
    }
    __syncthreads();
    const int nst = nsc / 16;
    for (int t = w; t < nst * nct; t += 4) {
      const int st = t / nct, ct = t - st * nct;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int kc = 0; kc < nkc; ++kc) {
        const int k = 16 * kc + 4 * g;
        mfma_k16(ld4_lds(al + (16 * st + r16) * LS + k), ld4_lds(xt + (16 * ct + r16) * LS + k), acc);
      }
      const int c = c0 + 16 * ct + r16;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int s = sb + 16 * st + 4 * g + r;
        if (s < S && c < C) Z[((long)b * S + s) * C + c] = acc[r] * inv_l;
      }
    }
    __syncthreads();   // the next chunk overwrites al
  }
}

// Backward part 1: grid (B, ceil(S / 16)); block 256.  da[b, s, q] = (1/HW) sum_c dZ[b, s, c] x[b, q, c] for
// the block's 16 tokens (MFMA, both operands as float4 runs of their rows straight from L2), kept in registers;
// then per token the fp64 sums over this sample's pixels of g1, g1 xh, g1 (m - mbar), g1 (v - vbar) ->
// part[(b * S + s) * NBS + j] (summed over the pixel tiles in a fixed order), and (round 6) per pixel the fp64
// sums over the block's 16 tokens of w0_s gi_s g1 and w1_s gi_s g1 (gi = gamma invstd) -> apart[((b * nsb +
// blockIdx.y) * HW + q) * 2 + j]: the token-sum part of the pixel gradients, so tl_bwd_dx needs neither da nor a
// per-token loop (the batch-statistics part of df is affine in the pixel's (max, mean), section below).
// Up to TLDA_W waves per block: one 16-pixel tile per wave up to HW = 16 TLDA_W (a wave with two tiles doubled
// the block's chain of dependent k-chunk loads).  Round 6: the block has exactly min(tiles, TLDA_W) waves (hsi1:
// 6, hsi2: 4) -- the round-5 blocks of 8 carried 2 / 4 idle waves whose registers and slots the concurrent
// selective-scan backward could not use; the per-token sums over the missing waves were exact zeros, so the
// results are unchanged bit for bit
constexpr int TLDA_W = 8;
__global__ __launch_bounds__(64 * TLDA_W) void tl_bwd_da(int B, int HW, int C, int S, const float* __restrict__ x,
                                                         long ldx, const float* __restrict__ mx,
                                                         const float* __restrict__ avg, const float* __restrict__ par,
                                                         const double* __restrict__ stats,
                                                         const float* __restrict__ dZ, double* __restrict__ part,
                                                         double* __restrict__ apart) {
  __shared__ double tsum[TLDA_W][16][NBS];   // [wave][token][sum]
  const int b = blockIdx.x, s0 = blockIdx.y * 16;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r16 = lane & 15, g = lane >> 4;
  const int Lp = (HW + 15) & ~15, nqt = Lp / 16, nkc = (C + 15) / 16;
  const int nw = blockDim.x >> 6;
  const double mbar = stats[2 * S + 1], vbar = stats[2 * S + 2];
  const float inv_l = 1.f / (float)HW;
  // this lane's A row (token s0 + r16) and the tokens of its accumulator rows (s0 + 4 g + r)
  const int sa = s0 + r16;
  const float* arow = dZ + ((long)b * S + min(sa, S - 1)) * C;
  float tp[4][TPAR];
  double tmean[4], tinv[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int s = s0 + 4 * g + r;
    const bool ok = s < S;
#pragma unroll
    for (int j = 0; j < TPAR; ++j) tp[r][j] = ok ? par[(long)s * TPAR + j] : 0.f;
    tmean[r] = ok ? stats[2 * s] : 0.0;
    tinv[r] = ok ? stats[2 * s + 1] : 0.0;
  }
  double v[4][NBS];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < NBS; ++j) v[r][j] = 0.0;
  for (int qt = w; qt < nqt; qt += nw) {
    const int qb = 16 * qt + r16;   // this lane's B column (pixel)
    const float* brow = x + ((long)b * HW + min(qb, HW - 1)) * ldx;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    constexpr int KB = 4;   // k chunks whose loads are issued together (8: 182 VGPRs, slower)
    for (int kc0 = 0; kc0 < nkc; kc0 += KB) {
      f32x4 av[KB], bv[KB];
#pragma unroll
      for (int u = 0; u < KB; ++u) {
        const int k = 16 * (kc0 + u) + 4 * g;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const bool kok = kc0 + u < nkc && k < C;
        av[u] = (kok && sa < S) ? *reinterpret_cast<const f32x4*>(arow + k) : z;
        bv[u] = (kok && qb < HW) ? *reinterpret_cast<const f32x4*>(brow + k) : z;
      }
#pragma unroll
      for (int u = 0; u < KB; ++u)
        if (kc0 + u < nkc) mfma_k16(av[u], bv[u], acc);
    }
    // acc[r] = da(token s0 + 4 g + r, pixel qb') with qb' = 16 qt + r16 for the C/D layout: col = lane % 16
    const int q = 16 * qt + r16;
    const float m = q < HW ? mx[(long)b * HW + q] : 0.f, vq = q < HW ? avg[(long)b * HW + q] : 0.f;
    double a0 = 0.0, a1 = 0.0;   // this lane's 4 tokens of sum_s w0 gi g1, sum_s w1 gi g1 (token order)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int s = s0 + 4 * g + r;
      const float dav = acc[r] * inv_l;
      if (s < S && q < HW) {
        double xh;
        const double g1 = tl_g1(m, vq, tp[r], tmean[r], tinv[r], dav, xh);
        v[r][0] += g1;
        v[r][1] += g1 * xh;
        v[r][2] += g1 * ((double)m - mbar);
        v[r][3] += g1 * ((double)vq - vbar);
        const double gg = (double)tp[r][3] * tinv[r] * g1;
        a0 += (double)tp[r][0] * gg;
        a1 += (double)tp[r][1] * gg;
      }
    }
    // the 4 lane groups (tokens 4 g .. 4 g + 3) pairwise: (g0 + g1) + (g2 + g3)
    a0 += __shfl_xor(a0, 16, 64);
    a1 += __shfl_xor(a1, 16, 64);
    a0 += __shfl_xor(a0, 32, 64);
    a1 += __shfl_xor(a1, 32, 64);
    if (g == 0 && q < HW) {
      double* ap = apart + (((long)b * gridDim.y + blockIdx.y) * HW + q) * 2;
      ap[0] = a0;
      ap[1] = a1;
    }
  }
  // per token: the 16 pixel lanes of the row group, then the waves in order
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int j = 0; j < NBS; ++j) {
      double t = v[r][j];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o, 64);
      v[r][j] = t;
    }
  if (r16 == 0)
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < NBS; ++j) tsum[w][4 * g + r][j] = v[r][j];
  __syncthreads();
  if (threadIdx.x < 16 * NBS) {
    const int tl = threadIdx.x / NBS, j = threadIdx.x - tl * NBS, s = s0 + tl;
    double t = tsum[0][tl][j];
#pragma unroll
    for (int ww = 1; ww < nw; ++ww) t += tsum[ww][tl][j];   // the waves in order
    if (s < S) part[((long)b * S + s) * NBS + j] = t;
  }
}

// Backward part 2: grid (B, ceil(C / 64)); block 256.  The tokens' s1 / s2 over the batch (the per-sample
// partials summed in 4 interleaved sample quarters, then the quarters in order), then for the block's sample
// and 64 channels
//   dx[b, q, c] = (1/HW) sum_s a[s][q] dZ[b, s, c]                      (MFMA; a as the forward wrote it)
//               + (sum_s w1_s df_s[q]) / C + [c == argmax_q] sum_s w0_s df_s[q]
// with df_s[q] = gi_s (g1 - s1/n - xh s2/n) (train; eval gi g1), gi = gamma invstd.  Round 6: the pixel sums
// split as  sum_s wj_s df_s[q] = A_j[q] - K_j - (alpha_j m_q + beta_j v_q + gamma_j)  with A_j = sum_s wj_s gi_s g1
// (tl_bwd_da's per-16-token partials, summed here in token-block order) and -- xh being affine in the pixel's
// pooled (m, v) -- K_j, alpha_j, beta_j, gamma_j per-batch scalars from the tokens' statistics (fp64 block sums);
// the round-5 form recomputed every token's g1 for every pixel in each of a sample's channel blocks.
// Block (0, 0) also writes the tokens' 5 parameter gradients (dparams).  The product runs as dx^T [c][q]: the
// A operand (dZ rows, 16 channels x 4 tokens per MFMA) and the B operand (a [s][q]) from LDS.  The pixels go
// through a and the MFMA tiles in chunks of QC (a multiple of 16 chosen on the host so the LDS fits: all Lp
// pixels at once for the model's patches); every sum is over tokens, so the results do not depend on QC.
// LDS (dynamic): q4 [4][S][2], tsum [2][S], tst [2][S] doubles; dzl [S4][68], al [S4][QC + 4],
// tpar [S][TPAR] (rounded up to 4), gq [2][QC] floats.
constexpr int TLDX_RED = 8 * 4;   // doubles of tl_bwd_dx's static reduction buffer
__global__ __launch_bounds__(256) void tl_bwd_dx(int train, int B, int HW, int C, int S, int QC,
                                                 const float* __restrict__ mx, const float* __restrict__ avg,
                                                 const int* __restrict__ amx, const float* __restrict__ par,
                                                 const double* __restrict__ stats, const float* __restrict__ a,
                                                 const float* __restrict__ dZ, const double* __restrict__ part,
                                                 const double* __restrict__ apart, float* __restrict__ dx, long lddx,
                                                 float* __restrict__ gpar) {
  extern __shared__ __attribute__((aligned(16))) float sm_f[];
  __shared__ double red[TLDX_RED];
  const int b = blockIdx.x, c0 = blockIdx.y * TL_CT;
  const bool b00 = blockIdx.x == 0 && blockIdx.y == 0;
  const int S4 = (S + 3) & ~3, Lp = (HW + 15) & ~15, QS = QC + 4;
  const int nsb = (S + 15) / 16;   // tl_bwd_da's token blocks
  constexpr int DZS = TL_CT + 4;
  double* q4 = reinterpret_cast<double*>(sm_f);   // [4][S][2] per token, 4 sample-quarter sums of two columns
  double* tsum = q4 + 8 * S;                      // [2][S]  s1 / n, s2 / n
  double* tst = tsum + 2 * S;                     // [2][S]  mean, invstd
  float* dzl = reinterpret_cast<float*>(tst + 2 * S);   // [S4][DZS]  dZ[b, s, c0 + cl] (zero padded; 16-B aligned)
  float* al = dzl + S4 * DZS;                     // [S4][QS]  a[s][q0 + ql] (zero padded)
  float* tpar = al + S4 * QS;                     // [S][TPAR]
  float* gq = tpar + ((S * TPAR + 3) & ~3);       // [2][QC] per pixel: sum_s w0 df, (sum_s w1 df) / C
  const long n = (long)B * HW;
  const double nd = (double)n;
  for (int i = threadIdx.x; i < S4 * (TL_CT / 4); i += 256) {   // float4 runs of the block's 64 channels
    const int s = i / (TL_CT / 4), c4 = 4 * (i - s * (TL_CT / 4)), c = c0 + c4;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (s < S) {
      const float* src = dZ + ((long)b * S + s) * C + c;
      if (c + 3 < C) v = *reinterpret_cast<const f32x4*>(src);
      else
        for (int j = 0; j < 4; ++j)
          if (c + j < C) v[j] = src[j];
    }
    *reinterpret_cast<f32x4*>(dzl + s * DZS + c4) = v;
  }
  for (int i = threadIdx.x; i < S * TPAR; i += 256) tpar[i] = par[i];
  for (int s = threadIdx.x; s < S; s += 256) {
    tst[s] = stats[2 * s];
    tst[S + s] = stats[2 * s + 1];
  }
  // the batch sums of partial columns j0, j0 + 1: 4 interleaved sample quarters, then the quarters in order
  auto batch_sums = [&](int j0) {
    for (int i = threadIdx.x; i < 4 * S; i += 256) {
      const int s = i >> 2, u = i & 3;
      double t0 = 0.0, t1 = 0.0;
      if (B <= 64) {   // every load of the quarter issued at once (one latency), summed in the loop's order
        double p0[16], p1[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int bb = u + 16 * (k >> 2) + 4 * (k & 3);
          p0[k] = bb < B ? part[((long)bb * S + s) * NBS + j0] : 0.0;
          p1[k] = bb < B ? part[((long)bb * S + s) * NBS + j0 + 1] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          t0 += p0[k];
          t1 += p1[k];
        }
        q4[(u * S + s) * 2] = t0;
        q4[(u * S + s) * 2 + 1] = t1;
        continue;
      }
      for (int bb0 = u; bb0 < B; bb0 += 16) {
        double p0[4], p1[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int bb = bb0 + 4 * k;
          p0[k] = bb < B ? part[((long)bb * S + s) * NBS + j0] : 0.0;
          p1[k] = bb < B ? part[((long)bb * S + s) * NBS + j0 + 1] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          t0 += p0[k];
          t1 += p1[k];
        }
      }
      q4[(u * S + s) * 2] = t0;
      q4[(u * S + s) * 2 + 1] = t1;
    }
    __syncthreads();
  };
  auto qsum = [&](int s, int j) {
    return ((q4[s * 2 + j] + q4[(S + s) * 2 + j]) + q4[(2 * S + s) * 2 + j]) + q4[(3 * S + s) * 2 + j];
  };
  batch_sums(0);
  for (int s = threadIdx.x; s < S; s += 256) {
    tsum[s] = qsum(s, 0) / nd;
    tsum[S + s] = qsum(s, 1) / nd;
  }
  __syncthreads();
  // the per-batch scalars of the pixel sums (train): per token, t_j = w_j gi, u = (s2 / n) invstd;
  //   K_j = sum t_j s1/n, alpha_j = sum t_j u w0, beta_j = sum t_j u w1, gamma_j = sum t_j u (bc - mean)
  double sc[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  if (train) {
    for (int s = threadIdx.x; s < S; s += 256) {   // a thread's tokens in order
      const float* ps = tpar + s * TPAR;
      const double gi = (double)ps[3] * tst[S + s];
      const double t0 = (double)ps[0] * gi, t1 = (double)ps[1] * gi, u = tsum[S + s] * tst[S + s];
      const double w0 = ps[0], w1 = ps[1], bm = (double)ps[2] - tst[s];
      sc[0] += t0 * tsum[s];
      sc[1] += t0 * u * w0;
      sc[2] += t0 * u * w1;
      sc[3] += t0 * u * bm;
      sc[4] += t1 * tsum[s];
      sc[5] += t1 * u * w0;
      sc[6] += t1 * u * w1;
      sc[7] += t1 * u * bm;
    }
  }
  block256_sums_d<8>(sc, red);   // (uniform: every thread takes part)
  if (b00) {   // parameter gradients: the other two partial columns too
    batch_sums(2);
    for (int s = threadIdx.x; s < S; s += 256) {
      const double t0 = tsum[s] * nd, t1 = tsum[S + s] * nd;
      const double t2 = qsum(s, 0);
      const double t3 = qsum(s, 1);
      const float* ps = tpar + s * TPAR;
      const double w0 = ps[0], w1 = ps[1], gam = ps[3];
      const double invstd = tst[S + s];
      const double* mom = stats + 2 * S;   // n, mbar, vbar, Cmm, Cmv, Cvv
      double gw0, gw1, gb;
      if (train) {
        const double k = t1 / nd * invstd;
        gw0 = gam * invstd * (t2 - k * (w0 * mom[3] + w1 * mom[4]));
        gw1 = gam * invstd * (t3 - k * (w0 * mom[4] + w1 * mom[5]));
        gb = 0.0;   // sum_i df_i = gamma invstd (s1 - s1 - s2/n sum_i xh_i) and sum_i xh_i = 0
      } else {
        gw0 = gam * invstd * (t2 + mom[1] * t0);
        gw1 = gam * invstd * (t3 + mom[2] * t0);
        gb = gam * invstd * t0;
      }
      float* gp = gpar + (long)s * TPAR;
      gp[0] = (float)gw0;
      gp[1] = (float)gw1;
      gp[2] = (float)gb;
      gp[3] = (float)t1;
      gp[4] = (float)t0;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r16 = lane & 15, g = lane >> 4;
  const int nct = TL_CT / 16, nk = S4 / 4;
  const float inv_l = 1.f / (float)HW;
  for (int q0 = 0; q0 < Lp; q0 += QC) {
    const int nq = min(QC, Lp - q0);   // a multiple of 16
    // the attention maps of the chunk's pixels into LDS (rows of HW contiguous floats), zero padded
    for (int i = threadIdx.x; i < S4 * nq; i += 256) {
      const int sl = i / nq, ql = i - sl * nq, q = q0 + ql;
      al[sl * QS + ql] = (sl < S && q < HW) ? a[((long)b * S + sl) * HW + q] : 0.f;
    }
    // the pixel gradients: the token-block partials in order, then the affine batch-statistics part
    for (int ql = threadIdx.x; ql < nq; ql += 256) {
      const int q = q0 + ql;
      double gm = 0.0, ga = 0.0;
      if (q < HW) {
        const double* ap = apart + ((long)b * nsb * HW + q) * 2;
        for (int t = 0; t < nsb; ++t) {
          gm += ap[(long)t * HW * 2];
          ga += ap[(long)t * HW * 2 + 1];
        }
        if (train) {
          const double m = mx[(long)b * HW + q], v = avg[(long)b * HW + q];
          gm -= sc[0] + (sc[1] * m + sc[2] * v + sc[3]);
          ga -= sc[4] + (sc[5] * m + sc[6] * v + sc[7]);
        }
      }
      gq[ql] = (float)gm;
      gq[QC + ql] = (float)(ga / (double)C);
    }
    __syncthreads();
    // dx^T tiles: rows = channels (16 per tile), cols = pixels (16 per tile), k = tokens (4 per MFMA)
    const int nqt = nq / 16;
    for (int t = w; t < nqt * nct; t += 4) {
      const int ct = t / nqt, qt = t - ct * nqt;
      const int cl = 16 * ct + r16;   // this lane's A row (channel, block-local)
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < nk; ++k) {
        const int s = 4 * k + g;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(dzl[s * DZS + cl], al[s * QS + 16 * qt + r16], acc, 0, 0, 0);
      }
      // acc[r] = dx^T (channel c0 + 16 ct + 4 g + r, pixel q0 + 16 qt + r16): 4 adjacent channels of one pixel
      const int ql = 16 * qt + r16, q = q0 + ql, cb = c0 + 16 * ct + 4 * g;
      if (q < HW) {
        const float gmf = gq[ql], gaf = gq[QC + ql];
        const int am = amx[(long)b * HW + q];
        float* dr = dx + ((long)b * HW + q) * lddx;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = cb + r;
          if (c < C) dr[c] = acc[r] * inv_l + (gaf + (c == am ? gmf : 0.f));
        }
      }
    }
    __syncthreads();   // the next chunk overwrites al / gq
  }
}

// mask[(b*S + s)*HW + q] = (BN(1) output > 0): the ReLU decisions attn_fwd / attn_bwd / pixel_bwd take
__global__ __launch_bounds__(256) void attn_mask(int B, int HW, int S, const float* __restrict__ mx,
                                                 const float* __restrict__ avg, const float* __restrict__ par,
                                                 const double* __restrict__ stats, unsigned char* __restrict__ mask) {
  const int s = blockIdx.y;
  const long n = (long)B * HW, i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float* p = par + (long)s * TPAR;
  double xh;
  const float bn = tl_bnv(mx[i], avg[i], p[0], p[1], p[2], stats[2 * s], stats[2 * s + 1], p[3], p[4], xh);
  const long b = i / HW, q = i - b * HW;
  mask[(b * S + s) * HW + q] = bn > 0.f ? 1 : 0;
}

}  // namespace

static long tl_pix_partials(long M) { return (long)vc_cdiv(M, PS_ROWS) * NMOM; }

// fp64 scratch of one TokenLearner call site: the pixel_stats moment partials, the per-(sample, token) backward
// partials, and the backward's per-(sample, 16-token block, pixel) pixel-gradient partials
static long tl_apart(int B, int HW, int S) { return (long)B * ((S + 15) / 16) * HW * 2; }
VC_API int vc_tl_ws_floats(int B, int HW, int S) {
  if (B <= 0 || HW <= 0 || S <= 0) return -1;
  const long dbl = tl_pix_partials((long)B * HW) + (long)B * S * NBS + tl_apart(B, HW, S);
  return (int)(2 * dbl + 2);
}

VC_API int vc_tl_pixel_stats(long M, int C, const float* x, long ldx, float* mx, int* amx, float* avg, double* ws,
                             hipStream_t stream) {
  VC_REQUIRE(M >= 0 && C > 0 && C <= 512);
  VC_REQUIRE_I32(M);
  if (M == 0) return VC_OK;
  hipLaunchKernelGGL(pixel_stats, dim3(vc_cdiv(M, PS_ROWS)), dim3(256), 0, stream, (int)M, C, x, ldx, mx, amx, avg,
                     ws);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// LDS plans.  The dynamic allocation plus the kernel's static __shared__ arrays must fit the CU's 160 KB
constexpr size_t TL_LDS_MAX = 160 * 1024;
constexpr size_t TL_FWD_STATIC = NMOM * 4 * sizeof(double);   // tl_fwd_pool's `red`
static size_t tl_fwd_lds(int HW, int S, int SC) {
  const int Lp = (HW + 15) & ~15;
  return 2 * (size_t)S * sizeof(double) + (size_t)((TL_CT + SC) * (Lp + 4) + 2 * Lp + S * TPAR) * sizeof(float);
}
constexpr size_t TL_BWD_STATIC = TLDX_RED * sizeof(double);   // tl_bwd_dx's `red`
static size_t tl_bwd_lds(int S, int QC) {
  const int S4 = (S + 3) & ~3;
  return 12 * (size_t)S * sizeof(double) +
         (size_t)(S4 * (TL_CT + 4 + QC + 4) + ((S * TPAR + 3) & ~3) + 2 * QC) * sizeof(float);
}
// the token chunk of tl_fwd_pool: all tokens when they fit, else the largest multiple of 16 that does (0: none)
static int tl_fwd_sc(int HW, int S) {
  for (int sc = (S + 15) & ~15; sc >= 16; sc -= 16)
    if (tl_fwd_lds(HW, S, sc) + TL_FWD_STATIC <= TL_LDS_MAX) return sc;
  return 0;
}
// the pixel chunk of tl_bwd_dx, alike
static int tl_bwd_qc(int HW, int S) {
  for (int qc = (HW + 15) & ~15; qc >= 16; qc -= 16)
    if (tl_bwd_lds(S, qc) + TL_BWD_STATIC <= TL_LDS_MAX) return qc;
  return 0;
}

VC_API int vc_tl_check(int HW, int C, int S) {
  VC_REQUIRE(HW > 0 && C > 0 && C <= 512 && S > 0);
  VC_REQUIRE(tl_fwd_sc(HW, S) > 0 && tl_bwd_qc(HW, S) > 0);
  return VC_OK;
}

VC_API int vc_tl_fwd(int train, int B, int HW, int C, int S, const float* x, long ldx, const float* mx,
                     const float* avg, const float* params, float* bn_buffers, float eps, float momentum,
                     const double* ws, double* stats, float* a, float* Z, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && C > 0 && S > 0 && ws && stats && Z);
  const int SC = tl_fwd_sc(HW, S);
  VC_REQUIRE(SC > 0);
  VC_REQUIRE_I32((long)B * HW * (S > C ? S : C));
  const int P = vc_cdiv((long)B * HW, PS_ROWS);
  hipLaunchKernelGGL(tl_fwd_pool, dim3(B, vc_cdiv(C, TL_CT)), dim3(256), tl_fwd_lds(HW, S, SC), stream, train, B, HW,
                     C, S, SC, x, ldx, mx, avg, params, bn_buffers, eps, momentum, ws, P, stats, a, Z);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_tl_bwd(int train, int B, int HW, int C, int S, const float* x, long ldx, const float* mx,
                     const float* avg, const int* amx, const float* params, const double* stats, const float* a,
                     const float* dZ, double* ws, float* dx, long lddx, float* dparams, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && C > 0 && C % 4 == 0 && ldx % 4 == 0 && S > 0 && ws && a && dx);
  VC_REQUIRE(((uintptr_t)x & 15) == 0 && ((uintptr_t)dZ & 15) == 0);
  const int QC = tl_bwd_qc(HW, S);
  VC_REQUIRE(QC > 0);
  VC_REQUIRE_I32((long)B * HW * (S > C ? S : C));
  double* part = ws + tl_pix_partials((long)B * HW);
  double* apart = part + (long)B * S * NBS;
  const int da_waves = std::min(TLDA_W, (HW + 15) / 16);
  hipLaunchKernelGGL(tl_bwd_da, dim3(B, vc_cdiv(S, 16)), dim3(64 * da_waves), 0, stream, B, HW, C, S, x, ldx, mx, avg, params,
                     stats, dZ, part, apart);
  VC_CHECK_LAUNCH();
  hipLaunchKernelGGL(tl_bwd_dx, dim3(B, vc_cdiv(C, TL_CT)), dim3(256), tl_bwd_lds(S, QC), stream, train, B, HW, C, S,
                     QC, mx, avg, amx, params, stats, a, dZ, part, apart, dx, lddx, dparams);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_tl_relu_mask(int B, int HW, int S, const float* mx, const float* avg, const float* params,
                           const double* stats, unsigned char* mask, hipStream_t stream) {
  VC_REQUIRE(B > 0 && HW > 0 && S > 0);
  VC_REQUIRE_I32((long)B * HW);
  hipLaunchKernelGGL(attn_mask, dim3(vc_cdiv((long)B * HW, 256), S), dim3(256), 0, stream, B, HW, S, mx, avg, params,
                     stats, mask);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
