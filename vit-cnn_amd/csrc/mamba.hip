// Selective-state-space mixer of hsiMamba over its 10 scan orders, fused for CDNA4.
//
// Reference: hsiMamba.forward '81_2+8' / '49_2+8' (Mutimodality_Mamba7.py:608-701, :787-867)
// feeding transformers' MambaMixer torch fallback (modeling_mamba.py:359-481, selective scan
// :175-283).  The 10 direction copies are never materialised: LayerNorm and in_proj act per
// token (they commute with the permutations) and out_proj is linear and bias-free (it commutes
// with the gated sum), so the host computes LN + in_proj once per token, and these kernels
// gather each direction's sequence through an int32 order table:
//
//   u[k,b,t,:]  = SiLU(causal depthwise conv1d_k4(xz[b, order_k(t), :D]) + bias)      (dirconv)
//   xdbl        = u x_proj^T                                                          (vc_gemm)
//   yp[k,b,t,d] = sum_n C_t[n] h_t[d,n] + D_d u_t[d]                                   (scan)
//                 h_t = exp(dt*A) h_{t-1} + dt*B_t*u_t,  dt = softplus(W_dt dtr_t + b_dt)
//   YP[b,l,:]   = sum_k softmax(gate)_k yp[k, b, inv_k(l), :]                          (combine)
//   ysum[b,l,:] = YP[b,l,:] * SiLU(z[b,l,:])
// The SiLU(z) gate of each direction's output, y_k = yp_k * SiLU(z(token)), is token-wise, so
// it commutes with the un-permute and the gated sum: it is applied once per token after the
// combine, and its backward (dz, and d(yp) = g_k dysum SiLU(z)) is an elementwise pass outside
// the sequential scan (gate_bwd) instead of 10 x 16 redundant evaluations inside it.
//
// The scan runs one lane per channel with the 16-wide state in fp32 registers (see scan_fwd);
// the backward re-runs the recurrence from the forward's segment checkpoints (nothing of size
// [seq, D, L, N] is ever stored), and every reduction is fixed-order.
#include "common.h"

namespace {

constexpr int NST = 16;     // ssm state size (config state_size=16, Mutimodality_Mamba7.py:316)

// Direction gather + causal conv1d + SiLU.  A thread owns DC_T consecutive tokens of one (direction,
// sample, channel) and slides the 4-tap window along them, so each gathered input is loaded once
// (a thread per output would load it 4 times, with 4 order-table reads); lanes run along the channels
// (coalesced rows).  Index decomposition with launch-time FastDivs.  A tap before the sequence start
// contributes fma(w, 0, pre) = pre, i.e. it is skipped as in the reference's left zero padding.
constexpr int DC_T = 8;
__global__ void dirconv_fwd_run(int total, FastDiv fD, FastDiv fC, FastDiv fB, int L, const int* __restrict__ order,
                                const float* __restrict__ xz, const float* __restrict__ cw,
                                const float* __restrict__ cb, float* __restrict__ u) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int D = fD.div;
  int d, c, b;
  const int sc = fdivmod(idx, fD, d);
  const int sq = fdivmod(sc, fC, c);
  const int k = fdivmod(sq, fB, b);
  const int* ord = order + k * L;
  const float* xb = xz + (long)b * L * (2 * D) + d;
  const float w0 = cw[d * 4], w1 = cw[d * 4 + 1], w2 = cw[d * 4 + 2], w3 = cw[d * 4 + 3], bias = cb[d];
  const int t0 = c * DC_T;
  float x[DC_T + 3];
#pragma unroll
  for (int i = 0; i < DC_T + 3; ++i) {
    const int tau = t0 - 3 + i;
    x[i] = (tau >= 0 && tau < L) ? xb[ord[tau] * (2 * D)] : 0.f;
  }
  float* ub = u + ((long)sq * L + t0) * D + d;
#pragma unroll
  for (int i = 0; i < DC_T; ++i) {
    if (t0 + i < L) {
      float pre = fmaf(w0, x[i], bias);
      pre = fmaf(w1, x[i + 1], pre);
      pre = fmaf(w2, x[i + 2], pre);
      pre = fmaf(w3, x[i + 3], pre);
      ub[(long)i * D] = silu_f(pre);
    }
  }
}

__device__ __forceinline__ float gate_softmax(const float* logits, int ndir, int k) {
  float mx = logits[0];
  for (int i = 1; i < ndir; ++i) mx = fmaxf(mx, logits[i]);
  float den = 0.f;
  for (int i = 0; i < ndir; ++i) den += __expf(logits[i] - mx);
  return __expf(logits[k] - mx) / den;
}

struct ScanArgs {
  int B, L, D, R;
  const float* u;      // [nseq*L, D]
  const float* xdbl;   // [nseq*L, R+2N]
  const int* order;    // [ndir*L]
  const float* wdt;    // [D, R]
  const float* bdt;    // [D]
  const float* alog;   // [D, N]
  const float* dskip;  // [D]
};

// Selective scan.  Block = one sequence s = k*B + b (all channels); wave = 16 channels x 4 state
// groups: lane = q * 16 + c, row q holds states n = 4q..4q+3 of channel 16*wave + c.
//
// gfx950 issues one wave64 VALU instruction per 4 cycles (an exp per 8) and the scan has little
// else to do, so it is bounded by VALU issue; the mapping decides how much work is redundant and
// how many waves hide latency.  Per (token, channel) work (dt*u, du, ddt, the dt lookup) is repeated
// 4x (once per row) instead of 16x in a lane-per-state mapping, each lane's 4 states give 4
// independent chains, and 4x more waves than a lane-per-channel mapping keep every SIMD busy.
// Sums over the 16 states are 4 in-register terms plus one cross-row sum (two VALU half swaps);
// the backward's dB_t / dC_t (sums over channels) are a reduce-scatter inside each 16-lane row
// (DPP) and a fixed-order combine of the waves' partials in LDS.
//
// dt = softplus(W_dt x_t + b_dt) depends on the token only through x_t, so it is computed for all
// (token, channel) pairs up front into LDS, a pass without serial dependence.  The forward stores
// the state entering every SCK-token segment ([nseq][nseg][16][D]); the backward re-runs one
// segment at a time from those checkpoints (the segment's states stay in registers) and sweeps it
// in reverse, so nothing of size [seq, L, D, 16] is ever stored.
// 4 tokens per segment (measured on MI355X): the backward's per-segment registers (states, cached
// exp(dt A), prefetched operands) fit 128 VGPRs, i.e. 4 waves per SIMD, so all 640 sequence blocks
// of a launch are resident at once (8 tokens: 182 VGPRs, 2 waves per SIMD, 3 rounds of blocks;
// hsi1 backward 211 -> 156 us).  The checkpoints cost 16 * D floats per segment of HBM traffic.
constexpr int SCK = 4;
constexpr int NQ = 4;                   // states per lane
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

__device__ __forceinline__ int seg_count(int L) { return (L + SCK - 1) / SCK; }

// softplus(beta = 1, threshold = 20) with an accurate log1p: log1p(e) = log(1 + e) * e / ((1 + e) - 1)
__device__ __forceinline__ float softplus_c(float x) {
  const float e = __builtin_amdgcn_exp2f(x * LOG2E);
  const float u = 1.f + e;
  const float lp = u == 1.f ? e : __builtin_amdgcn_logf(u) * LN2 * (e * __builtin_amdgcn_rcpf(u - 1.f));
  return x > 20.f ? x : lp;
}

// exp(x) - 1 without cancellation near 0: a degree-6 Taylor polynomial for |x| < 1/4 (truncation
// < 5e-8 relative), exp(x) - 1 elsewhere
__device__ __forceinline__ float expm1_c(float x) {
  const float p = x * (1.f + x * (0.5f + x * (1.f / 6 + x * (1.f / 24 + x * (1.f / 120 + x * (1.f / 720))))));
  float e = __builtin_amdgcn_exp2f(x * LOG2E) - 1.f;
  asm volatile("" : "+v"(e));   // both sides computed, then a select: no divergent branch
  return fabsf(x) < 0.25f ? p : e;
}

// LDS image of one sequence (Lp = SCK * segments tokens; rows L..Lp-1 zero):
//   Bs [Lp][16], Cs [Lp][16] (lane (q, c) reads its 4 states of a token as one ds_read_b128),
//   dts [Lp][Dp] dt per (token, channel), Dp = 16 * waves; xr [Lp][R] the dt-rank columns.
struct SeqLds {
  float *Bs, *Cs, *dts, *xr;
  __device__ SeqLds(float* base, int Lp, int R, int Dp) {
    Bs = base;
    Cs = Bs + Lp * NST;
    dts = Cs + Lp * NST;
    xr = dts + Lp * Dp;
  }
};
static size_t seq_lds_floats(int L, int R, int Dp) {
  const size_t Lp = (size_t)((L + SCK - 1) / SCK) * SCK;
  return Lp * (2 * NST + Dp + R);
}

// raw buffer access (MUBUF, vector memory): a resource over [p, p + bytes), 32-bit byte offsets;
// loads past the end return 0, stores past the end are dropped
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const float* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float buf_ld(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void buf_st(__amdgpu_buffer_rsrc_t r, unsigned off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}

template <int RT>
__device__ __forceinline__ void stage_dt(const ScanArgs& a, const SeqLds& m, int Lp, int Dp);

template <int RT>
__device__ __forceinline__ void stage_seq(const ScanArgs& a, int s, const SeqLds& m, int Lp, int Dp) {
  const int R = RT ? RT : a.R;
  const int XW = R + 2 * NST;
  const float* src = a.xdbl + (long)s * a.L * XW;
  const int n = a.L * XW, tot = Lp * XW;
  const int nt = blockDim.x;
  constexpr int SB = 8;
  // rows past L read 0 (buffer range check); each element's LDS destination is selected, not branched
  const auto r_src = buf_rsrc(src, (unsigned)(n * 4));
  for (int base = 0; base < tot; base += SB * nt) {
    float v[SB];
#pragma unroll
    for (int j = 0; j < SB; ++j) v[j] = buf_ld(r_src, (unsigned)(base + j * nt + threadIdx.x) * 4u);
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      const int i = base + j * nt + threadIdx.x;
      if (i < tot) {
        const int t = i / XW, col = i - t * XW;
        float* dst = col < R ? m.xr + t * R + col
                             : (col < R + NST ? m.Bs + t * NST + (col - R) : m.Cs + t * NST + (col - R - NST));
        *dst = v[j];
      }
    }
  }
  stage_dt<RT>(a, m, Lp, Dp);
}

// dt for every (token, channel) from the staged dt-rank columns m.xr (barriers on both sides): the block
// has 4 * Dp threads, so thread i handles channel c = i % Dp of tokens i / Dp, i / Dp + 4, ...; its W_dt
// row and bias are loaded once
template <int RT>
__device__ __forceinline__ void stage_dt(const ScanArgs& a, const SeqLds& m, int Lp, int Dp) {
  const int R = RT ? RT : a.R;
  const int nt = blockDim.x;
  const int c = threadIdx.x % Dp;
  const bool valid = c < a.D;
  const int cc = valid ? c : 0;
  float w[RT ? RT : 64];
#pragma unroll
  for (int r = 0; r < R; ++r) w[r] = valid ? a.wdt[(long)cc * R + r] : 0.f;
  const float bias = valid ? a.bdt[cc] : 0.f;
  __syncthreads();
  for (int t = threadIdx.x / Dp; t < Lp; t += nt / Dp) {
    const float* row = m.xr + t * R;
    float dtl = bias;
#pragma unroll
    for (int r = 0; r < R; ++r) dtl += w[r] * row[r];
    m.dts[t * Dp + c] = softplus_c(dtl);
  }
  __syncthreads();
}

// ---------------------------------------------------------------- fused front end (scan_fwd<RT, true>)
// The direction conv and x_proj of a sequence computed inside the scan block, before its scan:
//   phase 1  u[t, c] = SiLU(conv1d_k4(xz[b, order_k(t), c]) + bias) -> LDS image UD [Lp][Dp] (the dts
//            region, not yet in use) and U in HBM (read by the scan below and by the backward).  Thread
//            (c = i % Dp, g = i / Dp) slides the 4-tap window along tokens [g nseg, (g + 1) nseg), each
//            gathered input loaded once; dirconv_fwd_run's fma order, so U is bit-identical to it.
//   phase 2  xdbl[t, j] = sum_c u[t, c] W_x[j, c] on v_mfma_f32_16x16x4_f32: 16 x 16 (token, j) tiles,
//            A = UD rows, B = W_x rows (a wave's W_x fragments for every k chunk loaded at once and kept
//            while its tiles share the column tile); step s of lane group g pairs channel 16 kc + 4 g + s
//            on both operands -> the dt-rank / B / C columns of the LDS image and XD in HBM.
//   phase 3  dt = softplus(W_dt xr + b) over UD (stage_dt).
// Replaces the dirconv_fwd launch, the x_proj GEMM launch and the scan's staging of xdbl from HBM.
constexpr int FMAX_KC = 8;   // Dp / 16 <= 8 (D <= 128)
struct FusedFwd {
  const float* xz;       // [B*L, 2D] in_proj output (token order)
  const float* conv_w;   // [D, 4]
  const float* conv_b;   // [D]
  const float* wx;       // [R+2N, D] x_proj weight
  float* u;              // [nseq*L, D] out
  float* xdbl;           // [nseq*L, R+2N] out
};

__device__ __forceinline__ float cf_ld(const float* p, int i, bool ok) { return ok ? p[i] : 0.f; }

// phase 1: order table in `ord` (LDS, L ints) already staged; barrier after
__device__ __forceinline__ void fused_conv_seq(const ScanArgs& a, const FusedFwd& f, int s, const int* ord,
                                               float* UD, int nseg, int Dp) {
  const int L = a.L, D = a.D;
  const int b = s % a.B;
  const int c = threadIdx.x % Dp, g = threadIdx.x / Dp;
  const bool cv = c < D;
  const int cc = cv ? c : 0;
  const float w0 = cf_ld(f.conv_w, cc * 4, cv), w1 = cf_ld(f.conv_w, cc * 4 + 1, cv),
              w2 = cf_ld(f.conv_w, cc * 4 + 2, cv), w3 = cf_ld(f.conv_w, cc * 4 + 3, cv),
              bias = cf_ld(f.conv_b, cc, cv);
  const float* xb = f.xz + (long)b * L * (2 * D) + cc;
  float* ub = f.u + (long)s * L * D + cc;
  const int t0 = g * nseg;
  float x0, x1, x2;
  {
    float xv[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int tau = t0 - 3 + i;
      xv[i] = (cv && tau >= 0 && tau < L) ? xb[ord[tau] * (2 * D)] : 0.f;
    }
    x0 = xv[0], x1 = xv[1], x2 = xv[2];
  }
  constexpr int CH = 12;   // gathered inputs loaded together (a 21-token run: two rounds)
  for (int i0 = 0; i0 < nseg; i0 += CH) {
    float xv[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int t = t0 + i0 + i;
      xv[i] = (cv && i0 + i < nseg && t < L) ? xb[ord[t] * (2 * D)] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int t = t0 + i0 + i;
      if (i0 + i < nseg) {
        float pre = fmaf(w0, x0, bias);
        pre = fmaf(w1, x1, pre);
        pre = fmaf(w2, x2, pre);
        pre = fmaf(w3, xv[i], pre);
        const bool ok = cv && t < L;
        const float uu = ok ? silu_f(pre) : 0.f;
        UD[t * Dp + c] = uu;
        if (ok) ub[(long)t * D] = uu;
        x0 = x1;
        x1 = x2;
        x2 = xv[i];
      }
    }
  }
}

// phase 2 (after a barrier behind phase 1): xdbl = u W_x^T into the LDS columns and XD in HBM.  Needs D % 4 == 0.
__device__ __forceinline__ void fused_xproj_seq(const ScanArgs& a, const FusedFwd& f, int s, const SeqLds& m,
                                                const float* UD, int Lp, int Dp) {
  const int R = a.R, XW = R + 2 * NST, D = a.D, L = a.L;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int ntm = (Lp + 15) / 16, ntj = (XW + 15) / 16, nkc = Dp / 16;
  float* xd = f.xdbl + (long)s * L * XW;
  f32x4 bw[FMAX_KC];
  int cur_tj = -1;
  // column-tile-major tile order: a wave's consecutive tiles mostly share tj (its W_x fragments)
  for (int tile = wave; tile < ntm * ntj; tile += nw) {
    const int tj = tile / ntm, tm = tile - tj * ntm;
    if (tj != cur_tj) {
      cur_tj = tj;
      const int bj = min(16 * tj + r, XW - 1);   // B column = x_proj output j (clamped, discarded)
#pragma unroll
      for (int kc = 0; kc < FMAX_KC; ++kc) {
        const int k0 = 16 * kc + 4 * g;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        bw[kc] = (kc < nkc && k0 < D) ? *reinterpret_cast<const f32x4*>(f.wx + (long)bj * D + k0) : z;
      }
    }
    const int ar = min(16 * tm + r, Lp - 1);   // A row = token (rows past Lp: clamped, discarded)
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < FMAX_KC; ++kc)
      if (kc < nkc) {
        const f32x4 av = *reinterpret_cast<const f32x4*>(UD + ar * Dp + 16 * kc + 4 * g);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.x, bw[kc].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.y, bw[kc].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.z, bw[kc].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av.w, bw[kc].w, acc, 0, 0, 0);
      }
    // C[t = 16 tm + 4 g + i][j = 16 tj + r]
    const int j = 16 * tj + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 16 * tm + 4 * g + i;
      if (t < Lp && j < XW) {
        float* dst = j < R ? m.xr + t * R + j : (j < R + NST ? m.Bs + t * NST + (j - R) : m.Cs + t * NST + (j - R - NST));
        *dst = acc[i];
        if (t < L) xd[(long)t * XW + j] = acc[i];
      }
    }
  }
}

template <int RT, bool FUSED>
__global__ __launch_bounds__(512) void scan_fwd(ScanArgs a, float* __restrict__ y, float* __restrict__ ckpt,
                                                FusedFwd f) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int R = RT ? RT : a.R;
  const int nseg = seg_count(a.L), Lp = nseg * SCK;
  const int Dp = (blockDim.x >> 6) * 16;
  const SeqLds m(smem, Lp, R, Dp);
  const int s = blockIdx.x, lane = threadIdx.x & 63, q = lane >> 4;
  const int d = (threadIdx.x >> 6) * 16 + (lane & 15);
  const bool valid = d < a.D;
  const int dc = valid ? d : 0;
  float A2[NQ];
#pragma unroll
  for (int j = 0; j < NQ; ++j) A2[j] = valid ? -__expf(a.alog[dc * NST + NQ * q + j]) * LOG2E : 0.f;
  const float Dd = valid ? a.dskip[dc] : 0.f;
  // buffer resources over this sequence's rows (as in scan_bwd): padding tokens / channels and null
  // outputs (a zero-sized resource) fall out of range -- loads give 0, stores are dropped
  const unsigned seq_bytes = (unsigned)(a.L * a.D * 4);
  const unsigned lane_b = valid ? (unsigned)d * 4u : 0x80000000u;
  const auto r_u = buf_rsrc(a.u + (long)s * a.L * a.D, seq_bytes);
  const auto r_y = buf_rsrc(y ? y + (long)s * a.L * a.D : nullptr, y ? seq_bytes : 0u);
  const auto r_ck = buf_rsrc(ckpt ? ckpt + (long)s * nseg * NST * a.D : nullptr,
                             ckpt ? (unsigned)(nseg * NST * a.D * 4) : 0u);
  float h[NQ] = {0.f, 0.f, 0.f, 0.f};
  float un[SCK];
  if (FUSED) {
    int* ord = reinterpret_cast<int*>(m.xr + Lp * R);   // [L] this direction's token order
    const int k = s / a.B;
    for (int t = threadIdx.x; t < a.L; t += blockDim.x) ord[t] = a.order[k * a.L + t];
    __syncthreads();
    fused_conv_seq(a, f, s, ord, m.dts, nseg, Dp);
    __syncthreads();   // UD complete; U in HBM visible to the block
#pragma unroll
    for (int i = 0; i < SCK; ++i) un[i] = buf_ld(r_u, (unsigned)(i * a.D * 4) + lane_b);
    fused_xproj_seq(a, f, s, m, m.dts, Lp, Dp);
    stage_dt<RT>(a, m, Lp, Dp);   // its leading barrier orders phase 2's UD reads before the dt writes
  } else {
#pragma unroll
    for (int i = 0; i < SCK; ++i) un[i] = buf_ld(r_u, (unsigned)(i * a.D * 4) + lane_b);
    stage_seq<RT>(a, s, m, Lp, Dp);   // the first segment's u loads are in flight meanwhile
  }
  for (int c = 0; c < nseg; ++c) {
    const int t0 = c * SCK;
#pragma unroll
    for (int j = 0; j < NQ; ++j) buf_st(r_ck, (unsigned)((c * NST + NQ * q + j) * a.D * 4) + lane_b, h[j]);
    float uc[SCK];
#pragma unroll
    for (int i = 0; i < SCK; ++i) {
      uc[i] = un[i];
      un[i] = buf_ld(r_u, (unsigned)((t0 + SCK + i) * a.D * 4) + lane_b);   // prefetch the next segment
    }
    float yv[SCK];   // this lane's 4-state partial of C_t . h_t per token
#pragma unroll
    for (int i = 0; i < SCK; ++i) {
      const int t = t0 + i;
      const float4 bv = *reinterpret_cast<const float4*>(m.Bs + t * NST + NQ * q);
      const float4 cv = *reinterpret_cast<const float4*>(m.Cs + t * NST + NQ * q);
      const float dt = m.dts[t * Dp + d];
      const float dtu = dt * uc[i];
      // h = dtu * B + exp(dt A) h (the product exp(dt A) h rounded first: the backward's recompute
      // reuses it and so reproduces these states exactly)
      h[0] = fmaf(dtu, bv.x, __builtin_amdgcn_exp2f(dt * A2[0]) * h[0]);
      h[1] = fmaf(dtu, bv.y, __builtin_amdgcn_exp2f(dt * A2[1]) * h[1]);
      h[2] = fmaf(dtu, bv.z, __builtin_amdgcn_exp2f(dt * A2[2]) * h[2]);
      h[3] = fmaf(dtu, bv.w, __builtin_amdgcn_exp2f(dt * A2[3]) * h[3]);
      yv[i] = fmaf(h[3], cv.w, fmaf(h[2], cv.z, fmaf(h[1], cv.y, h[0] * cv.x)));
    }
    // the segment's 4 cross-row sums as one reduce-scatter: row q finishes token t0 + q and stores
    // it (one store per segment; padding tokens fall out of range)
    const float yt = row_scatter4(yv[0], yv[1], yv[2], yv[3]) + Dd * row_select4(uc, q);
    buf_st(r_y, (unsigned)((t0 + q) * a.D * 4) + lane_b, yt);
  }
}

// Sum of 8 per-lane values over the 16 lanes of each row, scattered: lane l of the row returns the
// total of value (l & 15) >> 1.  Partners: row_mirror (15 - l), row_half_mirror (7 - l within 8),
// quad_perm xor 2, xor 1 — each stage pairs lanes that hold the same value set, so the contributor
// sets stay disjoint; fixed order, deterministic.
__device__ __forceinline__ float reduce_scatter8_row(const float (&v)[8]) {
  const int l = threadIdx.x & 15;
  const bool b3 = l & 8, b2 = l & 4, b1 = l & 2;
  float y4[4], z[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float keep = b3 ? v[j + 4] : v[j], send = b3 ? v[j] : v[j + 4];
    y4[j] = keep + dpp_mov<0x140>(send);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float keep = b2 ? y4[j + 2] : y4[j], send = b2 ? y4[j] : y4[j + 2];
    z[j] = keep + dpp_mov<0x141>(send);
  }
  const float keep = b1 ? z[1] : z[0], send = b1 ? z[0] : z[1];
  const float w = keep + dpp_mov<0x4E>(send);
  return w + dpp_mov<0xB1>(w);
}

// The first two stages of reduce_scatter8_row without the selects: the lanes that keep value a and
// the lanes that keep value b sit in different 4-lane banks (bit 3: banks 0,1 vs 2,3; bit 2: banks
// 0,2 vs 1,3), so each output is two bank-masked DPP adds (own + partner's same value), each lane
// written by exactly one of them.  Same partners and operand order as reduce_scatter8_row, so the
// result is bit-identical.  s_nop 1: the DPP operands may have been written by the two preceding VALU
// instructions.
#ifndef VC_DPP_PAIRWISE
#define VC_DPP_PAIRWISE 0   // 1: the per-pair blocks below (one s_nop each) instead of dpp_stage12
#endif
template <int CTRL_ASM>
__device__ __forceinline__ float dpp_pair_add(float a, float b);
template <>
__device__ __forceinline__ float dpp_pair_add<0>(float a, float b) {   // row_mirror, bit 3
  float r;
  asm volatile(
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %1, %1 row_mirror row_mask:0xf bank_mask:0x3 bound_ctrl:1\n\t"
      "v_add_f32_dpp %0, %2, %2 row_mirror row_mask:0xf bank_mask:0xc bound_ctrl:1"
      : "=&v"(r) : "v"(a), "v"(b));
  return r;
}
template <>
__device__ __forceinline__ float dpp_pair_add<1>(float a, float b) {   // row_half_mirror, bit 2
  float r;
  asm volatile(
      "s_nop 1\n\t"
      "v_add_f32_dpp %0, %1, %1 row_half_mirror row_mask:0xf bank_mask:0x5 bound_ctrl:1\n\t"
      "v_add_f32_dpp %0, %2, %2 row_half_mirror row_mask:0xf bank_mask:0xa bound_ctrl:1"
      : "=&v"(r) : "v"(a), "v"(b));
  return r;
}
// Both bank-masked stages in one block: 12 DPP adds behind ONE s_nop.  Every stage-2 operand was
// written at least two instructions earlier (y0 at 1, y2 at 5 -> read at 9; y1 at 3, y3 at 7 -> read
// at 11), so only the block's entry needs the wait states; the per-pair form paid 6 s_nop per token.
__device__ __forceinline__ void dpp_stage12(const float (&v)[8], float& z0, float& z1) {
  float y0, y1, y2, y3;
  asm volatile(
      "s_nop 1\n\t"
      "v_add_f32_dpp %2, %6, %6 row_mirror row_mask:0xf bank_mask:0x3 bound_ctrl:1\n\t"
      "v_add_f32_dpp %2, %10, %10 row_mirror row_mask:0xf bank_mask:0xc bound_ctrl:1\n\t"
      "v_add_f32_dpp %3, %7, %7 row_mirror row_mask:0xf bank_mask:0x3 bound_ctrl:1\n\t"
      "v_add_f32_dpp %3, %11, %11 row_mirror row_mask:0xf bank_mask:0xc bound_ctrl:1\n\t"
      "v_add_f32_dpp %4, %8, %8 row_mirror row_mask:0xf bank_mask:0x3 bound_ctrl:1\n\t"
      "v_add_f32_dpp %4, %12, %12 row_mirror row_mask:0xf bank_mask:0xc bound_ctrl:1\n\t"
      "v_add_f32_dpp %5, %9, %9 row_mirror row_mask:0xf bank_mask:0x3 bound_ctrl:1\n\t"
      "v_add_f32_dpp %5, %13, %13 row_mirror row_mask:0xf bank_mask:0xc bound_ctrl:1\n\t"
      "v_add_f32_dpp %0, %2, %2 row_half_mirror row_mask:0xf bank_mask:0x5 bound_ctrl:1\n\t"
      "v_add_f32_dpp %0, %4, %4 row_half_mirror row_mask:0xf bank_mask:0xa bound_ctrl:1\n\t"
      "v_add_f32_dpp %1, %3, %3 row_half_mirror row_mask:0xf bank_mask:0x5 bound_ctrl:1\n\t"
      "v_add_f32_dpp %1, %5, %5 row_half_mirror row_mask:0xf bank_mask:0xa bound_ctrl:1"
      : "=&v"(z0), "=&v"(z1), "=&v"(y0), "=&v"(y1), "=&v"(y2), "=&v"(y3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]));
}
__device__ __forceinline__ float reduce_scatter8_row_bm(const float (&v)[8]) {
  const int l = threadIdx.x & 15;
  const bool b1 = l & 2;
  float z[2];
#if VC_DPP_PAIRWISE
  float y4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) y4[j] = dpp_pair_add<0>(v[j], v[j + 4]);
#pragma unroll
  for (int j = 0; j < 2; ++j) z[j] = dpp_pair_add<1>(y4[j], y4[j + 2]);
#else
  dpp_stage12(v, z[0], z[1]);
#endif
  const float keep = b1 ? z[1] : z[0], send = b1 ? z[0] : z[1];
  const float w = keep + dpp_mov<0x4E>(send);
  return w + dpp_mov<0xB1>(w);
}

// ---------------------------------------------------------------- fused tail (scan_bwd<RT, BM, true>)
// After the reverse sweep the block holds its sequence's du (the scan's part, over the dts region) and
// dB / dC (over Bs / Cs) in LDS, and d(dt_lin) in HBM.  The tail finishes the sequence's backward
// through dt_proj, x_proj and the direction conv, replacing three launches (the dt_proj and x_proj
// data-gradient GEMMs and dirconv_bwd_wgrad) and du's HBM round trip:
//   (a) dxr[t, j] = sum_c ddtl[t, c] W_dt[c, j]            (v_mfma_f32_16x16x4_f32, k = channel; A from
//                                                            HBM, W_dt staged over the dead dB / dC
//                                                            partial buffers) -> a [Lp][16] LDS image
//   (b) du[t, c] += sum_j dxdbl[t, j] W_x[j, c]            (MFMA, k = j in three 16-wide chunks: the
//                                                            dxr image | dB (Bs) | dC (Cs))
//   (c) dpre = du SiLU'(pre), pre recomputed from the 4 gathered taps (dirconv_fwd_run's fma order; xz is
//       L2-resident), written to HBM; the sequence's conv weight / bias partials [nseq][5D]
//       (c*4 + j | 4D + c), summed over its tokens in a fixed order.
// Global operands are issued ahead of their MFMAs (W_x fragments once per wave, the gathered taps for
// two token tiles at a time).  In (b) / (c) wave w owns channels 16 w .. 16 w + 15, so a channel's conv
// partials never leave its wave.  Needs R <= 16.
struct FusedBwd {
  const float* xz;       // [B*L, 2D]
  const float* conv_w;   // [D, 4]
  const float* conv_b;   // [D]
  const float* wx;       // [R+2N, D]
  float* conv_part;      // [nseq][5D] out
  int tail;              // 7 (all); measurement masks (VITCNN_SCAN_TAIL, results incomplete): bit 0 the
                         // tail at all, bit 1 phase (a), bit 2 phases (b) + (c)
};

struct ScanBwdOut {
  float* du;        // [nseq*L, D]
  float* ddtl;      // [nseq*L, D]  grad of W_dt dtr + b_dt (pre-softplus)
  float* dxdbl;     // [nseq*L, XW] B / C columns written
  float* da_part;   // [nseq][D*N]
  float* dd_part;   // [nseq][D]
  float* dg_part;   // [nseq]
};

template <int RT>
__device__ __forceinline__ void fused_bwd_tail(const ScanArgs& a, const FusedBwd& fb, const ScanBwdOut& o, int s,
                                               int b, const SeqLds& m, const int* ord, float* red, int Lp,
                                               int Dp) {
  const int R = RT ? RT : a.R, XW = R + 2 * NST, D = a.D, L = a.L;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int ntm = (Lp + 15) / 16, nkc = Dp / 16;
  const long base = (long)s * L;
  float* DX16 = red;                 // [Lp][16] dxr, columns R..15 zero
  float* wdt_lds = red + Lp * 16;    // [D][R]
  {   // W_dt: all of a thread's loads issued before its stores (one latency, not one per trip)
    constexpr int WS = 8;   // D R <= 128 x 16 over >= 256 threads
    float wv[WS];
#pragma unroll
    for (int j = 0; j < WS; ++j) {
      const int i = threadIdx.x + j * blockDim.x;
      wv[j] = i < D * R ? a.wdt[i] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < WS; ++j) {
      const int i = threadIdx.x + j * blockDim.x;
      if (i < D * R) wdt_lds[i] = wv[j];
    }
  }
  __syncthreads();
  // (a) A = ddtl rows from HBM (this block's sweep wrote them), B[k = c][col = j] = W_dt[c, j] (LDS);
  // a wave's (at most two, ntm <= 2 nw) token tiles' A rows loaded at once
  f32x4 avs[2][FMAX_KC];
  const int nu = (fb.tail & 2) ? 2 : 0;   // measurement mask (see FusedBwd::tail)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int ta = 16 * (wave + u * nw) + r;
    const bool tok = ta < L;
    const float* arow = o.ddtl + (base + (tok ? ta : 0)) * D;
#pragma unroll
    for (int kc = 0; kc < FMAX_KC; ++kc) {
      const int k0 = 16 * kc + 4 * g;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      avs[u][kc] = (kc < nkc && tok && k0 < D) ? *reinterpret_cast<const f32x4*>(arow + k0) : z;
    }
  }
#pragma unroll
  for (int u = 0; u < nu; ++u) {
    const int tm = wave + u * nw;
    if (tm >= ntm) break;
    const f32x4* av = avs[u];   // (tiles past 2 nw: none for the fused shapes, host check)
    const bool jok = r < R;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < FMAX_KC; ++kc)
      if (kc < nkc) {
        const int k0 = 16 * kc + 4 * g;
        float bv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[e] = (jok && k0 + e < D) ? wdt_lds[(k0 + e) * R + r] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc].x, bv[0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc].y, bv[1], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc].z, bv[2], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kc].w, bv[3], acc, 0, 0, 0);
      }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int t = 16 * tm + 4 * g + i;
      if (t < Lp) {
        DX16[t * 16 + r] = jok ? acc[i] : 0.f;
        if (jok && t < L) o.dxdbl[(base + t) * XW + r] = acc[i];
      }
    }
  }
  // the wave's W_x fragments for (b): B[k = j][col = dl], chunk 0 = dt-rank rows, 1 = B rows, 2 = C rows
  // (in flight across the barrier)
  const int dl = 16 * wave + r;
  const bool dok = dl < D;
  const int dcl = dok ? dl : 0;
  f32x4 bw[3];
#pragma unroll
  for (int kc = 0; kc < 3; ++kc)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int jj = 4 * g + e;
      const int j = kc == 0 ? jj : R + 16 * (kc - 1) + jj;
      bw[kc][e] = (dok && (kc > 0 || jj < R)) ? fb.wx[(long)j * D + dcl] : 0.f;
    }
  __syncthreads();
  // (b) + (c)
  const unsigned lb = dok ? (unsigned)dl * 4u : 0x80000000u;   // padding channels: stores dropped
  const auto r_dp = buf_rsrc(o.du + base * D, (unsigned)(L * D * 4));
  const float w0 = cf_ld(fb.conv_w, dcl * 4, dok), w1 = cf_ld(fb.conv_w, dcl * 4 + 1, dok),
              w2 = cf_ld(fb.conv_w, dcl * 4 + 2, dok), w3 = cf_ld(fb.conv_w, dcl * 4 + 3, dok),
              bias = cf_ld(fb.conv_b, dcl, dok);
  const float* xb = fb.xz + (long)b * L * (2 * D) + dcl;
  float cacc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  constexpr int TG = 3;   // token tiles whose gathered taps are issued together (more spills the 128-VGPR budget)
  const int ntm_c = (fb.tail & 4) ? ntm : 0;   // measurement mask
  for (int tm0 = 0; tm0 < ntm_c; tm0 += TG) {
    float xv[TG][7];   // taps tq - 3 .. tq + 3 of this lane's tokens tq .. tq + 3
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      const int tq = 16 * (tm0 + u) + 4 * g;
#pragma unroll
      for (int e = 0; e < 7; ++e) {
        const int tau = tq - 3 + e;
        xv[u][e] = (dok && tau >= 0 && tau < L) ? xb[ord[tau] * (2 * D)] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < TG; ++u) {
      const int tm = tm0 + u;
      if (tm >= ntm) break;
      const int ar = min(16 * tm + r, Lp - 1);
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(DX16 + ar * 16 + 4 * g);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(m.Bs + ar * NST + 4 * g);
      const f32x4 a2 = *reinterpret_cast<const f32x4*>(m.Cs + ar * NST + 4 * g);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, bw[0].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, bw[0].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, bw[0].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, bw[0].w, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, bw[1].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, bw[1].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, bw[1].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, bw[1].w, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a2.x, bw[2].x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a2.y, bw[2].y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a2.z, bw[2].z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a2.w, bw[2].w, acc, 0, 0, 0);
      // C[t = 16 tm + 4 g + i][dl]
      const int tq = 16 * tm + 4 * g;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (tq + i < L) {
          float pre = fmaf(w0, xv[u][i], bias);
          pre = fmaf(w1, xv[u][i + 1], pre);
          pre = fmaf(w2, xv[u][i + 2], pre);
          pre = fmaf(w3, xv[u][i + 3], pre);
          const float sg = sigmoid_f(pre);
          const float du = m.dts[(tq + i) * Dp + dl] + acc[i];
          const float gd = dok ? du * sg * (1.f + pre * (1.f - sg)) : 0.f;
          buf_st(r_dp, (unsigned)((tq + i) * D * 4) + lb, gd);
          cacc[4] += gd;
          cacc[0] += gd * xv[u][i];
          cacc[1] += gd * xv[u][i + 1];
          cacc[2] += gd * xv[u][i + 2];
          cacc[3] += gd * xv[u][i + 3];
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 5; ++e) cacc[e] = cross_row_sum(cacc[e]);
  if (g == 0 && dok) {
    float* cp = fb.conv_part + (long)s * 5 * D;
#pragma unroll
    for (int e = 0; e < 4; ++e) cp[dl * 4 + e] = cacc[e];
    cp[4 * D + dl] = cacc[4];
  }
}

template <int RT, bool BM, bool FUSE>
__global__ __launch_bounds__(512, 4) void scan_bwd(ScanArgs a, int ndir, const float* __restrict__ gate_logits,
                                                const float* __restrict__ yp, const float* __restrict__ dyp,
                                                const float* __restrict__ ckpt, ScanBwdOut o, int rbs,
                                                FusedBwd fb) {
  extern __shared__ __attribute__((aligned(16))) float smem[];  // SeqLds, red [2 rbs][nw][SCK][32], [nw], ord
  const int R = RT ? RT : a.R;
  const int XW = R + 2 * NST;
  const int nseg = seg_count(a.L), Lp = nseg * SCK;
  const int nw = blockDim.x >> 6, Dp = nw * 16;
  const SeqLds m(smem, Lp, R, Dp);
  float* red = m.xr + Lp * R;
  const int nbuf = 2 * rbs;   // partial buffers: a combine every rbs segments, double-buffered
  // partial buffers; the fused tail reuses them for its dxr image and W_dt ([Lp][16] + [D][R])
  const int red_n = FUSE ? max(nbuf * nw * SCK * 32, Lp * 16 + a.D * R) : nbuf * nw * SCK * 32;
  int* ord = reinterpret_cast<int*>(red + red_n + nw);   // [L] this direction's order
  const int s = blockIdx.x, k = s / a.B, b = s - k * a.B;
  for (int t = threadIdx.x; t < a.L; t += blockDim.x) ord[t] = a.order[k * a.L + t];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, q = lane >> 4, cl = lane & 15;
  const int d = wave * 16 + cl;
  const bool valid = d < a.D;
  const int dc = valid ? d : 0;
  const float g = gate_softmax(gate_logits, ndir, k);
  float A2[NQ];
#pragma unroll
  for (int j = 0; j < NQ; ++j) A2[j] = valid ? -__expf(a.alog[dc * NST + NQ * q + j]) * LOG2E : 0.f;
  const float Dd = valid ? a.dskip[dc] : 0.f;
  const long base = (long)s * a.L;
  // the dB/dC column this lane's reduce-scatter total belongs to
  const int vi = cl >> 1;
  const int col = vi < 4 ? NQ * q + vi : NST + NQ * q + vi - 4;
  // the lane's 4 states as two packed pairs (v_pk_fma_f32 / v_pk_mul_f32: two states per instruction)
  const f2 A2v[2] = {f2{A2[0], A2[1]}, f2{A2[2], A2[3]}};
  f2 dh[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}}, dAacc[2] = {f2{0.f, 0.f}, f2{0.f, 0.f}};
  float dD_acc = 0.f, dg_acc = 0.f;
  // global operands of a segment: the entering state, u, the gathered d(yp) and yp (for the gate
  // gradient); the next segment's are loaded while this one is computed
  float hn[NQ], un[SCK], dn[SCK], yn[SCK];
  // The segment operands and the du / d(dt_lin) outputs go through buffer resources over this
  // sequence's rows: 32-bit offsets (no 64-bit address arithmetic per access), and the hardware range
  // check returns 0 for out-of-range loads / drops out-of-range stores, which takes the place of the
  // padding-token (t >= L) and padding-channel (d >= D) guards: such lanes get an offset past the end.
  const unsigned seq_bytes = (unsigned)(a.L * a.D * 4);
  const auto r_u = buf_rsrc(a.u + base * a.D, seq_bytes);
  const auto r_yp = buf_rsrc(yp + base * a.D, seq_bytes);
  const auto r_dyp = buf_rsrc(dyp + (long)b * a.L * a.D, seq_bytes);
  const auto r_du = buf_rsrc(o.du + base * a.D, seq_bytes);
  const auto r_ddtl = buf_rsrc(o.ddtl + base * a.D, seq_bytes);
  const auto r_ck = buf_rsrc(ckpt + (long)s * nseg * NST * a.D, (unsigned)(nseg * NST * a.D * 4));
  const auto r_dx = buf_rsrc(o.dxdbl + base * XW, (unsigned)(a.L * XW * 4));
  const unsigned lane_b = valid ? (unsigned)d * 4u : 0x80000000u;   // invalid lanes: out of range
  auto load_seg = [&](int c) {
    const int t0 = c * SCK;
#pragma unroll
    for (int j = 0; j < NQ; ++j) hn[j] = buf_ld(r_ck, (unsigned)((c * NST + NQ * q + j) * a.D * 4) + lane_b);
#pragma unroll
    for (int i = 0; i < SCK; ++i) {
      const int t = t0 + i;
      const unsigned row = (unsigned)(t * a.D * 4) + lane_b;   // t >= L: past the end
      un[i] = buf_ld(r_u, row);
      dn[i] = buf_ld(r_dyp, (unsigned)((t < a.L ? ord[t] : a.L) * a.D * 4) + lane_b);
      yn[i] = buf_ld(r_yp, row);
    }
  };
  __syncthreads();   // ord
  load_seg(nseg - 1);   // the last segment's operands are in flight while the sequence is staged
  stage_seq<RT>(a, s, m, Lp, Dp);
  for (int c = nseg - 1; c >= 0; --c) {
    const int t0 = c * SCK;
    f2 hs[SCK + 1][2];   // hs[i] = state entering token t0 + i
    float uc[SCK], dyr[SCK];
    hs[0][0] = f2{hn[0], hn[1]};
    hs[0][1] = f2{hn[2], hn[3]};
#pragma unroll
    for (int i = 0; i < SCK; ++i) {
      uc[i] = un[i];
      dyr[i] = dn[i];
      dg_acc += dyr[i] * yn[i];
    }
    if (c > 0) load_seg(c - 1);
    // recompute the segment's states as the forward did, element for element (keep exp(dt A) for the
    // reverse sweep)
    f2 dAs[SCK][2];
#pragma unroll
    for (int i = 0; i < SCK; ++i) {
      const int t = t0 + i;
      const float4 bv = *reinterpret_cast<const float4*>(m.Bs + t * NST + NQ * q);
      const float dt = m.dts[t * Dp + d];
      const float dtu = dt * uc[i];
      const f2 bb[2] = {f2{bv.x, bv.y}, f2{bv.z, bv.w}};
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const f2 e = f2{dt, dt} * A2v[p];
        dAs[i][p] = f2{__builtin_amdgcn_exp2f(e.x), __builtin_amdgcn_exp2f(e.y)};
        hs[i + 1][p] = fma2(f2{dtu, dtu}, bb[p], dAs[i][p] * hs[i][p]);
      }
    }
    // reverse sweep
    float* rb = red + (c % nbuf) * nw * SCK * 32;
    float Sv[SCK], Qv[SCK];   // this lane's 4-state partials of S and qa per token
#pragma unroll
    for (int i = SCK - 1; i >= 0; --i) {
      const int t = t0 + i;
      const float4 b4 = *reinterpret_cast<const float4*>(m.Bs + t * NST + NQ * q);
      const float4 c4 = *reinterpret_cast<const float4*>(m.Cs + t * NST + NQ * q);
      const f2 bv[2] = {f2{b4.x, b4.y}, f2{b4.z, b4.w}}, cv[2] = {f2{c4.x, c4.y}, f2{c4.z, c4.w}};
      const float dt = m.dts[t * Dp + d], ut = uc[i], dy = g * dyr[i];
      const float dtu = dt * ut;
      const f2 dy2 = f2{dy, dy}, dt2 = f2{dt, dt}, dtu2 = f2{dtu, dtu};
      f2 Sp, Qp, vB[2], vC[2];   // this lane's terms of sum_n dhn B and sum_n (dL/d(dA) dA) A, pairwise
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const f2 dhn = fma2(cv[p], dy2, dh[p]);                // dL/dh_t
        const f2 qq = dhn * (dAs[i][p] * hs[i][p]);            // dL/d(dA_t) * dA_t
        dAacc[p] = fma2(qq, dt2, dAacc[p]);
        Qp = p ? fma2(qq, A2v[p], Qp) : qq * A2v[p];
        Sp = p ? fma2(dhn, bv[p], Sp) : dhn * bv[p];
        vB[p] = dhn * dtu2;                                    // dL/dB_t[n], this channel
        vC[p] = dy2 * hs[i + 1][p];                            // dL/dC_t[n], this channel
        dh[p] = dhn * dAs[i][p];                               // carried to t - 1
      }
      const float S = Sp.x + Sp.y, qa = Qp.x + Qp.y;
      const float v[8] = {vB[0].x, vB[0].y, vB[1].x, vB[1].y, vC[0].x, vC[0].y, vC[1].x, vC[1].y};
      Sv[i] = S;
      Qv[i] = qa;
      rb[(wave * SCK + i) * 32 + col] = BM ? reduce_scatter8_row_bm(v) : reduce_scatter8_row(v);   // lanes 2j, 2j+1 store the same
    }
    {   // the sums over the 16 states (the wave's 4 rows) of the segment's 4 tokens as one
        // reduce-scatter: row q finishes token t0 + q (padding tokens / channels fall out of range;
        // their u and d(yp) loaded as 0)
      const float S = row_scatter4(Sv[0], Sv[1], Sv[2], Sv[3]);
      const float qa = row_scatter4(Qv[0], Qv[1], Qv[2], Qv[3]);
      const float dt = m.dts[(t0 + q) * Dp + d], ut = row_select4(uc, q), dy = g * row_select4(dyr, q);
      const unsigned row = (unsigned)((t0 + q) * a.D * 4) + lane_b;
      const float duv = dt * S + Dd * dy;
      // fused tail: du stays in LDS, over this token's dt (read for the last time above, by this wave
      // only: its channels); the tail adds x_proj's part and writes dpre
      if (FUSE) m.dts[(t0 + q) * Dp + d] = duv;
      else buf_st(r_du, row, duv);
      // softplus'(dt_lin) = sigmoid(dt_lin) = 1 - exp(-softplus(dt_lin))
      buf_st(r_ddtl, row, (qa * LN2 + ut * S) * -expm1_c(-dt));
      dD_acc += dy * ut;   // row q's tokens; the rows are summed at the end
    }
    // one barrier per rbs segments: segment c's partials go to buffer c % (2 rbs), so the next rbs
    // segments' stores (the other half of the buffers) need no barrier behind this combine; the
    // combine after them orders the reuse of these buffers
    if (c % rbs == 0) {
      __syncthreads();
      for (int j = threadIdx.x; j < rbs * SCK * 32; j += blockDim.x) {
        const int cs = c + j / (SCK * 32), jj = j % (SCK * 32);
        const int i = jj >> 5, cc = jj & 31, t = cs * SCK + i;
        const float* rbc = red + (cs % nbuf) * nw * SCK * 32;
        // the nw (<= 8) partials read together, then summed in wave order; tokens t >= L (and
        // segments past the last) fall out of the output resource's range
        float pv[8];
#pragma unroll
        for (int ww = 0; ww < 8; ++ww) pv[ww] = ww < nw ? rbc[(ww * SCK + i) * 32 + cc] : 0.f;
        float sum = pv[0];
#pragma unroll
        for (int ww = 1; ww < 8; ++ww)
          if (ww < nw) sum += pv[ww];
        buf_st(r_dx, (unsigned)(t * XW + R + cc) * 4u, sum);
        // fused tail: dB / dC kept in LDS over the token's B / C rows (swept by every wave before the
        // barrier above; later segments read only their own rows)
        if (FUSE && t < Lp) (cc < NST ? m.Bs + t * NST + cc : m.Cs + t * NST + (cc - NST))[0] = sum;
      }
    }
  }
  dD_acc = cross_row_sum(dD_acc);
  if (valid) {
    float* dap = o.da_part + ((long)s * a.D + d) * NST + NQ * q;
#pragma unroll
    for (int j = 0; j < NQ; ++j) dap[j] = dAacc[j >> 1][j & 1] * A2[j] * LN2;   // dL/dA_log = dL/dA * A
    if (q == 0) o.dd_part[(long)s * a.D + d] = dD_acc;
  }
  const float v = wave_sum(q == 0 ? dg_acc : 0.f);
  float* rg = red + red_n;
  if (lane == 0) rg[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float sum = 0.f;
    for (int ww = 0; ww < nw; ++ww) sum += rg[ww];
    o.dg_part[s] = sum;
  }
  if (FUSE && (fb.tail & 1)) fused_bwd_tail<RT>(a, fb, o, s, b, m, ord, red, Lp, Dp);   // the barrier above: LDS images complete
}

// token-wise SiLU(z) gate of the combined output, backward:
//   dyp = dysum * SiLU(z);   dz = dysum * YP * SiLU'(z)  -> the z half of dxz (ld 2D)
__global__ void gate_bwd(int total, FastDiv fD, const float* __restrict__ xz, const float* __restrict__ ypsum,
                         const float* __restrict__ dysum, float* __restrict__ dyp, float* __restrict__ dxz) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int D = fD.div;
  int d;
  const int r = fdivmod(idx, fD, d);
  const float z = xz[(long)r * 2 * D + D + d];
  const float sg = sigmoid_f(z);
  const float g = dysum[idx];
  dyp[idx] = g * z * sg;
  dxz[(long)r * 2 * D + D + d] = g * ypsum[idx] * sg * (1.f + z * (1.f - sg));
}

// YP[b, l, :] = sum_k softmax(gate)_k y[k, b, inv_k(l), :], ysum = YP * SiLU(z).  The ndir (<= MAXK)
// order-table entries are read first and the gathered rows after them (one round of dependent loads
// instead of ndir), then summed in direction order.
template <int MAXK>
__global__ void combine_fwd(int total, FastDiv fD, FastDiv fL, int B, int ndir, const int* __restrict__ inv,
                            const float* __restrict__ logits, const float* __restrict__ y,
                            const float* __restrict__ xz, float* __restrict__ ypsum, float* __restrict__ out) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int D = fD.div, L = fL.div;
  int d, l;
  const int bl = fdivmod(idx, fD, d);
  const int b = fdivmod(bl, fL, l);
  float mx = logits[0];
  for (int i = 1; i < ndir; ++i) mx = fmaxf(mx, logits[i]);
  float den = 0.f;
  for (int i = 0; i < ndir; ++i) den += __expf(logits[i] - mx);
  const float rden = 1.f / den;
  float acc = 0.f;
  for (int k0 = 0; k0 < ndir; k0 += MAXK) {
    int tk[MAXK];
#pragma unroll
    for (int kk = 0; kk < MAXK; ++kk) tk[kk] = k0 + kk < ndir ? inv[(k0 + kk) * L + l] : 0;
    float yv[MAXK];
#pragma unroll
    for (int kk = 0; kk < MAXK; ++kk)
      yv[kk] = k0 + kk < ndir ? y[((long)((k0 + kk) * B + b) * L + tk[kk]) * D + d] : 0.f;
#pragma unroll
    for (int kk = 0; kk < MAXK; ++kk)
      if (k0 + kk < ndir) {
        const float gk = __expf(logits[k0 + kk] - mx) * rden;
        acc += gk * yv[kk];
      }
  }
  ypsum[idx] = acc;
  out[idx] = acc * silu_f(xz[(long)bl * 2 * D + D + d]);
}

// dlogit_j = g_j (dg_j - sum_k g_k dg_k),  dg_k = sum over the k-th direction's partials (one 256-thread block)
__device__ __forceinline__ void gate_grad_body(int ndir, int per_dir, const float* __restrict__ logits,
                                               const float* __restrict__ part, float* __restrict__ dlogits,
                                               float* dg, float* gg) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int kk = wave; kk < ndir; kk += 4) {
    float s = 0.f;
    for (int i = lane; i < per_dir; i += 64) s += part[(long)kk * per_dir + i];
    s = wave_sum(s);
    if (lane == 0) {
      dg[kk] = s;
      gg[kk] = gate_softmax(logits, ndir, kk);
    }
  }
  __syncthreads();
  if (threadIdx.x < ndir) {
    float dot = 0.f;
    for (int i = 0; i < ndir; ++i) dot += gg[i] * dg[i];
    dlogits[threadIdx.x] = gg[threadIdx.x] * (dg[threadIdx.x] - dot);
  }
}

__global__ __launch_bounds__(256) void gate_grad(int ndir, int per_dir, const float* __restrict__ logits,
                                                 const float* __restrict__ part, float* __restrict__ dlogits) {
  __shared__ float dg[64], gg[64];
  gate_grad_body(ndir, per_dir, logits, part, dlogits, dg, gg);
}

// Every per-sequence partial of a hsiMamba block's scan backward reduced in ONE launch (round 6): column blocks of
// 16 columns x 16 partial lanes over [dA_log 16D | D skip D | conv1d weight 4D | conv1d bias D] (sum_rows_kernel's
// fixed order; the columns of one block may straddle two tensors), and one last block for the gate gradient --
// instead of two two-phase column sums, the gate kernel and the conv row sum (6 launches at the end of the step)
__global__ __launch_bounds__(256) void mamba_params(int nseq, int D, int ndir, int ncb, const float* __restrict__ logits,
                                                    const float* __restrict__ pa, const float* __restrict__ pd,
                                                    const float* __restrict__ pg, const float* __restrict__ cp,
                                                    float* __restrict__ dA, float* __restrict__ dDs,
                                                    float* __restrict__ dgl, float* __restrict__ dcw,
                                                    float* __restrict__ dcb) {
  __shared__ float sh[16][17];
  __shared__ float dg[64], gg[64];
  if ((int)blockIdx.x == ncb) {
    gate_grad_body(ndir, nseq / ndir, logits, pg, dgl, dg, gg);
    return;
  }
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  const float* src = nullptr;
  long stride = 0;
  float* dst = nullptr;
  int cc = 0;
  if (c < NST * D) src = pa, stride = (long)NST * D, dst = dA, cc = c;
  else if (c < (NST + 1) * D) src = pd, stride = D, dst = dDs, cc = c - NST * D;
  else if (c < (NST + 5) * D) src = cp, stride = 5L * D, dst = dcw, cc = c - (NST + 1) * D;
  else if (c < (NST + 6) * D) src = cp + 4L * D, stride = 5L * D, dst = dcb, cc = c - (NST + 5) * D;
  float s = 0.f;
  if (src) {
#pragma unroll 4
    for (int p = pl; p < nseq; p += 16) s += src[(long)p * stride + cc];
  }
  sh[pl][cl] = s;
  __syncthreads();
  if (pl == 0 && src) {
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) v += sh[i][cl];
    dst[cc] = v;
  }
}


// dxz[b,l,d] = sum_k sum_j w[d,j] dpre[k,b,inv_k(l)+3-j,d]   (the x half; gate_bwd writes the z half)
// dxz[b, l, d] = sum_k sum_j w[d, j] dpre[k, b, inv_k(l) + 3 - j, d].  All ndir (<= MAXK) order-table
// entries are read first and the 4 ndir taps issued after them (one round of dependent loads instead
// of ndir); taps past the sequence end read as 0.  Same accumulation order for every ndir.
template <int MAXK>
__global__ void dirconv_bwd_gather(int total, FastDiv fD, FastDiv fL, int B, int ndir, const int* __restrict__ inv,
                                   const float* __restrict__ cw, const float* __restrict__ dpre,
                                   float* __restrict__ dxz) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int D = fD.div, L = fL.div;
  int d, l;
  const int bl = fdivmod(idx, fD, d);
  const int b = fdivmod(bl, fL, l);
  float w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = cw[d * 4 + j];
  float acc = 0.f;
  for (int k0 = 0; k0 < ndir; k0 += MAXK) {
    int tk[MAXK];
#pragma unroll
    for (int kk = 0; kk < MAXK; ++kk) tk[kk] = k0 + kk < ndir ? inv[(k0 + kk) * L + l] : L;
    float v[MAXK][4];
#pragma unroll
    for (int kk = 0; kk < MAXK; ++kk) {
      const float* base = dpre + (long)((k0 + kk) * B + b) * L * D + d;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int t = tk[kk] + 3 - j;
        v[kk][j] = t < L ? base[(long)t * D] : 0.f;
      }
    }
#pragma unroll
    for (int kk = 0; kk < MAXK; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc = fmaf(w[j], v[kk][j], acc);
  }
  dxz[(long)bl * 2 * D + d] = acc;
}

// Fused SiLU backward + conv1d weight/bias partial sums over a chunk of (seq, token-run) items:
//   dpre = du * SiLU'(pre) (pre recomputed from the 4 gathered taps as dirconv_fwd_run does, written in
//   place over du), part[p][d*4 + j] = sum dpre * x_{t-3+j},  part[p][4D + d] = sum dpre
// block = 16 channels x 16 item lanes; an item is DC_T consecutive tokens of one sequence, walked with
// the forward's sliding tap window (each gathered input loaded once).  Fixed order, deterministic.
__global__ __launch_bounds__(256) void dirconv_bwd_wgrad(int D, int L, FastDiv fC, FastDiv fB,
                                                         const int* __restrict__ order, const float* __restrict__ xz,
                                                         const float* __restrict__ cw, const float* __restrict__ cb,
                                                         float* __restrict__ du, int items, int items_per,
                                                         float* __restrict__ part) {
  __shared__ float sh[5][16][17];
  const int dlc = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int d = blockIdx.x * 16 + dlc;
  const int i0 = blockIdx.y * items_per, i1 = min(items, i0 + items_per);
  float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if (d < D) {
    const float w0 = cw[d * 4], w1 = cw[d * 4 + 1], w2 = cw[d * 4 + 2], w3 = cw[d * 4 + 3], bias = cb[d];
    for (int it = i0 + rl; it < i1; it += 16) {
      int c, b;
      const int sq = fdivmod(it, fC, c);
      const int k = fdivmod(sq, fB, b);
      const int* ord = order + k * L;
      const float* xb = xz + (long)b * L * (2 * D) + d;
      const int t0 = c * DC_T;
      float x[DC_T + 3];
#pragma unroll
      for (int i = 0; i < DC_T + 3; ++i) {
        const int tau = t0 - 3 + i;
        x[i] = (tau >= 0 && tau < L) ? xb[ord[tau] * (2 * D)] : 0.f;
      }
      float* gp = du + ((long)sq * L + t0) * D + d;
#pragma unroll
      for (int i = 0; i < DC_T; ++i) {
        if (t0 + i < L) {
          float pre = fmaf(w0, x[i], bias);
          pre = fmaf(w1, x[i + 1], pre);
          pre = fmaf(w2, x[i + 2], pre);
          pre = fmaf(w3, x[i + 3], pre);
          const float sg = sigmoid_f(pre);
          const float g = gp[(long)i * D] * sg * (1.f + pre * (1.f - sg));
          gp[(long)i * D] = g;
          acc[4] += g;
          // taps before the sequence start are 0 (the forward skipped them)
          acc[0] += g * x[i];
          acc[1] += g * x[i + 1];
          acc[2] += g * x[i + 2];
          acc[3] += g * x[i + 3];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 5; ++j) sh[j][rl][dlc] = acc[j];
  __syncthreads();
  if (threadIdx.x < 80) {
    const int j = threadIdx.x >> 4, dd = threadIdx.x & 15, dg = blockIdx.x * 16 + dd;
    if (dg < D) {
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) v += sh[j][i][dd];
      part[(long)blockIdx.y * 5 * D + (j < 4 ? dg * 4 + j : 4 * D + dg)] = v;
    }
  }
}

}  // namespace

VC_API int vc_mamba_dirconv_fwd(int B, int L, int D, int ndir, const int* order, const float* xz, const float* conv_w,
                                const float* conv_b, float* u, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && L > 0 && D > 0 && ndir > 0);
  long total = (long)ndir * B * L * D;
  if (total == 0) return VC_OK;
  VC_REQUIRE_I32(total);
  VC_REQUIRE_I32((long)B * L * 2 * D);
  const int nch = vc_cdiv(L, DC_T);
  const long runs = (long)ndir * B * nch * D;
  VC_REQUIRE_I32(runs);
  hipLaunchKernelGGL(dirconv_fwd_run, dim3(vc_cdiv(runs, 256)), dim3(256), 0, stream, (int)runs, make_fastdiv(D),
                     make_fastdiv(nch), make_fastdiv(B), L, order, xz, conv_w, conv_b, u);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

static int seg_count_h(int L) { return (L + SCK - 1) / SCK; }

VC_API int vc_mamba_scan_ckpt_floats(int B, int L, int D, int ndir) {
  if (B <= 0 || L <= 0 || D <= 0 || ndir <= 0) return -1;
  const long n = (long)ndir * B * seg_count_h(L) * NST * D;
  return n < (1L << 31) ? (int)n : -1;
}

VC_API int vc_mamba_scan_fwd(int B, int L, int D, int R, int ndir, const float* u, const float* xdbl,
                             const int* order, const float* dt_w, const float* dt_b, const float* A_log,
                             const float* Dskip, float* y, float* ckpt, hipStream_t stream) {
  VC_REQUIRE(B > 0 && L > 0 && D > 0 && D <= 128 && R > 0 && R <= 64 && ndir > 0);
  const dim3 grid(ndir * B), block(vc_cdiv(D, 16) * 64);
  VC_REQUIRE(block.x <= 512);
  const size_t sm = sizeof(float) * seq_lds_floats(L, R, block.x / 4);
  VC_REQUIRE(sm <= 160 * 1024);
  VC_REQUIRE_I32((long)ndir * B * L * (R + 2 * NST));
  ScanArgs a{B, L, D, R, u, xdbl, order, dt_w, dt_b, A_log, Dskip};
  if (R == 9) hipLaunchKernelGGL((scan_fwd<9, false>), grid, block, sm, stream, a, y, ckpt, FusedFwd{});
  else if (R == 16) hipLaunchKernelGGL((scan_fwd<16, false>), grid, block, sm, stream, a, y, ckpt, FusedFwd{});
  else hipLaunchKernelGGL((scan_fwd<0, false>), grid, block, sm, stream, a, y, ckpt, FusedFwd{});
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_mamba_combine_fwd(int B, int L, int D, int ndir, const int* inv_order, const float* gate_logits,
                                const float* y, const float* xz, float* ypsum, float* ysum, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && L > 0 && D > 0 && ndir > 0 && ndir <= 64);
  long total = (long)B * L * D;
  if (total == 0) return VC_OK;
  VC_REQUIRE_I32((long)ndir * total);
  if (ndir <= 10)   // the model's 10 scan orders
    hipLaunchKernelGGL(combine_fwd<10>, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total,
                       make_fastdiv(D), make_fastdiv(L), B, ndir, inv_order, gate_logits, y, xz, ypsum, ysum);
  else
    hipLaunchKernelGGL(combine_fwd<4>, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total,
                       make_fastdiv(D), make_fastdiv(L), B, ndir, inv_order, gate_logits, y, xz, ypsum, ysum);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_mamba_gate_bwd(int B, int L, int D, const float* xz, const float* ypsum, const float* dysum, float* dyp,
                             float* dxz, hipStream_t stream) {
  VC_REQUIRE(B >= 0 && L > 0 && D > 0);
  long total = (long)B * L * D;
  if (total == 0) return VC_OK;
  VC_REQUIRE_I32(2 * total);
  hipLaunchKernelGGL(gate_bwd, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total, make_fastdiv(D), xz,
                     ypsum, dysum, dyp, dxz);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

static int scan_param_reduce(int B, int D, int ndir, const float* gate_logits, const float* p_a, const float* p_d,
                             const float* p_g, float* dA_log, float* dDskip, float* dgate_logits, float* scratch,
                             long scratch_floats, hipStream_t stream) {
  const int nseq = ndir * B;
  int rc = dA_log ? vc_colsum(nseq, D * NST, p_a, (long)D * NST, dA_log, 0.f, scratch, scratch_floats, stream) : 0;
  if (rc) return rc;
  rc = dDskip ? vc_colsum(nseq, D, p_d, (long)D, dDskip, 0.f, scratch, scratch_floats, stream) : 0;
  if (rc) return rc;
  if (!dgate_logits) return VC_OK;
  // dg partials are laid out [k][b]: per direction B contiguous values
  hipLaunchKernelGGL(gate_grad, dim3(1), dim3(256), 0, stream, ndir, B, gate_logits, p_g, dgate_logits);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// Backward of scan + gate-weighted combine, given dyp = d(YP) per token (vc_mamba_gate_bwd).
// Writes du, ddt_lin (per sequence position), the B/C columns of dxdbl (ld R+2N), and
// dA_log / dD / d(gate logits) (overwrite).  ckpt: the segment states vc_mamba_scan_fwd stored
// (null: they are recomputed into ws first).
// ws needs (nseq*D*N + nseq*D + nseq + 2048*ceil(D*N/64)*64) floats (+ vc_mamba_scan_ckpt_floats
// without ckpt).
// the fused front end / tail need float4 rows of W_x / d(dt_lin) (D % 4 == 0) and R <= 16 (one 16-wide
// chunk of dt-rank columns); the model: (D, R) = (72, 9), (128, 16)
static bool scan_fusable(int D, int R) { return D % 4 == 0 && R <= 16; }

static int scan_bwd_impl(int B, int L, int D, int R, int ndir, const float* u, const float* xdbl,
                         const int* order, const float* dt_w, const float* dt_b, const float* A_log,
                         const float* Dskip, const float* gate_logits, const float* y, const float* dyp,
                         const float* ckpt, float* du, float* ddt_lin, float* dxdbl, float* dA_log,
                         float* dDskip, float* dgate_logits, float* ws, long ws_floats, const FusedBwd* fb,
                         hipStream_t stream) {
  VC_REQUIRE(B > 0 && L > 0 && D > 0 && D <= 128 && R > 0 && R <= 64 && ndir > 0 && ndir <= 64);
  VC_REQUIRE(!fb || (ckpt && scan_fusable(D, R)));
  const int nseq = ndir * B;
  const long need_a = (long)nseq * D * NST, need_d = (long)nseq * D, need_g = nseq;
  long need_ck = 0;
  if (!ckpt) {
    const int n = vc_mamba_scan_ckpt_floats(B, L, D, ndir);
    VC_REQUIRE(n > 0);
    need_ck = n;
  }
  VC_REQUIRE(need_a + need_d + need_g + need_ck <= ws_floats);
  const int nw = vc_cdiv(D, 16);
  VC_REQUIRE(nw <= 8);
  // dB / dC partial combine every rbs segments (2; knob SCAN_RBS in the probe library), when the LDS still
  // holds three blocks per CU; else every segment
  int rbs = (int)std::max(1L, std::min(4L, vc_knob("VITCNN_SCAN_RBS", 2)));
  const long tail_n = fb ? (long)seg_count_h(L) * SCK * 16 + (long)D * R : 0;
  auto lds_bytes = [&](int r) {
    return sizeof(float) * (seq_lds_floats(L, R, nw * 16) + std::max<long>(2L * r * nw * SCK * 32, tail_n) + nw + L);
  };
  while (rbs > 1 && lds_bytes(rbs) > 160 * 1024 / 3 && lds_bytes(1) <= 160 * 1024 / 3) --rbs;
  const size_t sm = lds_bytes(rbs);
  VC_REQUIRE(sm <= 160 * 1024);
  // the tail's (a) takes at most two token tiles per wave
  VC_REQUIRE(!fb || (R <= 16 && (seg_count_h(L) * SCK + 15) / 16 <= 2 * nw));
  VC_REQUIRE_I32((long)nseq * L * (R + 2 * NST));
  float* p_a = ws;
  float* p_d = p_a + need_a;
  float* p_g = p_d + need_d;
  float* p_ck = p_g + need_g;
  float* p_rest = p_ck + need_ck;
  long rest = ws_floats - (need_a + need_d + need_g + need_ck);
  ScanArgs a{B, L, D, R, u, xdbl, order, dt_w, dt_b, A_log, Dskip};
  const dim3 grid(nseq), block(nw * 64);
  if (!ckpt) {
    const size_t smf = sizeof(float) * seq_lds_floats(L, R, nw * 16);
    if (R == 9) hipLaunchKernelGGL((scan_fwd<9, false>), grid, block, smf, stream, a, nullptr, p_ck, FusedFwd{});
    else if (R == 16) hipLaunchKernelGGL((scan_fwd<16, false>), grid, block, smf, stream, a, nullptr, p_ck, FusedFwd{});
    else hipLaunchKernelGGL((scan_fwd<0, false>), grid, block, smf, stream, a, nullptr, p_ck, FusedFwd{});
    VC_CHECK_LAUNCH();
    ckpt = p_ck;
  }
  ScanBwdOut o{du, ddt_lin, dxdbl, p_a, p_d, p_g};
  // dB / dC reduce-scatter: bank-masked DPP adds (default) or the select-based form (knob SCAN_SELECT_RS=1,
  // probe library; bit-identical, kept for the A/B measurement and its test)
  const bool bm = vc_knob("VITCNN_SCAN_SELECT_RS", 0) == 0;
#define VC_SCAN_BWD(RV)                                                                                     \
  do {                                                                                                      \
    if (fb) hipLaunchKernelGGL((scan_bwd<RV, true, true>), grid, block, sm, stream, a, ndir, gate_logits, y, dyp, ckpt, o, rbs, *fb); \
    else if (bm) hipLaunchKernelGGL((scan_bwd<RV, true, false>), grid, block, sm, stream, a, ndir, gate_logits, y, dyp, ckpt, o, rbs, FusedBwd{}); \
    else hipLaunchKernelGGL((scan_bwd<RV, false, false>), grid, block, sm, stream, a, ndir, gate_logits, y, dyp, ckpt, o, rbs, FusedBwd{}); \
  } while (0)
  if (R == 9) VC_SCAN_BWD(9);
  else if (R == 16) VC_SCAN_BWD(16);
  else VC_SCAN_BWD(0);
#undef VC_SCAN_BWD
  VC_CHECK_LAUNCH();
  // the three parameter-gradient outputs are optional (the per-sequence partials stay in ws, for
  // vc_mamba_scan_bwd_params)
  return scan_param_reduce(B, D, ndir, gate_logits, p_a, p_d, p_g, dA_log, dDskip, dgate_logits, p_rest, rest, stream);
}

VC_API int vc_mamba_scan_bwd(int B, int L, int D, int R, int ndir, const float* u, const float* xdbl,
                             const int* order, const float* dt_w, const float* dt_b, const float* A_log,
                             const float* Dskip, const float* gate_logits, const float* y, const float* dyp,
                             const float* ckpt, float* du, float* ddt_lin, float* dxdbl, float* dA_log,
                             float* dDskip, float* dgate_logits, float* ws, long ws_floats, hipStream_t stream) {
  return scan_bwd_impl(B, L, D, R, ndir, u, xdbl, order, dt_w, dt_b, A_log, Dskip, gate_logits, y, dyp, ckpt, du,
                       ddt_lin, dxdbl, dA_log, dDskip, dgate_logits, ws, ws_floats, nullptr, stream);
}

VC_API int vc_mamba_scan_bwd_fused(int B, int L, int D, int R, int ndir, const float* u, const float* xdbl,
                                   const int* order, const float* xz, const float* conv_w, const float* conv_b,
                                   const float* x_proj_w, const float* dt_w, const float* dt_b, const float* A_log,
                                   const float* Dskip, const float* gate_logits, const float* y, const float* dyp,
                                   const float* ckpt, float* dpre, float* ddt_lin, float* dxdbl, float* conv_part,
                                   float* dA_log, float* dDskip, float* dgate_logits, float* ws, long ws_floats,
                                   hipStream_t stream) {
  VC_REQUIRE(xz && conv_w && conv_b && x_proj_w && conv_part);
  VC_REQUIRE_I32((long)B * L * 2 * D);
  // tail phase mask: 7 = every phase (the product); the probe library's knob SCAN_TAIL times phases alone
  const FusedBwd fb{xz, conv_w, conv_b, x_proj_w, conv_part, (int)vc_knob("VITCNN_SCAN_TAIL", 7)};
  return scan_bwd_impl(B, L, D, R, ndir, u, xdbl, order, dt_w, dt_b, A_log, Dskip, gate_logits, y, dyp, ckpt, dpre,
                       ddt_lin, dxdbl, dA_log, dDskip, dgate_logits, ws, ws_floats, &fb, stream);
}

VC_API int vc_mamba_scan_fwd_fused(int B, int L, int D, int R, int ndir, const float* xz, const int* order,
                                   const float* conv_w, const float* conv_b, const float* x_proj_w,
                                   const float* dt_w, const float* dt_b, const float* A_log, const float* Dskip,
                                   float* u, float* xdbl, float* y, float* ckpt, hipStream_t stream) {
  VC_REQUIRE(B > 0 && L > 0 && D > 0 && D <= 128 && R > 0 && R <= 64 && ndir > 0);
  VC_REQUIRE(xz && order && conv_w && conv_b && x_proj_w && u && xdbl && scan_fusable(D, R));
  const dim3 grid(ndir * B), block(vc_cdiv(D, 16) * 64);
  VC_REQUIRE(block.x <= 512);
  const size_t sm = sizeof(float) * (seq_lds_floats(L, R, block.x / 4) + L);   // + the order table
  VC_REQUIRE(sm <= 160 * 1024);
  VC_REQUIRE_I32((long)ndir * B * L * (R + 2 * NST));
  VC_REQUIRE_I32((long)B * L * 2 * D);
  const ScanArgs a{B, L, D, R, u, xdbl, order, dt_w, dt_b, A_log, Dskip};
  const FusedFwd f{xz, conv_w, conv_b, x_proj_w, u, xdbl};
  if (R == 9) hipLaunchKernelGGL((scan_fwd<9, true>), grid, block, sm, stream, a, y, ckpt, f);
  else if (R == 16) hipLaunchKernelGGL((scan_fwd<16, true>), grid, block, sm, stream, a, y, ckpt, f);
  else hipLaunchKernelGGL((scan_fwd<0, true>), grid, block, sm, stream, a, y, ckpt, f);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// the x half of dxz from the per-direction dpre (vc_mamba_scan_bwd_fused's output): dirconv_bwd_gather alone
VC_API int vc_mamba_dirconv_bwd_gather(int B, int L, int D, int ndir, const int* inv_order, const float* conv_w,
                                       const float* dpre, float* dxz, hipStream_t stream) {
  VC_REQUIRE(B > 0 && L > 0 && D > 0 && ndir > 0);
  VC_REQUIRE_I32((long)ndir * B * L * D);
  const long tot2 = (long)B * L * D;
  if (ndir <= 10)
    hipLaunchKernelGGL(dirconv_bwd_gather<10>, dim3(vc_cdiv(tot2, 256)), dim3(256), 0, stream, (int)tot2,
                       make_fastdiv(D), make_fastdiv(L), B, ndir, inv_order, conv_w, dpre, dxz);
  else
    hipLaunchKernelGGL(dirconv_bwd_gather<4>, dim3(vc_cdiv(tot2, 256)), dim3(256), 0, stream, (int)tot2,
                       make_fastdiv(D), make_fastdiv(L), B, ndir, inv_order, conv_w, dpre, dxz);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// conv1d weight [D,4] / bias [D] gradients (overwrite) from vc_mamba_scan_bwd_fused's per-sequence partials
VC_API int vc_mamba_conv_params(int B, int D, int ndir, const float* conv_part, float* dconv_w, float* dconv_b,
                                hipStream_t stream) {
  VC_REQUIRE(B > 0 && D > 0 && ndir > 0 && conv_part && dconv_w && dconv_b);
  const int nseq = ndir * B;
  if (dconv_b == dconv_w + 4L * D) return launch_sum_rows(nseq, 5 * D, conv_part, 5L * D, 0L, dconv_w, 0.f, stream);
  const int rc = launch_sum_rows(nseq, 4 * D, conv_part, 5L * D, 0L, dconv_w, 0.f, stream);
  if (rc) return rc;
  return launch_sum_rows(nseq, D, conv_part, 5L * D, 4L * D, dconv_b, 0.f, stream);
}

// vc_mamba_scan_bwd_params + vc_mamba_conv_params in one launch (mamba_params): ws as vc_mamba_scan_bwd_params,
// conv_part as vc_mamba_conv_params; every output overwritten
VC_API int vc_mamba_bwd_params(int B, int D, int ndir, const float* gate_logits, const float* ws, const float* conv_part,
                               float* dA_log, float* dDskip, float* dgate_logits, float* dconv_w, float* dconv_b,
                               hipStream_t stream) {
  VC_REQUIRE(B > 0 && D > 0 && ndir > 0 && ndir <= 64 && gate_logits && ws && conv_part && dA_log && dDskip &&
             dgate_logits && dconv_w && dconv_b);
  const int nseq = ndir * B;
  const float* p_a = ws;
  const float* p_d = p_a + (long)nseq * D * NST;
  const float* p_g = p_d + (long)nseq * D;
  const int ncb = vc_cdiv((NST + 6) * D, 16);
  hipLaunchKernelGGL(mamba_params, dim3(ncb + 1), dim3(256), 0, stream, nseq, D, ndir, ncb, gate_logits, p_a, p_d,
                     p_g, conv_part, dA_log, dDskip, dgate_logits, dconv_w, dconv_b);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// The parameter-gradient reductions of vc_mamba_scan_bwd, run separately (later, or on another
// stream): ws is the workspace a vc_mamba_scan_bwd call with null dA_log / dDskip / dgate_logits left
// its per-sequence partials in (it must not have been written since; given ckpt, ws_floats as then).
// scratch: the column sums' temporary.  Bit-identical to the fused call.
VC_API int vc_mamba_scan_bwd_params(int B, int D, int ndir, const float* gate_logits, const float* ws,
                                    float* dA_log, float* dDskip, float* dgate_logits, float* scratch,
                                    long scratch_floats, hipStream_t stream) {
  VC_REQUIRE(B > 0 && D > 0 && ndir > 0 && ws);
  const int nseq = ndir * B;
  const float* p_a = ws;
  const float* p_d = p_a + (long)nseq * D * NST;
  const float* p_g = p_d + (long)nseq * D;
  return scan_param_reduce(B, D, ndir, gate_logits, p_a, p_d, p_g, dA_log, dDskip, dgate_logits, scratch,
                           scratch_floats, stream);
}


// Backward of the direction gather + causal conv1d + SiLU.  dpre overwrites du in place;
// the x half of dxz (ld 2D) is overwritten (vc_mamba_gate_bwd writes the z half); conv grads
// overwritten.
VC_API int vc_mamba_dirconv_bwd(int B, int L, int D, int ndir, const int* order, const int* inv_order, const float* xz,
                                const float* conv_w, const float* conv_b, float* du, float* dxz,
                                float* dconv_w, float* dconv_b, float* ws, long ws_floats, hipStream_t stream) {
  VC_REQUIRE(B > 0 && L > 0 && D > 0 && ndir > 0);
  const long rows = (long)ndir * B * L;
  VC_REQUIRE_I32(rows * D);
  const int nch = vc_cdiv(L, DC_T);
  const long items = (long)ndir * B * nch;   // DC_T-token runs
  int items_per = std::max<long>(16, (items + 255) / 256);
  while ((long)vc_cdiv(items, items_per) * D * 5 > ws_floats) items_per *= 2;
  const int P = vc_cdiv(items, items_per);
  hipLaunchKernelGGL(dirconv_bwd_wgrad, dim3(vc_cdiv(D, 16), P), dim3(256), 0, stream, D, L, make_fastdiv(nch),
                     make_fastdiv(B), order, xz, conv_w, conv_b, du, (int)items, items_per, ws);
  VC_CHECK_LAUNCH();
  const long tot2 = (long)B * L * D;
  if (ndir <= 10)   // the model's 10 scan orders: one round of loads
    hipLaunchKernelGGL(dirconv_bwd_gather<10>, dim3(vc_cdiv(tot2, 256)), dim3(256), 0, stream, (int)tot2,
                       make_fastdiv(D), make_fastdiv(L), B, ndir, inv_order, conv_w, du, dxz);
  else
    hipLaunchKernelGGL(dirconv_bwd_gather<4>, dim3(vc_cdiv(tot2, 256)), dim3(256), 0, stream, (int)tot2,
                       make_fastdiv(D), make_fastdiv(L), B, ndir, inv_order, conv_w, du, dxz);
  VC_CHECK_LAUNCH();
  if (dconv_b == dconv_w + 4L * D) return launch_sum_rows(P, 5 * D, ws, 5L * D, 0L, dconv_w, 0.f, stream);
  int rc = launch_sum_rows(P, 4 * D, ws, 5L * D, 0L, dconv_w, 0.f, stream);
  if (rc) return rc;
  rc = launch_sum_rows(P, D, ws, 5L * D, 4L * D, dconv_b, 0.f, stream);
  if (rc) return rc;
  return VC_OK;
}
