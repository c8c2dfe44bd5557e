// Row chains of the hsiMamba block: two dense projections with a LayerNorm between them, computed for a
// block of 32 token rows in ONE launch, the intermediate rows kept in LDS.
//
// Reference: hsiMamba.forward (Mutimodality_Mamba7.py:642-701) --
//   front:  T = patch_embed(x) + pos_embed (:651-654), Xn = pre_norm(T) (:656), xz = in_proj(Xn)
//           (transformers modeling_mamba.py:433 / 372);
//   back:   the gated combine of the 10 directions (:694-701, modeling_mamba.py:274), T2 = out_proj(y) + T
//           (modeling_mamba.py:481 + the residual), G = ln1(T2) (:985), CD = change_dim(G) (:1068).
// The separate path is vc_gemm (patch_embed, pos addend) + vc_layernorm_fwd + vc_gemm (in_proj), and
// vc_mamba_combine_fwd + vc_gemm (out_proj, residual addend) + vc_layernorm_fwd + vc_gemm (change_dim):
// seven launches per block on the critical chain, most of them latency-bound (a 5184 x 144 x 144 GEMM is
// ~1.4 us of MFMA work at peak but 14-23 us as a launch).  Here each chain is one launch:
//   A phase   the 32 x K0 operand rows into LDS (front: the block input; back: the combine, whose YP / YS
//             are also written -- bit-identical to vc_mamba_combine_fwd);
//   G1        out1 = A W1^T + addend on v_mfma_f32_16x16x4_f32 (8 waves split the 16-column tiles; a
//             wave's W1 fragments for every k chunk are loaded at once from L2), rows kept in LDS;
//   LN        a wave per row, two-pass mean / variance as vc_layernorm_fwd, in place in LDS;
//   G2        out2 = Xn W2^T (+ bias) the same way.
// Every output the backward reads (T / T2, Xn / G, mean, rstd, xz / CD) is written.  fp32 throughout
// (also in the bf16 precision mode: these products are latency-bound, not MFMA-bound).
#include "common.h"

namespace {

// rows per block BM: 32 (two 16-row MFMA tiles) when that still gives >= 160 blocks, else 16 (hsi2's 3136
// rows: 196 blocks instead of 98 -- the products are fp32-MFMA-bound per block, so the row count per
// block sets the per-block time and the block count the share of the 256 CUs that work)
constexpr int RC_THREADS = 512;  // backward chains: 8 waves; forward chains: one wave per 16-column tile,
                                 // 8..16 waves
constexpr int RC_KC = 16;        // k chunks of 16: K <= 256

struct ChainArgs {
  int rows, K0, E, N2;
  const float* A0;                     // [rows, K0] (front)
  const float* W1;                     // [E][K0]
  const float* add1;                   // addend row (r % add_mod) * E
  int add_mod;
  float* out1;                         // [rows, E]
  const float *lnw, *lnb;
  float eps;
  float *xn, *mu, *rs;                 // [rows, E], [rows], [rows]
  const float* W2;                     // [N2][E]
  const float* b2;                     // [N2] nullable
  float* out2;                         // [rows, N2]
  // combine prologue (back chain): D = K0
  int B, L, ndir;
  const int* inv;                      // [ndir][L]
  const float* glog;                   // [ndir]
  const float* Y;                      // [ndir*B*L, D]
  const float* xz;                     // [B*L, 2D] (z half read)
  float *yp, *ys;                      // [B*L, D]
};

__host__ __device__ __forceinline__ int kpad(int k) { return (k + 15) / 16 * 16; }

// raw buffer loads (32-bit offsets; past the resource's end they return 0): the per-lane part of the
// offset in a VGPR, the part shared by the wave in an SGPR
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rc_rsrc(const float* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float rc_ld(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0));
}

// The block's BM rows of a [rows, K] matrix (K % 4 == 0) into LDS rows of stride lda, zero past the last
// row and in columns K..lda-1: float4 loads, all of a thread's (<= RC_STAGE) issued before any store, so
// the phase costs one load latency instead of one per loop trip.
constexpr int RC_STAGE = 5;   // ceil(32 rows x (256 + 4) floats / 4 / 512 threads)
template <int BM>
__device__ __forceinline__ void stage_rows(float* As, int lda, const float* __restrict__ src, int K, int r0, int nrow) {
  const int q = lda / 4;   // float4 per LDS row (lda % 4 == 0)
  const int kq = K / 4;
  const int nt = blockDim.x;
  for (int base = 0; base < BM * q; base += RC_STAGE * nt) {   // one trip for every shape here
    f32x4 v[RC_STAGE];
#pragma unroll
    for (int j = 0; j < RC_STAGE; ++j) {
      const int i = base + threadIdx.x + j * nt;
      const int rr = i / q, k4 = i - rr * q;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      v[j] = (i < BM * q && rr < nrow && k4 < kq) ? *reinterpret_cast<const f32x4*>(src + (long)(r0 + rr) * K + 4 * k4)
                                                   : z;
    }
#pragma unroll
    for (int j = 0; j < RC_STAGE; ++j) {
      const int i = base + threadIdx.x + j * nt;
      if (i < BM * q) reinterpret_cast<f32x4*>(As)[i] = v[j];
    }
  }
}

// C[16 MT x N] = A[16 MT x K] (LDS, row stride lda, columns K..kpad(K)-1 zero) op(W); op(W) = W[N][K]^T
// (TW = false: a projection, float4 fragment loads along k) or W[K][N] (TW = true: its data gradient,
// four k rows per fragment).  For each output element calls epi(row, col, value) (col < N).  MT = 2: one
// accumulator per 16-row tile; MT = 1: the even and the odd k chunks in two accumulators (two independent
// MFMA chains: the 40-cycle dependent latency of v_mfma_f32_16x16x4_f32 hidden behind its 32-cycle issue).
template <int MT, bool TW = false, typename Epi>
__device__ __forceinline__ void block_gemm(const float* A, int lda, int K, const float* __restrict__ W, int N,
                                           Epi epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int nkc = kpad(K) / 16, ntn = (N + 15) / 16;
  for (int tn = wave; tn < ntn; tn += nw) {
    const int n = 16 * tn + r;
    const int nc = min(n, N - 1);
    f32x4 bw[RC_KC];
    // TW: element (k, n) = W[k N + n]; lane (g, r) reads rows k = 16 kc + 4 g + e: the lane part
    // (4 g N + n) in the VGPR offset, (16 kc + e) N in the SGPR one; rows past K fall out of the resource
    const auto rw = rc_rsrc(W, TW ? (unsigned)(K * N * 4) : 0u);
    const unsigned vo = (unsigned)((4 * g * N + nc) * 4);
#pragma unroll
    for (int kc = 0; kc < RC_KC; ++kc) {
      const int k0 = 16 * kc + 4 * g;
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      if (TW) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bw[kc][e] = kc < nkc ? rc_ld(rw, vo, (unsigned)((16 * kc + e) * N * 4)) : 0.f;
      } else {
        bw[kc] = (kc < nkc && k0 < K) ? *reinterpret_cast<const f32x4*>(W + (long)nc * K + k0) : z;
      }
    }
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < RC_KC; ++kc)
      if (kc < nkc) {
        const int k0 = 16 * kc + 4 * g;
        if (MT == 2) {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(A + r * lda + k0);
          const f32x4 a1 = *reinterpret_cast<const f32x4*>(A + (16 + r) * lda + k0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, bw[kc].x, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, bw[kc].x, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, bw[kc].y, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, bw[kc].y, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, bw[kc].z, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, bw[kc].z, acc1, 0, 0, 0);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, bw[kc].w, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, bw[kc].w, acc1, 0, 0, 0);
        } else {
          const f32x4 a0 = *reinterpret_cast<const f32x4*>(A + r * lda + k0);
          f32x4& acc = (kc & 1) ? acc1 : acc0;
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, bw[kc].x, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, bw[kc].y, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, bw[kc].z, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, bw[kc].w, acc, 0, 0, 0);
        }
      }
    if (n < N) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (MT == 2) {
          epi(4 * g + i, n, acc0[i]);
          epi(16 + 4 * g + i, n, acc1[i]);
        } else {
          epi(4 * g + i, n, acc0[i] + acc1[i]);
        }
      }
    }
  }
}

// MODE 0: front chain (A = block input rows), MODE 1: back chain (A = the gated combine)
template <int MODE, int BM>
__global__ __launch_bounds__(1024) void rowchain_fwd(ChainArgs c) {
  constexpr int MT = BM / 16;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lda = kpad(c.K0) + 4, ldt = kpad(c.E) + 4;   // +4 floats: rows start 4 banks apart
  float* As = sm;                 // [BM][lda]
  float* Ts = sm + BM * lda;      // [BM][ldt]
  const int r0 = blockIdx.x * BM;
  const int nrow = min(BM, c.rows - r0);
  // ---- A phase (zero rows past the end and columns past K0)
  if (MODE == 0) {
    stage_rows<BM>(As, lda, c.A0, c.K0, r0, nrow);
  } else {
    // vc_mamba_combine_fwd per element (same operation order): YP = sum_k softmax(g)_k y_k[inv_k(l)],
    // YS = YP SiLU(z).  A thread takes 4 consecutive channels of a row (float4 gathers) and issues the
    // order-table reads of its items, then their gathers, before any arithmetic.
    const int D = c.K0, q = lda / 4, dq = D / 4;
    float mx = c.glog[0];
    for (int i = 1; i < c.ndir; ++i) mx = fmaxf(mx, c.glog[i]);
    float den = 0.f;
    for (int i = 0; i < c.ndir; ++i) den += __expf(c.glog[i] - mx);
    const float rden = 1.f / den;
    constexpr int NI = 2;   // items per thread per round (32 rows x 33 float4 / 512 threads: 3 at most)
    const int nt = blockDim.x;
    for (int i0 = threadIdx.x; i0 < BM * q; i0 += NI * nt) {
      int tk[NI][10];
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int i = i0 + u * nt, rr = i / q, d4 = i - rr * q;
        const bool ok = i < BM * q && rr < nrow && d4 < dq;
        const int bl = r0 + rr, l = bl % c.L;
#pragma unroll
        for (int kk = 0; kk < 10; ++kk) tk[u][kk] = (ok && kk < c.ndir) ? c.inv[kk * c.L + l] : 0;
      }
      f32x4 yv[NI][10];
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int i = i0 + u * nt, rr = i / q, d4 = i - rr * q;
        const bool ok = i < BM * q && rr < nrow && d4 < dq;
        const int bl = r0 + rr, b = bl / c.L;
#pragma unroll
        for (int kk = 0; kk < 10; ++kk) {
          const f32x4 z = {0.f, 0.f, 0.f, 0.f};
          yv[u][kk] = (ok && kk < c.ndir)
                          ? *reinterpret_cast<const f32x4*>(c.Y + ((long)(kk * c.B + b) * c.L + tk[u][kk]) * D + 4 * d4)
                          : z;
        }
      }
#pragma unroll
      for (int u = 0; u < NI; ++u) {
        const int i = i0 + u * nt, rr = i / q, d4 = i - rr * q;
        if (i >= BM * q) continue;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (rr < nrow && d4 < dq) {
          const long bl = r0 + rr;
          f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int kk = 0; kk < 10; ++kk)
            if (kk < c.ndir) {
              const float gk = __expf(c.glog[kk] - mx) * rden;
              acc.x += gk * yv[u][kk].x;
              acc.y += gk * yv[u][kk].y;
              acc.z += gk * yv[u][kk].z;
              acc.w += gk * yv[u][kk].w;
            }
          const f32x4 zz = *reinterpret_cast<const f32x4*>(c.xz + bl * 2 * D + D + 4 * d4);
          *reinterpret_cast<f32x4*>(c.yp + bl * D + 4 * d4) = acc;
          v.x = acc.x * silu_f(zz.x);
          v.y = acc.y * silu_f(zz.y);
          v.z = acc.z * silu_f(zz.z);
          v.w = acc.w * silu_f(zz.w);
          *reinterpret_cast<f32x4*>(c.ys + bl * D + 4 * d4) = v;
        }
        reinterpret_cast<f32x4*>(As)[i] = v;
      }
    }
  }
  __syncthreads();
  // ---- G1: out1 = A W1^T + addend -> HBM and Ts
  block_gemm<MT>(As, lda, c.K0, c.W1, c.E, [&](int rr, int n, float v) {
    const int row = r0 + rr;
    float o = 0.f;
    if (rr < nrow) {
      o = v + c.add1[(long)(row % c.add_mod) * c.E + n];
      c.out1[(long)row * c.E + n] = o;
    }
    Ts[rr * ldt + n] = o;
  });
  // zero the padding columns E..kpad(E)-1 (read as k by G2)
  for (int i = threadIdx.x; i < BM * (kpad(c.E) - c.E); i += blockDim.x) {
    const int w = kpad(c.E) - c.E, rr = i / w;
    Ts[rr * ldt + c.E + (i - rr * w)] = 0.f;
  }
  __syncthreads();
  // ---- LN (vc_layernorm_fwd's arithmetic: lanes own columns lane + 64 j, two-pass variance)
  {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int rr = wave; rr < nrow; rr += nw) {
      float v[4];
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = lane + 64 * j;
        v[j] = col < c.E ? Ts[rr * ldt + col] : 0.f;
        s += v[j];
      }
      const float mean = wave_sum(s) / c.E;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = lane + 64 * j;
        const float d = col < c.E ? v[j] - mean : 0.f;
        q += d * d;
      }
      const float rstd = rsqrtf(wave_sum(q) / c.E + c.eps);
      const long row = r0 + rr;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = lane + 64 * j;
        if (col < c.E) {
          const float y = (v[j] - mean) * rstd * c.lnw[col] + c.lnb[col];
          Ts[rr * ldt + col] = y;
          c.xn[row * c.E + col] = y;
        }
      }
      if (lane == 0) {
        c.mu[row] = mean;
        c.rs[row] = rstd;
      }
    }
  }
  __syncthreads();
  // ---- G2: out2 = Xn W2^T (+ bias)
  block_gemm<MT>(Ts, ldt, c.E, c.W2, c.N2, [&](int rr, int n, float v) {
    if (rr < nrow) c.out2[(long)(r0 + rr) * c.N2 + n] = v + (c.b2 ? c.b2[n] : 0.f);
  });
}

// ---------------------------------------------------------------- backward chains
// back (MODE 0): dG = dCD W_cd (change_dim's data gradient), the ln1 backward (dT = LN grad written; the
//   block's dw / db partials [blk][2E]), dYS = dT W_out (out_proj's data gradient) and the SiLU(z) gate
//   backward (vc_mamba_gate_bwd's arithmetic): dYP and the z half of dxz.
// front (MODE 1): dXn = dXZ W_in (in_proj's data gradient), the pre_norm backward with the residual
//   gradient (dTt = dT + LN grad written; partials), and dX (+)= dTt W_pe (patch_embed's data gradient,
//   accumulated: the caller orders it after the other branches' writes to dX).
// The weight gradients of the three projections stay separate launches (they reduce over all rows) and
// run off the critical path; ln_params sums the LN partials.
struct BwdChainArgs {
  int rows, K0, E, N2;
  const float* dIn;                    // [rows, K0]: dCD (back) / dXZ (front)
  const float* W1;                     // [K0][E]: W_cd (back) / W_in (front)
  const float *x, *mu, *rs, *lnw;      // the LN input [rows, E] and its statistics / weight
  const float* res;                    // [rows, E] residual gradient (front) or null
  float* dln;                          // [rows, E] out: dT (back) / dTt (front)
  float* part;                         // [blocks][2E] out: LN dw / db partials
  const float* W2;                     // [E][N2]: W_out (back: N2 = D) / W_pe (front: N2 = Cin)
  float* dout;                         // front: dX [rows, N2] (+)=, null = skip
  float beta;                          // front: 0 overwrite, 1 accumulate
  const float* dadd;                   // front: [rows, N2] added to dX (nullable: another branch's share)
  const float *xz, *yp;                // back: gate operands ([rows, 2D], [rows, D])
  float *dyp, *dxz;                    // back: outputs ([rows, D], z half of [rows, 2D])
};

template <int MODE, int BM>
__global__ __launch_bounds__(RC_THREADS) void rowchain_bwd(BwdChainArgs c) {
  constexpr int MT = BM / 16;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int lda = kpad(c.K0) + 4, ldt = kpad(c.E) + 4;
  float* As = sm;                 // [BM][lda]
  float* Ts = sm + BM * lda;      // [BM][ldt]
  float* Ps = Ts + BM * ldt;      // [8 waves][2][256] LN partials
  const int r0 = blockIdx.x * BM;
  const int nrow = min(BM, c.rows - r0);
  stage_rows<BM>(As, lda, c.dIn, c.K0, r0, nrow);
  __syncthreads();
  // ---- G1: dY(LN output) = dIn W1
  block_gemm<MT, true>(As, lda, c.K0, c.W1, c.E, [&](int rr, int n, float v) { Ts[rr * ldt + n] = v; });
  for (int i = threadIdx.x; i < BM * (kpad(c.E) - c.E); i += blockDim.x) {
    const int w = kpad(c.E) - c.E, rr = i / w;
    Ts[rr * ldt + c.E + (i - rr * w)] = 0.f;
  }
  __syncthreads();
  // ---- LN backward (ln_bwd's arithmetic): dx = rs (g - mean(g) - xhat mean(g xhat)), g = dy w
  {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    float pw[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f};
    // the wave's rows (wave, wave + 8, ...: 4 of the 32) -- their LN inputs, statistics and residual
    // gradients loaded at once
    constexpr int WR = BM / (RC_THREADS / 64);
    float xr[WR][4], rsd[WR][4], mur[WR], rsr[WR], wl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wl[j] = lane + 64 * j < c.E ? c.lnw[lane + 64 * j] : 0.f;
#pragma unroll
    for (int u = 0; u < WR; ++u) {
      const int rr = wave + u * nw;
      const bool rok = rr < nrow;
      const long row = r0 + (rok ? rr : 0);
      mur[u] = rok ? c.mu[row] : 0.f;
      rsr[u] = rok ? c.rs[row] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = lane + 64 * j;
        const bool ok = rok && col < c.E;
        xr[u][j] = ok ? c.x[row * c.E + col] : 0.f;
        rsd[u][j] = (ok && c.res) ? c.res[row * c.E + col] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < WR; ++u) {
      const int rr = wave + u * nw;
      if (rr >= nrow) break;
      const long row = r0 + rr;
      const float mu = mur[u], rs = rsr[u];
      float xh[4], gg[4], dd[4];
      float sg = 0.f, sgx = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = lane + 64 * j;
        const bool ok = col < c.E;
        const float d = ok ? Ts[rr * ldt + col] : 0.f;
        const float xv = xr[u][j];
        const float wc = wl[j];
        xh[j] = (xv - mu) * rs;
        gg[j] = d * wc;
        dd[j] = d;
        sg += gg[j];
        sgx += gg[j] * xh[j];
      }
      sg = wave_sum(sg) / c.E;
      sgx = wave_sum(sgx) / c.E;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = lane + 64 * j;
        pw[j] += dd[j] * xh[j];
        pb[j] += dd[j];
        if (col < c.E) {
          const float v = rs * (gg[j] - sg - xh[j] * sgx) + rsd[u][j];
          c.dln[row * c.E + col] = v;
          Ts[rr * ldt + col] = v;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      Ps[(wave * 2) * 256 + lane + 64 * j] = pw[j];
      Ps[(wave * 2 + 1) * 256 + lane + 64 * j] = pb[j];
    }
  }
  __syncthreads();
  for (int col = threadIdx.x; col < c.E; col += blockDim.x) {   // fixed wave order
    float a = 0.f, bb = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
      a += Ps[(w * 2) * 256 + col];
      bb += Ps[(w * 2 + 1) * 256 + col];
    }
    c.part[(long)blockIdx.x * 2 * c.E + col] = a;
    c.part[(long)blockIdx.x * 2 * c.E + c.E + col] = bb;
  }
  // ---- G2
  if (MODE == 0) {
    // dYS = dT W_out, then the gate backward (vc_mamba_gate_bwd)
    const int D = c.N2;
    block_gemm<MT, true>(Ts, ldt, c.E, c.W2, D, [&](int rr, int n, float v) {
      if (rr < nrow) {
        const long row = r0 + rr;
        const float z = c.xz[row * 2 * D + D + n];
        const float sg = sigmoid_f(z);
        c.dyp[row * D + n] = v * z * sg;
        c.dxz[row * 2 * D + D + n] = v * c.yp[row * D + n] * sg * (1.f + z * (1.f - sg));
      }
    });
  } else if (c.dout) {
    block_gemm<MT, true>(Ts, ldt, c.E, c.W2, c.N2, [&](int rr, int n, float v) {
      if (rr < nrow) {
        const long o = (long)(r0 + rr) * c.N2 + n;
        float* p = c.dout + o;
        *p = (c.beta != 0.f ? *p * c.beta : 0.f) + v + (c.dadd ? c.dadd[o] : 0.f);
      }
    });
  }
}

int rc_bm(int rows) { return vc_cdiv(rows, 32) >= 160 ? 32 : 16; }
size_t chain_lds(int bm, int K0, int E) { return sizeof(float) * bm * ((kpad(K0) + 4) + (kpad(E) + 4)); }
// forward chains: a wave per 16-column tile of the wider product, 8..16 waves
int chain_threads(int n1, int n2) { return 64 * std::min(16, std::max(8, std::max(vc_cdiv(n1, 16), vc_cdiv(n2, 16)))); }

size_t bwd_chain_lds(int bm, int K0, int E) { return chain_lds(bm, K0, E) + sizeof(float) * 16 * 256; }

}  // namespace

VC_API int vc_rowchain_front(int rows, int K0, int E, int N2, const float* x, const float* w_embed, const float* pos,
                             int L, float* t, const float* ln_w, const float* ln_b, float eps, float* xn, float* mean,
                             float* rstd, const float* w_proj, float* out, hipStream_t stream) {
  VC_REQUIRE(rows > 0 && K0 > 0 && K0 <= 256 && K0 % 4 == 0 && E > 0 && E <= 256 && E % 4 == 0 && N2 > 0 && L > 0);
  VC_REQUIRE(x && w_embed && pos && t && ln_w && ln_b && xn && mean && rstd && w_proj && out);
  VC_REQUIRE_I32((long)rows * std::max(std::max(K0, E), N2));
  ChainArgs c{};
  c.rows = rows, c.K0 = K0, c.E = E, c.N2 = N2, c.A0 = x, c.W1 = w_embed, c.add1 = pos, c.add_mod = L, c.out1 = t;
  c.lnw = ln_w, c.lnb = ln_b, c.eps = eps, c.xn = xn, c.mu = mean, c.rs = rstd, c.W2 = w_proj, c.b2 = nullptr;
  c.out2 = out;
  const int bm = rc_bm(rows);
  if (bm == 32)
    hipLaunchKernelGGL((rowchain_fwd<0, 32>), dim3(vc_cdiv(rows, 32)), dim3(chain_threads(E, N2)), chain_lds(32, K0, E),
                       stream, c);
  else
    hipLaunchKernelGGL((rowchain_fwd<0, 16>), dim3(vc_cdiv(rows, 16)), dim3(chain_threads(E, N2)), chain_lds(16, K0, E),
                       stream, c);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_rowchain_back(int B, int L, int D, int ndir, const int* inv_order, const float* gate_logits,
                            const float* y, const float* xz, float* ypsum, float* ysum, int E, const float* w_out,
                            const float* residual, float* t2, const float* ln_w, const float* ln_b, float eps,
                            float* g, float* mean, float* rstd, int N2, const float* w_proj, const float* b_proj,
                            float* out, hipStream_t stream) {
  VC_REQUIRE(B > 0 && L > 0 && D > 0 && D <= 256 && D % 4 == 0 && ndir > 0 && ndir <= 10 && E > 0 && E <= 256 &&
             E % 4 == 0 && N2 > 0);
  VC_REQUIRE(inv_order && gate_logits && y && xz && ypsum && ysum && w_out && residual && t2 && ln_w && ln_b && g &&
             mean && rstd && w_proj && out);
  const long rows = (long)B * L;
  VC_REQUIRE_I32((long)ndir * rows * D);
  VC_REQUIRE_I32(rows * std::max(std::max(2 * D, E), N2));
  ChainArgs c{};
  c.rows = (int)rows, c.K0 = D, c.E = E, c.N2 = N2, c.A0 = nullptr, c.W1 = w_out, c.add1 = residual,
  c.add_mod = (int)rows, c.out1 = t2;
  c.lnw = ln_w, c.lnb = ln_b, c.eps = eps, c.xn = g, c.mu = mean, c.rs = rstd, c.W2 = w_proj, c.b2 = b_proj;
  c.out2 = out;
  c.B = B, c.L = L, c.ndir = ndir, c.inv = inv_order, c.glog = gate_logits, c.Y = y, c.xz = xz, c.yp = ypsum,
  c.ys = ysum;
  const int bm = rc_bm((int)rows);
  if (bm == 32)
    hipLaunchKernelGGL((rowchain_fwd<1, 32>), dim3(vc_cdiv(rows, 32)), dim3(chain_threads(E, N2)), chain_lds(32, D, E),
                       stream, c);
  else
    hipLaunchKernelGGL((rowchain_fwd<1, 16>), dim3(vc_cdiv(rows, 16)), dim3(chain_threads(E, N2)), chain_lds(16, D, E),
                       stream, c);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_rowchain_back_bwd(int rows, int Cout, int E, int D, const float* dcd, const float* w_cd, const float* t2,
                                const float* mean, const float* rstd, const float* ln_w, float* dt, float* ln_part,
                                const float* w_out, const float* xz, const float* ypsum, float* dyp, float* dxz,
                                hipStream_t stream) {
  VC_REQUIRE(rows > 0 && Cout > 0 && Cout <= 256 && E > 0 && E <= 256 && D > 0);
  VC_REQUIRE(dcd && w_cd && t2 && mean && rstd && ln_w && dt && ln_part && w_out && xz && ypsum && dyp && dxz);
  VC_REQUIRE_I32((long)rows * std::max(std::max(Cout, E), 2 * D));
  BwdChainArgs c{};
  c.rows = rows, c.K0 = Cout, c.E = E, c.N2 = D, c.dIn = dcd, c.W1 = w_cd, c.x = t2, c.mu = mean, c.rs = rstd;
  c.lnw = ln_w, c.res = nullptr, c.dln = dt, c.part = ln_part, c.W2 = w_out, c.xz = xz, c.yp = ypsum, c.dyp = dyp;
  c.dxz = dxz;
  const int bm = rc_bm(rows);
  if (bm == 32)
    hipLaunchKernelGGL((rowchain_bwd<0, 32>), dim3(vc_cdiv(rows, 32)), dim3(RC_THREADS), bwd_chain_lds(32, Cout, E),
                       stream, c);
  else
    hipLaunchKernelGGL((rowchain_bwd<0, 16>), dim3(vc_cdiv(rows, 16)), dim3(RC_THREADS), bwd_chain_lds(16, Cout, E),
                       stream, c);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_API int vc_rowchain_front_bwd(int rows, int K0, int E, int Cin, const float* dxz, const float* w_in, const float* t,
                                 const float* mean, const float* rstd, const float* ln_w, const float* res, float* dtt,
                                 float* ln_part, const float* w_embed, float* dx, float beta, const float* dx_add,
                                 hipStream_t stream) {
  VC_REQUIRE(rows > 0 && K0 > 0 && K0 <= 256 && E > 0 && E <= 256 && Cin > 0);
  VC_REQUIRE(dxz && w_in && t && mean && rstd && ln_w && dtt && ln_part && (!dx || w_embed));
  VC_REQUIRE_I32((long)rows * std::max(std::max(K0, E), Cin));
  BwdChainArgs c{};
  c.rows = rows, c.K0 = K0, c.E = E, c.N2 = Cin, c.dIn = dxz, c.W1 = w_in, c.x = t, c.mu = mean, c.rs = rstd;
  c.lnw = ln_w, c.res = res, c.dln = dtt, c.part = ln_part, c.W2 = w_embed, c.dout = dx, c.beta = beta, c.dadd = dx_add;
  const int bm = rc_bm(rows);
  if (bm == 32)
    hipLaunchKernelGGL((rowchain_bwd<1, 32>), dim3(vc_cdiv(rows, 32)), dim3(RC_THREADS), bwd_chain_lds(32, K0, E),
                       stream, c);
  else
    hipLaunchKernelGGL((rowchain_bwd<1, 16>), dim3(vc_cdiv(rows, 16)), dim3(RC_THREADS), bwd_chain_lds(16, K0, E),
                       stream, c);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// LayerNorm weight / bias gradients (dw = beta dw + sum, db likewise) from a backward chain's partials
VC_API int vc_rowchain_ln_params(int rows, int E, const float* ln_part, float* dw, float* db, float beta,
                                 hipStream_t stream) {
  VC_REQUIRE(rows > 0 && E > 0 && ln_part && dw && db);
  const int P = vc_cdiv(rows, rc_bm(rows));
  if (db == dw + E) return launch_sum_rows(P, 2 * E, ln_part, 2L * E, 0L, dw, beta, stream);
  const int rc = launch_sum_rows(P, E, ln_part, 2L * E, 0L, dw, beta, stream);
  if (rc) return rc;
  return launch_sum_rows(P, E, ln_part, 2L * E, (long)E, db, beta, stream);
}

VC_API int vc_rowchain_ln_part_floats(int rows, int E) {
  if (rows <= 0 || E <= 0) return -1;
  const long n = (long)vc_cdiv(rows, rc_bm(rows)) * 2 * E;
  return n < (1L << 31) ? (int)n : -1;
}
