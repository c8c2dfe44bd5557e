// GEMM on CDNA4 matrix cores: fp32 (v_mfma_f32_16x16x4_f32, an exact fp32 fma chain) or bf16
// operands with fp32 accumulation (v_mfma_f32_16x16x32_bf16, the config-2 precision mode), plus
// split-K reduction and deterministic column sums.
//
// Every dense contraction of the ViT-CNN step goes through vc_gemm: the 1x1 convolutions
// (patch_embed, change_dim, channel_feature, NonLocal theta/phi/g/W, fusion layers;
// Mutimodality_Mamba7.py:258, :1068, :1071, :101-134, :1098, :1124), the im2col'ed 3x3
// convolutions (:1040), the Mamba in/x/dt/out projections (transformers
// modeling_mamba.py:372, :433, :438, :481), the TokenLearner weighted pooling (:47) and
// every weight / input gradient of those.  Activations are channels-last [rows, C], so a
// 1x1 conv is C[M,N] = X[M,K] * W[N,K]^T (transB=1) and its weight gradient is
// dW[N,K] = dY[M,N]^T * X[M,K] (transA=1, split over M).
#include "common.h"
#include "mfma_tiles.h"

namespace {

constexpr int BM = 64, BN = 64;
constexpr int LDS_STRIDE = 81;  // 64 + 17: conflict-free fragment reads, <=2-way stores

enum { F_RELU = 1, F_BF16 = 2, F_LEGACY = 4, F_V2 = 8, F_PIPE = 16, F_NOPIPE = 32, F_MASK = 64 };

struct Epi {
  float alpha, beta;
  const float* bias;     // [N] or null
  const float* addend;   // addend[(m % add_mod) * add_ld + n] or null; with F_MASK a ReLU output mask
  long add_ld;
  int add_mod;
  int flags;
};

__device__ __forceinline__ float epilogue(const Epi& e, float acc, const float* cptr, int m, int n) {
  float v = e.alpha * acc;
  if (e.beta != 0.f) v += e.beta * (*cptr);
  if (e.bias) v += e.bias[n];
  if (e.addend) {
    const float a = e.addend[(long)(m % e.add_mod) * e.add_ld + n];
    if (e.flags & F_MASK) v = a > 0.f ? v : 0.f;   // ReLU backward through the layer output `a`
    else v += a;
  }
  if (e.flags & F_RELU) v = fmaxf(v, 0.f);
  return v;
}

struct GemmArgs {
  int M, N, K, Ne, k_chunk, nsplit;   // Ne = N + 1 when the implicit ones column (bias gradient) is on
  const float* A;
  long lda, sA;
  const float* B;
  long ldb, sB;
  float* C;
  long ldc, sC;
  float* bias_grad;                   // [M]: column N of the product (sum over K of A)
  float* part;                        // split-K partial slabs [batch*nsplit][M][Ne]
  unsigned int* cnt;                  // per-tile arrival counters (zero on entry, left zero) or null
  Epi epi;
  // BatchNorm statistics of the output (gemm_pipe, nsplit == 1 only; vc_gemm_colstats): per 64-row tile ym and
  // column n, fp64 sum (y - shift[n]) -> colstats[ym * 2 N + n] and sum (y - shift[n])^2 -> [... + N + n]
  double* colstats = nullptr;
  const float* shift = nullptr;
};

__device__ __forceinline__ void store_out(const GemmArgs& g, int zb, int m, int n, float acc) {
  if (n < g.N) {
    float* cp = g.C + (long)zb * g.sC + (long)m * g.ldc + n;
    *cp = epilogue(g.epi, acc, cp, m, n);
  } else {
    float* bp = g.bias_grad + m;
    *bp = g.epi.alpha * acc + (g.epi.beta != 0.f ? g.epi.beta * *bp : 0.f);
  }
}

// A element (m,k): TA ? A[k*lda + m] : A[m*lda + k];  B element (k,n): TB ? B[n*ldb + k] : B[k*ldb + n]
// 64x64 output tile per 256-thread block (4 waves of 32x32 = 2x2 v_mfma_f32_16x16x4_f32), BK = 32
// K steps staged through LDS (k-major, 81-float rows, 20.7 KB) with a one-tile register prefetch
// issued before the tile's 32 MFMAs per wave (1024 cycles per SIMD), which covers an HBM miss.
// Each thread moves NE = 8 elements of each operand per K step.  VA / VB: the operand is 16-B
// aligned with a leading dimension divisible by 4, so those 8 elements are two float4 loads
// (edges fall back to guarded scalar loads).
constexpr int BK = 32;
constexpr int NE = BM * BK / 256;  // 8

// tile coordinates (row-of-operand r in [0,64), k in [0,BK)) of this thread's e-th element
template <bool T, bool V>
__device__ __forceinline__ void tile_idx(int tid, int e, int& r, int& k) {
  if (V) {
    if (T) { k = (tid >> 4) + 16 * (e >> 2); r = (tid & 15) * 4 + (e & 3); }  // r contiguous in memory
    else   { r = tid >> 2; k = (tid & 3) * 8 + e; }                          // k contiguous in memory
  } else {
    if (T) { r = tid & 63; k = (tid >> 6) + 4 * e; }
    else   { k = tid & 31; r = (tid >> 5) + 8 * e; }
  }
}

// The fixed summation order of split-K slices (every combine path of every kernel): G interleaved partial sums
// s_g = sum over z = g, g+G, ... (ascending), then s_0 + s_1 + ... + s_{G-1} left to right.  G (a
// power of two <= 16) depends on nsplit only (slab_groups), so the in-launch and the separate
// combine give bit-identical results.
__host__ __device__ inline int slab_groups(int nsplit) {
  int g = 1;
  while (g < 16 && 4 * (2 * g) <= nsplit) g *= 2;
  return g;
}

__device__ __forceinline__ float slab_sum(const float* p, long slab, int nsplit, int G) {
  float s[16];
#pragma unroll
  for (int g = 0; g < 16; ++g) s[g] = 0.f;
  for (int z0 = 0; z0 < nsplit; z0 += G) {
#pragma unroll
    for (int g = 0; g < 16; ++g)
      if (g < G && z0 + g < nsplit) s[g] += p[(z0 + g) * slab];
  }
  float t = s[0];
#pragma unroll
  for (int g = 1; g < 16; ++g)
    if (g < G) t += s[g];
  return t;
}

// One 64x64 output tile (bx, by) of K slice / batch bz; tn x tm tiles per slice (the arrival-counter
// index of the in-launch combine).  Shared by the single-problem kernel and the grouped one, which
// own the LDS (As, Bs: BK * LDS_STRIDE floats each, `last`: one int).
template <bool TA, bool TB, bool VA, bool VB, int PD>
__device__ __forceinline__ void gemm_f32_tile(const GemmArgs& g, int bx, int by, int bz, int tn, int tm,
                                              float* __restrict__ As, float* __restrict__ Bs, int* last) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = bx * BN, m0 = by * BM;
  const int zb = bz / g.nsplit, zs = bz % g.nsplit;
  const int kbeg = zs * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const float* A = g.A + (long)zb * g.sA;
  const float* Bp = g.B + (long)zb * g.sB;
  const bool ones = g.Ne > g.N;

  // PD register sets of staged operand tiles: the global loads of k-tiles t+1 .. t+PD-1 are in
  // flight while tile t is multiplied (the small-grid GEMMs of the step are bound by the load
  // latency of their few k-tiles, not by the MFMAs); the k order and the MFMA sequence are those of
  // PD = 1, so the results are bit-identical for every depth.
  float ra[PD][NE], rb[PD][NE];
  auto a_at = [&](int gm, int gk) -> float {
    return (gm < g.M && gk < kend) ? (TA ? A[(long)gk * g.lda + gm] : A[(long)gm * g.lda + gk]) : 0.f;
  };
  auto b_at = [&](int gn, int gk) -> float {
    if (gk >= kend) return 0.f;
    if (gn < g.N) return TB ? Bp[(long)gn * g.ldb + gk] : Bp[(long)gk * g.ldb + gn];
    return (ones && gn == g.N) ? 1.f : 0.f;
  };
  auto load = [&](int k0, float (&xa)[NE], float (&xb)[NE]) {
#pragma unroll
    for (int v = 0; v < NE / 4; ++v) {
      if (VA) {
        int m, k;
        tile_idx<TA, true>(tid, 4 * v, m, k);
        const int gm = m0 + m, gk = k0 + k;
        const bool full = TA ? (gk < kend && gm + 3 < g.M) : (gm < g.M && gk + 3 < kend);
        if (full) {
          const float4 x = *reinterpret_cast<const float4*>(TA ? A + (long)gk * g.lda + gm : A + (long)gm * g.lda + gk);
          xa[4 * v] = x.x; xa[4 * v + 1] = x.y; xa[4 * v + 2] = x.z; xa[4 * v + 3] = x.w;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) xa[4 * v + i] = TA ? a_at(gm + i, gk) : a_at(gm, gk + i);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int m, k;
          tile_idx<TA, false>(tid, 4 * v + i, m, k);
          xa[4 * v + i] = a_at(m0 + m, k0 + k);
        }
      }
      if (VB) {
        int n, k;
        tile_idx<!TB, true>(tid, 4 * v, n, k);
        const int gn = n0 + n, gk = k0 + k;
        const bool full = TB ? (gn < g.N && gk + 3 < kend) : (gk < kend && gn + 3 < g.N);
        if (full) {
          const float4 x = *reinterpret_cast<const float4*>(TB ? Bp + (long)gn * g.ldb + gk : Bp + (long)gk * g.ldb + gn);
          xb[4 * v] = x.x; xb[4 * v + 1] = x.y; xb[4 * v + 2] = x.z; xb[4 * v + 3] = x.w;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) xb[4 * v + i] = TB ? b_at(gn, gk + i) : b_at(gn + i, gk);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int n, k;
          tile_idx<!TB, false>(tid, 4 * v + i, n, k);
          xb[4 * v + i] = b_at(n0 + n, k0 + k);
        }
      }
    }
  };
  auto store = [&](const float (&xa)[NE], const float (&xb)[NE]) {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      int m, k;
      tile_idx<TA, VA>(tid, e, m, k);
      As[k * LDS_STRIDE + m] = xa[e];
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      int n, k;
      tile_idx<!TB, VB>(tid, e, n, k);
      Bs[k * LDS_STRIDE + n] = xb[e];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = lane >> 4;
  const int nk = kbeg < kend ? (kend - kbeg + BK - 1) / BK : 0;
#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (p < nk) load(kbeg + p * BK, ra[p], rb[p]);
  for (int t0 = 0; t0 < nk; t0 += PD) {
#pragma unroll
    for (int s = 0; s < PD; ++s) {
      const int t = t0 + s;
      if (t < nk) {
        store(ra[s], rb[s]);
        __syncthreads();
        if (t + PD < nk) load(kbeg + (t + PD) * BK, ra[s], rb[s]);
#pragma unroll
        for (int ks = 0; ks < BK / 4; ++ks) {
          const int kk = ks * 4 + fk;
          const float a0 = As[kk * LDS_STRIDE + wm * 32 + fr];
          const float a1 = As[kk * LDS_STRIDE + wm * 32 + 16 + fr];
          const float b0 = Bs[kk * LDS_STRIDE + wn * 32 + fr];
          const float b1 = Bs[kk * LDS_STRIDE + wn * 32 + 16 + fr];
          acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
          acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
          acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
      }
    }
  }

  // C/D map of 16x16x4: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + mi * 16 + fk * 4 + r;
        const int n = n0 + wn * 32 + ni * 16 + fr;
        if (m < g.M && n < g.Ne) {
          if (g.nsplit > 1) g.part[((long)bz * g.M + m) * g.Ne + n] = acc[mi][ni][r];
          else store_out(g, zb, m, n, acc[mi][ni][r]);
        }
      }
  if (g.nsplit == 1 || !g.cnt) return;

  // In-launch split-K combine (cdna_hip_programming.md, "In-launch split-K reduction"): every
  // slice publishes its slab (stores drained, barrier, one agent-scope release), takes a ticket;
  // the tile's last arriver acquires and sums all slices in slab_sum's fixed order — the same order
  // as the separate reduce, so results do not depend on which slice arrives last — then re-zeroes the
  // counter for the next launch on this stream.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int tile = (zb * tm + by) * tn + bx;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(&g.cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last = (t == (unsigned)(g.nsplit - 1));
  }
  __syncthreads();
  if (!*last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const long slab = (long)g.M * g.Ne;
  const float* pz = g.part + (long)zb * g.nsplit * slab;
  for (int e = tid; e < BM * BN; e += 256) {
    const int m = m0 + (e >> 6), n = n0 + (e & 63);
    if (m >= g.M || n >= g.Ne) continue;
    store_out(g, zb, m, n, slab_sum(pz + (long)m * g.Ne + n, slab, g.nsplit, slab_groups(g.nsplit)));
  }
  if (tid == 0) __hip_atomic_store(&g.cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool TA, bool TB, bool VA, bool VB, int PD>
__global__ __launch_bounds__(256) void gemm_f32_mfma(GemmArgs g) {
  __shared__ float As[BK * LDS_STRIDE];
  __shared__ float Bs[BK * LDS_STRIDE];
  __shared__ int last;
  gemm_f32_tile<TA, TB, VA, VB, PD>(g, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x, gridDim.y, As, Bs, &last);
}

// Grouped launch: up to GROUP_MAX independent problems in one grid (a horizontal fusion of GEMMs that
// would otherwise be separate launches on one stream).  Block b belongs to the problem p with
// start[p] <= b < start[p + 1] and runs its tile (b - start[p]) in (x fastest, y, z) order; the
// (TA, TB, VA, VB) variant is a runtime switch (registers: the largest variant's).
constexpr int GROUP_MAX = 8;
struct GemmGroup {
  int n;
  int start[GROUP_MAX + 1];
  int tn[GROUP_MAX], tm[GROUP_MAX], variant[GROUP_MAX];
  GemmArgs g[GROUP_MAX];
};

// The kernel arguments are indexed with constants only (an unrolled select), so the problem's
// descriptor is read with scalar loads from the argument segment instead of a dynamically indexed
// private copy.
struct GroupSel {
  GemmArgs g;
  int start, tn, tm, variant;
};

__device__ __forceinline__ GroupSel group_select(const GemmGroup& G, int b) {
  GroupSel s;
  s.g = G.g[0];
  s.start = G.start[0];
  s.tn = G.tn[0];
  s.tm = G.tm[0];
  s.variant = G.variant[0];
#pragma unroll
  for (int k = 1; k < GROUP_MAX; ++k)
    if (k < G.n && b >= G.start[k]) {
      s.g = G.g[k];
      s.start = G.start[k];
      s.tn = G.tn[k];
      s.tm = G.tm[k];
      s.variant = G.variant[k];
    }
  return s;
}

template <int PD>
__global__ __launch_bounds__(256) void gemm_f32_group(GemmGroup G) {
  __shared__ float As[BK * LDS_STRIDE];
  __shared__ float Bs[BK * LDS_STRIDE];
  __shared__ int last;
  const int b = blockIdx.x;
  const GroupSel s = group_select(G, b);
  const int local = b - s.start;
  const int tn = s.tn, tm = s.tm;
  const int bx = local % tn, by = (local / tn) % tm, bz = local / (tn * tm);
  const GemmArgs& g = s.g;
#define VC_TILE(V_, TA_, TB_, VA_, VB_) \
  case V_: gemm_f32_tile<TA_, TB_, VA_, VB_, PD>(g, bx, by, bz, tn, tm, As, Bs, &last); break;
  switch (s.variant) {
    VC_TILE(0, false, false, false, false) VC_TILE(1, false, false, false, true)
    VC_TILE(2, false, false, true, false) VC_TILE(3, false, false, true, true)
    VC_TILE(4, false, true, false, false) VC_TILE(5, false, true, false, true)
    VC_TILE(6, false, true, true, false) VC_TILE(7, false, true, true, true)
    VC_TILE(8, true, false, false, false) VC_TILE(9, true, false, false, true)
    VC_TILE(10, true, false, true, false) VC_TILE(11, true, false, true, true)
    VC_TILE(12, true, true, false, false) VC_TILE(13, true, true, false, true)
    VC_TILE(14, true, true, true, false) VC_TILE(15, true, true, true, true)
    default: break;
  }
#undef VC_TILE
}

// Column sums: block (cx, ry) sums rows [ry*rows_per, ...) of 64 columns (4 row lanes, combined in
// order).  One row block (P == 1) writes out directly; else it writes part[ry][Cn] and the fixed-order
// reduction over the P partials (colsum_reduce: 4 partial lanes p = l, l+4, ..., then the lanes in
// order) runs in the last-arriving block of the column group (cnt) or in colsum_final.
__device__ __forceinline__ void colsum_reduce(int P, int Cn, const float* __restrict__ part, int cx,
                                              float* __restrict__ out, float beta) {
  __shared__ float shr[4][64];
  const int cl = threadIdx.x & 63, pl = threadIdx.x >> 6;
  const int c = cx * 64 + cl;
  float s = 0.f;
  if (c < Cn) {
#pragma unroll 4
    for (int p = pl; p < P; p += 4) s += part[(long)p * Cn + c];
  }
  shr[pl][cl] = s;
  __syncthreads();
  if (pl == 0 && c < Cn)
    out[c] = (beta != 0.f ? beta * out[c] : 0.f) + ((shr[0][cl] + shr[1][cl]) + (shr[2][cl] + shr[3][cl]));
}

__global__ __launch_bounds__(256) void colsum_partial(int R, int Cn, const float* __restrict__ X, long ldx,
                                                      int rows_per, float* __restrict__ part,
                                                      unsigned int* __restrict__ cnt, float* __restrict__ out,
                                                      float beta) {
  __shared__ float sh[4][64];
  const int cl = threadIdx.x & 63;
  const int c = blockIdx.x * 64 + cl;
  const int rl = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(R, r0 + rows_per);
  float s = 0.f;
  if (c < Cn) {
#pragma unroll 4
    for (int r = r0 + rl; r < r1; r += 4) s += X[(long)r * ldx + c];
  }
  sh[rl][cl] = s;
  __syncthreads();
  if (gridDim.y == 1) {
    if (rl == 0 && c < Cn)
      out[c] = (beta != 0.f ? beta * out[c] : 0.f) + ((sh[0][cl] + sh[1][cl]) + (sh[2][cl] + sh[3][cl]));
    return;
  }
  if (rl == 0 && c < Cn) part[(long)blockIdx.y * Cn + c] = (sh[0][cl] + sh[1][cl]) + (sh[2][cl] + sh[3][cl]);
  if (!cnt || !block_last_arriver(cnt + blockIdx.x, gridDim.y)) return;
  colsum_reduce(gridDim.y, Cn, part, blockIdx.x, out, beta);
}

__global__ __launch_bounds__(256) void colsum_final(int P, int Cn, const float* __restrict__ part,
                                                    float* __restrict__ out, float beta) {
  colsum_reduce(P, Cn, part, blockIdx.x, out, beta);
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// gemm_mfma: K-contiguous LDS images, fp32 (v_mfma_f32_16x16x4_f32) or bf16 operands
// (v_mfma_f32_16x16x32_bf16, fp32 accumulation).
//
// Both operands are staged as K-contiguous LDS images: a tile row holds 128 B of k (32 fp32 or 64
// bf16) as eight 16-B chunks, chunk c of row r at slot c ^ ((r >> 1) & 7).  The XOR makes the
// fragment reads (ds_read_b128: rows lane&15, chunks lane>>4) and the staging writes
// (ds_write_b128) bank-conflict-free.  A lane reads one 16-B chunk per operand, 16-row tile and
// sub-step: in bf16 that is the 8-element k fragment of one 16x16x32 MFMA; in fp32 its 4 elements
// feed four 16x16x4 MFMAs in which lane group g = lane>>4 supplies k = 4g + j (the k order inside
// a 16-wide step is permuted identically for A and B: the same products, summed in another
// order).  Two LDS stages and one barrier per k-tile: the next tile's global loads are in flight
// while the current one is multiplied.  bf16 operands are rounded (RNE, v_cvt_pk_bf16_f32) as
// they are staged, so activations stay fp32 in HBM and the mode only changes the contraction.
namespace g2 {

using ::slab_groups;
using ::slab_sum;

// Block = 4 waves (2 x 2) over a BM x BN output tile, each wave (BM/2) x (BN/2).  1-D grid of
// nsplit * tn * tm * batch blocks in XCD-aware order: the hardware deals block i to XCD i % 8, and
// each XCD gets a contiguous run of logical blocks (split slice fastest, then n, m, batch): the K
// slices of one tile run together on one XCD, so the in-launch combine reads their slabs from that
// XCD's L2, and tiles sharing an A row panel meet in the same L2.
template <bool BF, int BM, int BN, bool TA, bool TB, int PF>
__global__ __launch_bounds__(256) void gemm_mfma(GemmArgs g, int tn, int tm, unsigned total, int va, int vb,
                                                  int G, int zfast) {
  constexpr int KT = BF ? 64 : 32;
  constexpr int MT = BM / 32, NT = BN / 32;
  constexpr int STAGE = (BM + BN) * ROWB;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const unsigned bid = blockIdx.x, q8 = total >> 3, r8 = total & 7, x8 = bid & 7;
  const unsigned lin = x8 * q8 + min(x8, r8) + (bid >> 3);
  // zfast: split slice fastest (the slices of a tile share an XCD: L2-local in-launch combine);
  // else tiles fastest (the tiles of one K slice share an XCD: its A / B rows are fetched once)
  int zs, xn, ym, zb;
  if (zfast) {
    zs = (int)(lin % (unsigned)g.nsplit);
    const unsigned t1 = lin / (unsigned)g.nsplit;
    xn = (int)(t1 % (unsigned)tn);
    const unsigned t2 = t1 / (unsigned)tn;
    ym = (int)(t2 % (unsigned)tm);
    zb = (int)(t2 / (unsigned)tm);
  } else {
    xn = (int)(lin % (unsigned)tn);
    const unsigned t1 = lin / (unsigned)tn;
    ym = (int)(t1 % (unsigned)tm);
    const unsigned t2 = t1 / (unsigned)tm;
    zs = (int)(t2 % (unsigned)g.nsplit);
    zb = (int)(t2 / (unsigned)g.nsplit);
  }
  const int z = zb * g.nsplit + zs;
  const int m0 = ym * BM, n0 = xn * BN;
  const int kbeg = zs * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const float* A = g.A + (long)zb * g.sA;
  const float* Bp = g.B + (long)zb * g.sB;
  const bool ones = g.Ne > g.N;

  typedef Stage<BF, TA, BM, false> SA;
  typedef Stage<BF, !TB, BN, true> SB;
  SA sa[PF];
  SB sb[PF];
  constexpr int NC = BF ? 1 : 2;
  f32x4 acc[NC][MT][NT];
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[c][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // PF = register sets of staged tiles: PF = 2 keeps two k-tiles of global loads in flight behind
  // the MFMAs of the current one (for the bandwidth-bound shapes), PF = 1 one.
  const int nk = kend > kbeg ? (kend - kbeg + KT - 1) / KT : 0;
  if (nk > 0) {
#pragma unroll
    for (int p = 0; p < PF; ++p)
      if (p < nk) {
        sa[p].load(A, g.lda, g.M, m0, kbeg + p * KT, kend, false, va, tid);
        sb[p].load(Bp, g.ldb, g.N, n0, kbeg + p * KT, kend, ones, vb, tid);
      }
    sa[0].store(smem, tid);
    sb[0].store(smem + BM * ROWB, tid);
    __syncthreads();
    for (int t = 0; t < nk; ++t) {
      char* cur = smem + (t & 1) * STAGE;
      char* nxt = smem + ((t & 1) ^ 1) * STAGE;
      if (PF == 1) {
        if (t + 1 < nk) {
          sa[0].load(A, g.lda, g.M, m0, kbeg + (t + 1) * KT, kend, false, va, tid);
          sb[0].load(Bp, g.ldb, g.N, n0, kbeg + (t + 1) * KT, kend, ones, vb, tid);
        }
        mma_ktile<BF, MT, NT, SA, SB, NC>(cur, cur + BM * ROWB, wm * (BM / 2), wn * (BN / 2), lane, acc);
        if (t + 1 < nk) {
          sa[0].store(nxt, tid);
          sb[0].store(nxt + BM * ROWB, tid);
        }
      } else {
        // tile t+1 sits in set (t+1)&1 (issued one iteration ago), tile t+2 goes into set t&1,
        // whose tile t reached LDS in the previous iteration
        if (t + 2 < nk) {
          const int k2 = kbeg + (t + 2) * KT;
          if (t & 1) {
            sa[1 % PF].load(A, g.lda, g.M, m0, k2, kend, false, va, tid);
            sb[1 % PF].load(Bp, g.ldb, g.N, n0, k2, kend, ones, vb, tid);
          } else {
            sa[0].load(A, g.lda, g.M, m0, k2, kend, false, va, tid);
            sb[0].load(Bp, g.ldb, g.N, n0, k2, kend, ones, vb, tid);
          }
        }
        mma_ktile<BF, MT, NT, SA, SB, NC>(cur, cur + BM * ROWB, wm * (BM / 2), wn * (BN / 2), lane, acc);
        if (t + 1 < nk) {
          if (t & 1) {
            sa[0].store(nxt, tid);
            sb[0].store(nxt + BM * ROWB, tid);
          } else {
            sa[1 % PF].store(nxt, tid);
            sb[1 % PF].store(nxt + BM * ROWB, tid);
          }
        }
      }
      __syncthreads();
    }
  }

  // C/D map of the 16x16 MFMAs: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * (BM / 2) + mi * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * (BN / 2) + ni * 16 + (lane & 15);
        float v = acc[0][mi][ni][r];
#pragma unroll
        for (int c = 1; c < NC; ++c) v += acc[c][mi][ni][r];
        if (m < g.M && n < g.Ne) {
          if (g.nsplit > 1) g.part[((long)z * g.M + m) * g.Ne + n] = v;
          else store_out(g, zb, m, n, v);
        }
      }
  if (g.nsplit == 1 || !g.cnt) return;

  // In-launch split-K combine (cdna_hip_programming.md, "In-launch split-K reduction"), as in the
  // fp32 kernel above; the "last arriver" flag travels through the (now idle) staging LDS.
  int* last = reinterpret_cast<int*>(smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int tile = (zb * tm + ym) * tn + xn;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned tk = __hip_atomic_fetch_add(&g.cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last = (tk == (unsigned)(g.nsplit - 1));
  }
  __syncthreads();
  if (!*last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const long slab = (long)g.M * g.Ne;
  const float* pz = g.part + (long)zb * g.nsplit * slab;
  for (int e = tid; e < BM * BN; e += 256) {
    const int m = m0 + e / BN, n = n0 + e % BN;
    if (m >= g.M || n >= g.Ne) continue;
    store_out(g, zb, m, n, slab_sum(pz + (long)m * g.Ne + n, slab, g.nsplit, G));
  }
  if (tid == 0) __hip_atomic_store(&g.cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Separate split-K combine for large slab volumes: a block covers 256/G lanes x 4 consecutive output
// elements (row-major over [batch][M][Ne], so rows wrap) x G z-groups (z = g, g+G, ...); the G
// partial sums meet in LDS and are added in slab_sum's order (bit-identical to the in-launch path).
// block `blk` of the reduce over nelem = batch * M * Ne elements
__device__ __forceinline__ void reduce4_block(const GemmArgs& g, long nelem, int G, long blk, float* sh) {
  const int lanes = 256 / G;
  const int lane = threadIdx.x % lanes, zg = threadIdx.x / lanes;
  const int per_block = 4 * lanes;
  const int e0 = (int)(blk * per_block) + 4 * lane;   // nelem < 2^31 (host check)
  const int slab = g.M * g.Ne;
  const long zs = slab;
  // the 4 elements' slab columns first, then z outer / element inner: 4 x 8 independent loads in
  // flight per thread while each element's adds stay in ascending z
  const float* p[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = min(e0 + i, (int)nelem - 1);
    const int b = e / slab, w = e - b * slab;
    p[i] = g.part + (long)b * g.nsplit * zs + w;
  }
  float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
  for (int z = zg; z < g.nsplit; z += G) {
#pragma unroll
    for (int i = 0; i < 4; ++i) s[i] += p[i][z * zs];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) sh[zg * per_block + 4 * lane + i] = s[i];
  __syncthreads();
  for (int t = threadIdx.x; t < per_block; t += 256) {
    const long e = blk * per_block + t;
    if (e >= nelem) break;
    float v = sh[t];
    for (int q = 1; q < G; ++q) v += sh[q * per_block + t];
    const int b = (int)e / slab, w = (int)e - b * slab;
    store_out(g, b, w / g.Ne, w % g.Ne, v);
  }
}

__global__ __launch_bounds__(256) void splitk_reduce4(GemmArgs g, long nelem, int G) {
  __shared__ float sh[1024];
  reduce4_block(g, nelem, G, blockIdx.x, sh);
}

}  // namespace g2

// ------------------------------------------------------------------------------------------------
// gemm_pipe: the fp32 GEMM of the step's mid shapes (M 1600-5184, N 72-1296, K 128-3136; the 3x3
// convs, the fusion / non-local 1x1 convs and their data / weight gradients), k-pipelined.
//
// The k-major kernel above stages one k-tile in registers and waits for it behind ~1000 cycles of
// MFMAs per wave: these shapes run at 1-2 blocks per CU, so the L2 / Infinity-Cache latency of every
// k-tile is exposed (the largest conv at 0.30 of the fp32 peak, MFMA busy 0.155).  Here the
// operand tiles go HBM/L2 -> LDS by LDS-DMA (buffer_load ... lds, 16 B per lane: no VGPRs, no
// ds_write pass), into a ring of NS stages, so NS - 1 k-tiles of loads are in flight behind the MFMAs;
// one raw s_barrier per k-tile with a COUNTED vmcnt wait (the stage being read has landed, the later
// ones stay in flight).  The buffer descriptors' range checks zero-fill everything past the operand
// (rows >= M / N, k >= K) and a per-lane out-of-range offset masks k past a split-K slice.
//
// LDS images (the same layouts and fragment reads as g2::Stage, fp32):
//  * K-contiguous operand ([row][k]: A of C = A W^T, W of a 1x1 conv): 128-B rows, chunk c of row r at
//    slot c ^ ((r >> 1) & 7); one DMA wave-instruction fills 8 rows (lane -> row lane>>3, slot lane&7,
//    the source address pre-swizzled);
//  * row-contiguous operand ([k][row]: dY / X of a weight gradient, W of a data gradient): ROWS floats
//    per k-row, 16-column blocks XOR-swizzled by (k >> 2) & 1; one DMA wave-instruction fills
//    256 / ROWS k-rows.
// Wave tile (BM/2) x (BN/2) of 16x16 v_mfma_f32_16x16x4_f32 tiles (2 x 2 waves), one accumulator chain
// per output tile; MT * NT >= 4 independent chains keep the 32-cycle issue rate.
namespace gp {

// bf16 operands (config 2) over the same fp32 stage: a lane's two fp32 fragments of the k-tile (sub-steps
// 0 and 1, k = 4g + j and 16 + 4g + j) rounded RNE to bf16 (v_cvt_pk_bf16_f32, g2's staging rounding) and
// fed to ONE v_mfma_f32_16x16x32_bf16 per output tile -- the MFMA's k order is a permutation applied to
// both operands alike, so the products are the k-tile's.  Same LDS reads as the fp32 path, 1/8 of the MFMAs.
template <int MT, int NT, class SA, class SB>
__device__ __forceinline__ void mma_ktile_bf(const char* As, const char* Bs, int arow, int brow, int lane,
                                             f32x4 (&acc)[MT][NT]) {
  uint4 a[MT], b[NT];
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) {
    const uint4 f0 = SA::frag(As, arow + 16 * mi, 0, lane), f1 = SA::frag(As, arow + 16 * mi, 1, lane);
    a[mi] = uint4{g2::pk_bf16(__uint_as_float(f0.x), __uint_as_float(f0.y)),
                  g2::pk_bf16(__uint_as_float(f0.z), __uint_as_float(f0.w)),
                  g2::pk_bf16(__uint_as_float(f1.x), __uint_as_float(f1.y)),
                  g2::pk_bf16(__uint_as_float(f1.z), __uint_as_float(f1.w))};
  }
#pragma unroll
  for (int ni = 0; ni < NT; ++ni) {
    const uint4 f0 = SB::frag(Bs, brow + 16 * ni, 0, lane), f1 = SB::frag(Bs, brow + 16 * ni, 1, lane);
    b[ni] = uint4{g2::pk_bf16(__uint_as_float(f0.x), __uint_as_float(f0.y)),
                  g2::pk_bf16(__uint_as_float(f0.z), __uint_as_float(f0.w)),
                  g2::pk_bf16(__uint_as_float(f1.x), __uint_as_float(f1.y)),
                  g2::pk_bf16(__uint_as_float(f1.z), __uint_as_float(f1.w))};
  }
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
      acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(g2::bf16x8, a[mi]),
                                                            __builtin_bit_cast(g2::bf16x8, b[ni]), acc[mi][ni], 0, 0, 0);
}

// The block's output tile: (xn, ym) of K slice zs / batch zb, tn x tm tiles per slice (the arrival
// counter's index of the in-launch combine, g.cnt; null = slabs for a separate reduce).  `smem` is the
// block's LDS ring (ring_bytes), shared by the single-problem and the grouped kernel.
//
// KS = 2 (fp32): twice the waves, the k-split pair of each wave tile sharing the ring -- wave half kh runs
// sub-step kh of every k-tile (g2::mma_substep), so each SIMD holds two waves whose LDS waits and DMA
// issue overlap the other's MFMAs (one wave per SIMD left the 16x16x4 issue idle ~half the time on a
// one-block-per-CU grid); the halves' accumulators are g2's NC = 2 partials, summed acc0 + acc1 through
// the idle ring before the epilogue, which the kh = 0 waves run.
//
// KM = 2 (round 6): each ring stage holds two consecutive 32-wide k-tiles (two A and two B images), so the block
// runs one DMA wait + barrier per 64 of K instead of per 32 -- the per-k-tile overhead, not the MFMAs, sets the
// time of the step's latency-bound shapes (more so with bf16 MFMAs, 1/8 of the fp32 count).  Same MFMAs in the
// same order: bit-identical to KM = 1.
template <int BM, int BN, int WM, int WN, bool TA, bool TB, int NS, bool BF = false, int KS = 1, int KM = 1>
__device__ __forceinline__ void pipe_tile(const GemmArgs& g, int zb, int zs, int xn, int ym, int tn, int tm, int G,
                                          char* smem) {
  constexpr int NWT = WM * WN;                  // waves per k-split half
  constexpr int NW = NWT * KS, NTH = 64 * NW;   // all waves (they share the DMA of a stage)
  constexpr int WTM = BM / WM, WTN = BN / WN;   // wave tile
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int SA_B = BM * 128, SUB = (BM + BN) * 128, STAGE = KM * SUB;
  constexpr int LOADS = KM * (BM / 8 + BN / 8) / NW;   // DMA wave-instructions per wave and stage
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  static_assert(KM == 1 || (KM == 2 && KS == 1), "two k-tiles per stage: without k-split waves");
  static_assert(KS == 1 || (KS == 2 && !BF), "k-split waves: fp32 only");
  static_assert(KS == 1 || NWT * MT * NT * 4 * 64 * 4 <= ring_bytes<BM, BN, NS>(), "partials fit the ring");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kh = wave / NWT, wt = wave % NWT;
  const int wm = wt / WN, wn = wt % WN;
  const bool out_wave = kh == 0;
  const int z = zb * g.nsplit + zs;
  const int m0 = ym * BM, n0 = xn * BN;
  const int kbeg = zs * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const bool ones = g.Ne > g.N;
  // operand descriptors (wave-uniform): the batch's whole operand, so the range check covers its edges
  const unsigned a_bytes = (unsigned)((TA ? (long)g.K * g.lda : (long)g.M * g.lda) * 4);
  const unsigned b_bytes = (unsigned)((TB ? (long)g.N * g.ldb : (long)g.K * g.ldb) * 4);
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.A + (long)zb * g.sA), (short)0,
                                                    (int)a_bytes, 0x00020000);
  const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.B + (long)zb * g.sB), (short)0,
                                                    (int)b_bytes, 0x00020000);
  typedef g2::Stage<false, TA, BM, false> SA;
  typedef g2::Stage<false, !TB, BN, true> SB;
  f32x4 acc[1][MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[0][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (kend - kbeg + KM * KT - 1) / (KM * KT) : 0;   // stages
  auto issue = [&](int t) {
#pragma unroll
    for (int u = 0; u < KM; ++u) {
      char* st = smem + (t % NS) * STAGE + u * SUB;
      const int k0 = kbeg + (t * KM + u) * KT;
      fill<TA, BM, NW>(ra, st, m0, k0, kend, g.lda, wave, lane);
      fill<!TB, BN, NW>(rb, st + SA_B, n0, k0, kend, g.ldb, wave, lane);
    }
  };
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) issue(p);
  // the implicit ones column of op(B) (bias gradient, B row-contiguous only): column N of the tile
  const int ones_col = (ones && g.N >= n0 && g.N < n0 + BN) ? g.N - n0 : -1;
  for (int t = 0; t < nk; ++t) {
    // stage t has landed once at most the later stages' DMAs are outstanding
    const int later = min(NS - 2, nk - 1 - t);
    if (NS >= 4 && later >= 2) vm_wait<2 * LOADS>();
    else if (NS >= 3 && later >= 1) vm_wait<LOADS>();
    else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of the slot refilled below
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");                          // no LDS read moves above the barrier
    if (t + NS - 1 < nk) issue(t + NS - 1);
    if (ones_col >= 0) {
      if (tid < KM * KT) {
        const int u = tid / KT, kk = tid - u * KT;
        const int k = kbeg + (t * KM + u) * KT + kk;
        char* img = smem + (t % NS) * STAGE + u * SUB + SA_B;
        *reinterpret_cast<float*>(img + SB::rc_off(kk, ones_col)) = k < kend ? 1.f : 0.f;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
#pragma unroll
    for (int u = 0; u < KM; ++u) {
      if (KM > 1 && kbeg + (t * KM + u) * KT >= kend) break;   // a ragged last stage (uniform)
      const char* cur = smem + (t % NS) * STAGE + u * SUB;
      if constexpr (BF) mma_ktile_bf<MT, NT, SA, SB>(cur, cur + SA_B, wm * WTM, wn * WTN, lane, acc[0]);
      else if constexpr (KS == 2) g2::mma_substep<MT, NT, SA, SB>(cur, cur + SA_B, wm * WTM, wn * WTN, lane, kh, acc[0]);
      else g2::mma_ktile<false, MT, NT, SA, SB, 1>(cur, cur + SA_B, wm * WTM, wn * WTN, lane, acc);
    }
  }
  if constexpr (KS == 2) {   // acc = sub-step-0 partial + sub-step-1 partial (g2's NC = 2 order)
    float* xch = reinterpret_cast<float*>(smem);   // [NWT][MT][NT][4][64]
    __syncthreads();                               // every wave past its last ring read
    if (kh == 1)
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r) xch[(((wt * MT + mi) * NT + ni) * 4 + r) * 64 + lane] = acc[0][mi][ni][r];
    __syncthreads();
    if (kh == 0)
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[0][mi][ni][r] = acc[0][mi][ni][r] + xch[(((wt * MT + mi) * NT + ni) * 4 + r) * 64 + lane];
  }

  // C/D map of the 16x16 MFMAs: col = lane & 15, row = (lane >> 4) * 4 + r
  if (g.colstats) {   // the output's BatchNorm statistics partials (single slice: the values are final)
    double cs[NT][2];
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) {
      const int n = n0 + wn * WTN + ni * 16 + (lane & 15);
      const double k = n < g.N ? (double)g.shift[n] : 0.0;
      double s1 = 0.0, s2 = 0.0;
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + r;
          if (out_wave && m < g.M && n < g.N) {
            float* cp = g.C + (long)m * g.ldc + n;
            const float v = epilogue(g.epi, acc[0][mi][ni][r], cp, m, n);
            *cp = v;
            const double d = (double)v - k;
            s1 += d;
            s2 += d * d;
          }
        }
      // the 4 row groups of the wave (lanes c, c + 16, c + 32, c + 48), pairwise in a fixed order
      s1 += __shfl_xor(s1, 16, 64);
      s2 += __shfl_xor(s2, 16, 64);
      s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      cs[ni][0] = s1;
      cs[ni][1] = s2;
    }
    // the WM row waves of the tile: through the idle LDS ring (all waves are past their last k-tile reads)
    double* red = reinterpret_cast<double*>(smem);   // [2][WM][BN]
    __syncthreads();
    if (out_wave && lane < 16)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
#pragma unroll
        for (int j = 0; j < 2; ++j) red[(j * WM + wm) * BN + wn * WTN + ni * 16 + lane] = cs[ni][j];
    __syncthreads();
    for (int t = tid; t < 2 * BN; t += NTH) {
      const int j = t / BN, cl = t - j * BN, n = n0 + cl;
      if (n >= g.N) continue;
      double v = red[(j * WM) * BN + cl];
#pragma unroll
      for (int w2 = 1; w2 < WM; ++w2) v += red[(j * WM + w2) * BN + cl];
      g.colstats[(long)ym * 2 * g.N + (long)j * g.N + n] = v;
    }
    return;
  }
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * WTN + ni * 16 + (lane & 15);
        if (out_wave && m < g.M && n < g.Ne) {
          if (g.nsplit > 1) g.part[((long)z * g.M + m) * g.Ne + n] = acc[0][mi][ni][r];
          else store_out(g, zb, m, n, acc[0][mi][ni][r]);
        }
      }
  if (g.nsplit == 1 || !g.cnt) return;
  // in-launch split-K combine (as g2::gemm_mfma; flag through the idle ring)
  int* last = reinterpret_cast<int*>(smem);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int tile = (zb * tm + ym) * tn + xn;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned tk = __hip_atomic_fetch_add(&g.cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *last = (tk == (unsigned)(g.nsplit - 1));
  }
  __syncthreads();
  if (!*last) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  const long slab = (long)g.M * g.Ne;
  const float* pz = g.part + (long)zb * g.nsplit * slab;
  for (int e = tid; e < BM * BN; e += NTH) {
    const int m = m0 + e / BN, n = n0 + e % BN;
    if (m >= g.M || n >= g.Ne) continue;
    store_out(g, zb, m, n, g2::slab_sum(pz + (long)m * g.Ne + n, slab, g.nsplit, G));
  }
  if (tid == 0) __hip_atomic_store(&g.cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int BM, int BN, int WM, int WN, bool TA, bool TB, int NS, bool BF = false, int KS = 1, int KM = 1>
__global__ __launch_bounds__(64 * WM * WN * KS) void gemm_pipe(GemmArgs g, int tn, int tm, unsigned total, int G,
                                                                int zfast) {
  __shared__ __attribute__((aligned(1024))) char smem[ring_bytes<BM, BN, NS, KM>()];
  int zs, xn, ym, zb;
  tile_coords(xcd_linear(blockIdx.x, total), g.nsplit, tn, tm, zfast, zs, xn, ym, zb);
  pipe_tile<BM, BN, WM, WN, TA, TB, NS, BF, KS, KM>(g, zb, zs, xn, ym, tn, tm, G, smem);
}

// Grouped launch: up to GROUP_MAX independent problems (any of the four layouts, a runtime switch) in one
// grid; problem p owns the logical blocks [start[p], start[p + 1]) of the XCD-ordered grid (slices of a
// tile fastest); no in-launch combine (the group's split-K slabs go to one grouped reduce).
struct PipeGroup {
  int n;
  int start[GROUP_MAX + 1];
  int tn[GROUP_MAX], tm[GROUP_MAX], variant[GROUP_MAX];   // variant = 4 BF + 2 TA + TB
  GemmArgs g[GROUP_MAX];
};

// KS = 2: fp32 problems only (the host launches a group holding a bf16 problem with KS = 1).
template <int BM, int BN, int WM, int WN, int NS, int KS = 1, int KM = 1>
__global__ __launch_bounds__(64 * WM * WN * KS) void gemm_pipe_group(PipeGroup P, unsigned total) {
  __shared__ __attribute__((aligned(1024))) char smem[ring_bytes<BM, BN, NS, KM>()];
  const unsigned lin = xcd_linear(blockIdx.x, total);
  int p = 0;
#pragma unroll
  for (int k = 1; k < GROUP_MAX; ++k)
    if (k < P.n && (int)lin >= P.start[k]) p = k;
  // the selected problem's descriptor by constant indices only (scalar loads from the argument segment)
  GemmArgs g = P.g[0];
  int tn = P.tn[0], tm = P.tm[0], variant = P.variant[0], start = P.start[0];
#pragma unroll
  for (int k = 1; k < GROUP_MAX; ++k)
    if (k == p) {
      g = P.g[k];
      tn = P.tn[k];
      tm = P.tm[k];
      variant = P.variant[k];
      start = P.start[k];
    }
  int zs, xn, ym, zb;
  tile_coords(lin - (unsigned)start, g.nsplit, tn, tm, 1, zs, xn, ym, zb);
  switch (variant) {   // 4 BF + 2 TA + TB
    case 0: pipe_tile<BM, BN, WM, WN, false, false, NS, false, KS, KM>(g, zb, zs, xn, ym, tn, tm, 1, smem); break;
    case 1: pipe_tile<BM, BN, WM, WN, false, true, NS, false, KS, KM>(g, zb, zs, xn, ym, tn, tm, 1, smem); break;
    case 2: pipe_tile<BM, BN, WM, WN, true, false, NS, false, KS, KM>(g, zb, zs, xn, ym, tn, tm, 1, smem); break;
    case 3: pipe_tile<BM, BN, WM, WN, true, true, NS, false, KS, KM>(g, zb, zs, xn, ym, tn, tm, 1, smem); break;
    default:
      if constexpr (KS == 1) {
        switch (variant) {
          case 4: pipe_tile<BM, BN, WM, WN, false, false, NS, true, 1, KM>(g, zb, zs, xn, ym, tn, tm, 1, smem); break;
          case 5: pipe_tile<BM, BN, WM, WN, false, true, NS, true, 1, KM>(g, zb, zs, xn, ym, tn, tm, 1, smem); break;
          case 6: pipe_tile<BM, BN, WM, WN, true, false, NS, true, 1, KM>(g, zb, zs, xn, ym, tn, tm, 1, smem); break;
          default: pipe_tile<BM, BN, WM, WN, true, true, NS, true, 1, KM>(g, zb, zs, xn, ym, tn, tm, 1, smem); break;
        }
      }
      break;
  }
}

// Grouped split-K reduce: g2::splitk_reduce4's blocks (G z-groups per element, combined in slab_sum's
// order) of up to RGROUP_MAX problems in one grid, so
// a GEMM gives the same bits grouped or alone
constexpr int RGROUP_MAX = 2 * GROUP_MAX;   // a group's k-major and pipelined problems
struct ReduceGroup {
  int n;
  int start[RGROUP_MAX + 1];
  int G[RGROUP_MAX];
  long nelem[RGROUP_MAX];
  GemmArgs g[RGROUP_MAX];
};

__global__ __launch_bounds__(256) void splitk_reduce_sum_group(ReduceGroup R) {
  __shared__ float sh[1024];
  const int b = blockIdx.x;
  int p = 0;
#pragma unroll
  for (int k = 1; k < RGROUP_MAX; ++k)
    if (k < R.n && b >= R.start[k]) p = k;
  GemmArgs g = R.g[0];
  int G = R.G[0], start = R.start[0];
  long nelem = R.nelem[0];
#pragma unroll
  for (int k = 1; k < RGROUP_MAX; ++k)
    if (k == p) {
      g = R.g[k];
      G = R.G[k];
      start = R.start[k];
      nelem = R.nelem[k];
    }
  g2::reduce4_block(g, nelem, G, b - start, sh);
}

}  // namespace gp


// C[b] = alpha * op(A[b]) * op(B[b]) + beta * C[b] (+ bias[n]) (+ addend[(m % add_mod), n]) (relu);
// bias_grad (optional): bias_grad[m] = alpha * sum_k op(A)(m,k) + beta * bias_grad[m]
// tuning override (vc_gemm_tune): 0 / -1 fields = automatic choice
struct G2Tune {
  int bm, bn, nsplit, pf, combine;
};
#ifdef VC_PROBE
static G2Tune g_tune = {0, 0, 0, 0, -1};
#else
static constexpr G2Tune g_tune = {0, 0, 0, 0, -1};   // the product library keeps no tuning state
#endif

VC_EXPORT int vc_gemm_tune(int bm, int bn, int nsplit, int pf, int combine) {
  VC_REQUIRE((bm == 0 || bm == 64 || bm == 128) && (bn == 0 || bn == 64 || bn == 128));
  VC_REQUIRE(nsplit >= 0 && nsplit <= 4096 && pf >= 0 && pf <= 2 && combine >= -1 && combine <= 1);
#ifdef VC_PROBE
  g_tune = G2Tune{bm, bn, nsplit, pf, combine};
#else
  // product library: only the automatic configuration (the forced ones exist in libvitcnn_probe.so)
  VC_REQUIRE(bm == 0 && bn == 0 && nsplit == 0 && pf == 0 && combine == -1);
#endif
  return VC_OK;
}

// largest per-tile slab volume (bytes) combined in-launch by the last-arriving slice (else a separate
// reduce kernel); knob SPLITK_COMBINE (probe library)
static long g2_combine_limit() { return vc_knob("VITCNN_SPLITK_COMBINE", 4096); }

// largest per-tile slab volume (bytes) the k-major kernel's last-arriving slice combines in-launch;
// knob LEGACY_COMBINE (probe library)
static long legacy_combine_limit() { return vc_knob("VITCNN_LEGACY_COMBINE", 4096); }

// the k-major fp32 kernel (LDS [k][row], 16x16x4 f32): launch configuration of one problem
struct LegacyPlan {
  GemmArgs g;
  int tn, tm, nz, variant;
  bool reduce;        // separate split-K reduce launch
  long ws_floats;     // split-K slab floats used
  int counters;       // arrival counters used (in-launch combine)
};

static LegacyPlan plan_legacy(int transA, int transB, int M, int N, int K, float alpha,
                              const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                              float beta, float* C, long ldc, long strideC, int batch,
                              const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                              float* bias_grad, float* ws, long ws_floats, unsigned int* tile_counters,
                              int n_counters) {
  Epi epi{alpha, beta, bias, addend, add_ld, add_mod > 0 ? add_mod : M, flags};
  const int Ne = N + (bias_grad ? 1 : 0);
  const int tn = vc_cdiv(Ne, BN), tm = vc_cdiv(M, BM);
  const long tiles = (long)tn * tm * batch;
  // Split K when the output grid leaves the chip short of ~3 blocks per CU (768 blocks): each
  // K slice keeps >= 128 of K (4 BK steps), the slabs must fit the workspace, and the slices are
  // summed in fixed order (slab_sum) so results do not depend on the split's scheduling.
  int nsplit = 1;
  constexpr long kTargetBlocks = 768;
  if (ws && K >= 256 && tiles < kTargetBlocks / 2) {
    const long want = (kTargetBlocks + tiles - 1) / tiles;
    const long maxk = K / 128;
    nsplit = (int)std::min<long>(std::min<long>(want, maxk), 256);
    while (nsplit > 1 && (long)nsplit * batch * M * Ne > ws_floats) --nsplit;
    if (nsplit < 1) nsplit = 1;
  }
  int k_chunk = K;
  if (nsplit > 1) {
    k_chunk = vc_cdiv(vc_cdiv(K, nsplit), BK) * BK;
    nsplit = vc_cdiv(K, k_chunk);
  }
  // the in-launch combine pays only while the last arriver's serial slab read stays small
  // (<= 4 KB of slabs per tile, measured: tools/gemm_census.py); wider splits keep the parallel
  // reduce kernel
  const long slab_bytes = (long)nsplit * std::min(BM, M) * std::min(BN, Ne) * 4;
  unsigned int* cnt = (nsplit > 1 && tile_counters && tiles <= n_counters && slab_bytes <= legacy_combine_limit())
                          ? tile_counters
                          : nullptr;
  LegacyPlan pl;
  pl.g = GemmArgs{M, N, K, Ne, k_chunk, nsplit, A, lda, strideA, B, ldb, strideB, C, ldc, strideC, bias_grad, ws, cnt,
                  epi};
  pl.tn = tn;
  pl.tm = tm;
  pl.nz = batch * nsplit;
  const bool va = ((uintptr_t)A % 16 == 0) && (lda % 4 == 0) && (batch == 1 || strideA % 4 == 0);
  const bool vb = ((uintptr_t)B % 16 == 0) && (ldb % 4 == 0) && (batch == 1 || strideB % 4 == 0);
  pl.variant = (transA ? 8 : 0) | (transB ? 4 : 0) | (va ? 2 : 0) | (vb ? 1 : 0);
  pl.reduce = nsplit > 1 && !cnt;
  pl.ws_floats = nsplit > 1 ? (long)nsplit * batch * M * Ne : 0;
  pl.counters = cnt ? (int)tiles : 0;
  return pl;
}

// register sets of staged k-tiles in the k-major kernel: 1.  Deeper sets (bit-identical results) measured
// slower on the whole step -- PD 1 / 2 / 3 / 4: 2.148 / 2.19 / 2.19 / 2.245 ms (round 3,
// tools/ab_env.sh, profiles/r03_ab_gemm_pd.log): the extra VGPRs cost more occupancy than the earlier
// loads save latency.  Knob GEMM_PD=2 (probe library) selects the two-set build for measurements.
static int legacy_pd() { return (int)std::max(1L, std::min(2L, vc_knob("VITCNN_GEMM_PD", 1))); }

template <int PD>
static int launch_plan_pd(const LegacyPlan& pl, hipStream_t stream) {
  const GemmArgs& g = pl.g;
  dim3 grid(pl.tn, pl.tm, pl.nz), block(256);
#define VC_L(V_, TA_, TB_, VA_, VB_) \
  case V_: hipLaunchKernelGGL((gemm_f32_mfma<TA_, TB_, VA_, VB_, PD>), grid, block, 0, stream, g); break;
  switch (pl.variant) {
    VC_L(0, false, false, false, false) VC_L(1, false, false, false, true)
    VC_L(2, false, false, true, false) VC_L(3, false, false, true, true)
    VC_L(4, false, true, false, false) VC_L(5, false, true, false, true)
    VC_L(6, false, true, true, false) VC_L(7, false, true, true, true)
    VC_L(8, true, false, false, false) VC_L(9, true, false, false, true)
    VC_L(10, true, false, true, false) VC_L(11, true, false, true, true)
    VC_L(12, true, true, false, false) VC_L(13, true, true, false, true)
    VC_L(14, true, true, true, false) VC_L(15, true, true, true, true)
    default: return VC_EINVAL;
  }
#undef VC_L
  VC_CHECK_LAUNCH();
  if (pl.reduce) {
    const long nelem = (long)(pl.nz / g.nsplit) * g.M * g.Ne;
    const int G = g2::slab_groups(g.nsplit);
    VC_REQUIRE(nelem < (1L << 31));
    hipLaunchKernelGGL(g2::splitk_reduce4, dim3(vc_cdiv(nelem, 1024 / G)), dim3(256), 0, stream, g, nelem, G);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

static int launch_plan(const LegacyPlan& pl, hipStream_t stream) {
  return legacy_pd() == 2 ? launch_plan_pd<2>(pl, stream) : launch_plan_pd<1>(pl, stream);
}

// ---- gemm_pipe launch configuration
// Can the pipelined kernel take this problem?  fp32, one batch, 16-B aligned operands with leading
// dimensions divisible by 4 and K % 4 == 0 (whole 16-B chunks along k), operands < 2 GB (32-bit buffer
// offsets), the bias-gradient ones column only on a row-contiguous B.
static bool pipe_fits(int transA, int transB, int M, int N, int K, const float* A, long lda, const float* B, long ldb,
                      int batch, const float* bias_grad) {
  if (batch != 1 || K % 4 || lda % 4 || ldb % 4 || ((uintptr_t)A % 16) || ((uintptr_t)B % 16)) return false;
  if (bias_grad && transB) return false;
  const long ab = (transA ? (long)K * lda : (long)M * lda) * 4, bb = (transB ? (long)N * ldb : (long)K * ldb) * 4;
  return ab < (1L << 31) && bb < (1L << 31);
}

// the shapes it pays on (tools/gemm_census.py, profiles/r04_gemm_census.log): enough work per launch that the
// pipeline fills, and (round 5) the small ones of the step with K <= 4096 and an output of >= 2048 elements --
// the NonLocal / hsi2 products of 1600 rows, 2-3 us faster each than on the k-major kernel; the long-K skinny
// weight gradients (K = 10 B L rows, M or N < 64) stay on the k-major kernel, which was faster there
static bool pipe_wanted(int M, int N, int K) {
  if (!vc_knob("VITCNN_GEMM_PIPE", 1)) return false;
  if ((long)M * N * K >= (1L << 24) && K >= 128 && M >= 128 && N >= 64) return true;
  return vc_knob("VITCNN_GEMM_PIPE_SMALL", 1) && K <= 4096 && M >= 16 && N >= 16 && (long)M * N >= 2048;
}

struct PipePlan {
  int bm, bn, ns, nsplit, k_chunk, tn, tm;
};

// bf16 64 x 64 tiles on 8 waves (2 x 4 of 32 x 16: two waves per SIMD, half the DMA pieces per wave) instead of 4
// (knob: probe library)
static int pipe_bf_w8() { return vc_knob("VITCNN_PIPE_BF_W8", 1) ? 1 : 0; }
// the same for fp32 tiles: equal or 1-5 % faster on every shape of the step, step 1.714 -> 1.690 ms
// (profiles/r05_gemm_f32_w8.log; knob: probe library)
static int pipe_f32_w8() { return vc_knob("VITCNN_PIPE_F32_W8", 1) ? 1 : 0; }
// k-tiles per ring stage of the 8-wave 64 x 64 kernels (pipe_tile KM; knob: probe library)
static int pipe_km() { return vc_knob("VITCNN_PIPE_KM", 1) == 2 ? 2 : 1; }

// k-split waves (gp::pipe_tile KS = 2) for fp32 64 x 64 tiles.  Rule 0: where the grid is at most one block per CU
// and K is long (the local 3x3 convs, M = B 49, K = 9 C: 34.1 -> 31.8 us; elsewhere equal or slower,
// profiles/r05_gemm_ks.log).  Superseded by the 8-wave 2 x 4 layout (pipe_f32_w8: 32.1 us on the local conv and
// faster elsewhere), so the default is 1 = never.  Knob (probe library): 0 = the rule, 1 = never, 2 = always.
static int pipe_ks(long tiles = 0, int nsplit = 1, int K = 0) {
  const int k = vc_knob("VITCNN_PIPE_KS", 1);
  if (k) return k == 2 ? 2 : 1;
  return (nsplit == 1 && tiles > 0 && tiles <= 256 && K >= 1024) ? 2 : 1;
}

// Launch plan (tools/gemm_lab.hip sweep over the step's 21 critical-path shapes, profiles/r04_gemm_lab.log):
// 64 x 64 tiles on 4 waves with a 2-stage ring (32 KB: up to 5 blocks per CU) won or tied on nearly every
// shape; a grid of >= 128 tiles runs unsplit (the split-K slab reduce costs more than the extra blocks
// gain), a smaller one splits K towards ~512 blocks in slices of >= 4 k-tiles (the weight gradients,
// K = 1600-5184 rows over a 2 x 5 ... 4 x 21 tile grid).
static PipePlan plan_pipe(int M, int Ne, int K, long ws_floats, bool have_ws, bool bf = false) {
  PipePlan p;
  p.bm = 64;
  p.bn = 64;
  p.ns = vc_knob("VITCNN_PIPE_NS", 2) == 4 ? 4 : 2;   // ring depth (knob: probe library)
  if (g_tune.bm) p.bm = g_tune.bm;
  if (g_tune.bn) p.bn = g_tune.bn;
  if (bf && p.bm == 128 && p.bn == 128) p.bn = 64;   // (no 128 x 128 build)
  p.tn = vc_cdiv(Ne, p.bn);
  p.tm = vc_cdiv(M, p.bm);
  const long tiles = (long)p.tn * p.tm;
  const int kt = vc_cdiv(K, gp::KT);
  int nsplit = 1;
  const long target = vc_knob("VITCNN_PIPE_SPLIT_BLOCKS", 512);   // blocks a split aims at (knob: probe library)
  if (have_ws && tiles < vc_knob("VITCNN_PIPE_SPLIT_BELOW", 128)) {   // (knob: probe library)
    const int cap = (int)std::max<long>(1, std::min<long>(kt / 4, 64));
    const int n0 = (int)std::max<long>(1, std::min<long>((target + tiles - 1) / tiles, cap));
    nsplit = n0;
    // round 6: of the splits n0 .. 2 n0, the one whose grid fills whole rounds of the 256 CUs best (the slices
    // after rounding to k-tiles; ties: fewer slabs), e.g. 84 tiles: 9 slices = 756 blocks, not 7 = 588 (ViT-CNN
    // step -0.011 ms median of 6).  Only for modest splits (n0 <= 16, grids of >= 32 tiles): the deep splits of
    // tiny grids (S2EFT's weight gradients, K = 9344) lost ~1 % with more slabs (profiles/r06_ab_split_fill.log)
    if (vc_knob("VITCNN_PIPE_SPLIT_FILL", 1) && n0 <= 16) {
      constexpr long NCU = 256;
      double best = -1.0;
      for (int n = n0; n <= std::min(2 * n0, cap); ++n) {
        const int kc = vc_cdiv(vc_cdiv(K, n), gp::KT) * gp::KT;
        const long blocks = tiles * vc_cdiv(K, kc);
        const double fill = (double)blocks / (double)(vc_cdiv(blocks, NCU) * NCU);
        if (fill > best + 1e-9) {
          best = fill;
          nsplit = n;
        }
      }
    }
  }
  if (g_tune.nsplit) nsplit = std::min(g_tune.nsplit, std::max(1, kt));
  while (nsplit > 1 && (long)nsplit * M * Ne > ws_floats) --nsplit;
  p.k_chunk = kt * gp::KT;
  if (nsplit > 1) {
    p.k_chunk = vc_cdiv(vc_cdiv(K, nsplit), gp::KT) * gp::KT;
    nsplit = vc_cdiv(K, p.k_chunk);
  }
  p.nsplit = nsplit;
  return p;
}

static int launch_pipe(int transA, int transB, int M, int N, int K, float alpha, const float* A, long lda,
                       const float* B, long ldb, float beta, float* C, long ldc, const float* bias,
                       const float* addend, long add_ld, int add_mod, int flags, float* bias_grad, float* ws,
                       long ws_floats, unsigned int* tile_counters, int n_counters, hipStream_t stream) {
  Epi epi{alpha, beta, bias, addend, add_ld, add_mod > 0 ? add_mod : M, flags};
  const int Ne = N + (bias_grad ? 1 : 0);
  const bool bf = (flags & F_BF16) != 0;
  const PipePlan p = plan_pipe(M, Ne, K, ws_floats, ws != nullptr, bf);
  const long tiles = (long)p.tn * p.tm;
  const long slab_bytes = (long)p.nsplit * std::min(p.bm, M) * std::min(p.bn, Ne) * 4;
  bool inl = slab_bytes <= g2_combine_limit();
  if (g_tune.combine >= 0) inl = g_tune.combine == 1;
  unsigned int* cnt = (p.nsplit > 1 && tile_counters && tiles <= n_counters && inl) ? tile_counters : nullptr;
  GemmArgs g{M, N, K, Ne, p.k_chunk, p.nsplit, A, lda, 0, B, ldb, 0, C, ldc, 0, bias_grad, ws, cnt, epi};
  const long total = tiles * p.nsplit;
  VC_REQUIRE(total < (1L << 31));
  const int G = g2::slab_groups(p.nsplit);
  // split slice fastest in the block order: a tile's K slices run side by side on one XCD (measured
  // faster for every split shape of the step, tools/gemm_lab.hip; the in-launch combine reads its slabs there)
  const int zfast = 1;
  dim3 grid((unsigned)total);
#define VC_GP(BM_, BN_, WM_, WN_, NS_, KS_, KM_)                                                                \
  do {                                                                                                           \
    const dim3 blk(64 * WM_ * WN_ * KS_);                                                                        \
    if (transA && transB)                                                                                        \
      hipLaunchKernelGGL((gp::gemm_pipe<BM_, BN_, WM_, WN_, true, true, NS_, false, KS_, KM_>), grid, blk, 0, stream, g, p.tn, p.tm, (unsigned)total, G, zfast);   \
    else if (transA)                                                                                             \
      hipLaunchKernelGGL((gp::gemm_pipe<BM_, BN_, WM_, WN_, true, false, NS_, false, KS_, KM_>), grid, blk, 0, stream, g, p.tn, p.tm, (unsigned)total, G, zfast);  \
    else if (transB)                                                                                             \
      hipLaunchKernelGGL((gp::gemm_pipe<BM_, BN_, WM_, WN_, false, true, NS_, false, KS_, KM_>), grid, blk, 0, stream, g, p.tn, p.tm, (unsigned)total, G, zfast);  \
    else                                                                                                         \
      hipLaunchKernelGGL((gp::gemm_pipe<BM_, BN_, WM_, WN_, false, false, NS_, false, KS_, KM_>), grid, blk, 0, stream, g, p.tn, p.tm, (unsigned)total, G, zfast); \
  } while (0)
#define VC_GP_T(NS_)                                                \
  do {                                                              \
    if (p.bm == 128 && p.bn == 64) VC_GP(128, 64, 4, 2, NS_, 1, 1);     \
    else if (p.bm == 64 && p.bn == 128) VC_GP(64, 128, 2, 4, NS_, 1, 1); \
    else if (pipe_ks(tiles, p.nsplit, K) == 2) VC_GP(64, 64, 2, 2, NS_, 2, 1); \
    else if (pipe_f32_w8() && km == 2) VC_GP(64, 64, 2, 4, NS_, 1, 2);  \
    else if (pipe_f32_w8()) VC_GP(64, 64, 2, 4, NS_, 1, 1);            \
    else VC_GP(64, 64, 2, 2, NS_, 1, 1);                               \
  } while (0)
#define VC_GPB(BM_, BN_, WM_, WN_, TA_, TB_, NS_, KM_) \
  hipLaunchKernelGGL((gp::gemm_pipe<BM_, BN_, WM_, WN_, TA_, TB_, NS_, true, 1, KM_>), grid, dim3(64 * WM_ * WN_), 0, stream, g, p.tn, p.tm, (unsigned)total, G, zfast)
#define VC_GPB_L(BM_, BN_, WM_, WN_, NS_, KM_)                          \
  do {                                                                  \
    if (transA && transB) VC_GPB(BM_, BN_, WM_, WN_, true, true, NS_, KM_); \
    else if (transA) VC_GPB(BM_, BN_, WM_, WN_, true, false, NS_, KM_);     \
    else if (transB) VC_GPB(BM_, BN_, WM_, WN_, false, true, NS_, KM_);     \
    else VC_GPB(BM_, BN_, WM_, WN_, false, false, NS_, KM_);                \
  } while (0)
  const int km = pipe_km();
  if (bf) {   // tiles other than 64 x 64 / 2 stages: measurement knobs (probe library)
    if (p.bm == 128 && p.bn == 64) VC_GPB_L(128, 64, 4, 2, 2, 1);
    else if (p.bm == 64 && p.bn == 128) VC_GPB_L(64, 128, 2, 4, 2, 1);
    else if (p.ns == 4) VC_GPB_L(64, 64, 2, 2, 4, 1);
    else if (pipe_bf_w8() && km == 2) VC_GPB_L(64, 64, 2, 4, 2, 2);
    else if (pipe_bf_w8()) VC_GPB_L(64, 64, 2, 4, 2, 1);
    else VC_GPB_L(64, 64, 2, 2, 2, 1);
  } else if (p.ns == 4) VC_GP_T(4);
  else VC_GP_T(2);
#undef VC_GPB_L
#undef VC_GPB
#undef VC_GP_T
#undef VC_GP
  VC_CHECK_LAUNCH();
  if (p.nsplit > 1 && !cnt) {
    const long nelem = (long)M * Ne;
    VC_REQUIRE(nelem < (1L << 31));
    hipLaunchKernelGGL(g2::splitk_reduce4, dim3(vc_cdiv(nelem, 1024 / G)), dim3(256), 0, stream, g, nelem, G);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

// ---- grouped launches: the problems added to a group (vc_gemm_group_add) launch at vc_gemm_group_end as
// one gemm_f32_group grid (the k-major problems), one gemm_pipe_group grid (the pipelined ones) and ONE
// grouped split-K reduce over both (each problem's slabs summed in the order its ungrouped launch uses, so
// a GEMM gives the same bits grouped or alone); each problem takes its own slice of the workspace and of
// the arrival counters.  The group state lives in caller-owned host memory (VC_GEMM_GROUP_BYTES), so the
// library keeps none and distinct groups are independent.
struct PipeRec {
  GemmArgs g;
  int tn, tm, variant;   // variant = 2 transA + transB
};

struct GroupState {
  unsigned magic;          // GROUP_MAGIC between begin and end
  hipStream_t stream;
  int n, np;
  LegacyPlan plans[GROUP_MAX];
  PipeRec pipes[GROUP_MAX];
  long ws_used;
  int cnt_used;
  int err;
};
constexpr unsigned GROUP_MAGIC = 0x56434747u;   // "VCGG"
static_assert(sizeof(GroupState) <= VC_GEMM_GROUP_BYTES, "VC_GEMM_GROUP_BYTES too small");

struct ReduceItems {
  gp::ReduceGroup R;
  long total = 0;
  void add(const GemmArgs& g, int G, int batch) {
    R.start[R.n] = (int)total;
    R.g[R.n] = g;
    R.G[R.n] = G;
    R.nelem[R.n] = (long)batch * g.M * g.Ne;
    ++R.n;
    total += (R.nelem[R.n - 1] + 1024 / G - 1) / (1024 / G);
  }
};

static int group_flush(GroupState& st) {
  const int n = st.n, np = st.np;
  st.n = st.np = 0;
  st.ws_used = 0;
  st.cnt_used = 0;
  if (n + np == 0) return VC_OK;
  if (n == 1 && np == 0) return launch_plan(st.plans[0], st.stream);
  ReduceItems red;
  red.R.n = 0;
  if (n == 1) {
    // one k-major problem: its own launch, its reduce (if any) joins the grouped one
    LegacyPlan pl = st.plans[0];
    const bool reduce = pl.reduce;
    pl.reduce = false;
    const int rc = launch_plan(pl, st.stream);
    if (rc) return rc;
    if (reduce) red.add(pl.g, g2::slab_groups(pl.g.nsplit), pl.nz / pl.g.nsplit);
  } else if (n > 1) {
    GemmGroup G;
    G.n = n;
    long total = 0;
    for (int p = 0; p < n; ++p) {
      const LegacyPlan& pl = st.plans[p];
      G.start[p] = (int)total;
      G.tn[p] = pl.tn;
      G.tm[p] = pl.tm;
      G.variant[p] = pl.variant;
      G.g[p] = pl.g;
      total += (long)pl.tn * pl.tm * pl.nz;
      if (pl.reduce) red.add(pl.g, g2::slab_groups(pl.g.nsplit), pl.nz / pl.g.nsplit);
    }
    G.start[n] = (int)total;
    VC_REQUIRE(total < (1L << 31));
    if (legacy_pd() == 2) hipLaunchKernelGGL(gemm_f32_group<2>, dim3((unsigned)total), dim3(256), 0, st.stream, G);
    else hipLaunchKernelGGL(gemm_f32_group<1>, dim3((unsigned)total), dim3(256), 0, st.stream, G);
    VC_CHECK_LAUNCH();
  }
  if (np > 0) {
    gp::PipeGroup P;
    P.n = np;
    long total = 0;
    for (int p = 0; p < np; ++p) {
      const PipeRec& pr = st.pipes[p];
      P.start[p] = (int)total;
      P.tn[p] = pr.tn;
      P.tm[p] = pr.tm;
      P.variant[p] = pr.variant;
      P.g[p] = pr.g;
      total += (long)pr.tn * pr.tm * pr.g.nsplit;
      if (pr.g.nsplit > 1) red.add(pr.g, g2::slab_groups(pr.g.nsplit), 1);
    }
    P.start[np] = (int)total;
    VC_REQUIRE(total < (1L << 31));
    bool any_bf = false;
    for (int p = 0; p < np; ++p) any_bf |= st.pipes[p].variant >= 4;
    if (!any_bf && vc_knob("VITCNN_PIPE_KS", 0) == 2)   // (grouped problems: measured no gain)
      hipLaunchKernelGGL((gp::gemm_pipe_group<64, 64, 2, 2, 2, 2>), dim3((unsigned)total), dim3(512), 0, st.stream, P,
                         (unsigned)total);
    else if (((any_bf && pipe_bf_w8()) || (!any_bf && pipe_f32_w8())) && pipe_km() == 2)   // 8 waves, 2 k-tiles
      hipLaunchKernelGGL((gp::gemm_pipe_group<64, 64, 2, 4, 2, 1, 2>), dim3((unsigned)total), dim3(512), 0, st.stream,
                         P, (unsigned)total);
    else if ((any_bf && pipe_bf_w8()) || (!any_bf && pipe_f32_w8()))   // 8 waves of 32 x 16
      hipLaunchKernelGGL((gp::gemm_pipe_group<64, 64, 2, 4, 2>), dim3((unsigned)total), dim3(512), 0, st.stream, P,
                         (unsigned)total);
    else
      hipLaunchKernelGGL((gp::gemm_pipe_group<64, 64, 2, 2, 2>), dim3((unsigned)total), dim3(256), 0, st.stream, P,
                         (unsigned)total);
    VC_CHECK_LAUNCH();
  }
  if (red.R.n) {
    red.R.start[red.R.n] = (int)red.total;
    for (int p = 0; p < red.R.n; ++p) VC_REQUIRE(red.R.nelem[p] < (1L << 31));
    VC_REQUIRE(red.total < (1L << 31));
    hipLaunchKernelGGL(gp::splitk_reduce_sum_group, dim3((unsigned)red.total), dim3(256), 0, st.stream, red.R);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

static GroupState* group_of(void* group) {
  if (!group || ((uintptr_t)group % alignof(GroupState)) != 0) return nullptr;
  return reinterpret_cast<GroupState*>(group);
}

VC_EXPORT int vc_gemm_group_begin(void* group, hipStream_t stream) {
  GroupState* st = group_of(group);
  VC_REQUIRE(st);
  st->magic = GROUP_MAGIC;
  st->stream = stream;
  st->n = st->np = 0;
  st->ws_used = 0;
  st->cnt_used = 0;
  st->err = 0;
  return VC_OK;
}

VC_EXPORT int vc_gemm_group_end(void* group) {
  GroupState* st = group_of(group);
  VC_REQUIRE(st && st->magic == GROUP_MAGIC);
  st->magic = 0;
  const int err = st->err;
  const int rc = group_flush(*st);
  return err ? err : rc;
}

static int launch_legacy(int transA, int transB, int M, int N, int K, float alpha,
                         const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                         float beta, float* C, long ldc, long strideC, int batch,
                         const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                         float* bias_grad, float* ws, long ws_floats, unsigned int* tile_counters,
                         int n_counters, hipStream_t stream, GroupState* st) {
  // the plan (split-K slices, combine path) depends on the problem and the caller's whole workspace /
  // counter arrays only -- never on what a group has used of them -- so a GEMM gives the same bits
  // grouped or alone, whatever its neighbours (tests/test_model_gpu.py::test_lane_schedules_*)
  LegacyPlan pl = plan_legacy(transA, transB, M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C, ldc, strideC,
                              batch, bias, addend, add_ld, add_mod, flags, bias_grad, ws, ws_floats, tile_counters,
                              n_counters);
  if (!st) return launch_plan(pl, stream);
  const long need = (pl.ws_floats + 63) / 64 * 64;
  if (st->n == GROUP_MAX || st->ws_used + need > ws_floats || st->cnt_used + pl.counters > n_counters) {
    const int rc = group_flush(*st);   // launch what is recorded; this problem starts a new group
    if (rc) return rc;
  }
  // this problem's slices of the workspace and the counters follow the earlier problems' slices
  if (pl.g.nsplit > 1) pl.g.part = ws + st->ws_used;
  if (pl.g.cnt) pl.g.cnt = tile_counters + st->cnt_used;
  st->ws_used += need;
  st->cnt_used += pl.counters;
  st->plans[st->n++] = pl;
  return VC_OK;
}

static int gemm_impl(int transA, int transB, int M, int N, int K, float alpha,
                     const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                     float beta, float* C, long ldc, long strideC, int batch,
                     const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                     float* bias_grad, float* ws, long ws_floats, unsigned int* tile_counters,
                     int n_counters, hipStream_t stream, GroupState* group);

// a problem of the group: the fp32 k-major ones wait for vc_gemm_group_end; any other (bf16 operands,
// K >= 4096) launches at once on the group's stream
VC_EXPORT int vc_gemm_group_add(void* group, int transA, int transB, int M, int N, int K, float alpha,
                                const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                                float beta, float* C, long ldc, long strideC, int batch,
                                const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                                float* bias_grad, float* ws, long ws_floats, unsigned int* tile_counters,
                                int n_counters) {
  GroupState* st = group_of(group);
  VC_REQUIRE(st && st->magic == GROUP_MAGIC);
  const int rc = gemm_impl(transA, transB, M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C, ldc, strideC,
                           batch, bias, addend, add_ld, add_mod, flags, bias_grad, ws, ws_floats, tile_counters,
                           n_counters, st->stream, st);
  if (rc && !st->err) st->err = rc;
  return rc;
}

// C[M, N] = A[M, K] W[N, K]^T + bias (fp32 or, flags & 2, bf16 operands) on the pipelined kernel without split-K,
// with the BatchNorm statistics partials of C written by the epilogue (shift = bias): colstats [ceil(M/64)][2][N]
// fp64, the layout vc_bn_apply_partials reduces.  Needs the pipelined kernel's operand alignment (else 1).
VC_EXPORT int vc_gemm_colstats(int M, int N, int K, const float* A, long lda, const float* W, long ldw,
                               const float* bias, float* C, long ldc, int flags, double* colstats, hipStream_t stream) {
  VC_REQUIRE(M > 0 && N > 0 && K > 0 && bias && colstats);
  VC_REQUIRE(pipe_fits(0, 1, M, N, K, A, lda, W, ldw, 1, nullptr));
  const bool bf = (flags & F_BF16) != 0;
  PipePlan p = plan_pipe(M, N, K, 0, false, bf);   // no workspace: no split
  VC_REQUIRE(p.nsplit == 1 && p.bm == 64 && p.bn == 64 && p.ns == 2);
  Epi epi{1.f, 0.f, bias, nullptr, 0, M, 0};
  GemmArgs g{M, N, K, N, p.k_chunk, 1, A, lda, 0, W, ldw, 0, C, ldc, 0, nullptr, nullptr, nullptr, epi};
  g.colstats = colstats;
  g.shift = bias;
  const long total = (long)p.tn * p.tm;
  dim3 grid((unsigned)total);
  if (bf) {
    if (pipe_bf_w8())
      hipLaunchKernelGGL((gp::gemm_pipe<64, 64, 2, 4, false, true, 2, true>), grid, dim3(512), 0, stream, g, p.tn,
                         p.tm, (unsigned)total, 1, 1);
    else
      hipLaunchKernelGGL((gp::gemm_pipe<64, 64, 2, 2, false, true, 2, true>), grid, dim3(256), 0, stream, g, p.tn,
                         p.tm, (unsigned)total, 1, 1);
  } else if (pipe_ks(total, 1, K) == 2)
    hipLaunchKernelGGL((gp::gemm_pipe<64, 64, 2, 2, false, true, 2, false, 2>), grid, dim3(512), 0, stream, g, p.tn,
                       p.tm, (unsigned)total, 1, 1);
  else if (pipe_f32_w8())
    hipLaunchKernelGGL((gp::gemm_pipe<64, 64, 2, 4, false, true, 2>), grid, dim3(512), 0, stream, g, p.tn, p.tm,
                       (unsigned)total, 1, 1);
  else
    hipLaunchKernelGGL((gp::gemm_pipe<64, 64, 2, 2, false, true, 2>), grid, dim3(256), 0, stream, g, p.tn, p.tm,
                       (unsigned)total, 1, 1);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_EXPORT int vc_gemm_ex(int transA, int transB, int M, int N, int K, float alpha,
                         const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                         float beta, float* C, long ldc, long strideC, int batch,
                         const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                         float* bias_grad, float* ws, long ws_floats, unsigned int* tile_counters,
                         int n_counters, hipStream_t stream) {
  return gemm_impl(transA, transB, M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C, ldc, strideC, batch,
                   bias, addend, add_ld, add_mod, flags, bias_grad, ws, ws_floats, tile_counters, n_counters, stream,
                   nullptr);
}

static int gemm_impl(int transA, int transB, int M, int N, int K, float alpha,
                     const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                     float beta, float* C, long ldc, long strideC, int batch,
                     const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                     float* bias_grad, float* ws, long ws_floats, unsigned int* tile_counters,
                     int n_counters, hipStream_t stream, GroupState* group) {
  VC_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1);
  VC_REQUIRE(!bias_grad || batch == 1);
  if (M == 0 || N == 0) return VC_OK;
  const bool bf = (flags & F_BF16) != 0;
  // mid shapes: the LDS-DMA pipelined kernel, fp32 or (F_BF16) bf16 MFMAs over the same fp32 stages
  // (F_PIPE forces it where it fits, F_NOPIPE keeps the older kernels: tests, census).  The choice depends on the problem only: a grouped problem that
  // takes it launches at once on the group's stream
  if (!(flags & (F_LEGACY | F_V2 | F_NOPIPE)) &&
      pipe_fits(transA, transB, M, N, K, A, lda, B, ldb, batch, bias_grad) &&
      ((flags & F_PIPE) || pipe_wanted(M, N, K))) {
    const int fl = flags & ~(F_PIPE | F_NOPIPE);
    const int Ne = N + (bias_grad ? 1 : 0);
    const PipePlan p = plan_pipe(M, Ne, K, ws_floats, ws != nullptr, bf);
    if (group) {
      // a problem whose own grid fills the chip launches alone (knob GEMM_GROUP_MAXB: the largest grid
      // that joins a group; probe library)
      const long own = (long)p.tn * p.tm * p.nsplit;
      if (p.bm == 64 && p.bn == 64 && p.ns == 2 && own <= vc_knob("VITCNN_GEMM_GROUP_MAXB", 1L << 30)) {
        const long need = p.nsplit > 1 ? ((long)p.nsplit * M * Ne + 63) / 64 * 64 : 0;
        GroupState& st = *group;
        if (st.np == GROUP_MAX || st.ws_used + need > ws_floats) {
          const int rc = group_flush(st);
          if (rc) return rc;
        }
        Epi epi{alpha, beta, bias, addend, add_ld, add_mod > 0 ? add_mod : M, fl};
        PipeRec& pr = st.pipes[st.np++];
        pr.g = GemmArgs{M, N, K, Ne, p.k_chunk, p.nsplit, A, lda, 0, B, ldb, 0, C, ldc, 0, bias_grad,
                        p.nsplit > 1 ? ws + st.ws_used : ws, nullptr, epi};
        pr.tn = p.tn;
        pr.tm = p.tm;
        pr.variant = (bf ? 4 : 0) | (transA ? 2 : 0) | (transB ? 1 : 0);
        st.ws_used += need;
        return VC_OK;
      }
    }
    return launch_pipe(transA, transB, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, bias, addend, add_ld, add_mod,
                       fl, bias_grad, ws, ws_floats, tile_counters, n_counters, stream);
  }
  // fp32: the k-major kernel (faster on every shape of the ViT-CNN step, tools/gemm_census.py) except
  // long contractions (K >= 4096, e.g. FusAtNet's 3x3 convs over 1024-2193 channels), where the
  // K-contiguous kernel's two accumulator chains and <= 2048-long slices keep the fp32 rounding at
  // the CPU reference's level (tools/gemm_err.py).  F_LEGACY / F_V2 force either (tests, census).
  const bool legacy = !bf && !(flags & F_V2) && ((flags & F_LEGACY) || K < 4096 || transA);
  if (legacy)
    return launch_legacy(transA, transB, M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C, ldc, strideC,
                         batch, bias, addend, add_ld, add_mod, flags, bias_grad, ws, ws_floats, tile_counters,
                         n_counters, stream, group);
  Epi epi{alpha, beta, bias, addend, add_ld, add_mod > 0 ? add_mod : M, flags};
  const int Ne = N + (bias_grad ? 1 : 0);
  const int KT = bf ? 64 : 32;
  // Configuration from the sweep of the step's shapes (tools/gemm_sweep.py):
  //  * 64 x 64 tiles; bf16 takes 128-row tiles for grids of >= 1024 tiles (fewer B re-reads);
  //  * split K when the grid is small (< 192 tiles) or K is long (>= 1024): slices of >= 2 k-tiles,
  //    up to ~4 blocks per CU (1024 blocks), at most 256 slices; the weight gradients (K = rows,
  //    tiny grids) end at 64-256 slices of 2-3 k-tiles each;
  //  * two k-tiles of loads in flight (pf 2) for bf16 weight gradients, else one.
  const int tiles64 = vc_cdiv(Ne, 64) * vc_cdiv(M, 64) * batch;
  int BM = (bf && tiles64 >= 1024) ? 128 : 64;
  int BN = 64;
  if (g_tune.bm) BM = g_tune.bm;
  if (g_tune.bn) BN = g_tune.bn;
  const int tn = vc_cdiv(Ne, BN), tm = vc_cdiv(M, BM);
  const long tiles = (long)tn * tm * batch;
  int nsplit = 1;
  if (K >= 4 * KT && (tiles < 192 || K >= 1024)) {
    const long by_k = K / (2 * KT);
    const long by_blocks = std::max<long>(1, 1024 / tiles);
    nsplit = (int)std::min<long>(std::min<long>(by_k, by_blocks), 256);
  }
  if (!bf) nsplit = std::max(nsplit, vc_cdiv(K, 2048));  // fp32: slices of <= 2048 (accuracy)
  if (g_tune.nsplit) nsplit = std::min(g_tune.nsplit, std::max(1, K / KT));
  if (!ws) nsplit = 1;
  while (nsplit > 1 && (long)nsplit * batch * M * Ne > ws_floats) --nsplit;
  int k_chunk = vc_cdiv(K, KT) * KT;
  if (nsplit > 1) {
    k_chunk = vc_cdiv(vc_cdiv(K, nsplit), KT) * KT;
    nsplit = vc_cdiv(K, k_chunk);
  }
  const int pf = g_tune.pf ? g_tune.pf : ((bf && transA) ? 2 : 1);
  // the slices of a tile run side by side on one XCD (split index fastest in the block order), so
  // the last arriver's slab reads are L2 hits: combine in-launch unless the tile's slabs are large
  const long slab_bytes = (long)nsplit * std::min(BM, M) * std::min(BN, Ne) * 4;
  bool inl = slab_bytes <= g2_combine_limit();
  if (g_tune.combine >= 0) inl = g_tune.combine == 1;
  unsigned int* cnt = (nsplit > 1 && tile_counters && tiles <= n_counters && inl) ? tile_counters : nullptr;
  GemmArgs g{M, N, K, Ne, k_chunk, nsplit, A, lda, strideA, B, ldb, strideB, C, ldc, strideC, bias_grad, ws, cnt, epi};
  const long total = tiles * nsplit;
  VC_REQUIRE(total < (1L << 31));
  // vector staging (float4 along the contiguous axis): 16-B aligned base, ld % 4, batch stride % 4
  auto vec_ok = [&](const float* p, long ld, long stride) {
    return ((uintptr_t)p % 16 == 0) && (ld % 4 == 0) && (batch == 1 || stride % 4 == 0);
  };
  const int va = vec_ok(A, lda, strideA);
  const int vb = vec_ok(B, ldb, strideB);
  const int G = g2::slab_groups(nsplit);
  const int zfast = cnt ? 1 : 0;
  dim3 grid((unsigned)total), block(256);
#define VC_G2(BF_, BM_, BN_, PF_)                                                                                 \
  do {                                                                                                            \
    if (transA && transB)                                                                                         \
      hipLaunchKernelGGL((g2::gemm_mfma<BF_, BM_, BN_, true, true, PF_>), grid, block, 0, stream, g, tn, tm, (unsigned)total, va, vb, G, zfast);   \
    else if (transA)                                                                                              \
      hipLaunchKernelGGL((g2::gemm_mfma<BF_, BM_, BN_, true, false, PF_>), grid, block, 0, stream, g, tn, tm, (unsigned)total, va, vb, G, zfast);  \
    else if (transB)                                                                                              \
      hipLaunchKernelGGL((g2::gemm_mfma<BF_, BM_, BN_, false, true, PF_>), grid, block, 0, stream, g, tn, tm, (unsigned)total, va, vb, G, zfast);  \
    else                                                                                                          \
      hipLaunchKernelGGL((g2::gemm_mfma<BF_, BM_, BN_, false, false, PF_>), grid, block, 0, stream, g, tn, tm, (unsigned)total, va, vb, G, zfast); \
  } while (0)
#define VC_G2_T(BF_, PF_)                                  \
  do {                                                     \
    if (BM == 128 && BN == 128) VC_G2(BF_, 128, 128, PF_); \
    else if (BM == 128) VC_G2(BF_, 128, 64, PF_);          \
    else if (BN == 128) VC_G2(BF_, 64, 128, PF_);          \
    else VC_G2(BF_, 64, 64, PF_);                          \
  } while (0)
  if (bf) {
    if (pf == 2) VC_G2_T(true, 2);
    else VC_G2_T(true, 1);
  } else {
    if (pf == 2) VC_G2_T(false, 2);
    else VC_G2_T(false, 1);
  }
#undef VC_G2_T
#undef VC_G2
  VC_CHECK_LAUNCH();
  if (nsplit > 1 && !cnt) {
    const long nelem = (long)batch * M * Ne;
    VC_REQUIRE(nelem < (1L << 31));
    hipLaunchKernelGGL(g2::splitk_reduce4, dim3(vc_cdiv(nelem, 1024 / G)), dim3(256), 0, stream, g, nelem, G);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

VC_EXPORT int vc_gemm(int transA, int transB, int M, int N, int K, float alpha,
                      const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                      float beta, float* C, long ldc, long strideC, int batch,
                      const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                      float* bias_grad, float* ws, long ws_floats, hipStream_t stream) {
  return vc_gemm_ex(transA, transB, M, N, K, alpha, A, lda, strideA, B, ldb, strideB, beta, C, ldc, strideC, batch,
                    bias, addend, add_ld, add_mod, flags, bias_grad, ws, ws_floats, nullptr, 0, stream);
}

// out[c] = beta * out[c] + sum_r X[r * ldx + c]   (deterministic: fixed-order partials).  counters
// (optional): >= ceil(Cn/64) zeroed arrival counters (left zero) -- the partials are then reduced in
// the last-arriving block of each column group instead of a second launch.
VC_EXPORT int vc_colsum_ex(int R, int Cn, const float* X, long ldx, float* out, float beta, float* ws, long ws_floats,
                           unsigned int* counters, int n_counters, hipStream_t stream) {
  VC_REQUIRE(R >= 0 && Cn >= 0);
  if (Cn == 0) return VC_OK;
  // ~64-128 rows per partial block, at most 128 partials (the reduction reads P/4 per thread)
  int rows_per = std::max(64, vc_cdiv(R, 128));
  int P = std::max(1, vc_cdiv(R, rows_per));
  while (P > 1 && (long)P * Cn > ws_floats && rows_per < (1 << 30)) {
    rows_per *= 2;
    P = std::max(1, vc_cdiv(R, rows_per));
  }
  VC_REQUIRE(P == 1 || (long)P * Cn <= ws_floats);
  VC_REQUIRE(P <= 65535);
  unsigned int* cnt = (P > 1 && counters && n_counters >= vc_cdiv(Cn, 64)) ? counters : nullptr;
  hipLaunchKernelGGL(colsum_partial, dim3(vc_cdiv(Cn, 64), P), dim3(256), 0, stream, R, Cn, X, ldx, rows_per, ws, cnt,
                     out, beta);
  VC_CHECK_LAUNCH();
  if (P > 1 && !cnt) {
    hipLaunchKernelGGL(colsum_final, dim3(vc_cdiv(Cn, 64)), dim3(256), 0, stream, P, Cn, ws, out, beta);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

VC_EXPORT int vc_colsum(int R, int Cn, const float* X, long ldx, float* out, float beta, float* ws, long ws_floats,
                        hipStream_t stream) {
  return vc_colsum_ex(R, Cn, X, ldx, out, beta, ws, ws_floats, nullptr, 0, stream);
}
