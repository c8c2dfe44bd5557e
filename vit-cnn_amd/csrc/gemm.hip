// fp32 GEMM on CDNA4 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32 fma chain),
// plus split-K reduction and deterministic column sums.
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

namespace {

constexpr int BM = 64, BN = 64;
constexpr int LDS_STRIDE = 81;  // 64 + 17: conflict-free fragment reads, <=2-way stores

enum { F_RELU = 1 };

struct Epi {
  float alpha, beta;
  const float* bias;     // [N] or null
  const float* addend;   // addend[(m % add_mod) * add_ld + n] or null
  long add_ld;
  int add_mod;
  int flags;
};

__device__ __forceinline__ float epilogue(const Epi& e, float acc, const float* cptr, int m, int n) {
  float v = e.alpha * acc;
  if (e.beta != 0.f) v += e.beta * (*cptr);
  if (e.bias) v += e.bias[n];
  if (e.addend) v += e.addend[(long)(m % e.add_mod) * e.add_ld + n];
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

template <bool TA, bool TB, bool VA, bool VB>
__global__ __launch_bounds__(256) void gemm_f32_mfma(GemmArgs g) {
  __shared__ float As[BK * LDS_STRIDE];
  __shared__ float Bs[BK * LDS_STRIDE];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int zb = blockIdx.z / g.nsplit, zs = blockIdx.z % g.nsplit;
  const int kbeg = zs * g.k_chunk;
  const int kend = min(g.K, kbeg + g.k_chunk);
  const float* A = g.A + (long)zb * g.sA;
  const float* Bp = g.B + (long)zb * g.sB;
  const bool ones = g.Ne > g.N;

  float ra[NE], rb[NE];
  auto a_at = [&](int gm, int gk) -> float {
    return (gm < g.M && gk < kend) ? (TA ? A[(long)gk * g.lda + gm] : A[(long)gm * g.lda + gk]) : 0.f;
  };
  auto b_at = [&](int gn, int gk) -> float {
    if (gk >= kend) return 0.f;
    if (gn < g.N) return TB ? Bp[(long)gn * g.ldb + gk] : Bp[(long)gk * g.ldb + gn];
    return (ones && gn == g.N) ? 1.f : 0.f;
  };
  auto load = [&](int k0) {
#pragma unroll
    for (int v = 0; v < NE / 4; ++v) {
      if (VA) {
        int m, k;
        tile_idx<TA, true>(tid, 4 * v, m, k);
        const int gm = m0 + m, gk = k0 + k;
        const bool full = TA ? (gk < kend && gm + 3 < g.M) : (gm < g.M && gk + 3 < kend);
        if (full) {
          const float4 x = *reinterpret_cast<const float4*>(TA ? A + (long)gk * g.lda + gm : A + (long)gm * g.lda + gk);
          ra[4 * v] = x.x; ra[4 * v + 1] = x.y; ra[4 * v + 2] = x.z; ra[4 * v + 3] = x.w;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) ra[4 * v + i] = TA ? a_at(gm + i, gk) : a_at(gm, gk + i);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int m, k;
          tile_idx<TA, false>(tid, 4 * v + i, m, k);
          ra[4 * v + i] = a_at(m0 + m, k0 + k);
        }
      }
      if (VB) {
        int n, k;
        tile_idx<!TB, true>(tid, 4 * v, n, k);
        const int gn = n0 + n, gk = k0 + k;
        const bool full = TB ? (gn < g.N && gk + 3 < kend) : (gk < kend && gn + 3 < g.N);
        if (full) {
          const float4 x = *reinterpret_cast<const float4*>(TB ? Bp + (long)gn * g.ldb + gk : Bp + (long)gk * g.ldb + gn);
          rb[4 * v] = x.x; rb[4 * v + 1] = x.y; rb[4 * v + 2] = x.z; rb[4 * v + 3] = x.w;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) rb[4 * v + i] = TB ? b_at(gn, gk + i) : b_at(gn + i, gk);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int n, k;
          tile_idx<!TB, false>(tid, 4 * v + i, n, k);
          rb[4 * v + i] = b_at(n0 + n, k0 + k);
        }
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      int m, k;
      tile_idx<TA, VA>(tid, e, m, k);
      As[k * LDS_STRIDE + m] = ra[e];
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      int n, k;
      tile_idx<!TB, VB>(tid, e, n, k);
      Bs[k * LDS_STRIDE + n] = rb[e];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fk = lane >> 4;
  if (kbeg < kend) {
    load(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
      store();
      __syncthreads();
      if (k0 + BK < kend) load(k0 + BK);
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
          if (g.nsplit > 1) g.part[((long)blockIdx.z * g.M + m) * g.Ne + n] = acc[mi][ni][r];
          else store_out(g, zb, m, n, acc[mi][ni][r]);
        }
      }
  if (g.nsplit == 1 || !g.cnt) return;

  // In-launch split-K combine (cdna_hip_programming.md, "In-launch split-K reduction"): every
  // slice publishes its slab (stores drained, barrier, one agent-scope release), takes a ticket;
  // the tile's last arriver acquires and sums all slices in fixed z order — the same order as
  // splitk_reduce, so results do not depend on which slice arrives last — then re-zeroes the
  // counter for the next launch on this stream.
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int tile = (zb * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(&g.cnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = (t == (unsigned)(g.nsplit - 1));
  }
  __syncthreads();
  if (!last) return;
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
    const float* p = pz + (long)m * g.Ne + n;
    float sum = 0.f;
#pragma unroll 8
    for (int z = 0; z < g.nsplit; ++z) sum += p[z * slab];
    store_out(g, zb, m, n, sum);
  }
  if (tid == 0) __hip_atomic_store(&g.cnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// grid (ceil(Ne/64), M, batch): one thread per output element, no index division; the
// nsplit slab reads are independent (unrolled) and summed in fixed z order (deterministic)
__global__ __launch_bounds__(64) void splitk_reduce(GemmArgs g) {
  const int n = blockIdx.x * 64 + threadIdx.x;
  if (n >= g.Ne) return;
  const int m = blockIdx.y, b = blockIdx.z;
  const long slab = (long)g.M * g.Ne;
  const float* p = g.part + (long)b * g.nsplit * slab + (long)m * g.Ne + n;
  float s = 0.f;
#pragma unroll 8
  for (int z = 0; z < g.nsplit; ++z) s += p[z * slab];
  store_out(g, b, m, n, s);
}

// stage 1 of a column sum: block (cx, ry) sums rows [ry*rows_per, ...) of 64 columns
__global__ __launch_bounds__(256) void colsum_partial(int R, int Cn, const float* __restrict__ X, long ldx,
                                                      int rows_per, float* __restrict__ part) {
  __shared__ float sh[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(R, r0 + rows_per);
  float s = 0.f;
  if (c < Cn)
    for (int r = r0 + rl; r < r1; r += 4) s += X[(long)r * ldx + c];
  sh[rl][threadIdx.x & 63] = s;
  __syncthreads();
  if (rl == 0 && c < Cn) part[(long)blockIdx.y * Cn + c] = sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x];
}

}  // namespace

// C[b] = alpha * op(A[b]) * op(B[b]) + beta * C[b] (+ bias[n]) (+ addend[(m % add_mod), n]) (relu);
// bias_grad (optional): bias_grad[m] = alpha * sum_k op(A)(m,k) + beta * bias_grad[m]
VC_EXPORT int vc_gemm_ex(int transA, int transB, int M, int N, int K, float alpha,
                         const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                         float beta, float* C, long ldc, long strideC, int batch,
                         const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                         float* bias_grad, float* ws, long ws_floats, unsigned int* tile_counters,
                         int n_counters, hipStream_t stream) {
  VC_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1);
  VC_REQUIRE(!bias_grad || batch == 1);
  if (M == 0 || N == 0) return VC_OK;
  Epi epi{alpha, beta, bias, addend, add_ld, add_mod > 0 ? add_mod : M, flags};
  const int Ne = N + (bias_grad ? 1 : 0);
  const int tn = vc_cdiv(Ne, BN), tm = vc_cdiv(M, BM);
  const long tiles = (long)tn * tm * batch;
  // Split K when the output grid leaves the chip short of ~3 blocks per CU (768 blocks): each
  // K slice keeps >= 128 of K (4 BK steps), the slabs must fit the workspace, and the slices are
  // summed in fixed order (splitk_reduce) so results do not depend on the split's scheduling.
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
  unsigned int* cnt =
      (nsplit > 1 && tile_counters && tiles <= n_counters && slab_bytes <= 4096) ? tile_counters : nullptr;
  GemmArgs g{M, N, K, Ne, k_chunk, nsplit, A, lda, strideA, B, ldb, strideB, C, ldc, strideC, bias_grad, ws, cnt, epi};
  dim3 grid(tn, tm, batch * nsplit), block(256);
  const bool va = ((uintptr_t)A % 16 == 0) && (lda % 4 == 0) && (batch == 1 || strideA % 4 == 0);
  const bool vb = ((uintptr_t)B % 16 == 0) && (ldb % 4 == 0) && (batch == 1 || strideB % 4 == 0);
#define VC_LAUNCH_GEMM(TA_, TB_)                                                                           \
  do {                                                                                                     \
    if (va && vb) hipLaunchKernelGGL((gemm_f32_mfma<TA_, TB_, true, true>), grid, block, 0, stream, g);    \
    else if (va) hipLaunchKernelGGL((gemm_f32_mfma<TA_, TB_, true, false>), grid, block, 0, stream, g);    \
    else if (vb) hipLaunchKernelGGL((gemm_f32_mfma<TA_, TB_, false, true>), grid, block, 0, stream, g);    \
    else hipLaunchKernelGGL((gemm_f32_mfma<TA_, TB_, false, false>), grid, block, 0, stream, g);           \
  } while (0)
  if (transA && transB) VC_LAUNCH_GEMM(true, true);
  else if (transA) VC_LAUNCH_GEMM(true, false);
  else if (transB) VC_LAUNCH_GEMM(false, true);
  else VC_LAUNCH_GEMM(false, false);
#undef VC_LAUNCH_GEMM
  VC_CHECK_LAUNCH();
  if (nsplit > 1 && !cnt) {
    hipLaunchKernelGGL(splitk_reduce, dim3(vc_cdiv(Ne, 64), M, batch), dim3(64), 0, stream, g);
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

// out[c] = beta * out[c] + sum_r X[r * ldx + c]   (deterministic two-stage; ws >= 2048 * ceil(C/64)*64)
VC_EXPORT int vc_colsum(int R, int Cn, const float* X, long ldx, float* out, float beta, float* ws, long ws_floats,
                        hipStream_t stream) {
  VC_REQUIRE(R >= 0 && Cn >= 0);
  if (Cn == 0) return VC_OK;
  // ~64-128 rows per partial block, at most 512 partials, then a 16x16 parallel final sum
  int rows_per = std::max(64, vc_cdiv(R, 512));
  int P = std::max(1, vc_cdiv(R, rows_per));
  while ((long)P * Cn > ws_floats && rows_per < (1 << 30)) {
    rows_per *= 2;
    P = std::max(1, vc_cdiv(R, rows_per));
  }
  VC_REQUIRE((long)P * Cn <= ws_floats);
  if (P == 1) {  // small R: a single pass writes the result directly
    hipLaunchKernelGGL(colsum_partial, dim3(vc_cdiv(Cn, 64), 1), dim3(256), 0, stream, R, Cn, X, ldx, rows_per, ws);
    VC_CHECK_LAUNCH();
    return launch_sum_rows(1, Cn, ws, Cn, 0, out, beta, stream);
  }
  hipLaunchKernelGGL(colsum_partial, dim3(vc_cdiv(Cn, 64), P), dim3(256), 0, stream, R, Cn, X, ldx, rows_per, ws);
  VC_CHECK_LAUNCH();
  return launch_sum_rows(P, Cn, ws, Cn, 0, out, beta, stream);
}
