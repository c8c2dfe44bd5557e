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

constexpr int BM = 64, BN = 64, BK = 16;
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

// A element (m,k): TA ? A[k*lda + m] : A[m*lda + k];  B element (k,n): TB ? B[n*ldb + k] : B[k*ldb + n]
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_mfma(int M, int N, int K, int k_chunk, int nsplit,
                                                     const float* __restrict__ A, long lda, long sA,
                                                     const float* __restrict__ B, long ldb, long sB,
                                                     float* __restrict__ C, long ldc, long sC, Epi epi,
                                                     float* __restrict__ part) {
  __shared__ float As[BK * LDS_STRIDE];
  __shared__ float Bs[BK * LDS_STRIDE];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n0 = blockIdx.x * BN, m0 = blockIdx.y * BM;
  const int zb = blockIdx.z / nsplit, zs = blockIdx.z % nsplit;
  const int kbeg = zs * k_chunk;
  const int kend = min(K, kbeg + k_chunk);
  A += (long)zb * sA;
  B += (long)zb * sB;

  float ra[4], rb[4];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int m, k;
      if (TA) { m = tid & 63; k = (tid >> 6) + 4 * i; }
      else    { k = tid & 15; m = (tid >> 4) + 16 * i; }
      int gm = m0 + m, gk = k0 + k;
      float v = 0.f;
      if (gm < M && gk < kend) v = TA ? A[(long)gk * lda + gm] : A[(long)gm * lda + gk];
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int n, k;
      if (TB) { k = tid & 15; n = (tid >> 4) + 16 * i; }
      else    { n = tid & 63; k = (tid >> 6) + 4 * i; }
      int gn = n0 + n, gk = k0 + k;
      float v = 0.f;
      if (gn < N && gk < kend) v = TB ? B[(long)gn * ldb + gk] : B[(long)gk * ldb + gn];
      rb[i] = v;
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int m, k;
      if (TA) { m = tid & 63; k = (tid >> 6) + 4 * i; }
      else    { k = tid & 15; m = (tid >> 4) + 16 * i; }
      As[k * LDS_STRIDE + m] = ra[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      int n, k;
      if (TB) { k = tid & 15; n = (tid >> 4) + 16 * i; }
      else    { n = tid & 63; k = (tid >> 6) + 4 * i; }
      Bs[k * LDS_STRIDE + n] = rb[i];
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
        float a0 = As[kk * LDS_STRIDE + wm * 32 + fr];
        float a1 = As[kk * LDS_STRIDE + wm * 32 + 16 + fr];
        float b0 = Bs[kk * LDS_STRIDE + wn * 32 + fr];
        float b1 = Bs[kk * LDS_STRIDE + wn * 32 + 16 + fr];
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
        if (m < M && n < N) {
          if (nsplit > 1) {
            part[((long)blockIdx.z * M + m) * N + n] = acc[mi][ni][r];
          } else {
            float* cp = C + (long)zb * sC + (long)m * ldc + n;
            *cp = epilogue(epi, acc[mi][ni][r], cp, m, n);
          }
        }
      }
}

__global__ void splitk_reduce(int M, int N, int nsplit, int batch, const float* __restrict__ part,
                              float* __restrict__ C, long ldc, long sC, Epi epi) {
  long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  long total = (long)batch * M * N;
  if (idx >= total) return;
  int n = idx % N;
  int m = (idx / N) % M;
  int b = idx / ((long)M * N);
  float s = 0.f;
  for (int z = 0; z < nsplit; ++z) s += part[(((long)b * nsplit + z) * M + m) * N + n];
  float* cp = C + (long)b * sC + (long)m * ldc + n;
  *cp = epilogue(epi, s, cp, m, n);
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

__global__ void colsum_final(int P, int Cn, const float* __restrict__ part, float* __restrict__ out, float beta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= Cn) return;
  float s = 0.f;
  for (int p = 0; p < P; ++p) s += part[(long)p * Cn + c];
  out[c] = (beta != 0.f ? beta * out[c] : 0.f) + s;
}

}  // namespace

// C[b] = alpha * op(A[b]) * op(B[b]) + beta * C[b] (+ bias[n]) (+ addend[(m % add_mod), n]) (relu)
VC_EXPORT int vc_gemm(int transA, int transB, int M, int N, int K, float alpha,
                      const float* A, long lda, long strideA, const float* B, long ldb, long strideB,
                      float beta, float* C, long ldc, long strideC, int batch,
                      const float* bias, const float* addend, long add_ld, int add_mod, int flags,
                      float* ws, long ws_floats, hipStream_t stream) {
  VC_REQUIRE(M >= 0 && N >= 0 && K >= 0 && batch >= 1);
  if (M == 0 || N == 0) return VC_OK;
  Epi epi{alpha, beta, bias, addend, add_ld, add_mod > 0 ? add_mod : M, flags};
  const int tn = vc_cdiv(N, BN), tm = vc_cdiv(M, BM);
  long tiles = (long)tn * tm * batch;
  // split K when the output grid cannot fill the 256 CUs (weight gradients: M,N small, K = rows)
  int nsplit = 1;
  if (ws && tiles < 256 && K >= 4 * BK) {
    long want = (512 + tiles - 1) / tiles;
    long maxk = K / (2 * BK);
    nsplit = (int)std::min<long>(std::min<long>(want, maxk), 64);
    while (nsplit > 1 && (long)nsplit * batch * M * N > ws_floats) --nsplit;
    if (nsplit < 1) nsplit = 1;
  }
  int k_chunk = K;
  if (nsplit > 1) {
    k_chunk = vc_cdiv(vc_cdiv(K, nsplit), BK) * BK;
    nsplit = vc_cdiv(K, k_chunk);
  }
  dim3 grid(tn, tm, batch * nsplit), block(256);
#define VC_LAUNCH_GEMM(TA_, TB_)                                                                          \
  hipLaunchKernelGGL((gemm_f32_mfma<TA_, TB_>), grid, block, 0, stream, M, N, K, k_chunk, nsplit, A, lda, \
                     strideA, B, ldb, strideB, C, ldc, strideC, epi, ws)
  if (transA && transB) VC_LAUNCH_GEMM(true, true);
  else if (transA) VC_LAUNCH_GEMM(true, false);
  else if (transB) VC_LAUNCH_GEMM(false, true);
  else VC_LAUNCH_GEMM(false, false);
#undef VC_LAUNCH_GEMM
  VC_CHECK_LAUNCH();
  if (nsplit > 1) {
    long total = (long)batch * M * N;
    hipLaunchKernelGGL(splitk_reduce, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, M, N, nsplit, batch, ws, C,
                       ldc, strideC, epi);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

// out[c] = beta * out[c] + sum_r X[r * ldx + c]   (deterministic two-stage; ws >= 2048 * ceil(C/64)*64)
VC_EXPORT int vc_colsum(int R, int Cn, const float* X, long ldx, float* out, float beta, float* ws, long ws_floats,
                        hipStream_t stream) {
  VC_REQUIRE(R >= 0 && Cn >= 0);
  if (Cn == 0) return VC_OK;
  int rows_per = 256;
  int P = std::max(1, vc_cdiv(R, rows_per));
  while ((long)P * Cn > ws_floats && rows_per < (1 << 30)) {
    rows_per *= 2;
    P = std::max(1, vc_cdiv(R, rows_per));
  }
  VC_REQUIRE((long)P * Cn <= ws_floats);
  hipLaunchKernelGGL(colsum_partial, dim3(vc_cdiv(Cn, 64), P), dim3(256), 0, stream, R, Cn, X, ldx, rows_per, ws);
  VC_CHECK_LAUNCH();
  hipLaunchKernelGGL(colsum_final, dim3(vc_cdiv(Cn, 256)), dim3(256), 0, stream, P, Cn, ws, out, beta);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
