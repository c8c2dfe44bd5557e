// GEMM design lab (standalone, GPU): variants of the k-pipelined fp32 MFMA GEMM on the step's shapes.
// C[M,N] = A[M,K] B[N,K]^T (both operands K-contiguous: the conv / 1x1-conv forward form), timed with
// HIP events and checked against an fp64 reference.  Not product code: the winner's structure goes to
// vit-cnn_amd/csrc/gemm.hip.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_lab.hip -o tools/gemm_lab
//   run:   tools/gemm_lab [reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int KT = 32;
constexpr unsigned OOB = 0x80000000u;

__device__ __forceinline__ int lds_off(int r, int c) { return (r << 7) + ((c ^ ((r >> 1) & 7)) << 4); }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const char* lds, unsigned voff) {
  const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(const lds_void*)lds);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(dst), "s"(r)
      : "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// row-contiguous image [32 k][ROWS]: 16-column blocks XOR-swizzled by (k >> 2) & 1 (g2::Stage::rc_off)
template <int ROWS>
__device__ __forceinline__ int rc_off(int k, int col) {
  return k * (ROWS * 4) + ((((col >> 4) ^ ((k >> 2) & 1))) << 6) + ((col & 15) << 2);
}

// one operand's stage, filled by NW waves; T: row-contiguous source (r, k) at k * ld + r
template <bool T, int ROWS, int NW>
__device__ __forceinline__ void fill(__amdgpu_buffer_rsrc_t r, char* img, int row0, int k0, int kend, long ld,
                                     int wave, int lane) {
  static_assert((ROWS / 8) % NW == 0, "fill split");
#pragma unroll
  for (int q = 0; q < ROWS / 8 / NW; ++q) {
    const int i = wave + NW * q;
    unsigned voff;
    if constexpr (!T) {
      const int row = 8 * i + (lane >> 3), slot = lane & 7;
      const int k = k0 + 4 * (slot ^ ((row >> 1) & 7));
      voff = k < kend ? (unsigned)(((long)(row0 + row) * ld + k) * 4) : OOB;
    } else {
      constexpr int KR = 256 / ROWS, SL = ROWS / 4;
      const int kr = KR * i + lane / SL, sq = lane % SL;
      const int col = ((((sq >> 2) ^ ((kr >> 2) & 1))) << 4) + ((sq & 3) << 2);
      const int k = k0 + kr;
      voff = k < kend ? (unsigned)(((long)k * ld + row0 + col) * 4) : OOB;
    }
    dma16(r, img + i * 1024, voff);
  }
}

template <bool T, int ROWS>
__device__ __forceinline__ uint4 frag(const char* img, int rowbase, int s, int lane) {
  const int g = lane >> 4, l16 = lane & 15;
  if constexpr (!T) {
    return *reinterpret_cast<const uint4*>(img + lds_off(rowbase + l16, 4 * s + g));
  } else {
    uint4 o;
    const int k = 16 * s + 4 * g, col = rowbase + l16;
    o.x = *reinterpret_cast<const uint32_t*>(img + rc_off<ROWS>(k, col));
    o.y = *reinterpret_cast<const uint32_t*>(img + rc_off<ROWS>(k + 1, col));
    o.z = *reinterpret_cast<const uint32_t*>(img + rc_off<ROWS>(k + 2, col));
    o.w = *reinterpret_cast<const uint32_t*>(img + rc_off<ROWS>(k + 3, col));
    return o;
  }
}

// C[M,N] = op(A) op(B): op(A)(m,k) = TA ? A[k*M + m] : A[m*K + k]; op(B)(k,n) = TB ? B[n*K + k] : B[k*N + n]
template <int BM, int BN, int WM, int WN, int NS, bool TA, bool TB>
__global__ __launch_bounds__(64 * WM * WN) void gemm_lab(const float* A, const float* B, float* C, int M, int N,
                                                         int K, int k_chunk, int nsplit, int tn, int tm) {
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int SA_B = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int LOADS = (BM / 8 + BN / 8) / NW;
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const unsigned total = gridDim.x, bid = blockIdx.x, q8 = total >> 3, r8 = total & 7, x8 = bid & 7;
  const unsigned lin = x8 * q8 + min(x8, r8) + (bid >> 3);
  const int zs = (int)(lin % (unsigned)nsplit);
  const unsigned t1 = lin / (unsigned)nsplit;
  const int xn = (int)(t1 % (unsigned)tn), ym = (int)(t1 / (unsigned)tn);
  const int m0 = ym * BM, n0 = xn * BN;
  const int kbeg = zs * k_chunk, kend = min(K, kbeg + k_chunk);
  const long lda = TA ? M : K, ldb = TB ? K : N;
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), (short)0, (int)((long)M * K * 4), 0x00020000);
  const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B), (short)0, (int)((long)N * K * 4), 0x00020000);
  const int nk = kend > kbeg ? (kend - kbeg + KT - 1) / KT : 0;
  auto issue = [&](int t) {
    char* st = smem + (t % NS) * STAGE;
    const int k0 = kbeg + t * KT;
    fill<TA, BM, NW>(ra, st, m0, k0, kend, lda, wave, lane);
    fill<!TB, BN, NW>(rb, st + SA_B, n0, k0, kend, ldb, wave, lane);
  };
  f32x4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int p = 0; p < NS - 1; ++p)
    if (p < nk) issue(p);
  for (int t = 0; t < nk; ++t) {
    const int later = min(NS - 2, nk - 1 - t);
    if (NS >= 4 && later >= 2) vm_wait<2 * LOADS>();
    else if (NS >= 3 && later >= 1) vm_wait<LOADS>();
    else vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < nk) issue(t + NS - 1);
    const char* As = smem + (t % NS) * STAGE;
    const char* Bs = As + SA_B;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      uint4 a[MT], b[NT];
#pragma unroll
      for (int mi = 0; mi < MT; ++mi) a[mi] = frag<TA, BM>(As, wm * WTM + 16 * mi, s, lane);
#pragma unroll
      for (int ni = 0; ni < NT; ++ni) b[ni] = frag<!TB, BN>(Bs, wn * WTN + 16 * ni, s, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
#pragma unroll
          for (int ni = 0; ni < NT; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[mi][j]), __uint_as_float(b[ni][j]),
                                                               acc[mi][ni], 0, 0, 0);
    }
  }
  float* out = C + (long)zs * M * N;
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + r;
        const int n = n0 + wn * WTN + ni * 16 + (lane & 15);
        if (m < M && n < N) out[(long)m * N + n] = acc[mi][ni][r];
      }
}

__global__ void ref_gemm(const float* A, const float* B, double* C, int M, int N, int K, int ta, int tb) {
  const int n = blockIdx.x * 64 + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  double s = 0;
  for (int k = 0; k < K; ++k)
    s += (double)(ta ? A[(long)k * M + m] : A[(long)m * K + k]) * (double)(tb ? B[(long)n * K + k] : B[(long)k * N + n]);
  C[(long)m * N + n] = s;
}

__global__ void sum_slabs(const float* P, float* C, long n, int ns) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int z = 0; z < ns; ++z) s += P[z * n + i];
  C[i] = s;
}

struct Shape {
  int ta, tb, M, N, K;
};

struct Res {
  double us;
  char name[64];
};

template <int BM, int BN, int WM, int WN, int NS, bool TA, bool TB>
Res run(const char* name, const Shape& sh, int nsplit, const float* A, const float* B, float* P, float* C,
        const std::vector<double>& ref, int reps) {
  const int M = sh.M, N = sh.N, K = sh.K;
  const int tn = (N + BN - 1) / BN, tm = (M + BM - 1) / BM;
  const int k_chunk = ((K + nsplit - 1) / nsplit + KT - 1) / KT * KT;
  nsplit = (K + k_chunk - 1) / k_chunk;
  const int grid = tn * tm * nsplit;
  auto launch = [&]() {
    hipLaunchKernelGGL((gemm_lab<BM, BN, WM, WN, NS, TA, TB>), dim3(grid), dim3(64 * WM * WN), 0, 0, A, B,
                       nsplit > 1 ? P : C, M, N, K, k_chunk, nsplit, tn, tm);
    if (nsplit > 1)
      hipLaunchKernelGGL(sum_slabs, dim3(((long)M * N + 255) / 256), dim3(256), 0, 0, P, C, (long)M * N, nsplit);
  };
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / reps;
  std::vector<float> got((size_t)M * N);
  CK(hipMemcpy(got.data(), C, got.size() * 4, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  for (size_t i = 0; i < got.size(); ++i) {
    err = std::max(err, std::fabs(got[i] - ref[i]));
    mx = std::max(mx, std::fabs(ref[i]));
  }
  printf("  %-22s ks=%2d ns=%2d grid=%5d  %7.1f us  %6.1f TF  err %.1e\n", name, 0, nsplit, grid, us,
         2.0 * M * N * K / us * 1e-6, err / mx);
  Res r;
  r.us = us;
  snprintf(r.name, sizeof(r.name), "%s ns%d", name, nsplit);
  return r;
}

template <bool TA, bool TB>
void sweep(const Shape& sh, const float* A, const float* B, float* P, float* C, const std::vector<double>& ref,
           int reps) {
  std::vector<Res> rs;
  const int kt = (sh.K + KT - 1) / KT;
  for (int ks : {1, 2, 4, 8}) {
    if (ks > 1 && kt / ks < 4) continue;
    rs.push_back(run<64, 64, 2, 2, 2, TA, TB>("64x64 w2x2 ns2", sh, ks, A, B, P, C, ref, reps));
    rs.push_back(run<64, 64, 2, 2, 4, TA, TB>("64x64 w2x2 ns4", sh, ks, A, B, P, C, ref, reps));
    rs.push_back(run<128, 64, 4, 2, 2, TA, TB>("128x64 w4x2 ns2", sh, ks, A, B, P, C, ref, reps));
    rs.push_back(run<64, 128, 2, 4, 2, TA, TB>("64x128 w2x4 ns2", sh, ks, A, B, P, C, ref, reps));
    rs.push_back(run<128, 128, 4, 2, 3, TA, TB>("128x128 w4x2 ns3", sh, ks, A, B, P, C, ref, reps));
  }
  size_t b = 0;
  for (size_t i = 1; i < rs.size(); ++i)
    if (rs[i].us < rs[b].us) b = i;
  printf("BEST ta=%d tb=%d M=%d N=%d K=%d: %s %.1f us (%.1f TF)\n", sh.ta, sh.tb, sh.M, sh.N, sh.K, rs[b].name, rs[b].us,
         2.0 * sh.M * sh.N * sh.K / rs[b].us * 1e-6);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 30;
  // the step's critical-path GEMMs (tools/gemm_pipe_bench.py SHAPES)
  std::vector<Shape> shapes = {{0, 1, 3136, 256, 1296}, {0, 0, 3136, 1296, 256}, {1, 0, 256, 1296, 3136},
                               {0, 1, 1600, 144, 2304}, {1, 0, 144, 2304, 1600}, {0, 0, 1600, 2304, 144},
                               {1, 0, 256, 512, 3136},  {0, 0, 3136, 512, 256},  {0, 1, 3136, 256, 512},
                               {1, 0, 256, 144, 5184},  {0, 0, 5184, 144, 256},  {0, 1, 5184, 256, 144},
                               {0, 1, 3136, 256, 256},  {0, 1, 3136, 256, 128},  {0, 0, 3136, 256, 256},
                               {1, 0, 256, 256, 3136},  {1, 0, 128, 256, 3136},  {0, 1, 3136, 128, 272},
                               {0, 1, 1600, 144, 288},  {1, 0, 144, 288, 1600},  {0, 0, 1600, 288, 144}};
  float *A, *B, *C, *P;
  double* R;
  const size_t maxe = 8 << 20;
  CK(hipMalloc(&A, maxe * 4));
  CK(hipMalloc(&B, maxe * 4));
  CK(hipMalloc(&C, maxe * 4));
  CK(hipMalloc(&P, 64 * maxe));
  CK(hipMalloc(&R, maxe * 8));
  for (const Shape& sh : shapes) {
    std::vector<float> ha((size_t)sh.M * sh.K), hb((size_t)sh.N * sh.K);
    srand(1);
    for (auto& v : ha) v = (float)rand() / (float)RAND_MAX * 2 - 1;
    for (auto& v : hb) v = (float)rand() / (float)RAND_MAX * 2 - 1;
    CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(ref_gemm, dim3((sh.N + 63) / 64, sh.M), dim3(64), 0, 0, A, B, R, sh.M, sh.N, sh.K, sh.ta, sh.tb);
    std::vector<double> ref((size_t)sh.M * sh.N);
    CK(hipMemcpy(ref.data(), R, ref.size() * 8, hipMemcpyDeviceToHost));
    printf("ta=%d tb=%d M=%d N=%d K=%d\n", sh.ta, sh.tb, sh.M, sh.N, sh.K);
    if (sh.ta && sh.tb) sweep<true, true>(sh, A, B, P, C, ref, reps);
    else if (sh.ta) sweep<true, false>(sh, A, B, P, C, ref, reps);
    else if (sh.tb) sweep<false, true>(sh, A, B, P, C, ref, reps);
    else sweep<false, false>(sh, A, B, P, C, ref, reps);
  }
  return 0;
}
