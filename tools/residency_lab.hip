// Co-residency probe: how many blocks of one launch are running at the same time?  Each block
// arrives at a counter and waits (bounded) until all `n` blocks have arrived; the launch reports how
// many blocks gave up waiting.  Swept over grid sizes, block LDS sizes and poll styles, it tells
// whether a group barrier (vit-cnn_amd/csrc/common.h block_group_sync) can be used for a grid.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/residency_lab tools/residency_lab.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

template <int LDS_FLOATS>
__global__ __launch_bounds__(256) void wait_all(unsigned* cnt, unsigned n, unsigned* gave_up, unsigned* max_seen,
                                                int poll_rmw, float* sink) {
  __shared__ float pad[LDS_FLOATS];
  pad[threadIdx.x % LDS_FLOATS] = (float)threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned zero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    unsigned seen = 0;
    int it = 0;
    for (; it < (1 << 20); ++it) {
      seen = poll_rmw ? __hip_atomic_fetch_add(cnt, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (seen >= n) break;
      __builtin_amdgcn_s_sleep(4);
    }
    if (seen < n) __hip_atomic_fetch_add(gave_up, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_max(max_seen, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 1) sink[blockIdx.x] = pad[(threadIdx.x + 7) % LDS_FLOATS];
}

template <int LDS_FLOATS>
static void run(unsigned n, int poll_rmw, unsigned* d, float* sink) {
  hipMemset(d, 0, 3 * sizeof(unsigned));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(wait_all<LDS_FLOATS>, dim3(n), dim3(256), 0, 0, d, n, d + 1, d + 2, poll_rmw, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned h[3];
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("lds %6d B  grid %5u  poll %s  gave_up %5u  max_seen %5u  %.3f ms\n", LDS_FLOATS * 4, n,
         poll_rmw ? "rmw " : "load", h[1], h[2], ms);
  fflush(stdout);
}


// BN-shaped group barrier (norm.hip bn_bwd_fused): grid (groups, P); each block streams its rows of a
// [M][C] map (64 channels x rows_per rows), publishes a partial, meets its group's P blocks (counter pair
// cnt[2 g], cnt[2 g + 1], as common.h block_group_sync / block_group_leave), reads all P partials and
// writes its rows again.  gave_up counts blocks whose wait hit the bound.
__global__ __launch_bounds__(256) void bn_like(const float* x, int M, int C, int rows_per, float* part, unsigned* cnt,
                                               unsigned* gave_up, float* y, int poll_rmw, int use_fence) {
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * rows_per, r1 = min(M, r0 + rows_per);
  float s = 0.f;
  for (int r = r0 + rl; r < r1; r += 4) s += x[(long)r * C + c];
  __shared__ float sh[4][64];
  sh[rl][cl] = s;
  __syncthreads();
  if (rl == 0) part[blockIdx.y * C + c] = sh[0][cl] + sh[1][cl] + sh[2][cl] + sh[3][cl];
  unsigned* arrive = cnt + 2 * blockIdx.x;
  const unsigned n = gridDim.y;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (use_fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned zero;
    asm volatile("v_mov_b32 %0, 0" : "=v"(zero));
    unsigned seen = 0;
    for (int it = 0; it < (1 << 20); ++it) {
      seen = poll_rmw ? __hip_atomic_fetch_add(arrive, zero, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : __hip_atomic_load(arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (seen >= n) break;
      __builtin_amdgcn_s_sleep(4);
    }
    if (seen < n) __hip_atomic_fetch_add(gave_up, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (use_fence) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  float tot = 0.f;
  for (int p = 0; p < (int)n; ++p) tot += part[p * C + c];
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(arrive + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == n - 1) {
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(arrive + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  for (int r = r0 + rl; r < r1; r += 4) y[(long)r * C + c] = x[(long)r * C + c] - tot / (float)M;
}

static void run_bn(int M, int C, int rows_per, int poll_rmw, int use_fence, float* x, float* part, unsigned* cnt,
                   unsigned* gu, float* y) {
  const int P = (M + rows_per - 1) / rows_per;
  hipMemset(gu, 0, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL(bn_like, dim3((C + 63) / 64, P), dim3(256), 0, 0, x, M, C, rows_per, part, cnt, gu, y, poll_rmw,
                       use_fence);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned h[2], left[32];
  hipMemcpy(h, gu, 4, hipMemcpyDeviceToHost);
  hipMemcpy(left, cnt, sizeof(left), hipMemcpyDeviceToHost);
  unsigned nz = 0;
  for (int i = 0; i < 32; ++i) nz += left[i] != 0;
  printf("bn_like M %5d C %4d P %3d grid %4d poll %s fence %d: gave_up %u  counters left nonzero %u  %.3f ms / 3\n", M, C,
         P, (C + 63) / 64 * P, poll_rmw ? "rmw " : "load", use_fence, h[0], nz, ms);
  fflush(stdout);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  printf("%s  CUs %d  LDS/block max %zu\n", p.gcnArchName, p.multiProcessorCount, p.sharedMemPerBlock);
  unsigned* d;
  float* sink;
  hipMalloc(&d, 64);
  hipMalloc(&sink, 4096 * sizeof(float));
  for (int rmw = 0; rmw < 2; ++rmw)
    for (unsigned n : {64u, 128u, 256u, 512u, 1024u}) {
      run<256>(n, rmw, d, sink);
      run<8448>(n, rmw, d, sink);
    }
  float *x, *part, *y;
  unsigned *cnt, *gu;
  hipMalloc(&x, 3136L * 512 * 4);
  hipMalloc(&y, 3136L * 512 * 4);
  hipMalloc(&part, 1024L * 512 * 4);
  hipMalloc(&cnt, 4096);
  hipMalloc(&gu, 64);
  hipMemset(x, 0, 3136L * 512 * 4);
  hipMemset(cnt, 0, 4096);
  for (int rmw = 0; rmw < 2; ++rmw)
    for (int fence = 0; fence < 2; ++fence) {
      run_bn(3136, 256, 49, rmw, fence, x, part, cnt, gu, y);
      run_bn(3136, 512, 49, rmw, fence, x, part, cnt, gu, y);
      run_bn(5184, 144, 81, rmw, fence, x, part, cnt, gu, y);
    }
  hipFree(d);
  hipFree(sink);
  return 0;
}
