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
  hipFree(d);
  hipFree(sink);
  return 0;
}
