// Confusion matrix of a whole-image prediction, counted on the device: the counting step of the
// reference's metrics() (utils.py:585-663) — ignored target labels dropped (:596-601), then
// sklearn confusion_matrix(target, prediction, labels=range(n_classes)) (:608-611): rows are
// target labels, columns predictions, pairs outside the label set are not counted.
//
// Integer histogram, HBM-bound: 16 B read per pixel (int64 target + int64 prediction).  Each
// block counts its grid-stride share into an LDS histogram (n_classes^2 <= 4096 uint32 bins,
// 16 KB) with LDS atomics, then adds its non-zero bins into the global uint64 matrix.  Integer
// addition: the result does not depend on the schedule.
#include "common.h"

namespace {

constexpr int MAXC = 64;

__global__ __launch_bounds__(256) void confusion_count(long n, const long long* __restrict__ target,
                                                      const long long* __restrict__ pred, int ncls,
                                                      const unsigned char* __restrict__ ignored,
                                                      unsigned long long* __restrict__ cm) {
  __shared__ unsigned int h[MAXC * MAXC];
  const int nb = ncls * ncls;
  for (int i = threadIdx.x; i < nb; i += 256) h[i] = 0u;
  __syncthreads();
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long long t = target[i], p = pred[i];
    if (t < 0 || t >= ncls || p < 0 || p >= ncls || ignored[t]) continue;
    atomicAdd(&h[t * ncls + p], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += 256)
    if (h[i]) atomicAdd(&cm[i], (unsigned long long)h[i]);
}

}  // namespace

VC_EXPORT int vc_confusion_matrix(long n, const long long* target, const long long* pred, int n_classes,
                                  const unsigned char* ignored, unsigned long long* cm, hipStream_t stream) {
  VC_REQUIRE(n >= 0 && n_classes > 0 && n_classes <= MAXC && target && pred && ignored && cm);
  if (n == 0) return VC_OK;
  // ~8 pixels per thread, at most 2048 blocks (8 per CU)
  const int blocks = (int)std::min<long>(std::max(1, vc_cdiv(n, 256 * 8)), 2048);
  hipLaunchKernelGGL(confusion_count, dim3(blocks), dim3(256), 0, stream, n, target, pred, n_classes, ignored, cm);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
