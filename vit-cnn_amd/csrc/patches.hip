// Patch windows on the device: gather [n][C][P][P] model inputs from an HBM-resident image cube
// and scatter window logits into the centre-pixel probability map.
//
// Replaces the host-side patch cutting of the reference: MultiModalX.__getitem__
// (datasets.py:550-593, incl. the flip/rot90 augmentation of :511-526) and the whole-image
// sliding_window / grouper / np.copy loop of test() (utils.py:357-415, :567-582;
// model_utils.py:1067-1132).
//
// HBM-bound byte movement (no arithmetic): per window C*P*P*4 bytes read + the same written.
// The cube keeps its source layout img[x][y][c] (band-contiguous), so one patch row (fixed x,
// P consecutive y) is P*C contiguous floats: the block reads it coalesced into LDS, then writes
// the channel-major [C][P][P] output coalesced over (i, j) with the optional flip/rotation folded
// into the LDS read index.
#include "common.h"

namespace {

constexpr int CT = 32;  // channels per LDS pass

struct Win {
  int W, H, P, step, ny;
};

__device__ __forceinline__ void corner(const Win& w, const int* corners, long k, int& x, int& y) {
  if (corners) {
    x = corners[2 * k];
    y = corners[2 * k + 1];
  } else {
    const long ix = k / w.ny, iy = k % w.ny;
    x = (int)min((long)w.W - w.P, ix * w.step);
    y = (int)min((long)w.H - w.P, iy * w.step);
  }
}

// output (i, j) of the transformed patch <- source (si, sj) of the window
__device__ __forceinline__ void src_of(int code, int P, int i, int j, int& si, int& sj) {
  si = i;
  sj = j;
  if (code & 3) {
    if (code & 1) sj = P - 1 - sj;  // np.fliplr: axis 1 (y)
    if (code & 2) si = P - 1 - si;  // np.flipud: axis 0 (x)
  } else {
    const int k = (code >> 2) & 3;  // np.rot90(a, k): out[i][j] = a[j][P-1-i] for k = 1
    if (k == 1) { si = j; sj = P - 1 - i; }
    else if (k == 2) { si = P - 1 - i; sj = P - 1 - j; }
    else if (k == 3) { si = P - 1 - j; sj = i; }
  }
}

__global__ __launch_bounds__(256) void patch_gather(Win w, int C, const float* __restrict__ cube,
                                                    const int* __restrict__ corners, long k0,
                                                    const unsigned char* __restrict__ xform,
                                                    float* __restrict__ out) {
  extern __shared__ float tile[];  // [P*P][CT+1]
  const int P = w.P, PP = P * P;
  const long i = blockIdx.x;
  int x, y;
  corner(w, corners, k0 + i, x, y);
  const int code = xform ? xform[i] : 0;
  float* o = out + i * (long)C * PP;
  for (int c0 = 0; c0 < C; c0 += CT) {
    const int cn = min(CT, C - c0);
    // load: for each pixel (ii, jj) the cn channels [c0, c0+cn) — consecutive threads walk channels
    for (int e = threadIdx.x; e < PP * cn; e += blockDim.x) {
      const int p = e / cn, c = e - p * cn;
      const int ii = p / P, jj = p - ii * P;
      tile[p * (CT + 1) + c] = cube[((long)(x + ii) * w.H + (y + jj)) * C + c0 + c];
    }
    __syncthreads();
    for (int e = threadIdx.x; e < cn * PP; e += blockDim.x) {
      const int c = e / PP, q = e - c * PP;
      const int oi = q / P, oj = q - oi * P;
      int si, sj;
      src_of(code, P, oi, oj, si, sj);
      o[(long)(c0 + c) * PP + q] = tile[(si * P + sj) * (CT + 1) + c];
    }
    __syncthreads();
  }
}

__global__ void center_accumulate(Win w, int ncls, const int* __restrict__ corners, long k0, int n,
                                  const float* __restrict__ logits, double* __restrict__ probs) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (long)n * ncls) return;
  const long i = e / ncls;
  const int c = (int)(e - i * ncls);
  int x, y;
  corner(w, corners, k0 + i, x, y);
  const int h = w.P / 2;
  probs[((long)(x + h) * w.H + (y + h)) * ncls + c] += (double)logits[e];
}

// number of sliding-window positions along one axis (utils.py:389-399)
long axis_count(int L, int P, int step) {
  const int off = (L - P) % step;
  return (long)((L - P + off) / step) + 1;
}

Win make_win(int W, int H, int P, int step) {
  Win w;
  w.W = W;
  w.H = H;
  w.P = P;
  w.step = step;
  w.ny = (int)axis_count(H, P, step);
  return w;
}

}  // namespace

VC_EXPORT int vc_window_count(int W, int H, int P, int step, long* count) {
  VC_REQUIRE(count && P > 0 && step > 0 && W >= P && H >= P);
  *count = axis_count(W, P, step) * axis_count(H, P, step);
  return VC_OK;
}

VC_EXPORT int vc_patch_gather(int W, int H, int C, int P, const float* cube, const int* corners, long k0, int step,
                              int n, const unsigned char* xform, float* out, hipStream_t stream) {
  VC_REQUIRE(P > 0 && C > 0 && W >= P && H >= P && n >= 0 && (corners || step > 0));
  VC_REQUIRE(P * P * (CT + 1) * 4 <= 64 * 1024);
  if (n == 0) return VC_OK;
  if (!corners) {
    long total = 0;
    vc_window_count(W, H, P, step, &total);
    VC_REQUIRE(k0 >= 0 && k0 + n <= total);
  }
  const Win w = make_win(W, H, P, corners ? 1 : step);
  hipLaunchKernelGGL(patch_gather, dim3(n), dim3(256), P * P * (CT + 1) * sizeof(float), stream, w, C, cube,
                     corners, k0, xform, out);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_EXPORT int vc_center_accumulate(int W, int H, int P, int ncls, const int* corners, long k0, int step, int n,
                                   const float* logits, double* probs, hipStream_t stream) {
  VC_REQUIRE(P > 0 && ncls > 0 && W >= P && H >= P && n >= 0 && (corners || step > 0));
  if (n == 0) return VC_OK;
  const Win w = make_win(W, H, P, corners ? 1 : step);
  const long total = (long)n * ncls;
  hipLaunchKernelGGL(center_accumulate, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, w, ncls, corners, k0, n,
                     logits, probs);
  VC_CHECK_LAUNCH();
  return VC_OK;
}
