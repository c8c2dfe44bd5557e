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

// Counter-based randomness of the noise augmentations: splitmix64 finaliser over
// (seed, global sample id, stream, element).  oracle/patch_noise_oracle.py restates it.
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ unsigned long long noise_key(unsigned long long seed, long long gid, int stream) {
  return mix64(seed ^ mix64(((unsigned long long)gid << 2) | (unsigned long long)stream));
}
// standard normal (Box-Muller on two 24-bit uniforms in (0, 1))
__device__ __forceinline__ float gauss(unsigned long long key, int e) {
  const unsigned long long r = mix64(key + (unsigned long long)e);
  const float u1 = ((float)(r >> 40) + 0.5f) * (1.f / 16777216.f);
  const float u2 = ((float)(r & 0xFFFFFFull) + 0.5f) * (1.f / 16777216.f);
  return sqrtf(-2.f * logf(u1)) * cosf(6.283185307179586f * u2);
}

// one thread per element of x (sample-major, then channel, then pixel): coalesced reads / writes of
// the patches; the mixture source spectrum is a gather of one cube row (band-contiguous) per pixel
__global__ __launch_bounds__(256) void patch_noise(int total, FastDiv fCPP, FastDiv fPP, int C, int H,
                                                   float* __restrict__ x, const float* __restrict__ lab,
                                                   const float* __restrict__ rad, const float* __restrict__ mix,
                                                   const int* __restrict__ off, const int* __restrict__ pix, int nlab,
                                                   const float* __restrict__ cube, unsigned long long seed,
                                                   long long gid0) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int PP = fPP.div;
  int rem, c, p;
  const int s = fdivmod(idx, fCPP, rem);
  c = fdivmod(rem, fPP, p);
  const float a = rad[s], a1 = mix[2 * s], a2 = mix[2 * s + 1];
  if (a == 0.f && !(a1 > 0.f)) return;
  float v = x[idx];
  const long long gid = gid0 + s;
  if (a != 0.f) v = fmaf(a, v, 0.04f * gauss(noise_key(seed, gid, 0), c * PP + p));
  if (a1 > 0.f) {
    const int lv = (int)lab[(long)s * PP + p];
    float d2 = 0.f;
    if (lv >= 0 && lv < nlab) {
      const int o0 = off[lv], cnt = off[lv + 1] - o0;
      if (cnt > 0) {
        const unsigned long long r = mix64(noise_key(seed, gid, 2) + (unsigned long long)p);
        const int j = (int)((r >> 32) % (unsigned long long)cnt);
        d2 = cube[(long)pix[o0 + j] * C + c];
      }
    }
    v = (a1 * v + a2 * d2) / (a1 + a2) + 0.04f * gauss(noise_key(seed, gid, 1), c * PP + p);
  }
  x[idx] = v;
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

VC_EXPORT int vc_patch_noise(int n, int C, int P, int H, float* x, const float* lab, const float* rad,
                             const float* mix, const int* off, const int* pix, int nlab, const float* cube,
                             unsigned long long seed, long long gid0, hipStream_t stream) {
  VC_REQUIRE(n >= 0 && C > 0 && P > 0 && H > 0 && nlab >= 0 && x && rad && mix);
  VC_REQUIRE(nlab == 0 || (lab && off && pix && cube));
  if (n == 0) return VC_OK;
  const long total = (long)n * C * P * P;
  VC_REQUIRE_I32(total);
  hipLaunchKernelGGL(patch_noise, dim3(vc_cdiv(total, 256)), dim3(256), 0, stream, (int)total,
                     make_fastdiv(C * P * P), make_fastdiv(P * P), C, H, x, lab, rad, mix, off, pix, nlab, cube, seed,
                     gid0);
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
