// LayerNorm and BatchNorm (train + eval) for channels-last activations [rows, C].
//
// LayerNorm(eps=1e-6) rows: hsiMamba pre_norm / ln1 (Mutimodality_Mamba7.py:349, :353,
// applied at :656, :985), GlobalLocalBlock ln3 / ln4 (:1069, :1073).  One wave64 per row,
// shuffle reductions, two-pass variance.
// BatchNorm2d (eps 1e-5, momentum 0.1): ms_conv_bn_relu.bn (:1039), FusionLayer BN (:1103,
// :1129), NonLocal W[1] (:113).  Train mode normalises with the biased batch variance over
// all rows (B*H*W) and updates running_var with the unbiased one; eval mode uses the
// running statistics.  Reductions are deterministic (fixed-order partials + Chan merge).
#include "common.h"

namespace {

constexpr int LN_MAXV = 8;  // C <= 512

__global__ __launch_bounds__(256) void ln_fwd(int R, int C, const float* __restrict__ x, long ldx,
                                              const float* __restrict__ w, const float* __restrict__ b, float eps,
                                              float* __restrict__ y, long ldy, float* __restrict__ mean_out,
                                              float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= R) return;
  const float* xr = x + r * ldx;
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    int c = lane + 64 * j;
    v[j] = (c < C) ? xr[c] : 0.f;
    s += v[j];
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    int c = lane + 64 * j;
    float d = (c < C) ? v[j] - mean : 0.f;
    q += d * d;
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
  float* yr = y + r * ldy;
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    int c = lane + 64 * j;
    if (c < C) yr[c] = (v[j] - mean) * rstd * w[c] + b[c];
  }
  if (lane == 0) {
    mean_out[r] = mean;
    rstd_out[r] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * w ; per-block partial dw / db
__global__ __launch_bounds__(256) void ln_bwd(int R, int C, int rows_per_block, const float* __restrict__ dy,
                                              long lddy, const float* __restrict__ x, long ldx,
                                              const float* __restrict__ w, const float* __restrict__ mean,
                                              const float* __restrict__ rstd, float* __restrict__ dx, long lddx,
                                              float beta_dx, float* __restrict__ part) {
  __shared__ float sh[4][2][512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float pw[LN_MAXV], pb[LN_MAXV];
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) pw[j] = pb[j] = 0.f;
  const long rbeg = (long)blockIdx.x * rows_per_block;
  const long rend = min((long)R, rbeg + rows_per_block);
  for (long r = rbeg + wv; r < rend; r += 4) {
    const float mu = mean[r], rs = rstd[r];
    float xh[LN_MAXV], g[LN_MAXV];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAXV; ++j) {
      int c = lane + 64 * j;
      float d = 0.f, xv = 0.f, wc = 0.f;
      if (c < C) {
        d = dy[r * lddy + c];
        xv = x[r * ldx + c];
        wc = w[c];
      }
      xh[j] = (xv - mu) * rs;
      g[j] = d * wc;
      sg += g[j];
      sgx += g[j] * xh[j];
      pw[j] += d * xh[j];
      pb[j] += d;
    }
    sg = wave_sum(sg) / C;
    sgx = wave_sum(sgx) / C;
#pragma unroll
    for (int j = 0; j < LN_MAXV; ++j) {
      int c = lane + 64 * j;
      if (c < C) {
        float v = rs * (g[j] - sg - xh[j] * sgx);
        float* p = dx + r * lddx + c;
        *p = (beta_dx != 0.f ? *p * beta_dx : 0.f) + v;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < LN_MAXV; ++j) {
    int c = lane + 64 * j;
    if (c < 512) {
      sh[wv][0][c] = pw[j];
      sh[wv][1][c] = pb[j];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = sh[0][0][c] + sh[1][0][c] + sh[2][0][c] + sh[3][0][c];
    float bb = sh[0][1][c] + sh[1][1][c] + sh[2][1][c] + sh[3][1][c];
    part[(long)blockIdx.x * 2 * C + c] = a;
    part[(long)blockIdx.x * 2 * C + C + c] = bb;
  }
}

// ---------------------------------------------------------------- BatchNorm (channels-last)
__global__ __launch_bounds__(256) void bn_stats_partial(int M, int C, const float* __restrict__ x, long ldx,
                                                        int rows_per, double* __restrict__ part) {
  __shared__ double sh[3][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = min((long)M, r0 + rows_per);
  double n = 0.0, mean = 0.0, m2 = 0.0;
  if (c < C) {
    for (long r = r0 + rl; r < r1; r += 4) {
      const double v = x[r * ldx + c];
      n += 1.0;
      const double d = v - mean;
      mean += d / n;
      m2 += d * (v - mean);
    }
  }
  sh[0][rl][cl] = n;
  sh[1][rl][cl] = mean;
  sh[2][rl][cl] = m2;
  __syncthreads();
  if (rl == 0 && c < C) {
    for (int k = 1; k < 4; ++k) welford_merge(n, mean, m2, sh[0][k][cl], sh[1][k][cl], sh[2][k][cl]);
    double* p = part + (long)blockIdx.y * 3 * C + c;
    p[0] = n;
    p[C] = mean;
    p[2 * C] = m2;
  }
}

// block = 16 channels x 16 partial lanes; each lane Chan-merges its partials, then a fixed-order
// 16-way merge in LDS
__global__ __launch_bounds__(256) void bn_stats_final(int P, int C, long M, const double* __restrict__ part, float eps,
                                                      float momentum, float* __restrict__ save_mean,
                                                      float* __restrict__ save_invstd, float* __restrict__ run_mean,
                                                      float* __restrict__ run_var) {
  __shared__ double sh[3][16][17];
  const int cl = threadIdx.x & 15, pl = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  if (c < C)
    for (int p = pl; p < P; p += 16) {
      const double* q = part + (long)p * 3 * C + c;
      welford_merge(n, mean, m2, q[0], q[C], q[2 * C]);
    }
  sh[0][pl][cl] = n;
  sh[1][pl][cl] = mean;
  sh[2][pl][cl] = m2;
  __syncthreads();
  if (pl != 0 || c >= C) return;
  for (int k = 1; k < 16; ++k) welford_merge(n, mean, m2, sh[0][k][cl], sh[1][k][cl], sh[2][k][cl]);
  const double var = m2 / (double)M;
  save_mean[c] = (float)mean;
  save_invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    const double unb = M > 1 ? m2 / (double)(M - 1) : var;
    run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * mean);
    run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
  }
}

__global__ void bn_eval_prep(int C, const float* __restrict__ run_mean, const float* __restrict__ run_var, float eps,
                             float* __restrict__ save_mean, float* __restrict__ save_invstd) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  save_mean[c] = run_mean[c];
  save_invstd[c] = rsqrtf(run_var[c] + eps);
}

__global__ void bn_apply(int total, FastDiv fC, const float* __restrict__ x, long ldx, const float* __restrict__ mean,
                         const float* __restrict__ invstd, const float* __restrict__ w, const float* __restrict__ b,
                         int relu, float* __restrict__ y, long ldy) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  int c;
  const long r = fdivmod(idx, fC, c);
  float v = (x[r * ldx + c] - mean[c]) * invstd[c] * w[c] + b[c];
  if (relu) v = fmaxf(v, 0.f);
  y[r * ldy + c] = v;
}

// partial sums of dyv and dyv*xhat,  dyv = dy * (relu_out > 0 if relu_out)
__global__ __launch_bounds__(256) void bn_bwd_partial(int M, int C, const float* __restrict__ dy, long lddy,
                                                      const float* __restrict__ x, long ldx,
                                                      const float* __restrict__ relu_out, long ldo,
                                                      const float* __restrict__ mean, const float* __restrict__ invstd,
                                                      int rows_per, double* __restrict__ part) {
  __shared__ double sh[2][4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const long r0 = (long)blockIdx.y * rows_per;
  const long r1 = min((long)M, r0 + rows_per);
  double s1 = 0.0, s2 = 0.0;
  if (c < C) {
    const float mu = mean[c], is = invstd[c];
    for (long r = r0 + rl; r < r1; r += 4) {
      float d = dy[r * lddy + c];
      if (relu_out && !(relu_out[r * ldo + c] > 0.f)) d = 0.f;
      s1 += d;
      s2 += (double)d * ((x[r * ldx + c] - mu) * is);
    }
  }
  sh[0][rl][cl] = s1;
  sh[1][rl][cl] = s2;
  __syncthreads();
  if (rl == 0 && c < C) {
    double* p = part + (long)blockIdx.y * 2 * C + c;
    p[0] = sh[0][0][cl] + sh[0][1][cl] + sh[0][2][cl] + sh[0][3][cl];
    p[C] = sh[1][0][cl] + sh[1][1][cl] + sh[1][2][cl] + sh[1][3][cl];
  }
}

// dw/db from the reduced sums (sums[0:C] = sum dyv, sums[C:2C] = sum dyv*xhat)
__global__ void bn_bwd_finish(int C, const double* __restrict__ sums, float* __restrict__ dw, float* __restrict__ db,
                              float beta_w) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  if (dw) dw[c] = (beta_w != 0.f ? beta_w * dw[c] : 0.f) + (float)sums[C + c];
  if (db) db[c] = (beta_w != 0.f ? beta_w * db[c] : 0.f) + (float)sums[c];
}

// train: dx = w*invstd*(dyv - s1/M - xhat*s2/M);  eval (sums == null): dx = w*invstd*dyv
__global__ void bn_bwd_apply(int M, FastDiv fC, const float* __restrict__ dy, long lddy, const float* __restrict__ x,
                             long ldx, const float* __restrict__ relu_out, long ldo, const float* __restrict__ mean,
                             const float* __restrict__ invstd, const float* __restrict__ w,
                             const double* __restrict__ sums, float* __restrict__ dx, long lddx, float beta_dx,
                             const double* __restrict__ red, float* __restrict__ dw, float* __restrict__ db,
                             float beta_w) {
  const int C = fC.div;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < C) {
    if (dw) dw[idx] = (beta_w != 0.f ? beta_w * dw[idx] : 0.f) + (float)red[C + idx];
    if (db) db[idx] = (beta_w != 0.f ? beta_w * db[idx] : 0.f) + (float)red[idx];
  }
  if (idx >= M * C) return;
  int c;
  const long r = fdivmod(idx, fC, c);
  float d = dy[r * lddy + c];
  if (relu_out && !(relu_out[r * ldo + c] > 0.f)) d = 0.f;
  const float is = invstd[c];
  float v;
  if (sums) {
    const float invM = 1.f / (float)M;
    const float xh = (x[r * ldx + c] - mean[c]) * is;
    v = w[c] * is * (d - (float)sums[c] * invM - xh * ((float)sums[C + c] * invM));
  } else {
    v = w[c] * is * d;
  }
  float* p = dx + r * lddx + c;
  *p = (beta_dx != 0.f ? beta_dx * *p : 0.f) + v;
}

int bn_rows_per(long M, int C, long ws_floats, int per_row_floats) {
  int rows_per = std::max<long>(32, (M + 255) / 256);
  while ((long)vc_cdiv(M, rows_per) * C * per_row_floats > ws_floats || vc_cdiv(M, rows_per) > 2048) rows_per *= 2;
  return rows_per;
}

}  // namespace

VC_EXPORT int vc_layernorm_fwd(int R, int C, const float* x, long ldx, const float* w, const float* b, float eps,
                               float* y, long ldy, float* mean, float* rstd, hipStream_t stream) {
  VC_REQUIRE(C > 0 && C <= 64 * LN_MAXV && R >= 0);
  if (R == 0) return VC_OK;
  hipLaunchKernelGGL(ln_fwd, dim3(vc_cdiv(R, 4)), dim3(256), 0, stream, R, C, x, ldx, w, b, eps, y, ldy, mean, rstd);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// dx = beta_dx*dx + LNgrad;  dw = beta_w*dw + sum dy*xhat;  db = beta_w*db + sum dy
VC_EXPORT int vc_layernorm_bwd(int R, int C, const float* dy, long lddy, const float* x, long ldx, const float* w,
                               const float* mean, const float* rstd, float* dx, long lddx, float beta_dx, float* dw,
                               float* db, float beta_w, float* ws, long ws_floats, hipStream_t stream) {
  VC_REQUIRE(C > 0 && C <= 64 * LN_MAXV && R >= 0);
  if (R == 0) return VC_OK;
  int rows_per = std::max(16, vc_cdiv(R, 256));
  while ((long)vc_cdiv(R, rows_per) * 2 * C > ws_floats) rows_per *= 2;
  const int P = vc_cdiv(R, rows_per);
  hipLaunchKernelGGL(ln_bwd, dim3(P), dim3(256), 0, stream, R, C, rows_per, dy, lddy, x, ldx, w, mean, rstd, dx,
                     lddx, beta_dx, ws);
  VC_CHECK_LAUNCH();
  if (dw && db == dw + C) return launch_sum_rows(P, 2 * C, ws, (long)2 * C, 0L, dw, beta_w, stream);  // adjacent
  if (dw) {
    int rc = launch_sum_rows(P, C, ws, (long)2 * C, 0L, dw, beta_w, stream);
    if (rc) return rc;
  }
  if (db) {
    int rc = launch_sum_rows(P, C, ws, (long)2 * C, (long)C, db, beta_w, stream);
    if (rc) return rc;
  }
  return VC_OK;
}

// Train: batch statistics -> save_mean / save_invstd, running stats updated (if run_mean).
// Eval (train == 0): save_* filled from the running statistics.
VC_EXPORT int vc_bn_stats(int train, long M, int C, const float* x, long ldx, float eps, float momentum,
                          float* save_mean, float* save_invstd, float* run_mean, float* run_var, float* ws,
                          long ws_floats, hipStream_t stream) {
  VC_REQUIRE(C > 0 && M >= 0);
  if (!train) {
    hipLaunchKernelGGL(bn_eval_prep, dim3(vc_cdiv(C, 256)), dim3(256), 0, stream, C, run_mean, run_var, eps,
                       save_mean, save_invstd);
    VC_CHECK_LAUNCH();
    return VC_OK;
  }
  VC_REQUIRE(M > 0 && ((uintptr_t)ws & 7) == 0);
  // partial (count, mean, M2) triples are fp64: the workspace holds ws_floats/2 doubles
  double* wsd = reinterpret_cast<double*>(ws);
  const long ws_doubles = ws_floats / 2;
  const int rows_per = bn_rows_per(M, C, ws_doubles, 3);
  const int P = vc_cdiv(M, rows_per);
  VC_REQUIRE((long)P * C * 3 <= ws_doubles);
  hipLaunchKernelGGL(bn_stats_partial, dim3(vc_cdiv(C, 64), P), dim3(256), 0, stream, (int)M, C, x, ldx, rows_per,
                     wsd);
  VC_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_stats_final, dim3(vc_cdiv(C, 16)), dim3(256), 0, stream, P, C, M, wsd, eps, momentum,
                     save_mean, save_invstd, run_mean, run_var);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_EXPORT int vc_bn_apply(long M, int C, const float* x, long ldx, const float* mean, const float* invstd,
                          const float* w, const float* b, int relu, float* y, long ldy, hipStream_t stream) {
  VC_REQUIRE(C > 0 && M >= 0);
  if (M == 0) return VC_OK;
  VC_REQUIRE_I32(M * C);
  hipLaunchKernelGGL(bn_apply, dim3(vc_cdiv(M * C, 256)), dim3(256), 0, stream, (int)(M * C), make_fastdiv(C), x, ldx,
                     mean, invstd, w, b,
                     relu, y, ldy);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

// BN backward (optionally through a following ReLU whose output is relu_out).
// dx = beta_dx*dx + ...;  dw/db = beta_w*dw/db + ... (either may be null).
VC_EXPORT int vc_bn_bwd(int train, long M, int C, const float* dy, long lddy, const float* x, long ldx,
                        const float* relu_out, long ldo, const float* mean, const float* invstd, const float* w,
                        float* dx, long lddx, float beta_dx, float* dw, float* db, float beta_w, float* ws,
                        long ws_floats, hipStream_t stream) {
  VC_REQUIRE(C > 0 && M > 0 && ((uintptr_t)ws & 7) == 0);
  // per-row-block partial sums [P][2][C] and the final [2][C] sums are fp64
  double* wsd = reinterpret_cast<double*>(ws);
  const long ws_doubles = ws_floats / 2;
  const int rows_per = bn_rows_per(M, C, ws_doubles - 2L * C, 2);
  const int P = vc_cdiv(M, rows_per);
  VC_REQUIRE((long)P * C * 2 + 2L * C <= ws_doubles);
  double* sums = wsd + (long)P * C * 2;
  hipLaunchKernelGGL(bn_bwd_partial, dim3(vc_cdiv(C, 64), P), dim3(256), 0, stream, (int)M, C, dy, lddy, x, ldx,
                     relu_out, ldo, mean, invstd, rows_per, wsd);
  VC_CHECK_LAUNCH();
  // one pass over the [P][2C] partials gives both sums (sum dy, sum dy*xhat)
  hipLaunchKernelGGL(sum_rows_d_kernel, dim3(vc_cdiv(2L * C, 16)), dim3(256), 0, stream, P, 2 * C, wsd, 2L * C, 0L,
                     sums);
  VC_CHECK_LAUNCH();
  if (dx) {
    VC_REQUIRE_I32(M * C);
    hipLaunchKernelGGL(bn_bwd_apply, dim3(vc_cdiv(std::max<long>(M * C, C), 256)), dim3(256), 0, stream, (int)M,
                       make_fastdiv(C), dy,
                       lddy, x, ldx, relu_out, ldo, mean, invstd, w, train ? sums : (const double*)nullptr, dx, lddx,
                       beta_dx, sums, dw, db, beta_w);
    VC_CHECK_LAUNCH();
  } else {
    hipLaunchKernelGGL(bn_bwd_finish, dim3(vc_cdiv(C, 256)), dim3(256), 0, stream, C, sums, dw, db, beta_w);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}
