// FusAtNet's 3x3 convolutions (stride 1, padding 0 or 1; FusAtNet.py:10-62 ConvUnit / ConvUnit_NP /
// Residual_Unit, :168-186) as implicit GEMMs over a TAP-MAJOR contraction index k = tap * C + c.
//
// The im2col formulation (vc_im2col3x3_pad + vc_gemm) orders k channel-major (c * 9 + tap, the
// torch weight layout), so every k-tile of the col matrix mixes channels and taps and has to be
// materialised: for the 2193-channel concat of the fusion module that is 611 MB written and read
// per conv, plus a col2im scatter in the backward.  With k tap-major, a k-tile of 32 consecutive k
// is 32 consecutive channels of ONE tap, i.e. for every output pixel a contiguous 128-B piece of
// one channels-last input row: the operand tile is a row GATHER with one address per row and tap,
// loaded as float4s like a plain matrix.  No col matrix and no col2im: the data gradient is the
// same gather over the output gradient with the mirrored tap offsets.  The weights are repacked
// tap-major once per step (vc_conv3x3_pack); the backward reads the same repacked copy.
//
//   fwd   : y[p][o]        = b[o] + sum_{tap,c} x[in(p,tap)][c] Wt[o][tap][c]      M = pixels, N = O,  K = 9C
//   wgrad : dWt[o][tap][c] = sum_p dy[p][o] x[in(p,tap)][c]                        M = O, N = 9C,      K = pixels
//   dgrad : dx[q][c]      (+)= sum_{tap,o} dy[out(q,tap)][o] Wt[o][tap][c]         M = pixels, N = C,  K = 9O
//
// Block = 256 threads = 4 waves (2 x 2) over a 128 x 128 output tile, each wave 64 x 64 = 2 x 2
// tiles of v_mfma_f32_32x32x2_f32 (f32 operands, exact f32 fma chains; 64-cycle issue; four
// independent accumulators per wave).  k-tiles of 32 go through LDS as k-major images [k][row], so a
// fragment read is 32 consecutive rows per half-wave (conflict-free): operands whose source rows are
// k-contiguous are transposed by scalar stores into a pitch-129 image (a 32-lane group's 8 k-chunks x
// 4 rows land in 32 distinct banks), k-outer sources are stored as float4s into a pitch-132 image.
// One register set of the next k-tile's loads is in flight behind the MFMAs.  Against the 64 x 64
// im2col GEMM the 128 x 128 tile halves the operand bytes per flop (the long-K convs were
// operand-bandwidth-bound at ~50 TF/s).
#include "common.h"
#include "mfma_tiles.h"

#include <algorithm>

namespace {

constexpr int TM = 128, TN = 128, TK = 32;
constexpr int PK = 129;   // LDS pitch of images transposed from k-contiguous rows
constexpr int PO = 132;   // LDS pitch of images stored from k-outer rows

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { FWD = 0, WGRAD = 1, DGRAD = 2 };

struct TapArgs {
  int nb;                  // batch
  int H, W, C, O, pad, OH, OW;
  int Cw;                  // Wt row pitch per tap: C rounded up to 4 (zero padding)
  int M, N;                // GEMM output extents (N: total output columns; wgrad 9C)
  int P;                   // wgrad: number of output pixels (the contraction)
  int nk;                  // k-tiles in all
  int tpt;                 // fwd / dgrad: k-tiles per tap; wgrad: n-tiles per tap
  int kper;                // k-tiles per split slice
  const float* x;  long ldx;     // input activations (fwd, wgrad), channels-last rows
  const float* dy; long lddy;    // output gradient (wgrad, dgrad), channels-last rows
  const float* w;                // Wt [O][9][C] (fwd, dgrad)
  const float* bias;             // fwd (optional)
  float* out; long ldo;          // fwd: y [M][ldo]; wgrad: dWt [O][9C] (ldo = 9C); dgrad: dx [M][ldo]
  float beta;                    // dgrad: dx = beta dx + ...
  float* part;                   // split-K slabs [nsplit][M][N]
  int oihw;                      // wgrad: out is the torch layout [O][C][3][3] (else dWt [O][9C])
  float* dbias;                  // wgrad (nullable): the bias gradient sum_p dy[p][o], from the n-tile-0
                                 // blocks' staged dy tiles (split: column 9C of the slabs, a.N = 9C + 1)
  int vx, vdy, vw;               // float4 loads allowed (16-B aligned base, ld % 4 == 0)
  FastDiv fOW, fOHW, fW, fHW;
};

__device__ __forceinline__ int tap_di(int tap) { return tap >= 6 ? 2 : (tap >= 3 ? 1 : 0); }

// the output-pixel decomposition (fwd rows, wgrad k) and the input-pixel one (dgrad rows)
__device__ __forceinline__ void split_out(const TapArgs& a, int p, int& b, int& i, int& j) {
  int r1;
  b = fdivmod(p, a.fOHW, r1);
  i = fdivmod(r1, a.fOW, j);
}
__device__ __forceinline__ void split_in(const TapArgs& a, int q, int& b, int& i, int& j) {
  int r1;
  b = fdivmod(q, a.fHW, r1);
  i = fdivmod(r1, a.fW, j);
}
// input row of output pixel (b, i, j) through tap t, -1 outside the (padded) image
__device__ __forceinline__ int in_row(const TapArgs& a, int b, int i, int j, int tap) {
  const int di = tap_di(tap), dj = tap - 3 * di;
  const int y = i + di - a.pad, x = j + dj - a.pad;
  return (b >= 0 && y >= 0 && y < a.H && x >= 0 && x < a.W) ? (b * a.H + y) * a.W + x : -1;
}
// output row reading input pixel (b, i, j) through tap t, -1 if none
__device__ __forceinline__ int out_row(const TapArgs& a, int b, int i, int j, int tap) {
  const int di = tap_di(tap), dj = tap - 3 * di;
  const int y = i - di + a.pad, x = j - dj + a.pad;
  return (b >= 0 && y >= 0 && y < a.OH && x >= 0 && x < a.OW) ? (b * a.OH + y) * a.OW + x : -1;
}

// 4 consecutive floats of row `row` (ld `ld`) from column c, columns >= cend read 0; row < 0 -> 0
__device__ __forceinline__ void load4(const float* base, long ld, int row, int c, int cend, bool vec, float* v) {
  if (row < 0) {
    v[0] = v[1] = v[2] = v[3] = 0.f;
    return;
  }
  const float* p = base + (long)row * ld + c;
  if (vec && c + 3 < cend) {
    const float4 q = *reinterpret_cast<const float4*>(p);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = c + e < cend ? p[e] : 0.f;
  }
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void conv_tap(TapArgs a) {
  constexpr int PA = MODE == WGRAD ? PO : PK;   // A: dy^T (k-outer) for wgrad, row gathers (k-contiguous) else
  constexpr int PB = MODE == FWD ? PK : PO;     // B: Wt rows (k-contiguous) for fwd, k-outer else
  __shared__ __attribute__((aligned(16))) float As[TK * PA];
  __shared__ __attribute__((aligned(16))) float Bs[TK * PB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1, l31 = lane & 31, h = lane >> 5;
  const int m0 = blockIdx.y * TM;
  const int nt = blockIdx.x;
  const int kt0 = blockIdx.z * a.kper, kt1 = min(a.nk, kt0 + a.kper);
  const int ntap = MODE == WGRAD ? nt / a.tpt : 0;                       // wgrad: the n-tile's tap
  const int n0 = MODE == WGRAD ? (nt - ntap * a.tpt) * TN : nt * TN;      // first channel / column
  const int Kt = MODE == FWD ? a.C : a.O;                                  // per-tap k extent (fwd, dgrad)

  // k-contiguous staging: rows kr + 32 i, k-chunk kc (4 consecutive k); k-outer staging: k rows
  // ok + 8 i, column chunk oc (4 consecutive columns)
  const int kr = tid >> 3, kc = tid & 7;
  const int ok = tid >> 5, oc = tid & 31;
  // fwd / dgrad: this thread's 4 gathered A rows, decomposed once (b = -1: past the last row)
  int rb_[4], ri_[4], rj_[4];
  if constexpr (MODE != WGRAD) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = m0 + kr + 32 * i;
      if (r < a.M) {
        if (MODE == FWD) split_out(a, r, rb_[i], ri_[i], rj_[i]);
        else split_in(a, r, rb_[i], ri_[i], rj_[i]);
      } else {
        rb_[i] = -1; ri_[i] = rj_[i] = 0;
      }
    }
  }

  float ra[16], rbv[16];
  auto load = [&](int kt) {
    if constexpr (MODE == WGRAD) {
      const int p0 = kt * TK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = p0 + ok + 8 * i;
        // A(m = o, k = p) = dy[p][o]
        load4(a.dy, a.lddy, p < a.P ? p : -1, m0 + 4 * oc, a.O, a.vdy, ra + 4 * i);
        // B(k = p, n = (tap, c)) = x[in(p, tap)][c]
        int row = -1;
        if (p < a.P) {
          int b, y, x;
          split_out(a, p, b, y, x);
          row = in_row(a, b, y, x, ntap);
        }
        load4(a.x, a.ldx, row, n0 + 4 * oc, a.C, a.vx, rbv + 4 * i);
      }
    } else {
      const int tap = kt / a.tpt, c0 = (kt - tap * a.tpt) * TK;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (MODE == FWD) {
          const int row = in_row(a, rb_[i], ri_[i], rj_[i], tap);
          load4(a.x, a.ldx, row, c0 + 4 * kc, Kt, a.vx, ra + 4 * i);
          // B(k = (tap, c), n = o) = Wt[o][tap][c]: rows o = n0 + kr + 32 i
          const int o = n0 + kr + 32 * i;
          load4(a.w + (long)tap * a.Cw, 9L * a.Cw, o < a.O ? o : -1, c0 + 4 * kc, a.Cw, a.vw, rbv + 4 * i);
        } else {
          const int row = out_row(a, rb_[i], ri_[i], rj_[i], tap);
          load4(a.dy, a.lddy, row, c0 + 4 * kc, Kt, a.vdy, ra + 4 * i);
          // B(k = (tap, o), n = c) = Wt[o][tap][c] (the forward's layout read with row stride 9 Cw):
          // k rows o = c0 + ok + 8 i
          const int o = c0 + ok + 8 * i;
          load4(a.w + (long)tap * a.Cw, 9L * a.Cw, o < a.O ? o : -1, n0 + 4 * oc, a.Cw, a.vw, rbv + 4 * i);
        }
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (MODE == WGRAD) {
        *reinterpret_cast<float4*>(As + (ok + 8 * i) * PA + 4 * oc) =
            make_float4(ra[4 * i], ra[4 * i + 1], ra[4 * i + 2], ra[4 * i + 3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) As[(4 * kc + e) * PA + kr + 32 * i] = ra[4 * i + e];
      }
      if constexpr (MODE == FWD) {
#pragma unroll
        for (int e = 0; e < 4; ++e) Bs[(4 * kc + e) * PB + kr + 32 * i] = rbv[4 * i + e];
      } else {
        *reinterpret_cast<float4*>(Bs + (ok + 8 * i) * PB + 4 * oc) =
            make_float4(rbv[4 * i], rbv[4 * i + 1], rbv[4 * i + 2], rbv[4 * i + 3]);
      }
    }
  };

  // wgrad bias gradient: the blocks of n-tile 0 also sum their staged dy^T tile over k (thread: output
  // row tid & 127, k half tid >> 7; fixed order: k within the half, k-tiles in order, then the halves)
  const bool do_b = MODE == WGRAD && a.dbias && blockIdx.x == 0;
  float bacc = 0.f;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (kt0 < kt1) {
    load(kt0);
    for (int kt = kt0; kt < kt1; ++kt) {
      store();
      __syncthreads();
      if (kt + 1 < kt1) load(kt + 1);
      if (do_b) {
        const int mm = tid & 127, hh = tid >> 7;
#pragma unroll
        for (int k = 0; k < TK / 2; ++k) bacc += As[(hh * (TK / 2) + k) * PA + mm];
      }
#pragma unroll
      for (int ks = 0; ks < TK / 2; ++ks) {
        const int k = 2 * ks + h;
        const float a0 = As[k * PA + wm * 64 + l31];
        const float a1 = As[k * PA + wm * 64 + 32 + l31];
        const float b0 = Bs[k * PB + wn * 64 + l31];
        const float b1 = Bs[k * PB + wn * 64 + 32 + l31];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
      }
      __syncthreads();
    }
  }

  // C/D of 32x32: column = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  const bool split = gridDim.z > 1;
  if (do_b) {   // (block-uniform) the two k halves combined through the idle B image
    const int mm = tid & 127, hh = tid >> 7;
    if (hh == 1) Bs[mm] = bacc;
    __syncthreads();
    const int row = m0 + mm;
    if (hh == 0 && row < a.M) {
      const float v = bacc + Bs[mm];
      if (split) a.part[((long)blockIdx.z * a.M + row) * a.N + 9 * a.C] = v;
      else a.dbias[row] = v;
    }
  }
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      // one 32x32 accumulator at a time: the data gradient's read of dx (beta) is not batched over
      // all 64 outputs (that raised the kernel past 3 waves per SIMD)
      asm volatile("" ::: "memory");
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 64 + mi * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int cl = n0 + wn * 64 + ni * 32 + l31;         // column within the tile's range
        int col;
        bool ok_ = row < a.M;
        if (MODE == WGRAD) {
          ok_ = ok_ && cl < a.C;
          col = ntap * a.C + cl;
        } else {
          ok_ = ok_ && cl < (MODE == FWD ? a.O : a.C);
          col = cl;
        }
        if (!ok_) continue;
        const float v = acc[mi][ni][r];
        if (split) {
          a.part[((long)blockIdx.z * a.M + row) * a.N + col] = v;
        } else if (MODE == WGRAD && a.oihw) {
          a.out[((long)row * a.C + cl) * 9 + ntap] = v;
        } else {
          float* o = a.out + (long)row * a.ldo + col;
          if (MODE == FWD) *o = v + (a.bias ? a.bias[col] : 0.f);
          else if (MODE == DGRAD) *o = (a.beta != 0.f ? a.beta * *o : 0.f) + v;
          else *o = v;
        }
      }
    }
}

// one combined element: the mode's epilogue
template <int MODE>
__device__ __forceinline__ void tap_reduce_store(const TapArgs& a, long e, float s) {
  const int row = (int)(e / a.N), col = (int)(e - (long)row * a.N);
  if (MODE == WGRAD && col == 9 * a.C) {   // the bias-gradient column (a.N = 9C + 1)
    a.dbias[row] = s;
    return;
  }
  if (MODE == WGRAD && a.oihw) {   // torch layout [O][C][3][3]: col = tap * C + c
    const int tap = col / a.C, c = col - tap * a.C;
    a.out[((long)row * a.C + c) * 9 + tap] = s;
    return;
  }
  float* o = a.out + (long)row * a.ldo + col;
  if (MODE == FWD) *o = s + (a.bias ? a.bias[col] : 0.f);
  else if (MODE == DGRAD) *o = (a.beta != 0.f ? a.beta * *o : 0.f) + s;
  else *o = s;
}

// split-K combine in fixed slice order, then the mode's epilogue.  vec: a thread sums 4 consecutive
// elements of the flattened [M][N] slabs as float4s (slab size and workspace 16-B aligned), else one
template <int MODE>
__global__ __launch_bounds__(256) void conv_tap_reduce(TapArgs a, int nsplit, int vec) {
  const long slab = (long)a.M * a.N;
  if (vec) {
    const long e0 = ((long)blockIdx.x * 256 + threadIdx.x) * 4;
    if (e0 >= slab) return;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 8
    for (int z = 0; z < nsplit; ++z) {   // 8 slab loads in flight, each element summed in z order
      const float4 v = *reinterpret_cast<const float4*>(a.part + z * slab + e0);
      s.x += v.x;
      s.y += v.y;
      s.z += v.z;
      s.w += v.w;
    }
    const float sv[4] = {s.x, s.y, s.z, s.w};
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (e0 + i < slab) tap_reduce_store<MODE>(a, e0 + i, sv[i]);
    return;
  }
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= slab) return;
  float s = 0.f;
#pragma unroll 8
  for (int z = 0; z < nsplit; ++z) s += a.part[z * slab + e];   // 8 slab loads in flight, summed in z order
  tap_reduce_store<MODE>(a, e, s);
}

// weight layouts: w [O][C][9] (torch) -> Wt [O][9][Cw] (mode 0; Cw = C rounded up to 4, zero padding, so
// the fwd / dgrad weight rows are 16-B aligned and load as float4 at any C) / W2 [9][O][C] (mode 1);
// mode 2: w = beta w + unpack(dWt [O][9][C])
__global__ __launch_bounds__(256) void conv_pack(int O, int C, int mode, const float* __restrict__ src,
                                                 float* __restrict__ dst, float beta) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (mode == 0) {   // e indexes Wt [O][9][Cw]: a gather from the torch layout, padding columns 0
    const int Cw = (C + 3) & ~3;
    if (e >= (long)O * 9 * Cw) return;
    const int c = (int)(e % Cw);
    const long ot = e / Cw;
    const int tap = (int)(ot % 9), o = (int)(ot / 9);
    dst[e] = c < C ? src[((long)o * C + c) * 9 + tap] : 0.f;
    return;
  }
  const long n = (long)O * C * 9;
  if (e >= n) return;
  // e indexes the torch layout: o, c, tap
  const int tap = (int)(e % 9);
  const long oc_ = e / 9;
  const int c = (int)(oc_ % C), o = (int)(oc_ / C);
  if (mode == 1) dst[((long)tap * O + o) * C + c] = src[e];
  else dst[e] = (beta != 0.f ? beta * dst[e] : 0.f) + src[((long)o * 9 + tap) * C + c];
}

// mode-0 packs of up to PACK_MAX convs in one launch: conv i owns blocks [start[i], start[i + 1]) of the
// 1-D grid (256 elements of its Wt [O][9][Cw] each), the same element map as conv_pack mode 0
constexpr int PACK_MAX = 48;
struct PackMany {
  int n;
  int start[PACK_MAX + 1];
  int O[PACK_MAX], C[PACK_MAX];
  const float* src[PACK_MAX];
  float* dst[PACK_MAX];
};

// thread -> (o, c): its 9 taps are 36 contiguous source bytes (a wave reads one contiguous run) and 9
// stores at consecutive c (each a contiguous wave run)
__global__ __launch_bounds__(256) void conv_pack_many(PackMany P) {
  const int b = blockIdx.x;
  int i = 0;
  for (int k = 1; k < P.n; ++k)
    if (b >= P.start[k]) i = k;
  const int O = P.O[i], C = P.C[i], Cw = (C + 3) & ~3;
  const long e = (long)(b - P.start[i]) * 256 + threadIdx.x;
  if (e >= (long)O * Cw) return;
  const int c = (int)(e % Cw), o = (int)(e / Cw);
  float v[9];
  const float* s = P.src[i] + ((long)o * C + c) * 9;
#pragma unroll
  for (int t = 0; t < 9; ++t) v[t] = c < C ? s[t] : 0.f;
  float* d = P.dst[i] + (long)o * 9 * Cw + c;
#pragma unroll
  for (int t = 0; t < 9; ++t) d[(long)t * Cw] = v[t];
}

// ---- conv_pipe: the same three implicit GEMMs on the LDS-DMA pipeline of the GEMM kernels (gemm.hip
// gp::gemm_pipe, mfma_tiles.h): 64 x 64 output tiles on 4 waves, a 2-stage ring of 32-wide k-tiles filled
// by buffer_load ... lds (one 16-B chunk per lane, no register staging, no LDS transposes), counted vmcnt
// waits, one barrier per k-tile, v_mfma_f32_16x16x4_f32.  The gathers become per-lane DMA offsets: a
// K-contiguous image row is one gathered input / output-gradient row (FWD / DGRAD A) or a weight row (FWD B);
// a row-contiguous image k-row is one dy row (WGRAD A), one gathered input row (WGRAD B) or a weight row
// (DGRAD B).  Rows outside the (padded) image, channels past C / O and pixels past the slice get an offset
// past the buffer's end: the DMA writes zeros.  Needs C, O, ldx, lddy multiples of 4 and 16-B aligned bases
// (otherwise conv_tap above).  On FusAtNet-sized products the pipelined GEMM runs at 100-110 TF/s against
// conv_tap's 77-91 (tools/gemm_one.py, round 4).
constexpr int CP_B = 64;   // output tile (both sides)

// NW = 8 (round 5): the tile on 2 x 4 waves of 32 x 16 (two waves per SIMD, one DMA piece per operand per wave),
// as gemm.hip's pipelined kernel
template <int MODE, int NW = 4>
__global__ __launch_bounds__(64 * NW) void conv_pipe(TapArgs a, int tn, int nsplit, unsigned total) {
  constexpr int BM = CP_B, BN = CP_B, WN = NW / 2, NS = 2, QN = 8 / NW;
  constexpr int WTM = BM / 2, WTN = BN / WN, MT = WTM / 16, NT = WTN / 16;
  constexpr int SA_B = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int LOADS = (BM / 8 + BN / 8) / NW;
  constexpr bool TA = MODE == WGRAD;   // A image [k][m] (row-contiguous) for the weight gradient
  constexpr bool TB = MODE != FWD;     // B image [k][n] for the data and weight gradients
  typedef g2::Stage<false, TA, BM, false> SA;
  typedef g2::Stage<false, TB, BN, false> SB;
  __shared__ __attribute__((aligned(1024))) char smem[gp::ring_bytes<BM, BN, NS>()];
  __shared__ float bsh[NW][64];
  int zs, xn, ym, zb;
  const int tm = (a.M + BM - 1) / BM;
  gp::tile_coords(gp::xcd_linear(blockIdx.x, total), nsplit, tn, tm, 1, zs, xn, ym, zb);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int m0 = ym * BM;
  const int ntap = MODE == WGRAD ? xn / a.tpt : 0;
  const int n0 = MODE == WGRAD ? (xn - ntap * a.tpt) * BN : xn * BN;
  const int kt0 = zs * a.kper, kt1 = min(a.nk, kt0 + a.kper);
  const unsigned OOB = gp::OOB;
  const long in_rows = (long)a.nb * a.H * a.W, out_rows = (long)a.nb * a.OH * a.OW;
  const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.x), (short)0,
                                                    a.x ? (int)(in_rows * a.ldx * 4) : 0, 0x00020000);
  const auto rdy = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.dy), (short)0,
                                                     a.dy ? (int)(out_rows * a.lddy * 4) : 0, 0x00020000);
  const auto rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.w), (short)0,
                                                    a.w ? (int)((long)a.O * 9 * a.Cw * 4) : 0, 0x00020000);
  // K-contiguous fills (FWD A / B, DGRAD A): this lane's two image rows, decomposed once
  int kb_[QN], ki_[QN], kj_[QN];
  bool kok_[QN];
  if constexpr (MODE != WGRAD) {
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      const int rloc = 8 * (wave + NW * q) + (lane >> 3);
      const int m = m0 + rloc;
      kok_[q] = m < a.M;
      if (MODE == FWD) split_out(a, kok_[q] ? m : 0, kb_[q], ki_[q], kj_[q]);
      else split_in(a, kok_[q] ? m : 0, kb_[q], ki_[q], kj_[q]);
    }
  }
  auto issue = [&](int t) {
    char* st = smem + (t % NS) * STAGE;
    const int kt = kt0 + t;
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      const int i = wave + NW * q;   // wave-instruction: 1 KB of each image
      // K-contiguous chunk coordinates
      const int rloc = 8 * i + (lane >> 3), kk = 4 * ((lane & 7) ^ ((rloc >> 1) & 7));
      // row-contiguous chunk coordinates (4 k-rows x 16 chunks per instruction)
      const int kr = 4 * i + (lane >> 4), sq = lane & 15;
      const int col = (((sq >> 2) ^ ((kr >> 2) & 1)) << 4) + ((sq & 3) << 2);
      unsigned va, vb;
      if constexpr (MODE == FWD) {
        const int tap = kt / a.tpt, c = (kt - tap * a.tpt) * 32 + kk;
        const int row = in_row(a, kb_[q], ki_[q], kj_[q], tap);
        va = (kok_[q] && row >= 0 && c < a.C) ? (unsigned)(((long)row * a.ldx + c) * 4) : OOB;
        const int o = n0 + rloc;
        vb = (o < a.O && c < a.Cw) ? (unsigned)(((long)o * 9 * a.Cw + (long)tap * a.Cw + c) * 4) : OOB;
      } else if constexpr (MODE == DGRAD) {
        const int tap = kt / a.tpt, o0 = (kt - tap * a.tpt) * 32;
        const int row = out_row(a, kb_[q], ki_[q], kj_[q], tap), o = o0 + kk;
        va = (kok_[q] && row >= 0 && o < a.O) ? (unsigned)(((long)row * a.lddy + o) * 4) : OOB;
        const int ob = o0 + kr, c = n0 + col;
        vb = (ob < a.O && c < a.Cw) ? (unsigned)(((long)ob * 9 * a.Cw + (long)tap * a.Cw + c) * 4) : OOB;
      } else {
        const int p = kt * 32 + kr, o = m0 + col, c = n0 + col;
        va = (p < a.P && o < a.O) ? (unsigned)(((long)p * a.lddy + o) * 4) : OOB;
        int row = -1;
        if (p < a.P) {
          int b, y, x;
          split_out(a, p, b, y, x);
          row = in_row(a, b, y, x, ntap);
        }
        vb = (row >= 0 && c < a.C) ? (unsigned)(((long)row * a.ldx + c) * 4) : OOB;
      }
      if constexpr (MODE == WGRAD) gp::dma16(rdy, st + i * 1024, va);
      else if constexpr (MODE == FWD) gp::dma16(rx, st + i * 1024, va);
      else gp::dma16(rdy, st + i * 1024, va);
      if constexpr (MODE == FWD) gp::dma16(rw, st + SA_B + i * 1024, vb);
      else if constexpr (MODE == DGRAD) gp::dma16(rw, st + SA_B + i * 1024, vb);
      else gp::dma16(rx, st + SA_B + i * 1024, vb);
    }
  };
  f32x4 acc[1][MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[0][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // weight gradient's bias column: the n-tile-0 blocks sum their staged dy tile (A, [k][m]) over k --
  // thread (m = tid & 63, k quarter tid >> 6), k-tiles in order, the quarters in order at the end
  const bool do_b = MODE == WGRAD && a.dbias && xn == 0;
  float bacc = 0.f;
  const int nk = kt1 > kt0 ? kt1 - kt0 : 0;
  if (nk > 0) issue(0);
  for (int t = 0; t < nk; ++t) {
    gp::vm_wait<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of the slot refilled below
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + 1 < nk) issue(t + 1);
    const char* cur = smem + (t % NS) * STAGE;
    if (do_b) {
      const int mm = tid & 63, kq = tid >> 6;
#pragma unroll
      for (int k = 0; k < 32 / NW; ++k)
        bacc += *reinterpret_cast<const float*>(cur + SA::rc_off((32 / NW) * kq + k, mm));
    }
    g2::mma_ktile<false, MT, NT, SA, SB, 1>(cur, cur + SA_B, wm * WTM, wn * WTN, lane, acc);
  }
  (void)LOADS;
  const bool split = nsplit > 1;
  if (do_b) {
    const int mm = tid & 63, kq = tid >> 6;
    bsh[kq][mm] = bacc;
    __syncthreads();
    const int row = m0 + mm;
    if (kq == 0 && row < a.M) {
      float v = bsh[0][mm];
#pragma unroll
      for (int w2 = 1; w2 < NW; ++w2) v += bsh[w2][mm];   // the k groups in order
      if (split) a.part[((long)zs * a.M + row) * a.N + 9 * a.C] = v;
      else a.dbias[row] = v;
    }
  }
  // C/D map of the 16x16 MFMAs: col = lane & 15, row = (lane >> 4) * 4 + r
#pragma unroll
  for (int mi = 0; mi < MT; ++mi)
#pragma unroll
    for (int ni = 0; ni < NT; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * WTM + mi * 16 + (lane >> 4) * 4 + r;
        const int nl = n0 + wn * WTN + ni * 16 + (lane & 15);
        const int nmax = MODE == FWD ? a.O : a.C;
        if (m >= a.M || nl >= nmax) continue;
        const float v = acc[0][mi][ni][r];
        const int col = MODE == WGRAD ? ntap * a.C + nl : nl;
        if (split) {
          a.part[((long)zs * a.M + m) * a.N + col] = v;
        } else if (MODE == WGRAD && a.oihw) {
          a.out[((long)m * a.C + nl) * 9 + ntap] = v;
        } else {
          float* o = a.out + (long)m * a.ldo + col;
          if (MODE == FWD) *o = v + (a.bias ? a.bias[col] : 0.f);
          else if (MODE == DGRAD) *o = (a.beta != 0.f ? a.beta * *o : 0.f) + v;
          else *o = v;
        }
      }
}

bool vec_ok(const float* p, long ld) { return p && ((uintptr_t)p % 16 == 0) && (ld % 4 == 0); }

template <int MODE>
int launch_tap(TapArgs& a, int grid_n, int grid_m, float* ws, long ws_floats, hipStream_t stream) {
  // split K so the grid fills one round of resident blocks (256 CUs x 3 blocks: 164 VGPRs, 34 KB LDS)
  // without a ragged second round; slices of >= 4 k-tiles; the slabs must fit the workspace
  const long tiles = (long)grid_n * grid_m;
  int nsplit = 1;
  if (vc_knob("VITCNN_TAP_NOSPLIT", 0)) ws = nullptr;
  const long target = vc_knob("VITCNN_TAP_TARGET", 768);   // blocks the split aims at (knob: probe library)
  if (ws && tiles < target && a.nk >= 8) {
    nsplit = (int)std::max<long>(1, std::min<long>(target / tiles, a.nk / 4));
    while (nsplit > 1 && (long)nsplit * a.M * a.N > ws_floats) --nsplit;
  }
  a.kper = vc_cdiv(a.nk, nsplit);
  nsplit = vc_cdiv(a.nk, a.kper);
  a.part = nsplit > 1 ? ws : nullptr;
  VC_REQUIRE(grid_m < 65536 && nsplit < 65536);
  hipLaunchKernelGGL(conv_tap<MODE>, dim3(grid_n, grid_m, nsplit), dim3(256), 0, stream, a);
  VC_CHECK_LAUNCH();
  if (nsplit > 1) {
    const long n = (long)a.M * a.N;
    const int vec = (n % 4 == 0) && ((uintptr_t)ws % 16 == 0);
    hipLaunchKernelGGL(conv_tap_reduce<MODE>, dim3(vc_cdiv(vec ? n / 4 : n, 256)), dim3(256), 0, stream, a, nsplit,
                       vec);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

// the pipelined kernel's launch: split K (slices of >= 4 k-tiles, towards ~512 blocks) only for grids
// of < 128 tiles -- the plan of gemm.hip's plan_pipe; the same split-K combine as conv_tap
template <int MODE>
int launch_conv_pipe(TapArgs& a, int grid_n, float* ws, long ws_floats, hipStream_t stream) {
  const int tm = vc_cdiv(a.M, CP_B);
  const long tiles = (long)grid_n * tm;
  int nsplit = 1;
  // grids smaller than this split K (knobs; per direction).  Forward / data gradient 512, weight gradient 1024:
  // FusAtNet's B=64 step 17.20 -> 17.07 ms against 1024 for all three (profiles/r06_ab_conv_pipe_tiles.log)
  static const char* const knob[3] = {"VITCNN_CONV_PIPE_TILES_F", "VITCNN_CONV_PIPE_TILES_W", "VITCNN_CONV_PIPE_TILES_D"};
  static const long below_default[3] = {512, 1024, 512};
  const long below = vc_knob(knob[MODE], below_default[MODE]);
  if (ws && tiles < below)
    nsplit = (int)std::max<long>(1, std::min<long>(std::min<long>((4 * below + tiles - 1) / tiles, a.nk / 4), 64));
  while (nsplit > 1 && (long)nsplit * a.M * a.N > ws_floats) --nsplit;
  a.kper = vc_cdiv(a.nk, nsplit);
  nsplit = vc_cdiv(a.nk, a.kper);
  a.part = nsplit > 1 ? ws : nullptr;
  const long total = tiles * nsplit;
  VC_REQUIRE(total < (1L << 31));
  if (vc_knob("VITCNN_CONV_PIPE_W8", 1))   // 8 waves (knob: probe library)
    hipLaunchKernelGGL((conv_pipe<MODE, 8>), dim3((unsigned)total), dim3(512), 0, stream, a, grid_n, nsplit,
                       (unsigned)total);
  else
    hipLaunchKernelGGL((conv_pipe<MODE, 4>), dim3((unsigned)total), dim3(256), 0, stream, a, grid_n, nsplit,
                       (unsigned)total);
  VC_CHECK_LAUNCH();
  if (nsplit > 1) {
    const long n = (long)a.M * a.N;
    const int vec = (n % 4 == 0) && ((uintptr_t)ws % 16 == 0);
    hipLaunchKernelGGL(conv_tap_reduce<MODE>, dim3(vc_cdiv(vec ? n / 4 : n, 256)), dim3(256), 0, stream, a, nsplit,
                       vec);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

// can the pipelined kernel take this conv: whole 16-B chunks everywhere (O and the leading dimensions multiples
// of 4, 16-B aligned bases) and operands under 2 GB (32-bit buffer offsets).  Round 5, with the 8-wave
// conv_pipe: every direction (FusAtNet step 18.21 -> 18.04-18.06 ms; wgrad only 18.14,
// profiles/r05_fusat_conv_pipe_w8.log); knob TAP_PIPE = direction bit mask (probe library).
// Round 6: C need not be a multiple of 4 (FusAtNet's 2193-channel concat, rows padded to 2196): with ldx % 4 == 0
// the last 16-B chunk of an input row covers channels up to C rounded to 4, which meet the packed weights' zero
// padding (forward; the caller keeps those columns finite, include/vitcnn.h) or land only in output columns >= C,
// which are not stored (weight and data gradients)
bool conv_pipe_ok(int mode, const TapArgs& a, const void* p0, long ld0, const void* p1, long ld1) {
  const long in_b = (long)a.nb * a.H * a.W * 4, out_b = (long)a.nb * a.OH * a.OW * 4;
  return (vc_knob("VITCNN_TAP_PIPE", 7) >> mode & 1) && a.O % 4 == 0 && ld0 % 4 == 0 && ld1 % 4 == 0 &&
         ((uintptr_t)p0 % 16) == 0 && ((uintptr_t)p1 % 16) == 0 && in_b * std::max(ld0, ld1) < (1L << 31) &&
         out_b * std::max(ld0, ld1) < (1L << 31) && (long)a.O * 9 * a.Cw * 4 < (1L << 31);
}

TapArgs geo(int B, int H, int W, int C, int O, int pad) {
  TapArgs a{};
  a.nb = B;
  a.H = H; a.W = W; a.C = C; a.O = O; a.pad = pad;
  a.Cw = (C + 3) & ~3;
  a.OH = H + 2 * pad - 2; a.OW = W + 2 * pad - 2;
  a.fOW = make_fastdiv(a.OW); a.fOHW = make_fastdiv(a.OH * a.OW);
  a.fW = make_fastdiv(W); a.fHW = make_fastdiv(H * W);
  return a;
}

}  // namespace

VC_EXPORT int vc_conv3x3_pack(int O, int C, int mode, const float* src, float* dst, float beta, hipStream_t stream) {
  VC_REQUIRE(O > 0 && C > 0 && mode >= 0 && mode <= 2 && src && dst);
  const long n = (long)O * ((C + 3) & ~3) * 9;   // mode 0 writes the padded layout
  VC_REQUIRE_I32(n);
  hipLaunchKernelGGL(conv_pack, dim3(vc_cdiv(n, 256)), dim3(256), 0, stream, O, C, mode, src, dst, beta);
  VC_CHECK_LAUNCH();
  return VC_OK;
}

VC_EXPORT int vc_conv3x3_pack_many(int n, const int* shapes, const float* const* src, float* const* dst,
                                   hipStream_t stream) {
  VC_REQUIRE(n >= 0 && (n == 0 || (shapes && src && dst)));
  for (int i0 = 0; i0 < n; i0 += PACK_MAX) {   // PACK_MAX convs per launch
    PackMany P;
    P.n = std::min(PACK_MAX, n - i0);
    long total = 0;
    for (int k = 0; k < P.n; ++k) {
      const int O = shapes[2 * (i0 + k)], C = shapes[2 * (i0 + k) + 1];
      VC_REQUIRE(O > 0 && C > 0 && src[i0 + k] && dst[i0 + k]);
      P.O[k] = O;
      P.C[k] = C;
      P.src[k] = src[i0 + k];
      P.dst[k] = dst[i0 + k];
      P.start[k] = (int)total;
      total += vc_cdiv((long)O * ((C + 3) & ~3), 256);
      VC_REQUIRE(total < (1L << 31));
    }
    P.start[P.n] = (int)total;
    hipLaunchKernelGGL(conv_pack_many, dim3((unsigned)total), dim3(256), 0, stream, P);
    VC_CHECK_LAUNCH();
  }
  return VC_OK;
}

VC_EXPORT int vc_conv3x3_tap_fwd(int B, int H, int W, int C, int O, int pad, const float* x, long ldx, const float* wt,
                                 const float* bias, float* y, long ldy, float* ws, long ws_floats, hipStream_t stream) {
  VC_REQUIRE(B > 0 && H >= 3 - 2 * pad && W >= 3 - 2 * pad && C > 0 && O > 0 && (pad == 0 || pad == 1));
  VC_REQUIRE(x && wt && y && ldx >= C && ldy >= O);
  TapArgs a = geo(B, H, W, C, O, pad);
  a.M = B * a.OH * a.OW;
  a.N = O;
  VC_REQUIRE_I32((long)B * H * W * ldx);
  VC_REQUIRE_I32((long)a.M * ldy);
  a.tpt = vc_cdiv(C, TK);
  a.nk = 9 * a.tpt;
  a.x = x; a.ldx = ldx; a.w = wt; a.bias = bias; a.out = y; a.ldo = ldy;
  a.vx = vec_ok(x, ldx); a.vw = vec_ok(wt, a.Cw);
  if (conv_pipe_ok(FWD, a, x, ldx, wt, 4)) return launch_conv_pipe<FWD>(a, vc_cdiv(O, CP_B), ws, ws_floats, stream);
  return launch_tap<FWD>(a, vc_cdiv(O, TN), vc_cdiv(a.M, TM), ws, ws_floats, stream);
}

static int tap_wgrad(int B, int H, int W, int C, int O, int pad, const float* x, long ldx, const float* dy, long lddy,
                     float* dwt, int oihw, float* db, float* ws, long ws_floats, hipStream_t stream) {
  VC_REQUIRE(B > 0 && H >= 3 - 2 * pad && W >= 3 - 2 * pad && C > 0 && O > 0 && (pad == 0 || pad == 1));
  VC_REQUIRE(x && dy && dwt && ldx >= C && lddy >= O);
  TapArgs a = geo(B, H, W, C, O, pad);
  a.M = O;
  a.N = 9 * C;
  a.P = B * a.OH * a.OW;
  VC_REQUIRE_I32((long)B * H * W * ldx);
  VC_REQUIRE_I32((long)a.P * lddy);
  a.tpt = vc_cdiv(C, TN);
  a.nk = vc_cdiv(a.P, TK);
  a.x = x; a.ldx = ldx; a.dy = dy; a.lddy = lddy; a.out = dwt; a.ldo = 9L * C;
  a.oihw = oihw;
  a.dbias = db;
  if (db) a.N = 9 * C + 1;   // the split slabs' bias column
  a.vx = vec_ok(x, ldx); a.vdy = vec_ok(dy, lddy);
  if (conv_pipe_ok(WGRAD, a, x, ldx, dy, lddy)) {
    a.tpt = vc_cdiv(C, CP_B);   // n-tiles per tap
    return launch_conv_pipe<WGRAD>(a, 9 * a.tpt, ws, ws_floats, stream);
  }
  return launch_tap<WGRAD>(a, 9 * a.tpt, vc_cdiv(O, TM), ws, ws_floats, stream);
}

VC_EXPORT int vc_conv3x3_tap_wgrad(int B, int H, int W, int C, int O, int pad, const float* x, long ldx,
                                   const float* dy, long lddy, float* dwt, float* ws, long ws_floats,
                                   hipStream_t stream) {
  return tap_wgrad(B, H, W, C, O, pad, x, ldx, dy, lddy, dwt, 0, nullptr, ws, ws_floats, stream);
}

VC_EXPORT int vc_conv3x3_tap_wgrad_oihw(int B, int H, int W, int C, int O, int pad, const float* x, long ldx,
                                        const float* dy, long lddy, float* dw, float* db, float* ws, long ws_floats,
                                        hipStream_t stream) {
  return tap_wgrad(B, H, W, C, O, pad, x, ldx, dy, lddy, dw, 1, db, ws, ws_floats, stream);
}

VC_EXPORT int vc_conv3x3_tap_dgrad(int B, int H, int W, int C, int O, int pad, const float* dy, long lddy,
                                   const float* wt, float beta, float* dx, long lddx, float* ws, long ws_floats,
                                   hipStream_t stream) {
  VC_REQUIRE(B > 0 && H >= 3 - 2 * pad && W >= 3 - 2 * pad && C > 0 && O > 0 && (pad == 0 || pad == 1));
  VC_REQUIRE(dy && wt && dx && lddy >= O && lddx >= C);
  TapArgs a = geo(B, H, W, C, O, pad);
  a.M = B * H * W;
  a.N = C;
  VC_REQUIRE_I32((long)a.M * lddx);
  VC_REQUIRE_I32((long)B * a.OH * a.OW * lddy);
  a.tpt = vc_cdiv(O, TK);
  a.nk = 9 * a.tpt;
  a.dy = dy; a.lddy = lddy; a.w = wt; a.out = dx; a.ldo = lddx; a.beta = beta;
  a.vdy = vec_ok(dy, lddy); a.vw = vec_ok(wt, a.Cw);
  if (conv_pipe_ok(DGRAD, a, dy, lddy, wt, 4)) return launch_conv_pipe<DGRAD>(a, vc_cdiv(C, CP_B), ws, ws_floats, stream);
  return launch_tap<DGRAD>(a, vc_cdiv(C, TN), vc_cdiv(a.M, TM), ws, ws_floats, stream);
}
