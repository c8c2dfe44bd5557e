// MFMA tile primitives shared by the GEMM kernels (gemm.hip) and the tap-major conv kernels
// (conv_tap.hip): the K-contiguous / row-contiguous LDS images and their fragment reads (g2::Stage), the
// per-k-tile MFMA step (g2::mma_ktile), the LDS-DMA staging of the pipelined kernels (gp::dma16, gp::fill)
// and the XCD-aware block order.
#pragma once
#include "common.h"

namespace g2 {

constexpr int ROWB = 128;  // bytes of k per LDS tile row and k-tile

__device__ __forceinline__ int lds_off(int r, int c) { return (r << 7) + ((c ^ ((r >> 1) & 7)) << 4); }

typedef float vf2 __attribute__((ext_vector_type(2)));
typedef __bf16 vb2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((vf2){lo, hi}, vb2));
}

// One operand's share of a k-tile.  Element (r, k) of the operand is T ? p[k*ld + r] : p[r*ld + k]
// for r < R and k < kend, else 0; with ONES, row R reads 1.0 (op(B)'s implicit ones column).
// Both images of a tile take ROWS x 128 B of LDS, laid out after the source's contiguous axis:
//  * K-contiguous sources (T = 0): [row][k] — eight 16-B k-chunks per row, chunk c of row r at
//    slot c ^ ((r >> 1) & 7).  A thread owns chunks (row (tid>>3) + 32i, chunk tid&7) and reads
//    each as float4s; a fragment is one ds_read_b128 (rows lane&15, chunk lane>>4).
//  * row-contiguous sources (T = 1, the weight gradients' dY / X and the data gradients' W): [k][row]
//    — a thread reads float4s along rows (16 lanes = 64 rows = 256 coalesced bytes at one k) and
//    stores them as one 16-B (fp32) / 8-B (bf16) piece.  fp32 fragments are four ds_read_b32 (one
//    k each); bf16 fragments two ds_read_b64_tr_b16 (4 k-rows x 16 columns each, delivered
//    column-major: the hardware transpose).  16-column blocks are XOR-swizzled by k so the
//    fragment reads and the stores are bank-conflict-free.
// Fragment k order (both images, so A and B always pair the same k): bf16 lane group g = lane>>4 of
// sub-step s holds k = 32s + 8g + j (j < 8); fp32 element j of group g holds k = 16s + 4g + j.
// `vec`: the operand allows the vector loads (alignment, leading dimension), a uniform flag.
template <bool BF, bool T, int ROWS, bool ONES>
struct Stage {
  static constexpr int KT = BF ? 64 : 32;      // k per tile
  static constexpr int NR = KT * ROWS / 256;   // staged floats per thread
  static constexpr int E = BF ? 8 : 4;         // KC: elements per 16-B chunk
  float raw[NR];

  __device__ __forceinline__ static float at(const float* p, long ld, int R, int kend, bool ones, int r, int k) {
    if (k >= kend) return 0.f;
    if (r < R) return T ? p[(long)k * ld + r] : p[(long)r * ld + k];
    return (ONES && ones && r == R) ? 1.f : 0.f;
  }

  // RC image offsets
  __device__ __forceinline__ static int rc_off(int k, int col) {
    if (BF) {
      const int x = ROWS == 64 ? (((k >> 1) & 1) | (((k >> 3) & 1) << 1)) : ((k & 3) | (((k >> 3) & 1) << 2));
      return k * (ROWS * 2) + ((((col >> 4) ^ x)) << 5) + ((col & 15) << 1);
    }
    return k * (ROWS * 4) + ((((col >> 4) ^ ((k >> 2) & 1))) << 6) + ((col & 15) << 2);
  }

  __device__ __forceinline__ void load(const float* p, long ld, int R, int row0, int k0, int kend, bool ones,
                                       bool vec, int tid) {
    if constexpr (!T) {
#pragma unroll
      for (int i = 0; i < NR / E; ++i) {
        const int r = row0 + (tid >> 3) + 32 * i, k = k0 + (tid & 7) * E;
        if (vec && r < R && k + E <= kend) {
          const float* s = p + (long)r * ld + k;
#pragma unroll
          for (int v = 0; v < E / 4; ++v) {
            const float4 x = *reinterpret_cast<const float4*>(s + 4 * v);
            raw[i * E + 4 * v] = x.x;
            raw[i * E + 4 * v + 1] = x.y;
            raw[i * E + 4 * v + 2] = x.z;
            raw[i * E + 4 * v + 3] = x.w;
          }
        } else {
#pragma unroll
          for (int j = 0; j < E; ++j) raw[i * E + j] = at(p, ld, R, kend, ones, r, k + j);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < NR / 4; ++i) {
        const int idx = tid + 256 * i;
        const int k = k0 + idx / (ROWS / 4), r = row0 + 4 * (idx % (ROWS / 4));
        if (vec && r + 3 < R && k < kend) {
          const float4 x = *reinterpret_cast<const float4*>(p + (long)k * ld + r);
          raw[4 * i] = x.x;
          raw[4 * i + 1] = x.y;
          raw[4 * i + 2] = x.z;
          raw[4 * i + 3] = x.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) raw[4 * i + j] = at(p, ld, R, kend, ones, r + j, k);
        }
      }
    }
  }

  __device__ __forceinline__ void store(char* lds, int tid) const {
    if constexpr (!T) {
#pragma unroll
      for (int i = 0; i < NR / E; ++i) {
        const int r = (tid >> 3) + 32 * i, c = tid & 7;
        uint4 w;
        if (BF) {
          w.x = pk_bf16(raw[i * E], raw[i * E + 1]);
          w.y = pk_bf16(raw[i * E + 2], raw[i * E + 3]);
          w.z = pk_bf16(raw[i * E + 4 % E], raw[i * E + 5 % E]);
          w.w = pk_bf16(raw[i * E + 6 % E], raw[i * E + 7 % E]);
        } else {
          w.x = __float_as_uint(raw[i * E]);
          w.y = __float_as_uint(raw[i * E + 1]);
          w.z = __float_as_uint(raw[i * E + 2 % E]);
          w.w = __float_as_uint(raw[i * E + 3 % E]);
        }
        *reinterpret_cast<uint4*>(lds + lds_off(r, c)) = w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NR / 4; ++i) {
        const int idx = tid + 256 * i;
        const int k = idx / (ROWS / 4), col = 4 * (idx % (ROWS / 4));
        if (BF) {
          uint2 w;
          w.x = pk_bf16(raw[4 * i], raw[4 * i + 1]);
          w.y = pk_bf16(raw[4 * i + 2], raw[4 * i + 3]);
          *reinterpret_cast<uint2*>(lds + rc_off(k, col)) = w;
        } else {
          *reinterpret_cast<float4*>(lds + rc_off(k, col)) =
              make_float4(raw[4 * i], raw[4 * i + 1], raw[4 * i + 2], raw[4 * i + 3]);
        }
      }
    }
  }

  // the lane's fragment of the 16-row block starting at `rowbase`, sub-step s (bit pattern: 4 fp32
  // or 8 bf16 in the k order above)
  __device__ __forceinline__ static uint4 frag(const char* lds, int rowbase, int s, int lane) {
    const int g = lane >> 4, l16 = lane & 15;
    if constexpr (!T) {
      return *reinterpret_cast<const uint4*>(lds + lds_off(rowbase + l16, 4 * s + g));
    } else if constexpr (BF) {
      typedef short s4 __attribute__((ext_vector_type(4)));
      typedef __attribute__((address_space(3))) s4 lds_s4;
      const int q = l16 >> 2, pcol = l16 & 3;
      uint4 out;
      const s4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s4*)(lds + rc_off(32 * s + 8 * g + q, rowbase + 4 * pcol)));
      const s4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (lds_s4*)(lds + rc_off(32 * s + 8 * g + 4 + q, rowbase + 4 * pcol)));
      out.x = (uint32_t)(uint16_t)v0[0] | ((uint32_t)(uint16_t)v0[1] << 16);
      out.y = (uint32_t)(uint16_t)v0[2] | ((uint32_t)(uint16_t)v0[3] << 16);
      out.z = (uint32_t)(uint16_t)v1[0] | ((uint32_t)(uint16_t)v1[1] << 16);
      out.w = (uint32_t)(uint16_t)v1[2] | ((uint32_t)(uint16_t)v1[3] << 16);
      return out;
    } else {
      uint4 out;
      const int k = 16 * s + 4 * g, col = rowbase + l16;
      out.x = *reinterpret_cast<const uint32_t*>(lds + rc_off(k, col));
      out.y = *reinterpret_cast<const uint32_t*>(lds + rc_off(k + 1, col));
      out.z = *reinterpret_cast<const uint32_t*>(lds + rc_off(k + 2, col));
      out.w = *reinterpret_cast<const uint32_t*>(lds + rc_off(k + 3, col));
      return out;
    }
  }
};

// the wave's MT x NT tiles of 16x16 over one k-tile (two sub-steps).  fp32 keeps NC = 2 partial
// accumulators per tile, one per sub-step s: two fma chains of half the length (long-K accuracy,
// tools/gemm_err.py; with slices capped at 2048 of K the chains stay <= 1024 deep), and the MFMAs of
// one fragment element go round all MT*NT accumulators before the next element (dependent issues
// MT*NT >= 4 apart; 16x16x4 f32: 32-cycle issue, 40-cycle dependent latency).
template <bool BF, int MT, int NT, class SA, class SB, int NC>
__device__ __forceinline__ void mma_ktile(const char* As, const char* Bs, int arow, int brow, int lane,
                                          f32x4 (&acc)[NC][MT][NT]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    uint4 a[MT], b[NT];
#pragma unroll
    for (int mi = 0; mi < MT; ++mi) a[mi] = SA::frag(As, arow + 16 * mi, s, lane);
#pragma unroll
    for (int ni = 0; ni < NT; ++ni) b[ni] = SB::frag(Bs, brow + 16 * ni, s, lane);
    if (BF) {
#pragma unroll
      for (int mi = 0; mi < MT; ++mi)
#pragma unroll
        for (int ni = 0; ni < NT; ++ni)
          acc[0][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[mi]),
                                                                   __builtin_bit_cast(bf16x8, b[ni]), acc[0][mi][ni], 0, 0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int mi = 0; mi < MT; ++mi)
#pragma unroll
          for (int ni = 0; ni < NT; ++ni)
            acc[s % NC][mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                __uint_as_float(a[mi][j]), __uint_as_float(b[ni][j]), acc[s % NC][mi][ni], 0, 0, 0);
    }
  }
}

// One sub-step s (k = 16 s .. 16 s + 15 of the k-tile) of mma_ktile's fp32 path into one accumulator set:
// the pipelined kernel's k-split waves (gp::pipe_tile, KS = 2) each run one sub-step of every k-tile, so
// their two accumulators are mma_ktile's NC = 2 partials (k = 16 s + 4 g + j, the same fma chains).
template <int MT, int NT, class SA, class SB>
__device__ __forceinline__ void mma_substep(const char* As, const char* Bs, int arow, int brow, int lane, int s,
                                            f32x4 (&acc)[MT][NT]) {
  uint4 a[MT], b[NT];
#pragma unroll
  for (int mi = 0; mi < MT; ++mi) a[mi] = SA::frag(As, arow + 16 * mi, s, lane);
#pragma unroll
  for (int ni = 0; ni < NT; ++ni) b[ni] = SB::frag(Bs, brow + 16 * ni, s, lane);
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int mi = 0; mi < MT; ++mi)
#pragma unroll
      for (int ni = 0; ni < NT; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[mi][j]), __uint_as_float(b[ni][j]),
                                                            acc[mi][ni], 0, 0, 0);
}

}  // namespace g2

namespace gp {

constexpr int KT = 32;   // k per stage (fp32: 128-B LDS rows)
constexpr unsigned OOB = 0x80000000u;   // a voffset past every operand: the DMA writes zeros

typedef __attribute__((address_space(3))) void lds_void;

// One 16-B-per-lane LDS-DMA wave-instruction: lane i's 16 source bytes (buffer offset voff) land at LDS
// byte lds + 16 i.  Written as asm on purpose: for the builtin form hipcc's wait-count pass cannot tell
// which ring slot a DMA writes, so it drains every outstanding DMA (vmcnt(0)) before each ds_read of any
// slot -- no k-tile would stay in flight.  Here the kernel counts them itself (vm_wait before the barrier
// that precedes the reads).  M0 is compiler-reserved: saved and restored inside the statement
// (cdna_hip_programming.md section 5.7); `lds` must be wave-uniform.
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

// one operand's share of a stage: ROWS rows of the operand (r in [row0, row0 + ROWS)), k in
// [k0, k0 + KT) masked at kend; T = row-contiguous source (element (r, k) at k * ld + r) else
// K-contiguous (r * ld + k).  Wave w of NW issues the wave-instructions w, w + NW, ... (ROWS / 8 / NW each).
template <bool T, int ROWS, int NW>
__device__ __forceinline__ void fill(__amdgpu_buffer_rsrc_t r, char* img, int row0, int k0, int kend, long ld,
                                     int wave, int lane) {
  static_assert((ROWS / 8) % NW == 0, "the waves split the stage's wave-instructions evenly");
#pragma unroll
  for (int q = 0; q < ROWS / 8 / NW; ++q) {
    const int i = wave + NW * q;   // wave-instruction: 1 KB of the image
    unsigned voff;
    if constexpr (!T) {
      const int row = 8 * i + (lane >> 3), slot = lane & 7;
      const int k = k0 + 4 * (slot ^ ((row >> 1) & 7));
      voff = k < kend ? (unsigned)(((long)(row0 + row) * ld + k) * 4) : OOB;
    } else {
      constexpr int KR = 256 / ROWS;          // k-rows per wave-instruction
      constexpr int SL = ROWS / 4;            // 16-B slots per k-row
      const int kr = KR * i + lane / SL, sq = lane % SL;
      const int col = ((((sq >> 2) ^ ((kr >> 2) & 1))) << 4) + ((sq & 3) << 2);
      const int k = k0 + kr;
      voff = k < kend ? (unsigned)(((long)k * ld + row0 + col) * 4) : OOB;
    }
    dma16(r, img + i * 1024, voff);
  }
}

template <int BM, int BN, int NS, int KM = 1>
constexpr int ring_bytes() { return NS * KM * (BM + BN) * 128; }

// 1-D grid in XCD-aware order (g2::gemm_mfma): block i runs on XCD i % 8, each XCD gets a contiguous
// run of logical blocks -- with zfast the K slices of a tile side by side
__device__ __forceinline__ unsigned xcd_linear(unsigned bid, unsigned total) {
  const unsigned q8 = total >> 3, r8 = total & 7, x8 = bid & 7;
  return x8 * q8 + min(x8, r8) + (bid >> 3);
}

__device__ __forceinline__ void tile_coords(unsigned lin, int nsplit, int tn, int tm, int zfast, int& zs, int& xn,
                                            int& ym, int& zb) {
  if (zfast) {
    zs = (int)(lin % (unsigned)nsplit);
    const unsigned t1 = lin / (unsigned)nsplit;
    xn = (int)(t1 % (unsigned)tn);
    const unsigned t2 = t1 / (unsigned)tn;
    ym = (int)(t2 % (unsigned)tm);
    zb = (int)(t2 / (unsigned)tm);
  } else {
    xn = (int)(lin % (unsigned)tn);
    const unsigned t1 = lin / (unsigned)tn;
    ym = (int)(t1 % (unsigned)tm);
    const unsigned t2 = t1 / (unsigned)tm;
    zs = (int)(t2 % (unsigned)nsplit);
    zb = (int)(t2 / (unsigned)nsplit);
  }
}

}  // namespace gp
