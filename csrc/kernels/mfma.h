// MFMA / LDS-image helpers shared by the GEMM and attention kernels (gfx950).
//
// LDS images hold tiles of row-major bf16 matrices, copied row by row from
// HBM in 16-byte chunks.  Each chunk's physical slot is XOR-swizzled by row so
// that BOTH access patterns an MFMA operand needs are bank-conflict free
// (bank rules: cdna_hip_programming.md §2, T2, T10):
//   * row reads  - ds_read_b128, a lane reads 16 B (8 consecutive k) of its
//                  own row; 16-lane groups see 16 distinct rows;
//   * tr reads   - ds_read_b64_tr_b16, a half wave reads 4 consecutive rows x
//                  64 B and receives them transposed (4 k values per lane).
// 128-byte rows: slot = c ^ g((r>>1)&7) with g(x) = x ^ ((x&1)<<2): row pairs
// alternate 64-byte halves, so the 4 rows of a tr read hit 4 bank quarters.
// 256-byte rows: slot = c ^ (((r&3)<<2) | ((r>>2)&3))  (guide T10 image (b)).
#pragma once
#include "common.h"

namespace ffk {

typedef bf16x4 __attribute__((address_space(3))) * lds_b4_ptr;

template <int ROW_BYTES>
__device__ __forceinline__ int swz_chunk(int r, int c) {
  if constexpr (ROW_BYTES == 128) {
    const int x = (r >> 1) & 7;
    return c ^ (x ^ ((x & 1) << 2));
  } else if constexpr (ROW_BYTES == 256) {
    return c ^ (((r & 3) << 2) | ((r >> 2) & 3));
  } else {
    static_assert(ROW_BYTES == 128 || ROW_BYTES == 256, "unsupported LDS image row size");
    return c;
  }
}
template <int ROW_BYTES>
__device__ __forceinline__ int img_off(int r, int c) {
  return r * ROW_BYTES + swz_chunk<ROW_BYTES>(r, c) * 16;
}

__device__ __forceinline__ bf16x8 lds_read16(const unsigned char* base, int off) {
  return *reinterpret_cast<const bf16x8*>(base + off);
}
__device__ __forceinline__ bf16x4 lds_tr(const unsigned char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4_ptr)(base + off));
}
__device__ __forceinline__ bf16x8 cat44(bf16x4 a, bf16x4 b) {
  bf16x8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
  r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
  return r;
}
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Row-read operand: lane holds image[row0 + (lane&31)][k0 + 8*(lane>>5) .. +8]
// (k0 a multiple of 16 elements).
template <int ROW_BYTES>
__device__ __forceinline__ bf16x8 row_frag(const unsigned char* img, int row0, int k0, int lane) {
  return lds_read16(img, img_off<ROW_BYTES>(row0 + (lane & 31), (k0 >> 3) + (lane >> 5)));
}

// Transposed operand with NATURAL k order: the image is [k][x]; lane holds
// image[k0 + 8*(lane>>5) + j][x0 + (lane&31)] for j = 0..7.
template <int ROW_BYTES>
__device__ __forceinline__ bf16x8 tr_frag_nat(const unsigned char* img, int k0, int x0, int lane) {
  const int h = lane >> 5, g = (lane >> 4) & 1, i = lane & 15;
  const int col = x0 + 16 * g + 4 * (i & 3);
  const int ra = k0 + 8 * h + (i >> 2);
  const int oa = img_off<ROW_BYTES>(ra, col >> 3) + (col & 7) * 2;
  const int ob = img_off<ROW_BYTES>(ra + 4, col >> 3) + (col & 7) * 2;
  return cat44(lds_tr(img, oa), lds_tr(img, ob));
}

// Same read issued from inline asm.  hipcc cannot see which LDS bytes an
// intrinsic ds_read_b64_tr_b16 touches and waits vmcnt(0) for every LDS-DMA
// in flight before it, draining a DMA pipeline that spans barriers (gemmp.hip).
// The asm form is invisible to that analysis: the CALLER must retire the
// reads itself (s_waitcnt lgkmcnt(0) + sched_barrier before the consumer).
__device__ __forceinline__ bf16x4 lds_tr_asm(const unsigned char* base, int off) {
  bf16x4 r;
  const unsigned addr = static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const unsigned char*)(base + off)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}
template <int ROW_BYTES>
__device__ __forceinline__ bf16x8 tr_frag_nat_asm(const unsigned char* img, int k0, int x0, int lane) {
  const int h = lane >> 5, g = (lane >> 4) & 1, i = lane & 15;
  const int col = x0 + 16 * g + 4 * (i & 3);
  const int ra = k0 + 8 * h + (i >> 2);
  const int oa = img_off<ROW_BYTES>(ra, col >> 3) + (col & 7) * 2;
  const int ob = img_off<ROW_BYTES>(ra + 4, col >> 3) + (col & 7) * 2;
  return cat44(lds_tr_asm(img, oa), lds_tr_asm(img, ob));
}

// Transposed operand with the ACCUMULATOR k order (pairs with an f32x16
// accumulator converted by acc_to_frag): element j of lane half h holds
// image[k0 + 8*(j>>2) + 4*h + (j&3)][x0 + (lane&31)].
template <int ROW_BYTES>
__device__ __forceinline__ bf16x8 tr_frag_acc(const unsigned char* img, int k0, int x0, int lane) {
  const int h = lane >> 5, g = (lane >> 4) & 1, i = lane & 15;
  const int col = x0 + 16 * g + 4 * (i & 3);
  const int ra = k0 + 4 * h + (i >> 2);
  const int oa = img_off<ROW_BYTES>(ra, col >> 3) + (col & 7) * 2;
  const int ob = img_off<ROW_BYTES>(ra + 8, col >> 3) + (col & 7) * 2;
  return cat44(lds_tr(img, oa), lds_tr(img, ob));
}

// Accumulator registers 8s..8s+7 -> bf16 operand fragment for k-step s.
__device__ __forceinline__ bf16x8 acc_to_frag(const f32x16& acc, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(acc[8 * s + j]);
  return r;
}

// Bijective XCD-aware block remap (guide §5 "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD (shared L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8, idx = orig / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace ffk
