// One-wave-per-SIMD bf16 GEMM for gfx950 (GemmPParams.variant = 3).
//
// Geometry (the shape hipBLASLt's fastest gfx950 kernels use on these
// problems, MT256x256x64 MI16x16 with an 8 x 8 MFMA wave tile): a 256 x 256
// output tile per workgroup of 4 waves (2 x 2), a 128 x 128 tile per wave =
// 8 x 8 v_mfma_f32_16x16x32_bf16 blocks whose accumulators (256 registers)
// live in AGPRs: with one wave per SIMD the unified register file holds 512
// per lane.  Per 32-deep k-step a wave reads 8 A + 8 B fragments for 64
// MFMAs: half the LDS read traffic per MFMA of a 128 x 64 wave tile.
//
// K loop, one barrier per 64-deep K-tile, two phases:
//   A: MFMAs of k-step 0 (fragments F0)      | read F1 (k-step 1 of this tile),
//                                              write the staged registers of tile
//                                              t+1 to the other LDS buffer, issue
//                                              the global loads of tile t+2
//   -- lgkmcnt(0), barrier --
//   B: MFMAs of k-step 1 (F1)                | read F0 (k-step 0 of tile t+1)
// so fragment reads run one phase ahead of their MFMAs and global loads one
// K-tile ahead of their LDS writes (register staging, guide T14; no LDS-DMA
// issue cost in the MFMA stream).  WAR: a buffer is rewritten in phase A of
// tile t+2, after every wave passed the barrier of tile t+1, which follows
// its last reads of it (lgkmcnt(0) before the barrier).
//
// Operand images (bank-conflict-free reads AND writes):
//   K-contiguous operand [outer][k]: [256 outer][64 k], 128-B rows, 16-B slot
//     = chunk ^ ((row >> 1) & 7); read by ds_read_b128 (lane -> row lane & 15)
//   K-outer operand [k][outer]: two halves [64 k][128 outer] (one per wave
//     row / column), 256-B rows, mfma.h 256-B swizzle; read by two
//     ds_read_b64_tr_b16 per fragment.
// Global loads: buffer_load_dwordx4 with per-lane voffsets fixed per tile and
// the K advance in the scalar soffset.
//
// Accumulators hold C^T (mfma(B fragment, A fragment)): D column lane & 15 ->
// m, D row 4 (lane >> 4) + e -> n: a lane owns 4 consecutive n of one row.
// Epilogues as gemmp.hip: plain (+ beta C, bf16 / fp32), bias + activation
// (+ pre-activation), activation-gradient (+ bias-gradient column sums),
// split-K fp32 slabs.
#include <type_traits>
#include <utility>

#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int TM = 256, TN = 256, TK = 64, NTHREADS = 256;
constexpr int HALF = 16 * 1024;   // 32 KB per operand tile per buffer
constexpr int BUFT = 4 * HALF;    // A tile + B tile
constexpr int GROUP = 4;
typedef float f32x4t __attribute__((ext_vector_type(4)));
typedef int i32x4t __attribute__((ext_vector_type(4)));

struct GemmTArgs {
  const bf16* A;
  const bf16* B;
  void* C;
  float* ws;
  const bf16* bias;
  bf16* pre;
  const bf16* aux;
  float* dbias;
  int M, N, K, lda, ldb, ldc;
  float alpha, beta;
  int act, act_bwd, out_f32, splits;
  unsigned bytesA, bytesB;
  int dbg;   // ablation bits (timing experiments, tools/gemm_ablate.py)
};

// activation code (elementwise.hip numbering) fixed at compile time: a run-time
// switch here keeps hipcc from unrolling the epilogue, which then indexes the
// AGPR accumulators dynamically through scratch
template <int ACT>
__device__ __forceinline__ float t_act(float x) {
  if (ACT == 1) return x > 0.f ? x : 0.f;
  if (ACT == 2) return 1.f / (1.f + __expf(-x));
  if (ACT == 3) return fast_tanh(x);
  if (ACT == 4) return gelu_tanh(x);
  return x;
}
template <int ACT>
__device__ __forceinline__ float t_act_grad(float x) {
  if (ACT == 1) return x > 0.f ? 1.f : 0.f;
  if (ACT == 2) {
    const float s = 1.f / (1.f + __expf(-x));
    return s * (1.f - s);
  }
  if (ACT == 3) {
    const float t = fast_tanh(x);
    return 1.f - t * t;
  }
  if (ACT == 4) return gelu_tanh_grad(x);
  return 1.f;
}

typedef float f32x2t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2t __attribute__((ext_vector_type(2)));

// activation (gradient) of an element pair: float2 arithmetic lowers to
// v_pk_mul / v_pk_fma / v_pk_add (two lanes' worth per VALU issue); only the
// v_exp / v_rcp transcendentals stay per element
__device__ __forceinline__ f32x2t gelu_sig2(f32x2t x, f32x2t x2) {
  constexpr float k1 = 0.044715f, c = -2.f * 0.7978845608028654f * 1.4426950408889634f;
  const f32x2t arg = x * __builtin_elementwise_fma(x2, f32x2t{c * k1, c * k1}, f32x2t{c, c});
  const f32x2t d = f32x2t{__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)} + 1.f;
  return f32x2t{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
template <int ACT>
__device__ __forceinline__ f32x2t t_act2(f32x2t x) {
  if (ACT == 1) return f32x2t{x.x > 0.f ? x.x : 0.f, x.y > 0.f ? x.y : 0.f};
  if (ACT == 4) return x * gelu_sig2(x, x * x);
  return f32x2t{t_act<ACT>(x.x), t_act<ACT>(x.y)};
}
// g * act'(x)
template <int ACT>
__device__ __forceinline__ f32x2t t_dact2(f32x2t g, f32x2t x) {
  if (ACT == 1) return f32x2t{x.x > 0.f ? g.x : 0.f, x.y > 0.f ? g.y : 0.f};
  if (ACT == 4) {
    constexpr float k0x2 = 2.f * 0.7978845608028654f, k1x3 = 3.f * 0.044715f;
    const f32x2t x2 = x * x;
    const f32x2t sg = gelu_sig2(x, x2);
    const f32x2t w = x * __builtin_elementwise_fma(x2, f32x2t{k0x2 * k1x3, k0x2 * k1x3}, f32x2t{k0x2, k0x2});
    return g * __builtin_elementwise_fma(w, sg - sg * sg, sg);
  }
  return f32x2t{g.x * t_act_grad<ACT>(x.x), g.y * t_act_grad<ACT>(x.y)};
}
// bf16 pair (one dword) -> float2: low half << 16, high half masked
__device__ __forceinline__ f32x2t unpack2(unsigned u) {
  return f32x2t{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
}

__device__ __forceinline__ int t_slot128(int r, int c) { return c ^ ((r >> 1) & 7); }

__device__ __forceinline__ f32x4t mfma16(bf16x8 a, bf16x8 b, f32x4t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Staging map: chunk i (0..7) of thread tid for one operand tile.
//  K-contiguous: row = (tid >> 3) + 32 i, 16-B chunk c = tid & 7
//  K-outer:      flat = tid + 256 i: half h = flat >> 10, k row r = (flat >> 4) & 63, chunk c = flat & 15
// The per-lane part of the byte offset is chunk 0's (one VGPR per operand);
// the chunk index and the K advance are wave-uniform and go in soffset.
// Rows / columns past the operand's edge are not clamped: they read zeros
// (buffer range check) or in-range bytes of another row, and only feed
// masked outputs.
template <bool KOUTER>
__device__ __forceinline__ unsigned stage_voff(int ld, int outer0, int tid) {
  if (KOUTER) {
    const int r = tid >> 4, c = tid & 15;
    return (static_cast<unsigned>(r) * static_cast<unsigned>(ld) + static_cast<unsigned>(outer0 + c * 8)) * 2u;
  }
  const int row = outer0 + (tid >> 3);
  return (static_cast<unsigned>(row) * static_cast<unsigned>(ld) + static_cast<unsigned>((tid & 7) * 8)) * 2u;
}
template <bool KOUTER>
__device__ __forceinline__ unsigned stage_soff(int ld, int i) {
  if (KOUTER) return static_cast<unsigned>(16 * (i & 3)) * static_cast<unsigned>(ld) * 2u + (i >> 2) * 256u;
  return static_cast<unsigned>(32 * i) * static_cast<unsigned>(ld) * 2u;
}
template <bool KOUTER>
__device__ __forceinline__ int stage_lds(int i, int tid) {
  if (KOUTER) {
    const int flat = tid + 256 * i;
    const int h = flat >> 10, r = (flat >> 4) & 63, c = flat & 15;
    return h * HALF + r * 256 + swz_chunk<256>(r, c) * 16;
  }
  const int row = (tid >> 3) + 32 * i, c = tid & 7;
  return row * 128 + t_slot128(row, c) * 16;
}

// LDS-DMA staging of one operand tile (32 KB = 32 x 1 KiB wave pieces, 8 per
// wave).  The DMA writes lane-linearly (base + 16 lane), so each lane's
// global source is the logical chunk that the image's swizzle stores in its
// physical slot (guide rule 21).  Piece i of wave w is image KiB j = 8 w + i.
//  K-contiguous image: KiB j = rows 8j..8j+7; the chunk swizzle depends on i
//    through bit 2 ((row >> 1) & 7 gains 4 i) -> two per-lane voffsets.
//  K-outer image: KiB j = half j >> 4 (= w >> 1), rows 4 (j & 15) + lane >> 4;
//    the swizzle depends on i & 3 -> four per-lane voffsets.
template <bool KOUTER>
__device__ __forceinline__ unsigned dma_voff(int ld, int outer0, int i, int wave, int lane) {
  const int j = wave * 8 + i;
  if (KOUTER) {
    const int h = j >> 4, r = 4 * (j & 15) + (lane >> 4);
    const int c = swz_chunk<256>(r, lane & 15);
    return (static_cast<unsigned>(r) * static_cast<unsigned>(ld) + static_cast<unsigned>(outer0 + h * 128 + c * 8)) * 2u;
  }
  const int row = 8 * j + (lane >> 3);
  const int c = t_slot128(row, lane & 7);
  return (static_cast<unsigned>(outer0 + row) * static_cast<unsigned>(ld) + static_cast<unsigned>(c * 8)) * 2u;
}

__device__ __forceinline__ bf16x8 row16(const unsigned char* img, int o0, int ks, int lane) {
  const int r = o0 + (lane & 15);
  return lds_read16(img, r * 128 + (t_slot128(r, ks * 4 + (lane >> 4)) << 4));
}
// ds_read_b64_tr_b16 hidden from the compiler's wait-count pass: with LDS-DMA
// in flight it treats the intrinsic as a possible reader of the DMA target and
// drains vmcnt(0) before every one (8 full drains per K-tile).  The caller
// waits lgkmcnt itself before the first MFMA that consumes these registers.
__device__ __forceinline__ bf16x4 lds_tr_asm(const unsigned char* base, int off) {
  bf16x4 r;
  const unsigned a = static_cast<unsigned>(reinterpret_cast<uintptr_t>(
      (const __attribute__((address_space(3))) unsigned char*)(base + off)));
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}
template <bool ASM = false>
__device__ __forceinline__ bf16x8 tr16(const unsigned char* img, int ks, int o0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = o0 + 4 * (i & 3);
  const int r = ks * 32 + 8 * g + (i >> 2);
  const int oa = img_off<256>(r, col >> 3) + (col & 7) * 2;
  const int ob = img_off<256>(r + 4, col >> 3) + (col & 7) * 2;
  if (ASM) return cat44(lds_tr_asm(img, oa), lds_tr_asm(img, ob));
  return cat44(lds_tr(img, oa), lds_tr(img, ob));
}

// kEpiPlain: bf16 C = alpha * AB (16-B paired stores); kEpiGeneral: fp32
// output and / or beta != 0 (kept apart: its extra live registers in a shared
// epilogue made the allocator shuttle accumulators through VGPRs in the loop)
// kEpiBias: bf16 C = AB + bias (no activation, no pre-activation copy)
// kEpiAccum: bf16 C += AB (alpha 1, beta != 0: the input-gradient GEMMs that
// accumulate into a residual branch's gradient) on the paired 16-B path, the
// fp32 values exchanged before packing so the sum is rounded once
enum Epi : int { kEpiPlain = 0, kEpiBiasAct = 1, kEpiDact = 2, kEpiSplit = 3, kEpiGeneral = 4, kEpiBias = 5,
                 kEpiAccum = 6 };

// one v_cvt_pk_bf16_f32 per pair (per-element casts pack through perm/alignbit)
__device__ __forceinline__ unsigned pack2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2t{a, b}, bf16x2t));
}
__device__ __forceinline__ uint2 pack4(const float (&v)[4]) { return uint2{pack2(v[0], v[1]), pack2(v[2], v[3])}; }
__device__ __forceinline__ unsigned pack2v(f32x2t v) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2t));
}

// Store the 8 bf16x4 groups of one row block (blocks nb = 0..7, lane row
// r = lane >> 4 holding columns 4r..4r+3 of each) as 16-byte stores: for each
// block pair (2j, 2j+1) one v_permlane16_swap per dword exchanges the odd
// 16-lane rows of block 2j with the even rows of block 2j+1, after which row
// r holds 8 consecutive columns, (r >> 1) * 8 .. +8, of block 2j + (r & 1)
// (guide T21: the store tail is issue-bound; half the instructions).
template <bool NT = false>
__device__ __forceinline__ void store_row16(bf16* C, int64_t row_off, int ncol0, int N, bool mok, const uint2 (&o)[8],
                                            int lane) {
  const int r = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const auto sx = __builtin_amdgcn_permlane16_swap(o[2 * j].x, o[2 * j + 1].x, false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(o[2 * j].y, o[2 * j + 1].y, false, false);
    const int n = ncol0 + (2 * j + (r & 1)) * 16 + (r >> 1) * 8;
    if (mok && n < N) {
      if (NT) {   // streamed past L2: keep the operands resident
        const i32x4t v{static_cast<int>(sx[0]), static_cast<int>(sy[0]), static_cast<int>(sx[1]),
                       static_cast<int>(sy[1])};
        __builtin_nontemporal_store(v, reinterpret_cast<i32x4t*>(C + row_off + n));
      } else {
        *reinterpret_cast<uint4*>(C + row_off + n) = uint4{sx[0], sy[0], sx[1], sy[1]};
      }
    }
  }
}

// kEpiAccum store of one row block: per block pair (2j, 2j+1) four fp32
// v_permlane16_swaps give lane row r 8 consecutive columns (the layout of
// store_row16), then one 16-B read of C, fp32 adds and one 16-B store.
__device__ __forceinline__ void accum_row16(bf16* C, int64_t row_off, int ncol0, int N, bool mok,
                                            const f32x4t (&a)[8], float beta, int lane) {
  const int r = lane >> 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned s[4][2];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const auto w = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[2 * j][e]), __float_as_uint(a[2 * j + 1][e]),
                                                      false, false);
      s[e][0] = w[0];
      s[e][1] = w[1];
    }
    const int n = ncol0 + (2 * j + (r & 1)) * 16 + (r >> 1) * 8;
    if (mok && n < N) {
      uint4* p = reinterpret_cast<uint4*>(C + row_off + n);
      const uint4 old = *p;
      const unsigned ow[4] = {old.x, old.y, old.z, old.w};
      unsigned nw[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // dword q holds columns 2q, 2q+1: elements (e = 2 (q & 1), +1) of swap half q >> 1
        const int h = q >> 1, e0 = 2 * (q & 1);
        const f32x2t v{__uint_as_float(s[e0][h]), __uint_as_float(s[e0 + 1][h])};
        nw[q] = pack2v(v + beta * unpack2(ow[q]));
      }
      *p = uint4{nw[0], nw[1], nw[2], nw[3]};
    }
  }
}

// LDS-staged C (one 128 x 128 bf16 wave tile = 32 KB, rows of 256 B, 16-B
// chunk slot = chunk ^ (row & 15)): the row block's paired 16-B groups go to
// LDS, and the tile leaves as whole rows, 4 rows x 256 contiguous bytes per
// store instruction (8 full 128-B lines instead of 16 half lines).
__device__ __forceinline__ void stage_row16(unsigned char* st, int mb, const uint2 (&o)[8], int lane) {
  const int r = lane >> 4;
  const int row = mb * 16 + (lane & 15);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const auto sx = __builtin_amdgcn_permlane16_swap(o[2 * j].x, o[2 * j + 1].x, false, false);
    const auto sy = __builtin_amdgcn_permlane16_swap(o[2 * j].y, o[2 * j + 1].y, false, false);
    const int chunk = 4 * j + 2 * (r & 1) + (r >> 1);
    *reinterpret_cast<i32x4t*>(st + row * 256 + ((chunk ^ (row & 15)) << 4)) =
        i32x4t{static_cast<int>(sx[0]), static_cast<int>(sy[0]), static_cast<int>(sx[1]), static_cast<int>(sy[1])};
  }
}
__device__ __forceinline__ void flush_rows(const unsigned char* st, bf16* C, int mrow0, int ncol0, int M, int N,
                                           int ldc, int lane) {
  const int c = lane & 15;
  const int col = ncol0 + c * 8;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int row = 4 * i + (lane >> 4);
    const i32x4t v = *reinterpret_cast<const i32x4t*>(st + row * 256 + ((c ^ (row & 15)) << 4));
    const int m = mrow0 + row;
    if (m < M && col < N) *reinterpret_cast<i32x4t*>(C + static_cast<int64_t>(m) * ldc + col) = v;
  }
}

// acc[mb][nb]: row m = m0 + wm*128 + mb*16 + (lane & 15);
// columns n = n0 + wn*128 + nb*16 + 4 (lane >> 4) + e.
template <int EPI, int ACT, bool NT = false, bool STAGE = false>
__device__ __forceinline__ void epilogue(const GemmTArgs& g, f32x4t (&acc)[8][8], int m0, int n0, int split, int wm,
                                         int wn, int lane, unsigned char* st = nullptr) {
  const int nl = 4 * (lane >> 4);
  const int ncol0 = n0 + wn * 128;
  const int nbase = ncol0 + nl;
  // bf16 results (and pre-activations) go out through the paired 16-B path
  constexpr bool WIDE = EPI == kEpiBiasAct || EPI == kEpiDact || EPI == kEpiPlain || EPI == kEpiBias;
  float csum[8][4];
  if (EPI == kEpiDact) {
#pragma unroll
    for (int b = 0; b < 8; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c) csum[b][c] = 0.f;
  }
  // bias of this lane's 32 columns, loaded once (not per row block)
  float bv[8][4];
  if (EPI == kEpiBiasAct || EPI == kEpiBias) {
    if (g.bias) {
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
        const bf16x4 bb = *reinterpret_cast<const bf16x4*>(g.bias + min(nbase + nb * 16, g.N - 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[nb][e] = bf2f(bb[e]);
      }
    } else {
#pragma unroll
      for (int nb = 0; nb < 8; ++nb)
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[nb][e] = 0.f;
    }
  }
  // activation-gradient inputs, prefetched one row block ahead
  uint2 xa[2][8];
  auto row_of = [&](int mb) {
    const int m_raw = m0 + wm * 128 + mb * 16 + (lane & 15);
    return m_raw < g.M ? m_raw : g.M - 1;
  };
  if (EPI == kEpiDact) {
    const int64_t r0 = static_cast<int64_t>(row_of(0)) * g.ldc;
#pragma unroll
    for (int nb = 0; nb < 8; ++nb)
      xa[0][nb] = *reinterpret_cast<const uint2*>(g.aux + r0 + min(nbase + nb * 16, g.N - 4));
  }
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int m_raw = m0 + wm * 128 + mb * 16 + (lane & 15);
    const bool mok = m_raw < g.M;
    const int m = mok ? m_raw : g.M - 1;
    const int64_t roff = static_cast<int64_t>(m) * g.ldc;
    const float mf = mok ? 1.f : 0.f;
    if (EPI == kEpiDact && mb < 7) {
      const int64_t r1 = static_cast<int64_t>(row_of(mb + 1)) * g.ldc;
#pragma unroll
      for (int nb = 0; nb < 8; ++nb)
        xa[(mb + 1) & 1][nb] = *reinterpret_cast<const uint2*>(g.aux + r1 + min(nbase + nb * 16, g.N - 4));
    }
    // re-pin this row block's accumulators: one pin per block here (rather than
    // all 64 at the loop exit) keeps hipcc from permuting the AGPRs first
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[mb][j]));
    if (EPI == kEpiAccum) {
      accum_row16(static_cast<bf16*>(g.C), roff, ncol0, g.N, mok, acc[mb], g.beta, lane);
      continue;
    }
    uint2 ob[8], pb[8];
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) {
      const int n_raw = nbase + nb * 16;
      const bool ok = mok && n_raw < g.N;  // N % 8 == 0: a 4-group is all-in or all-out
      const int n = ok ? n_raw : min(n_raw, g.N - 4);
      const int64_t off = roff + n;
      if (EPI == kEpiBiasAct || EPI == kEpiDact || EPI == kEpiBias) {  // alpha 1 (gemmt_supported); pairs
        f32x2t v[2] = {f32x2t{acc[mb][nb][0], acc[mb][nb][1]}, f32x2t{acc[mb][nb][2], acc[mb][nb][3]}};
        if (EPI == kEpiBias) {
#pragma unroll
          for (int h = 0; h < 2; ++h) v[h] += f32x2t{bv[nb][2 * h], bv[nb][2 * h + 1]};
        } else if (EPI == kEpiBiasAct) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            v[h] += f32x2t{bv[nb][2 * h], bv[nb][2 * h + 1]};
            (h ? pb[nb].y : pb[nb].x) = pack2v(v[h]);  // the pre-activation
            v[h] = t_act2<ACT>(v[h]);
          }
        } else {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            v[h] = t_dact2<ACT>(v[h], unpack2(h ? xa[mb & 1][nb].y : xa[mb & 1][nb].x));
            csum[nb][2 * h] += mf * v[h].x;  // masked rows add 0 (fp32 sum of the gradient)
            csum[nb][2 * h + 1] += mf * v[h].y;
          }
        }
        ob[nb] = uint2{pack2v(v[0]), pack2v(v[1])};
        continue;
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = EPI == kEpiPlain ? acc[mb][nb][e] : g.alpha * acc[mb][nb][e];  // plain: alpha 1
      if (EPI == kEpiSplit) {
        float* Wp = g.ws + (static_cast<int64_t>(split) * g.M + m) * g.N + n;
        if (ok) *reinterpret_cast<f32x4t*>(Wp) = f32x4t{v[0], v[1], v[2], v[3]};
        continue;
      }
      if (EPI == kEpiGeneral) {
        if (g.beta != 0.f) {
          if (g.out_f32) {
            const f32x4t o = *reinterpret_cast<const f32x4t*>(static_cast<const float*>(g.C) + off);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += g.beta * o[e];
          } else {
            const bf16x4 o = *reinterpret_cast<const bf16x4*>(static_cast<const bf16*>(g.C) + off);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += g.beta * bf2f(o[e]);
          }
        }
        if (g.out_f32) {
          if (ok) *reinterpret_cast<f32x4t*>(static_cast<float*>(g.C) + off) = f32x4t{v[0], v[1], v[2], v[3]};
        } else if (ok) {
          *reinterpret_cast<uint2*>(static_cast<bf16*>(g.C) + off) = pack4(v);
        }
        continue;
      }
      ob[nb] = pack4(v);
    }
    if (WIDE && STAGE) {
      stage_row16(st, mb, ob, lane);
      if (EPI == kEpiBiasAct && g.pre) store_row16<NT>(g.pre, roff, ncol0, g.N, mok, pb, lane);
    } else if (WIDE) {
      store_row16<NT>(static_cast<bf16*>(g.C), roff, ncol0, g.N, mok, ob, lane);
      if (EPI == kEpiBiasAct && g.pre) store_row16<NT>(g.pre, roff, ncol0, g.N, mok, pb, lane);
    }
  }
  if (WIDE && STAGE) {
    asm volatile("" ::: "memory");  // LDS is in order within a wave: no wait, no barrier
    flush_rows(st, static_cast<bf16*>(g.C), m0 + wm * 128, ncol0, g.M, g.N, g.ldc, lane);
  }
  if (EPI == kEpiDact && g.dbias) {
    // column sums over the 16 lanes of a row group (lane & 15) as a
    // reduce-scatter: each xor step halves the live values (30 shuffles, not
    // 128), leaving lane 2 values: k = 16 b3 + 8 b2 + 4 b1 + 2 b0 + {0, 1}
    float cv[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) cv[k] = csum[k >> 2][k & 3];
#pragma unroll
    for (int st = 0, c = 32; st < 4; ++st, c >>= 1) {
      const int o = 8 >> st;
      const bool hi = (lane & o) != 0;
#pragma unroll
      for (int i = 0; i < c / 2; ++i) {
        const float send = hi ? cv[i] : cv[i + c / 2];
        const float keep = hi ? cv[i + c / 2] : cv[i];
        cv[i] = keep + __shfl_xor(send, o, 64);
      }
    }
    const int kb = 16 * ((lane >> 3) & 1) + 8 * ((lane >> 2) & 1) + 4 * ((lane >> 1) & 1) + 2 * (lane & 1);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = kb + t;
      const int n = nbase + (k >> 2) * 16 + (k & 3);
      if (n < g.N) atomicAdd(g.dbias + n, cv[t]);
    }
  }
}

// 16 bytes per lane straight into LDS (kept out of the kernel template: the
// builtin inside a lambda of a kernel template drops the host launch stub)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// STG: 0 = both operands staged through registers; 1 = B by LDS-DMA (issued
// in phase B, two phases ahead of its first read), A through registers; 2 =
// both by LDS-DMA (no staging registers, no ds_write in the loop)
// DBG (timing ablations only, results are garbage): 1 = no global loads in
// the loop, 2 = no LDS writes in the loop, 4 = no mid-tile barrier, 8 = no
// epilogue; 256 (STG 2, a schedule variant with valid results): each
// group's fragment reads (and phase B's DMA issues) interleaved 1:1 with its
// MFMAs
template <bool TA, bool TB, int EPI, int ACT, int STG, int DBG = 0>
__global__ __launch_bounds__(NTHREADS, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemmt_kernel(
    GemmTArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUFT];  // the ONE LDS object
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  // ---- tile (bijective XCD remap + grouped raster, guide T1)
  const int gm = (g.M + TM - 1) / TM, gn = (g.N + TN - 1) / TN;
  const int nwg = gm * gn;
  const int W = nwg * g.splits;
  const int bid = xcd_remap(blockIdx.x, W);
  const int split = bid / nwg, t = bid % nwg;
  const int per_group = GROUP * gn;
  const int first_m = (t / per_group) * GROUP;
  const int gsize = min(gm - first_m, GROUP);
  const int m0 = (first_m + (t % per_group) % gsize) * TM;
  const int n0 = ((t % per_group) / gsize) * TN;
  // K-tiles of this split: the remainder goes one each to the first splits
  const int KT = g.K / TK, Lb = KT / g.splits, rem = KT % g.splits;
  const int L = Lb + (split < rem ? 1 : 0);
  const int kt0 = split * Lb + min(split, rem);

  // ---- global staging (A: KOUTER = TA, B: KOUTER = !TB)
  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.A), static_cast<short>(0), g.bytesA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.B), static_cast<short>(0), g.bytesB, 0x00020000);
  const unsigned kstepA = TA ? static_cast<unsigned>(TK * g.lda * 2) : TK * 2u;
  const unsigned kstepB = !TB ? static_cast<unsigned>(TK * g.ldb * 2) : TK * 2u;
  const unsigned voA = stage_voff<TA>(g.lda, m0, tid);
  const unsigned voB = stage_voff<!TB>(g.ldb, n0, tid);
  constexpr int NDV = !TB ? 4 : 2;  // B DMA voffsets (K-outer: by i & 3, K-contiguous: by i & 1)
  unsigned dvB[NDV];
#pragma unroll
  for (int i = 0; i < NDV; ++i) dvB[i] = STG >= 1 ? dma_voff<!TB>(g.ldb, n0, i, wave, lane) : 0u;
  constexpr int NDA = TA ? 4 : 2;   // A DMA voffsets (STG 2)
  unsigned dvA[NDA];
#pragma unroll
  for (int i = 0; i < NDA; ++i) dvA[i] = STG == 2 ? dma_voff<TA>(g.lda, m0, i, wave, lane) : 0u;
  auto dsoffA = [&](int i) -> unsigned {
    return TA ? static_cast<unsigned>(4 * (i - (i & 3))) * static_cast<unsigned>(g.lda) * 2u
              : static_cast<unsigned>(8 * (i - (i & 1))) * static_cast<unsigned>(g.lda) * 2u;
  };
  // scalar part of B DMA piece i's offset (rows beyond piece i % NDV's)
  auto dsoffB = [&](int i) -> unsigned {
    return !TB ? static_cast<unsigned>(4 * (i - (i & 3))) * static_cast<unsigned>(g.ldb) * 2u
               : static_cast<unsigned>(8 * (i - (i & 1))) * static_cast<unsigned>(g.ldb) * 2u;
  };
  constexpr int NR = STG == 1 ? 8 : 16;
  i32x4t R[16];
  (void)NR;
  auto gload = [&](int kt) {  // issue the register-staged global loads of K-tile kt
    const unsigned ka = static_cast<unsigned>(kt) * kstepA;
    const unsigned kb = static_cast<unsigned>(kt) * kstepB;
    if (STG == 2) return;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      R[i] = __builtin_amdgcn_raw_buffer_load_b128(
          rA, voA, __builtin_amdgcn_readfirstlane(ka + stage_soff<TA>(g.lda, i)), 0);
    if (STG == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        R[8 + i] = __builtin_amdgcn_raw_buffer_load_b128(
            rB, voB, __builtin_amdgcn_readfirstlane(kb + stage_soff<!TB>(g.ldb, i)), 0);
    }
  };
  auto swrite = [&](unsigned char* buf) {  // R -> LDS image of one K-tile
    if (STG == 2) return;
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<i32x4t*>(buf + stage_lds<TA>(i, tid)) = R[i];
    if (STG == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) *reinterpret_cast<i32x4t*>(buf + 2 * HALF + stage_lds<!TB>(i, tid)) = R[8 + i];
    }
  };
  auto dmaB = [&](unsigned char* buf, int kt, int i) {  // B DMA piece i of K-tile kt into buf
    const unsigned kb = static_cast<unsigned>(kt) * kstepB + dsoffB(i);
    dma16(rB, buf + 2 * HALF + (wave * 8 + i) * 1024, dvB[i % NDV], __builtin_amdgcn_readfirstlane(kb));
  };
  auto dmaA = [&](unsigned char* buf, int kt, int i) {  // A DMA piece i of K-tile kt into buf (STG 2)
    const unsigned ka = static_cast<unsigned>(kt) * kstepA + dsoffA(i);
    dma16(rA, buf + (wave * 8 + i) * 1024, dvA[i % NDA], __builtin_amdgcn_readfirstlane(ka));
  };

  // ---- fragments
  auto rdA = [&](const unsigned char* buf, int mb, int ks) -> bf16x8 {
    return TA ? tr16<STG >= 1>(buf + wm * HALF, ks, mb * 16, lane) : row16(buf, wm * 128 + mb * 16, ks, lane);
  };
  auto rdB = [&](const unsigned char* buf, int nb, int ks) -> bf16x8 {
    const unsigned char* b = buf + 2 * HALF;
    return TB ? row16(b, wn * 128 + nb * 16, ks, lane) : tr16<STG >= 1>(b + wn * HALF, ks, nb * 16, lane);
  };

  f32x4t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4t{};
  // fa[mb] is re-read for the next k-step right after its last MFMA; the B
  // fragments alternate between two named sets (all 8 live through a k-step)
  bf16x8 fa[8], fbx[8], fby[8];

  // ---- prologue: tile 0 -> buffer 0, tile 1 in flight, k-step 0 fragments
  gload(kt0);
  if (STG >= 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (STG == 2) dmaA(smem, kt0, i);
      dmaB(smem, kt0, i);
    }
  }
  swrite(smem);
  gload(kt0 + 1);
  if (STG == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) dmaB(smem + BUFT, kt0 + 1, i);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // B of tile 0 landed (A / B of tile 1 in flight)
  }
  if (STG == 2) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      dmaA(smem + BUFT, kt0 + 1, i);
      dmaB(smem + BUFT, kt0 + 1, i);
    }
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 landed (tile 1 in flight)
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa[i] = rdA(smem, i, 0);
    fbx[i] = rdB(smem, i, 0);
  }

  // LDS read instructions per (A, B) fragment pair: ds_read_b128 = 1, transposed = 2
  constexpr int NRD = (TA ? 2 : 1) + (TB ? 1 : 2);
  // One straight-line body per K-tile (no branches: past the last K-tile the
  // global loads read zeros or unused in-range bytes and land in a buffer
  // nobody reads).  Program order IS the schedule: each 8-MFMA group (one A
  // fragment x the 8 B fragments, 128 cycles of matrix work) carries the
  // re-read of that A fragment and of one B fragment for the next k-step,
  // and in phase A also two LDS writes of the staged tile and the two global
  // loads that refill those registers; sched_barrier(0) between groups keeps
  // hipcc from hoisting all LDS / memory work out of the MFMA stream.
  for (int kt = 0; kt < L; ++kt) {
    unsigned char* cur = smem + (kt & 1) * BUFT;
    unsigned char* nxt = smem + ((kt + 1) & 1) * BUFT;
    const unsigned ka = static_cast<unsigned>(kt0 + kt + 2) * kstepA;
    const unsigned kb = static_cast<unsigned>(kt0 + kt + 2) * kstepB;
    // asm-issued transposed reads (STG 1) are invisible to the compiler's
    // counters: the k-step 0 fragments of the previous phase B land here
    if (STG >= 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // ---- phase A: k-step 0 (fa, fbx) | read k-step 1 into (fa, fby), stage tile kt+1, load tile kt+2
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = mfma16(fbx[nb], fa[mb], acc[mb][nb]);
      fa[mb] = rdA(cur, mb, 1);
      fby[mb] = rdB(cur, mb, 1);
      // LDS writes + refills: STG 0: chunks 2mb, 2mb+1 (A chunks for mb < 4,
      // B after); STG 1: A chunk mb
#pragma unroll
      for (int h = 0; h < (STG == 2 ? 0 : STG == 1 ? 1 : 2); ++h) {
        const int c = STG == 1 ? mb : 2 * mb + h;
        if (c < 8) {
          if (!(DBG & 2)) *reinterpret_cast<i32x4t*>(nxt + stage_lds<TA>(c, tid)) = R[c];
          if (!(DBG & 1))
            R[c] = __builtin_amdgcn_raw_buffer_load_b128(
                rA, voA, __builtin_amdgcn_readfirstlane(ka + stage_soff<TA>(g.lda, c)), 0);
        } else {
          if (!(DBG & 2)) *reinterpret_cast<i32x4t*>(nxt + 2 * HALF + stage_lds<!TB>(c - 8, tid)) = R[c];
          if (!(DBG & 1))
            R[c] = __builtin_amdgcn_raw_buffer_load_b128(
                rB, voB, __builtin_amdgcn_readfirstlane(kb + stage_soff<!TB>(g.ldb, c - 8)), 0);
        }
      }
      // one memory instruction between MFMAs (an MFMA leaves the SIMD's issue
      // free for 8 of its 16 cycles); the fragment re-reads go last, after
      // the group's final use of fa[mb]
      if (STG == 2 && (DBG & 256)) {   // reads interleaved 1:1 with the group's MFMAs
#pragma unroll
        for (int r = 0; r < NRD; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8 - NRD, 0);
      } else if (STG == 2) {
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      if (STG == 2) {
      } else if (STG == 0) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      } else {
        __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
      }
      if (!(STG == 2 && (DBG & 256))) __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    // (DBG 128: no wait — a timing ablation of the exposed load latency)
    if (STG == 1 && !(DBG & 128)) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // B of tile kt+1 landed
    if (STG == 2 && !(DBG & 128)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt+1 landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // k-step 1 reads + LDS writes done
    if (!(DBG & 4)) __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // ---- phase B: k-step 1 (fa, fby) | read k-step 0 of tile kt+1 into (fa, fbx)
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = mfma16(fby[nb], fa[mb], acc[mb][nb]);
      fa[mb] = rdA(nxt, mb, 0);
      fbx[mb] = rdB(nxt, mb, 0);
      if (STG == 2) dmaA(cur, kt0 + kt + 2, mb);
      if (STG >= 1) dmaB(cur, kt0 + kt + 2, mb);  // tile kt's buffer: its reads retired at the barrier
      if (STG == 2 && (DBG & 256)) {   // reads, then the two DMA issues, one per MFMA
#pragma unroll
        for (int r = 0; r < NRD; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 8 - NRD - 2, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // pin the accumulators to AGPRs at the loop exit: otherwise the epilogue's
  // VALU use of them can tip the allocator into keeping some in VGPRs and
  // shuttling them (v_accvgpr_read / write) inside the loop
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) if (0) asm volatile("" : "+a"(acc[i][j]));
  constexpr bool STAGE_C = (DBG & 32) != 0;
  if (STAGE_C) __syncthreads();  // every wave is past its last K-loop LDS read
  if (!(DBG & 8))
    epilogue<EPI, ACT, (DBG & 16) != 0, STAGE_C>(g, acc, m0, n0, split, wm, wn, lane, smem + wave * 32768);
}

// ---- Both operands K-outer (C = A^T B, the weight-gradient GEMMs), LDS-DMA
// staged into PADDED images so every fragment read is one base VGPR plus an
// immediate offset.
//
// The swizzled 256-B-row image above spreads the 8 rows a 32-lane group reads
// over the banks by XOR-ing the 16-B chunk with row bits, i.e. with the bits
// that also select the 16-column block mb: each (mb, half) fragment address
// is a different per-lane value, and the loop spent 104 v_add_u32 per K-tile
// (next to 128 MFMAs and 64 transposed reads) re-forming them from the buffer
// pointer.  Here a half image is 64 k-rows of 128 columns at a 288-B pitch
// (256 B + 32 B pad, so consecutive physical rows start 32 B = 8 banks
// apart) with k-row bits 2 and 3 swapped: the rows a 32-lane group reads,
// 8g + {0..3} for g = 0, 1 (and + 4 for the second read, + 16 for g = 2, 3),
// land on 8 consecutive physical rows = 8 distinct 32-B bank groups.  A
// fragment address is then
//   lane base + buffer * KK_PT + ks * 32 rows + mb * 32 B (+ 4 rows for the
//   second half-read)
// with everything after the lane base a compile-time immediate of
// ds_read_b64_tr_b16 (< 64 KiB with the LDS order [A0][A1][B0][B1]).
// The DMA writes each 1-KiB piece lane-linearly; a lane's global source is
// the element its physical slot holds (pad slots re-load a neighbour's 16 B
// of the same row).  A half is 18 pieces: 9 per wave per operand.
constexpr int KK_PITCH = 288;
constexpr int KK_PH = 64 * KK_PITCH;   // one 128-column half image (18 KiB)
constexpr int KK_PT = 2 * KK_PH;       // one operand tile
constexpr int KK_NP = 9;               // DMA pieces per wave per operand tile

__device__ __forceinline__ int kk_swap23(int r) { return (r & ~12) | ((r & 4) << 1) | ((r & 8) >> 1); }

// per-lane voffset (bytes, K-tile 0) of DMA piece i of `wave` (half wave >> 1)
__device__ __forceinline__ unsigned kk_dma_voff(int ld, int outer0, int i, int wave, int lane) {
  const int b = (9 * (wave & 1) + i) * 1024 + lane * 16;
  const int prow = b / KK_PITCH;
  int w = b - prow * KK_PITCH;
  if (w >= 256) w -= 32;   // pad slot: same row, a neighbour's bytes
  const int r = kk_swap23(prow);
  const int col = (wave >> 1) * 128 + w / 2;
  return (static_cast<unsigned>(r) * static_cast<unsigned>(ld) + static_cast<unsigned>(outer0 + col)) * 2u;
}

template <int OFF>
__device__ __forceinline__ bf16x4 kk_tr(unsigned a) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
// fragment (k-step KS, 16-column block MB) of buffer BUF; base = lane base
// fragment (k-step KS, 16-column block MB) of the buffer whose lane base is `base`
template <int KS, int MB>
__device__ __forceinline__ bf16x8 kk_frag(unsigned base) {
  constexpr int O = KS * 32 * KK_PITCH + MB * 32;
  return cat44(kk_tr<O>(base), kk_tr<O + 8 * KK_PITCH>(base));   // k-row + 4 = physical row + 8
}

// K-contiguous A operand (gemmt_kernel's 128-B-row image): 16-row block MB
// of the k-step whose lane base is `base`
template <int MB>
__device__ __forceinline__ bf16x8 kk_row(unsigned base) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "i"(MB * 16 * 128));
  return r;
}

template <typename F, int... I>
__device__ __forceinline__ void kk_for(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}

// TA: A K-outer (padded image, as B); !TA: A K-contiguous (gemmt_kernel's
// swizzled 128-B-row image, ds_read_b128 at lane base + immediate)
// RS: the K-tile after next is loaded into registers (buffer_load_dwordx4,
// one 16-B piece per lane per DMA piece) in phase A and written lane-linearly
// with ds_write_b128 into the SAME image the LDS-DMA builds, one K-tile later.
// An LDS-DMA piece costs the issuing wave 60-185 cycles of issue among MFMAs
// (MI355X_MICROARCH.md cycle constants, 'LDS-DMA piece issue cost'); a
// buffer_load + ds_write_b128 pair ~20, inside the MFMA gaps, and the loads
// get a whole K-tile (not one phase) to land.
template <bool TA, int EPI, int ACT, int SCH = 0, bool TB = false, bool RS = false>
__global__ __launch_bounds__(NTHREADS, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemmt_kk_kernel(
    GemmTArgs g) {
  constexpr int SA = TA ? KK_PT : 2 * HALF;   // A tile bytes per buffer
  constexpr int SB = TB ? 2 * HALF : KK_PT;   // B tile bytes per buffer (TB: K-contiguous image)
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * SA + 2 * SB];  // [A0][A1][B0][B1]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int gm = (g.M + TM - 1) / TM, gn = (g.N + TN - 1) / TN;
  const int nwg = gm * gn;
  const int bid = xcd_remap(blockIdx.x, nwg * g.splits);
  const int split = bid / nwg, t = bid % nwg;
  const int per_group = GROUP * gn;
  const int first_m = (t / per_group) * GROUP;
  const int gsize = min(gm - first_m, GROUP);
  const int m0 = (first_m + (t % per_group) % gsize) * TM;
  const int n0 = ((t % per_group) / gsize) * TN;
  const int KT = g.K / TK, Lb = KT / g.splits, rem = KT % g.splits;
  const int L = Lb + (split < rem ? 1 : 0);
  const int kt0 = split * Lb + min(split, rem);

  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.A), static_cast<short>(0), g.bytesA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.B), static_cast<short>(0), g.bytesB, 0x00020000);
  const unsigned kstepA = TA ? static_cast<unsigned>(TK * g.lda * 2) : TK * 2u;
  const unsigned kstepB = TB ? TK * 2u : static_cast<unsigned>(TK * g.ldb * 2);
  unsigned dvA[KK_NP], dvB[KK_NP];
#pragma unroll
  for (int i = 0; i < KK_NP; ++i) {
    dvA[i] = TA ? kk_dma_voff(g.lda, m0, i, wave, lane) : i < 2 ? dma_voff<false>(g.lda, m0, i, wave, lane) : 0u;
    dvB[i] = !TB ? kk_dma_voff(g.ldb, n0, i, wave, lane) : i < 2 ? dma_voff<false>(g.ldb, n0, i, wave, lane) : 0u;
  }
  // this wave's first DMA piece of an operand tile (buffer 0)
  const int dpiece = (wave >> 1) * KK_PH + 9 * (wave & 1) * 1024;
  unsigned char* const sA = smem;
  unsigned char* const sB = smem + 2 * SA;
  auto dmaB = [&](int buf, unsigned kbyte, int i) __attribute__((always_inline)) {
    if (!TB) {
      dma16(rB, sB + buf * SB + dpiece + i * 1024, dvB[i], __builtin_amdgcn_readfirstlane(kbyte));
    } else {
      const unsigned so = kbyte + static_cast<unsigned>(8 * (i - (i & 1))) * static_cast<unsigned>(g.ldb) * 2u;
      dma16(rB, sB + buf * SB + (wave * 8 + i) * 1024, dvB[i & 1], __builtin_amdgcn_readfirstlane(so));
    }
  };
  // K-contiguous A: 8 pieces per wave, KiB j = 8 wave + i = rows 8j..8j+7,
  // per-lane voffset by i & 1 and the rows beyond in the scalar offset
  auto dmaA = [&](int buf, unsigned kbyte, int i) __attribute__((always_inline)) {
    if (TA) {
      dma16(rA, sA + buf * SA + dpiece + i * 1024, dvA[i], __builtin_amdgcn_readfirstlane(kbyte));
    } else {
      const unsigned so = kbyte + static_cast<unsigned>(8 * (i - (i & 1))) * static_cast<unsigned>(g.lda) * 2u;
      dma16(rA, sA + buf * SA + (wave * 8 + i) * 1024, dvA[i & 1], __builtin_amdgcn_readfirstlane(so));
    }
  };

  // register staging (RS): piece i of A in R[i], of B in R[NPA + i]
  constexpr int NPA = TA ? KK_NP : 8, NPB = TB ? 8 : KK_NP;
  i32x4t R[RS ? NPA + NPB : 1];
  auto ldA = [&](unsigned kbyte, int i) __attribute__((always_inline)) {
    if constexpr (RS) {
      if (TA) {
        R[i] = __builtin_amdgcn_raw_buffer_load_b128(rA, dvA[i], __builtin_amdgcn_readfirstlane(kbyte), 0);
      } else {
        const unsigned so = kbyte + static_cast<unsigned>(8 * (i - (i & 1))) * static_cast<unsigned>(g.lda) * 2u;
        R[i] = __builtin_amdgcn_raw_buffer_load_b128(rA, dvA[i & 1], __builtin_amdgcn_readfirstlane(so), 0);
      }
    }
  };
  auto ldB = [&](unsigned kbyte, int i) __attribute__((always_inline)) {
    if constexpr (RS) {
      if (!TB) {
        R[NPA + i] = __builtin_amdgcn_raw_buffer_load_b128(rB, dvB[i], __builtin_amdgcn_readfirstlane(kbyte), 0);
      } else {
        const unsigned so = kbyte + static_cast<unsigned>(8 * (i - (i & 1))) * static_cast<unsigned>(g.ldb) * 2u;
        R[NPA + i] = __builtin_amdgcn_raw_buffer_load_b128(rB, dvB[i & 1], __builtin_amdgcn_readfirstlane(so), 0);
      }
    }
  };
  // the lane-linear LDS position the DMA would have written piece i to
  auto wrA = [&](int buf, int i) __attribute__((always_inline)) {
    if constexpr (RS) {
      unsigned char* d = sA + buf * SA + (TA ? dpiece + i * 1024 : (wave * 8 + i) * 1024) + lane * 16;
      *reinterpret_cast<i32x4t*>(d) = R[i];
    }
  };
  auto wrB = [&](int buf, int i) __attribute__((always_inline)) {
    if constexpr (RS) {
      unsigned char* d = sB + buf * SB + (!TB ? dpiece + i * 1024 : (wave * 8 + i) * 1024) + lane * 16;
      *reinterpret_cast<i32x4t*>(d) = R[NPA + i];
    }
  };

  // lane base of the fragment reads (LDS byte address)
  const int gq = lane >> 4, iq = lane & 15;
  const int lrow = kk_swap23(8 * gq + (iq >> 2));
  const unsigned lds0 = static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) unsigned char*)smem));
  const unsigned lbase = lds0 + static_cast<unsigned>(lrow * KK_PITCH + 8 * (iq & 3));

  // A lane bases of k-step 0 / 1 (the K-outer image takes the k-step as an immediate)
  auto rowbase = [&](int ks) -> unsigned {
    const int r = lane & 15;
    return lds0 + static_cast<unsigned>((wm * 128 + r) * 128 + (t_slot128(r, ks * 4 + (lane >> 4)) << 4));
  };
  const unsigned baseA0 = TA ? lbase + static_cast<unsigned>(wm * KK_PH) : rowbase(0);
  const unsigned baseA1 = TA ? baseA0 : rowbase(1);
  auto rowbaseB = [&](int ks) -> unsigned {
    const int r = lane & 15;
    return lds0 + static_cast<unsigned>(2 * SA + (wn * 128 + r) * 128 + (t_slot128(r, ks * 4 + (lane >> 4)) << 4));
  };
  const unsigned baseB0 = TB ? rowbaseB(0) : lbase + static_cast<unsigned>(2 * SA + wn * KK_PH);
  const unsigned baseB1 = TB ? rowbaseB(1) : baseB0;

  f32x4t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4t{};
  bf16x8 fa[8], fbx[8], fby[8];
  constexpr auto S8 = std::make_integer_sequence<int, 8>{};

  auto readA = [&](auto KSC, auto MBC, unsigned base) __attribute__((always_inline)) -> bf16x8 {
    constexpr int ks = decltype(KSC)::value, mb = decltype(MBC)::value;
    if constexpr (TA) return kk_frag<ks, mb>(base);
    else return kk_row<mb>(base);
  };
  auto readB = [&](auto KSC, auto MBC, unsigned base) __attribute__((always_inline)) -> bf16x8 {
    constexpr int ks = decltype(KSC)::value, mb = decltype(MBC)::value;
    if constexpr (TB) return kk_row<mb>(base);
    else return kk_frag<ks, mb>(base);
  };
  using K0 = std::integral_constant<int, 0>;
  using K1 = std::integral_constant<int, 1>;

  // ---- prologue: tile 0 -> buffer 0, tile 1 -> buffer 1 (RS: tile 0 ->
  // buffer 0 by DMA, tile 1 -> registers), k-step 0 fragments
  constexpr int NPT = (TA ? KK_NP : 8) + (TB ? 8 : KK_NP);   // DMA issues per K-tile per wave
  if constexpr (RS) {
#pragma unroll
    for (int i = 0; i < NPA; ++i) dmaA(0, static_cast<unsigned>(kt0) * kstepA, i);
#pragma unroll
    for (int i = 0; i < NPB; ++i) dmaB(0, static_cast<unsigned>(kt0) * kstepB, i);
#pragma unroll
    for (int i = 0; i < NPA; ++i) ldA(static_cast<unsigned>(kt0 + 1) * kstepA, i);
#pragma unroll
    for (int i = 0; i < NPB; ++i) ldB(static_cast<unsigned>(kt0 + 1) * kstepB, i);
  } else {
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
      for (int i = 0; i < NPA; ++i) dmaA(b, static_cast<unsigned>(kt0 + b) * kstepA, i);
#pragma unroll
      for (int i = 0; i < NPB; ++i) dmaB(b, static_cast<unsigned>(kt0 + b) * kstepB, i);
    }
  }
  // tile 0 landed (tile 1's 18 / 17 / 16 pieces in flight, by DMA or into registers)
  if constexpr (NPT == 18) asm volatile("s_waitcnt vmcnt(18)" ::: "memory");
  else if constexpr (NPT == 17) asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  kk_for([&](auto MB) __attribute__((always_inline)) {
    constexpr int mb = decltype(MB)::value;
    fa[mb] = readA(K0{}, MB, baseA0);
    fbx[mb] = readB(K0{}, MB, baseB0);
  }, S8);

  // SCH 1: one side instruction after each MFMA of an 8-MFMA group (the B
  // fragment's two reads, the A fragment's read(s), then the group's DMA
  // pieces), each pinned by sched_barrier, instead of the group's reads
  // clustered after its 8 MFMAs
  auto group = [&](auto MBC, auto KSC, const bf16x8 (&fin)[8], bf16x8 (&fout)[8], unsigned aB, unsigned bB,
                   int dbuf, unsigned ka_, unsigned kb_, int wbuf = -1) __attribute__((always_inline)) {
    constexpr int mb = decltype(MBC)::value, ks = decltype(KSC)::value;
    constexpr int OB = ks * 32 * KK_PITCH + mb * 32;
    bf16x4 b0, b1, a0, a1;
    bf16x8 ar, br;
    __builtin_amdgcn_sched_barrier(0);
    acc[mb][0] = mfma16(fin[0], fa[mb], acc[mb][0]);
    if constexpr (TB) br = kk_row<mb>(bB);
    else b0 = kk_tr<OB>(bB);
    __builtin_amdgcn_sched_barrier(0);
    acc[mb][1] = mfma16(fin[1], fa[mb], acc[mb][1]);
    if constexpr (!TB) b1 = kk_tr<OB + 8 * KK_PITCH>(bB);
    __builtin_amdgcn_sched_barrier(0);
    acc[mb][2] = mfma16(fin[2], fa[mb], acc[mb][2]);
    if constexpr (TA) a0 = kk_tr<OB>(aB);
    else ar = kk_row<mb>(aB);
    __builtin_amdgcn_sched_barrier(0);
    acc[mb][3] = mfma16(fin[3], fa[mb], acc[mb][3]);
    if constexpr (TA) a1 = kk_tr<OB + 8 * KK_PITCH>(aB);
    __builtin_amdgcn_sched_barrier(0);
    acc[mb][4] = mfma16(fin[4], fa[mb], acc[mb][4]);
    if (dbuf >= 0) dmaA(dbuf, ka_, mb);
    if (RS && wbuf >= 0) {
      wrA(wbuf, mb);
      ldA(ka_, mb);
    }
    __builtin_amdgcn_sched_barrier(0);
    acc[mb][5] = mfma16(fin[5], fa[mb], acc[mb][5]);
    if (dbuf >= 0) dmaB(dbuf, kb_, mb);
    if (RS && wbuf >= 0) {
      wrB(wbuf, mb);
      ldB(kb_, mb);
    }
    __builtin_amdgcn_sched_barrier(0);
    acc[mb][6] = mfma16(fin[6], fa[mb], acc[mb][6]);
    if (dbuf >= 0 && mb == 7 && TA) dmaA(dbuf, ka_, 8);
    if (RS && wbuf >= 0 && mb == 7 && TA) {
      wrA(wbuf, 8);
      ldA(ka_, 8);
    }
    __builtin_amdgcn_sched_barrier(0);
    acc[mb][7] = mfma16(fin[7], fa[mb], acc[mb][7]);
    if (dbuf >= 0 && mb == 7 && !TB) dmaB(dbuf, kb_, 8);
    if (RS && wbuf >= 0 && mb == 7 && !TB) {
      wrB(wbuf, 8);
      ldB(kb_, 8);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (TB) fout[mb] = br;
    else fout[mb] = cat44(b0, b1);
    if constexpr (TA) fa[mb] = cat44(a0, a1);
    else fa[mb] = ar;
  };

  // same two-phase schedule as gemmt_kernel STG 2; the buffer's lane bases
  // are the only per-tile VALU work (4 adds)
  for (int kt = 0; kt < L; ++kt) {
    const int cur = kt & 1;
    const unsigned pa = static_cast<unsigned>(cur * SA), pna = static_cast<unsigned>((cur ^ 1) * SA);
    const unsigned pb = static_cast<unsigned>(cur * SB), pnb = static_cast<unsigned>((cur ^ 1) * SB);
    const unsigned aC = baseA1 + pa, bC = baseB1 + pb, aN = baseA0 + pna, bN = baseB0 + pnb;
    const unsigned ka = static_cast<unsigned>(kt0 + kt + 2) * kstepA;
    const unsigned kb = static_cast<unsigned>(kt0 + kt + 2) * kstepB;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // phase A: k-step 0 (fa, fbx) | read k-step 1 of the current buffer into (fa, fby)
    kk_for([&](auto MB) __attribute__((always_inline)) {
      constexpr int mb = decltype(MB)::value;
      if constexpr (SCH == 0) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = mfma16(fbx[nb], fa[mb], acc[mb][nb]);
        fa[mb] = readA(K1{}, MB, aC);
        fby[mb] = readB(K1{}, MB, bC);
      } else if constexpr (RS) {
        // stage tile kt+1 (registers) into the next buffer, load tile kt+2
        group(MB, K1{}, fbx, fby, aC, bC, -1, ka, kb, cur ^ 1);
      } else {
        group(MB, K1{}, fbx, fby, aC, bC, -1, 0u, 0u);
      }
    }, S8);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (!RS) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // tile kt+1 (next buffer) landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // k-step 1 reads (RS: and the staging writes) done
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // phase B: k-step 1 (fa, fby) | read k-step 0 of the next buffer into (fa, fbx),
    // DMA tile kt+2 into the current one (its reads retired at the barrier)
    kk_for([&](auto MB) __attribute__((always_inline)) {
      constexpr int mb = decltype(MB)::value;
      if constexpr (SCH == 0) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = mfma16(fby[nb], fa[mb], acc[mb][nb]);
        fa[mb] = readA(K0{}, MB, aN);
        fbx[mb] = readB(K0{}, MB, bN);
        dmaA(cur, ka, mb);
        dmaB(cur, kb, mb);
        if (mb == 7) {
          if (TA) dmaA(cur, ka, 8);
          if (!TB) dmaB(cur, kb, 8);
        }
      } else {
        group(MB, K0{}, fby, fbx, aN, bN, RS ? -1 : cur, ka, kb);
      }
    }, S8);
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) if (0) asm volatile("" : "+a"(acc[i][j]));
  epilogue<EPI, ACT, false, false>(g, acc, m0, n0, split, wm, wn, lane, nullptr);
}

// Persistent form (variant 5): one workgroup per CU walks its work items
// (tiles x K-splits) b, b + grid, ...; the K-tile stream runs on across item
// boundaries, so the last two iterations of an item already stage the next
// item's first two K-tiles and read its first fragments, and the epilogue of
// item i overlaps the in-flight global loads of item i + 1 (no prologue
// bubble per tile).  Requires L = K / 64 / splits >= 2.
template <bool TA, bool TB, int EPI, int ACT>
__global__ __launch_bounds__(NTHREADS, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemmt_pers_kernel(
    GemmTArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUFT];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;

  const int gm = (g.M + TM - 1) / TM, gn = (g.N + TN - 1) / TN;
  const int nwg = gm * gn;
  const int W = nwg * g.splits;
  const int L = g.K / TK / g.splits;
  const int per_group = GROUP * gn;
  // item -> (m0, n0, split); item % 8 is the XCD the workgroup runs on
  // (gridDim.x is a multiple of 8 or equal to W), so the bijective remap keeps
  // the tiles that run together on one XCD adjacent in the grouped raster
  auto geom = [&](int item, int& m0, int& n0, int& split) {
    const int bid = xcd_remap(item, W);
    split = bid / nwg;
    const int t = bid % nwg;
    const int first_m = (t / per_group) * GROUP;
    const int gsize = min(gm - first_m, GROUP);
    m0 = (first_m + (t % per_group) % gsize) * TM;
    n0 = ((t % per_group) / gsize) * TN;
  };

  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.A), static_cast<short>(0), g.bytesA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.B), static_cast<short>(0), g.bytesB, 0x00020000);
  const unsigned kstepA = TA ? static_cast<unsigned>(TK * g.lda * 2) : TK * 2u;
  const unsigned kstepB = !TB ? static_cast<unsigned>(TK * g.ldb * 2) : TK * 2u;

  int item = blockIdx.x;
  int m0, n0, split;
  geom(item, m0, n0, split);
  int nitem = item + static_cast<int>(gridDim.x);
  int m0n = m0, n0n = n0, splitn = split;
  if (nitem < W) geom(nitem, m0n, n0n, splitn);
  unsigned voA = stage_voff<TA>(g.lda, m0, tid), voB = stage_voff<!TB>(g.ldb, n0, tid);
  unsigned voAn = stage_voff<TA>(g.lda, m0n, tid), voBn = stage_voff<!TB>(g.ldb, n0n, tid);
  int kt0 = split * L, kt0n = splitn * L;

  i32x4t R[16];
  auto rdA = [&](const unsigned char* buf, int mb, int ks) -> bf16x8 {
    return TA ? tr16(buf + wm * HALF, ks, mb * 16, lane) : row16(buf, wm * 128 + mb * 16, ks, lane);
  };
  auto rdB = [&](const unsigned char* buf, int nb, int ks) -> bf16x8 {
    const unsigned char* b = buf + 2 * HALF;
    return TB ? row16(b, wn * 128 + nb * 16, ks, lane) : tr16(b + wn * HALF, ks, nb * 16, lane);
  };

  f32x4t acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4t{};
  bf16x8 fa[8], fbx[8], fby[8];

  // ---- prologue (first item only): K-tile 0 -> buffer 0, K-tile 1 in flight
  {
    const unsigned ka = static_cast<unsigned>(kt0) * kstepA, kb = static_cast<unsigned>(kt0) * kstepB;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      R[i] = __builtin_amdgcn_raw_buffer_load_b128(rA, voA, __builtin_amdgcn_readfirstlane(ka + stage_soff<TA>(g.lda, i)),
                                                   0);
      R[8 + i] = __builtin_amdgcn_raw_buffer_load_b128(
          rB, voB, __builtin_amdgcn_readfirstlane(kb + stage_soff<!TB>(g.ldb, i)), 0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      *reinterpret_cast<i32x4t*>(smem + stage_lds<TA>(i, tid)) = R[i];
      *reinterpret_cast<i32x4t*>(smem + 2 * HALF + stage_lds<!TB>(i, tid)) = R[8 + i];
    }
    const unsigned ka1 = ka + kstepA, kb1 = kb + kstepB;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      R[i] = __builtin_amdgcn_raw_buffer_load_b128(rA, voA,
                                                   __builtin_amdgcn_readfirstlane(ka1 + stage_soff<TA>(g.lda, i)), 0);
      R[8 + i] = __builtin_amdgcn_raw_buffer_load_b128(
          rB, voB, __builtin_amdgcn_readfirstlane(kb1 + stage_soff<!TB>(g.ldb, i)), 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa[i] = rdA(smem, i, 0);
    fbx[i] = rdB(smem, i, 0);
  }

  constexpr int NRD = (TA ? 2 : 1) + (TB ? 1 : 2);
  int pos = 0;  // K-tiles this workgroup has consumed: the LDS buffer of K-tile kt is (pos + kt) & 1
  for (;;) {
    for (int kt = 0; kt < L; ++kt) {
      unsigned char* cur = smem + ((pos + kt) & 1) * BUFT;
      unsigned char* nxt = smem + ((pos + kt + 1) & 1) * BUFT;
      // the loads issued now are for stream position kt + 2: this item's or the next one's
      const bool nx = kt + 2 >= L;
      const unsigned vA = nx ? voAn : voA, vB = nx ? voBn : voB;
      const unsigned kk = static_cast<unsigned>(nx ? kt0n + kt + 2 - L : kt0 + kt + 2);
      const unsigned ka = kk * kstepA, kb = kk * kstepB;
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = mfma16(fbx[nb], fa[mb], acc[mb][nb]);
        fa[mb] = rdA(cur, mb, 1);
        fby[mb] = rdB(cur, mb, 1);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int c = 2 * mb + h;
          if (c < 8) {
            *reinterpret_cast<i32x4t*>(nxt + stage_lds<TA>(c, tid)) = R[c];
            R[c] = __builtin_amdgcn_raw_buffer_load_b128(rA, vA,
                                                         __builtin_amdgcn_readfirstlane(ka + stage_soff<TA>(g.lda, c)), 0);
          } else {
            *reinterpret_cast<i32x4t*>(nxt + 2 * HALF + stage_lds<!TB>(c - 8, tid)) = R[c];
            R[c] = __builtin_amdgcn_raw_buffer_load_b128(
                rB, vB, __builtin_amdgcn_readfirstlane(kb + stage_soff<!TB>(g.ldb, c - 8)), 0);
          }
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, NRD, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = mfma16(fby[nb], fa[mb], acc[mb][nb]);
        fa[mb] = rdA(nxt, mb, 0);
        fbx[mb] = rdB(nxt, mb, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+a"(acc[i][j]));
    epilogue<EPI, ACT>(g, acc, m0, n0, split, wm, wn, lane);
    if (nitem >= W) break;   // uniform: every wave of the workgroup leaves together
    pos += L;
    item = nitem;
    m0 = m0n, n0 = n0n, split = splitn, voA = voAn, voB = voBn, kt0 = kt0n;
    nitem = item + static_cast<int>(gridDim.x);
    if (nitem < W) {
      geom(nitem, m0n, n0n, splitn);
      voAn = stage_voff<TA>(g.lda, m0n, tid);
      voBn = stage_voff<!TB>(g.ldb, n0n, tid);
      kt0n = splitn * L;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4t{};
  }
  // drain the (unused) loads of the stream's last two positions before exit
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool TA, bool TB>
void launch_pers(const GemmTArgs& g, dim3 grid, dim3 block, int epi, int act, hipStream_t st) {
  switch (epi * 8 + act) {
    case kEpiPlain * 8: hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiPlain, 0>), grid, block, 0, st, g); break;
    case kEpiSplit * 8: hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiSplit, 0>), grid, block, 0, st, g); break;
    case kEpiGeneral * 8:
      hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiGeneral, 0>), grid, block, 0, st, g);
      break;
    case kEpiAccum * 8: hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiAccum, 0>), grid, block, 0, st, g); break;
    case kEpiBiasAct * 8 + 0:
      hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiBiasAct, 0>), grid, block, 0, st, g);
      break;
    case kEpiBias * 8:
      hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiBias, 0>), grid, block, 0, st, g);
      break;
    case kEpiBiasAct * 8 + 1:
      hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiBiasAct, 1>), grid, block, 0, st, g);
      break;
    case kEpiBiasAct * 8 + 4:
      hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiBiasAct, 4>), grid, block, 0, st, g);
      break;
    case kEpiDact * 8 + 1: hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiDact, 1>), grid, block, 0, st, g); break;
    case kEpiDact * 8 + 4: hipLaunchKernelGGL((gemmt_pers_kernel<TA, TB, kEpiDact, 4>), grid, block, 0, st, g); break;
    default: throw std::invalid_argument("gemmt: activation without an instantiated epilogue");
  }
}

template <bool TA, bool TB, int S>
void launch_dbg(const GemmTArgs& g, dim3 grid, dim3 block, hipStream_t st) {
  if constexpr (S != 0) {   // LDS-DMA forms: the load-wait ablation only
    switch (g.dbg) {
      case 128: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, S, 128>), grid, block, 0, st, g); break;
      case 256: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, S, 256>), grid, block, 0, st, g); break;
      case 136: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, S, 136>), grid, block, 0, st, g); break;
      case 8: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, S, 8>), grid, block, 0, st, g); break;
      default: throw std::invalid_argument("gemmt: unsupported ablation bits");
    }
    return;
  }
  switch (g.dbg) {
    case 1: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, 0, 1>), grid, block, 0, st, g); break;
    case 2: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, 0, 2>), grid, block, 0, st, g); break;
    case 3: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, 0, 3>), grid, block, 0, st, g); break;
    case 4: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, 0, 4>), grid, block, 0, st, g); break;
    case 8: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, 0, 8>), grid, block, 0, st, g); break;
    case 15: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, 0, 15>), grid, block, 0, st, g); break;
    case 16: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, 0, 16>), grid, block, 0, st, g); break;
    case 32: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, 0, 32>), grid, block, 0, st, g); break;
    default: throw std::invalid_argument("gemmt: unsupported ablation bits");
  }
}

template <bool TA, bool TB, int S>
void launch_t(const GemmTArgs& g, dim3 grid, dim3 block, int epi, int act, hipStream_t st) {
  if constexpr (!TA) {
    if (g.dbg && epi == kEpiPlain) return launch_dbg<TA, TB, S>(g, grid, block, st);
  }
  switch (epi * 8 + act) {
    case kEpiPlain * 8: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiPlain, 0, S>), grid, block, 0, st, g); break;
    case kEpiSplit * 8: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiSplit, 0, S>), grid, block, 0, st, g); break;
    case kEpiGeneral * 8:
      hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiGeneral, 0, S>), grid, block, 0, st, g);
      break;
    case kEpiAccum * 8: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiAccum, 0, S>), grid, block, 0, st, g); break;
    case kEpiBiasAct * 8 + 0:
      hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiBiasAct, 0, S>), grid, block, 0, st, g);
      break;
    case kEpiBias * 8: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiBias, 0, S>), grid, block, 0, st, g); break;
    case kEpiBiasAct * 8 + 1:
      hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiBiasAct, 1, S>), grid, block, 0, st, g);
      break;
    case kEpiBiasAct * 8 + 4:
      hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiBiasAct, 4, S>), grid, block, 0, st, g);
      break;
    case kEpiDact * 8 + 1: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiDact, 1, S>), grid, block, 0, st, g); break;
    case kEpiDact * 8 + 4: hipLaunchKernelGGL((gemmt_kernel<TA, TB, kEpiDact, 4, S>), grid, block, 0, st, g); break;
    default: throw std::invalid_argument("gemmt: activation without an instantiated epilogue");
  }
}

template <bool TA, int SCH, bool TB, bool RS = false>
void launch_kk_s(const GemmTArgs& g, dim3 grid, dim3 block, int epi, int act, hipStream_t st) {
  switch (epi * 8 + act) {
    case kEpiPlain * 8:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiPlain, 0, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiSplit * 8:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiSplit, 0, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiGeneral * 8:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiGeneral, 0, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiAccum * 8:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiAccum, 0, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiBiasAct * 8 + 0:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiBiasAct, 0, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiBias * 8:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiBias, 0, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiBiasAct * 8 + 1:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiBiasAct, 1, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiBiasAct * 8 + 4:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiBiasAct, 4, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiDact * 8 + 1:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiDact, 1, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    case kEpiDact * 8 + 4:
      hipLaunchKernelGGL((gemmt_kk_kernel<TA, kEpiDact, 4, SCH, TB, RS>), grid, block, 0, st, g);
      break;
    default: throw std::invalid_argument("gemmt: activation without an instantiated epilogue");
  }
}

// interleaved group schedule by default: 1.5-11 % faster per GEMM and +0.7 %
// on the BERT-large step (profiles/r4/ab_gemmt_kk_sched_r4.txt);
// FFK_GEMMT_KK_SCHED=0 keeps the clustered one
template <bool TA, bool TB = false>
void launch_kk(const GemmTArgs& g, dim3 grid, dim3 block, int epi, int act, hipStream_t st) {
  static const int sch = [] {
    const char* e = std::getenv("FFK_GEMMT_KK_SCHED");
    return e != nullptr && e[0] == '0' ? 0 : 1;
  }();
  if (sch == 1) launch_kk_s<TA, 1, TB>(g, grid, block, epi, act, st);
  else launch_kk_s<TA, 0, TB>(g, grid, block, epi, act, st);
}

// padded-image kernel for A^T B and A B (FFK_GEMMT_KK=0 keeps the
// swizzled-image gemmt_kernel).  A/B on the BERT-large shapes
// (profiles/r4/ab_gemmt_kk_r4.txt): forward A B 1.5-4% faster, dW out 10%,
// dW qkv 2% slower, the rest within 1%
bool kk_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("FFK_GEMMT_KK");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

// A B^T through the same kernel (both operands K-contiguous, reads at lane
// base + immediate issued from asm, so hipcc's waitcnt pass does not make
// each LDS-DMA issue wait for the older fragment reads: 12 waits per K-tile
// in gemmt_kernel's loop, 3 here).  0.7-5.6 % faster per GEMM than
// gemmt_kernel on the BERT input-gradient shapes (hipBLASLt still ahead on
// most, profiles/r4/ab_gemmt_kk_nt_r4.txt); FFK_GEMMT_KK_NT=0 for A/B runs
bool kk_nt_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("FFK_GEMMT_KK_NT");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

}  // namespace

// the bias / activation / activation-gradient and plain bf16 epilogues take
// alpha = 1 (their callers' only use); other alphas go to gemmq
bool gemmt_supported(const GemmPParams& p) {
  const bool fused = p.bias || p.pre || p.act || p.act_bwd;
  return (p.act == 0 || p.act == 1 || p.act == 4) && (!fused || p.alpha == 1.f);
}

void gemmt_launch(const GemmPParams& p, int splits, int stage_mode, hipStream_t st) {
  auto bytes = [](int rows, int ld) {
    const uint64_t b = static_cast<uint64_t>(rows) * static_cast<uint64_t>(ld) * 2u;
    return static_cast<unsigned>(b > 0xFFFFFFFFull ? 0xFFFFFFFFull : b);
  };
  GemmTArgs g{static_cast<const bf16*>(p.A), static_cast<const bf16*>(p.B), p.C, p.workspace,
              static_cast<const bf16*>(p.bias), static_cast<bf16*>(p.pre), static_cast<const bf16*>(p.aux), p.dbias,
              p.M, p.N, p.K, p.lda, p.ldb, p.ldc, p.alpha, p.beta, p.act, p.act_bwd ? 1 : 0, p.out_f32, splits,
              bytes(p.trans_a ? p.K : p.M, p.lda), bytes(p.trans_b ? p.N : p.K, p.ldb), p.dbg};
  const int items = ((p.M + TM - 1) / TM) * ((p.N + TN - 1) / TN) * splits;
  dim3 grid(items), block(NTHREADS);
  const int epi = splits > 1                        ? kEpiSplit
                  : p.act_bwd                       ? kEpiDact
                  : (p.bias && !p.pre && !p.act)    ? kEpiBias
                  : (p.bias || p.pre || p.act)      ? kEpiBiasAct
                  : (!p.out_f32 && p.beta != 0.f && p.alpha == 1.f && !(p.dbg & 64) &&
                     (reinterpret_cast<uintptr_t>(p.C) & 15) == 0 && p.ldc % 8 == 0) ? kEpiAccum
                  : (p.out_f32 || p.beta != 0.f || p.alpha != 1.f) ? kEpiGeneral
                                                                   : kEpiPlain;
  const int L = p.K / TK / splits;
  if (stage_mode == 2 && L >= 2 && (p.K / TK) % splits == 0) {
    static int n_cu = [] {
      int dev = 0, n = 0;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                  hipSuccess || n <= 0)
        n = 256;
      return n;
    }();
    // a multiple of 8 workgroups (XCD-aware item mapping) unless all items fit
    const int pg = items <= n_cu ? items : (n_cu / 8) * 8;
    dim3 pgrid(pg);
    if (!p.trans_a && !p.trans_b) launch_pers<false, false>(g, pgrid, block, epi, p.act, st);
    else if (!p.trans_a && p.trans_b) launch_pers<false, true>(g, pgrid, block, epi, p.act, st);
    else if (p.trans_a && !p.trans_b) launch_pers<true, false>(g, pgrid, block, epi, p.act, st);
    else launch_pers<true, true>(g, pgrid, block, epi, p.act, st);
  } else if (stage_mode == 7 && !(p.trans_a && p.trans_b)) {   // kk images, register-staged (variant 10)
    if (!p.trans_a && !p.trans_b) launch_kk_s<false, 1, false, true>(g, grid, block, epi, p.act, st);
    else if (!p.trans_a && p.trans_b) launch_kk_s<false, 1, true, true>(g, grid, block, epi, p.act, st);
    else launch_kk_s<true, 1, false, true>(g, grid, block, epi, p.act, st);
  } else if (stage_mode == 3 || stage_mode == 7) {   // both operands by LDS-DMA
    const bool kk = kk_enabled() && !p.dbg;
    if (!p.trans_a && !p.trans_b) {
      if (kk) launch_kk<false>(g, grid, block, epi, p.act, st);
      else launch_t<false, false, 2>(g, grid, block, epi, p.act, st);
    } else if (!p.trans_a && p.trans_b) {
      if (kk && kk_nt_enabled()) launch_kk<false, true>(g, grid, block, epi, p.act, st);
      else launch_t<false, true, 2>(g, grid, block, epi, p.act, st);
    } else if (p.trans_a && !p.trans_b) {
      if (kk) launch_kk<true>(g, grid, block, epi, p.act, st);
      else launch_t<true, false, 2>(g, grid, block, epi, p.act, st);
    } else {
      launch_t<true, true, 2>(g, grid, block, epi, p.act, st);
    }
  } else if (stage_mode == 1) {
    if (!p.trans_a && !p.trans_b) launch_t<false, false, 1>(g, grid, block, epi, p.act, st);
    else if (!p.trans_a && p.trans_b) launch_t<false, true, 1>(g, grid, block, epi, p.act, st);
    else if (p.trans_a && !p.trans_b) launch_t<true, false, 1>(g, grid, block, epi, p.act, st);
    else launch_t<true, true, 1>(g, grid, block, epi, p.act, st);
  } else {
    if (!p.trans_a && !p.trans_b) launch_t<false, false, 0>(g, grid, block, epi, p.act, st);
    else if (!p.trans_a && p.trans_b) launch_t<false, true, 0>(g, grid, block, epi, p.act, st);
    else if (p.trans_a && !p.trans_b) launch_t<true, false, 0>(g, grid, block, epi, p.act, st);
    else launch_t<true, true, 0>(g, grid, block, epi, p.act, st);
  }
  FFK_LAUNCH_CHECK("gemmt");
}

}  // namespace ffk
