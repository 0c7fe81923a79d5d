// Eight-wave ping-pong bf16 GEMM for gfx950 (GemmPParams.variant = 11).
//
// C[M][N] (+)= A[M][K] B[N][K]^T (+ bias), both operands K-contiguous: the
// input-gradient products dX = dY W^T of every Linear and the vocabulary
// head's -- the signatures hipBLASLt still won against the one-wave-per-SIMD
// kernels (gemmt.hip), whose MFMA pipe idles whenever its only wave waits on
// a barrier, an LDS read or pays an LDS-DMA issue (60-185 cycles among
// MFMAs, MI355X_MICROARCH.md cycle constants).  Parity:
// lib/kernels/src/cuda/ops/linear_kernels.cu:303 (the dX cublasGemmEx).
//
// Geometry: a 256 x 256 x 64 tile per workgroup of 8 waves.  Waves 0-3
// (group 0) own output rows 0-127 of the tile, waves 4-7 (group 1) rows
// 128-255; inside a group the waves are 2 x 2, a 64 x 128 sub-tile each =
// 4 x 8 v_mfma_f32_16x16x32_bf16 blocks (128 accumulator registers).  Wave
// w and w + 4 share a SIMD (waves are dealt to SIMDs cyclically), so every
// SIMD holds one wave of each group.
//
// Schedule: every wave runs the same loop -- load half (issue the LDS-DMA of
// tile t + 1, read all 24 fragments of tile t), barrier, compute half (64
// MFMAs from registers), barrier -- and group 1 starts one barrier late, so
//   half-period 2t:     group 0 loads tile t      | group 1 computes tile t - 1
//   half-period 2t + 1: group 0 computes tile t   | group 1 loads tile t
// and each SIMD's matrix pipe alternates between its two waves, never
// waiting on memory (cdna_hip_programming.md, two waves per SIMD).  One
// instruction stream for both groups keeps hipcc from giving the two roles
// separate fragment registers joined by copies (a role-branched version
// spilled ~400 registers).
// LDS: two buffers x (A + B) x 32 KiB; the 128-B-row images use the chunk
// swizzle c ^ ((row >> 1) & 7) (bank-conflict-free ds_read_b128 and DMA
// writes), each 1-KiB DMA piece lane-linear with the logical chunk its
// physical slot holds as each lane's source.
// WAR / RAW: tile t + 1 goes to buffer (t + 1) & 1 in half-period 2t, after
// both groups' reads of tile t - 1 (half-periods 2t - 2 and 2t - 1); group 0
// waits for its pieces (vmcnt(0)) at the end of its compute half 2t + 1,
// before the barrier that precedes the first reads of tile t + 1.
// DS = 1 splits the DMA: group 0 issues A, group 1 issues B of tile t + 1 in
// its own load half (2t + 1) and waits for it at that half's end.
// Accumulators hold C^T (mfma(B fragment, A fragment)): lane & 15 -> m,
// 4 (lane >> 4) + e -> n.  Epilogues: plain bf16, C += AB (beta, one
// rounding), + bias.  Group 0 stores beside group 1's last MFMAs.
//
// Measured (profiles/r5/ab_gemmpp_r5.txt, BERT-large dX shapes): correct to
// the bf16 output rounding; 5-6 % ahead of the one-wave kernels on dX QKV /
// FFN1, 2-4 % behind them on dX FFN2 / head, 8-20 % behind hipBLASLt.  The
// ablations place the cost: MFMA + barriers alone run the head shape at
// 1.92 PFLOP/s (the ping-pong itself is efficient), the fragment reads add
// 8 %, the LDS-DMA another 33 % -- the load half is bound by the DMA pieces'
// issue cost (100-185 cycles each beside 24 ds_read_b128), not by their
// latency (a third A buffer, prefetch distance 2, moved it < 1 %).  Moving 2-4
// of each wave's DMA pieces into its compute half did not help either
// (profiles/r5/ab_gemmpp_cn_r5.txt): what the DMA costs is not issue slots
// alone but its LDS writes beside the fragment reads.
#include <utility>

#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int QM = 256, QN = 256, QK = 64, QTH = 512;
constexpr int QOP = 256 * 128;   // one operand image per buffer (32 KiB)
constexpr int QGROUP = 4;        // M-tiles per raster group
typedef float q4f __attribute__((ext_vector_type(4)));
typedef float q2f __attribute__((ext_vector_type(2)));
typedef __bf16 qbf2 __attribute__((ext_vector_type(2)));

enum { kQPlain = 0, kQAccum = 1, kQBias = 2 };

struct GemmQArgs {
  const bf16* A;
  const bf16* B;
  bf16* C;
  const bf16* bias;
  int M, N, K, lda, ldb, ldc;
  float beta;
  unsigned bytesA, bytesB;
};

__device__ __forceinline__ q4f qmfma(bf16x8 a, bf16x8 b, q4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// fragment read at lane base + immediate, hidden from hipcc's wait-count
// pass (the caller waits lgkmcnt(0) before the consumer)
template <int OFF>
__device__ __forceinline__ bf16x8 qrd(unsigned base) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(base), "i"(OFF));
  return r;
}

__device__ __forceinline__ void qdma(__amdgpu_buffer_rsrc_t r, unsigned char* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// per-lane voffset (bytes, K-tile 0) of DMA piece parity `par` of issuing
// wave q: the piece covers rows 8 (8 q + i) .. +8, lane -> row + (lane >> 3),
// physical slot lane & 7 holds logical chunk slot ^ ((row >> 1) & 7), which
// depends on the piece index only through i & 1
__device__ __forceinline__ unsigned q_dma_voff(int ld, int outer0, int par, int q, int lane) {
  const int row = 8 * (8 * q + par) + (lane >> 3);
  const int c = (lane & 7) ^ ((row >> 1) & 7);
  return (static_cast<unsigned>(outer0 + row) * static_cast<unsigned>(ld) + static_cast<unsigned>(c * 8)) * 2u;
}

__device__ __forceinline__ unsigned q_pack2(q2f v) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, qbf2));
}

template <typename F, int... I>
__device__ __forceinline__ void q_for(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}

template <int EPI, int DS, int PRIO>
__global__ __launch_bounds__(QTH, 1) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemmpp_kernel(GemmQArgs g) {
  // DS 2: [A0][A1][A2][B0][B1] = 160 KiB (the whole LDS); else [A0][A1][B0][B1]
  constexpr int NA = DS == 2 ? 3 : 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[(NA + 2) * QOP];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wave >> 2, q = wave & 3;
  const int wm = q >> 1, wn = q & 1;

  // ---- tile: bijective XCD remap + grouped raster (QGROUP M-tiles share B in L2)
  const int gm = (g.M + QM - 1) / QM, gn = (g.N + QN - 1) / QN;
  const int nwg = gm * gn;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int per_group = QGROUP * gn;
  const int first_m = (t / per_group) * QGROUP;
  const int gsize = min(gm - first_m, QGROUP);
  const int m0 = (first_m + (t % per_group) % gsize) * QM;
  const int n0 = ((t % per_group) / gsize) * QN;
  const int L = g.K / QK;

  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.A), static_cast<short>(0), g.bytesA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.B), static_cast<short>(0), g.bytesB, 0x00020000);
  const unsigned dvA0 = q_dma_voff(g.lda, m0, 0, q, lane), dvA1 = q_dma_voff(g.lda, m0, 1, q, lane);
  const unsigned dvB0 = q_dma_voff(g.ldb, n0, 0, q, lane), dvB1 = q_dma_voff(g.ldb, n0, 1, q, lane);
  unsigned char* const sA = smem;
  unsigned char* const sB = smem + NA * QOP;
  // the 8 pieces of one operand tile issued by wave q of the issuing group
  auto dmaA = [&](int buf, int kt) __attribute__((always_inline)) {
    const unsigned kb = static_cast<unsigned>(kt) * (QK * 2u);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const unsigned so = kb + static_cast<unsigned>(8 * (i & ~1)) * static_cast<unsigned>(g.lda) * 2u;
      qdma(rA, sA + buf * QOP + (8 * q + i) * 1024, (i & 1) ? dvA1 : dvA0, __builtin_amdgcn_readfirstlane(so));
    }
  };
  auto dmaB = [&](int buf, int kt) __attribute__((always_inline)) {
    const unsigned kb = static_cast<unsigned>(kt) * (QK * 2u);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const unsigned so = kb + static_cast<unsigned>(8 * (i & ~1)) * static_cast<unsigned>(g.ldb) * 2u;
      qdma(rB, sB + buf * QOP + (8 * q + i) * 1024, (i & 1) ? dvB1 : dvB0, __builtin_amdgcn_readfirstlane(so));
    }
  };

  // fragment lane bases: rows o0 + (lane & 15) (o0 % 16 == 0), k-step ks:
  // byte (lane & 15) * 128 + (((4 ks + (lane >> 4)) ^ (((lane & 15) >> 1) & 7)) << 4) + o0 * 128
  const unsigned lds0 = static_cast<unsigned>(
      reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) unsigned char*)smem));
  const int li = lane & 15;
  auto lbase = [&](int ks) -> unsigned {
    return static_cast<unsigned>(li * 128 + ((((4 * ks) + (lane >> 4)) ^ ((li >> 1) & 7)) << 4));
  };
  const unsigned aB0 = lds0 + static_cast<unsigned>((grp * 128 + wm * 64) * 128) + lbase(0);
  const unsigned aB1 = lds0 + static_cast<unsigned>((grp * 128 + wm * 64) * 128) + lbase(1);
  const unsigned bB0 = lds0 + static_cast<unsigned>(NA * QOP + wn * 128 * 128) + lbase(0);
  const unsigned bB1 = lds0 + static_cast<unsigned>(NA * QOP + wn * 128 * 128) + lbase(1);

  q4f acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = q4f{};
  bf16x8 fa0[4], fa1[4], fb0[8], fb1[8];
  constexpr auto S4 = std::make_integer_sequence<int, 4>{};
  constexpr auto S8 = std::make_integer_sequence<int, 8>{};

  // all 24 fragments of the tile in buffer `buf`, retired before returning
  auto memread = [&](int abuf, int bbuf) __attribute__((always_inline)) {
    const unsigned oa = static_cast<unsigned>(abuf * QOP), ob = static_cast<unsigned>(bbuf * QOP);
    const unsigned a0 = aB0 + oa, a1 = aB1 + oa, b0 = bB0 + ob, b1 = bB1 + ob;
    q_for([&](auto I) __attribute__((always_inline)) {
      constexpr int i = decltype(I)::value;
      fb0[i] = qrd<i * 2048>(b0);
      if constexpr (i < 4) fa0[i] = qrd<i * 2048>(a0);
    }, S8);
    q_for([&](auto I) __attribute__((always_inline)) {
      constexpr int i = decltype(I)::value;
      fb1[i] = qrd<i * 2048>(b1);
      if constexpr (i < 4) fa1[i] = qrd<i * 2048>(a1);
    }, S8);
  };
  // wait for the reads and pin the fragments behind the wait
  auto retire = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(fa0[i]), "+v"(fa1[i]));
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" : "+v"(fb0[i]), "+v"(fb1[i]));
    __builtin_amdgcn_sched_barrier(0);
  };
  auto compute = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = qmfma(fb0[nb], fa0[mb], acc[mb][nb]);
#pragma unroll
    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = qmfma(fb1[nb], fa1[mb], acc[mb][nb]);
    if (PRIO) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  };

  auto epilogue = [&]() __attribute__((always_inline)) {
    const int r = lane >> 4;
    const int ncol0 = n0 + wn * 128;
    float bv[8][4];
    if (EPI == kQBias) {
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
        const int n = min(ncol0 + nb * 16 + 4 * r, g.N - 4);
        const bf16x4 bb = *reinterpret_cast<const bf16x4*>(g.bias + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[nb][e] = bf2f(bb[e]);
      }
    }
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int m = m0 + grp * 128 + wm * 64 + mb * 16 + li;
      const bool mok = m < g.M;
      const int64_t roff = static_cast<int64_t>(mok ? m : g.M - 1) * g.ldc;
      if (EPI == kQAccum) {
        // per block pair: four fp32 permlane16 swaps give lane row r 8
        // consecutive columns, one 16-B read of C, fp32 adds, one 16-B store
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          unsigned s[4][2];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const auto w = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[mb][2 * j][e]),
                                                            __float_as_uint(acc[mb][2 * j + 1][e]), false, false);
            s[e][0] = w[0];
            s[e][1] = w[1];
          }
          const int n = ncol0 + (2 * j + (r & 1)) * 16 + (r >> 1) * 8;
          if (mok && n < g.N) {
            uint4* p = reinterpret_cast<uint4*>(g.C + roff + n);
            const uint4 old = *p;
            const unsigned ow[4] = {old.x, old.y, old.z, old.w};
            unsigned nw[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const int h = c >> 1, e0 = 2 * (c & 1);
              const q2f v{__uint_as_float(s[e0][h]), __uint_as_float(s[e0 + 1][h])};
              const q2f o{__uint_as_float(ow[c] << 16), __uint_as_float(ow[c] & 0xFFFF0000u)};
              nw[c] = q_pack2(v + g.beta * o);
            }
            *p = uint4{nw[0], nw[1], nw[2], nw[3]};
          }
        }
        continue;
      }
      uint2 ob[8];
#pragma unroll
      for (int nb = 0; nb < 8; ++nb) {
        q2f v0{acc[mb][nb][0], acc[mb][nb][1]}, v1{acc[mb][nb][2], acc[mb][nb][3]};
        if (EPI == kQBias) {
          v0 += q2f{bv[nb][0], bv[nb][1]};
          v1 += q2f{bv[nb][2], bv[nb][3]};
        }
        ob[nb] = uint2{q_pack2(v0), q_pack2(v1)};
      }
      // 16-B stores: v_permlane16_swap pairs the odd 16-lane rows of block 2j
      // with the even rows of block 2j + 1 (row r then holds 8 consecutive
      // columns of block 2j + (r & 1))
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const auto sx = __builtin_amdgcn_permlane16_swap(ob[2 * j].x, ob[2 * j + 1].x, false, false);
        const auto sy = __builtin_amdgcn_permlane16_swap(ob[2 * j].y, ob[2 * j + 1].y, false, false);
        const int n = ncol0 + (2 * j + (r & 1)) * 16 + (r >> 1) * 8;
        if (mok && n < g.N) *reinterpret_cast<uint4*>(g.C + roff + n) = uint4{sx[0], sy[0], sx[1], sy[1]};
      }
    }
  };

  // ---- one instruction stream for both groups, group 1 one barrier behind
  // (no role-dependent register data flow: hipcc keeps one fragment set)
  if (grp == 0) {
    dmaA(0, 0);
    if (DS == 2) dmaA(1, 1);
    if (DS == 0) dmaB(0, 0);
  } else if (DS != 0) {
    dmaB(0, 0);
  }
  if (DS == 2 && grp == 0 && L > 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // A(0) landed, A(1) in flight
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if (grp != 0) {
    __builtin_amdgcn_s_barrier();   // group 1 runs one half-period behind
    asm volatile("" ::: "memory");
  }
  int abuf = 0;   // kt % NA
  for (int kt = 0; kt < L; ++kt) {
    const int buf = kt & 1;
    const int anext = abuf + 2 >= NA ? abuf + 2 - NA : abuf + 2;   // DS 2: (kt + 2) % 3
    // ---- load half: the DMA of a later tile into a buffer both groups have
    // finished reading, then this tile's fragments
    if (DS == 2) {
      if (grp == 0 && kt + 2 < L) dmaA(anext, kt + 2);
      if (grp != 0 && kt + 1 < L) dmaB(buf ^ 1, kt + 1);
    } else if (kt + 1 < L) {
      if (grp == 0) {
        dmaA(buf ^ 1, kt + 1);
        if (DS == 0) dmaB(buf ^ 1, kt + 1);
      } else if (DS == 1) {
        dmaB(buf ^ 1, kt + 1);
      }
    }
    memread(DS == 2 ? abuf : buf, buf);
    retire();
    if (DS != 0 && grp != 0 && kt + 1 < L) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // B(kt + 1) landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // ---- compute half
    compute();
    if (grp == 0 && kt + 1 < L) {   // A (DS 0: and B) of tile kt + 1 landed
      if (DS == 2 && kt + 2 < L) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // A(kt + 2) may fly on
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    abuf = abuf + 1 == NA ? 0 : abuf + 1;
  }
  epilogue();
  if (grp == 0) {
    __builtin_amdgcn_s_barrier();   // pairs with group 1's last one (its final compute)
    asm volatile("" ::: "memory");
  }
}

template <int DS, int PRIO>
void launch_q(const GemmQArgs& g, int epi, dim3 grid, hipStream_t st) {
  switch (epi) {
    case kQAccum: hipLaunchKernelGGL((gemmpp_kernel<kQAccum, DS, PRIO>), grid, dim3(QTH), 0, st, g); break;
    case kQBias: hipLaunchKernelGGL((gemmpp_kernel<kQBias, DS, PRIO>), grid, dim3(QTH), 0, st, g); break;
    default: hipLaunchKernelGGL((gemmpp_kernel<kQPlain, DS, PRIO>), grid, dim3(QTH), 0, st, g); break;
  }
}

}  // namespace

bool gemmpp_supported(const GemmPParams& p) {
  const uint64_t a_bytes = uint64_t(p.M) * uint64_t(p.lda) * 2u;
  const uint64_t b_bytes = uint64_t(p.N) * uint64_t(p.ldb) * 2u;
  return !p.trans_a && p.trans_b && p.K % QK == 0 && p.K / QK >= 2 && p.lda % 8 == 0 && p.ldb % 8 == 0 &&
         p.N % 8 == 0 && p.ldc % 8 == 0 && !p.out_f32 && p.alpha == 1.f && !p.act && !p.pre && !p.act_bwd &&
         !p.dbias && !(p.bias && p.beta != 0.f) && a_bytes < (1ull << 32) && b_bytes < (1ull << 32) &&
         ((reinterpret_cast<uintptr_t>(p.A) | reinterpret_cast<uintptr_t>(p.B) | reinterpret_cast<uintptr_t>(p.C)) &
          15) == 0 &&
         (!p.bias || (reinterpret_cast<uintptr_t>(p.bias) & 7) == 0);
}

// FFK_GEMMPP_MODE (or GemmPParams.dbg with bit 4 set): bits 0-1 = DS (0, 1,
// 2), bit 2 = s_setprio 1 over each compute half (timing A/Bs; default 6)
void gemmpp_launch(const GemmPParams& p, hipStream_t st) {
  if (!gemmpp_supported(p)) throw std::invalid_argument("gemmpp: unsupported layout / epilogue / alignment");
  GemmQArgs g{static_cast<const bf16*>(p.A), static_cast<const bf16*>(p.B), static_cast<bf16*>(p.C),
              static_cast<const bf16*>(p.bias), p.M, p.N, p.K, p.lda, p.ldb, p.ldc, p.beta,
              static_cast<unsigned>(uint64_t(p.M) * uint64_t(p.lda) * 2u),
              static_cast<unsigned>(uint64_t(p.N) * uint64_t(p.ldb) * 2u)};
  const int epi = p.bias ? kQBias : p.beta != 0.f ? kQAccum : kQPlain;
  const dim3 grid(((p.M + QM - 1) / QM) * ((p.N + QN - 1) / QN));
  static const int env_mode = [] {
    const char* e = std::getenv("FFK_GEMMPP_MODE");
    return e ? std::atoi(e) : 6;
  }();
  // dbg (bit 4 set): same-process A/Bs (tools/gemm_ab.py)
  const int mode = (p.dbg & 16) ? (p.dbg & 15) : env_mode;
  switch (mode & 7) {
    case 0: launch_q<0, 0>(g, epi, grid, st); break;
    case 1: launch_q<1, 0>(g, epi, grid, st); break;
    case 2: launch_q<2, 0>(g, epi, grid, st); break;
    case 4: launch_q<0, 1>(g, epi, grid, st); break;
    case 5: launch_q<1, 1>(g, epi, grid, st); break;
    default: launch_q<2, 1>(g, epi, grid, st); break;
  }
  FFK_LAUNCH_CHECK("gemmpp");
}

}  // namespace ffk
