// gemmp's phase pipeline on v_mfma_f32_16x16x32_bf16 (GemmPParams.variant = 1).
//
// Same tile (256 x 256 x 64, 8 waves as 2 (M) x 4 (N), a 128 x 64 output per
// wave), the same four 16 KiB operand units per K-tile read in exactly one
// phase each, the same counted vmcnt(8) across raw barriers and the same
// persistent work-item stream with fused training epilogues as gemmp.hip.
// What differs is the matrix instruction: each phase is 16 x 16x32 MFMAs
// (one 64 x 32 quadrant of the wave's output, K = 64) instead of 8 x 32x32x16.
// Equal cycles per FLOP, but on random bf16 operands the chip holds a higher
// clock on the 16x16x32 shape (MI355X_MICROARCH.md 'DVFS give-back' item 7:
// 1.12-1.15x the FLOP/s of 32x32x16 loops reading operands from LDS).
//
// Operand images: K-contiguous operands as [128 outer][64 k] with 128-B rows
// and slot = chunk ^ ((row >> 1) & 7): a 16x16x32 row read (lane -> row
// lane & 15, chunk + (lane >> 4), ds_read_b128) covers 16 distinct 16-B slots
// in each of its four lane groups (conflict-free; gemmp's 128-B swizzle is
// 2-way for this read pattern).  K-outer operands as [64 k][128 outer] with
// 256-B rows (mfma.h swizzle) read by two ds_read_b64_tr_b16 per fragment,
// also conflict-free.  tools/lds_conflicts.py checks both.
//
// Accumulators hold C^T: D column (lane & 15) -> m, D row 4 * (lane >> 4) + e
// -> n, so a lane owns 4 consecutive n of one row (8-byte bf16 stores).
#include <type_traits>

#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int TM = 256, TN = 256, TK = 64, NTHREADS = 512;
constexpr int UNIT = 16 * 1024;  // 128 outer x 64 k bf16
constexpr int BUF = 4 * UNIT;    // one K-tile: units A0 A1 B0 B1
constexpr int GROUP = 4;
typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef float f32x4q __attribute__((ext_vector_type(4)));

struct GemmQArgs {
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
  int dbg;
};

__device__ __forceinline__ float q_act(int act, float x) {
  switch (act) {
    case 1: return x > 0.f ? x : 0.f;
    case 2: return 1.f / (1.f + __expf(-x));
    case 3: return fast_tanh(x);
    case 4: return gelu_tanh(x);
    default: return x;
  }
}
__device__ __forceinline__ float q_act_grad(int act, float x) {
  switch (act) {
    case 1: return x > 0.f ? 1.f : 0.f;
    case 2: {
      const float s = 1.f / (1.f + __expf(-x));
      return s * (1.f - s);
    }
    case 3: {
      const float t = fast_tanh(x);
      return 1.f - t * t;
    }
    case 4: return gelu_tanh_grad(x);
    default: return 1.f;
  }
}

// 128-B-row image slot of logical 16-B chunk c in row r (an involution in c)
__device__ __forceinline__ int q_slot128(int r, int c) { return c ^ ((r >> 1) & 7); }

__device__ __forceinline__ f32x4q mfma16(bf16x8 a, bf16x8 b, f32x4q c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <bool IS_A>
__device__ __forceinline__ int unit_outer(int u, int o) {
  if (IS_A) return (o >> 6) * 128 + u * 64 + (o & 63);
  return (o >> 5) * 64 + u * 32 + (o & 31);
}

// Stage unit u of one operand (K-tile at k0) into `img`: 16 x 1 KiB LDS-DMA
// pieces, 2 per wave.  The DMA destination is lane-linear, so the swizzle is
// applied to the per-lane global source address (guide rule 21).
template <bool IS_A, bool KOUTER>
__device__ __forceinline__ void stage_unit(const bf16* __restrict__ P, int ld, int outer0, int n_outer, int k0, int u,
                                           unsigned char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = wave * 2 + i;
    const bf16* src;
    if (KOUTER) {
      const int r = 4 * j + (lane >> 4);
      const int c = swz_chunk<256>(r, lane & 15);
      int col = outer0 + unit_outer<IS_A>(u, c * 8);
      col = min(col, n_outer - 8);
      src = P + static_cast<int64_t>(k0 + r) * ld + col;
    } else {
      const int r = 8 * j + (lane >> 3);
      const int c = q_slot128(r, lane & 7);
      const int row = min(outer0 + unit_outer<IS_A>(u, r), n_outer - 1);
      src = P + static_cast<int64_t>(row) * ld + k0 + c * 8;
    }
    __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)(img + j * 1024), 16, 0, 0);
  }
}

// 16x16x32 operand fragment, K-contiguous image: lane holds
// image[o0 + (lane & 15)][32 ks + 8 (lane >> 4) .. +8].
__device__ __forceinline__ bf16x8 row16(const unsigned char* img, int o0, int ks, int lane) {
  const int r = o0 + (lane & 15);
  return lds_read16(img, r * 128 + (q_slot128(r, ks * 4 + (lane >> 4)) << 4));
}
// 16x16x32 operand fragment, K-outer image [k][outer]: lane holds
// image[32 ks + 8 (lane >> 4) + j][o0 + (lane & 15)], j = 0..7, from two
// transposed reads (guide T10: lane 4q+p of each 16-lane group addresses
// row q, columns 4p..4p+3 of a 4 x 16 block).
__device__ __forceinline__ bf16x8 tr16(const unsigned char* img, int ks, int o0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = o0 + 4 * (i & 3);
  const int r = ks * 32 + 8 * g + (i >> 2);
  const int oa = img_off<256>(r, col >> 3) + (col & 7) * 2;
  const int ob = img_off<256>(r + 4, col >> 3) + (col & 7) * 2;
  return cat44(lds_tr_asm(img, oa), lds_tr_asm(img, ob));
}

__device__ __forceinline__ void lds_ready() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void phase_sync(bool pipelined, int dbg = 0) {
  if (!(dbg & 1)) {
    if (!pipelined) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  if (!(dbg & 2)) __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

enum Epi : int { kEpiPlain = 0, kEpiBiasAct = 1, kEpiDact = 2, kEpiSplit = 3 };

// acc[qn][qm][mb][nb]: 16 x 16 C^T blocks.  Row m = m0 + wm*128 + qm*64 +
// mb*16 + (lane & 15); columns n = n0 + wn*64 + qn*32 + nb*16 + 4 (lane >> 4) + e.
template <int EPI>
__device__ __forceinline__ void epilogue(const GemmQArgs& g, f32x4q (&acc)[2][2][4][2], int m0, int n0, int split,
                                         int wm, int wn, int lane) {
  const int nl = 4 * (lane >> 4);
  bf16x4 bias[2][2];
  if (EPI == kEpiBiasAct) {
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) {
        const int n = min(n0 + wn * 64 + qn * 32 + nb * 16 + nl, g.N - 4);
        bias[qn][nb] = g.bias ? *reinterpret_cast<const bf16x4*>(g.bias + n) : bf16x4{};
      }
  }
  float csum[2][2][4];
  if (EPI == kEpiDact) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int c = 0; c < 4; ++c) csum[a][b][c] = 0.f;
  }
#pragma unroll
  for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int m_raw = m0 + wm * 128 + qm * 64 + mb * 16 + (lane & 15);
      const bool mok = m_raw < g.M;
      const int m = mok ? m_raw : g.M - 1;
      bf16x4 xa[2][2];
      f32x4q old[2][2];
      if (EPI == kEpiDact || (EPI == kEpiPlain && g.beta != 0.f)) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) {
            const int n = min(n0 + wn * 64 + qn * 32 + nb * 16 + nl, g.N - 4);
            const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
            if (EPI == kEpiDact) {
              xa[qn][nb] = *reinterpret_cast<const bf16x4*>(g.aux + off);
            } else if (g.out_f32) {
              old[qn][nb] = *reinterpret_cast<const f32x4q*>(static_cast<const float*>(g.C) + off);
            } else {
              const bf16x4 o = *reinterpret_cast<const bf16x4*>(static_cast<const bf16*>(g.C) + off);
              old[qn][nb] = f32x4q{bf2f(o[0]), bf2f(o[1]), bf2f(o[2]), bf2f(o[3])};
            }
          }
      }
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const int n_raw = n0 + wn * 64 + qn * 32 + nb * 16 + nl;
          const bool ok = mok && n_raw < g.N;  // N % 8 == 0: a 4-group is all-in or all-out
          const int n = ok ? n_raw : min(n_raw, g.N - 4);
          const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[qn][qm][mb][nb][e];
          if (EPI == kEpiSplit) {
            float* W = g.ws + (static_cast<int64_t>(split) * g.M + m) * g.N + n;
            if (ok) *reinterpret_cast<f32x4q*>(W) = f32x4q{v[0], v[1], v[2], v[3]};
            continue;
          }
          if (EPI == kEpiBiasAct) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += bf2f(bias[qn][nb][e]);
            if (g.pre && ok) {
              bf16x4 pv;
#pragma unroll
              for (int e = 0; e < 4; ++e) pv[e] = f2bf(v[e]);
              *reinterpret_cast<bf16x4*>(g.pre + off) = pv;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = q_act(g.act, v[e]);
          }
          if (EPI == kEpiDact) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= q_act_grad(g.act, bf2f(xa[qn][nb][e]));
          }
          if (EPI == kEpiPlain && g.beta != 0.f) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += g.beta * old[qn][nb][e];
          }
          if (EPI == kEpiPlain && g.out_f32) {
            if (ok) *reinterpret_cast<f32x4q*>(static_cast<float*>(g.C) + off) = f32x4q{v[0], v[1], v[2], v[3]};
          } else {
            bf16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
            if (EPI == kEpiDact) {
#pragma unroll
              for (int e = 0; e < 4; ++e) csum[qn][nb][e] += ok ? bf2f(o[e]) : 0.f;
            }
            if (ok) *reinterpret_cast<bf16x4*>(static_cast<bf16*>(g.C) + off) = o;
          }
        }
      }
    }
  }
  if (EPI == kEpiDact && g.dbias) {
    // sum over the 16 rows (lanes) of each 16-lane group, one atomic per column
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float sm = csum[qn][nb][e];
#pragma unroll
          for (int o = 8; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
          const int n = n0 + wn * 64 + qn * 32 + nb * 16 + nl + e;
          if ((lane & 15) == 0 && n < g.N) atomicAdd(g.dbias + n, sm);
        }
  }
}

struct Geom {
  int m0, n0, kt0;
};

template <bool TA, bool TB, int EPI>
__global__ __launch_bounds__(NTHREADS, 1) void gemmq_kernel(GemmQArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF];  // the ONE LDS object
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;

  const int gm = (g.M + TM - 1) / TM, gn = (g.N + TN - 1) / TN;
  const int nwg = gm * gn;
  const int L = g.K / TK / g.splits;
  const int W = nwg * g.splits;
  const int G = gridDim.x;
  const int n_items = (W - static_cast<int>(blockIdx.x) + G - 1) / G;
  const int S = n_items * L;

  auto geom = [&](int i) {
    const int w = blockIdx.x + i * G;
    const int bid = xcd_remap(w, W);
    const int split = bid / nwg, t = bid % nwg;
    const int per_group = GROUP * gn;
    const int first_m = (t / per_group) * GROUP;
    const int gsize = min(gm - first_m, GROUP);
    const int tm = first_m + (t % per_group) % gsize;
    const int tn = (t % per_group) / gsize;
    return Geom{tm * TM, tn * TN, split * L};
  };
  auto unitA = [&](int s, int u) { return smem + (s & 1) * BUF + u * UNIT; };
  auto unitB = [&](int s, int u) { return smem + (s & 1) * BUF + (2 + u) * UNIT; };
  struct Pos {
    int s, item, j;
    Geom q;
  };
  auto advance = [&](Pos& p) {
    ++p.s;
    if (++p.j == L) {
      p.j = 0;
      ++p.item;
      if (p.s < S) p.q = geom(p.item);
    }
  };
  auto stA = [&](const Pos& p, int u) {
    if (p.s >= S) return;
    stage_unit<true, TA>(g.A, g.lda, p.q.m0, g.M, (p.q.kt0 + p.j) * TK, u, unitA(p.s, u), wave, lane);
  };
  auto stB = [&](const Pos& p, int u) {
    if (p.s >= S) return;
    stage_unit<false, !TB>(g.B, g.ldb, p.q.n0, g.N, (p.q.kt0 + p.j) * TK, u, unitB(p.s, u), wave, lane);
  };
  auto rdA = [&](const unsigned char* img, int mb, int ks) -> bf16x8 {
    return TA ? tr16(img, ks, wm * 64 + mb * 16, lane) : row16(img, wm * 64 + mb * 16, ks, lane);
  };
  auto rdB = [&](const unsigned char* img, int nb, int ks) -> bf16x8 {
    return TB ? row16(img, wn * 32 + nb * 16, ks, lane) : tr16(img, ks, wn * 32 + nb * 16, lane);
  };

  f32x4q acc[2][2][4][2];  // [qn][qm][mb][nb]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4q{};
  bf16x8 fa0[4][2], fa1[4][2], fb0[2][2], fb1[2][2];  // [block][kstep]

  Pos p1{0, 0, 0, geom(0)};
  stA(p1, 0);
  stB(p1, 0);
  stB(p1, 1);
  stA(p1, 1);
  advance(p1);
  stA(p1, 0);
  stB(p1, 0);
  stB(p1, 1);
  Pos p2 = p1;
  advance(p2);
  phase_sync(S >= 2);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) fa0[mb][ks] = rdA(unitA(0, 0), mb, ks);
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) fb0[nb][ks] = rdB(unitB(0, 0), nb, ks);
  }

  bool after_epilogue = false;
  for (int s = 0, j = 0, item = 0; s < S; ++s) {
    const bool more1 = s + 1 < S, more2 = s + 2 < S;
    // ---- P1: q0 x b0 | read B1(s) | stage A1(s+1)
    phase_sync(more1 && !after_epilogue, g.dbg);
    lds_ready();
    {
      const unsigned char* b1 = unitB(s, 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) acc[0][0][mb][nb] = mfma16(fb0[nb][ks], fa0[mb][ks], acc[0][0][mb][nb]);
          if (mb & 1) fb1[mb >> 1][ks] = rdB(b1, mb >> 1, ks);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    stA(p1, 1);
    // ---- P2: q0 x b1 | read A1(s) | stage A0(s+2)
    phase_sync(more1, g.dbg);
    lds_ready();
    {
      const unsigned char* a1 = unitA(s, 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) acc[1][0][mb][nb] = mfma16(fb1[nb][ks], fa0[mb][ks], acc[1][0][mb][nb]);
          fa1[mb][ks] = rdA(a1, mb, ks);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    stA(p2, 0);
    // ---- P3: q1 x b0 | - | stage B0(s+2)
    phase_sync(more2, g.dbg);
    lds_ready();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[0][1][mb][nb] = mfma16(fb0[nb][ks], fa1[mb][ks], acc[0][1][mb][nb]);
    __builtin_amdgcn_s_setprio(0);
    stB(p2, 0);
    // ---- P4: q1 x b1 | read A0(s+1), B0(s+1) | stage B1(s+2)
    phase_sync(more2, g.dbg);
    lds_ready();
    {
      const unsigned char* a0 = unitA(s + 1, 0);
      const unsigned char* b0 = unitB(s + 1, 0);
      const bool rd = more1 && j + 1 < L;  // at an item's end: after its epilogue
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) acc[1][1][mb][nb] = mfma16(fb1[nb][ks], fa1[mb][ks], acc[1][1][mb][nb]);
          if (rd) {
            fa0[mb][ks] = rdA(a0, mb, ks);
            if (mb & 1) fb0[mb >> 1][ks] = rdB(b0, mb >> 1, ks);
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    stB(p2, 1);
    p1 = p2;
    advance(p2);

    after_epilogue = false;
    if (++j == L) {
      const Geom q = geom(item);
      epilogue<EPI>(g, acc, q.m0, q.n0, (q.kt0 / L), wm, wn, lane);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4q{};
      j = 0;
      ++item;
      after_epilogue = true;
      if (more1) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) fa0[mb][ks] = rdA(unitA(s + 1, 0), mb, ks);
#pragma unroll
          for (int nb = 0; nb < 2; ++nb) fb0[nb][ks] = rdB(unitB(s + 1, 0), nb, ks);
        }
      }
    }
  }
}

}  // namespace

void gemmq_launch(const GemmPParams& p, int splits, int n_cu, hipStream_t st) {
  GemmQArgs g{static_cast<const bf16*>(p.A), static_cast<const bf16*>(p.B), p.C, p.workspace,
              static_cast<const bf16*>(p.bias), static_cast<bf16*>(p.pre), static_cast<const bf16*>(p.aux), p.dbias,
              p.M, p.N, p.K, p.lda, p.ldb, p.ldc, p.alpha, p.beta, p.act, p.act_bwd ? 1 : 0, p.out_f32, splits,
              p.dbg};
  const int items = ((p.M + TM - 1) / TM) * ((p.N + TN - 1) / TN) * splits;
  dim3 grid(std::min(items, n_cu)), block(NTHREADS);
  const int epi = splits > 1 ? kEpiSplit : p.act_bwd ? kEpiDact : (p.bias || p.pre || p.act) ? kEpiBiasAct : kEpiPlain;
  auto launch = [&](auto ta, auto tb) {
    constexpr bool TA = decltype(ta)::value, TB = decltype(tb)::value;
    switch (epi) {
      case kEpiPlain: hipLaunchKernelGGL((gemmq_kernel<TA, TB, kEpiPlain>), grid, block, 0, st, g); break;
      case kEpiBiasAct: hipLaunchKernelGGL((gemmq_kernel<TA, TB, kEpiBiasAct>), grid, block, 0, st, g); break;
      case kEpiDact: hipLaunchKernelGGL((gemmq_kernel<TA, TB, kEpiDact>), grid, block, 0, st, g); break;
      default: hipLaunchKernelGGL((gemmq_kernel<TA, TB, kEpiSplit>), grid, block, 0, st, g); break;
    }
  };
  using F = std::false_type;
  using T = std::true_type;
  if (!p.trans_a && !p.trans_b) launch(F{}, F{});
  else if (!p.trans_a && p.trans_b) launch(F{}, T{});
  else if (p.trans_a && !p.trans_b) launch(T{}, F{});
  else launch(T{}, T{});
  FFK_LAUNCH_CHECK("gemmq");
}

}  // namespace ffk
