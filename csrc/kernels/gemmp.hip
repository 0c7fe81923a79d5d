// Phase-pipelined 256x256 bf16 MFMA GEMM for gfx950 (the production GEMM of
// the transformer path), with fused training epilogues.
//
//   C = epi(alpha * op(A) op(B))       epi = [+bias] [pre := .] [act | * act'(aux)]
//                                            [dbias += colsum] [+ beta * C]
//   split-K: fp32 partial slabs + splitk_reduce (gemm256.hip) for the long-K
//   weight gradients.
//
// Why a second 256^2 kernel: gemm256.hip retires every K-tile's LDS-DMA with
// vmcnt(0) + __syncthreads (a full pipeline drain per K step, ~830 TF on the
// BERT shapes vs hipBLASLt's 950-1370).  Here each K-tile is computed in FOUR
// phases, one per 64x32 quadrant of a wave's 128x64 output, and the operand
// tiles are staged in four 16 KiB UNITS laid out so that every unit is read
// in exactly one phase:
//
//   unit A0 = tile rows {0..63, 128..191}   (quadrant rows q = 0 of both wave rows)
//   unit A1 = tile rows {64..127, 192..255} (q = 1)
//   unit B0 = tile cols {wn*64 + 0..31}     (quadrant cols 0 of the 4 wave cols)
//   unit B1 = tile cols {wn*64 + 32..63}
//
//   phase  ds_read            LDS-DMA issued (2 x global_load_lds_dwordx4 / lane)   MFMA (8 x 32x32x16)
//   P1     A0, B0 (tile t)     B1 (t+1)                                              q0 x b0
//   P2     B1 (t)              A1 (t+1)                                              q0 x b1
//   P3     A1 (t)              A0 (t+2)                                              q1 x b0
//   P4     -                   B0 (t+2)                                              q1 x b1
//
// Two LDS buffers (tile parity) x 4 units = 128 KiB.  Every unit is restaged
// >= 2 phases after its last read (WAR: the reading wave's ds_reads retire
// before its MFMAs, which precede the next phase's barrier), and the counted
// s_waitcnt vmcnt(8) before each phase's barrier retires exactly the unit the
// NEXT phase reads (RAW) while four units (one whole K-tile) stay in flight
// across the barrier — the pipeline never drains inside the K loop (guide §5
// "Pipelining across barriers", T3/T4).  One raw s_barrier per phase; the
// tail (no more tiles to stage) waits vmcnt(0).  MFMA clusters sit between
// s_setprio(1)/(0) (T5).  Operand images: XOR-swizzled rows (mfma.h), swizzle
// applied to the per-lane GLOBAL source address because the DMA destination
// is lane-linear (rule 21); K-outer operands read with ds_read_b64_tr_b16.
// Bijective XCD remap + grouped raster (T1).
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

struct GemmPArgs {
  const bf16* A;
  const bf16* B;
  void* C;
  float* ws;          // split-K partials [S][M][N]
  const bf16* bias;   // [N]
  bf16* pre;          // pre-activation out (ldc)
  const bf16* aux;    // pre-activation in for the activation-gradient epilogue (ldc)
  float* dbias;       // column sums of the final value (fp32 atomics)
  int M, N, K, lda, ldb, ldc;
  float alpha, beta;
  int act, act_bwd, out_f32, splits;
  int dbg;  // ablation bits (timing experiments only; results are garbage): 1 no vm waits, 2 no barriers
};

__device__ __forceinline__ float act_fn(int act, float x) {
  switch (act) {
    case 1: return x > 0.f ? x : 0.f;
    case 2: return 1.f / (1.f + __expf(-x));
    case 3: return fast_tanh(x);
    case 4: return gelu_tanh(x);
    default: return x;
  }
}
__device__ __forceinline__ float act_grad_fn(int act, float x) {
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

// Tile-local outer index of image row / column o (0..127) of unit u.
template <bool IS_A>
__device__ __forceinline__ int unit_outer(int u, int o) {
  if (IS_A) return (o >> 6) * 128 + u * 64 + (o & 63);
  return (o >> 5) * 64 + u * 32 + (o & 31);
}

// Stage unit u of one operand (K-tile at k0) into `img` (16 KiB): 16 DMA
// instructions per unit, 2 per wave.
//  KOUTER: operand stored [K][outer]: image [64 k][128 outer], 256 B rows.
//  else:   operand stored [outer][K]: image [128 outer][64 k], 128 B rows.
template <bool IS_A, bool KOUTER>
__device__ __forceinline__ void stage_unit(const bf16* __restrict__ P, int ld, int outer0, int n_outer, int k0, int u,
                                           unsigned char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int j = wave * 2 + i;  // which KiB of the unit
    const bf16* src;
    if (KOUTER) {
      const int r = 4 * j + (lane >> 4);                 // k row
      const int c = swz_chunk<256>(r, lane & 15);        // logical 8-wide outer chunk stored in slot lane&15
      int col = outer0 + unit_outer<IS_A>(u, c * 8);
      col = min(col, n_outer - 8);                       // clamped columns only feed masked outputs
      src = P + static_cast<int64_t>(k0 + r) * ld + col;
    } else {
      const int r = 8 * j + (lane >> 3);                 // outer row
      const int c = swz_chunk<128>(r, lane & 7);
      const int row = min(outer0 + unit_outer<IS_A>(u, r), n_outer - 1);
      src = P + static_cast<int64_t>(row) * ld + k0 + c * 8;
    }
    __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)(img + j * 1024), 16, 0, 0);
  }
}

// Before a phase's MFMAs: retire this phase's LDS reads (the asm tr reads are
// not tracked by the compiler) and keep the MFMAs below the wait (rule 18).
__device__ __forceinline__ void lds_ready() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // no LDS access moves across the barrier
}

// Phase head: counted wait + barrier.  Unstaggered: vmcnt(8) leaves the 4
// most recent units (8 DMA instructions) in flight.  Staggered: vmcnt(6), 3
// units — the lagging wave group's wait retires a unit one phase later.
__device__ __forceinline__ void phase_sync(bool pipelined, int dbg = 0) {
  if (!(dbg & 1)) {
    if (!pipelined) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (dbg & 4) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  if (!(dbg & 2)) __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");  // no LDS access moves across the barrier
}

// Epilogue modes (compile-time, so each instantiation holds only the registers it needs)
enum Epi : int { kEpiPlain = 0, kEpiBiasAct = 1, kEpiDact = 2, kEpiSplit = 3 };

// Epilogue of one 256x256 tile: acc[qn][q][t] holds C^T (lane -> m, registers -> n).
//  plain:    C = alpha*acc + beta*C                       (bf16 or fp32 C)
//  bias_act: C = act(alpha*acc + bias) [pre := alpha*acc + bias]
//  dact:     C = alpha*acc * act'(aux) [dbias += colsum(C)]
//  split:    ws[split] = alpha*acc                        (fp32 partial slab)
template <int EPI>
__device__ __forceinline__ void epilogue(const GemmPArgs& g, f32x16 (&acc)[2][2][2], int m0, int n0, int split,
                                         int wm, int wn, int lane) {
  const int h = lane >> 5;
  bf16x4 bias[2][4];
  if (EPI == kEpiBiasAct) {
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int n = min(n0 + wn * 64 + qn * 32 + 8 * g4 + 4 * h, g.N - 4);
        bias[qn][g4] = g.bias ? *reinterpret_cast<const bf16x4*>(g.bias + n) : bf16x4{};
      }
  }
  float csum[2][4][4];  // [qn][g4][e] column partial sums (dbias)
  if (EPI == kEpiDact) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int c = 0; c < 4; ++c) csum[a][b][c] = 0.f;
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      // every load's value is consumed on every path (math is unconditional,
      // only the stores are masked): no load is left pending into the K loop,
      // where hipcc would otherwise drain vmcnt before reusing its registers
      const int m_raw = m0 + wm * 128 + q * 64 + t * 32 + (lane & 31);
      const bool mok = m_raw < g.M;
      const int m = mok ? m_raw : g.M - 1;
      // loads first (aux / old C for all 8 column groups of this row), then math + stores
      bf16x4 xa[2][4];
      f32x4 old[2][4];
      if (EPI == kEpiDact || (EPI == kEpiPlain && g.beta != 0.f)) {
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int n = min(n0 + wn * 64 + qn * 32 + 8 * g4 + 4 * h, g.N - 4);
            const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
            if (EPI == kEpiDact) {
              xa[qn][g4] = *reinterpret_cast<const bf16x4*>(g.aux + off);
            } else if (g.out_f32) {
              old[qn][g4] = *reinterpret_cast<const f32x4*>(static_cast<const float*>(g.C) + off);
            } else {
              const bf16x4 o = *reinterpret_cast<const bf16x4*>(static_cast<const bf16*>(g.C) + off);
              old[qn][g4] = f32x4{bf2f(o[0]), bf2f(o[1]), bf2f(o[2]), bf2f(o[3])};
            }
          }
      }
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int n_raw = n0 + wn * 64 + qn * 32 + 8 * g4 + 4 * h;
          const bool ok = mok && n_raw < g.N;  // N % 8 == 0: a 4-group is all-in or all-out
          const int n = ok ? n_raw : min(n_raw, g.N - 4);
          const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[qn][q][t][4 * g4 + e];
          if (EPI == kEpiSplit) {
            float* W = g.ws + (static_cast<int64_t>(split) * g.M + m) * g.N + n;
            if (ok) *reinterpret_cast<f32x4*>(W) = f32x4{v[0], v[1], v[2], v[3]};
            continue;
          }
          if (EPI == kEpiBiasAct) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += bf2f(bias[qn][g4][e]);
            if (g.pre && ok) {
              bf16x4 pv;
#pragma unroll
              for (int e = 0; e < 4; ++e) pv[e] = f2bf(v[e]);
              *reinterpret_cast<bf16x4*>(g.pre + off) = pv;
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = act_fn(g.act, v[e]);
          }
          if (EPI == kEpiDact) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= act_grad_fn(g.act, bf2f(xa[qn][g4][e]));
          }
          if (EPI == kEpiPlain && g.beta != 0.f) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += g.beta * old[qn][g4][e];
          }
          if (EPI == kEpiPlain && g.out_f32) {
            if (ok) *reinterpret_cast<f32x4*>(static_cast<float*>(g.C) + off) = f32x4{v[0], v[1], v[2], v[3]};
          } else {
            bf16x4 o;
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
            if (EPI == kEpiDact) {
#pragma unroll
              for (int e = 0; e < 4; ++e) csum[qn][g4][e] += ok ? bf2f(o[e]) : 0.f;  // the stored (rounded) value
            }
            if (ok) *reinterpret_cast<bf16x4*>(static_cast<bf16*>(g.C) + off) = o;
          }
        }
      }
    }
  }
  if (EPI == kEpiDact && g.dbias) {
    // reduce over the 32 rows of each lane half, then one atomic per column
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float sm = csum[qn][g4][e];
#pragma unroll
          for (int o = 16; o > 0; o >>= 1) sm += __shfl_xor(sm, o, 64);
          const int n = n0 + wn * 64 + qn * 32 + 8 * g4 + 4 * h + e;
          if ((lane & 31) == 0 && n < g.N) atomicAdd(g.dbias + n, sm);
        }
  }
}

struct Geom {
  int m0, n0, kt0;
};

template <bool TA, bool TB, int EPI>
__global__ __launch_bounds__(NTHREADS, 1) void gemmp_kernel(GemmPArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF];  // the ONE LDS object (guide §5 4a)
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // wave group = M half; on 4 SIMDs wave w and w + 4 share a SIMD, one of each group
  const int wm = wave >> 2, wn = wave & 3;
  const bool stagger = g.dbg & 4;

  // persistent: work item w (tile x K-split) = blockIdx.x + i * gridDim.x
  const int gm = (g.M + TM - 1) / TM, gn = (g.N + TN - 1) / TN;
  const int nwg = gm * gn;
  const int L = g.K / TK / g.splits;  // K-tiles per item (host: splits | K/64)
  const int W = nwg * g.splits;
  const int G = gridDim.x;
  const int n_items = (W - static_cast<int>(blockIdx.x) + G - 1) / G;
  const int S = n_items * L;  // this block's K-tile stream

  auto geom = [&](int i) {
    const int w = blockIdx.x + i * G;
    const int bid = xcd_remap(w, W);  // contiguous logical items per XCD in every round
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
  // stream-position geometry, advanced incrementally (the full tile mapping,
  // with its scalar divisions, runs once per work item, not per phase)
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
  auto rdA = [&](const unsigned char* img, int t, int ks) -> bf16x8 {
    return TA ? tr_frag_nat_asm<256>(img, ks * 16, wm * 64 + t * 32, lane)
              : row_frag<128>(img, wm * 64 + t * 32, ks * 16, lane);
  };
  auto rdB = [&](const unsigned char* img, int ks) -> bf16x8 {
    return TB ? row_frag<128>(img, wn * 32, ks * 16, lane) : tr_frag_nat_asm<256>(img, ks * 16, wn * 32, lane);
  };

  f32x16 acc[2][2][2];  // [qn][q][t]: 32x32 C^T tiles (lane -> m, registers -> n)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[a][b][c] = f32x16{};
  bf16x8 fa0[2][4], fa1[2][4], fb0[4], fb1[4];  // fragments [t][kstep] / [kstep]

  // prologue: the steady-state issue order up to stream position 1, then the
  // first fragments (A0(0), B0(0): "phase P4 of position -1")
  Pos p1{0, 0, 0, geom(0)};  // becomes s + 1
  stA(p1, 0);
  stB(p1, 0);
  stB(p1, 1);
  stA(p1, 1);
  advance(p1);
  stA(p1, 0);
  stB(p1, 0);
  stB(p1, 1);
  Pos p2 = p1;  // s + 2
  advance(p2);
  phase_sync(S >= 2);
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
    for (int t = 0; t < 2; ++t) fa0[t][ks] = rdA(unitA(0, 0), t, ks);
    fb0[ks] = rdB(unitB(0, 0), ks);
  }
  // Staggered schedule (guide §5 8-phase template): a second barrier after
  // every MFMA cluster and group 1 one barrier behind, so one group's MFMAs
  // run while the other group issues its DMA and waits — the two waves of a
  // SIMD take turns on the matrix pipe.
  if (stagger && wm == 1) bar();

  bool after_epilogue = false;
  for (int s = 0, j = 0, item = 0; s < S; ++s) {
    const bool more1 = s + 1 < S, more2 = s + 2 < S;
    // ---- P1: q0 x b0 | read B1(s) | stage A1(s+1)
    phase_sync(more1 && !after_epilogue, g.dbg);  // the epilogue's stores share the vm counter
    lds_ready();
    {
      const unsigned char* b1 = unitB(s, 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[0][0][t] = mfma32(fb0[ks], fa0[t][ks], acc[0][0][t]);
        fb1[ks] = rdB(b1, ks);
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (stagger) bar();
    stA(p1, 1);
    // ---- P2: q0 x b1 | read A1(s) | stage A0(s+2)
    phase_sync(more1, g.dbg);
    lds_ready();
    {
      const unsigned char* a1 = unitA(s, 1);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          acc[1][0][t] = mfma32(fb1[ks], fa0[t][ks], acc[1][0][t]);
          fa1[t][ks] = rdA(a1, t, ks);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (stagger) bar();
    stA(p2, 0);
    // ---- P3: q1 x b0 | - | stage B0(s+2)
    phase_sync(more2, g.dbg);
    lds_ready();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[0][1][t] = mfma32(fb0[ks], fa1[t][ks], acc[0][1][t]);
    __builtin_amdgcn_s_setprio(0);
    if (stagger) bar();
    stB(p2, 0);
    // ---- P4: q1 x b1 | read A0(s+1), B0(s+1) | stage B1(s+2)
    phase_sync(more2, g.dbg);
    lds_ready();
    {
      const unsigned char* a0 = unitA(s + 1, 0);
      const unsigned char* b0 = unitB(s + 1, 0);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
        for (int t = 0; t < 2; ++t) acc[1][1][t] = mfma32(fb1[ks], fa1[t][ks], acc[1][1][t]);
        if (more1 && j + 1 < L) {  // at an item's end: after its epilogue (no fragments live across it)
#pragma unroll
          for (int t = 0; t < 2; ++t) fa0[t][ks] = rdA(a0, t, ks);
          fb0[ks] = rdB(b0, ks);
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    if (stagger) bar();
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
          for (int c = 0; c < 2; ++c) acc[a][b][c] = f32x16{};
      j = 0;
      ++item;
      after_epilogue = true;
      if (more1) {
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
          for (int t = 0; t < 2; ++t) fa0[t][ks] = rdA(unitA(s + 1, 0), t, ks);
          fb0[ks] = rdB(unitB(s + 1, 0), ks);
        }
      }
    }
  }
  if (stagger && wm == 0) bar();  // equal barrier counts in both groups
}

}  // namespace

bool gemmp_supported(int M, int N, int K, int lda, int ldb, bool trans_a, bool trans_b) {
  if (M < 8 || N < 8 || K < TK || K % TK) return false;
  if (M % 8 || N % 8 || lda % 8 || ldb % 8) return false;
  (void)trans_a;
  (void)trans_b;
  return true;
}

void gemmp_bf16(const GemmPParams& p, hipStream_t st) {
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return;
  if (!gemmp_supported(p.M, p.N, p.K, p.lda, p.ldb, p.trans_a, p.trans_b))
    throw std::invalid_argument("gemmp: needs K % 64 == 0, M/N/lda/ldb multiples of 8");
  if ((reinterpret_cast<uintptr_t>(p.A) | reinterpret_cast<uintptr_t>(p.B)) & 15)
    throw std::invalid_argument("gemmp: operands must be 16-byte aligned");
  if (p.ldc % 4 || (reinterpret_cast<uintptr_t>(p.C) & (p.out_f32 ? 15 : 7)))
    throw std::invalid_argument("gemmp: C alignment (16 B fp32 / 8 B bf16) and ldc % 4");
  if ((p.pre && (reinterpret_cast<uintptr_t>(p.pre) & 7)) || (p.aux && (reinterpret_cast<uintptr_t>(p.aux) & 7)) ||
      (p.bias && (reinterpret_cast<uintptr_t>(p.bias) & 7)))
    throw std::invalid_argument("gemmp: bias / pre / aux must be 8-byte aligned");
  if (p.act_bwd && (!p.aux || !p.act))
    throw std::invalid_argument("gemmp: the activation-gradient epilogue needs aux and an activation");
  const int nk = p.K / TK;
  int splits = std::max(1, std::min(p.splits, nk));
  // gemmr / gemmt address their operands with 32-bit buffer offsets
  const uint64_t a_bytes = uint64_t(p.trans_a ? p.K : p.M) * uint64_t(p.lda) * 2u;
  const uint64_t b_bytes = uint64_t(p.trans_b ? p.N : p.K) * uint64_t(p.ldb) * 2u;
  const bool small = a_bytes < (1ull << 32) && b_bytes < (1ull << 32);
  // the non-persistent gemmt spreads the remainder K-tiles over the first
  // splits (QKV dW: 48 tiles x 5 splits = 240 workgroups); every other
  // kernel streams the same number of K-tiles per work item
  const bool uneven = ((p.variant == 3 || p.variant == 4 || p.variant == 6 || p.variant == 10) && small &&
                       gemmt_supported(p)) ||
                      p.variant == 8;
  if (!uneven)
    while (nk % splits) --splits;
  if (splits > 1) {
    if (p.bias || p.pre || p.act || p.dbias)
      throw std::invalid_argument("gemmp: split-K has no bias / activation / dbias epilogue");
    if (!p.workspace || (reinterpret_cast<uintptr_t>(p.workspace) & 15))
      throw std::invalid_argument("gemmp: split-K needs a 16-byte aligned fp32 workspace of splits*M*N");
  }
  GemmPArgs g{static_cast<const bf16*>(p.A), static_cast<const bf16*>(p.B), p.C, p.workspace,
              static_cast<const bf16*>(p.bias), static_cast<bf16*>(p.pre), static_cast<const bf16*>(p.aux), p.dbias,
              p.M, p.N, p.K, p.lda, p.ldb, p.ldc, p.alpha, p.beta, p.act, p.act_bwd ? 1 : 0, p.out_f32, splits,
              p.dbg};
  static const int n_cu = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return std::max(8, n);
  }();
  if (p.variant == 11 && splits == 1 && gemmpp_supported(p)) {
    gemmpp_launch(p, st);
    return;
  }
  if (p.variant == 9 && splits == 1 && gemmn_supported(p)) {
    gemmn_launch(p, st);
    return;
  }
  if (p.variant == 8) {
    gemms_launch(p, splits, st);
    if (splits > 1) splitk_reduce(p.workspace, p.C, p.M, p.N, p.ldc, splits, p.beta, p.out_f32, st);
    return;
  }
  // 9 / 11 (eight-wave A B^T kernels) fall back to gemmt for other layouts / epilogues
  if ((p.variant >= 1 && p.variant <= 6) || p.variant == 9 || p.variant == 10 || p.variant == 11) {
    if (p.variant == 2 && small) gemmr_launch(p, splits, n_cu, st);
    else if (p.variant >= 3 && small && gemmt_supported(p)) {
      if (p.variant >= 11) {   // the eight-wave kernels' dbg is their mode, not gemmt's ablation bits
        GemmPParams q = p;
        q.dbg = 0;
        gemmt_launch(q, splits, p.variant - 3, st);
      } else {
        gemmt_launch(p, splits, p.variant - 3, st);
      }
    }
    else gemmq_launch(p, splits, n_cu, st);
    if (splits > 1) splitk_reduce(p.workspace, p.C, p.M, p.N, p.ldc, splits, p.beta, p.out_f32, st);
    return;
  }
  const int items = ((p.M + TM - 1) / TM) * ((p.N + TN - 1) / TN) * splits;
  dim3 grid(std::min(items, n_cu)), block(NTHREADS);  // persistent: one workgroup per CU
  const int epi = splits > 1 ? kEpiSplit : p.act_bwd ? kEpiDact : (p.bias || p.pre || p.act) ? kEpiBiasAct : kEpiPlain;
  if (epi == kEpiBiasAct && p.beta != 0.f) throw std::invalid_argument("gemmp: bias / activation epilogue has no beta");
  if (epi == kEpiDact && (p.beta != 0.f || p.out_f32 || p.bias || p.pre))
    throw std::invalid_argument("gemmp: the activation-gradient epilogue writes bf16, no beta / bias / pre");
  if (p.dbias && epi != kEpiDact) throw std::invalid_argument("gemmp: dbias needs the activation-gradient epilogue");
  if (epi == kEpiBiasAct && p.out_f32) throw std::invalid_argument("gemmp: bias / activation epilogue writes bf16");
  auto launch = [&](auto ta, auto tb) {
    constexpr bool TA = decltype(ta)::value, TB = decltype(tb)::value;
    switch (epi) {
      case kEpiPlain: hipLaunchKernelGGL((gemmp_kernel<TA, TB, kEpiPlain>), grid, block, 0, st, g); break;
      case kEpiBiasAct: hipLaunchKernelGGL((gemmp_kernel<TA, TB, kEpiBiasAct>), grid, block, 0, st, g); break;
      case kEpiDact: hipLaunchKernelGGL((gemmp_kernel<TA, TB, kEpiDact>), grid, block, 0, st, g); break;
      default: hipLaunchKernelGGL((gemmp_kernel<TA, TB, kEpiSplit>), grid, block, 0, st, g); break;
    }
  };
  using F = std::false_type;
  using T = std::true_type;
  if (!p.trans_a && !p.trans_b) launch(F{}, F{});
  else if (!p.trans_a && p.trans_b) launch(F{}, T{});
  else if (p.trans_a && !p.trans_b) launch(T{}, F{});
  else launch(T{}, T{});
  FFK_LAUNCH_CHECK("gemmp");
  if (splits > 1) splitk_reduce(p.workspace, p.C, p.M, p.N, p.ldc, splits, p.beta, p.out_f32, st);
}

}  // namespace ffk
