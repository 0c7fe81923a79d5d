// Ping-pong phase GEMM on v_mfma_f32_16x16x32_bf16 (GemmPParams.variant = 2).
//
// Tile 256 x 256 x 64, 8 waves as 2 (M) x 4 (N), a 128 x 64 output per wave,
// the operand tiles staged by LDS-DMA in four 16 KiB units per K-tile (A0 =
// tile rows {0..63, 128..191}, A1 = rows {64..127, 192..255}, B0 / B1 = the
// left / right 32 columns of every wave's 64) — the same units, images and
// swizzles as gemmq.hip.  What differs is the schedule:
//
//  * Each phase is split into a LOAD segment (this phase's fragment reads +
//    one unit of LDS-DMA) and a COMPUTE segment (16 MFMAs, one 64 x 32
//    quadrant x K 64), each closed by a barrier.  Wave group 1 (waves 4-7)
//    runs one barrier behind group 0, and waves w and w + 4 share a SIMD, so
//    each SIMD alternates one wave's MFMAs with its partner's loads: the DMA
//    issue and the LDS reads hide behind the partner's matrix work instead
//    of idling the matrix pipe at every phase boundary (guide §5 8-phase
//    template, MI355X_MICROARCH.md 'Two waves per SIMD').
//  * The fragment reads of a phase are for that phase's MFMAs, ordered so
//    that every phase reads one unit: P1 A0(s), P2 B1(s), P3 A1(s), P4
//    B0(s+1) — a single unit stream ... B0(s) A0(s) B1(s) A1(s) B0(s+1) ...
//    read one unit per phase, 8 / 4 / 8 / 4 ds_read_b128 (balanced).
//  * The DMA runs D = 6 units ahead of the reads in the same stream (8 LDS
//    slots: 2 K-tile buffers x 4 units).  RAW: the unit read in group 0's
//    load segment of phase k must be retired by every wave before the
//    barrier that opens it; group 0 waits for it just before that barrier,
//    group 1 (one barrier behind) before its previous compute barrier, both
//    with vmcnt(2 (D - 1)) in the steady state.  WAR: a slot is refilled 6
//    phases after the unit it held was read, i.e. after both groups retired
//    those reads (lgkmcnt(0) before their compute barriers).
//  * DMA through buffer_load ... lds with per-lane voffsets computed once per
//    output tile and the K advance in the scalar soffset: no address VALU in
//    the K loop.
//
// Epilogues as gemmp.hip / gemmq.hip (C^T accumulators: a lane owns 4
// consecutive n of one row).
#include <type_traits>

#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int TM = 256, TN = 256, TK = 64, NTHREADS = 512;
constexpr int UNIT = 16 * 1024;
constexpr int BUF = 4 * UNIT;
constexpr int GROUP = 4;
constexpr int DIST = 6;  // DMA distance (units = phases); WAR needs DIST <= 7
typedef float f32x4r __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_void_ptr;

struct GemmRArgs {
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
};

__device__ __forceinline__ float r_act(int act, float x) {
  switch (act) {
    case 1: return x > 0.f ? x : 0.f;
    case 2: return 1.f / (1.f + __expf(-x));
    case 3: return fast_tanh(x);
    case 4: return gelu_tanh(x);
    default: return x;
  }
}
__device__ __forceinline__ float r_act_grad(int act, float x) {
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

__device__ __forceinline__ int r_slot128(int r, int c) { return c ^ ((r >> 1) & 7); }

__device__ __forceinline__ f32x4r mfma16(bf16x8 a, bf16x8 b, f32x4r c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <bool IS_A>
__device__ __forceinline__ int unit_outer(int u, int o) {
  if (IS_A) return (o >> 6) * 128 + u * 64 + (o & 63);
  return (o >> 5) * 64 + u * 32 + (o & 31);
}

// Byte voffset of this lane's 16-B DMA piece i (0, 1) of unit u for a tile
// whose outer origin is outer0 (K-tile 0; the K advance goes in soffset).
template <bool IS_A, bool KOUTER>
__device__ __forceinline__ unsigned dma_voff(int ld, int outer0, int n_outer, int u, int i, int wave, int lane) {
  const int j = wave * 2 + i;
  if (KOUTER) {
    const int r = 4 * j + (lane >> 4);
    const int c = swz_chunk<256>(r, lane & 15);
    const int col = min(outer0 + unit_outer<IS_A>(u, c * 8), n_outer - 8);
    return (static_cast<unsigned>(r) * static_cast<unsigned>(ld) + static_cast<unsigned>(col)) * 2u;
  }
  const int r = 8 * j + (lane >> 3);
  const int c = r_slot128(r, lane & 7);
  const int row = min(outer0 + unit_outer<IS_A>(u, r), n_outer - 1);
  return (static_cast<unsigned>(row) * static_cast<unsigned>(ld) + static_cast<unsigned>(c * 8)) * 2u;
}

__device__ __forceinline__ bf16x8 row16(const unsigned char* img, int o0, int ks, int lane) {
  const int r = o0 + (lane & 15);
  return lds_read16(img, r * 128 + (r_slot128(r, ks * 4 + (lane >> 4)) << 4));
}
__device__ __forceinline__ bf16x8 tr16(const unsigned char* img, int ks, int o0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const int col = o0 + 4 * (i & 3);
  const int r = ks * 32 + 8 * g + (i >> 2);
  const int oa = img_off<256>(r, col >> 3) + (col & 7) * 2;
  const int ob = img_off<256>(r + 4, col >> 3) + (col & 7) * 2;
  return cat44(lds_tr_asm(img, oa), lds_tr_asm(img, ob));
}

__device__ __forceinline__ void bar() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// s_waitcnt vmcnt(2 n) for a run-time n in [0, DIST - 1] (wave-uniform)
__device__ __forceinline__ void wait_units(int n) {
  switch (n) {
    case 5: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}
static_assert(DIST - 1 <= 5, "wait_units covers up to DIST - 1 = 5 units in flight");

enum Epi : int { kEpiPlain = 0, kEpiBiasAct = 1, kEpiDact = 2, kEpiSplit = 3 };

template <int EPI>
__device__ __forceinline__ void epilogue(const GemmRArgs& g, f32x4r (&acc)[2][2][4][2], int m0, int n0, int split,
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
      f32x4r old[2][2];
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
              old[qn][nb] = *reinterpret_cast<const f32x4r*>(static_cast<const float*>(g.C) + off);
            } else {
              const bf16x4 o = *reinterpret_cast<const bf16x4*>(static_cast<const bf16*>(g.C) + off);
              old[qn][nb] = f32x4r{bf2f(o[0]), bf2f(o[1]), bf2f(o[2]), bf2f(o[3])};
            }
          }
      }
#pragma unroll
      for (int qn = 0; qn < 2; ++qn) {
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const int n_raw = n0 + wn * 64 + qn * 32 + nb * 16 + nl;
          const bool ok = mok && n_raw < g.N;
          const int n = ok ? n_raw : min(n_raw, g.N - 4);
          const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
          float v[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[qn][qm][mb][nb][e];
          if (EPI == kEpiSplit) {
            float* Wp = g.ws + (static_cast<int64_t>(split) * g.M + m) * g.N + n;
            if (ok) *reinterpret_cast<f32x4r*>(Wp) = f32x4r{v[0], v[1], v[2], v[3]};
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
            for (int e = 0; e < 4; ++e) v[e] = r_act(g.act, v[e]);
          }
          if (EPI == kEpiDact) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] *= r_act_grad(g.act, bf2f(xa[qn][nb][e]));
          }
          if (EPI == kEpiPlain && g.beta != 0.f) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += g.beta * old[qn][nb][e];
          }
          if (EPI == kEpiPlain && g.out_f32) {
            if (ok) *reinterpret_cast<f32x4r*>(static_cast<float*>(g.C) + off) = f32x4r{v[0], v[1], v[2], v[3]};
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
__global__ __launch_bounds__(NTHREADS, 1) void gemmr_kernel(GemmRArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF];  // the ONE LDS object
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const bool grp1 = wm == 1;  // wave-uniform: runs one barrier behind group 0

  const int gm = (g.M + TM - 1) / TM, gn = (g.N + TN - 1) / TN;
  const int nwg = gm * gn;
  const int L = g.K / TK / g.splits;
  const int W = nwg * g.splits;
  const int G = gridDim.x;
  const int n_items = (W - static_cast<int>(blockIdx.x) + G - 1) / G;
  const int S = n_items * L;     // K-tiles in this block's stream
  const int last = 4 * S - 2;    // last unit of the read stream (B0 of tile S does not exist)

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

  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.A), static_cast<short>(0), g.bytesA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.B), static_cast<short>(0), g.bytesB, 0x00020000);
  const unsigned kstepA = TA ? static_cast<unsigned>(TK * g.lda * 2) : TK * 2u;   // soffset per K-tile
  const unsigned kstepB = !TB ? static_cast<unsigned>(TK * g.ldb * 2) : TK * 2u;

  // ---- DMA side: the stream position of the next unit to stage
  unsigned voA[2][2], voB[2][2];  // [unit][piece] per-lane byte voffsets of the DMA tile
  int d_item = 0, d_j = -1, d_s = -1;  // item, K-tile within it, global stream tile of the last B0 issued
  unsigned d_kA = 0, d_kB = 0;         // soffsets of the DMA K-tile
  auto set_dma_geom = [&](int item) {
    const Geom q = geom(item);
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        voA[u][i] = dma_voff<true, TA>(g.lda, q.m0, g.M, u, i, wave, lane);
        voB[u][i] = dma_voff<false, !TB>(g.ldb, q.n0, g.N, u, i, wave, lane);
      }
    d_kA = q.kt0 * kstepA;
    d_kB = q.kt0 * kstepB;
  };
  // stage the next unit of the stream; T = unit type (0 B0, 1 A0, 2 B1, 3 A1)
  auto dma = [&](auto tc) {
    constexpr int T = decltype(tc)::value;
    if (T == 0) {  // first unit of a K-tile: advance the DMA tile
      ++d_s;
      if (++d_j == L) {
        d_j = 0;
        ++d_item;
        set_dma_geom(d_item);
      } else if (d_s > 0) {
        d_kA += kstepA;
        d_kB += kstepB;
      }
    }
    constexpr bool IS_A = T & 1;
    constexpr int u = T >> 1;
    unsigned char* img = smem + (d_s & 1) * BUF + (IS_A ? u * UNIT : (2 + u) * UNIT) + wave * 2048;
    // soffset provably wave-uniform (guide T20: otherwise hipcc wraps each
    // buffer op in a readfirstlane waterfall loop)
    const unsigned koff = __builtin_amdgcn_readfirstlane(IS_A ? d_kA : d_kB);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (IS_A)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rA, (lds_void_ptr)(img + i * 1024), 16, voA[u][i], koff, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rB, (lds_void_ptr)(img + i * 1024), 16, voB[u][i], koff, 0, 0);
    }
  };

  auto rdA = [&](const unsigned char* img, int mb, int ks) -> bf16x8 {
    return TA ? tr16(img, ks, wm * 64 + mb * 16, lane) : row16(img, wm * 64 + mb * 16, ks, lane);
  };
  auto rdB = [&](const unsigned char* img, int nb, int ks) -> bf16x8 {
    return TB ? row16(img, wn * 32 + nb * 16, ks, lane) : tr16(img, ks, wn * 32 + nb * 16, lane);
  };

  f32x4r acc[2][2][4][2];  // [qn][qm][mb][nb]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4r{};
  bf16x8 fa0[4][2], fa1[4][2], fb0[2][2], fb1[2][2];  // [block][kstep]

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // ---- prologue: stage units -1 .. DIST-2 (B0 A0 B1 A1 of tile 0, B0 A0 of tile 1)
  set_dma_geom(0);
  dma(I0{});
  if (last >= 0) dma(I1{});
  if (last >= 1) dma(I2{});
  if (last >= 2) dma(I3{});
  if (last >= 3) dma(I0{});
  if (last >= 4) dma(I1{});
  // units in flight after the reads of unit k are retired (k read in L(k)):
  // group 0 waits before the barrier opening L(k), having issued through
  // unit k - 1 + DIST; group 1 before the barrier opening C(k - 1), having
  // issued through the same unit.
  // An epilogue's stores also count in vmcnt and are younger than every DMA
  // issued before them, so after one the same counts only wait longer (safe).
  auto n_after = [&](int k) { return min(k - 1 + DIST, last) - k; };
  auto wait_for = [&](int k) { wait_units(n_after(k)); };

  // phase -1: read B0(0)
  if (grp1) {
    wait_for(-1);
    bar();   // group 1 runs one barrier behind from here on
  } else {
    wait_for(-1);
  }
  bar();
  if (last >= 5) dma(I2{});  // unit DIST - 1 = B1 of tile 1
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) fb0[nb][ks] = rdB(smem + 2 * UNIT, nb, ks);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (grp1) wait_for(0);
  bar();   // (empty compute segment of phase -1)

  int c_item = 0, c_j = 0;
  for (int s = 0; s < S; ++s) {
    const int k0 = 4 * s;
    unsigned char* cur = smem + (s & 1) * BUF;
    unsigned char* nxt = smem + ((s + 1) & 1) * BUF;
    // ================= P1: L reads A0(s), stages unit k+6 (A1 of s+1); C q0 x b0
    if (!grp1) wait_for(k0);
    bar();
    if (k0 + DIST <= last) dma(I3{});
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) fa0[mb][ks] = rdA(cur, mb, ks);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (grp1) wait_for(k0 + 1);
    bar();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[0][0][mb][nb] = mfma16(fb0[nb][ks], fa0[mb][ks], acc[0][0][mb][nb]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    // ================= P2: L reads B1(s), stages B0 of s+2; C q0 x b1
    if (!grp1) wait_for(k0 + 1);
    bar();
    if (k0 + 1 + DIST <= last) dma(I0{});
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nb = 0; nb < 2; ++nb) fb1[nb][ks] = rdB(cur + 3 * UNIT, nb, ks);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (grp1) wait_for(k0 + 2);
    bar();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[1][0][mb][nb] = mfma16(fb1[nb][ks], fa0[mb][ks], acc[1][0][mb][nb]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    // ================= P3: L reads A1(s), stages A0 of s+2; C q1 x b0
    if (!grp1) wait_for(k0 + 2);
    bar();
    if (k0 + 2 + DIST <= last) dma(I1{});
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) fa1[mb][ks] = rdA(cur + UNIT, mb, ks);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (grp1) wait_for(k0 + 3);
    bar();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[0][1][mb][nb] = mfma16(fb0[nb][ks], fa1[mb][ks], acc[0][1][mb][nb]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    // ================= P4: L reads B0(s+1), stages B1 of s+2; C q1 x b1
    if (!grp1) wait_for(k0 + 3);
    bar();
    if (k0 + 3 + DIST <= last) dma(I2{});
    if (k0 + 3 <= last) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) fb0[nb][ks] = rdB(nxt + 2 * UNIT, nb, ks);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (grp1) wait_for(k0 + 4);
    bar();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mb = 0; mb < 4; ++mb)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) acc[1][1][mb][nb] = mfma16(fb1[nb][ks], fa1[mb][ks], acc[1][1][mb][nb]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (++c_j == L) {
      const Geom q = geom(c_item);
      epilogue<EPI>(g, acc, q.m0, q.n0, q.kt0 / L, wm, wn, lane);
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int d = 0; d < 2; ++d) acc[a][b][c][d] = f32x4r{};
      c_j = 0;
      ++c_item;
    }
  }
  if (!grp1) bar();  // equal barrier counts in both groups
}

}  // namespace

void gemmr_launch(const GemmPParams& p, int splits, int n_cu, hipStream_t st) {
  auto bytes = [](int rows, int ld) {
    const uint64_t b = static_cast<uint64_t>(rows) * static_cast<uint64_t>(ld) * 2u;
    return static_cast<unsigned>(b > 0xFFFFFFFFull ? 0xFFFFFFFFull : b);
  };
  const int a_rows = p.trans_a ? p.K : p.M;
  const int b_rows = p.trans_b ? p.N : p.K;
  GemmRArgs g{static_cast<const bf16*>(p.A), static_cast<const bf16*>(p.B), p.C, p.workspace,
              static_cast<const bf16*>(p.bias), static_cast<bf16*>(p.pre), static_cast<const bf16*>(p.aux), p.dbias,
              p.M, p.N, p.K, p.lda, p.ldb, p.ldc, p.alpha, p.beta, p.act, p.act_bwd ? 1 : 0, p.out_f32, splits,
              bytes(a_rows, p.lda), bytes(b_rows, p.ldb)};
  const int items = ((p.M + TM - 1) / TM) * ((p.N + TN - 1) / TN) * splits;
  dim3 grid(std::min(items, n_cu)), block(NTHREADS);
  const int epi = splits > 1 ? kEpiSplit : p.act_bwd ? kEpiDact : (p.bias || p.pre || p.act) ? kEpiBiasAct : kEpiPlain;
  auto launch = [&](auto ta, auto tb) {
    constexpr bool TA = decltype(ta)::value, TB = decltype(tb)::value;
    switch (epi) {
      case kEpiPlain: hipLaunchKernelGGL((gemmr_kernel<TA, TB, kEpiPlain>), grid, block, 0, st, g); break;
      case kEpiBiasAct: hipLaunchKernelGGL((gemmr_kernel<TA, TB, kEpiBiasAct>), grid, block, 0, st, g); break;
      case kEpiDact: hipLaunchKernelGGL((gemmr_kernel<TA, TB, kEpiDact>), grid, block, 0, st, g); break;
      default: hipLaunchKernelGGL((gemmr_kernel<TA, TB, kEpiSplit>), grid, block, 0, st, g); break;
    }
  };
  using F = std::false_type;
  using T = std::true_type;
  if (!p.trans_a && !p.trans_b) launch(F{}, F{});
  else if (!p.trans_a && p.trans_b) launch(F{}, T{});
  else if (p.trans_a && !p.trans_b) launch(T{}, F{});
  else launch(T{}, T{});
  FFK_LAUNCH_CHECK("gemmr");
}

}  // namespace ffk
