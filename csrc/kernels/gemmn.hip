// Eight-wave multistage bf16 GEMM for the NT layout (GemmPParams.variant = 9).
//
// C[M][N] (+)= A[M][K] B[N][K]^T with both operands K-contiguous: the
// input-gradient products dX = dY W^T of every Linear (and the vocabulary
// head's), the signatures hipBLASLt still won in round 3
// (profiles/autotune_report_bert_b64_r3.txt).
//
//   * 256 x 256 output tile per workgroup of 8 waves (2 x 4); a wave owns a
//     128 x 64 sub-tile = 8 x 4 blocks of v_mfma_f32_16x16x32_bf16 (128
//     accumulator registers), two waves per SIMD;
//   * K-tiles of 32 in a four-stage LDS ring (4 x 32 KiB): every operand
//     stage is 16 subtiles of 16 rows x 32 k (1 KiB) with the st_16x32
//     swizzle (byte bit 5 ^= bit 9: the 16 lanes of a ds_read_b128 group hit
//     eight distinct 16-B slots), filled by LDS-DMA (buffer_load ... lds, one
//     1-KiB subtile per wave instruction, rows past the operand read zeros);
//   * one barrier per K-tile: wait for this tile's DMA with a COUNTED vmcnt
//     (the two younger tiles stay in flight), barrier, issue the DMA of tile
//     t + 3 into the stage tile t - 1 used (every wave is past its reads),
//     then 32 MFMAs per wave;
//   * C^T accumulators (mfma(B, A)): a lane holds 4 consecutive n of one m;
//     epilogue: plain bf16 / fp32, beta accumulate.
// Bijective XCD remap + grouped raster (cdna_hip_programming.md T1).
#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int NM = 256, NN = 256, NK = 32, NTH = 512, NSTAGE = 4;
constexpr int NSUB = 1024;                 // one 16 x 32 subtile
constexpr int NOP = 16 * NSUB;             // one operand stage (256 rows x 32 k)
constexpr int NSTG = 2 * NOP;              // A + B
constexpr int NGROUP = 8;
typedef float nf32x4 __attribute__((ext_vector_type(4)));

struct GemmNArgs {
  const bf16* A;
  const bf16* B;
  void* C;
  int M, N, K, lda, ldb, ldc;
  float alpha, beta;
  int out_f32;
  unsigned bytesA, bytesB;
};

__device__ __forceinline__ void dma16n(__amdgpu_buffer_rsrc_t r, unsigned char* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// the logical 16-B chunk a DMA lane stores into physical slot `lane` of a
// subtile (the swizzle is an involution)
__device__ __forceinline__ int n_chunk(int lane) { return lane ^ (((lane >> 5) & 1) << 1); }

// byte offset of lane's operand fragment (row lane & 15, k group lane >> 4)
// inside a subtile
__device__ __forceinline__ int n_frag_off(int lane) {
  const int r = lane & 15, byte = r * 64 + (lane >> 4) * 16;
  return byte ^ (((r >> 3) & 1) << 5);
}

__device__ __forceinline__ nf32x4 mfma16n(bf16x8 a, bf16x8 b, nf32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int EPI>  // 0: plain bf16 (alpha), 1: general (beta and / or fp32 out)
__global__ __launch_bounds__(NTH, 1) void gemmn_kernel(GemmNArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[NSTAGE * NSTG];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;

  const int gm = (g.M + NM - 1) / NM, gn = (g.N + NN - 1) / NN;
  const int nwg = gm * gn;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_group = NGROUP * gn;
  const int first_m = (bid / per_group) * NGROUP;
  const int gsize = min(gm - first_m, NGROUP);
  const int m0 = (first_m + (bid % per_group) % gsize) * NM;
  const int n0 = ((bid % per_group) / gsize) * NN;

  const __amdgpu_buffer_rsrc_t rA =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.A), static_cast<short>(0), g.bytesA, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(g.B), static_cast<short>(0), g.bytesB, 0x00020000);
  // wave w fills subtiles 2w and 2w + 1 of each operand stage: rows
  // 32 w + 16 j + (chunk >> 2), k chunk (chunk & 3)
  const int ch = n_chunk(lane);
  unsigned voA[2], voB[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = 32 * wave + 16 * j + (ch >> 2);
    voA[j] = (static_cast<unsigned>(m0 + row) * static_cast<unsigned>(g.lda) + static_cast<unsigned>((ch & 3) * 8)) * 2u;
    voB[j] = (static_cast<unsigned>(n0 + row) * static_cast<unsigned>(g.ldb) + static_cast<unsigned>((ch & 3) * 8)) * 2u;
  }
  auto issue = [&](int kt) {
    unsigned char* st = smem + (kt % NSTAGE) * NSTG;
    const unsigned ks = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(kt) * NK * 2u);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      dma16n(rA, st + (2 * wave + j) * NSUB, voA[j], ks);
      dma16n(rB, st + NOP + (2 * wave + j) * NSUB, voB[j], ks);
    }
  };

  nf32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = nf32x4{};
  const int fo = n_frag_off(lane);

  const int T = g.K / NK;
  issue(0);
  if (T > 1) issue(1);
  if (T > 2) issue(2);
  for (int t = 0; t < T; ++t) {
    // this wave's DMA of tile t landed; tiles t + 1, t + 2 may stay in flight
    const int younger = min(2, T - 1 - t);
    if (younger == 2) vm_wait<8>();
    else if (younger == 1) vm_wait<4>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();   // every wave's DMA of tile t landed; every wave is past tile t - 1
    asm volatile("" ::: "memory");
    if (t + 3 < T) issue(t + 3);    // into tile t - 1's stage
    const unsigned char* st = smem + (t % NSTAGE) * NSTG;
    // all 12 fragment reads first (the compiler's counted lgkmcnt waits then
    // release each MFMA group as soon as its A fragment has landed)
    bf16x8 fb[4], fa[8];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) fb[nb] = lds_read16(st + NOP + (wc * 4 + nb) * NSUB, fo);
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) fa[mb] = lds_read16(st + (wr * 8 + mb) * NSUB, fo);
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[mb][nb] = mfma16n(fb[nb], fa[mb], acc[mb][nb]);
  }

  // ---- epilogue: acc[mb][nb] -> row m0 + 128 wr + 16 mb + (lane & 15),
  // columns n0 + 64 wc + 16 nb + 4 (lane >> 4) + e
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int m = m0 + wr * 128 + mb * 16 + (lane & 15);
    if (m >= g.M) continue;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      const int n = n0 + wc * 64 + nb * 16 + 4 * (lane >> 4);
      if (n >= g.N) continue;   // N % 8 == 0 (host-checked): a 4-group is all in or all out
      const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[mb][nb][e];
      if (g.out_f32) {
        float* C = static_cast<float*>(g.C) + off;
        nf32x4 o = nf32x4{v[0], v[1], v[2], v[3]};
        if (EPI == 1 && g.beta != 0.f) {
          const nf32x4 old = *reinterpret_cast<const nf32x4*>(C);
          o += g.beta * old;
        }
        *reinterpret_cast<nf32x4*>(C) = o;
      } else {
        bf16* C = static_cast<bf16*>(g.C) + off;
        if (EPI == 1 && g.beta != 0.f) {
          const bf16x4 old = *reinterpret_cast<const bf16x4*>(C);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += g.beta * bf2f(old[e]);
        }
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
        *reinterpret_cast<bf16x4*>(C) = o;
      }
    }
  }
}

}  // namespace

bool gemmn_supported(const GemmPParams& p) {
  if (p.trans_a || !p.trans_b || p.bias || p.pre || p.act || p.act_bwd || p.dbias) return false;
  if (p.K % NK || p.N % 8 || p.lda % 8 || p.ldb % 8 || p.ldc % 4) return false;
  const uint64_t a = uint64_t(p.M) * uint64_t(p.lda) * 2u, b = uint64_t(p.N) * uint64_t(p.ldb) * 2u;
  return a < (1ull << 32) && b < (1ull << 32);
}

void gemmn_launch(const GemmPParams& p, hipStream_t st) {
  if (!gemmn_supported(p)) throw std::invalid_argument("gemmn: NT layout, plain epilogue, K % 32, N % 8");
  GemmNArgs g{static_cast<const bf16*>(p.A), static_cast<const bf16*>(p.B), p.C, p.M, p.N, p.K, p.lda, p.ldb, p.ldc,
              p.alpha, p.beta, p.out_f32,
              static_cast<unsigned>(uint64_t(p.M) * uint64_t(p.lda) * 2u),
              static_cast<unsigned>(uint64_t(p.N) * uint64_t(p.ldb) * 2u)};
  const int nwg = ((p.M + NM - 1) / NM) * ((p.N + NN - 1) / NN);
  if (p.beta != 0.f || p.out_f32) hipLaunchKernelGGL((gemmn_kernel<1>), dim3(nwg), dim3(NTH), 0, st, g);
  else hipLaunchKernelGGL((gemmn_kernel<0>), dim3(nwg), dim3(NTH), 0, st, g);
  FFK_LAUNCH_CHECK("gemmn");
}

}  // namespace ffk
