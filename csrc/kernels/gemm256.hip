// 256x256-tile bf16 MFMA GEMM with LDS-DMA staging and split-K, gfx950.
//
//   C = act(alpha * op(A) op(B) + bias) + beta * C       (split-K: partial
//   fp32 slabs + a reduce pass; used for the long-K weight gradients
//   dW = X^T dY, K = tokens, whose few output tiles cannot fill 256 CUs).
//
// Structure (cdna_hip_programming.md §5 "glds, 2 LDS buffers, BK=64"):
//  * block = 8 waves (2 along M x 4 along N), 256x256 output, each wave
//    128x64 = 4x2 v_mfma_f32_32x32x16_bf16 tiles (32 MFMAs per K-step);
//  * operands staged HBM/L2 -> LDS by global_load_lds_dwordx4 (no VGPR
//    round trip, 1 KiB per wave instruction), two buffers: the next K-tile's
//    DMA is in flight while the current one feeds the MFMAs;
//  * the LDS image is lane-linear (DMA destination = base + 16*lane), so the
//    bank-conflict swizzle is applied to the per-lane GLOBAL source address
//    and undone by the same XOR on the fragment read (rule 21);
//  * each 256-wide operand image is two 128-wide sub-images so the existing
//    128 B / 256 B row swizzles (mfma.h) serve both K-inner (ds_read_b128) and
//    K-outer (ds_read_b64_tr_b16) operands;
//  * C^T formulation as in gemm.hip: a lane owns one output row and 4
//    consecutive columns per register group (16-byte fp32 / 8-byte bf16 stores);
//  * bijective XCD remap + grouped raster for L2 reuse; split index in
//    blockIdx.y.
#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int TM = 256, TN = 256, TK = 64, NTHREADS = 512;
constexpr int SUB = 128 * TK * 2;  // 16 KiB sub-image
constexpr int IMG = 2 * SUB;       // 32 KiB operand image
constexpr int GROUP = 4;
typedef __attribute__((address_space(3))) void* lds_void_ptr;

struct Gemm256Args {
  const bf16* A;
  const bf16* B;
  void* C;
  float* ws;  // split-K partials [S][M][N] (S > 1)
  const bf16* bias;
  bf16* pre;
  int M, N, K, lda, ldb, ldc;
  float alpha, beta;
  int act, out_f32, splits;
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

// One operand tile (256 outer x 64 k) -> LDS image by 4 DMA instructions per wave.
//  KOUTER: operand stored [K][outer] (row = k); sub-image [64 k][128 outer], 256 B rows.
//  else:   operand stored [outer][K] (row = outer); sub-image [128 outer][64 k], 128 B rows.
template <bool KOUTER>
__device__ __forceinline__ void stage(const bf16* __restrict__ P, int ld, int outer0, int n_outer, int k0,
                                      unsigned char* img, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = wave * 4 + i;  // 0..31: which KiB of the image
    const int sub = q >> 4, j = q & 15;
    const bf16* src;
    if (KOUTER) {
      const int r = 4 * j + (lane >> 4);                // k row within the tile
      const int c = swz_chunk<256>(r, lane & 15);       // logical 8-element chunk stored at slot lane&15
      int col = outer0 + sub * 128 + c * 8;
      col = min(col, n_outer - 8);                      // out-of-range columns only feed masked outputs
      src = P + static_cast<int64_t>(k0 + r) * ld + col;
    } else {
      const int r = 8 * j + (lane >> 3);
      const int c = swz_chunk<128>(r, lane & 7);
      const int row = min(outer0 + sub * 128 + r, n_outer - 1);
      src = P + static_cast<int64_t>(row) * ld + k0 + c * 8;
    }
    __builtin_amdgcn_global_load_lds(src, (lds_void_ptr)(img + sub * SUB + j * 1024), 16, 0, 0);
  }
}

template <bool TA, bool TB>
__global__ __launch_bounds__(NTHREADS, 1) void gemm256_kernel(Gemm256Args g) {
  // ONE shared array (a second __shared__ object can de-pipeline the DMA
  // waits, guide §5 item 4a): [buf][A img | B img]
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * 2 * IMG];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave & 1, wn = wave >> 1;

  const int gm = (g.M + TM - 1) / TM, gn = (g.N + TN - 1) / TN;
  const int nwg = gm * gn;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_group = GROUP * gn;
  const int first_m = (bid / per_group) * GROUP;
  const int gsize = min(gm - first_m, GROUP);
  const int tm = first_m + (bid % per_group) % gsize;
  const int tn = (bid % per_group) / gsize;
  const int m0 = tm * TM, n0 = tn * TN;

  const int nk = g.K / TK;
  const int split = blockIdx.y;
  const int kb = static_cast<int>((static_cast<int64_t>(nk) * split) / g.splits);
  const int ke = static_cast<int>((static_cast<int64_t>(nk) * (split + 1)) / g.splits);

  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};

  if (kb < ke) {
    stage<TA>(g.A, g.lda, m0, g.M, kb * TK, smem, wave, lane);
    stage<!TB>(g.B, g.ldb, n0, g.N, kb * TK, smem + IMG, wave, lane);
  }
  __syncthreads();

  for (int kt = kb; kt < ke; ++kt) {
    const int buf = (kt - kb) & 1;
    const unsigned char* Ai = smem + buf * 2 * IMG;
    const unsigned char* Bi = Ai + IMG;
    if (kt + 1 < ke) {  // next tile's DMA overlaps this tile's MFMAs
      unsigned char* nxt = smem + (buf ^ 1) * 2 * IMG;
      stage<TA>(g.A, g.lda, m0, g.M, (kt + 1) * TK, nxt, wave, lane);
      stage<!TB>(g.B, g.ldb, n0, g.N, (kt + 1) * TK, nxt + IMG, wave, lane);
    }
    const unsigned char* Asub = Ai + wm * SUB;          // this wave's 128 rows of M
    const unsigned char* Bsub = Bi + (wn >> 1) * SUB;   // its 64 columns of N live in one 128-wide sub-image
    const int nb = (wn & 1) * 64;
#pragma unroll
    for (int ks = 0; ks < TK / 16; ++ks) {
      bf16x8 bf[2], af[4];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (TB) bf[t] = row_frag<128>(Bsub, nb + t * 32, ks * 16, lane);
        else bf[t] = tr_frag_nat<256>(Bsub, ks * 16, nb + t * 32, lane);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (!TA) af[t] = row_frag<128>(Asub, t * 32, ks * 16, lane);
        else af[t] = tr_frag_nat<256>(Asub, ks * 16, t * 32, lane);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[nt][mt] = mfma32(bf[nt], af[mt], acc[nt][mt]);
    }
    __syncthreads();  // drains this wave's DMA (vmcnt(0)) and orders it for every reader
  }

  // ---- epilogue: acc[nt][mt] = C^T tile; lane -> m, registers -> n
  const int h = lane >> 5;
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
    const int m = m0 + wm * 128 + mt * 32 + (lane & 31);
    if (m >= g.M) continue;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int n = n0 + wn * 64 + nt * 32 + 8 * g4 + 4 * h;
        if (n >= g.N) continue;  // N % 8 == 0 (host check): a 4-group is all-in or all-out
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[nt][mt][4 * g4 + e];
        if (g.splits > 1) {
          float* W = g.ws + (static_cast<int64_t>(split) * g.M + m) * g.N + n;
          *reinterpret_cast<f32x4*>(W) = f32x4{v[0], v[1], v[2], v[3]};
          continue;
        }
        if (g.bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bf2f(g.bias[n + e]);
        }
        const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
        if (g.pre) {
          bf16x4 pv;
#pragma unroll
          for (int e = 0; e < 4; ++e) pv[e] = f2bf(v[e]);
          *reinterpret_cast<bf16x4*>(g.pre + off) = pv;
        }
        if (g.act) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = act_fn(g.act, v[e]);
        }
        if (g.out_f32) {
          float* C = static_cast<float*>(g.C) + off;
          f32x4 o = f32x4{};
          if (g.beta != 0.f) o = *reinterpret_cast<f32x4*>(C);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = v[e] + g.beta * o[e];
          *reinterpret_cast<f32x4*>(C) = o;
        } else {
          bf16* C = static_cast<bf16*>(g.C) + off;
          if (g.beta != 0.f) {
            bf16x4 old = *reinterpret_cast<bf16x4*>(C);
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
}

// out[m][n] = sum_s ws[s][m][n] + beta * out[m][n]   (4 columns per thread)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, void* out, int M, int N,
                                                            int ldc, int S, float beta, int out_f32) {
  const int64_t n4 = static_cast<int64_t>(M) * N / 4;
  const int64_t slab = static_cast<int64_t>(M) * N;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t e0 = i * 4;
    const int m = static_cast<int>(e0 / N), n = static_cast<int>(e0 % N);
    f32x4 s = reinterpret_cast<const f32x4*>(ws + e0)[0];
    for (int z = 1; z < S; ++z) {
      const f32x4 t = reinterpret_cast<const f32x4*>(ws + z * slab + e0)[0];
#pragma unroll
      for (int e = 0; e < 4; ++e) s[e] += t[e];
    }
    const int64_t off = static_cast<int64_t>(m) * ldc + n;
    if (out_f32) {
      float* C = static_cast<float*>(out) + off;
      if (beta != 0.f) {
        const f32x4 o = *reinterpret_cast<f32x4*>(C);
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += beta * o[e];
      }
      *reinterpret_cast<f32x4*>(C) = s;
    } else {
      bf16* C = static_cast<bf16*>(out) + off;
      if (beta != 0.f) {
        const bf16x4 o = *reinterpret_cast<bf16x4*>(C);
#pragma unroll
        for (int e = 0; e < 4; ++e) s[e] += beta * bf2f(o[e]);
      }
      bf16x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = f2bf(s[e]);
      *reinterpret_cast<bf16x4*>(C) = r;
    }
  }
}

}  // namespace

void splitk_reduce(const float* ws, void* out, int M, int N, int ldc, int S, float beta, int out_f32,
                   hipStream_t st) {
  const int64_t n4 = static_cast<int64_t>(M) * N / 4;
  const int rgrid = static_cast<int>(std::min<int64_t>((n4 + 255) / 256, 2048));
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(rgrid), dim3(256), 0, st, ws, out, M, N, ldc, S, beta, out_f32);
  FFK_LAUNCH_CHECK("splitk_reduce");
}

bool gemm256_supported(int M, int N, int K, int lda, int ldb, bool trans_a, bool trans_b) {
  if (M < 8 || N < 8 || K < TK || K % TK) return false;
  if (M % 8 || N % 8 || lda % 8 || ldb % 8) return false;
  (void)trans_a;
  (void)trans_b;
  return true;
}

void gemm256_bf16(const void* A, const void* B, void* C, const void* bias, void* pre, int M, int N, int K, int lda,
                  int ldb, int ldc, bool trans_a, bool trans_b, int act, float alpha, float beta, int out_f32,
                  int splits, float* workspace, hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0) return;
  if (!gemm256_supported(M, N, K, lda, ldb, trans_a, trans_b))
    throw std::invalid_argument("gemm256: needs K % 64 == 0, M/N/lda/ldb multiples of 8");
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15)
    throw std::invalid_argument("gemm256: operands must be 16-byte aligned");
  if (ldc % 4 || (reinterpret_cast<uintptr_t>(C) & (out_f32 ? 15 : 7)))
    throw std::invalid_argument("gemm256: C alignment (16 B fp32 / 8 B bf16) and ldc % 4");
  splits = std::max(1, std::min(splits, K / TK));
  if (splits > 1) {
    if (bias || pre || act) throw std::invalid_argument("gemm256: split-K has no bias/activation epilogue");
    if (!workspace || (reinterpret_cast<uintptr_t>(workspace) & 15))
      throw std::invalid_argument("gemm256: split-K needs a 16-byte aligned fp32 workspace of splits*M*N");
  }
  Gemm256Args g{static_cast<const bf16*>(A), static_cast<const bf16*>(B), C, workspace,
                static_cast<const bf16*>(bias), static_cast<bf16*>(pre), M, N, K, lda, ldb, ldc, alpha, beta,
                act, out_f32, splits};
  const int nwg = ((M + TM - 1) / TM) * ((N + TN - 1) / TN);
  dim3 grid(nwg, splits), block(NTHREADS);
  if (!trans_a && !trans_b) hipLaunchKernelGGL((gemm256_kernel<false, false>), grid, block, 0, st, g);
  else if (!trans_a && trans_b) hipLaunchKernelGGL((gemm256_kernel<false, true>), grid, block, 0, st, g);
  else if (trans_a && !trans_b) hipLaunchKernelGGL((gemm256_kernel<true, false>), grid, block, 0, st, g);
  else hipLaunchKernelGGL((gemm256_kernel<true, true>), grid, block, 0, st, g);
  FFK_LAUNCH_CHECK("gemm256");
  if (splits > 1) splitk_reduce(workspace, C, M, N, ldc, splits, beta, out_f32, st);
}

}  // namespace ffk
