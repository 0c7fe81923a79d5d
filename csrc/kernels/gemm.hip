// bf16 MFMA GEMM with fused epilogues for gfx950.
//
//   C[m][n] = act(alpha * sum_k Aop[m][k] * Bop[k][n] + bias[n]) + beta * C[m][n]
//   Aop = A (row-major [M][K], lda) or A^T (A stored [K][M]) ; same for B.
//   Optional: store the pre-activation (bf16) for the activation backward;
//             fp32 output (weight gradients straight into the flat fp32
//             gradient buffer, beta = 1 accumulates micro-batches).
//
// Parity: lib/kernels/src/cuda/ops/linear_kernels.cu (cublasGemmEx forward
// :131, bias GEMM :152, activation :173/:185; dW :231, db :280, dX :303) and
// batch_matmul_kernels.cu — there one library call per step plus separate
// activation / bias launches; here one launch per product with the epilogue
// fused.
//
// CDNA4 structure (cdna_hip_programming.md §5): 128x128x64 block tile, 4
// waves as 2x2, each wave 64x64 = 2x2 tiles of v_mfma_f32_32x32x16_bf16
// (16 MFMAs per wave per K-step); register-staged double-buffered LDS with the
// next tile's loads issued before the MFMAs and written after them (one
// barrier per K-step); both operand layouts are served from one row-copied LDS
// image by ds_read_b128 (k-contiguous rows) or ds_read_b64_tr_b16 (transposed)
// with swizzles that are conflict-free for both (mfma.h); the product is
// computed as C^T so a lane owns 4 consecutive output columns per register
// group (8/16-byte stores); bijective XCD remap + grouped tile order for L2
// reuse (T1).
#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int IMG_BYTES = BM * BK * 2;  // 16 KiB per operand image
constexpr int GROUP_M = 8;

struct GemmArgs {
  const bf16* A;
  const bf16* B;
  void* C;
  const bf16* bias;
  bf16* pre;
  int M, N, K, lda, ldb, ldc;
  float alpha, beta;
  int act;
  int out_f32;
  float* ws;   // split-K: fp32 partial slabs [splits][M][N] (epilogue applied by splitk_epi_kernel)
  int splits;
};

__device__ __forceinline__ float apply_act(int act, float x) {
  switch (act) {
    case 1: return x > 0.f ? x : 0.f;
    case 2: return 1.f / (1.f + __expf(-x));
    case 3: return fast_tanh(x);
    case 4: return gelu_tanh(x);
    default: return x;
  }
}

// Stage one operand tile (global -> 4 x 16-byte registers per thread).
// ROWS x ROWB image; the global row r of the tile is `rowptr(r)`.
template <bool K_CONTIG>
struct Stager {
  bf16x8 reg[4];
  // K_CONTIG: image rows = the 128 "outer" indices (m or n), 8 chunks of k.
  //          else: image rows = the 64 k indices, 16 chunks of m or n.
  __device__ __forceinline__ void load(const bf16* P, int ld, int outer0, int n_outer, int k0, int K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = threadIdx.x + 256 * i;
      int r, ch;
      bool ok;
      const bf16* src;
      if (K_CONTIG) {
        r = c >> 3;
        ch = c & 7;
        ok = (outer0 + r < n_outer) && (k0 + ch * 8 < K);
        src = P + static_cast<int64_t>(outer0 + r) * ld + k0 + ch * 8;
      } else {
        r = c >> 4;
        ch = c & 15;
        ok = (k0 + r < K) && (outer0 + ch * 8 < n_outer);
        src = P + static_cast<int64_t>(k0 + r) * ld + outer0 + ch * 8;
      }
      reg[i] = ok ? *reinterpret_cast<const bf16x8*>(src) : bf16x8{};
    }
  }
  __device__ __forceinline__ void store(unsigned char* img) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = threadIdx.x + 256 * i;
      if (K_CONTIG) *reinterpret_cast<bf16x8*>(img + img_off<128>(c >> 3, c & 7)) = reg[i];
      else *reinterpret_cast<bf16x8*>(img + img_off<256>(c >> 4, c & 15)) = reg[i];
    }
  }
};

template <bool TA, bool TB>
__global__ __launch_bounds__(256, 2) void gemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[4 * IMG_BYTES];  // A0 B0 A1 B1
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  // ---- tile order: XCD remap, then GROUP_M-grouped raster
  const int gm = (g.M + BM - 1) / BM, gn = (g.N + BN - 1) / BN;
  const int nwg = gm * gn;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_group = GROUP_M * gn;
  const int first_m = (bid / per_group) * GROUP_M;
  const int gsize = min(gm - first_m, GROUP_M);
  const int tm = first_m + (bid % per_group) % gsize;
  const int tn = (bid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  Stager<!TA> sa;  // A: k-contiguous unless transposed
  Stager<TB> sb;   // B: k-contiguous only when transposed ([N][K])

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  // split-K: split blockIdx.y takes an (uneven) contiguous range of K-tiles
  const int nk_all = (g.K + BK - 1) / BK;
  const int sbase = nk_all / g.splits, srem = nk_all % g.splits, sp = blockIdx.y;
  const int kt0 = sp * sbase + min(sp, srem);
  const int nk = kt0 + sbase + (sp < srem ? 1 : 0);
  sa.load(g.A, g.lda, m0, g.M, kt0 * BK, g.K);
  sb.load(g.B, g.ldb, n0, g.N, kt0 * BK, g.K);
  sa.store(smem);
  sb.store(smem + IMG_BYTES);
  __syncthreads();

  for (int kt = kt0; kt < nk; ++kt) {
    const unsigned char* Ai = smem + ((kt - kt0) & 1) * 2 * IMG_BYTES;
    const unsigned char* Bi = Ai + IMG_BYTES;
    const bool has_next = kt + 1 < nk;
    if (has_next) {
      sa.load(g.A, g.lda, m0, g.M, (kt + 1) * BK, g.K);
      sb.load(g.B, g.ldb, n0, g.N, (kt + 1) * BK, g.K);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 bf[2], af[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (TB) bf[t] = row_frag<128>(Bi, wn * 64 + t * 32, ks * 16, lane);
        else bf[t] = tr_frag_nat<256>(Bi, ks * 16, wn * 64 + t * 32, lane);
        if (!TA) af[t] = row_frag<128>(Ai, wm * 64 + t * 32, ks * 16, lane);
        else af[t] = tr_frag_nat<256>(Ai, ks * 16, wm * 64 + t * 32, lane);
      }
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[nt][mt] = mfma32(bf[nt], af[mt], acc[nt][mt]);
    }
    if (has_next) {
      unsigned char* nxt = smem + ((kt + 1 - kt0) & 1) * 2 * IMG_BYTES;
      sa.store(nxt);
      sb.store(nxt + IMG_BYTES);
    }
    __syncthreads();
  }

  // ---- epilogue: acc[nt][mt] holds C^T; lane = m, registers = n
  const int h = lane >> 5;
  if (g.splits > 1) {  // raw alpha * partial into this split's slab (N % 4 == 0, host-checked)
    float* slab = g.ws + static_cast<int64_t>(sp) * g.M * g.N;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = m0 + wm * 64 + mt * 32 + (lane & 31);
      if (m >= g.M) continue;
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int n = n0 + wn * 64 + nt * 32 + 8 * g4 + 4 * h;
          if (n >= g.N) continue;
          f32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = g.alpha * acc[nt][mt][4 * g4 + e];
          *reinterpret_cast<f32x4*>(slab + static_cast<int64_t>(m) * g.N + n) = o;
        }
    }
    return;
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int m = m0 + wm * 64 + mt * 32 + (lane & 31);
    if (m >= g.M) continue;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int n = n0 + wn * 64 + nt * 32 + 8 * g4 + 4 * h;
        if (n >= g.N) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[nt][mt][4 * g4 + e];
        const bool full = n + 3 < g.N;
        if (g.bias) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (full || n + e < g.N) v[e] += bf2f(g.bias[n + e]);
        }
        const int64_t off = static_cast<int64_t>(m) * g.ldc + n;
        if (g.pre) {
          if (full) {
            bf16x4 pv;
#pragma unroll
            for (int e = 0; e < 4; ++e) pv[e] = f2bf(v[e]);
            *reinterpret_cast<bf16x4*>(g.pre + off) = pv;
          } else {
            for (int e = 0; e < 4 && n + e < g.N; ++e) g.pre[off + e] = f2bf(v[e]);
          }
        }
        if (g.act) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = apply_act(g.act, v[e]);
        }
        if (g.out_f32) {
          float* C = static_cast<float*>(g.C) + off;
          if (full) {
            f32x4 o;
            if (g.beta != 0.f) o = *reinterpret_cast<f32x4*>(C);
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = v[e] + (g.beta != 0.f ? g.beta * o[e] : 0.f);
            *reinterpret_cast<f32x4*>(C) = o;
          } else {
            for (int e = 0; e < 4 && n + e < g.N; ++e) C[e] = v[e] + (g.beta != 0.f ? g.beta * C[e] : 0.f);
          }
        } else {
          bf16* C = static_cast<bf16*>(g.C) + off;
          if (full) {
            bf16x4 o;
            if (g.beta != 0.f) {
              bf16x4 old = *reinterpret_cast<bf16x4*>(C);
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] += g.beta * bf2f(old[e]);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
            *reinterpret_cast<bf16x4*>(C) = o;
          } else {
            for (int e = 0; e < 4 && n + e < g.N; ++e)
              C[e] = f2bf(v[e] + (g.beta != 0.f ? g.beta * bf2f(C[e]) : 0.f));
          }
        }
      }
    }
  }
}

// Split-K finish with the full gemm epilogue: v = sum_s ws[s] + bias;
// pre := v; v = act(v); C = v + beta * C.  Four columns per thread.
__global__ __launch_bounds__(256) void splitk_epi_kernel(GemmArgs g) {
  const int64_t n4 = static_cast<int64_t>(g.M) * g.N / 4;
  const int64_t slab = static_cast<int64_t>(g.M) * g.N;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t e0 = i * 4;
    const int m = static_cast<int>(e0 / g.N), n = static_cast<int>(e0 % g.N);
    f32x4 v = *reinterpret_cast<const f32x4*>(g.ws + e0);
    for (int z = 1; z < g.splits; ++z) {
      const f32x4 t = *reinterpret_cast<const f32x4*>(g.ws + z * slab + e0);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += t[e];
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
      for (int e = 0; e < 4; ++e) v[e] = apply_act(g.act, v[e]);
    }
    if (g.out_f32) {
      float* C = static_cast<float*>(g.C) + off;
      f32x4 o;
      if (g.beta != 0.f) o = *reinterpret_cast<f32x4*>(C);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = v[e] + (g.beta != 0.f ? g.beta * o[e] : 0.f);
      *reinterpret_cast<f32x4*>(C) = o;
    } else {
      bf16* C = static_cast<bf16*>(g.C) + off;
      if (g.beta != 0.f) {
        const bf16x4 old = *reinterpret_cast<bf16x4*>(C);
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

}  // namespace

void gemm_bf16_ex(const void* A, const void* B, void* C, const void* bias, void* pre, int M, int N, int K, int lda,
                  int ldb, int ldc, bool trans_a, bool trans_b, int act, float alpha, float beta, int out_f32,
                  hipStream_t st, int splits, float* ws) {
  if (M <= 0 || N <= 0 || K <= 0) return;
  splits = std::max(1, std::min(splits, (K + BK - 1) / BK));
  // the split-K epilogue stores 4 columns per thread: f32x4 (16 B) into an
  // fp32 C, bf16x4 (8 B) into a bf16 C and into the pre-activation; an
  // output view that is not aligned for that runs the single-pass kernel
  if (splits > 1 && (((reinterpret_cast<uintptr_t>(C) & (out_f32 ? 15 : 7)) != 0) ||
                     (pre && (reinterpret_cast<uintptr_t>(pre) & 7) != 0)))
    splits = 1;
  if (splits > 1 && (!ws || N % 4 || ldc % 4 || (reinterpret_cast<uintptr_t>(ws) & 15)))
    throw std::invalid_argument("gemm: split-K needs a 16-byte aligned fp32 workspace and N % 4 == 0");
  // 16-byte global loads require 8-element aligned leading dims and
  // contiguous extents (checked here, on the host, before any launch).
  if (lda % 8 || ldb % 8) throw std::invalid_argument("gemm: lda/ldb must be multiples of 8");
  if (!trans_a && K % 8) throw std::invalid_argument("gemm: K must be a multiple of 8");
  if (trans_a && M % 8) throw std::invalid_argument("gemm: M must be a multiple of 8 when A is transposed");
  if (!trans_b && N % 8) throw std::invalid_argument("gemm: N must be a multiple of 8 when B is [K][N]");
  if (trans_b && K % 8) throw std::invalid_argument("gemm: K must be a multiple of 8");
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15)
    throw std::invalid_argument("gemm: operands must be 16-byte aligned");
  if (ldc % 4 || (reinterpret_cast<uintptr_t>(C) & 7)) throw std::invalid_argument("gemm: C must be 8-byte aligned, ldc%4==0");
  GemmArgs g{static_cast<const bf16*>(A), static_cast<const bf16*>(B), C, static_cast<const bf16*>(bias),
             static_cast<bf16*>(pre), M, N, K, lda, ldb, ldc, alpha, beta, act, out_f32, ws, splits};
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  dim3 grid(nwg, splits), block(256);
  if (!trans_a && !trans_b) hipLaunchKernelGGL((gemm_kernel<false, false>), grid, block, 0, st, g);
  else if (!trans_a && trans_b) hipLaunchKernelGGL((gemm_kernel<false, true>), grid, block, 0, st, g);
  else if (trans_a && !trans_b) hipLaunchKernelGGL((gemm_kernel<true, false>), grid, block, 0, st, g);
  else hipLaunchKernelGGL((gemm_kernel<true, true>), grid, block, 0, st, g);
  FFK_LAUNCH_CHECK("gemm_bf16");
  if (splits > 1) {
    const int64_t n4 = static_cast<int64_t>(M) * N / 4;
    const int rgrid = static_cast<int>(std::min<int64_t>((n4 + 255) / 256, 2048));
    hipLaunchKernelGGL(splitk_epi_kernel, dim3(rgrid), dim3(256), 0, st, g);
    FFK_LAUNCH_CHECK("gemm_bf16 split-K epilogue");
  }
}

void gemm_bf16(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda, int ldb,
               int ldc, bool trans_a, bool trans_b, int act, float alpha, float beta, int out_f32, hipStream_t st) {
  gemm_bf16_ex(A, B, C, bias, nullptr, M, N, K, lda, ldb, ldc, trans_a, trans_b, act, alpha, beta, out_f32, st);
}

}  // namespace ffk
