// Small-tile bf16 MFMA GEMM for MLP-sized products (GemmPParams.variant = 8).
//
// DLRM's MLPs multiply [1024, 512..1024] activations by [512..1024]^2 weights:
// a 256x256-tile kernel puts 16 workgroups on 256 CUs, and the library's
// 64x64 kernels (the Cijk_* MT64x64x64 of profiles/dlrm_kernels_r3.txt) run
// the bias and the activation in separate passes.  Here:
//   * 64 x 64 output tile per workgroup of 4 waves (2 x 2), each wave one
//     32 x 32 v_mfma_f32_32x32x16_bf16 accumulator (C^T: lane = m, registers =
//     4 consecutive n per group, as gemm.hip) -> a 1024 x 1024 output is 256
//     workgroups, one per CU; 32 KB of LDS lets four share a CU;
//   * K-tiles of 64, both operand images 128-byte rows (mfma.h swizzle: row
//     reads and transposed reads conflict free), register-staged double buffer,
//     one barrier per K-tile;
//   * the epilogues fused: bias + activation (+ pre-activation store), and the
//     activation gradient of the producer (result * act'(aux)) with the bias
//     gradient's column sums (wave shuffle reduction, one fp32 atomic per
//     column per wave half), plain alpha / beta (bf16 or fp32 out) and split-K
//     fp32 slabs (reduced by gemmp.hip's splitk_reduce).
// Bijective XCD remap + grouped raster as gemm.hip.
#include <type_traits>

#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int SM = 64, SN = 64, SK = 64, SNT = 256;
constexpr int SIMG = SM * SK * 2;  // 8 KiB per operand image
constexpr int SGROUP = 8;

enum SEpi : int { sPlain = 0, sBiasAct = 1, sDact = 2, sSplit = 3 };

struct GemmSArgs {
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
  int out_f32, splits;
  int64_t sA = 0, sB = 0, sC = 0;   // batched: element strides between the blockIdx.z products
};

template <int ACT>
__device__ __forceinline__ float s_act(float x) {
  if (ACT == 1) return x > 0.f ? x : 0.f;
  if (ACT == 2) return 1.f / (1.f + __expf(-x));
  if (ACT == 3) return fast_tanh(x);
  if (ACT == 4) return gelu_tanh(x);
  return x;
}
template <int ACT>
__device__ __forceinline__ float s_act_grad(float x) {
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

// Two 16-byte chunks per thread per operand tile.  K-contiguous operand:
// image row = the outer index (m or n), chunk = 8 k; K-outer operand: image
// row = k, chunk = 8 outer.  Both images: 64 rows x 128 B.
template <bool KC>
struct SStager {
  bf16x8 reg[2];
  __device__ __forceinline__ void load(const bf16* P, int ld, int outer0, int n_outer, int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = threadIdx.x + SNT * i;
      const int r = c >> 3, ch = c & 7;
      bool ok;
      const bf16* src;
      if (KC) {
        ok = outer0 + r < n_outer;
        src = P + static_cast<int64_t>(outer0 + r) * ld + k0 + ch * 8;
      } else {
        ok = outer0 + ch * 8 < n_outer;
        src = P + static_cast<int64_t>(k0 + r) * ld + outer0 + ch * 8;
      }
      reg[i] = ok ? *reinterpret_cast<const bf16x8*>(src) : bf16x8{};
    }
  }
  __device__ __forceinline__ void store(unsigned char* img) const {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = threadIdx.x + SNT * i;
      *reinterpret_cast<bf16x8*>(img + img_off<128>(c >> 3, c & 7)) = reg[i];
    }
  }
};

template <bool TA, bool TB, int EPI, int ACT>
__global__ __launch_bounds__(SNT) void gemms_kernel(GemmSArgs g) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[4 * SIMG];  // A0 B0 A1 B1
  if (blockIdx.z) {  // batched product z (plain epilogue)
    g.A += blockIdx.z * g.sA;
    g.B += blockIdx.z * g.sB;
    g.C = static_cast<void*>(static_cast<char*>(g.C) + blockIdx.z * g.sC * (g.out_f32 ? 4 : 2));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  const int gm = (g.M + SM - 1) / SM, gn = (g.N + SN - 1) / SN;
  const int nwg = gm * gn;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_group = SGROUP * gn;
  const int first_m = (bid / per_group) * SGROUP;
  const int gsize = min(gm - first_m, SGROUP);
  const int m0 = (first_m + (bid % per_group) % gsize) * SM;
  const int n0 = ((bid % per_group) / gsize) * SN;

  // split-K: split blockIdx.y takes a contiguous (uneven) range of K-tiles
  const int nk_all = g.K / SK;
  const int sb = nk_all / g.splits, sr = nk_all % g.splits, sp = blockIdx.y;
  const int kt0 = sp * sb + min(sp, sr);
  const int kt1 = kt0 + sb + (sp < sr ? 1 : 0);

  SStager<!TA> sa;
  SStager<TB> sbs;
  f32x16 acc = f32x16{};
  sa.load(g.A, g.lda, m0, g.M, kt0 * SK);
  sbs.load(g.B, g.ldb, n0, g.N, kt0 * SK);
  sa.store(smem);
  sbs.store(smem + SIMG);
  __syncthreads();
  for (int kt = kt0; kt < kt1; ++kt) {
    const unsigned char* Ai = smem + ((kt - kt0) & 1) * 2 * SIMG;
    const unsigned char* Bi = Ai + SIMG;
    const bool has_next = kt + 1 < kt1;
    if (has_next) {
      sa.load(g.A, g.lda, m0, g.M, (kt + 1) * SK);
      sbs.load(g.B, g.ldb, n0, g.N, (kt + 1) * SK);
    }
#pragma unroll
    for (int ks = 0; ks < SK / 16; ++ks) {
      const bf16x8 af = !TA ? row_frag<128>(Ai, wm * 32, ks * 16, lane) : tr_frag_nat<128>(Ai, ks * 16, wm * 32, lane);
      const bf16x8 bf = TB ? row_frag<128>(Bi, wn * 32, ks * 16, lane) : tr_frag_nat<128>(Bi, ks * 16, wn * 32, lane);
      acc = mfma32(bf, af, acc);
    }
    if (has_next) {
      unsigned char* nxt = smem + ((kt + 1 - kt0) & 1) * 2 * SIMG;
      sa.store(nxt);
      sbs.store(nxt + SIMG);
    }
    __syncthreads();
  }

  // ---- epilogue: lane row m, columns n = 8 g4 + 4 h + e (acc[4 g4 + e])
  const int h = lane >> 5;
  const int m = m0 + wm * 32 + (lane & 31);
  const bool mok = m < g.M;
  const int64_t roff = static_cast<int64_t>(mok ? m : g.M - 1) * g.ldc;
  float csum[16];
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int n = n0 + wn * 32 + 8 * g4 + 4 * h;
    const bool ok = mok && n < g.N;  // N % 8 == 0: a 4-group is all in or all out
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = g.alpha * acc[4 * g4 + e];
    if (EPI == sSplit) {
      if (ok)
        *reinterpret_cast<f32x4*>(g.ws + (static_cast<int64_t>(sp) * g.M + m) * g.N + n) = f32x4{v[0], v[1], v[2], v[3]};
      continue;
    }
    if (EPI == sBiasAct) {
      if (g.bias && n < g.N) {
        const bf16x4 bb = *reinterpret_cast<const bf16x4*>(g.bias + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += bf2f(bb[e]);
      }
      if (g.pre && ok) {
        bf16x4 pv;
#pragma unroll
        for (int e = 0; e < 4; ++e) pv[e] = f2bf(v[e]);
        *reinterpret_cast<bf16x4*>(g.pre + roff + n) = pv;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = s_act<ACT>(v[e]);
    }
    if (EPI == sDact) {
      bf16x4 xa{};
      if (ok) xa = *reinterpret_cast<const bf16x4*>(g.aux + roff + n);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] *= s_act_grad<ACT>(bf2f(xa[e]));
        csum[4 * g4 + e] = ok ? v[e] : 0.f;
      }
    }
    if (!ok) continue;
    if (g.out_f32) {
      float* C = static_cast<float*>(g.C) + roff + n;
      f32x4 o;
      if (EPI == sPlain && g.beta != 0.f) o = *reinterpret_cast<const f32x4*>(C);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = v[e] + ((EPI == sPlain && g.beta != 0.f) ? g.beta * o[e] : 0.f);
      *reinterpret_cast<f32x4*>(C) = o;
    } else {
      bf16* C = static_cast<bf16*>(g.C) + roff + n;
      if (EPI == sPlain && g.beta != 0.f) {
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
  if (EPI == sDact && g.dbias) {
    // column sums over the 32 rows of each wave half (lanes with equal h)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) csum[i] += __shfl_xor(csum[i], o, 64);
    }
    if ((lane & 31) == 0) {
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int n = n0 + wn * 32 + 8 * g4 + 4 * h;
        if (n < g.N) {
#pragma unroll
          for (int e = 0; e < 4; ++e) atomicAdd(g.dbias + n + e, csum[4 * g4 + e]);
        }
      }
    }
  }
}

}  // namespace

bool gemms_supported(const GemmPParams& p) {
  return p.K % SK == 0 && p.N % 8 == 0 && p.M % 8 == 0 && p.lda % 8 == 0 && p.ldb % 8 == 0;
}

void gemms_launch(const GemmPParams& p, int splits, hipStream_t st) { gemms_launch_batched(p, splits, 1, 0, 0, 0, st); }

void gemms_launch_batched(const GemmPParams& p, int splits, int batch, int64_t sA, int64_t sB, int64_t sC,
                          hipStream_t st) {
  if (!gemms_supported(p)) throw std::invalid_argument("gemms: needs K % 64, M / N / lda / ldb multiples of 8");
  const int epi = splits > 1 ? sSplit : p.act_bwd ? sDact : (p.bias || p.pre || p.act) ? sBiasAct : sPlain;
  if (epi == sBiasAct && (p.beta != 0.f || p.out_f32))
    throw std::invalid_argument("gemms: the bias / activation epilogue writes bf16 without beta");
  if (epi == sDact && (p.beta != 0.f || p.out_f32 || p.bias || p.pre))
    throw std::invalid_argument("gemms: the activation-gradient epilogue writes bf16, no beta / bias / pre");
  if (p.dbias && epi != sDact) throw std::invalid_argument("gemms: dbias needs the activation-gradient epilogue");
  GemmSArgs g{static_cast<const bf16*>(p.A), static_cast<const bf16*>(p.B), p.C, p.workspace,
              static_cast<const bf16*>(p.bias), static_cast<bf16*>(p.pre), static_cast<const bf16*>(p.aux), p.dbias,
              p.M, p.N, p.K, p.lda, p.ldb, p.ldc, p.alpha, p.beta, p.out_f32, splits, sA, sB, sC};
  if (batch > 1 && epi != sPlain) throw std::invalid_argument("gemms: batched products take the plain epilogue");
  const int nwg = ((p.M + SM - 1) / SM) * ((p.N + SN - 1) / SN);
  dim3 grid(nwg, splits, std::max(1, batch)), block(SNT);
  auto by_act = [&](auto ta, auto tb, auto e) {
    constexpr bool TA = decltype(ta)::value, TB = decltype(tb)::value;
    constexpr int EPI = decltype(e)::value;
    switch (EPI == sPlain || EPI == sSplit ? 0 : p.act) {
      case 1: hipLaunchKernelGGL((gemms_kernel<TA, TB, EPI, 1>), grid, block, 0, st, g); break;
      case 2: hipLaunchKernelGGL((gemms_kernel<TA, TB, EPI, 2>), grid, block, 0, st, g); break;
      case 3: hipLaunchKernelGGL((gemms_kernel<TA, TB, EPI, 3>), grid, block, 0, st, g); break;
      case 4: hipLaunchKernelGGL((gemms_kernel<TA, TB, EPI, 4>), grid, block, 0, st, g); break;
      default: hipLaunchKernelGGL((gemms_kernel<TA, TB, EPI, 0>), grid, block, 0, st, g); break;
    }
  };
  auto by_epi = [&](auto ta, auto tb) {
    switch (epi) {
      case sBiasAct: by_act(ta, tb, std::integral_constant<int, sBiasAct>{}); break;
      case sDact: by_act(ta, tb, std::integral_constant<int, sDact>{}); break;
      case sSplit: by_act(ta, tb, std::integral_constant<int, sSplit>{}); break;
      default: by_act(ta, tb, std::integral_constant<int, sPlain>{}); break;
    }
  };
  using F = std::false_type;
  using T = std::true_type;
  if (!p.trans_a && !p.trans_b) by_epi(F{}, F{});
  else if (!p.trans_a && p.trans_b) by_epi(F{}, T{});
  else if (p.trans_a && !p.trans_b) by_epi(T{}, F{});
  else by_epi(T{}, T{});
  FFK_LAUNCH_CHECK("gemms");
}

void bmm_bf16(const void* A, const void* B, void* C, int batch, int M, int N, int K, int lda, int ldb, int ldc,
              int64_t sA, int64_t sB, int64_t sC, bool trans_a, bool trans_b, float alpha, float beta, int out_f32,
              hipStream_t st) {
  if (batch <= 0 || M <= 0 || N <= 0 || K <= 0) return;
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B)) & 15 || (sA % 8) || (sB % 8))
    throw std::invalid_argument("bmm: operands and batch strides must be 16-byte aligned");
  if (ldc % 4 || sC % 4 || (reinterpret_cast<uintptr_t>(C) & (out_f32 ? 15 : 7)))
    throw std::invalid_argument("bmm: C alignment");
  GemmPParams p;
  p.A = A;
  p.B = B;
  p.C = C;
  p.M = M;
  p.N = N;
  p.K = K;
  p.lda = lda;
  p.ldb = ldb;
  p.ldc = ldc;
  p.trans_a = trans_a;
  p.trans_b = trans_b;
  p.alpha = alpha;
  p.beta = beta;
  p.out_f32 = out_f32;
  gemms_launch_batched(p, 1, batch, sA, sB, sC, st);
}

}  // namespace ffk
