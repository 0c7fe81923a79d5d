// fp32-accumulate implicit-GEMM family on the exact-f32 MFMA (gfx950):
//   * fp32 GEMMs  C = act(alpha op(A) op(B) + bias) (+ beta C), any transposes,
//     fp32 or bf16 output, optional pre-activation copy;
//   * 2-D convolution forward / data gradient / weight gradient over NHWC
//     activations and a [K][R][S][C/groups] weight, for fp32 AND bf16
//     tensors, with any number of groups (blockIdx.z = group).
//
// Parity: lib/kernels/src/cuda/ops/linear_kernels.cu:124-131 (the reference
// trains fp32 end to end: cublasGemmEx on fp32 operands) and
// conv_2d_kernels.cu:194-196,279-373 (cuDNN grouped convolution, groups set on
// the descriptor).  The bf16 ungrouped convolutions keep conv.hip's MFMA
// bf16 kernels; this file is what runs when the model computes in fp32 and
// for grouped convolutions (ResNeXt), which conv.hip does not tile.
//
// Matrix core: v_mfma_f32_32x32x2_f32 — f32 in, f32 accumulate, bit-for-bit a
// k-ordered fmaf chain (cdna_hip_programming.md §3 'FP32-input MFMA'), at the
// f32 vector rate (64 FLOP / clk / SIMD), one VGPR per operand per lane.  The
// A operand of lane l is A[i = l & 31][k = l >> 5], the B operand
// B[k = l >> 5][j = l & 31]; the accumulator holds D[row][col = l & 31] with
// row = (reg & 3) + 8 (reg >> 2) + 4 (l >> 5).
//
// Tile: BM = 128 rows (4 waves x 32) by BN = 32 or 64 columns, BK = 16, both
// operands staged through registers into K-major LDS images [k][outer]
// (fp32, converted from bf16 on load): every fragment read is 32 consecutive
// floats per half wave (ds_read_b32, conflict-free).  Two LDS buffers: the
// global loads of K-tile t + 1 are in flight while tile t's 16 MFMA steps run.
// Each operand is fetched in 8-element chunks along its contiguous axis
// (16-B / 32-B vector loads when the chunk is aligned and in range, else
// element by element with per-element bounds and tap checks).
#include <type_traits>

#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int QBM = 128, QBK = 16, QTHREADS = 256;
typedef float q16 __attribute__((ext_vector_type(16)));
typedef float q4 __attribute__((ext_vector_type(4)));

enum { Q_GEMM = 0, Q_FWD = 1, Q_DGRAD = 2, Q_WGRAD = 3 };

struct Q32Args {
  const void* A;     // GEMM A | FWD x | DGRAD dy | WGRAD dy
  const void* B;     // GEMM B | FWD / DGRAD w | WGRAD x
  void* C;           // GEMM C | FWD y | DGRAD dx | WGRAD dw (fp32)
  const void* bias;  // GEMM / FWD bias [N] (dtype of the inputs)
  void* pre;         // GEMM pre-activation copy (out dtype)
  int64_t M, N, K;   // GEMM sizes (per group for convolutions)
  int64_t lda, ldb, ldc;
  int64_t sa, sb, sc;  // GEMM batch strides (blockIdx.z = batch index)
  int ta, tb;        // GEMM transposes
  float alpha, beta;
  int act, out_f32;
  // convolution geometry (per group: Cg input / Kg output channels)
  int n, H, W, Cin, Kout, R, S, P, Q, sh, sw, ph, pw, dh, dw, Cg, Kg;
  int k_per_split;   // WGRAD: K-tiles per split (blockIdx.y)
  int vecA, vecB;    // 8-element chunks may use vector loads
};

__device__ __forceinline__ float q_act(int act, float x) {
  switch (act) {
    case 1: return x > 0.f ? x : 0.f;
    case 2: return 1.f / (1.f + __expf(-x));
    case 3: return tanhf(x);
    case 4: {
      const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    default: return x;
  }
}

template <typename T>
__device__ __forceinline__ float q_ld(const T* p) {
  if constexpr (std::is_same<T, float>::value) return *p;
  else return bf2f(*p);
}
// 8 consecutive elements (16-B aligned for bf16, 32-B for fp32)
template <typename T>
__device__ __forceinline__ void q_ld8(const T* p, float (&v)[8]) {
  if constexpr (std::is_same<T, float>::value) {
    const q4 a = *reinterpret_cast<const q4*>(p), b = *reinterpret_cast<const q4*>(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = a[e];
      v[4 + e] = b[e];
    }
  } else {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bf2f(a[e]);
  }
}

// ---- operand element maps.  Each returns the element pointer of (row o of
// the operand's outer axis, k) or null when the element is a structural
// zero (outside the image, outside the matrix).
// A side: outer = GEMM row m.  B side: outer = GEMM column n.
template <int MODE, typename T>
struct QOps {
  // contiguous axis of each operand: true = k (chunks of 8 consecutive k),
  // false = outer (chunks of 8 consecutive rows / columns)
  __device__ static bool a_kc(const Q32Args& g) {
    if (MODE == Q_GEMM) return !g.ta;
    return MODE != Q_WGRAD;
  }
  __device__ static bool b_kc(const Q32Args& g) {
    if (MODE == Q_GEMM) return g.tb;
    return MODE == Q_FWD;
  }
  __device__ static const T* a_ptr(const Q32Args& g, int grp, int64_t m, int64_t k) {
    if (m >= g.M || k >= g.K) return nullptr;
    const T* A = static_cast<const T*>(g.A);
    if (MODE == Q_GEMM) return A + grp * g.sa + (g.ta ? k * g.lda + m : m * g.lda + k);
    if (MODE == Q_FWD) {   // x gather: m = (n, p, q), k = (r, s, c)
      const int q = static_cast<int>(m % g.Q);
      const int64_t t = m / g.Q;
      const int p = static_cast<int>(t % g.P), nn = static_cast<int>(t / g.P);
      const int c = static_cast<int>(k % g.Cg), rs = static_cast<int>(k / g.Cg);
      const int s = rs % g.S, r = rs / g.S;
      const int ih = p * g.sh - g.ph + r * g.dh, iw = q * g.sw - g.pw + s * g.dw;
      if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return nullptr;
      return A + ((static_cast<int64_t>(nn) * g.H + ih) * g.W + iw) * g.Cin + grp * g.Cg + c;
    }
    if (MODE == Q_DGRAD) {  // dy gather: m = input pixel (n, h, w), k = (r, s, ko)
      const int w = static_cast<int>(m % g.W);
      const int64_t t = m / g.W;
      const int h = static_cast<int>(t % g.H), nn = static_cast<int>(t / g.H);
      const int ko = static_cast<int>(k % g.Kg), rs = static_cast<int>(k / g.Kg);
      const int s = rs % g.S, r = rs / g.S;
      const int yn = h + g.ph - r * g.dh, xn = w + g.pw - s * g.dw;
      if (yn < 0 || xn < 0) return nullptr;
      const int oh = yn / g.sh, ow = xn / g.sw;
      if (oh * g.sh != yn || ow * g.sw != xn || oh >= g.P || ow >= g.Q) return nullptr;
      return A + ((static_cast<int64_t>(nn) * g.P + oh) * g.Q + ow) * g.Kout + grp * g.Kg + ko;
    }
    // WGRAD: A[m = ko][k = output pixel] = dy[pixel][grp Kg + ko]
    return A + k * g.Kout + grp * g.Kg + m;
  }
  __device__ static const T* b_ptr(const Q32Args& g, int grp, int64_t n, int64_t k) {
    if (n >= g.N || k >= g.K) return nullptr;
    const T* B = static_cast<const T*>(g.B);
    if (MODE == Q_GEMM) return B + grp * g.sb + (g.tb ? n * g.ldb + k : k * g.ldb + n);
    if (MODE == Q_FWD) return B + (static_cast<int64_t>(grp) * g.Kg + n) * g.K + k;   // w[kout][(r,s,c)]
    if (MODE == Q_DGRAD) {  // w[grp Kg + ko][r][s][c = n], k = (r, s, ko)
      const int ko = static_cast<int>(k % g.Kg), rs = static_cast<int>(k / g.Kg);
      const int s = rs % g.S, r = rs / g.S;
      return B + ((((static_cast<int64_t>(grp) * g.Kg + ko) * g.R + r) * g.S + s) * g.Cg) + n;
    }
    // WGRAD: B[k = output pixel (n, p, q)][n = (r, s, c)] = x gather
    const int c = static_cast<int>(n % g.Cg), rs = static_cast<int>(n / g.Cg);
    const int s = rs % g.S, r = rs / g.S;
    const int q = static_cast<int>(k % g.Q);
    const int64_t t = k / g.Q;
    const int p = static_cast<int>(t % g.P), nn = static_cast<int>(t / g.P);
    const int ih = p * g.sh - g.ph + r * g.dh, iw = q * g.sw - g.pw + s * g.dw;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) return nullptr;
    return B + ((static_cast<int64_t>(nn) * g.H + ih) * g.W + iw) * g.Cin + grp * g.Cg + c;
  }
};

// One 8-element chunk of an operand tile [QBK k][BOUT outer]:
//   kc: row o = chunk >> 1, k = 8 (chunk & 1) ..+8   (BOUT * 2 chunks)
//   oc: k = chunk / (BOUT / 8), outer = 8 (chunk % (BOUT / 8)) ..+8
template <int MODE, typename T, bool ASIDE, int BOUT>
struct QChunk {
  float v[8];
  bool live;
  int o, k;   // tile-local coordinates of element 0
  bool kc;

  __device__ __forceinline__ void load(const Q32Args& g, int grp, int64_t o0, int64_t k0, int chunk, bool vec) {
    kc = ASIDE ? QOps<MODE, T>::a_kc(g) : QOps<MODE, T>::b_kc(g);
    constexpr int NCH = BOUT * 2;
    live = chunk < NCH;
    if (!live) return;
    if (kc) {
      o = chunk >> 1;
      k = 8 * (chunk & 1);
    } else {
      constexpr int CPR = BOUT / 8;
      k = chunk / CPR;
      o = 8 * (chunk % CPR);
    }
    auto ptr = [&](int e) -> const T* {
      const int64_t oo = o0 + o + (kc ? 0 : e), kk = k0 + k + (kc ? e : 0);
      return ASIDE ? QOps<MODE, T>::a_ptr(g, grp, oo, kk) : QOps<MODE, T>::b_ptr(g, grp, oo, kk);
    };
    if (vec) {
      // fast path: the chunk is 8 consecutive in-range elements of one row /
      // tap, so element 0's pointer and element 7's existence decide it
      const T* p0 = ptr(0);
      const T* p7 = ptr(7);
      if (p0 != nullptr && p7 == p0 + 7) {
        q_ld8<T>(p0, v);
        return;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const T* p = ptr(e);
      v[e] = p ? q_ld<T>(p) : 0.f;
    }
  }
  // LDS image [QBK][BOUT] fp32 (row = BOUT floats)
  __device__ __forceinline__ void store(float* img) const {
    if (!live) return;
    if (kc) {
#pragma unroll
      for (int e = 0; e < 8; ++e) img[(k + e) * BOUT + o] = v[e];
    } else {
      q4* d = reinterpret_cast<q4*>(img + k * BOUT + o);
      d[0] = q4{v[0], v[1], v[2], v[3]};
      d[1] = q4{v[4], v[5], v[6], v[7]};
    }
  }
};

template <int MODE, typename T, int BN>
__global__ __launch_bounds__(QTHREADS) void igemm32_kernel(Q32Args g) {
  constexpr int NB = BN / 32;                     // 32x32 blocks per wave
  constexpr int SA = QBK * QBM, SB = QBK * BN;    // floats per image
  __shared__ __attribute__((aligned(16))) float smem[2 * (SA + SB)];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = blockIdx.z;

  const int64_t gm = (g.M + QBM - 1) / QBM, gn = (g.N + BN - 1) / BN;
  const int64_t tile = blockIdx.x;
  // grouped raster: 8 row tiles share their column tiles in L2
  const int64_t per_group = 8 * gn;
  const int64_t first_m = (tile / per_group) * 8;
  const int64_t gsize = min(gm - first_m, int64_t(8));
  const int64_t m0 = (first_m + (tile % per_group) % gsize) * QBM;
  const int64_t n0 = ((tile % per_group) / gsize) * BN;

  const int64_t nkt = (g.K + QBK - 1) / QBK;
  int64_t kt0 = 0, kt1 = nkt;
  if (MODE == Q_WGRAD) {
    kt0 = static_cast<int64_t>(blockIdx.y) * g.k_per_split;
    kt1 = min(nkt, kt0 + g.k_per_split);
    if (kt0 >= kt1) return;
  }

  QChunk<MODE, T, true, QBM> ca;
  QChunk<MODE, T, false, BN> cb;
  auto load = [&](int64_t kt) {
    ca.load(g, grp, m0, kt * QBK, tid, g.vecA != 0);
    cb.load(g, grp, n0, kt * QBK, tid, g.vecB != 0);
  };
  auto store = [&](float* buf) {
    ca.store(buf);
    cb.store(buf + SA);
  };

  q16 acc[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) acc[j] = q16{};

  load(kt0);
  store(smem);
  __syncthreads();
  for (int64_t kt = kt0; kt < kt1; ++kt) {
    const float* As = smem + ((kt - kt0) & 1) * (SA + SB);
    const float* Bs = As + SA;
    const bool next = kt + 1 < kt1;
    if (next) load(kt + 1);
#pragma unroll
    for (int ks = 0; ks < QBK / 2; ++ks) {
      const int kr = 2 * ks + (lane >> 5);
      const float a = As[kr * QBM + wave * 32 + (lane & 31)];
      float b[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) b[j] = Bs[kr * BN + j * 32 + (lane & 31)];
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b[j], acc[j], 0, 0, 0);
    }
    if (next) store(smem + ((kt + 1 - kt0) & 1) * (SA + SB));
    __syncthreads();
  }

  // ---- epilogue: lane owns column n = n0 + 32 j + (lane & 31), 16 rows
  const int64_t rbase = m0 + wave * 32 + 4 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int64_t n = n0 + j * 32 + (lane & 31);
    if (n >= g.N) continue;
    if (MODE == Q_WGRAD) {
      float* dw = static_cast<float*>(g.C) + (static_cast<int64_t>(grp) * g.Kg) * g.N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = rbase + (r & 3) + 8 * (r >> 2);
        if (m >= g.M) continue;
        float* d = dw + m * g.N + n;
        if (gridDim.y > 1) atomicAdd(d, acc[j][r]);
        else *d += acc[j][r];
      }
      continue;
    }
    float bv = 0.f;
    if ((MODE == Q_GEMM || MODE == Q_FWD) && g.bias) {
      const int64_t bn = MODE == Q_FWD ? static_cast<int64_t>(grp) * g.Kg + n : n;
      bv = q_ld<T>(static_cast<const T*>(g.bias) + bn);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = rbase + (r & 3) + 8 * (r >> 2);
      if (m >= g.M) continue;
      int64_t off;
      if (MODE == Q_GEMM) off = grp * g.sc + m * g.ldc + n;
      else if (MODE == Q_FWD) off = m * g.Kout + static_cast<int64_t>(grp) * g.Kg + n;
      else off = m * g.Cin + static_cast<int64_t>(grp) * g.Cg + n;
      float v = (MODE == Q_GEMM ? g.alpha : 1.f) * acc[j][r] + bv;
      if (MODE != Q_DGRAD) {
        if (g.pre) {
          if (g.out_f32) static_cast<float*>(g.pre)[off] = v;
          else static_cast<bf16*>(g.pre)[off] = f2bf(v);
        }
        v = q_act(g.act, v);
      }
      if (g.out_f32) {
        float* o = static_cast<float*>(g.C) + off;
        *o = g.beta != 0.f ? v + g.beta * *o : v;
      } else {
        bf16* o = static_cast<bf16*>(g.C) + off;
        *o = f2bf(g.beta != 0.f ? v + g.beta * bf2f(*o) : v);
      }
    }
  }
}

template <int MODE, typename T>
void q_launch(const Q32Args& g, int bn, dim3 grid, hipStream_t st) {
  if (bn == 32) hipLaunchKernelGGL((igemm32_kernel<MODE, T, 32>), grid, dim3(QTHREADS), 0, st, g);
  else hipLaunchKernelGGL((igemm32_kernel<MODE, T, 64>), grid, dim3(QTHREADS), 0, st, g);
}

template <int MODE>
void q_dispatch(const Q32Args& g, int in_f32, int bn, dim3 grid, hipStream_t st) {
  if (in_f32) q_launch<MODE, float>(g, bn, grid, st);
  else q_launch<MODE, bf16>(g, bn, grid, st);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

dim3 q_grid(int64_t M, int64_t N, int bn, int ysplit, int groups) {
  const int64_t tiles = ((M + QBM - 1) / QBM) * ((N + bn - 1) / bn);
  if (tiles >= (int64_t(1) << 31)) throw std::invalid_argument("igemm32: too many tiles");
  return dim3(static_cast<unsigned>(tiles), static_cast<unsigned>(ysplit), static_cast<unsigned>(groups));
}

Q32Args conv_args(const ConvShape& cs, int groups) {
  if (groups <= 0 || cs.C % groups || cs.K % groups) throw std::invalid_argument("conv32: channels % groups != 0");
  if (cs.N <= 0 || cs.H <= 0 || cs.W <= 0 || cs.R <= 0 || cs.S <= 0 || cs.sh <= 0 || cs.sw <= 0 || cs.dh <= 0 ||
      cs.dw <= 0 || cs.ph < 0 || cs.pw < 0)
    throw std::invalid_argument("conv32: bad geometry");
  Q32Args g{};
  g.n = cs.N; g.H = cs.H; g.W = cs.W; g.Cin = cs.C; g.Kout = cs.K; g.R = cs.R; g.S = cs.S;
  g.sh = cs.sh; g.sw = cs.sw; g.ph = cs.ph; g.pw = cs.pw; g.dh = cs.dh; g.dw = cs.dw;
  g.P = (cs.H + 2 * cs.ph - cs.dh * (cs.R - 1) - 1) / cs.sh + 1;
  g.Q = (cs.W + 2 * cs.pw - cs.dw * (cs.S - 1) - 1) / cs.sw + 1;
  if (g.P <= 0 || g.Q <= 0) throw std::invalid_argument("conv32: empty output");
  g.Cg = cs.C / groups;
  g.Kg = cs.K / groups;
  g.alpha = 1.f;
  return g;
}

}  // namespace

void gemm_f32(const void* A, const void* B, void* C, const void* bias, void* pre, int64_t M, int64_t N, int64_t K,
              int64_t lda, int64_t ldb, int64_t ldc, bool trans_a, bool trans_b, int act, float alpha, float beta,
              int in_f32, int out_f32, hipStream_t st, int batch, int64_t sa, int64_t sb, int64_t sc) {
  if (M <= 0 || N <= 0 || batch <= 0) return;
  if (batch > 65535) throw std::invalid_argument("gemm_f32: batch > 65535");
  Q32Args g{};
  g.A = A; g.B = B; g.C = C; g.bias = bias; g.pre = pre;
  g.M = M; g.N = N; g.K = K; g.lda = lda; g.ldb = ldb; g.ldc = ldc;
  g.sa = sa; g.sb = sb; g.sc = sc;
  g.ta = trans_a; g.tb = trans_b; g.alpha = alpha; g.beta = beta; g.act = act; g.out_f32 = out_f32;
  // vector chunks: 8 consecutive elements along the contiguous axis start on
  // a multiple of 8 elements, so an aligned base, leading dim and batch
  // stride suffice
  g.vecA = aligned16(A) && lda % 8 == 0 && sa % 8 == 0;
  g.vecB = aligned16(B) && ldb % 8 == 0 && sb % 8 == 0;
  const int bn = N <= 32 ? 32 : 64;
  q_dispatch<Q_GEMM>(g, in_f32, bn, q_grid(M, N, bn, 1, batch), st);
  FFK_LAUNCH_CHECK("gemm_f32");
}

void conv32_fwd(const ConvShape& cs, int groups, const void* x, const void* w, const void* bias, void* y, int act,
                int in_f32, hipStream_t st) {
  Q32Args g = conv_args(cs, groups);
  g.A = x; g.B = w; g.C = y; g.bias = bias; g.act = act; g.out_f32 = in_f32;
  g.M = static_cast<int64_t>(g.n) * g.P * g.Q;
  g.N = g.Kg;
  g.K = static_cast<int64_t>(g.R) * g.S * g.Cg;
  g.vecA = aligned16(x) && g.Cg % 8 == 0 && g.Cin % 8 == 0;
  g.vecB = aligned16(w) && g.K % 8 == 0;
  const int bn = g.N <= 32 ? 32 : 64;
  q_dispatch<Q_FWD>(g, in_f32, bn, q_grid(g.M, g.N, bn, 1, groups), st);
  FFK_LAUNCH_CHECK("conv32_fwd");
}

void conv32_dgrad(const ConvShape& cs, int groups, const void* dy, const void* w, void* dx, float beta, int in_f32,
                  hipStream_t st) {
  Q32Args g = conv_args(cs, groups);
  g.A = dy; g.B = w; g.C = dx; g.beta = beta; g.out_f32 = in_f32;
  g.M = static_cast<int64_t>(g.n) * g.H * g.W;
  g.N = g.Cg;
  g.K = static_cast<int64_t>(g.R) * g.S * g.Kg;
  g.vecA = aligned16(dy) && g.Kg % 8 == 0 && g.Kout % 8 == 0;
  g.vecB = aligned16(w) && g.Cg % 8 == 0;
  const int bn = g.N <= 32 ? 32 : 64;
  q_dispatch<Q_DGRAD>(g, in_f32, bn, q_grid(g.M, g.N, bn, 1, groups), st);
  FFK_LAUNCH_CHECK("conv32_dgrad");
}

void conv32_wgrad(const ConvShape& cs, int groups, const void* x, const void* dy, float* dw, int in_f32,
                  hipStream_t st) {
  Q32Args g = conv_args(cs, groups);
  g.A = dy;     // A[m = ko][k = pixel]
  g.B = x;      // B[k = pixel][n = (r, s, c)], gathered
  g.C = dw;
  g.out_f32 = 1;
  g.M = g.Kg;
  g.N = static_cast<int64_t>(g.R) * g.S * g.Cg;
  g.K = static_cast<int64_t>(g.n) * g.P * g.Q;
  g.vecA = aligned16(dy) && g.Kg % 8 == 0 && g.Kout % 8 == 0;
  g.vecB = aligned16(x) && g.Cg % 8 == 0 && g.Cin % 8 == 0;
  const int bn = g.N <= 32 ? 32 : 64;
  const int64_t tiles = ((g.M + QBM - 1) / QBM) * ((g.N + bn - 1) / bn) * groups;
  const int64_t nkt = (g.K + QBK - 1) / QBK;
  // ~2048 workgroups, >= 16 K-tiles each; fp32 atomics combine the splits
  int64_t splits = std::max<int64_t>(1, std::min<int64_t>((2048 + tiles - 1) / tiles, nkt / 16));
  splits = std::min<int64_t>(splits, 65535);
  g.k_per_split = static_cast<int>((nkt + splits - 1) / splits);
  splits = (nkt + g.k_per_split - 1) / g.k_per_split;
  q_dispatch<Q_WGRAD>(g, in_f32, bn, q_grid(g.M, g.N, bn, static_cast<int>(splits), groups), st);
  FFK_LAUNCH_CHECK("conv32_wgrad");
}

}  // namespace ffk
