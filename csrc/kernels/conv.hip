// Implicit-GEMM convolution for gfx950 (NHWC bf16, fp32 accumulate on MFMA).
//
// Parity: lib/kernels/src/cuda/ops/conv_2d_kernels.cu (cudnnConvolutionForward
// :279 + bias/activation :303, BackwardFilter :346, BackwardData :362,
// BackwardBias :373; algorithms autotuned with cudnnFind*AlgorithmEx :8-115).
// There NCHW fp32 through cuDNN; here three hand-written MFMA kernels that
// never materialise im2col:
//
//   FWD   Y[m=(n,p,q)][k]      = sum_{(r,s,c)} X[n, p*sh-ph+r*dh, q*sw-pw+s*dw, c] * W[k][r][s][c]
//   DGRAD dX[m=(n,h,w)][c]     = sum_{(r,s,k)} dY[n, (h+ph-r*dh)/sh, (w+pw-s*dw)/sw, k] * W[k][r][s][c]
//   WGRAD dW[k][(r,s,c)]      += sum_{m=(n,p,q)} dY[m][k] * X[n, p*sh-ph+r*dh, q*sw-pw+s*dw, c]
//
// Layouts: activations NHWC (torch channels_last), the weight physically
// [K][R][S][C] so its GEMM K axis (r,s,c) is contiguous.  C and K must be
// multiples of 8 (a 16-byte chunk of 8 channels never straddles a filter tap;
// the stem's 3 input channels are zero-padded to 8 by the host).
//
// Structure: the 128xBN x64 register-staged, double-buffered LDS tile of
// gemm.hip (4 waves 2x2, v_mfma_f32_32x32x16_bf16, XOR-swizzled images read
// by ds_read_b128 or ds_read_b64_tr_b16), with the operand stagers replaced
// by gathers that compute the input coordinates of each 8-channel chunk
// (out-of-image taps and tile tails load zeros).  BN = 64 serves the
// 64-channel layers without wasting half the MFMAs.  Epilogues: FWD fuses
// bias + activation and (optionally) the per-channel sum / sum-of-squares a
// following training-mode BatchNorm needs (a wave-reduce per column into a
// per-tile partial slot, folded by reduce_rows — no same-address atomic
// storms), so BN never re-reads Y for its statistics; WGRAD is split-K over
// the pixel axis with per-split fp32 slabs summed by reduce_rows into the
// flat gradient buffer (+=); a single-split launch accumulates in place.
#include "kernels.h"
#include "mfma.h"

namespace ffk {

namespace {

constexpr int BM = 128, BK = 64;
enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

struct ConvArgs {
  const bf16* x;    // FWD/WGRAD input  [N][H][W][C]
  const bf16* w;    // FWD/DGRAD weight [K][R][S][C]
  const bf16* dy;   // DGRAD/WGRAD      [N][P][Q][K]
  void* out;        // FWD y [N][P][Q][K] bf16 | DGRAD dx [N][H][W][C] bf16 | WGRAD dw [K][R][S][C] f32
  const bf16* bias; // FWD only
  float* stats;     // FWD only: per-wave partials [gm*2][2][K] (sum, sum of squares)
  float* wpart;     // WGRAD split-K partial slabs [splits][K][R*S*C] (null: splits == 1)
  int N, H, W, C, K, R, S, P, Q;
  int sh, sw, ph, pw, dh, dw;
  int M, NG, KG;    // GEMM sizes
  int act;
  float beta;       // DGRAD: dx = result + beta * dx
  int kt_per_split; // WGRAD split-K
  // DGRAD parity class (strided convs): rows are the input pixels with
  // h % sh == pch, w % sw == pcw (Hc x Wc per image); the K axis runs only over
  // the taps r = rf + i*sh (i < nr), s = sf + j*sw (j < ns) that reach them.
  int par, pch, pcw, Hc, Wc, rf, sf, nr, ns;
};

// DGRAD output row of local row m (parity classes scatter to the full image)
__device__ __forceinline__ int64_t dgrad_row(const ConvArgs& g, int m) {
  if (!g.par) return m;
  const int ww = m % g.Wc, t = m / g.Wc, hh = t % g.Hc, n = t / g.Hc;
  return (static_cast<int64_t>(n) * g.H + hh * g.sh + g.pch) * g.W + ww * g.sw + g.pcw;
}
// (r, s) of tap index rs of the K axis
__device__ __forceinline__ void tap_of(const ConvArgs& g, int rs, int& r, int& s) {
  if (g.par) {
    const int j = rs % g.ns, i = rs / g.ns;
    r = g.rf + i * g.sh;
    s = g.sf + j * g.sw;
  } else {
    s = rs % g.S;
    r = rs / g.S;
  }
}

__device__ __forceinline__ float conv_act(int act, float x) {
  switch (act) {
    case 1: return x > 0.f ? x : 0.f;
    case 2: return 1.f / (1.f + __expf(-x));
    case 3: return fast_tanh(x);
    case 4: return gelu_tanh(x);
    default: return x;
  }
}

__device__ __forceinline__ bf16x8 ld8(const bf16* p, bool ok) {
  return ok ? *reinterpret_cast<const bf16x8*>(p) : bf16x8{};
}

// ---------------------------------------------------------------------------
// A operand, K-contiguous image [128 rows = m][64 k], 4 chunks per thread.
// FWD: m = output pixel (n,p,q), k = (r,s,c).  DGRAD: m = input pixel (n,h,w),
// k = (r,s,kout).  The pixel decode happens once; the tap decode once per tile.
template <int MODE>
struct AGather {
  bf16x8 reg[4];
  int64_t base[4];  // element offset of the image n (NHWC / NPQK)
  int ya[4], xa[4]; // FWD: p*sh-ph, q*sw-pw ; DGRAD: h+ph, w+pw ; INT_MIN = row past M

  __device__ __forceinline__ void init(const ConvArgs& g, int m0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + (threadIdx.x >> 3) + 32 * i;
      if (m >= g.M) {
        ya[i] = -0x3fffffff;
        xa[i] = 0;
        base[i] = 0;
        continue;
      }
      if (MODE == MODE_FWD) {
        const int q = m % g.Q, t = m / g.Q, p = t % g.P, n = t / g.P;
        ya[i] = p * g.sh - g.ph;
        xa[i] = q * g.sw - g.pw;
        base[i] = static_cast<int64_t>(n) * g.H * g.W * g.C;
      } else {
        int w, h, n;
        if (g.par) {
          const int ww = m % g.Wc, t = m / g.Wc, hh = t % g.Hc;
          n = t / g.Hc;
          h = hh * g.sh + g.pch;
          w = ww * g.sw + g.pcw;
        } else {
          const int t = m / g.W;
          w = m % g.W;
          h = t % g.H;
          n = t / g.H;
        }
        ya[i] = h + g.ph;
        xa[i] = w + g.pw;
        base[i] = static_cast<int64_t>(n) * g.P * g.Q * g.K;
      }
    }
  }
  __device__ __forceinline__ void load(const ConvArgs& g, int k0) {
    const int k = k0 + (threadIdx.x & 7) * 8;
    const bool kok = k < g.KG;
    const int CC = MODE == MODE_FWD ? g.C : g.K;
    const int cc = k % CC, rs = k / CC;
    int r, s;
    if (MODE == MODE_FWD) {
      s = rs % g.S;
      r = rs / g.S;
    } else {
      tap_of(g, rs, r, s);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool ok = kok;
      const bf16* src;
      if (MODE == MODE_FWD) {
        const int ih = ya[i] + r * g.dh, iw = xa[i] + s * g.dw;
        ok = ok && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        src = g.x + base[i] + (static_cast<int64_t>(ih) * g.W + iw) * g.C + cc;
      } else {
        const int yn = ya[i] - r * g.dh, xn = xa[i] - s * g.dw;
        const int oh = yn / g.sh, ow = xn / g.sw;
        ok = ok && yn >= 0 && xn >= 0 && yn == oh * g.sh && xn == ow * g.sw && oh < g.P && ow < g.Q;
        src = g.dy + base[i] + (static_cast<int64_t>(oh) * g.Q + ow) * g.K + cc;
      }
      reg[i] = ld8(src, ok);
    }
  }
  __device__ __forceinline__ void store(unsigned char* img) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = threadIdx.x + 256 * i;
      *reinterpret_cast<bf16x8*>(img + img_off<128>(c >> 3, c & 7)) = reg[i];
    }
  }
};

// Plain K-contiguous operand [OUTER rows][64 k] (FWD weight: [K][R*S*C]).
template <int OUTER>
struct RowStager {
  static constexpr int NL = OUTER / 32;
  bf16x8 reg[NL];
  __device__ __forceinline__ void load(const bf16* P, int ld, int outer0, int n_outer, int k0, int K) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = threadIdx.x + 256 * i, r = c >> 3, ch = c & 7;
      const bool ok = (outer0 + r < n_outer) && (k0 + ch * 8 < K);
      reg[i] = ld8(P + static_cast<int64_t>(outer0 + r) * ld + k0 + ch * 8, ok);
    }
  }
  __device__ __forceinline__ void store(unsigned char* img) const {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = threadIdx.x + 256 * i;
      *reinterpret_cast<bf16x8*>(img + img_off<128>(c >> 3, c & 7)) = reg[i];
    }
  }
};

// Operand stored [k][outer] ("transposed"), image [64 k rows][OUTER].
//   KIND 0: plain rows (WGRAD A = dY [pixels][K], outer = kout)
//   KIND 1: DGRAD B: row k = (r,s,kout) -> W[kout][r][s][c0..], outer = c
//   KIND 2: WGRAD B: row k = pixel (n,p,q), outer = (r,s,c) -> X gather
template <int OUTER, int KIND>
struct ColStager {
  static constexpr int CPR = OUTER / 8;         // chunks per image row
  static constexpr int NL = 64 * CPR / 256;     // chunks per thread
  static constexpr int RB = OUTER * 2;          // image row bytes
  bf16x8 reg[NL];
  // KIND 2: per-thread tap (fixed across tiles: the thread's chunk column is fixed)
  int tr_, ts_, tc_;
  bool tok_;

  __device__ __forceinline__ void init(const ConvArgs& g, int outer0) {
    if (KIND == 2) {
      const int n = outer0 + (threadIdx.x % CPR) * 8;
      tok_ = n < g.NG;
      tc_ = n % g.C;
      const int rs = n / g.C;
      ts_ = rs % g.S;
      tr_ = rs / g.S;
    }
  }
  __device__ __forceinline__ void load(const ConvArgs& g, const bf16* P, int ld, int outer0, int n_outer, int k0,
                                       int K) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = threadIdx.x + 256 * i, r = c / CPR, ch = c % CPR;
      const int k = k0 + r, o = outer0 + ch * 8;
      bool ok = (k < K) && (o < n_outer);
      const bf16* src;
      if (KIND == 0) {
        src = P + static_cast<int64_t>(k) * ld + o;
      } else if (KIND == 1) {
        const int kout = k % g.K, rs = k / g.K;
        int rr, s;
        tap_of(g, rs, rr, s);
        src = g.w + ((static_cast<int64_t>(kout) * g.R + rr) * g.S + s) * g.C + o;
      } else {
        const int q = k % g.Q, t = k / g.Q, p = t % g.P, n = t / g.P;
        const int ih = p * g.sh - g.ph + tr_ * g.dh, iw = q * g.sw - g.pw + ts_ * g.dw;
        ok = ok && tok_ && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
        src = g.x + ((static_cast<int64_t>(n) * g.H + ih) * g.W + iw) * g.C + tc_;
      }
      reg[i] = ld8(src, ok);
    }
  }
  __device__ __forceinline__ void store(unsigned char* img) const {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = threadIdx.x + 256 * i;
      *reinterpret_cast<bf16x8*>(img + img_off<RB>(c / CPR, c % CPR)) = reg[i];
    }
  }
};

// ---------------------------------------------------------------------------
template <int MODE, int BN>
__global__ __launch_bounds__(256, 2) void conv_igemm_kernel(ConvArgs g) {
  constexpr int IMG = BM * BK * 2;  // 16 KiB (A image; B image is BN*BK*2)
  constexpr int IMGB = BN * BK * 2;
  constexpr int NTN = BN / 64;      // 32-wide n subtiles per wave
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * (IMG + IMGB)];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 1, wn = wave >> 1;

  const int gm = (g.M + BM - 1) / BM, gn = (g.NG + BN - 1) / BN;
  const int ntile = gm * gn;
  int bid = blockIdx.x, split = 0;
  if (MODE == MODE_WGRAD) {
    split = bid / ntile;
    bid = bid % ntile;
  } else {
    bid = xcd_remap(bid, ntile);
  }
  // grouped raster (8 m-tiles share their B tiles in L2)
  const int per_group = 8 * gn;
  const int first_m = (bid / per_group) * 8;
  const int gsize = min(gm - first_m, 8);
  const int tm = first_m + (bid % per_group) % gsize;
  const int tn = (bid % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  const int nk_all = (g.KG + BK - 1) / BK;
  int kt0 = 0, kt1 = nk_all;
  if (MODE == MODE_WGRAD) {
    kt0 = split * g.kt_per_split;
    kt1 = min(nk_all, kt0 + g.kt_per_split);
    if (kt0 >= kt1) return;
  }

  // operand stagers
  AGather<MODE_FWD> afw;
  AGather<MODE_DGRAD> adg;
  ColStager<128, 0> awg;  // WGRAD A: dY [pix][K], outer = kout (M side)
  RowStager<BN> bfw;
  ColStager<BN, 1> bdg;
  ColStager<BN, 2> bwg;

  auto load = [&](int kt) {
    const int k0 = kt * BK;
    if (MODE == MODE_FWD) {
      afw.load(g, k0);
      bfw.load(g.w, g.KG, n0, g.NG, k0, g.KG);
    } else if (MODE == MODE_DGRAD) {
      adg.load(g, k0);
      bdg.load(g, nullptr, 0, n0, g.NG, k0, g.KG);
    } else {
      awg.load(g, g.dy, g.K, m0, g.M, k0, g.KG);
      bwg.load(g, nullptr, 0, n0, g.NG, k0, g.KG);
    }
  };
  auto store = [&](unsigned char* buf) {
    if (MODE == MODE_FWD) {
      afw.store(buf);
      bfw.store(buf + IMG);
    } else if (MODE == MODE_DGRAD) {
      adg.store(buf);
      bdg.store(buf + IMG);
    } else {
      awg.store(buf);
      bwg.store(buf + IMG);
    }
  };

  if (MODE == MODE_FWD) afw.init(g, m0);
  if (MODE == MODE_DGRAD) adg.init(g, m0);
  if (MODE == MODE_WGRAD) bwg.init(g, n0);

  f32x16 acc[NTN][2];
#pragma unroll
  for (int i = 0; i < NTN; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  load(kt0);
  store(smem);
  __syncthreads();

  for (int kt = kt0; kt < kt1; ++kt) {
    const unsigned char* Ai = smem + ((kt - kt0) & 1) * (IMG + IMGB);
    const unsigned char* Bi = Ai + IMG;
    const bool has_next = kt + 1 < kt1;
    if (has_next) load(kt + 1);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8 bf[NTN], af[2];
#pragma unroll
      for (int t = 0; t < NTN; ++t) {
        if (MODE == MODE_FWD) bf[t] = row_frag<128>(Bi, wn * (BN / 2) + t * 32, ks * 16, lane);
        else bf[t] = tr_frag_nat<BN * 2>(Bi, ks * 16, wn * (BN / 2) + t * 32, lane);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (MODE == MODE_WGRAD) af[t] = tr_frag_nat<256>(Ai, ks * 16, wm * 64 + t * 32, lane);
        else af[t] = row_frag<128>(Ai, wm * 64 + t * 32, ks * 16, lane);
      }
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[nt][mt] = mfma32(bf[nt], af[mt], acc[nt][mt]);
    }
    if (has_next) store(smem + ((kt + 1 - kt0) & 1) * (IMG + IMGB));
    __syncthreads();
  }

  // ---- epilogue: acc[nt][mt] holds C^T; lane&31 = m row, registers = 4 n columns
  const int h = lane >> 5;
  if (MODE == MODE_WGRAD) {
    // one writer per element: split 0 of a single-split launch accumulates into
    // dW directly; otherwise this split's slab (summed by reduce_rows)
    float* out = g.wpart ? g.wpart + static_cast<int64_t>(split) * g.M * g.NG : static_cast<float*>(g.out);
    const bool accumulate = g.wpart == nullptr;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int m = m0 + wm * 64 + mt * 32 + (lane & 31);
      if (m >= g.M) continue;
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int n = n0 + wn * (BN / 2) + nt * 32 + 8 * g4 + 4 * h;
          if (n >= g.NG) continue;
          f32x4* dst = reinterpret_cast<f32x4*>(out + static_cast<int64_t>(m) * g.NG + n);
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = acc[nt][mt][4 * g4 + e];
          if (accumulate) v += *dst;
          *dst = v;
        }
    }
    return;
  }

  bf16* out = static_cast<bf16*>(g.out);
  float csum[NTN][4][4], csq[NTN][4][4];
#pragma unroll
  for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
      for (int e = 0; e < 4; ++e) csum[nt][g4][e] = csq[nt][g4][e] = 0.f;

  // Epilogue through LDS: lanes own one row x 4 columns of the accumulator
  // (8-byte pieces of many rows), so the tile is first written to an LDS
  // image and then stored row-contiguously, 16 B per lane (full 128-B lines).
  constexpr int ROWB = BN * 2 + 16;  // padded row: conflict-free 8-B writes
  unsigned char* ctile = smem;       // 128 x ROWB <= the staging buffers (free after the K loop)
  static_assert(BM * ROWB <= 2 * (IMG + IMGB), "epilogue tile exceeds LDS");
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int ml = wm * 64 + mt * 32 + (lane & 31);
    const bool mok = m0 + ml < g.M;
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const int nl = wn * (BN / 2) + nt * 32 + 8 * g4 + 4 * h;
        const int n = n0 + nl;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[nt][mt][4 * g4 + e];
        if (MODE == MODE_FWD) {
          if (g.bias && n < g.NG) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += bf2f(g.bias[n + e]);
          }
          if (g.act) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = conv_act(g.act, v[e]);
          }
        }
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
        if (mok && n < g.NG) {  // NG % 8 == 0: a 4-group is all in or all out
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float r = bf2f(o[e]);  // statistics of the stored (rounded) value
            csum[nt][g4][e] += r;
            csq[nt][g4][e] += r * r;
          }
        }
        *reinterpret_cast<bf16x4*>(ctile + ml * ROWB + nl * 2) = o;
      }
  }
  __syncthreads();
  {
    constexpr int CPR = BN / 8;  // 16-byte chunks per tile row
#pragma unroll
    for (int i = 0; i < BM * CPR / 256; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int ml = c / CPR, ch = c % CPR;
      const int m = m0 + ml, n = n0 + ch * 8;
      if (m >= g.M || n >= g.NG) continue;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(ctile + ml * ROWB + ch * 16);
      bf16* dst = out + (MODE == MODE_DGRAD ? dgrad_row(g, m) : static_cast<int64_t>(m)) * g.NG + n;
      if (MODE == MODE_DGRAD && g.beta != 0.f) {
        const bf16x8 old = *reinterpret_cast<const bf16x8*>(dst);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + g.beta * bf2f(old[e]));
      }
      *reinterpret_cast<bf16x8*>(dst) = v;
    }
  }
  if (MODE == MODE_FWD && g.stats) {
    // per-wave column partials (no atomics: a slot per (m tile, wave row));
    // reduce_rows folds them into the [2][K] statistics
    float* part = g.stats + static_cast<int64_t>(tm * 2 + wm) * 2 * g.NG;
#pragma unroll
    for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float s = csum[nt][g4][e], q = csq[nt][g4][e];
#pragma unroll
          for (int o = 1; o < 32; o <<= 1) {
            s += __shfl_xor(s, o, 64);
            q += __shfl_xor(q, o, 64);
          }
          const int n = n0 + wn * (BN / 2) + nt * 32 + 8 * g4 + 4 * h + e;
          if ((lane & 31) == 0 && n < g.NG) {
            part[n] = s;
            part[g.NG + n] = q;
          }
        }
  }
}

// out[j] (+)= sum_r ws[r][j] over rows [blockIdx.y*per, +per); with several
// row chunks each writes its partial row of `out` (a [chunks][W] scratch),
// summed by a second single-chunk pass — no atomics anywhere.
__global__ __launch_bounds__(256) void reduce_rows_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                          int rows, int64_t W, int rows_per_chunk, int accumulate) {
  const int64_t j = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) * 4;
  if (j >= W) return;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(rows, r0 + rows_per_chunk);
  float* o = out + static_cast<int64_t>(blockIdx.y) * W;
  if (j + 3 < W) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 8
    for (int r = r0; r < r1; ++r) s += *reinterpret_cast<const f32x4*>(ws + static_cast<int64_t>(r) * W + j);
    f32x4* d = reinterpret_cast<f32x4*>(o + j);
    *d = accumulate ? *d + s : s;
  } else {
    for (int e = 0; j + e < W; ++e) {
      float t = 0.f;
      for (int r = r0; r < r1; ++r) t += ws[static_cast<int64_t>(r) * W + j + e];
      o[j + e] = accumulate ? o[j + e] + t : t;
    }
  }
}

constexpr int kMaxChunks = 256;

// tmp: kMaxChunks * W floats (null: single pass)
void reduce_rows(const float* ws, float* out, int rows, int64_t W, int accumulate, float* tmp, hipStream_t st) {
  const int64_t cols = (W + 1023) / 1024;
  int chunks = 1;
  if (tmp && rows >= 64)
    chunks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>({rows / 64, kMaxChunks / 2, 2048 / cols})));
  const int per = (rows + chunks - 1) / chunks;
  chunks = (rows + per - 1) / per;
  if (chunks == 1) {
    hipLaunchKernelGGL(reduce_rows_kernel, dim3(static_cast<unsigned>(cols), 1), dim3(256), 0, st, ws, out, rows, W,
                       rows, accumulate);
    return;
  }
  hipLaunchKernelGGL(reduce_rows_kernel, dim3(static_cast<unsigned>(cols), chunks), dim3(256), 0, st, ws, tmp, rows,
                     W, per, 0);
  hipLaunchKernelGGL(reduce_rows_kernel, dim3(static_cast<unsigned>(cols), 1), dim3(256), 0, st,
                     static_cast<const float*>(tmp), out, chunks, W, chunks, accumulate);
}

}  // namespace

namespace {

ConvArgs make_args(const ConvShape& cs) {
  ConvArgs g{};
  g.N = cs.N; g.H = cs.H; g.W = cs.W; g.C = cs.C; g.K = cs.K; g.R = cs.R; g.S = cs.S;
  g.sh = cs.sh; g.sw = cs.sw; g.ph = cs.ph; g.pw = cs.pw; g.dh = cs.dh; g.dw = cs.dw;
  g.P = (cs.H + 2 * cs.ph - cs.dh * (cs.R - 1) - 1) / cs.sh + 1;
  g.Q = (cs.W + 2 * cs.pw - cs.dw * (cs.S - 1) - 1) / cs.sw + 1;
  return g;
}

void check_shape(const ConvShape& cs, const char* who) {
  if (cs.C % 8 || cs.K % 8) throw std::invalid_argument(std::string(who) + ": C and K must be multiples of 8");
  if (cs.N <= 0 || cs.H <= 0 || cs.W <= 0 || cs.R <= 0 || cs.S <= 0 || cs.sh <= 0 || cs.sw <= 0 || cs.dh <= 0 ||
      cs.dw <= 0 || cs.ph < 0 || cs.pw < 0)
    throw std::invalid_argument(std::string(who) + ": bad geometry");
  const int64_t P = (cs.H + 2 * cs.ph - cs.dh * (cs.R - 1) - 1) / cs.sh + 1;
  const int64_t Q = (cs.W + 2 * cs.pw - cs.dw * (cs.S - 1) - 1) / cs.sw + 1;
  if (P <= 0 || Q <= 0) throw std::invalid_argument(std::string(who) + ": empty output");
  if (static_cast<int64_t>(cs.N) * cs.H * cs.W * cs.C >= (int64_t(1) << 31) ||
      static_cast<int64_t>(cs.N) * P * Q * cs.K >= (int64_t(1) << 31) ||
      static_cast<int64_t>(cs.N) * P * Q >= (int64_t(1) << 31))
    throw std::invalid_argument(std::string(who) + ": tensor too large for 32-bit pixel indexing");
}

template <int MODE>
void launch(const ConvArgs& g, int bn, int blocks, hipStream_t st) {
  if (bn == 64) hipLaunchKernelGGL((conv_igemm_kernel<MODE, 64>), dim3(blocks), dim3(256), 0, st, g);
  else hipLaunchKernelGGL((conv_igemm_kernel<MODE, 128>), dim3(blocks), dim3(256), 0, st, g);
}

}  // namespace

int conv2d_stats_ws_floats(const ConvShape& cs) {
  ConvArgs g = make_args(cs);
  const int64_t M = static_cast<int64_t>(g.N) * g.P * g.Q;
  return static_cast<int>((((M + BM - 1) / BM) * 2 + kMaxChunks) * 2 * cs.K);
}

void conv2d_fwd(const ConvShape& cs, const void* x, const void* w, const void* bias, void* y, float* stats,
                float* stats_ws, int act, hipStream_t st) {
  check_shape(cs, "conv2d_fwd");
  if (stats && !stats_ws) throw std::invalid_argument("conv2d_fwd: statistics need a workspace");
  ConvArgs g = make_args(cs);
  g.x = static_cast<const bf16*>(x);
  g.w = static_cast<const bf16*>(w);
  g.bias = static_cast<const bf16*>(bias);
  g.out = y;
  g.stats = stats ? stats_ws : nullptr;
  g.act = act;
  g.M = g.N * g.P * g.Q;
  g.NG = g.K;
  g.KG = g.R * g.S * g.C;
  const int bn = g.NG <= 64 ? 64 : 128;
  const int gm = (g.M + BM - 1) / BM;
  const int blocks = gm * ((g.NG + bn - 1) / bn);
  launch<MODE_FWD>(g, bn, blocks, st);
  FFK_LAUNCH_CHECK("conv2d_fwd");
  if (stats) {
    const int64_t W = 2 * static_cast<int64_t>(g.NG);
    reduce_rows(stats_ws, stats, gm * 2, W, 0, stats_ws + static_cast<int64_t>(gm) * 2 * W, st);
    FFK_LAUNCH_CHECK("conv2d_fwd stats");
  }
}

void conv2d_dgrad(const ConvShape& cs, const void* dy, const void* w, void* dx, float beta, hipStream_t st) {
  check_shape(cs, "conv2d_dgrad");
  ConvArgs g = make_args(cs);
  g.dy = static_cast<const bf16*>(dy);
  g.w = static_cast<const bf16*>(w);
  g.out = dx;
  g.beta = beta;
  g.NG = g.C;
  const int bn = g.NG <= 64 ? 64 : 128;
  if ((g.sh > 1 || g.sw > 1) && g.dh == 1 && g.dw == 1) {
    // strided: one launch per output-parity class, each a dense implicit GEMM
    // over only the taps that reach it (no MFMA work on structural zeros)
    g.par = 1;
    for (int pch = 0; pch < g.sh; ++pch)
      for (int pcw = 0; pcw < g.sw; ++pcw) {
        g.pch = pch;
        g.pcw = pcw;
        g.Hc = (g.H - pch + g.sh - 1) / g.sh;
        g.Wc = (g.W - pcw + g.sw - 1) / g.sw;
        if (g.Hc <= 0 || g.Wc <= 0) continue;
        g.rf = (pch + g.ph) % g.sh;
        g.sf = (pcw + g.pw) % g.sw;
        g.nr = g.rf < g.R ? (g.R - 1 - g.rf) / g.sh + 1 : 0;
        g.ns = g.sf < g.S ? (g.S - 1 - g.sf) / g.sw + 1 : 0;
        g.M = g.N * g.Hc * g.Wc;
        g.KG = g.nr * g.ns * g.K;
        const int blocks = ((g.M + BM - 1) / BM) * ((g.NG + bn - 1) / bn);
        launch<MODE_DGRAD>(g, bn, blocks, st);
      }
    FFK_LAUNCH_CHECK("conv2d_dgrad");
    return;
  }
  g.M = g.N * g.H * g.W;
  g.KG = g.R * g.S * g.K;
  const int blocks = ((g.M + BM - 1) / BM) * ((g.NG + bn - 1) / bn);
  launch<MODE_DGRAD>(g, bn, blocks, st);
  FFK_LAUNCH_CHECK("conv2d_dgrad");
}

namespace {
struct WgradPlan {
  int bn, tiles, splits, kt_per_split;
};
WgradPlan wgrad_plan(const ConvShape& cs, int splits) {
  ConvArgs g = make_args(cs);
  const int M = cs.K, NG = cs.R * cs.S * cs.C;
  const int64_t KG = static_cast<int64_t>(g.N) * g.P * g.Q;
  WgradPlan p;
  p.bn = NG <= 64 ? 64 : 128;
  p.tiles = ((M + BM - 1) / BM) * ((NG + p.bn - 1) / p.bn);
  const int nk = static_cast<int>((KG + BK - 1) / BK);
  if (splits <= 0) {
    // ~2048 blocks (8 per CU), >= 8 K-tiles per split, slabs <= 256 MiB
    splits = (2048 + p.tiles - 1) / p.tiles;
    splits = std::min(splits, std::max(1, nk / 8));
    const int64_t slab = static_cast<int64_t>(M) * NG * 4;
    splits = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(splits, (int64_t(256) << 20) / slab)));
  }
  splits = std::max(1, std::min(splits, nk));
  p.kt_per_split = (nk + splits - 1) / splits;
  p.splits = (nk + p.kt_per_split - 1) / p.kt_per_split;
  return p;
}
}  // namespace

int64_t conv2d_wgrad_ws_floats(const ConvShape& cs, int splits) {
  const WgradPlan p = wgrad_plan(cs, splits);
  const int64_t W = static_cast<int64_t>(cs.K) * cs.R * cs.S * cs.C;
  if (p.splits <= 1) return 0;
  // slabs + the two-pass reduce scratch when there are many slabs
  return static_cast<int64_t>(p.splits) * W + (p.splits >= 64 ? kMaxChunks * W : 0);
}

void conv2d_wgrad(const ConvShape& cs, const void* x, const void* dy, float* dw, float* ws, int splits,
                  hipStream_t st) {
  check_shape(cs, "conv2d_wgrad");
  const WgradPlan p = wgrad_plan(cs, splits);
  if (p.splits > 1 && !ws) throw std::invalid_argument("conv2d_wgrad: split-K needs a workspace");
  ConvArgs g = make_args(cs);
  g.x = static_cast<const bf16*>(x);
  g.dy = static_cast<const bf16*>(dy);
  g.out = dw;
  g.wpart = p.splits > 1 ? ws : nullptr;
  g.M = g.K;
  g.NG = g.R * g.S * g.C;
  g.KG = g.N * g.P * g.Q;
  g.kt_per_split = p.kt_per_split;
  launch<MODE_WGRAD>(g, p.bn, p.tiles * p.splits, st);
  FFK_LAUNCH_CHECK("conv2d_wgrad");
  if (p.splits > 1) {
    const int64_t W = static_cast<int64_t>(g.M) * g.NG;
    reduce_rows(ws, dw, p.splits, W, 1, p.splits >= 64 ? ws + static_cast<int64_t>(p.splits) * W : nullptr, st);
    FFK_LAUNCH_CHECK("conv2d_wgrad reduce");
  }
}

}  // namespace ffk
