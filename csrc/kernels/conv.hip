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

// n / d for n < 2^31 as (umulhi(n, m) + n) >> l, l = ceil(log2 d),
// m = floor(2^32 (2^l - d) / d) + 1 (division by invariant integers)
struct FastDiv {
  unsigned m;
  int l;
};
inline FastDiv make_fdiv(unsigned d) {
  int l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t m = (((1ull << l) - d) << 32) / d + 1;
  return FastDiv{static_cast<unsigned>(m), l};
}

struct ConvArgs {
  const bf16* x;    // FWD/WGRAD input  [N][H][W][C]
  const bf16* w;    // FWD/DGRAD weight [K][R][S][C]
  const bf16* dy;   // DGRAD/WGRAD      [N][P][Q][K]
  void* out;        // FWD y [N][P][Q][K] bf16 | DGRAD dx [N][H][W][C] bf16 | WGRAD dw [K][R][S][C] f32
  const bf16* bias; // FWD only
  float* stats;     // FWD only: per-wave partials [gm*2][2][K] (sum, sum of squares)
  float* wpart;     // WGRAD split-K partial slabs [splits][K][R*S*C] (null: splits == 1)
  int N, H, W, C, K, R, S, P, Q;   // C / K: channels of one (super-)group
  int ldx, ldk;     // pixel strides (channel counts) of X / dX and of Y / dY
  int sh, sw, ph, pw, dh, dw;
  int M, NG, KG;    // GEMM sizes
  int act;
  float beta;       // DGRAD: dx = result + beta * dx
  int kt_per_split; // WGRAD split-K
  // DGRAD parity class (strided convs): rows are the input pixels with
  // h % sh == pch, w % sw == pcw (Hc x Wc per image); the K axis runs only over
  // the taps r = rf + i*sh (i < nr), s = sf + j*sw (j < ns) that reach them.
  int par, pch, pcw, Hc, Wc, rf, sf, nr, ns;
  // magic divisors of the loaders and the operands' byte sizes (buffer range)
  FastDiv fC, fS, fK, fQ, fP, fW, fH, fWc, fHc, fns, fsh, fsw;
  unsigned bx, bw, bdy;
  // DGRAD of a convolution fed by a BatchNorm (+ReLU): the epilogue also
  // reduces that BN's backward sums over the stored gradient g (masked by the
  // forward's ReLU, recomputed from the BN input): sum g and sum g * xhat,
  // one partial row per M tile into `stats` (bn_reduce's pass then skipped)
  const bf16* bnx;            // BN input [N][H][W][C] (null: no BN sums)
  const float* bnmean;        // [C]
  const float* bnrstd;        // [C]
  const float* bnss;          // [2][C] scale, shift (null: no ReLU mask)
};

// DGRAD output row of local row m (parity classes scatter to the full image)
__device__ __forceinline__ int64_t dgrad_row(const ConvArgs& g, int m) {
  if (!g.par) return m;
  const int ww = m % g.Wc, t = m / g.Wc, hh = t % g.Hc, n = t / g.Hc;
  return (static_cast<int64_t>(n) * g.H + hh * g.sh + g.pch) * g.W + ww * g.sw + g.pcw;
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

// Branch-free gathers: every 16-B chunk is one buffer_load_dwordx4 whose
// offset is replaced by the tensor's byte size when the chunk is padding or
// past an edge (the buffer range check returns zeros), so the loaders carry
// no exec-mask branches; 32-bit offsets (check_shape bounds every tensor
// below 2^31 elements) and host-computed magic divisors (FastDiv) replace the
// 64-bit multiply-adds and integer divisions of the per-chunk address math.
__device__ __forceinline__ unsigned fdiv(unsigned n, FastDiv f) { return (__umulhi(n, f.m) + n) >> f.l; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t conv_rsrc(const bf16* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(p), static_cast<short>(0), bytes, 0x00020000);
}
__device__ __forceinline__ bf16x8 bld8(__amdgpu_buffer_rsrc_t r, int eoff, bool ok, unsigned oob) {
  const unsigned off = ok ? static_cast<unsigned>(eoff) * 2u : oob;
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// (r, s) of tap index rs of the DGRAD K axis
__device__ __forceinline__ void tap_of_f(const ConvArgs& g, int rs, int& r, int& s) {
  if (g.par) {
    const int i = static_cast<int>(fdiv(static_cast<unsigned>(rs), g.fns)), j = rs - i * g.ns;
    r = g.rf + i * g.sh;
    s = g.sf + j * g.sw;
  } else {
    r = static_cast<int>(fdiv(static_cast<unsigned>(rs), g.fS));
    s = rs - r * g.S;
  }
}

// ---------------------------------------------------------------------------
// A operand, K-contiguous image [128 rows = m][64 k], 4 chunks per thread.
// FWD: m = output pixel (n,p,q), k = (r,s,c).  DGRAD: m = input pixel (n,h,w),
// k = (r,s,kout).  The pixel decode happens once; the thread's tap (its k =
// k0 + 8 (tid & 7)) advances by 64 per K-tile without a division.
template <int MODE>
struct AGather {
  bf16x8 reg[4];
  int pix[4];       // FWD: element offset of x[n][ya][xa][0] (may be negative); DGRAD: of dy[n][0][0][0]
  int ya[4], xa[4]; // FWD: p*sh-ph, q*sw-pw ; DGRAD: h+ph, w+pw ; -2^30 = row past M
  int k, cc, r, s, rs;   // the thread's K index and its (channel, tap) decode

  __device__ __forceinline__ void init(const ConvArgs& g, int m0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + (threadIdx.x >> 3) + 32 * i;
      if (m >= g.M) {
        ya[i] = -0x3fffffff;
        xa[i] = 0;
        pix[i] = 0;
        continue;
      }
      if (MODE == MODE_FWD) {
        const int t = static_cast<int>(fdiv(static_cast<unsigned>(m), g.fQ)), q = m - t * g.Q;
        const int n = static_cast<int>(fdiv(static_cast<unsigned>(t), g.fP)), p = t - n * g.P;
        ya[i] = p * g.sh - g.ph;
        xa[i] = q * g.sw - g.pw;
        pix[i] = ((n * g.H + ya[i]) * g.W + xa[i]) * g.ldx;
      } else {
        int w, h, n;
        if (g.par) {
          const int t = static_cast<int>(fdiv(static_cast<unsigned>(m), g.fWc)), ww = m - t * g.Wc;
          n = static_cast<int>(fdiv(static_cast<unsigned>(t), g.fHc));
          const int hh = t - n * g.Hc;
          h = hh * g.sh + g.pch;
          w = ww * g.sw + g.pcw;
        } else {
          const int t = static_cast<int>(fdiv(static_cast<unsigned>(m), g.fW));
          w = m - t * g.W;
          n = static_cast<int>(fdiv(static_cast<unsigned>(t), g.fH));
          h = t - n * g.H;
        }
        ya[i] = h + g.ph;
        xa[i] = w + g.pw;
        pix[i] = n * g.P * g.Q * g.ldk;
      }
    }
    k = (threadIdx.x & 7) * 8;   // K-tile 0 (FWD / DGRAD never split K)
    const int CC = MODE == MODE_FWD ? g.C : g.K;
    const FastDiv fCC = MODE == MODE_FWD ? g.fC : g.fK;
    rs = static_cast<int>(fdiv(static_cast<unsigned>(k), fCC));
    cc = k - rs * CC;
    if (MODE == MODE_FWD) {
      r = static_cast<int>(fdiv(static_cast<unsigned>(rs), g.fS));
      s = rs - r * g.S;
    } else {
      tap_of_f(g, rs, r, s);
    }
  }
  // load the current K-tile's chunks, then step the tap to the next K-tile
  __device__ __forceinline__ void load(const ConvArgs& g, __amdgpu_buffer_rsrc_t rsrc, unsigned oob) {
    const bool kok = k < g.KG;
    if (MODE == MODE_FWD) {
      const int rr = r * g.dh, ss = s * g.dw;
      const int delta = (rr * g.W + ss) * g.ldx + cc;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        // bitwise & (no short-circuit): hipcc otherwise branches on kok around the
        // loads and serialises them with vmcnt(0) waits on the reused registers
        const bool ok = kok & (static_cast<unsigned>(ya[i] + rr) < static_cast<unsigned>(g.H)) &
                        (static_cast<unsigned>(xa[i] + ss) < static_cast<unsigned>(g.W));
        reg[i] = bld8(rsrc, pix[i] + delta, ok, oob);
      }
    } else {
      const int rr = r * g.dh, ss = s * g.dw;
      const bool unit = g.sh == 1 && g.sw == 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int yn = ya[i] - rr, xn = xa[i] - ss;
        int oh = yn, ow = xn;
        bool ok = kok & (yn >= 0) & (xn >= 0);
        if (!unit) {   // strided: only the parity class's taps reach these rows
          oh = static_cast<int>(fdiv(static_cast<unsigned>(max(yn, 0)), g.fsh));
          ow = static_cast<int>(fdiv(static_cast<unsigned>(max(xn, 0)), g.fsw));
          ok = ok & (yn == oh * g.sh) & (xn == ow * g.sw);
        }
        ok = ok & (oh < g.P) & (ow < g.Q);
        reg[i] = bld8(rsrc, pix[i] + (oh * g.Q + ow) * g.ldk + cc, ok, oob);
      }
    }
    // next K-tile: k += 64 (channel counts are multiples of 8: C = 8 wraps
    // eight times, C >= 64 at most once)
    const int CC = MODE == MODE_FWD ? g.C : g.K;
    k += BK;
    cc += BK;
    while (cc >= CC) {
      cc -= CC;
      ++rs;
      if (MODE == MODE_FWD) {
        if (++s == g.S) {
          s = 0;
          ++r;
        }
      }
    }
    if (MODE == MODE_DGRAD) tap_of_f(g, rs, r, s);
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
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rsrc, unsigned oob, int ld, int outer0, int n_outer,
                                       int k0, int K) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = threadIdx.x + 256 * i, r = c >> 3, ch = c & 7;
      const bool ok = (outer0 + r < n_outer) & (k0 + ch * 8 < K);
      reg[i] = bld8(rsrc, (outer0 + r) * ld + k0 + ch * 8, ok, oob);
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
  // KIND 1: per-chunk (kout, tap index) of the chunk's K row, stepped by 64 per tile
  int kout_[NL], rsi_[NL];

  __device__ __forceinline__ void init(const ConvArgs& g, int outer0) {
    if (KIND == 2) {
      const int n = outer0 + (threadIdx.x % CPR) * 8;
      tok_ = n < g.NG;
      const int rs = static_cast<int>(fdiv(static_cast<unsigned>(n), g.fC));
      tc_ = n - rs * g.C;
      tr_ = static_cast<int>(fdiv(static_cast<unsigned>(rs), g.fS));
      ts_ = rs - tr_ * g.S;
    }
    if (KIND == 1) {   // K-tile 0 (DGRAD never splits K)
#pragma unroll
      for (int i = 0; i < NL; ++i) {
        const int k = (threadIdx.x + 256 * i) / CPR;
        rsi_[i] = static_cast<int>(fdiv(static_cast<unsigned>(k), g.fK));
        kout_[i] = k - rsi_[i] * g.K;
      }
    }
  }
  __device__ __forceinline__ void load(const ConvArgs& g, __amdgpu_buffer_rsrc_t rsrc, unsigned oob, int ld,
                                       int outer0, int n_outer, int k0, int K) {
#pragma unroll
    for (int i = 0; i < NL; ++i) {
      const int c = threadIdx.x + 256 * i, r = c / CPR, ch = c % CPR;
      const int k = k0 + r, o = outer0 + ch * 8;
      bool ok = (k < K) & (o < n_outer);
      int off;
      if (KIND == 0) {
        off = k * ld + o;
      } else if (KIND == 1) {
        int rr, s;
        tap_of_f(g, rsi_[i], rr, s);
        off = ((kout_[i] * g.R + rr) * g.S + s) * g.C + o;
        kout_[i] += BK;   // next K-tile (K >= 8: wraps at most 8 times)
        while (kout_[i] >= g.K) {
          kout_[i] -= g.K;
          ++rsi_[i];
        }
      } else {
        const int t = static_cast<int>(fdiv(static_cast<unsigned>(k), g.fQ)), q = k - t * g.Q;
        const int n = static_cast<int>(fdiv(static_cast<unsigned>(t), g.fP)), p = t - n * g.P;
        const int ih = p * g.sh - g.ph + tr_ * g.dh, iw = q * g.sw - g.pw + ts_ * g.dw;
        ok = ok & tok_ & (static_cast<unsigned>(ih) < static_cast<unsigned>(g.H)) &
             (static_cast<unsigned>(iw) < static_cast<unsigned>(g.W));
        off = ((n * g.H + ih) * g.W + iw) * g.ldx + tc_;
      }
      reg[i] = bld8(rsrc, off, ok, oob);
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

  // grouped convolutions: blockIdx.z = super-group (a block-diagonal dense
  // conv over g.C input / g.K output channels at channel offsets cx0 / ck0
  // of the full tensors, its expanded weight the z-th [K][R][S][C] block)
  const int z = blockIdx.z;
  const int cx0 = z * g.C, ck0 = z * g.K;
  const int64_t wz = static_cast<int64_t>(z) * g.K * g.R * g.S * g.C;

  // operand stagers
  AGather<MODE_FWD> afw;
  AGather<MODE_DGRAD> adg;
  ColStager<128, 0> awg;  // WGRAD A: dY [pix][K], outer = kout (M side)
  RowStager<BN> bfw;
  ColStager<BN, 1> bdg;
  ColStager<BN, 2> bwg;

  // the buffer ranges start at the super-group's channel offset: a chunk
  // past the tensor's end still reads the range check's zeros
  const unsigned bxz = g.bx - 2u * cx0, bdyz = g.bdy - 2u * ck0;
  const __amdgpu_buffer_rsrc_t rx = conv_rsrc(g.x + cx0, bxz), rw = conv_rsrc(g.w + wz, g.bw),
                               rdy = conv_rsrc(g.dy + ck0, bdyz);
  auto load = [&](int kt) {
    const int k0 = kt * BK;
    if (MODE == MODE_FWD) {
      afw.load(g, rx, bxz);
      bfw.load(rw, g.bw, g.KG, n0, g.NG, k0, g.KG);
    } else if (MODE == MODE_DGRAD) {
      adg.load(g, rdy, bdyz);
      bdg.load(g, rw, g.bw, 0, n0, g.NG, k0, g.KG);
    } else {
      awg.load(g, rdy, bdyz, g.ldk, m0, g.M, k0, g.KG);
      bwg.load(g, rx, bxz, 0, n0, g.NG, k0, g.KG);
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
  if (MODE == MODE_DGRAD) {
    adg.init(g, m0);
    bdg.init(g, n0);
  }
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
    // every fragment of the K-tile requested before the first MFMA, so the
    // LDS latency of k-steps 1-3 hides under the earlier k-steps' MFMAs (one
    // lgkmcnt wait per k-step group instead of an exposed read per k-step)
    bf16x8 bf[BK / 16][NTN], af[BK / 16][2];
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
#pragma unroll
      for (int t = 0; t < NTN; ++t) {
        if (MODE == MODE_FWD) bf[ks][t] = row_frag<128>(Bi, wn * (BN / 2) + t * 32, ks * 16, lane);
        else bf[ks][t] = tr_frag_nat<BN * 2>(Bi, ks * 16, wn * (BN / 2) + t * 32, lane);
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (MODE == MODE_WGRAD) af[ks][t] = tr_frag_nat<256>(Ai, ks * 16, wm * 64 + t * 32, lane);
        else af[ks][t] = row_frag<128>(Ai, wm * 64 + t * 32, ks * 16, lane);
      }
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead (hipcc re-sinks them to save registers)
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks)
#pragma unroll
      for (int nt = 0; nt < NTN; ++nt)
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) acc[nt][mt] = mfma32(bf[ks][nt], af[ks][mt], acc[nt][mt]);
    __builtin_amdgcn_sched_barrier(0);
    if (has_next) store(smem + ((kt + 1 - kt0) & 1) * (IMG + IMGB));
    __syncthreads();
  }

  // ---- epilogue: acc[nt][mt] holds C^T; lane&31 = m row, registers = 4 n columns
  const int h = lane >> 5;
  if (MODE == MODE_WGRAD) {
    // one writer per element: split 0 of a single-split launch accumulates into
    // dW directly; otherwise this split's slab (summed by reduce_rows)
    const int64_t slab = static_cast<int64_t>(g.M) * g.NG;
    float* out = g.wpart ? g.wpart + (static_cast<int64_t>(split) * gridDim.z + z) * slab
                         : static_cast<float*>(g.out) + z * slab;
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

  // FWD writes output channels [ck0, ck0 + K) of Y, DGRAD input channels
  // [cx0, cx0 + C) of dX
  const int coff = MODE == MODE_FWD ? ck0 : cx0;
  const int ldo = MODE == MODE_FWD ? g.ldk : g.ldx;
  bf16* out = static_cast<bf16*>(g.out) + coff;

  // Epilogue through LDS: lanes own one row x 4 columns of the accumulator
  // (8-byte pieces of many rows), so the tile is first written to an LDS
  // image and then stored row-contiguously, 16 B per lane (full 128-B lines).
  constexpr int ROWB = BN * 2 + 16;  // padded row: conflict-free 8-B writes
  unsigned char* ctile = smem;       // 128 x ROWB <= the staging buffers (free after the K loop)
  static_assert(BM * ROWB <= 2 * (IMG + IMGB), "epilogue tile exceeds LDS");
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int ml = wm * 64 + mt * 32 + (lane & 31);
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
            for (int e = 0; e < 4; ++e) v[e] += bf2f(g.bias[ck0 + n + e]);
          }
          if (g.act) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = conv_act(g.act, v[e]);
          }
        }
        bf16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
        *reinterpret_cast<bf16x4*>(ctile + ml * ROWB + nl * 2) = o;
      }
  }
  constexpr int CPR = BN / 8;  // 16-byte chunks per tile row
  constexpr int NCH = BM * CPR / 256;   // chunks per thread
  const bool want_stats = (MODE == MODE_FWD || MODE == MODE_DGRAD) && g.stats != nullptr;
  // BN backward sums (DGRAD): a thread's chunks all sit in channel group
  // tid % CPR; its BN parameters and the BN input under its chunks are
  // requested here, before the barrier, so their latency hides behind it
  float bmu[8], brs[8], bsc[8], bsh[8];
  bf16x8 bxr[MODE == MODE_DGRAD ? NCH : 1];
  if (MODE == MODE_DGRAD && want_stats) {
    const int n = n0 + (threadIdx.x % CPR) * 8;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int m = m0 + (threadIdx.x + 256 * i) / CPR;
      if (m < g.M && n < g.NG) bxr[i] = *reinterpret_cast<const bf16x8*>(g.bnx + static_cast<int64_t>(m) * ldo + coff + n);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool ok = n + e < g.NG;
      bmu[e] = ok ? g.bnmean[n + e] : 0.f;
      brs[e] = ok ? g.bnrstd[n + e] : 0.f;
      bsc[e] = ok && g.bnss ? g.bnss[n + e] : 0.f;
      bsh[e] = ok && g.bnss ? g.bnss[g.NG + n + e] : 1.f;   // no mask: x*0 + 1 > 0
    }
  }
  __syncthreads();
  // Row-contiguous stores; a thread's chunks are one 8-column group (ch =
  // tid % CPR) of every (256 / CPR)-th row, so the BN statistics of the stored
  // (rounded) values accumulate per thread here, then reduce over the lanes of
  // that group (xor over lane bits >= log2 CPR) and over the 4 waves in LDS
  // into one partial row per M tile (reduce_rows folds the tiles): no
  // 320-shuffle column reduction of accumulator layouts.
  float cs[8], cq[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = cq[e] = 0.f;
#pragma unroll
  for (int i = 0; i < BM * CPR / 256; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int ml = c / CPR, ch = c % CPR;
    const int m = m0 + ml, n = n0 + ch * 8;
    if (m >= g.M || n >= g.NG) continue;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(ctile + ml * ROWB + ch * 16);
    bf16* dst = out + (MODE == MODE_DGRAD ? dgrad_row(g, m) : static_cast<int64_t>(m)) * ldo + n;
    if (MODE == MODE_DGRAD && g.beta != 0.f) {
      const bf16x8 old = *reinterpret_cast<const bf16x8*>(dst);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = f2bf(bf2f(v[e]) + g.beta * bf2f(old[e]));
    }
    *reinterpret_cast<bf16x8*>(dst) = v;
    if (MODE == MODE_DGRAD && want_stats) {   // beta == 0 and no parity classes (host checked)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xe = bf2f(bxr[MODE == MODE_DGRAD ? i : 0][e]);
        const float gr = xe * bsc[e] + bsh[e] > 0.f ? bf2f(v[e]) : 0.f;
        cs[e] += gr;
        cq[e] += gr * (xe - bmu[e]) * brs[e];
      }
    }
    if (MODE == MODE_FWD && want_stats) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float r = bf2f(v[e]);
        cs[e] += r;
        cq[e] += r * r;
      }
    }
  }
  if (want_stats) {
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        cs[e] += __shfl_xor(cs[e], o, 64);
        cq[e] += __shfl_xor(cq[e], o, 64);
      }
    __syncthreads();   // every wave is done reading the C tile: reuse its LDS
    float* red = reinterpret_cast<float*>(smem);   // [4 waves][CPR groups][16]
    if (lane < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * CPR + lane) * 16 + e] = cs[e];
        red[(wave * CPR + lane) * 16 + 8 + e] = cq[e];
      }
    }
    __syncthreads();
    if (threadIdx.x < CPR * 16) {
      const int chv = threadIdx.x >> 4, vv = threadIdx.x & 15;
      const float t = red[chv * 16 + vv] + red[(CPR + chv) * 16 + vv] + red[(2 * CPR + chv) * 16 + vv] +
                      red[(3 * CPR + chv) * 16 + vv];
      const int n = n0 + chv * 8 + (vv & 7);
      float* part = g.stats + static_cast<int64_t>(tm) * 2 * ldo;   // one partial row per M tile
      if (n < g.NG) part[(vv < 8 ? 0 : ldo) + coff + n] = t;
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
  g.ldx = cs.C;
  g.ldk = cs.K;
  g.sh = cs.sh; g.sw = cs.sw; g.ph = cs.ph; g.pw = cs.pw; g.dh = cs.dh; g.dw = cs.dw;
  g.P = (cs.H + 2 * cs.ph - cs.dh * (cs.R - 1) - 1) / cs.sh + 1;
  g.Q = (cs.W + 2 * cs.pw - cs.dw * (cs.S - 1) - 1) / cs.sw + 1;
  g.fC = make_fdiv(cs.C);
  g.fS = make_fdiv(cs.S);
  g.fK = make_fdiv(cs.K);
  g.fQ = make_fdiv(g.Q);
  g.fP = make_fdiv(g.P);
  g.fW = make_fdiv(cs.W);
  g.fH = make_fdiv(cs.H);
  g.fsh = make_fdiv(cs.sh);
  g.fsw = make_fdiv(cs.sw);
  g.fWc = g.fHc = g.fns = make_fdiv(1);
  g.bx = static_cast<unsigned>(static_cast<int64_t>(cs.N) * cs.H * cs.W * cs.C * 2);
  g.bdy = static_cast<unsigned>(static_cast<int64_t>(cs.N) * g.P * g.Q * cs.K * 2);
  g.bw = static_cast<unsigned>(static_cast<int64_t>(cs.K) * cs.R * cs.S * cs.C * 2);
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
void launch(const ConvArgs& g, int bn, int blocks, hipStream_t st, int zgroups = 1) {
  if (bn == 64) hipLaunchKernelGGL((conv_igemm_kernel<MODE, 64>), dim3(blocks, 1, zgroups), dim3(256), 0, st, g);
  else hipLaunchKernelGGL((conv_igemm_kernel<MODE, 128>), dim3(blocks, 1, zgroups), dim3(256), 0, st, g);
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
    reduce_rows(stats_ws, stats, gm, W, 0, stats_ws + static_cast<int64_t>(gm) * W, st);
    FFK_LAUNCH_CHECK("conv2d_fwd stats");
  }
}

void conv2d_dgrad(const ConvShape& cs, const void* dy, const void* w, void* dx, float beta, hipStream_t st,
                  const ConvBnBwd* bn_sums) {
  check_shape(cs, "conv2d_dgrad");
  ConvArgs g = make_args(cs);
  g.dy = static_cast<const bf16*>(dy);
  g.w = static_cast<const bf16*>(w);
  g.out = dx;
  g.beta = beta;
  g.NG = g.C;
  const int bn = g.NG <= 64 ? 64 : 128;
  const bool strided = (g.sh > 1 || g.sw > 1) && g.dh == 1 && g.dw == 1;
  if (bn_sums) {
    if (strided || beta != 0.f || !bn_sums->x || !bn_sums->mean || !bn_sums->rstd || !bn_sums->sums ||
        !bn_sums->ws)
      throw std::invalid_argument("conv2d_dgrad: BN sums need a stride-1 dgrad without accumulation");
    g.bnx = static_cast<const bf16*>(bn_sums->x);
    g.bnmean = bn_sums->mean;
    g.bnrstd = bn_sums->rstd;
    g.bnss = bn_sums->scale_shift;
    g.stats = bn_sums->ws;
  }
  if (strided) {
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
        g.fWc = make_fdiv(g.Wc);
        g.fHc = make_fdiv(g.Hc);
        g.fns = make_fdiv(std::max(g.ns, 1));
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
  const int gm = (g.M + BM - 1) / BM;
  const int blocks = gm * ((g.NG + bn - 1) / bn);
  launch<MODE_DGRAD>(g, bn, blocks, st);
  FFK_LAUNCH_CHECK("conv2d_dgrad");
  if (bn_sums) {
    const int64_t W = 2 * static_cast<int64_t>(g.NG);
    reduce_rows(bn_sums->ws, bn_sums->sums, gm, W, 0, bn_sums->ws + static_cast<int64_t>(gm) * W, st);
    FFK_LAUNCH_CHECK("conv2d_dgrad bn sums");
  }
}

int conv2d_dgrad_bn_ws_floats(const ConvShape& cs) {
  const int64_t M = static_cast<int64_t>(cs.N) * cs.H * cs.W;
  return static_cast<int>((((M + BM - 1) / BM) + kMaxChunks) * 2 * cs.C);
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


// ---------------------------------------------------------------------------
// Grouped convolutions (ResNeXt) on the bf16 MFMA kernels above.  `gps`
// consecutive groups form a super-group of Cs = gps * C/groups input and
// Ks = gps * K/groups output channels, run as ONE dense implicit GEMM over a
// block-diagonal expanded weight [Z][Ks][R][S][Cs] (zeros between the
// groups), blockIdx.z = super-group.  gps is the smallest divisor of
// `groups` with Cs, Ks multiples of 8 and Ks >= 64 (one 64-wide MFMA tile):
// ResNeXt-50 32x4d's Cg = 4 runs 16 groups per super-group.  The MFMAs on the
// zero blocks (gps x the useful work) are cheap next to what these layers
// move: the 3x3 grouped convs carry 1/8 of a dense 3x3's FLOPs per byte.
// Parity: conv_2d_kernels.cu:194-196 (cudnnSetConvolutionGroupCount, tensor
// op math), :279 / :346 / :362.
namespace {
struct GroupPlan {
  int Z, gps, Cs, Ks, Cg, Kg;
};
GroupPlan group_plan(const ConvShape& cs, int groups) {
  if (groups <= 0 || cs.C % groups || cs.K % groups)
    throw std::invalid_argument("conv2d_grouped: groups must divide C and K");
  GroupPlan p{};
  p.Cg = cs.C / groups;
  p.Kg = cs.K / groups;
  for (int gps = 1; gps <= groups; ++gps) {
    if (groups % gps) continue;
    const int Cs = gps * p.Cg, Ks = gps * p.Kg;
    if (Cs % 8 || Ks % 8) continue;
    if (Ks < 64 && gps != groups) continue;
    p.gps = gps;
    p.Cs = Cs;
    p.Ks = Ks;
    p.Z = groups / gps;
    return p;
  }
  throw std::invalid_argument("conv2d_grouped: no super-group with channel counts that are multiples of 8");
}
// the per-super-group dense shape; pixel strides are the full channel counts
ConvArgs grouped_args(const ConvShape& cs, const GroupPlan& p) {
  ConvShape s = cs;
  s.C = p.Cs;
  s.K = p.Ks;
  ConvArgs g = make_args(s);
  g.ldx = cs.C;
  g.ldk = cs.K;
  g.bx = static_cast<unsigned>(static_cast<int64_t>(cs.N) * cs.H * cs.W * cs.C * 2);
  g.bdy = static_cast<unsigned>(static_cast<int64_t>(cs.N) * g.P * g.Q * cs.K * 2);
  return g;
}

// wexp[k][rs][cl] = w[k][rs][cl - (kl / Kg) * Cg] on the diagonal block, else 0
__global__ __launch_bounds__(256) void group_expand_kernel(const bf16* __restrict__ w, bf16* __restrict__ wexp,
                                                           int64_t n, int RS, int Cs, int Ks, int Cg, int Kg) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int cl = static_cast<int>(i % Cs);
  const int64_t t = i / Cs;   // k * RS + rs
  const int rs = static_cast<int>(t % RS);
  const int64_t k = t / RS;
  const int kl = static_cast<int>(k % Ks);
  const int c0 = (kl / Kg) * Cg;
  wexp[i] = (cl >= c0 && cl < c0 + Cg) ? w[(k * RS + rs) * Cg + (cl - c0)] : static_cast<bf16>(0.f);
}
// dw[k][rs][c] += dwexp[k][rs][(kl / Kg) * Cg + c]
__global__ __launch_bounds__(256) void group_compress_kernel(const float* __restrict__ dwexp, float* __restrict__ dw,
                                                             int64_t n, int RS, int Cs, int Ks, int Cg, int Kg) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= n) return;
  const int c = static_cast<int>(i % Cg);
  const int64_t t = i / Cg;
  const int rs = static_cast<int>(t % RS);
  const int64_t k = t / RS;
  const int kl = static_cast<int>(k % Ks);
  dw[i] += dwexp[(k * RS + rs) * Cs + (kl / Kg) * Cg + c];
}
}  // namespace

int64_t conv2d_grouped_wexp_elems(const ConvShape& cs, int groups) {
  const GroupPlan p = group_plan(cs, groups);
  return static_cast<int64_t>(cs.K) * cs.R * cs.S * p.Cs;
}

void conv2d_grouped_expand(const ConvShape& cs, int groups, const void* w, void* wexp, hipStream_t st) {
  const GroupPlan p = group_plan(cs, groups);
  const int64_t n = static_cast<int64_t>(cs.K) * cs.R * cs.S * p.Cs;
  hipLaunchKernelGGL(group_expand_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, st,
                     static_cast<const bf16*>(w), static_cast<bf16*>(wexp), n, cs.R * cs.S, p.Cs, p.Ks, p.Cg, p.Kg);
  FFK_LAUNCH_CHECK("conv2d_grouped_expand");
}

void conv2d_grouped_fwd(const ConvShape& cs, int groups, const void* x, const void* wexp, const void* bias, void* y,
                        float* stats, float* stats_ws, int act, hipStream_t st) {
  check_shape(cs, "conv2d_grouped_fwd");
  if (stats && !stats_ws) throw std::invalid_argument("conv2d_grouped_fwd: statistics need a workspace");
  const GroupPlan p = group_plan(cs, groups);
  ConvArgs g = grouped_args(cs, p);
  g.x = static_cast<const bf16*>(x);
  g.w = static_cast<const bf16*>(wexp);
  g.bias = static_cast<const bf16*>(bias);
  g.out = y;
  g.stats = stats ? stats_ws : nullptr;
  g.act = act;
  g.M = g.N * g.P * g.Q;
  g.NG = g.K;
  g.KG = g.R * g.S * g.C;
  const int bn = g.NG <= 64 ? 64 : 128;
  const int gm = (g.M + BM - 1) / BM;
  launch<MODE_FWD>(g, bn, gm * ((g.NG + bn - 1) / bn), st, p.Z);
  FFK_LAUNCH_CHECK("conv2d_grouped_fwd");
  if (stats) {
    const int64_t W = 2 * static_cast<int64_t>(cs.K);
    reduce_rows(stats_ws, stats, gm, W, 0, stats_ws + static_cast<int64_t>(gm) * W, st);
    FFK_LAUNCH_CHECK("conv2d_grouped_fwd stats");
  }
}

void conv2d_grouped_dgrad(const ConvShape& cs, int groups, const void* dy, const void* wexp, void* dx, float beta,
                          hipStream_t st) {
  check_shape(cs, "conv2d_grouped_dgrad");
  const GroupPlan p = group_plan(cs, groups);
  ConvArgs g = grouped_args(cs, p);
  g.dy = static_cast<const bf16*>(dy);
  g.w = static_cast<const bf16*>(wexp);
  g.out = dx;
  g.beta = beta;
  g.NG = g.C;
  const int bn = g.NG <= 64 ? 64 : 128;
  const bool strided = (g.sh > 1 || g.sw > 1) && g.dh == 1 && g.dw == 1;
  if (strided) {
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
        g.fWc = make_fdiv(g.Wc);
        g.fHc = make_fdiv(g.Hc);
        g.fns = make_fdiv(std::max(g.ns, 1));
        g.M = g.N * g.Hc * g.Wc;
        g.KG = g.nr * g.ns * g.K;
        launch<MODE_DGRAD>(g, bn, ((g.M + BM - 1) / BM) * ((g.NG + bn - 1) / bn), st, p.Z);
      }
    FFK_LAUNCH_CHECK("conv2d_grouped_dgrad");
    return;
  }
  g.M = g.N * g.H * g.W;
  g.KG = g.R * g.S * g.K;
  launch<MODE_DGRAD>(g, bn, ((g.M + BM - 1) / BM) * ((g.NG + bn - 1) / bn), st, p.Z);
  FFK_LAUNCH_CHECK("conv2d_grouped_dgrad");
}

namespace {
WgradPlan grouped_wgrad_plan(const ConvShape& cs, const GroupPlan& gp) {
  ConvArgs g = grouped_args(cs, gp);
  const int M = gp.Ks, NG = cs.R * cs.S * gp.Cs;
  const int64_t KG = static_cast<int64_t>(g.N) * g.P * g.Q;
  WgradPlan p;
  p.bn = NG <= 64 ? 64 : 128;
  p.tiles = ((M + BM - 1) / BM) * ((NG + p.bn - 1) / p.bn);
  const int nk = static_cast<int>((KG + BK - 1) / BK);
  const int64_t tz = static_cast<int64_t>(p.tiles) * gp.Z;
  int splits = static_cast<int>((2048 + tz - 1) / tz);
  splits = std::min(splits, std::max(1, nk / 8));
  const int64_t slab = static_cast<int64_t>(gp.Z) * M * NG * 4;
  splits = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(splits, (int64_t(256) << 20) / slab)));
  splits = std::max(1, std::min(splits, nk));
  p.kt_per_split = (nk + splits - 1) / splits;
  p.splits = (nk + p.kt_per_split - 1) / p.kt_per_split;
  return p;
}
}  // namespace

int64_t conv2d_grouped_wgrad_ws_floats(const ConvShape& cs, int groups) {
  const GroupPlan gp = group_plan(cs, groups);
  const WgradPlan p = grouped_wgrad_plan(cs, gp);
  const int64_t W = static_cast<int64_t>(cs.K) * cs.R * cs.S * gp.Cs;   // the expanded gradient (all super-groups)
  // expanded gradient + split slabs + the two-pass reduce scratch
  return W + (p.splits > 1 ? static_cast<int64_t>(p.splits) * W + (p.splits >= 64 ? kMaxChunks * W : 0) : 0);
}

void conv2d_grouped_wgrad(const ConvShape& cs, int groups, const void* x, const void* dy, float* dw, float* ws,
                          hipStream_t st) {
  check_shape(cs, "conv2d_grouped_wgrad");
  if (!ws) throw std::invalid_argument("conv2d_grouped_wgrad: needs a workspace");
  const GroupPlan gp = group_plan(cs, groups);
  const WgradPlan p = grouped_wgrad_plan(cs, gp);
  ConvArgs g = grouped_args(cs, gp);
  const int64_t W = static_cast<int64_t>(cs.K) * cs.R * cs.S * gp.Cs;
  float* dwexp = ws;
  g.x = static_cast<const bf16*>(x);
  g.dy = static_cast<const bf16*>(dy);
  g.out = dwexp;
  // every launch writes (never accumulates): one split writes the expanded
  // gradient itself, several write slabs reduced into it
  g.wpart = p.splits > 1 ? ws + W : dwexp;
  g.M = g.K;
  g.NG = g.R * g.S * g.C;
  g.KG = g.N * g.P * g.Q;
  g.kt_per_split = p.kt_per_split;
  launch<MODE_WGRAD>(g, p.bn, p.tiles * p.splits, st, gp.Z);
  FFK_LAUNCH_CHECK("conv2d_grouped_wgrad");
  if (p.splits > 1) {
    reduce_rows(ws + W, dwexp, p.splits, W, 0, p.splits >= 64 ? ws + W + static_cast<int64_t>(p.splits) * W : nullptr,
                st);
    FFK_LAUNCH_CHECK("conv2d_grouped_wgrad reduce");
  }
  const int64_t n = static_cast<int64_t>(cs.K) * cs.R * cs.S * gp.Cg;
  hipLaunchKernelGGL(group_compress_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, st,
                     static_cast<const float*>(dwexp), dw, n, cs.R * cs.S, gp.Cs, gp.Ks, gp.Cg, gp.Kg);
  FFK_LAUNCH_CHECK("conv2d_grouped_wgrad compress");
}

// ---------------------------------------------------------------------------
// Channel padding of a convolution input (the RGB stem: 3 channels -> 8, so
// every 16-B gather chunk holds whole channels): one pass from any 4-d
// strided bf16 tensor [N][C][H][W] (NCHW or channels_last) to an NHWC image
// with Cp >= C channels, the pad channels zero; one output pixel (Cp / 8
// 16-B chunks) per thread.  Replaces a layout copy, a zero fill and a strided
// copy.
namespace {
__global__ __launch_bounds__(256) void pad_channels_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                           int64_t npix, int C, int H, int W, int64_t sn,
                                                           int64_t sc, int64_t sh, int64_t sw, int Cp) {
  const int64_t p = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (p >= npix) return;
  const int w = static_cast<int>(p % W);
  const int64_t t = p / W;
  const int h = static_cast<int>(t % H);
  const int64_t n = t / H;
  const bf16* src = x + n * sn + h * sh + w * sw;
  for (int c0 = 0; c0 < Cp; c0 += 8) {
    bf16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = c0 + e < C ? src[(c0 + e) * sc] : static_cast<bf16>(0.f);
    *reinterpret_cast<bf16x8*>(y + p * Cp + c0) = v;
  }
}
}  // namespace

void pad_channels_nhwc(const void* x, void* y, int64_t N, int C, int H, int W, int64_t sn, int64_t sc, int64_t sh,
                       int64_t sw, int Cp, hipStream_t st) {
  if (Cp % 8 || Cp < C) throw std::invalid_argument("pad_channels_nhwc: Cp must be a multiple of 8 and >= C");
  const int64_t npix = N * H * W;
  if (npix <= 0) return;
  hipLaunchKernelGGL(pad_channels_kernel, dim3(static_cast<unsigned>((npix + 255) / 256)), dim3(256), 0, st,
                     static_cast<const bf16*>(x), static_cast<bf16*>(y), npix, C, H, W, sn, sc, sh, sw, Cp);
  FFK_LAUNCH_CHECK("pad_channels_nhwc");
}

}  // namespace ffk
