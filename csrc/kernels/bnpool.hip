// BatchNorm (training mode) and 2-D pooling for NHWC bf16 activations (gfx950).
//
// Parity: lib/kernels/src/cuda/ops/batch_norm_kernels.cu
// (cudnnBatchNormalizationForwardTraining :35 with running statistics,
// fused ReLU, cudnnBatchNormalizationBackward :71 + reluBackward :68) and
// pool_2d_kernels.cu (cudnnPoolingForward :103 / Backward :123, max and
// average).
//
// Layout: activations are [M = N*H*W][C] (channels innermost, torch
// channels_last), so every thread moves 8 channels as one 16-byte vector and
// the per-channel parameters a thread needs are fixed for its whole life.
//   * statistics: per-channel (sum, sum of squares) — either produced by the
//     convolution epilogue (conv.hip) or by bn_stats here — then bn_finalize
//     turns them into scale/shift (+ running-stat update, + saved mean/rstd);
//   * bn_apply: y = x*scale + shift [+ residual] [ReLU] in one pass;
//   * backward: bn_bwd_reduce accumulates sum(g), sum(g*xhat) with g = dy
//     masked by the ReLU (recomputed from y), bn_bwd_coef folds them into
//     per-channel (A, B, D) and dgamma/dbeta, bn_bwd_apply writes
//     dx = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)) = A*g + B*x + D.
// Reductions: a block is RL row-lanes x GL channel-group lanes; each thread
// strides over rows with 8 fp32 accumulators per quantity, the block reduces
// its row-lanes through LDS and issues one fp32 atomic per channel.
// Pooling: forward one thread per (output pixel, 8 channels), max pooling
// records the winning tap as a byte; backward is a gather over the windows
// that cover an input pixel (no atomics, deterministic).
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace ffk {

namespace {

__device__ __forceinline__ void load8(const bf16* p, float (&v)[8]) {
  const bf16x8 t = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = bf2f(t[i]);
}
__device__ __forceinline__ void store8(bf16* p, const float (&v)[8]) {
  bf16x8 t;
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = f2bf(v[i]);
  *reinterpret_cast<bf16x8*>(p) = t;
}
__device__ __forceinline__ float ldp(const void* p, int dt, int i) {
  return dt == 1 ? bf2f(static_cast<const bf16*>(p)[i]) : static_cast<const float*>(p)[i];
}

constexpr int kBnBuckets = 16;

struct RedGeom {
  int GL, RL, G;  // group lanes, row lanes, channel groups
};
RedGeom red_geom(int C) {
  RedGeom r;
  r.G = C / 8;
  r.GL = 1;
  while (r.GL < r.G && r.GL < 64) r.GL <<= 1;
  r.RL = 256 / r.GL;
  return r;
}
// target workgroups of a reduction pass (FFK_BN_RED_BLOCKS, read once).
// 1024 (4 per CU): ResNet-50 8910 img/s vs 8794 at 2048, 8596 at 4096, 8257
// at 8192 (interleaved on one box, profiles/r5/ab_bn_red_blocks_r5.txt) --
// fewer, longer-running workgroups mean fewer bucket atomics and LDS tails
int red_blocks() {
  static const int b = [] {
    const char* e = getenv("FFK_BN_RED_BLOCKS");
    const int v = e ? atoi(e) : 1024;
    return v >= 256 && v <= 65536 ? v : 1024;
  }();
  return b;
}
dim3 red_grid(const RedGeom& r, int64_t M) {
  const int gy = (r.G + r.GL - 1) / r.GL;
  int64_t gx = (M + r.RL - 1) / r.RL;
  const int64_t want = std::max<int64_t>(1, red_blocks() / gy);
  gx = std::min(gx, want);
  return dim3(static_cast<unsigned>(std::max<int64_t>(gx, 1)), gy);
}

// MODE 0: stats of x  -> out[0:C] += sum x, out[C:2C] += sum x^2
// MODE 1: bwd reduce  -> out[0:C] += sum g,  out[C:2C] += sum g*xhat
// U rows per thread and iteration, their loads issued before any math (raw
// 16-B vectors, 4 VGPRs each): a wave keeps U (MODE 0) or 2U / 3U (MODE 1)
// KiB in flight instead of 1 / 2 / 3, which is what the HBM latency needs.
template <int MODE, int U>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                        const bf16* __restrict__ y, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, float* __restrict__ out,
                                                        int64_t M, int C, int GL, int relu,
                                                        const float* __restrict__ ss, int nbuckets) {
  __shared__ float red[2][256 * 8 + 8];
  const int RL = 256 / GL;
  const int gl = threadIdx.x % GL, rl = threadIdx.x / GL;
  const int grp = blockIdx.y * GL + gl;
  const bool gok = grp * 8 < C;
  const int c0 = grp * 8;
  float a[8], b[8], mu[8], rs[8], sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = b[i] = 0.f;
  if (MODE == 1 && gok) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      mu[i] = mean[c0 + i];
      rs[i] = rstd[c0 + i];
      sc[i] = relu == 2 ? ss[c0 + i] : 0.f;
      sh[i] = relu == 2 ? ss[C + c0 + i] : 0.f;
    }
  }
  if (gok) {
    const int64_t step = static_cast<int64_t>(gridDim.x) * RL;
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * RL + rl; r < M; r += U * step) {
      bf16x8 xr[U], gr[U], yr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = r + u * step;
        if (rr < M) {
          const int64_t off = rr * C + c0;
          xr[u] = *reinterpret_cast<const bf16x8*>(x + off);
          if (MODE == 1) {
            gr[u] = *reinterpret_cast<const bf16x8*>(dy + off);
            if (relu == 1) yr[u] = *reinterpret_cast<const bf16x8*>(y + off);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (r + u * step >= M) break;
        float xv[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] = bf2f(xr[u][i]);
        if (MODE == 0) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            a[i] += xv[i];
            b[i] += xv[i] * xv[i];
          }
        } else {
          float g[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) g[i] = bf2f(gr[u][i]);
          if (relu == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) g[i] = bf2f(yr[u][i]) > 0.f ? g[i] : 0.f;
          } else if (relu == 2) {  // ReLU mask recomputed from x (the forward's y is not re-read)
#pragma unroll
            for (int i = 0; i < 8; ++i) g[i] = xv[i] * sc[i] + sh[i] > 0.f ? g[i] : 0.f;
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            a[i] += g[i];
            b[i] += g[i] * (xv[i] - mu[i]) * rs[i];
          }
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[0][threadIdx.x * 8 + i] = a[i];
    red[1][threadIdx.x * 8 + i] = b[i];
  }
  __syncthreads();
  // column j of the block tile (GL*8 channels) reduced over RL row lanes
  for (int j = threadIdx.x; j < GL * 8 * 2; j += 256) {
    const int q = j / (GL * 8), col = j % (GL * 8);
    const int lg = col / 8, e = col % 8;
    float s = 0.f;
    for (int l = 0; l < RL; ++l) s += red[q][(l * GL + lg) * 8 + e];
    const int ch = blockIdx.y * GL * 8 + col;
    // blocks spread over `nbuckets` copies of [2][C] (the consumer sums them):
    // a few hundred same-address atomics, not thousands
    float* dst = out + static_cast<int64_t>(blockIdx.x % nbuckets) * 2 * C;
    if (ch < C) atomicAdd(dst + q * C + ch, s);
  }
}

// scale/shift from accumulated stats; running stats; saved mean / rstd.
__global__ void bn_finalize_kernel(const float* __restrict__ stats, const void* gamma, const void* beta, int pdt,
                                   float* running_mean, float* running_var, float* scale, float* shift, float* mean_o,
                                   float* rstd_o, int C, double count, float momentum, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double mean = stats[c] / count;
  double var = stats[C + c] / count - mean * mean;
  var = var > 0.0 ? var : 0.0;
  const float rstd = static_cast<float>(1.0 / sqrt(var + eps));
  const float g = gamma ? ldp(gamma, pdt, c) : 1.f;
  const float b = beta ? ldp(beta, pdt, c) : 0.f;
  scale[c] = g * rstd;
  shift[c] = b - static_cast<float>(mean) * g * rstd;
  if (mean_o) mean_o[c] = static_cast<float>(mean);
  if (rstd_o) rstd_o[c] = rstd;
  if (running_mean && momentum > 0.f) {
    const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * static_cast<float>(mean);
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * static_cast<float>(unbiased);
  }
}

template <int U>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, bf16* __restrict__ y,
                                                       int64_t nvec, int C, int relu) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t v0 = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; v0 < nvec; v0 += U * step) {
    bf16x8 xr[U], rr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + u * step;
      if (v < nvec) {
        xr[u] = *reinterpret_cast<const bf16x8*>(x + v * 8);
        if (res) rr[u] = *reinterpret_cast<const bf16x8*>(res + v * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + u * step;
      if (v >= nvec) break;
      const int64_t off = v * 8;
      const int c0 = static_cast<int>(off % C);
      float xv[8];
      const f32x4 s0 = *reinterpret_cast<const f32x4*>(scale + c0), s1 = *reinterpret_cast<const f32x4*>(scale + c0 + 4);
      const f32x4 h0 = *reinterpret_cast<const f32x4*>(shift + c0), h1 = *reinterpret_cast<const f32x4*>(shift + c0 + 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        xv[i] = bf2f(xr[u][i]) * s0[i] + h0[i];
        xv[i + 4] = bf2f(xr[u][i + 4]) * s1[i] + h1[i];
      }
      if (res) {
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] += bf2f(rr[u][i]);
      }
      if (relu) {
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] = xv[i] > 0.f ? xv[i] : 0.f;
      }
      store8(y + off, xv);
    }
  }
}

// per-channel backward coefficients: dx = A*g + B*x + D with
// A = gamma*rstd, B = -A*rstd*mean(g*xhat), D = -A*mean(g) - B*mean;
// also dgamma += sum(g*xhat), dbeta += sum(g).
__global__ void bn_bwd_coef_kernel(float* __restrict__ sums, const float* __restrict__ mean,
                                   const float* __restrict__ rstd, const void* gamma, int pdt, float* __restrict__ coef,
                                   float* dgamma, float* dbeta, int C, float inv_count, int reset, int nb) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s1 = 0.f, s2 = 0.f;
  for (int k = 0; k < nb; ++k) {
    s1 += sums[static_cast<int64_t>(k) * 2 * C + c];
    s2 += sums[static_cast<int64_t>(k) * 2 * C + C + c];
  }
  if (reset) {  // a persistent workspace leaves this kernel zeroed for the next reduction
    for (int k = 0; k < kBnBuckets; ++k) {
      sums[static_cast<int64_t>(k) * 2 * C + c] = 0.f;
      sums[static_cast<int64_t>(k) * 2 * C + C + c] = 0.f;
    }
  }
  const float A = (gamma ? ldp(gamma, pdt, c) : 1.f) * rstd[c];
  const float B = -A * rstd[c] * s2 * inv_count;
  coef[c] = A;
  coef[C + c] = B;
  coef[2 * C + c] = -A * s1 * inv_count - B * mean[c];
  if (dbeta) dbeta[c] += s1;
  if (dgamma) dgamma[c] += s2;
}

template <int U>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                           const bf16* __restrict__ y, const float* __restrict__ coef,
                                                           bf16* __restrict__ dx, bf16* __restrict__ dres,
                                                           int64_t nvec, int C, int relu,
                                                           const float* __restrict__ ss) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t v0 = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; v0 < nvec; v0 += U * step) {
    bf16x8 gr[U], xr[U], yr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + u * step;
      if (v < nvec) {
        gr[u] = *reinterpret_cast<const bf16x8*>(dy + v * 8);
        xr[u] = *reinterpret_cast<const bf16x8*>(x + v * 8);
        if (relu == 1) yr[u] = *reinterpret_cast<const bf16x8*>(y + v * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = v0 + u * step;
      if (v >= nvec) break;
      const int64_t off = v * 8;
      const int c0 = static_cast<int>(off % C);
      float g[8], xv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        g[i] = bf2f(gr[u][i]);
        xv[i] = bf2f(xr[u][i]);
      }
      if (relu == 1) {
#pragma unroll
        for (int i = 0; i < 8; ++i) g[i] = bf2f(yr[u][i]) > 0.f ? g[i] : 0.f;
      } else if (relu == 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 s4 = *reinterpret_cast<const f32x4*>(ss + c0 + 4 * h);
          const f32x4 h4 = *reinterpret_cast<const f32x4*>(ss + C + c0 + 4 * h);
#pragma unroll
          for (int i = 0; i < 4; ++i) g[4 * h + i] = xv[4 * h + i] * s4[i] + h4[i] > 0.f ? g[4 * h + i] : 0.f;
        }
      }
      if (dres) store8(dres + off, g);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 A = *reinterpret_cast<const f32x4*>(coef + c0 + 4 * h);
        const f32x4 B = *reinterpret_cast<const f32x4*>(coef + C + c0 + 4 * h);
        const f32x4 D = *reinterpret_cast<const f32x4*>(coef + 2 * C + c0 + 4 * h);
#pragma unroll
        for (int i = 0; i < 4; ++i) g[4 * h + i] = A[i] * g[4 * h + i] + B[i] * xv[4 * h + i] + D[i];
      }
      store8(dx + off, g);
    }
  }
}

// ---------------------------------------------------------------------------
struct PoolArgs {
  int N, H, W, C, P, Q, R, S, sh, sw, ph, pw;
  int avg, count_pad;
};

__global__ __launch_bounds__(256) void pool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                       unsigned char* __restrict__ arg, PoolArgs a, int64_t nthreads) {
  const int G = a.C / 8;
  for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < nthreads;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(t % G);
    int64_t pix = t / G;
    const int q = static_cast<int>(pix % a.Q);
    pix /= a.Q;
    const int p = static_cast<int>(pix % a.P);
    const int n = static_cast<int>(pix / a.P);
    const int h0 = p * a.sh - a.ph, w0 = q * a.sw - a.pw;
    float acc[8];
    unsigned char best[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc[i] = a.avg ? 0.f : -__builtin_inff();
      best[i] = 0;
    }
    int cnt = 0;
    for (int r = 0; r < a.R; ++r) {
      const int ih = h0 + r;
      if (ih < 0 || ih >= a.H) continue;
      for (int s = 0; s < a.S; ++s) {
        const int iw = w0 + s;
        if (iw < 0 || iw >= a.W) continue;
        float v[8];
        load8(x + ((static_cast<int64_t>(n) * a.H + ih) * a.W + iw) * a.C + g * 8, v);
        ++cnt;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (a.avg) {
            acc[i] += v[i];
          } else if (v[i] > acc[i]) {
            acc[i] = v[i];
            best[i] = static_cast<unsigned char>(r * a.S + s);
          }
        }
      }
    }
    const int64_t off = t * 8;
    if (a.avg) {
      const float div = a.count_pad ? static_cast<float>(a.R * a.S) : static_cast<float>(cnt > 0 ? cnt : 1);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] /= div;
    } else if (arg) {
      uint64_t packed = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) packed |= static_cast<uint64_t>(best[i]) << (8 * i);
      *reinterpret_cast<uint64_t*>(arg + off) = packed;
    }
    store8(y + off, acc);
  }
}

__global__ __launch_bounds__(256) void pool_bwd_kernel(const bf16* __restrict__ dy,
                                                       const unsigned char* __restrict__ arg,
                                                       bf16* __restrict__ dx, PoolArgs a, int64_t nthreads,
                                                       float beta) {
  const int G = a.C / 8;
  for (int64_t t = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; t < nthreads;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int g = static_cast<int>(t % G);
    int64_t pix = t / G;
    const int w = static_cast<int>(pix % a.W);
    pix /= a.W;
    const int h = static_cast<int>(pix % a.H);
    const int n = static_cast<int>(pix / a.H);
    // windows p with p*sh - ph <= h < p*sh - ph + R
    const int pl = max(0, (h + a.ph - a.R + a.sh) / a.sh), ph_ = min(a.P - 1, (h + a.ph) / a.sh);
    const int ql = max(0, (w + a.pw - a.S + a.sw) / a.sw), qh = min(a.Q - 1, (w + a.pw) / a.sw);
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    for (int p = pl; p <= ph_; ++p) {
      const int r = h - (p * a.sh - a.ph);
      if (r < 0 || r >= a.R) continue;
      for (int q = ql; q <= qh; ++q) {
        const int s = w - (q * a.sw - a.pw);
        if (s < 0 || s >= a.S) continue;
        const int64_t o = ((static_cast<int64_t>(n) * a.P + p) * a.Q + q) * a.C + g * 8;
        float d[8];
        load8(dy + o, d);
        if (a.avg) {
          float div;
          if (a.count_pad) {
            div = static_cast<float>(a.R * a.S);
          } else {
            const int h0 = p * a.sh - a.ph, w0 = q * a.sw - a.pw;
            const int nh = min(h0 + a.R, a.H) - max(h0, 0), nw = min(w0 + a.S, a.W) - max(w0, 0);
            div = static_cast<float>(max(nh * nw, 1));
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[i] += d[i] / div;
        } else {
          const uint64_t packed = *reinterpret_cast<const uint64_t*>(arg + o);
          const unsigned tap = static_cast<unsigned>(r * a.S + s);
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (((packed >> (8 * i)) & 0xff) == tap) acc[i] += d[i];
        }
      }
    }
    const int64_t off = t * 8;
    if (beta != 0.f) {
      float old[8];
      load8(dx + off, old);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += beta * old[i];
    }
    store8(dx + off, acc);
  }
}

int ew_blocks(int64_t n) { return static_cast<int>(std::min<int64_t>((n + 255) / 256, 8192)); }

}  // namespace

__global__ void bn_fold_buckets_kernel(float* __restrict__ ws, float* __restrict__ stats, int C2, int reset,
                                       int overwrite) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C2) return;
  float s = 0.f;
  for (int k = 0; k < kBnBuckets; ++k) s += ws[static_cast<int64_t>(k) * C2 + c];
  stats[c] = overwrite ? s : stats[c] + s;
  if (reset)
    for (int k = 0; k < kBnBuckets; ++k) ws[static_cast<int64_t>(k) * C2 + c] = 0.f;
}

// rows / vectors per thread and iteration of the reduction and apply passes
// (FFK_BN_UNROLL: 1, 2 or 4; read once).  1 measured fastest: 5.2-5.6 TB/s
// at the ResNet-50 layer-1 shapes, 2 and 4 up to 8 % slower, ResNet-50
// 8143 vs 7950 img/s (profiles/r5/bench_bn_unroll_r5.txt)
static int bn_unroll() {
  static const int u = [] {
    const char* e = getenv("FFK_BN_UNROLL");
    const int v = e ? atoi(e) : 1;
    return v == 2 || v == 4 ? v : 1;
  }();
  return u;
}
// workgroup cap of the BN apply passes (FFK_BN_APPLY_BLOCKS, read once)
static int bn_apply_blocks(int64_t n) {
  static const int cap = [] {
    const char* e = getenv("FFK_BN_APPLY_BLOCKS");
    const int v = e ? atoi(e) : 8192;
    return v >= 256 && v <= 65536 ? v : 8192;
  }();
  return static_cast<int>(std::min<int64_t>((n + 255) / 256, cap));
}
template <typename F>
static void with_unroll(F&& f) {
  switch (bn_unroll()) {
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    default: f(std::integral_constant<int, 1>{}); break;
  }
}

void bn_stats(const void* x, float* stats, int64_t M, int C, hipStream_t st, float* ws, int ws_clean) {
  if (C % 8) throw std::invalid_argument("bn_stats: C must be a multiple of 8");
  // ws_clean bit 1: overwrite `stats` instead of accumulating (needs ws)
  const int overwrite = (ws_clean & 2) && ws ? 1 : 0;
  ws_clean &= 1;
  if (M <= 0) {
    if (overwrite) (void)hipMemsetAsync(stats, 0, sizeof(float) * 2 * C, st);
    return;
  }
  const RedGeom r = red_geom(C);
  dim3 grid = red_grid(r, M);
  if (!ws) grid.x = std::min(grid.x, 256u);  // single [2][C] target: bound the same-address atomics
  else if (!ws_clean) (void)hipMemsetAsync(ws, 0, sizeof(float) * 2 * C * kBnBuckets, st);
  with_unroll([&](auto uu) {
    hipLaunchKernelGGL((bn_reduce_kernel<0, decltype(uu)::value>), grid, dim3(256), 0, st,
                       static_cast<const bf16*>(x), nullptr, nullptr, nullptr, nullptr, ws ? ws : stats, M, C, r.GL,
                       0, nullptr, ws ? kBnBuckets : 1);
  });
  if (ws)
    hipLaunchKernelGGL(bn_fold_buckets_kernel, dim3((2 * C + 255) / 256), dim3(256), 0, st, ws, stats, 2 * C,
                       ws_clean, overwrite);
  FFK_LAUNCH_CHECK("bn_stats");
}

void bn_finalize(const float* stats, const void* gamma, const void* beta, int param_dtype, float* running_mean,
                 float* running_var, float* scale, float* shift, float* mean, float* rstd, int C, double count,
                 float momentum, float eps, hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, stats, gamma, beta, param_dtype,
                     running_mean, running_var, scale, shift, mean, rstd, C, count, momentum, eps);
  FFK_LAUNCH_CHECK("bn_finalize");
}

void bn_apply(const void* x, const void* residual, const float* scale, const float* shift, void* y, int64_t M, int C,
              int relu, hipStream_t st) {
  if (C % 8) throw std::invalid_argument("bn_apply: C must be a multiple of 8");
  const int64_t nvec = M * C / 8;
  if (nvec <= 0) return;
  with_unroll([&](auto uu) {
    constexpr int U = decltype(uu)::value;
    hipLaunchKernelGGL(bn_apply_kernel<U>, dim3(bn_apply_blocks((nvec + U - 1) / U)), dim3(256), 0, st,
                       static_cast<const bf16*>(x), static_cast<const bf16*>(residual), scale, shift,
                       static_cast<bf16*>(y), nvec, C, relu);
  });
  FFK_LAUNCH_CHECK("bn_apply");
}

void bn_bwd(const void* dy, const void* x, const void* y, const float* mean, const float* rstd, const void* gamma,
            int param_dtype, void* dx, void* dres, float* dgamma, float* dbeta, float* ws, int64_t M, int C,
            int relu, hipStream_t st, const float* scale_shift, int ws_clean, const float* pre_sums) {
  if (C % 8) throw std::invalid_argument("bn_bwd: C must be a multiple of 8");
  if (relu == 1 && !y) throw std::invalid_argument("bn_bwd: ReLU mask from y needs y");
  if (relu == 2 && !scale_shift) throw std::invalid_argument("bn_bwd: ReLU mask from x needs the scale / shift");
  if (M <= 0) return;
  const RedGeom r = red_geom(C);
  float* coef = ws + 2 * C * kBnBuckets;
  if (pre_sums) {   // sums reduced by the consumer convolution's dgrad epilogue (conv.hip)
    hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, st, const_cast<float*>(pre_sums),
                       mean, rstd, gamma, param_dtype, coef, dgamma, dbeta, C, static_cast<float>(1.0 / M), 0, 1);
  } else {
    if (!ws_clean) (void)hipMemsetAsync(ws, 0, sizeof(float) * 2 * C * kBnBuckets, st);
    with_unroll([&](auto uu) {
      hipLaunchKernelGGL((bn_reduce_kernel<1, decltype(uu)::value>), red_grid(r, M), dim3(256), 0, st,
                         static_cast<const bf16*>(x), static_cast<const bf16*>(dy), static_cast<const bf16*>(y), mean,
                         rstd, ws, M, C, r.GL, relu, scale_shift, kBnBuckets);
    });
    hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, st, ws, mean, rstd, gamma,
                       param_dtype, coef, dgamma, dbeta, C, static_cast<float>(1.0 / M), ws_clean, kBnBuckets);
  }
  const int64_t nvec = M * C / 8;
  with_unroll([&](auto uu) {
    constexpr int U = decltype(uu)::value;
    hipLaunchKernelGGL(bn_bwd_apply_kernel<U>, dim3(bn_apply_blocks((nvec + U - 1) / U)), dim3(256), 0, st,
                       static_cast<const bf16*>(dy), static_cast<const bf16*>(x), static_cast<const bf16*>(y), coef,
                       static_cast<bf16*>(dx), static_cast<bf16*>(dres), nvec, C, relu, scale_shift);
  });
  FFK_LAUNCH_CHECK("bn_bwd");
}

static PoolArgs pool_args(const PoolShape& s) {
  if (s.C % 8) throw std::invalid_argument("pool2d: C must be a multiple of 8");
  if (s.R * s.S > 256) throw std::invalid_argument("pool2d: window larger than 256 taps");
  PoolArgs a{s.N, s.H, s.W, s.C, 0, 0, s.R, s.S, s.sh, s.sw, s.ph, s.pw, s.avg, s.count_pad};
  a.P = (s.H + 2 * s.ph - s.R) / s.sh + 1;
  a.Q = (s.W + 2 * s.pw - s.S) / s.sw + 1;
  if (a.P <= 0 || a.Q <= 0 || s.sh <= 0 || s.sw <= 0) throw std::invalid_argument("pool2d: bad geometry");
  return a;
}

void pool2d_fwd(const PoolShape& s, const void* x, void* y, void* argmax, hipStream_t st) {
  const PoolArgs a = pool_args(s);
  const int64_t n = static_cast<int64_t>(a.N) * a.P * a.Q * (a.C / 8);
  hipLaunchKernelGGL(pool_fwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, st, static_cast<const bf16*>(x),
                     static_cast<bf16*>(y), static_cast<unsigned char*>(argmax), a, n);
  FFK_LAUNCH_CHECK("pool2d_fwd");
}

void pool2d_bwd(const PoolShape& s, const void* dy, const void* argmax, void* dx, float beta, hipStream_t st) {
  const PoolArgs a = pool_args(s);
  if (!a.avg && !argmax) throw std::invalid_argument("pool2d_bwd: max pooling needs the argmax bytes");
  const int64_t n = static_cast<int64_t>(a.N) * a.H * a.W * (a.C / 8);
  hipLaunchKernelGGL(pool_bwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, st, static_cast<const bf16*>(dy),
                     static_cast<const unsigned char*>(argmax), static_cast<bf16*>(dx), a, n, beta);
  FFK_LAUNCH_CHECK("pool2d_bwd");
}

}  // namespace ffk
