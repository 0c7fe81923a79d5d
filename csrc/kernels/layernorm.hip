// Fused (residual add +) LayerNorm forward / backward for gfx950.
//
// Parity: lib/kernels/src/cuda/ops/layer_norm_kernels.cu (RowwiseMoments +
// LayerNormForward, ComputeInternalGradients + backward + GammaBetaBackward,
// :69-399).  Re-designed for CDNA4 rather than translated:
//  * one wave64 per row, the whole row held in registers (N = C*512 fast path,
//    C <= 8) -> a single HBM read of x (+ residual) and a single write of y;
//  * 16-byte vector loads/stores (8 x bf16 per lane);
//  * residual add fused (BERT/GPT post/pre-LN blocks), optional store of the
//    pre-norm sum for the backward pass;
//  * dgamma/dbeta accumulate in registers across the rows a wave visits,
//    reduce across the block's 4 waves through LDS, then one fp32 atomic per
//    column per block (grid is capped, so atomics are ~N * grid, not N * M).
#include "common.h"
#include <cstdlib>

#include "kernels.h"

namespace ffk {

template <typename T>
struct Vec8;
template <>
struct Vec8<bf16> {
  static __device__ __forceinline__ void load(const bf16* p, float* o) {
    u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = u2f(v[i]);
  }
  static __device__ __forceinline__ void store(bf16* p, const float* o) {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = f2bf(o[i]);
    *reinterpret_cast<bf16x8*>(p) = v;
  }
};
template <>
struct Vec8<float> {
  static __device__ __forceinline__ void load(const float* p, float* o) {
    f32x4 a = reinterpret_cast<const f32x4*>(p)[0];
    f32x4 b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[i] = a[i];
      o[4 + i] = b[i];
    }
  }
  static __device__ __forceinline__ void store(float* p, const float* o) {
    f32x4 a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = o[i];
      b[i] = o[4 + i];
    }
    reinterpret_cast<f32x4*>(p)[0] = a;
    reinterpret_cast<f32x4*>(p)[1] = b;
  }
};

// ---------------------------------------------------------------------------
template <typename T, int C>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                     T* __restrict__ sum_out, const T* __restrict__ gamma,
                                                     const T* __restrict__ beta, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int M, float eps) {
  constexpr int N = C * 512;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const size_t base = static_cast<size_t>(row) * N;
  float v[C][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int col = c * 512 + lane * 8;
    Vec8<T>::load(x + base + col, v[c]);
    if (res) {
      float r[8];
      Vec8<T>::load(res + base + col, r);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] += r[i];
      if (sum_out) Vec8<T>::store(sum_out + base + col, v[c]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[c][i];
  }
  const float mean = wave_sum(s) * (1.f / N);
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float d = v[c][i] - mean;
      q += d * d;
    }
  const float rstd = rsqrtf(wave_sum(q) * (1.f / N) + eps);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int col = c * 512 + lane * 8;
    float g[8], b[8], o[8];
    if (gamma) Vec8<T>::load(gamma + col, g);
    else
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = 1.f;
    if (beta) Vec8<T>::load(beta + col, b);
    else
#pragma unroll
      for (int i = 0; i < 8; ++i) b[i] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mean) * rstd * g[i] + b[i];
    Vec8<T>::store(y + base + col, o);
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Generic path: any N that is a multiple of 8; one 256-thread block per row,
// two passes over the row (L2 resident).
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_generic(const T* __restrict__ x, const T* __restrict__ res,
                                                      T* __restrict__ sum_out, const T* __restrict__ gamma,
                                                      const T* __restrict__ beta, T* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int M, int N, float eps) {
  __shared__ float scratch[4];
  const int row = blockIdx.x;
  const size_t base = static_cast<size_t>(row) * N;
  float s = 0.f, q = 0.f;
  for (int col = threadIdx.x * 8; col < N; col += 256 * 8) {
    float v[8];
    Vec8<T>::load(x + base + col, v);
    if (res) {
      float r[8];
      Vec8<T>::load(res + base + col, r);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += r[i];
      if (sum_out) Vec8<T>::store(sum_out + base + col, v);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s += v[i];
      q += v[i] * v[i];
    }
  }
  s = block_sum<256>(s, scratch);
  q = block_sum<256>(q, scratch);
  const float mean = s / N;
  const float var = fmaxf(q / N - mean * mean, 0.f);
  const float rstd = rsqrtf(var + eps);
  for (int col = threadIdx.x * 8; col < N; col += 256 * 8) {
    float v[8], g[8], b[8], o[8];
    Vec8<T>::load(x + base + col, v);
    if (res) {
      float r[8];
      Vec8<T>::load(res + base + col, r);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] += r[i];
    }
    if (gamma) Vec8<T>::load(gamma + col, g);
    else
      for (int i = 0; i < 8; ++i) g[i] = 1.f;
    if (beta) Vec8<T>::load(beta + col, b);
    else
      for (int i = 0; i < 8; ++i) b[i] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (v[i] - mean) * rstd * g[i] + b[i];
    Vec8<T>::store(y + base + col, o);
  }
  if (threadIdx.x == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// ---------------------------------------------------------------------------
// Backward: xhat = (s - mean) * rstd; g = dy * gamma
//   dx = rstd * (g - mean(g) - xhat * mean(g * xhat))
//   dgamma += dy * xhat, dbeta += dy
// One wave per row, two rows in flight per wave (their loads are issued
// together to hide HBM latency); dgamma / dbeta partials accumulate in
// registers across the rows a wave visits, are reduced over the block's 4
// waves in LDS and stored (plain stores, no atomics) as block partials
// ws[2][gridDim.x][N]; a column-sum pass finishes them.
template <typename T, int C>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ s,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const T* __restrict__ gamma,
                                                     T* __restrict__ dx, float* __restrict__ ws, int M,
                                                     const T* __restrict__ dres, float* __restrict__ ws_dx) {
  constexpr int N = C * 512;
  __shared__ float red[4][2][512];
  // ws_dx: per-block column sums of the final dx (the producing Linear's bias
  // gradient, reduced with the dgamma/dbeta partials); dres: a gradient that
  // reached the normalised SUM from another consumer (pre-LN residual stream)
  float pd[C][8];
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) pd[c][i] = 0.f;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  float pg[C][8], pb[C][8], gm[C][8];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (gamma) Vec8<T>::load(gamma + c * 512 + lane * 8, gm[c]);
    else
#pragma unroll
      for (int i = 0; i < 8; ++i) gm[c][i] = 1.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) pg[c][i] = pb[c][i] = 0.f;
  }
  const int stride = gridDim.x * 4;
  for (int row0 = blockIdx.x * 4 + wave; row0 < M; row0 += 2 * stride) {
    const int rows[2] = {row0, row0 + stride};
    float dv[2][C][8], sv[2][C][8], rv[2][C][8];
    float mean[2], rstd[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const bool ok = rows[k] < M;
      const size_t base = static_cast<size_t>(ok ? rows[k] : row0) * N;
      mean[k] = mean_in[ok ? rows[k] : row0];
      rstd[k] = rstd_in[ok ? rows[k] : row0];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        Vec8<T>::load(dy + base + c * 512 + lane * 8, dv[k][c]);
        Vec8<T>::load(s + base + c * 512 + lane * 8, sv[k][c]);
        // the residual-stream gradient is loaded with the row, not at the
        // store after the two row reductions (a dependent HBM latency per
        // row pair in a latency-bound kernel)
        if (dres) Vec8<T>::load(dres + base + c * 512 + lane * 8, rv[k][c]);
      }
      if (!ok)
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
          for (int i = 0; i < 8; ++i) dv[k][c][i] = 0.f;
    }
    float sum_g[2] = {0.f, 0.f}, sum_gx[2] = {0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xh = (sv[k][c][i] - mean[k]) * rstd[k];
          const float g = dv[k][c][i] * gm[c][i];
          sv[k][c][i] = xh;  // keep xhat
          sum_g[k] += g;
          sum_gx[k] += g * xh;
          pg[c][i] += dv[k][c][i] * xh;
          pb[c][i] += dv[k][c][i];
        }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      sum_g[k] = wave_sum(sum_g[k]) * (1.f / N);
      sum_gx[k] = wave_sum(sum_gx[k]) * (1.f / N);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (rows[k] >= M) continue;
      const size_t base = static_cast<size_t>(rows[k]) * N;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        float o[8];
#pragma unroll
        for (int i = 0; i < 8; ++i)
          o[i] = rstd[k] * (dv[k][c][i] * gm[c][i] - sum_g[k] - sv[k][c][i] * sum_gx[k]);
        if (dres) {
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += rv[k][c][i];
        }
        Vec8<T>::store(dx + base + c * 512 + lane * 8, o);
        if (ws_dx) {
#pragma unroll
          for (int i = 0; i < 8; ++i) pd[c][i] += o[i];
        }
      }
    }
  }
  if (ws_dx) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
#pragma unroll
      for (int i = 0; i < 8; ++i) red[wave][0][lane * 8 + i] = pd[c][i];
      __syncthreads();
      for (int j = threadIdx.x; j < 512; j += 256)
        ws_dx[static_cast<size_t>(blockIdx.x) * N + c * 512 + j] =
            red[0][0][j] + red[1][0][j] + red[2][0][j] + red[3][0][j];
      __syncthreads();
    }
  }
  if (!ws) return;
#pragma unroll
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[wave][0][lane * 8 + i] = pg[c][i];
      red[wave][1][lane * 8 + i] = pb[c][i];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 512; j += 256) {
      const float a = red[0][0][j] + red[1][0][j] + red[2][0][j] + red[3][0][j];
      const float b = red[0][1][j] + red[1][1][j] + red[2][1][j] + red[3][1][j];
      ws[static_cast<size_t>(blockIdx.x) * N + c * 512 + j] = a;
      ws[static_cast<size_t>(gridDim.x + blockIdx.x) * N + c * 512 + j] = b;
    }
    __syncthreads();
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_generic(const T* __restrict__ dy, const T* __restrict__ s,
                                                      const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in,
                                                      const T* __restrict__ gamma, T* __restrict__ dx,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta, int M,
                                                      int N, const T* __restrict__ dres, float* __restrict__ dsum) {
  __shared__ float scratch[4];
  const int row = blockIdx.x;
  const size_t base = static_cast<size_t>(row) * N;
  const float mean = mean_in[row], rstd = rstd_in[row];
  float sum_g = 0.f, sum_gx = 0.f;
  for (int col = threadIdx.x * 8; col < N; col += 256 * 8) {
    float dv[8], sv[8], gm[8];
    Vec8<T>::load(dy + base + col, dv);
    Vec8<T>::load(s + base + col, sv);
    if (gamma) Vec8<T>::load(gamma + col, gm);
    else
      for (int i = 0; i < 8; ++i) gm[i] = 1.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float xh = (sv[i] - mean) * rstd;
      float g = dv[i] * gm[i];
      sum_g += g;
      sum_gx += g * xh;
      if (dgamma) atomicAdd(dgamma + col + i, dv[i] * xh);
      if (dbeta) atomicAdd(dbeta + col + i, dv[i]);
    }
  }
  sum_g = block_sum<256>(sum_g, scratch) / N;
  sum_gx = block_sum<256>(sum_gx, scratch) / N;
  for (int col = threadIdx.x * 8; col < N; col += 256 * 8) {
    float dv[8], sv[8], gm[8], o[8];
    Vec8<T>::load(dy + base + col, dv);
    Vec8<T>::load(s + base + col, sv);
    if (gamma) Vec8<T>::load(gamma + col, gm);
    else
      for (int i = 0; i < 8; ++i) gm[i] = 1.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float xh = (sv[i] - mean) * rstd;
      o[i] = rstd * (dv[i] * gm[i] - sum_g - xh * sum_gx);
    }
    if (dres) {
      float r[8];
      Vec8<T>::load(dres + base + col, r);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] += r[i];
    }
    Vec8<T>::store(dx + base + col, o);
    if (dsum)
#pragma unroll
      for (int i = 0; i < 8; ++i) atomicAdd(dsum + col + i, o[i]);
  }
}

// ---------------------------------------------------------------------------
template <typename T>
static void ln_fwd_t(const void* x, const void* res, void* sum_out, const void* gamma, const void* beta, void* y,
                     float* mean, float* rstd, int M, int N, float eps, hipStream_t st) {
  auto X = static_cast<const T*>(x);
  auto R = static_cast<const T*>(res);
  auto S = static_cast<T*>(sum_out);
  auto G = static_cast<const T*>(gamma);
  auto B = static_cast<const T*>(beta);
  auto Y = static_cast<T*>(y);
  if (N % 512 == 0 && N <= 4096) {
    dim3 grid((M + 3) / 4);
    switch (N / 512) {
#define FFK_LN_CASE(c) \
  case c: hipLaunchKernelGGL((ln_fwd_kernel<T, c>), grid, dim3(256), 0, st, X, R, S, G, B, Y, mean, rstd, M, eps); break;
      FFK_LN_CASE(1) FFK_LN_CASE(2) FFK_LN_CASE(3) FFK_LN_CASE(4) FFK_LN_CASE(5) FFK_LN_CASE(6) FFK_LN_CASE(7)
      FFK_LN_CASE(8)
#undef FFK_LN_CASE
    }
  } else {
    hipLaunchKernelGGL((ln_fwd_generic<T>), dim3(M), dim3(256), 0, st, X, R, S, G, B, Y, mean, rstd, M, N, eps);
  }
  FFK_LAUNCH_CHECK("layernorm_fwd");
}

// Finishes the backward's column sums in ONE launch: out_j[c] += sum over the
// `rows` partial rows of slice j of ws[3][rows][N] (j = dgamma, dbeta, dsum;
// absent outputs are skipped).  Block = 64 columns x 4 row groups over a
// 64-row chunk (grid.z chunks, so every thread has only 16 loads in flight
// and the reduction is not latency bound); one fp32 atomic per column per block.
__global__ __launch_bounds__(256) void ln_ws_reduce_kernel(const float* __restrict__ ws, float* out0, float* out1,
                                                           float* out2, int rows, int N) {
  __shared__ float red[4][64];
  float* out = blockIdx.y == 0 ? out0 : (blockIdx.y == 1 ? out1 : out2);
  if (out == nullptr) return;
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cx;
  const float* src = ws + static_cast<size_t>(blockIdx.y) * rows * N;
  const int r0 = blockIdx.z * 64, r1 = min(rows, r0 + 64);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int r = r0 + ry + 4 * u;
      if (r < r1) acc[u & 3] += src[static_cast<size_t>(r) * N + c];
    }
  }
  red[ry][cx] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (ry == 0 && c < N) atomicAdd(out + c, (red[0][cx] + red[1][cx]) + (red[2][cx] + red[3][cx]));
}

template <typename T>
static void ln_bwd_t(const void* dy, const void* s, const float* mean, const float* rstd, const void* gamma,
                     void* dx, float* dgamma, float* dbeta, float* ws, int M, int N, const void* dres, float* dsum,
                     hipStream_t st) {
  auto DY = static_cast<const T*>(dy);
  auto S = static_cast<const T*>(s);
  auto G = static_cast<const T*>(gamma);
  auto DX = static_cast<T*>(dx);
  auto DR = static_cast<const T*>(dres);
  if (N % 512 == 0 && N <= 4096) {
    const int grid = layernorm_bwd_grid(M, N);
    float* W = (dgamma || dbeta) ? ws : nullptr;
    if ((dgamma || dbeta || dsum) && ws == nullptr) throw std::invalid_argument("layernorm_bwd: workspace required");
    float* WD = dsum ? ws + static_cast<size_t>(2) * grid * N : nullptr;
    switch (N / 512) {
#define FFK_LNB_CASE(c)                                                                                      \
  case c:                                                                                                    \
    hipLaunchKernelGGL((ln_bwd_kernel<T, c>), dim3(grid), dim3(256), 0, st, DY, S, mean, rstd, G, DX, W, M, DR, \
                       WD);                                                                                  \
    break;
      FFK_LNB_CASE(1) FFK_LNB_CASE(2) FFK_LNB_CASE(3) FFK_LNB_CASE(4) FFK_LNB_CASE(5) FFK_LNB_CASE(6)
      FFK_LNB_CASE(7) FFK_LNB_CASE(8)
#undef FFK_LNB_CASE
    }
    FFK_LAUNCH_CHECK("layernorm_bwd");
    if (dgamma || dbeta || dsum) {
      hipLaunchKernelGGL(ln_ws_reduce_kernel, dim3((N + 63) / 64, dsum ? 3 : 2, (grid + 63) / 64), dim3(256), 0, st,
                         ws, dgamma, dbeta, dsum, grid, N);
      FFK_LAUNCH_CHECK("layernorm_bwd_reduce");
    }
    return;
  } else {
    hipLaunchKernelGGL((ln_bwd_generic<T>), dim3(M), dim3(256), 0, st, DY, S, mean, rstd, G, DX, dgamma, dbeta, M,
                       N, DR, dsum);
  }
  FFK_LAUNCH_CHECK("layernorm_bwd");
}

void layernorm_fwd(int dtype, const void* x, const void* res, void* sum_out, const void* gamma, const void* beta,
                   void* y, float* mean, float* rstd, int M, int N, float eps, hipStream_t st) {
  if (N % 8 != 0) throw std::invalid_argument("layernorm: N must be a multiple of 8");
  if (dtype == kBF16) ln_fwd_t<bf16>(x, res, sum_out, gamma, beta, y, mean, rstd, M, N, eps, st);
  else if (dtype == kF32) ln_fwd_t<float>(x, res, sum_out, gamma, beta, y, mean, rstd, M, N, eps, st);
  else throw std::invalid_argument("layernorm: unsupported dtype");
}

int layernorm_bwd_grid(int M, int N) {
  // blocks of 4 waves; more blocks = more rows in flight (the kernel is
  // HBM-latency bound at 2 waves / SIMD), at the price of a larger partial-sum
  // workspace ws[3][grid][N] for the final reduction
  static const int cap = [] {
    const char* e = getenv("FFK_LN_BWD_GRID");
    return e ? std::max(64, atoi(e)) : 512;
  }();
  if (N % 512 == 0 && N <= 4096) return std::max(1, std::min((M + 7) / 8, cap));
  return 0;
}

void layernorm_bwd(int dtype, const void* dy, const void* s, const float* mean, const float* rstd,
                   const void* gamma, void* dx, float* dgamma, float* dbeta, float* ws, int M, int N,
                   hipStream_t st, const void* dres, float* dsum) {
  if (N % 8 != 0) throw std::invalid_argument("layernorm: N must be a multiple of 8");
  if (dtype == kBF16) ln_bwd_t<bf16>(dy, s, mean, rstd, gamma, dx, dgamma, dbeta, ws, M, N, dres, dsum, st);
  else if (dtype == kF32) ln_bwd_t<float>(dy, s, mean, rstd, gamma, dx, dgamma, dbeta, ws, M, N, dres, dsum, st);
  else throw std::invalid_argument("layernorm: unsupported dtype");
}

}  // namespace ffk
