// Elementwise / activation / reduction-by-column kernels for gfx950.
//
// Parity: lib/kernels/src/cuda/ops/element_unary_kernels.cu (ReLU / Sigmoid /
// Tanh / ELU / GELU / Exp / ... forward + backward), cuda_helper.cu
// (gelu_forward_kernel, relu/sigmoid backward, apply_add, scale), linear bias
// gradient (linear_kernels.cu:280, a GEMM with a ones vector there), dropout
// (dropout_kernels.cu, cuDNN there), cast_kernels.cu.
// CDNA4 design: every kernel moves 16 B per lane; the activation backward and
// the bias gradient are one pass (column sums kept in registers across rows,
// then an LDS reduce over the block and one fp32 atomic per column);
// dropout regenerates its mask from a counter hash instead of storing it.
#include <algorithm>
#include <cstdlib>

#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace ffk {

enum Act : int { kIdentity = 0, kRelu = 1, kSigmoid = 2, kTanh = 3, kGelu = 4, kElu = 5, kExp = 6 };

__device__ __forceinline__ float act_apply(int op, float x, float alpha) {
  switch (op) {
    case kRelu: return x > 0.f ? x : 0.f;
    case kSigmoid: return 1.f / (1.f + __expf(-x));
    case kTanh: return fast_tanh(x);
    case kGelu: return gelu_tanh(x);
    case kElu: return x > 0.f ? x : alpha * (__expf(x) - 1.f);
    case kExp: return __expf(x);
    default: return x;
  }
}
// derivative w.r.t. the pre-activation x
__device__ __forceinline__ float act_grad(int op, float x, float alpha) {
  switch (op) {
    case kRelu: return x > 0.f ? 1.f : 0.f;
    case kSigmoid: {
      float s = 1.f / (1.f + __expf(-x));
      return s * (1.f - s);
    }
    case kTanh: {
      float t = fast_tanh(x);
      return 1.f - t * t;
    }
    case kGelu: return gelu_tanh_grad(x);
    case kElu: return x > 0.f ? 1.f : alpha * __expf(x);
    case kExp: return __expf(x);
    default: return 1.f;
  }
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* o);
template <>
__device__ __forceinline__ void ld8<bf16>(const bf16* p, float* o) {
  u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = u2f(v[i]);
}
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float* o) {
  f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i] = a[i];
    o[i + 4] = b[i];
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* o);
template <>
__device__ __forceinline__ void st8<bf16>(bf16* p, const float* o) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = f2bf(o[i]);
  *reinterpret_cast<bf16x8*>(p) = v;
}
template <>
__device__ __forceinline__ void st8<float>(float* p, const float* o) {
  f32x4 a, b;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    a[i] = o[i];
    b[i] = o[i + 4];
  }
  reinterpret_cast<f32x4*>(p)[0] = a;
  reinterpret_cast<f32x4*>(p)[1] = b;
}

// ---------------------------------------------------------------------------
// y = act(x [+ bias]); optionally pre = x + bias.  x: [M, N] row-major; n8 = M*N/8.
template <typename T, int OP>
__global__ __launch_bounds__(256) void bias_act_fwd_kernel(const T* __restrict__ x, const T* __restrict__ bias,
                                                           T* __restrict__ pre, T* __restrict__ y, int64_t n8,
                                                           int N, float alpha) {
  constexpr int op = OP;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    float v[8];
    ld8<T>(x + i * 8, v);
    if (bias) {
      float b[8];
      ld8<T>(bias + (i * 8) % N, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += b[k];
      if (pre) st8<T>(pre + i * 8, v);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = act_apply(op, v[k], alpha);
    st8<T>(y + i * 8, v);
  }
}

// dx = dy * act'(pre).  Element-wise (no bias grad).
template <typename T, int OP>
__global__ __launch_bounds__(256) void act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ pre,
                                                      T* __restrict__ dx, int64_t n8, float alpha) {
  constexpr int op = OP;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    float d[8], p[8];
    ld8<T>(dy + i * 8, d);
    ld8<T>(pre + i * 8, p);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] *= act_grad(op, p[k], alpha);
    st8<T>(dx + i * 8, d);
  }
}

// Column-sum (bias gradient), optionally fused with the activation backward:
//   g = dy * act'(pre) (if pre) ; dx = g (if dx) ; dbias += sum_rows g
// grid = (ceil(N/512), row_splits); block = 4 waves over the same 512 columns.
template <typename T, int OP>
__global__ __launch_bounds__(256) void colsum_act_kernel(const T* __restrict__ dy, const T* __restrict__ pre,
                                                         T* __restrict__ dx, float* __restrict__ dbias, int M,
                                                         int N, float alpha) {
  constexpr int op = OP;  // compile-time activation: no per-element switch
  __shared__ float red[4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + lane * 8;
  const bool active = col < N;
  float acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
  const int rows_per = (M + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * rows_per;
  const int r1 = min(M, r0 + rows_per);
  constexpr int U = 8;  // rows in flight per wave: 8 x 16 B (x2 with pre) per lane
  if (active) {
    for (int r = r0 + wave; r < r1; r += 4 * U) {
      float d[U][8], p[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + 4 * u;
        if (rr < r1) {
          const size_t off = static_cast<size_t>(rr) * N + col;
          ld8<T>(dy + off, d[u]);
          if (pre) ld8<T>(pre + off, p[u]);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) d[u][k] = p[u][k] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int rr = r + 4 * u;
        if (pre)
#pragma unroll
          for (int k = 0; k < 8; ++k) d[u][k] *= act_grad(op, p[u][k], alpha);
        if (dx && rr < r1) st8<T>(dx + static_cast<size_t>(rr) * N + col, d[u]);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] += d[u][k];
      }
    }
  }
  if (!dbias) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) red[wave][lane * 8 + k] = acc[k];
  __syncthreads();
  for (int j = threadIdx.x; j < 512; j += 256) {
    const int c = blockIdx.x * 512 + j;
    if (c < N) atomicAdd(dbias + c, red[0][j] + red[1][j] + red[2][j] + red[3][j]);
  }
}

// ---------------------------------------------------------------------------
// Dropout with a regenerated mask: y = x * keep / (1-p)
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n8,
                                                      float p, uint64_t seed) {
  const float scale = 1.f / (1.f - p);
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    float v[8];
    ld8<T>(x + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = uniform01(seed, i * 8 + k) >= p ? v[k] * scale : 0.f;
    st8<T>(y + i * 8, v);
  }
}

// ---------------------------------------------------------------------------
template <typename TI, typename TO>
__global__ __launch_bounds__(256) void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, int64_t n8) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    float v[8];
    ld8<TI>(x + i * 8, v);
    st8<TO>(y + i * 8, v);
  }
}

// y = a*x + b*y
template <typename T>
__global__ __launch_bounds__(256) void axpby_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n8, float a,
                                                    float b) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    float u[8], v[8];
    ld8<T>(x + i * 8, u);
    ld8<T>(y + i * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = a * u[k] + b * v[k];
    st8<T>(y + i * 8, v);
  }
}

// ---------------------------------------------------------------------------
static void need8(int64_t n, const char* what) {
  if (n % 8 != 0) throw std::invalid_argument(std::string(what) + ": element count must be a multiple of 8");
}

// op code -> compile-time constant (one kernel instantiation per activation)
template <typename F>
static void dispatch_act(int op, F&& f) {
  switch (op) {
    case kIdentity: f(std::integral_constant<int, kIdentity>{}); break;
    case kRelu: f(std::integral_constant<int, kRelu>{}); break;
    case kSigmoid: f(std::integral_constant<int, kSigmoid>{}); break;
    case kTanh: f(std::integral_constant<int, kTanh>{}); break;
    case kGelu: f(std::integral_constant<int, kGelu>{}); break;
    case kElu: f(std::integral_constant<int, kElu>{}); break;
    case kExp: f(std::integral_constant<int, kExp>{}); break;
    default: throw std::invalid_argument("unknown activation code");
  }
}

void bias_act_fwd(int dtype, const void* x, const void* bias, void* pre, void* y, int64_t M, int64_t N, int op,
                  float alpha, hipStream_t st) {
  need8(N, "bias_act_fwd");
  int64_t n8 = M * N / 8;
  int grid = grid_for(n8, 256, 256 * 8);
  dispatch_act(op, [&](auto opc) {
    constexpr int OPC = decltype(opc)::value;
    if (dtype == kBF16)
      hipLaunchKernelGGL((bias_act_fwd_kernel<bf16, OPC>), dim3(grid), dim3(256), 0, st, static_cast<const bf16*>(x),
                         static_cast<const bf16*>(bias), static_cast<bf16*>(pre), static_cast<bf16*>(y), n8,
                         static_cast<int>(N), alpha);
    else if (dtype == kF32)
      hipLaunchKernelGGL((bias_act_fwd_kernel<float, OPC>), dim3(grid), dim3(256), 0, st,
                         static_cast<const float*>(x), static_cast<const float*>(bias), static_cast<float*>(pre),
                         static_cast<float*>(y), n8, static_cast<int>(N), alpha);
    else throw std::invalid_argument("bias_act_fwd: dtype");
  });
  FFK_LAUNCH_CHECK("bias_act_fwd");
}

void act_bwd(int dtype, const void* dy, const void* pre, void* dx, int64_t n, int op, float alpha, hipStream_t st) {
  need8(n, "act_bwd");
  int grid = grid_for(n / 8, 256, 256 * 8);
  dispatch_act(op, [&](auto opc) {
    constexpr int OPC = decltype(opc)::value;
    if (dtype == kBF16)
      hipLaunchKernelGGL((act_bwd_kernel<bf16, OPC>), dim3(grid), dim3(256), 0, st, static_cast<const bf16*>(dy),
                         static_cast<const bf16*>(pre), static_cast<bf16*>(dx), n / 8, alpha);
    else if (dtype == kF32)
      hipLaunchKernelGGL((act_bwd_kernel<float, OPC>), dim3(grid), dim3(256), 0, st, static_cast<const float*>(dy),
                         static_cast<const float*>(pre), static_cast<float*>(dx), n / 8, alpha);
    else throw std::invalid_argument("act_bwd: dtype");
  });
  FFK_LAUNCH_CHECK("act_bwd");
}

void colsum_act(int dtype, const void* dy, const void* pre, void* dx, float* dbias, int64_t M, int64_t N, int op,
                float alpha, hipStream_t st) {
  need8(N, "colsum_act");
  int gx = static_cast<int>((N + 511) / 512);
  // row splits: ~FFK_COLSUM_BLOCKS blocks in total (default 4 per CU) and at
  // least 64 rows per block, so every wave streams >= 2 pipelined batches
  static const int64_t target = [] {
    const char* e = std::getenv("FFK_COLSUM_BLOCKS");
    return e ? std::max<int64_t>(1, std::atoll(e)) : int64_t(1024);
  }();
  int gy = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((target + gx - 1) / gx, (M + 63) / 64)));
  if (!pre) op = kIdentity;
  auto launch = [&](auto tag) {
    using T = decltype(tag);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(gx, gy), dim3(256), 0, st, static_cast<const T*>(dy), static_cast<const T*>(pre),
                         static_cast<T*>(dx), dbias, static_cast<int>(M), static_cast<int>(N), alpha);
    };
    switch (op) {
      case kIdentity: go(colsum_act_kernel<T, kIdentity>); break;
      case kRelu: go(colsum_act_kernel<T, kRelu>); break;
      case kSigmoid: go(colsum_act_kernel<T, kSigmoid>); break;
      case kTanh: go(colsum_act_kernel<T, kTanh>); break;
      case kGelu: go(colsum_act_kernel<T, kGelu>); break;
      case kElu: go(colsum_act_kernel<T, kElu>); break;
      case kExp: go(colsum_act_kernel<T, kExp>); break;
      default: throw std::invalid_argument("colsum_act: activation");
    }
  };
  if (dtype == kBF16) launch(bf16{});
  else if (dtype == kF32) launch(float{});
  else throw std::invalid_argument("colsum_act: dtype");
  FFK_LAUNCH_CHECK("colsum_act");
}

void dropout_fwd(int dtype, const void* x, void* y, int64_t n, float p, uint64_t seed, hipStream_t st) {
  need8(n, "dropout");
  int grid = grid_for(n / 8, 256, 256 * 8);
  if (dtype == kBF16)
    hipLaunchKernelGGL(dropout_kernel<bf16>, dim3(grid), dim3(256), 0, st, static_cast<const bf16*>(x),
                       static_cast<bf16*>(y), n / 8, p, seed);
  else if (dtype == kF32)
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<const float*>(x),
                       static_cast<float*>(y), n / 8, p, seed);
  else throw std::invalid_argument("dropout: dtype");
  FFK_LAUNCH_CHECK("dropout");
}

void cast(int dtype_in, int dtype_out, const void* x, void* y, int64_t n, hipStream_t st) {
  need8(n, "cast");
  int grid = grid_for(n / 8, 256, 256 * 8);
  if (dtype_in == kF32 && dtype_out == kBF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(grid), dim3(256), 0, st, static_cast<const float*>(x),
                       static_cast<bf16*>(y), n / 8);
  else if (dtype_in == kBF16 && dtype_out == kF32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(grid), dim3(256), 0, st, static_cast<const bf16*>(x),
                       static_cast<float*>(y), n / 8);
  else throw std::invalid_argument("cast: unsupported dtype pair");
  FFK_LAUNCH_CHECK("cast");
}

void axpby(int dtype, const void* x, void* y, int64_t n, float a, float b, hipStream_t st) {
  need8(n, "axpby");
  int grid = grid_for(n / 8, 256, 256 * 8);
  if (dtype == kBF16)
    hipLaunchKernelGGL(axpby_kernel<bf16>, dim3(grid), dim3(256), 0, st, static_cast<const bf16*>(x),
                       static_cast<bf16*>(y), n / 8, a, b);
  else if (dtype == kF32)
    hipLaunchKernelGGL(axpby_kernel<float>, dim3(grid), dim3(256), 0, st, static_cast<const float*>(x),
                       static_cast<float*>(y), n / 8, a, b);
  else throw std::invalid_argument("axpby: dtype");
  FFK_LAUNCH_CHECK("axpby");
}

// zero `bytes` bytes (16-B stores, a byte tail): gradient buffers between
// steps, without a runtime fill or a torch kernel in the step
__global__ __launch_bounds__(256) void zero_kernel(unsigned char* __restrict__ p, int64_t n16, int64_t bytes) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n16; i += stride)
    reinterpret_cast<u16x8*>(p)[i] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  if (blockIdx.x == 0)
    for (int64_t b = n16 * 16 + threadIdx.x; b < bytes; b += 256) p[b] = 0;
}

void zero_fill(void* p, int64_t bytes, hipStream_t st) {
  if (bytes <= 0) return;
  if (reinterpret_cast<uintptr_t>(p) % 16) throw std::invalid_argument("zero_fill: pointer must be 16-B aligned");
  const int64_t n16 = bytes / 16;
  const int grid = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n16 + 255) / 256, 4096)));
  hipLaunchKernelGGL(zero_kernel, dim3(grid), dim3(256), 0, st, static_cast<unsigned char*>(p), n16, bytes);
  FFK_LAUNCH_CHECK("zero_fill");
}

// ------------------------------------------------------------ narrow Linear
// Linear layers with a narrow output, N <= 8 (DLRM's 1-wide sigmoid head, any
// width the 16-B-row GEMM epilogues cannot write): GEMV-shaped and bound by
// reading X once, so no MFMA tile fits them.  W (K x N, row-major) is held in
// LDS transposed as fp32 [N][K]; one wave per row, each lane 8 consecutive k
// per 512-column step (16-B loads).  The activation (forward) and its
// derivative (backward, from the saved pre-activation) are applied in the
// same passes, so no separate element-wise kernel runs for the head.
constexpr int kNarrowLds = 16384;   // floats: K * N <= 16384

template <int N>
__device__ __forceinline__ void narrow_stage_w(const bf16* __restrict__ w, float* wt, int K) {
  for (int i = threadIdx.x; i < K * N; i += blockDim.x) wt[(i % N) * K + i / N] = bf2f(w[i]);
  __syncthreads();
}

template <int N>
__global__ __launch_bounds__(256) void narrow_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                         const float* __restrict__ bias, bf16* __restrict__ y,
                                                         bf16* __restrict__ pre, int M, int K, int act) {
  __shared__ float wt[kNarrowLds];
  narrow_stage_w<N>(w, wt, K);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int m = blockIdx.x * 4 + wv; m < M; m += gridDim.x * 4) {
    float acc[N];
#pragma unroll
    for (int n = 0; n < N; ++n) acc[n] = 0.f;
    const bf16* xr = x + static_cast<int64_t>(m) * K;
    for (int k0 = lane * 8; k0 < K; k0 += 512) {
      float xv[8];
      ld8<bf16>(xr + k0, xv);
#pragma unroll
      for (int n = 0; n < N; ++n)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[n] = __builtin_fmaf(xv[j], wt[n * K + k0 + j], acc[n]);
    }
    float v = 0.f;
#pragma unroll
    for (int n = 0; n < N; ++n) {
      const float t = wave_sum(acc[n]);
      if (lane == n) v = t;
    }
    if (lane < N) {
      if (bias) v += bias[lane];
      const int64_t o = static_cast<int64_t>(m) * N + lane;
      if (pre) pre[o] = f2bf(v);
      y[o] = f2bf(act_apply(act, v, 1.f));
    }
  }
}

// g[n] = dy[m, n] * act'(pre[m, n]) of one row (every lane of the wave)
template <int N>
__device__ __forceinline__ void narrow_row_grad(const bf16* __restrict__ dy, const bf16* __restrict__ pre, int64_t m,
                                                int act, float* g) {
#pragma unroll
  for (int n = 0; n < N; ++n) {
    float d = bf2f(dy[m * N + n]);
    if (act != kIdentity) d *= act_grad(act, bf2f(pre[m * N + n]), 1.f);
    g[n] = d;
  }
}

// dX[m, :] = g[m, :] W^T (+ beta dX)
template <int N>
__global__ __launch_bounds__(256) void narrow_dgrad_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ pre,
                                                           const bf16* __restrict__ w, bf16* __restrict__ dx, int M,
                                                           int K, int act, float beta) {
  __shared__ float wt[kNarrowLds];
  narrow_stage_w<N>(w, wt, K);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int m = blockIdx.x * 4 + wv; m < M; m += gridDim.x * 4) {
    float g[N];
    narrow_row_grad<N>(dy, pre, m, act, g);
    bf16* dr = dx + static_cast<int64_t>(m) * K;
    for (int k0 = lane * 8; k0 < K; k0 += 512) {
      float o[8], prev[8];
      if (beta != 0.f) ld8<bf16>(dr + k0, prev);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = beta != 0.f ? beta * prev[j] : 0.f;
#pragma unroll
        for (int n = 0; n < N; ++n) v = __builtin_fmaf(g[n], wt[n * K + k0 + j], v);
        o[j] = v;
      }
      u16x8 pk;
#pragma unroll
      for (int j = 0; j < 8; ++j) pk[j] = f2u(o[j]);
      *reinterpret_cast<u16x8*>(dr + k0) = pk;
    }
  }
}

// per row block b: part[b][k][n] = sum_{m in b} x[m, k] g[m, n] (k < K),
// part[b][K][n] = sum_{m in b} g[m, n] (the bias gradient)
template <int N>
__global__ __launch_bounds__(256) void narrow_wgrad_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                           const bf16* __restrict__ pre, float* __restrict__ part,
                                                           int M, int K, int act, int rows) {
  const int m0 = blockIdx.x * rows, m1 = min(M, m0 + rows);
  float* out = part + static_cast<int64_t>(blockIdx.x) * (K + 1) * N;
  for (int k0 = threadIdx.x * 8; k0 < K; k0 += 256 * 8) {
    float acc[8][N];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int n = 0; n < N; ++n) acc[j][n] = 0.f;
    for (int m = m0; m < m1; ++m) {
      float g[N], xv[8];
      narrow_row_grad<N>(dy, pre, m, act, g);
      ld8<bf16>(x + static_cast<int64_t>(m) * K + k0, xv);
#pragma unroll
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int n = 0; n < N; ++n) acc[j][n] = __builtin_fmaf(xv[j], g[n], acc[j][n]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int n = 0; n < N; ++n) out[(k0 + j) * N + n] = acc[j][n];
  }
  if (threadIdx.x < N) {
    float sb = 0.f;
    for (int m = m0; m < m1; ++m) {
      float g[N];
      narrow_row_grad<N>(dy, pre, m, act, g);
#pragma unroll
      for (int n = 0; n < N; ++n)
        if (n == static_cast<int>(threadIdx.x)) sb += g[n];
    }
    out[K * N + threadIdx.x] = sb;
  }
}

// dW = beta dW + sum_b part[b][:K]; db += sum_b part[b][K]
template <typename TW>
__global__ __launch_bounds__(256) void narrow_wgrad_finish_kernel(const float* __restrict__ part, int blocks, int KN,
                                                                  int N, TW* __restrict__ dw, float beta,
                                                                  float* __restrict__ db) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= KN + N) return;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;   // four independent chains: loads in flight
  const int64_t ld = KN + N;
  int b = 0;
  for (; b + 4 <= blocks; b += 4) {
    s0 += part[(b + 0) * ld + i];
    s1 += part[(b + 1) * ld + i];
    s2 += part[(b + 2) * ld + i];
    s3 += part[(b + 3) * ld + i];
  }
  for (; b < blocks; ++b) s0 += part[b * ld + i];
  const float s = (s0 + s1) + (s2 + s3);
  if (i < KN) {
    if (dw) {
      const float prev = beta != 0.f ? static_cast<float>(dw[i]) * beta : 0.f;
      dw[i] = static_cast<TW>(prev + s);
    }
  } else if (db) {
    db[i - KN] += s;
  }
}

template <typename F>
static void narrow_dispatch(int N, const char* what, F&& f) {
  switch (N) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: f(std::integral_constant<int, 5>{}); break;
    case 6: f(std::integral_constant<int, 6>{}); break;
    case 7: f(std::integral_constant<int, 7>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    default: throw std::invalid_argument(std::string(what) + ": N must be 1..8");
  }
}

static void narrow_check(int64_t M, int64_t K, int64_t N, const char* what) {
  if (M <= 0 || K <= 0 || K % 8 || N < 1 || N > 8 || K * N > kNarrowLds || M > (1LL << 31) - 1)
    throw std::invalid_argument(std::string(what) + ": shape outside the narrow-Linear kernel (K % 8, K*N <= 16384)");
}

static int narrow_grid(int64_t M) { return static_cast<int>(std::min<int64_t>((M + 3) / 4, 1024)); }

void narrow_linear_fwd(const void* x, const void* w, const float* bias, void* y, void* pre, int64_t M, int64_t K,
                       int64_t N, int act, hipStream_t st) {
  narrow_check(M, K, N, "narrow_linear_fwd");
  narrow_dispatch(static_cast<int>(N), "narrow_linear_fwd", [&](auto nn) {
    hipLaunchKernelGGL(narrow_fwd_kernel<decltype(nn)::value>, dim3(narrow_grid(M)), dim3(256), 0, st,
                       static_cast<const bf16*>(x), static_cast<const bf16*>(w), bias, static_cast<bf16*>(y),
                       static_cast<bf16*>(pre), static_cast<int>(M), static_cast<int>(K), act);
  });
  FFK_LAUNCH_CHECK("narrow_linear_fwd");
}

void narrow_linear_dgrad(const void* dy, const void* pre, const void* w, void* dx, int64_t M, int64_t K, int64_t N,
                         int act, float beta, hipStream_t st) {
  narrow_check(M, K, N, "narrow_linear_dgrad");
  narrow_dispatch(static_cast<int>(N), "narrow_linear_dgrad", [&](auto nn) {
    hipLaunchKernelGGL(narrow_dgrad_kernel<decltype(nn)::value>, dim3(narrow_grid(M)), dim3(256), 0, st,
                       static_cast<const bf16*>(dy), static_cast<const bf16*>(pre), static_cast<const bf16*>(w),
                       static_cast<bf16*>(dx), static_cast<int>(M), static_cast<int>(K), act, beta);
  });
  FFK_LAUNCH_CHECK("narrow_linear_dgrad");
}

int narrow_wgrad_blocks(int64_t M) { return static_cast<int>(std::min<int64_t>(64, (M + 15) / 16)); }

void narrow_linear_wgrad(const void* x, const void* dy, const void* pre, float* part, int blocks, void* dw,
                         int dw_dtype, float beta, float* db, int64_t M, int64_t K, int64_t N, int act,
                         hipStream_t st) {
  narrow_check(M, K, N, "narrow_linear_wgrad");
  if (blocks < 1) throw std::invalid_argument("narrow_linear_wgrad: blocks");
  const int rows = static_cast<int>((M + blocks - 1) / blocks);
  narrow_dispatch(static_cast<int>(N), "narrow_linear_wgrad", [&](auto nn) {
    hipLaunchKernelGGL(narrow_wgrad_kernel<decltype(nn)::value>, dim3(blocks), dim3(256), 0, st,
                       static_cast<const bf16*>(x), static_cast<const bf16*>(dy), static_cast<const bf16*>(pre), part,
                       static_cast<int>(M), static_cast<int>(K), act, rows);
  });
  FFK_LAUNCH_CHECK("narrow_linear_wgrad");
  const int KN = static_cast<int>(K * N);
  const int g = (KN + static_cast<int>(N) + 255) / 256;
  if (dw_dtype == kF32 || dw == nullptr)
    hipLaunchKernelGGL(narrow_wgrad_finish_kernel<float>, dim3(g), dim3(256), 0, st, part, blocks, KN,
                       static_cast<int>(N), static_cast<float*>(dw), beta, db);
  else if (dw_dtype == kBF16)
    hipLaunchKernelGGL(narrow_wgrad_finish_kernel<bf16>, dim3(g), dim3(256), 0, st, part, blocks, KN,
                       static_cast<int>(N), static_cast<bf16*>(dw), beta, db);
  else
    throw std::invalid_argument("narrow_linear_wgrad: dW dtype");
  FFK_LAUNCH_CHECK("narrow_linear_wgrad_finish");
}

}  // namespace ffk
