// General tensor operators for gfx950: broadcast element-wise binary ops and
// their gradients, N-d permutation, slice copies (concat / split), reverse,
// gather / scatter-add, axis reductions, per-row top-k, scalar / unary math,
// MSE loss + metrics, and on-device parameter initialisers.
//
// Parity: element_binary_kernels.cu (cudnnOpTensor +
// elewise_binary_backward_kernel :26, broadcast-reduced gradients),
// element_unary_kernels.cu (scalar / unary forward + backward :99-204),
// transpose_kernels.cu :45, concat/split via cuda_helper copy_with_stride /
// add_with_stride :144-159, reverse_kernels.cu :24, gather_kernels.cu :26/:53,
// reduce_kernels.cu (cudnnReduceTensor), topk_kernels.cu :342/:410,
// loss_function_kernels.cu (MSE) + metrics_functions.cu, initializer_kernels.cu
// (curand uniform / normal, constant, zero).
//
// CDNA4 notes: contiguous same-shape and row-broadcast (bias-like) binary ops
// take a 16-byte vector path; everything else uses an N-d (<= 6) strided
// index decomposition.  Reductions keep one thread per output element walking
// the reduced sub-space (coalesced over the innermost kept dim).  Top-k is one
// wave per row (64-lane arg-max, k rounds).  Initialisers hash (seed, global
// element index) so every shard of a parameter generates exactly its slice of
// the same logical tensor, on any rank, with no broadcast.
#include <algorithm>
#include <cmath>
#include <string>
#include <type_traits>

#include "common.h"
#include "kernels.h"

namespace ffk {

namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p) {
  if constexpr (std::is_same<T, float>::value) return *p;
  else return bf2f(*p);
}
template <typename T>
__device__ __forceinline__ void st(T* p, float v) {
  if constexpr (std::is_same<T, float>::value) *p = v;
  else *p = f2bf(v);
}

__device__ __forceinline__ float bin_op(int op, float a, float b) {
  switch (op) {
    case 0: return a + b;
    case 1: return a - b;
    case 2: return a * b;
    case 3: return a / b;
    case 4: return fmaxf(a, b);
    case 5: return fminf(a, b);
    case 6: return a == b ? 1.f : 0.f;
    case 7: return a > b ? 1.f : 0.f;
    case 8: return a < b ? 1.f : 0.f;
    default: return 0.f;
  }
}

__device__ __forceinline__ int64_t nd_offset(int64_t i, const NdShape& s, const int64_t* strides) {
  int64_t off = 0;
  for (int d = s.nd - 1; d >= 0; --d) {
    const int64_t c = i % s.size[d];
    i /= s.size[d];
    off += c * strides[d];
  }
  return off;
}

// ---------------------------------------------------------------- binary
template <typename T>
__global__ __launch_bounds__(256) void binary_nd_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                        T* __restrict__ y, NdShape s, NdStrides sa, NdStrides sb,
                                                        int64_t n, int op) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256)
    st<T>(y + i, bin_op(op, ld<T>(a + nd_offset(i, s, sa.s)), ld<T>(b + nd_offset(i, s, sb.s))));
}

// same-shape contiguous operands: 8 elements (16 B of bf16) per thread
template <typename T>
__device__ __forceinline__ void ld8v(const T* p, float* o) {
  if constexpr (std::is_same<T, float>::value) {
    const f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[i] = a[i];
      o[i + 4] = b[i];
    }
  } else {
    const u16x8 v = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = u2f(v[i]);
  }
}
template <typename T>
__device__ __forceinline__ void st8v(T* p, const float* o) {
  if constexpr (std::is_same<T, float>::value) {
    reinterpret_cast<f32x4*>(p)[0] = f32x4{o[0], o[1], o[2], o[3]};
    reinterpret_cast<f32x4*>(p)[1] = f32x4{o[4], o[5], o[6], o[7]};
  } else {
    bf16x8 v;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = f2bf(o[i]);
    *reinterpret_cast<bf16x8*>(p) = v;
  }
}
template <typename T>
__global__ __launch_bounds__(256) void binary_flat8_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                           T* __restrict__ y, int64_t n8, int op) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    float x[8], z[8];
    ld8v<T>(a + i * 8, x);
    ld8v<T>(b + i * 8, z);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] = bin_op(op, x[k], z[k]);
    st8v<T>(y + i * 8, x);
  }
}

// gradient of a binary op w.r.t. a (which = 0) or b (which = 1), full output shape
template <typename T>
__global__ __launch_bounds__(256) void binary_grad_nd_kernel(const T* __restrict__ dy, const T* __restrict__ a,
                                                             const T* __restrict__ b, float* __restrict__ g,
                                                             NdShape s, NdStrides sa, NdStrides sb, int64_t n, int op,
                                                             int which) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const float d = ld<T>(dy + i);
    const float av = ld<T>(a + nd_offset(i, s, sa.s)), bv = ld<T>(b + nd_offset(i, s, sb.s));
    float r = 0.f;
    switch (op) {
      case 0: r = d; break;
      case 1: r = which ? -d : d; break;
      case 2: r = which ? d * av : d * bv; break;
      case 3: r = which ? -d * av / (bv * bv) : d / bv; break;
      case 4: r = (which ? (bv > av) : (av >= bv)) ? d : 0.f; break;
      case 5: r = (which ? (bv < av) : (av <= bv)) ? d : 0.f; break;
      default: r = 0.f;
    }
    g[i] = r;
  }
}

// out[j] = sum over the broadcast sub-space of full[...]; full has shape `s`
// (the op's output), the target keeps dims where keep[d] == 1.
template <typename T>
__global__ __launch_bounds__(256) void sum_to_kernel(const float* __restrict__ full, T* __restrict__ out, NdShape s,
                                                     NdShape keep_shape, NdShape red_shape, NdStrides full_st,
                                                     int64_t n_out, int64_t n_red, float beta) {
  for (int64_t j = blockIdx.x * 256 + threadIdx.x; j < n_out; j += static_cast<int64_t>(gridDim.x) * 256) {
    // coordinates of the kept dims (reduced dims have size 1 in keep_shape)
    int64_t base = 0, jj = j;
    for (int d = keep_shape.nd - 1; d >= 0; --d) {
      const int64_t c = jj % keep_shape.size[d];
      jj /= keep_shape.size[d];
      base += c * full_st.s[d];
    }
    float acc = 0.f;
    for (int64_t r = 0; r < n_red; ++r) {
      int64_t off = base, rr = r;
      for (int d = red_shape.nd - 1; d >= 0; --d) {
        const int64_t c = rr % red_shape.size[d];
        rr /= red_shape.size[d];
        off += c * full_st.s[d];
      }
      acc += full[off];
    }
    if (beta != 0.f) acc += beta * ld<T>(out + j);
    st<T>(out + j, acc);
  }
  (void)s;
}

// ------------------------------------------------------- permute / copies
template <typename T>
__global__ __launch_bounds__(256) void permute_kernel(const T* __restrict__ x, T* __restrict__ y, NdShape out_shape,
                                                      NdStrides in_strides_permuted, int64_t n) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256)
    y[i] = x[nd_offset(i, out_shape, in_strides_permuted.s)];
}

// y[o][off + j][i] (+)= x[o][j][i] for x of [outer, len, inner], y of [outer, total, inner]
template <typename T>
__global__ __launch_bounds__(256) void slice_copy_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t outer,
                                                         int64_t len, int64_t inner, int64_t total, int64_t off,
                                                         int to_slice, int accumulate) {
  const int64_t n = outer * len * inner;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t in = i % inner, j = (i / inner) % len, o = i / (inner * len);
    const int64_t big = (o * total + off + j) * inner + in;
    if (to_slice) {  // big tensor -> slice
      if (accumulate) st<T>(y + i, ld<T>(y + i) + ld<T>(x + big));
      else y[i] = x[big];
    } else {         // slice -> big tensor
      if (accumulate) st<T>(y + big, ld<T>(y + big) + ld<T>(x + i));
      else y[big] = x[i];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void reverse_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t outer,
                                                      int64_t len, int64_t inner) {
  const int64_t n = outer * len * inner;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t in = i % inner, j = (i / inner) % len, o = i / (inner * len);
    y[(o * len + (len - 1 - j)) * inner + in] = x[i];
  }
}

// gather along `dim`: x [outer, len_x, inner], idx/y [outer, len_i, inner]
template <typename T, typename I>
__global__ __launch_bounds__(256) void gather_kernel(const T* __restrict__ x, const I* __restrict__ idx,
                                                     T* __restrict__ y, int64_t outer, int64_t len_x, int64_t len_i,
                                                     int64_t inner) {
  const int64_t n = outer * len_i * inner;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t in = i % inner, o = i / (inner * len_i);
    int64_t k = static_cast<int64_t>(idx[i]);
    k = k < 0 ? k + len_x : k;
    if (k >= 0 && k < len_x) y[i] = x[(o * len_x + k) * inner + in];
    else st<T>(y + i, 0.f);
  }
}

template <typename T, typename I>
__global__ __launch_bounds__(256) void scatter_add_kernel(const T* __restrict__ dy, const I* __restrict__ idx,
                                                          float* __restrict__ dx, int64_t outer, int64_t len_x,
                                                          int64_t len_i, int64_t inner) {
  const int64_t n = outer * len_i * inner;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t in = i % inner, o = i / (inner * len_i);
    int64_t k = static_cast<int64_t>(idx[i]);
    k = k < 0 ? k + len_x : k;
    if (k >= 0 && k < len_x) atomicAdd(dx + (o * len_x + k) * inner + in, ld<T>(dy + i));
  }
}

// ------------------------------------------------------------- reductions
// x viewed as [outer, red, inner]; op: 0 sum, 1 mean, 2 max, 3 min, 4 prod
template <typename T>
__global__ __launch_bounds__(256) void reduce_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t outer,
                                                     int64_t red, int64_t inner, int op) {
  const int64_t n = outer * inner;
  for (int64_t j = blockIdx.x * 256 + threadIdx.x; j < n; j += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t in = j % inner, o = j / inner;
    const T* p = x + o * red * inner + in;
    float acc = op == 2 ? -INFINITY : (op == 3 ? INFINITY : (op == 4 ? 1.f : 0.f));
    for (int64_t r = 0; r < red; ++r) {
      const float v = ld<T>(p + r * inner);
      acc = op == 2 ? fmaxf(acc, v) : (op == 3 ? fminf(acc, v) : (op == 4 ? acc * v : acc + v));
    }
    if (op == 1) acc /= static_cast<float>(red);
    st<T>(y + j, acc);
  }
}

// ------------------------------------------------------------------ top-k
// one wave per row; values descending (sorted), indices int64
template <typename T>
__global__ __launch_bounds__(256) void topk_kernel(const T* __restrict__ x, T* __restrict__ vals,
                                                   int64_t* __restrict__ idx, int64_t rows, int n, int k) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + row * n;
  int last_idx = -1;
  float last_val = INFINITY;
  for (int t = 0; t < k; ++t) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int j = lane; j < n; j += 64) {
      const float v = ld<T>(xr + j);
      // strictly after the previous pick in (value desc, index asc) order
      const bool after = v < last_val || (v == last_val && j > last_idx);
      if (after && (v > best || (v == best && j < bi))) {
        best = v;
        bi = j;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ov > best || (ov == best && oi < bi)) {
        best = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      st<T>(vals + row * k + t, best);
      idx[row * k + t] = bi;
    }
    last_val = best;
    last_idx = bi;
  }
}

// --------------------------------------------------------- unary / scalar
// op: 0 scalar_add, 1 scalar_sub, 2 scalar_mul, 3 scalar_div, 4 pow, 5 log,
//     6 sqrt, 7 rsqrt, 8 sin, 9 cos, 10 leaky_relu, 11 ceil, 12 round, 13 identity
__device__ __forceinline__ float un_op(int op, float x, float s) {
  switch (op) {
    case 0: return x + s;
    case 1: return x - s;
    case 2: return x * s;
    case 3: return x / s;
    case 4: return __powf(x, s);
    case 5: return __logf(x);
    case 6: return sqrtf(x);
    case 7: return rsqrtf(x);
    case 8: return __sinf(x);
    case 9: return __cosf(x);
    case 10: return x > 0.f ? x : s * x;
    case 11: return ceilf(x);
    case 12: return rintf(x);
    default: return x;
  }
}
__device__ __forceinline__ float un_grad(int op, float x, float s) {
  switch (op) {
    case 0: case 1: case 13: return 1.f;
    case 2: return s;
    case 3: return 1.f / s;
    case 4: return s * __powf(x, s - 1.f);
    case 5: return 1.f / x;
    case 6: return 0.5f * rsqrtf(x);
    case 7: { const float r = rsqrtf(x); return -0.5f * r * r * r; }
    case 8: return __cosf(x);
    case 9: return -__sinf(x);
    case 10: return x > 0.f ? 1.f : s;
    default: return 0.f;  // ceil / round
  }
}

template <typename T>
__global__ __launch_bounds__(256) void unary_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                    T* __restrict__ y, int64_t n, int op, float s, int backward) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const float v = ld<T>(x + i);
    st<T>(y + i, backward ? ld<T>(dy + i) * un_grad(op, v, s) : un_op(op, v, s));
  }
}

// ------------------------------------------------------------------- MSE
// grad = scale * (p - y); metrics[0] += sum (p-y)^2, metrics[1] += sum |p-y|
// (``full``: the loss-metrics block of ops/loss.py, slots loss 0, count 2,
// squared error 3, absolute error 4: loss += sum (p-y)^2 / C, count += rows,
// so no element-wise torch kernels run around the loss).  Labels may be fp32
// or the prediction's dtype.
template <typename T, typename L>
__global__ __launch_bounds__(256) void mse_kernel(const T* __restrict__ p, const L* __restrict__ y,
                                                  T* __restrict__ grad, float* __restrict__ metrics, int64_t n,
                                                  float scale, int full, float inv_c, float rows) {
  float se = 0.f, ae = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const float d = ld<T>(p + i) - static_cast<float>(y[i]);
    se += d * d;
    ae += fabsf(d);
    if (grad) st<T>(grad + i, scale * d);
  }
  __shared__ float red[8];
  se = block_sum<256>(se, red);
  ae = block_sum<256>(ae, red + 4);
  if (threadIdx.x == 0 && metrics) {
    if (full) {
      atomicAdd(metrics + 0, se * inv_c);
      if (blockIdx.x == 0) atomicAdd(metrics + 2, rows);
      atomicAdd(metrics + 3, se);
      atomicAdd(metrics + 4, ae);
    } else {
      atomicAdd(metrics + 0, se);
      atomicAdd(metrics + 1, ae);
    }
  }
}

// ------------------------------------------------------------ initialisers
// kind: 0 uniform[a,b), 1 normal(a, b), 2 truncated normal(a, b) in [c, d],
//       3 constant a.  The element's GLOBAL linear index in the full logical
//       tensor is computed from the piece box, so shards agree.
template <typename T>
__global__ __launch_bounds__(256) void init_kernel(T* __restrict__ out, NdShape piece, NdShape full,
                                                   NdStrides box_lo, int64_t n, int kind, uint64_t seed, float a,
                                                   float b, float c, float d) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    int64_t rem = i, g = 0, mul = 1;
    for (int dd = piece.nd - 1; dd >= 0; --dd) {
      const int64_t cc = rem % piece.size[dd];
      rem /= piece.size[dd];
      g += (cc + box_lo.s[dd]) * mul;
      mul *= full.size[dd];
    }
    float v;
    if (kind == 3) {
      v = a;
    } else if (kind == 0) {
      v = a + (b - a) * uniform01(seed, 2 * g);
    } else {
      // Box-Muller from two counter-based uniforms; truncated: re-draw (bounded)
      float z = 0.f;
      for (int attempt = 0; attempt < 16; ++attempt) {
        const float u1 = fmaxf(uniform01(seed ^ (0x9E37ULL * (attempt + 1)), 2 * g), 1e-7f);
        const float u2 = uniform01(seed ^ (0x9E37ULL * (attempt + 1)), 2 * g + 1);
        z = a + b * sqrtf(-2.f * __logf(u1)) * __cosf(6.283185307f * u2);
        if (kind != 2 || (z >= c && z <= d)) break;
        z = fminf(fmaxf(z, c), d);
      }
      v = z;
    }
    st<T>(out + i, v);
  }
}

template <typename F>
void by_dtype(int dtype, const char* what, F&& f) {
  if (dtype == kBF16) f(bf16{});
  else if (dtype == kF32) f(float{});
  else throw std::invalid_argument(std::string(what) + ": dtype");
}

int grid1(int64_t n) { return grid_for(n, 256, 256); }

}  // namespace

void binary_nd(int dtype, const void* a, const void* b, void* y, const NdShape& s, const NdStrides& sa,
               const NdStrides& sb, int op, hipStream_t st) {
  int64_t n = 1;
  for (int d = 0; d < s.nd; ++d) n *= s.size[d];
  if (n == 0) return;
  // both operands contiguous with the output shape -> 16-byte vector path
  bool flat = true;
  int64_t acc = 1;
  for (int d = s.nd - 1; d >= 0; --d) {
    if (s.size[d] != 1 && (sa.s[d] != acc || sb.s[d] != acc)) flat = false;
    acc *= s.size[d];
  }
  const bool aligned = ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b) |
                         reinterpret_cast<uintptr_t>(y)) & 15) == 0;
  by_dtype(dtype, "binary", [&](auto t) {
    using T = decltype(t);
    if (flat && aligned && n % 8 == 0)
      hipLaunchKernelGGL(binary_flat8_kernel<T>, dim3(grid_for(n / 8, 256, 256 * 8)), dim3(256), 0, st,
                         static_cast<const T*>(a), static_cast<const T*>(b), static_cast<T*>(y), n / 8, op);
    else
      hipLaunchKernelGGL(binary_nd_kernel<T>, dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(a),
                         static_cast<const T*>(b), static_cast<T*>(y), s, sa, sb, n, op);
  });
  FFK_LAUNCH_CHECK("binary_nd");
}

void binary_grad_nd(int dtype, const void* dy, const void* a, const void* b, float* g, const NdShape& s,
                    const NdStrides& sa, const NdStrides& sb, int op, int which, hipStream_t st) {
  int64_t n = 1;
  for (int d = 0; d < s.nd; ++d) n *= s.size[d];
  if (n == 0) return;
  by_dtype(dtype, "binary_grad", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(binary_grad_nd_kernel<T>, dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(dy),
                       static_cast<const T*>(a), static_cast<const T*>(b), g, s, sa, sb, n, op, which);
  });
  FFK_LAUNCH_CHECK("binary_grad_nd");
}

void sum_to(int dtype, const float* full, void* out, const NdShape& s, const NdShape& target, float beta,
            hipStream_t st) {
  NdShape keep = s, red = s;
  NdStrides fs{};
  int64_t stride = 1, n_out = 1, n_red = 1;
  for (int d = s.nd - 1; d >= 0; --d) {
    fs.s[d] = stride;
    stride *= s.size[d];
  }
  for (int d = 0; d < s.nd; ++d) {
    const bool kept = target.size[d] == s.size[d];
    keep.size[d] = kept ? s.size[d] : 1;
    red.size[d] = kept ? 1 : s.size[d];
    n_out *= keep.size[d];
    n_red *= red.size[d];
  }
  by_dtype(dtype, "sum_to", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(sum_to_kernel<T>, dim3(grid1(n_out)), dim3(256), 0, st, full, static_cast<T*>(out), s, keep,
                       red, fs, n_out, n_red, beta);
  });
  FFK_LAUNCH_CHECK("sum_to");
}

void permute_nd(int dtype, const void* x, void* y, const NdShape& out_shape, const NdStrides& in_strides_permuted,
                hipStream_t st) {
  int64_t n = 1;
  for (int d = 0; d < out_shape.nd; ++d) n *= out_shape.size[d];
  if (n == 0) return;
  by_dtype(dtype, "permute", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(permute_kernel<T>, dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(x),
                       static_cast<T*>(y), out_shape, in_strides_permuted, n);
  });
  FFK_LAUNCH_CHECK("permute");
}

// Every piece of a concat / split in one launch (blockIdx.y = piece): a
// DLRM interaction concatenates 9 feature blocks forward and splits them
// back in the backward pass, 18 tiny launches per step as single copies.
template <typename T>
__global__ __launch_bounds__(256) void slice_copy_multi_kernel(SlicePieces p, T* __restrict__ big, int64_t outer,
                                                               int64_t inner, int64_t total, int to_slice) {
  const int k = blockIdx.y;
  T* sl = static_cast<T*>(p.ptr[k]);
  const int64_t len = p.len[k], off = p.off[k];
  const int64_t n = outer * len * inner;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t in = i % inner, j = (i / inner) % len, o = i / (inner * len);
    const int64_t b = (o * total + off + j) * inner + in;
    if (to_slice) sl[i] = big[b];
    else big[b] = sl[i];
  }
}

void slice_copy_multi(int dtype, void* big, const SlicePieces& p, int64_t outer, int64_t inner, int64_t total,
                      int to_slice, hipStream_t st) {
  if (p.n <= 0) return;
  if (p.n > kMaxSlicePieces) throw std::invalid_argument("slice_copy_multi: too many pieces");
  int64_t most = 0;
  for (int k = 0; k < p.n; ++k) most = std::max(most, outer * p.len[k] * inner);
  if (most == 0) return;
  by_dtype(dtype, "slice_copy_multi", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(slice_copy_multi_kernel<T>, dim3(grid1(most), p.n), dim3(256), 0, st, p, static_cast<T*>(big),
                       outer, inner, total, to_slice);
  });
  FFK_LAUNCH_CHECK("slice_copy_multi");
}

void slice_copy(int dtype, const void* x, void* y, int64_t outer, int64_t len, int64_t inner, int64_t total,
                int64_t off, int to_slice, int accumulate, hipStream_t st) {
  const int64_t n = outer * len * inner;
  if (n == 0) return;
  by_dtype(dtype, "slice_copy", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(slice_copy_kernel<T>, dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(x),
                       static_cast<T*>(y), outer, len, inner, total, off, to_slice, accumulate);
  });
  FFK_LAUNCH_CHECK("slice_copy");
}

void reverse_axis(int dtype, const void* x, void* y, int64_t outer, int64_t len, int64_t inner, hipStream_t st) {
  const int64_t n = outer * len * inner;
  if (n == 0) return;
  by_dtype(dtype, "reverse", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(reverse_kernel<T>, dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(x),
                       static_cast<T*>(y), outer, len, inner);
  });
  FFK_LAUNCH_CHECK("reverse");
}

void gather_axis(int dtype, int index_bits, const void* x, const void* idx, void* y, int64_t outer, int64_t len_x,
                 int64_t len_i, int64_t inner, hipStream_t st) {
  const int64_t n = outer * len_i * inner;
  if (n == 0) return;
  by_dtype(dtype, "gather", [&](auto t) {
    using T = decltype(t);
    if (index_bits == 64)
      hipLaunchKernelGGL((gather_kernel<T, int64_t>), dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(x),
                         static_cast<const int64_t*>(idx), static_cast<T*>(y), outer, len_x, len_i, inner);
    else
      hipLaunchKernelGGL((gather_kernel<T, int32_t>), dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(x),
                         static_cast<const int32_t*>(idx), static_cast<T*>(y), outer, len_x, len_i, inner);
  });
  FFK_LAUNCH_CHECK("gather");
}

void scatter_add_axis(int dtype, int index_bits, const void* dy, const void* idx, float* dx, int64_t outer,
                      int64_t len_x, int64_t len_i, int64_t inner, hipStream_t st) {
  const int64_t n = outer * len_i * inner;
  if (n == 0) return;
  by_dtype(dtype, "scatter_add", [&](auto t) {
    using T = decltype(t);
    if (index_bits == 64)
      hipLaunchKernelGGL((scatter_add_kernel<T, int64_t>), dim3(grid1(n)), dim3(256), 0, st,
                         static_cast<const T*>(dy), static_cast<const int64_t*>(idx), dx, outer, len_x, len_i, inner);
    else
      hipLaunchKernelGGL((scatter_add_kernel<T, int32_t>), dim3(grid1(n)), dim3(256), 0, st,
                         static_cast<const T*>(dy), static_cast<const int32_t*>(idx), dx, outer, len_x, len_i, inner);
  });
  FFK_LAUNCH_CHECK("scatter_add");
}

void reduce_axis(int dtype, const void* x, void* y, int64_t outer, int64_t red, int64_t inner, int op,
                 hipStream_t st) {
  const int64_t n = outer * inner;
  if (n == 0) return;
  by_dtype(dtype, "reduce", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(reduce_kernel<T>, dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(x),
                       static_cast<T*>(y), outer, red, inner, op);
  });
  FFK_LAUNCH_CHECK("reduce");
}

void topk_rows(int dtype, const void* x, void* vals, int64_t* idx, int64_t rows, int n, int k, hipStream_t st) {
  if (rows == 0) return;
  if (k > n) throw std::invalid_argument("topk: k > row length");
  const int grid = static_cast<int>((rows + 3) / 4);
  by_dtype(dtype, "topk", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(topk_kernel<T>, dim3(grid), dim3(256), 0, st, static_cast<const T*>(x), static_cast<T*>(vals),
                       idx, rows, n, k);
  });
  FFK_LAUNCH_CHECK("topk");
}

void unary_op(int dtype, const void* x, const void* dy, void* y, int64_t n, int op, float scalar, int backward,
              hipStream_t st) {
  if (n == 0) return;
  by_dtype(dtype, "unary", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(unary_kernel<T>, dim3(grid1(n)), dim3(256), 0, st, static_cast<const T*>(x),
                       static_cast<const T*>(dy), static_cast<T*>(y), n, op, scalar, backward);
  });
  FFK_LAUNCH_CHECK("unary");
}

void mse_loss(int dtype, const void* pred, const void* label, void* grad, float* metrics, int64_t n, float scale,
              hipStream_t st) {
  mse_loss_full(dtype, dtype, pred, label, grad, metrics, n, scale, 0, 1, 0, st);
}

void mse_loss_full(int dtype, int label_dtype, const void* pred, const void* label, void* grad, float* metrics,
                   int64_t n, float scale, int full, int64_t cols, int64_t rows, hipStream_t st) {
  if (n == 0) return;
  by_dtype(dtype, "mse", [&](auto t) {
    using T = decltype(t);
    auto go = [&](auto l) {
      using L = decltype(l);
      hipLaunchKernelGGL((mse_kernel<T, L>), dim3(std::min(grid1(n), 1024)), dim3(256), 0, st,
                         static_cast<const T*>(pred), static_cast<const L*>(label), static_cast<T*>(grad), metrics, n,
                         scale, full, 1.f / static_cast<float>(std::max<int64_t>(cols, 1)), static_cast<float>(rows));
    };
    if (label_dtype == dtype) go(T{});
    else if (label_dtype == kF32) go(float{});
    else throw std::invalid_argument("mse: label dtype");
  });
  FFK_LAUNCH_CHECK("mse");
}

void init_tensor(int dtype, void* out, const NdShape& piece, const NdShape& full, const NdStrides& box_lo, int kind,
                 uint64_t seed, float a, float b, float c, float d, hipStream_t st) {
  int64_t n = 1;
  for (int i = 0; i < piece.nd; ++i) n *= piece.size[i];
  if (n == 0) return;
  by_dtype(dtype, "init", [&](auto t) {
    using T = decltype(t);
    hipLaunchKernelGGL(init_kernel<T>, dim3(grid1(n)), dim3(256), 0, st, static_cast<T*>(out), piece, full, box_lo,
                       n, kind, seed, a, b, c, d);
  });
  FFK_LAUNCH_CHECK("init");
}

}  // namespace ffk
