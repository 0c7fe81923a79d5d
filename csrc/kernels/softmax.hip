// Softmax and fused softmax + cross-entropy (loss, gradient, metrics) for gfx950.
//
// Parity: lib/kernels/src/cuda/ops/softmax_kernels.cu (forward via cuDNN; its
// backward is a plain copy that is only right when fused with CE, :63-72),
// lib/kernels/src/cuda/loss_function_kernels.cu (sparse CCE grad = softmax -
// onehot, scaled by 1/batch, :21-137) and metrics_functions.cu (accuracy and
// CCE accumulated with atomics, :23-185).
// Here: a real softmax backward (dx = y * (dy - <dy, y>)), and one fused
// kernel for the training loss: a single online max/sum pass over the logits
// row (16-byte loads), then the gradient written IN PLACE over the logits
// (no separate probability tensor: for BERT's 30k-wide vocabulary that saves
// a full [tokens, vocab] buffer), plus loss-sum / correct-count atomics.
#include "common.h"
#include "kernels.h"

namespace ffk {

struct MaxSum {
  float m, s;
};
__device__ __forceinline__ MaxSum ms_merge(MaxSum a, MaxSum b) {
  float m = fmaxf(a.m, b.m);
  float s = (a.m == -INFINITY ? 0.f : a.s * __expf(a.m - m)) + (b.m == -INFINITY ? 0.f : b.s * __expf(b.m - m));
  return {m, s};
}

template <typename T>
__device__ __forceinline__ float ldf(const T* p);
template <>
__device__ __forceinline__ float ldf<bf16>(const bf16* p) {
  return bf2f(*p);
}
template <>
__device__ __forceinline__ float ldf<float>(const float* p) {
  return *p;
}
template <typename T>
__device__ __forceinline__ void stf(T* p, float v);
template <>
__device__ __forceinline__ void stf<bf16>(bf16* p, float v) {
  *p = f2bf(v);
}
template <>
__device__ __forceinline__ void stf<float>(float* p, float v) {
  *p = v;
}

// Block-level (max, sum, argmax) reduction for 256 threads.
__device__ __forceinline__ void block_reduce_msa(MaxSum& ms, float& best, int& best_idx) {
  __shared__ float sm[4], ss[4], sb[4];
  __shared__ int si[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    MaxSum other{__shfl_xor(ms.m, o, 64), __shfl_xor(ms.s, o, 64)};
    ms = ms_merge(ms, other);
    float ob = __shfl_xor(best, o, 64);
    int oi = __shfl_xor(best_idx, o, 64);
    if (ob > best || (ob == best && oi < best_idx)) {
      best = ob;
      best_idx = oi;
    }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = ms.m;
    ss[w] = ms.s;
    sb[w] = best;
    si[w] = best_idx;
  }
  __syncthreads();
  ms = {sm[0], ss[0]};
  best = sb[0];
  best_idx = si[0];
  for (int i = 1; i < 4; ++i) {
    ms = ms_merge(ms, MaxSum{sm[i], ss[i]});
    if (sb[i] > best || (sb[i] == best && si[i] < best_idx)) {
      best = sb[i];
      best_idx = si[i];
    }
  }
  __syncthreads();
}

// Per-row metric contributions.  With `row_stats` ([M, 3]) each row writes
// its own (loss, correct, counted) and ce_metrics_reduce_kernel sums them in
// one block: three same-address float atomics per row from every XCD had cost
// 0.32 ms per BERT-large step (16384 rows), most of the kernel.  Without it
// (a caller that passes no scratch) the atomics remain.
__device__ __forceinline__ void ce_row_metrics(float* metrics, float* row_stats, int row, float loss, bool correct,
                                               bool valid) {
  if (row_stats) {
    float* rs = row_stats + 3 * static_cast<size_t>(row);
    rs[0] = loss;
    rs[1] = correct ? 1.f : 0.f;
    rs[2] = valid ? 1.f : 0.f;
  } else if (valid) {
    atomicAdd(metrics + 0, loss);
    atomicAdd(metrics + 1, correct ? 1.f : 0.f);
    atomicAdd(metrics + 2, 1.f);
  }
}

__global__ __launch_bounds__(256) void ce_metrics_reduce_kernel(const float* __restrict__ row_stats, int M,
                                                                float* __restrict__ metrics) {
  __shared__ float scratch[4];
  float a = 0.f, b = 0.f, c = 0.f;
  for (int r = threadIdx.x; r < M; r += 256) {
    a += row_stats[3 * static_cast<size_t>(r)];
    b += row_stats[3 * static_cast<size_t>(r) + 1];
    c += row_stats[3 * static_cast<size_t>(r) + 2];
  }
  a = block_sum<256>(a, scratch);
  b = block_sum<256>(b, scratch);
  c = block_sum<256>(c, scratch);
  if (threadIdx.x == 0) {
    metrics[0] += a;
    metrics[1] += b;
    metrics[2] += c;
  }
}

// logits: [M, V] (row stride V); labels: [M] int32 or int64.
// Columns >= V_valid are padding (excluded from the softmax, grad 0).
template <typename T, typename L, bool VEC>
__global__ __launch_bounds__(256) void softmax_ce_kernel(T* __restrict__ logits, const L* __restrict__ labels,
                                                         float* __restrict__ row_loss, float* __restrict__ metrics,
                                                         float* __restrict__ row_stats,
                                                         int M, int V, int V_valid, float grad_scale,
                                                         int ignore_index, int write_grad) {
  const int row = blockIdx.x;
  T* x = logits + static_cast<size_t>(row) * V;
  MaxSum ms{-INFINITY, 0.f};
  float best = -INFINITY;
  int best_idx = 0;
  if (VEC) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      float v[8];
      if constexpr (sizeof(T) == 2) {
        u16x8 u = *reinterpret_cast<const u16x8*>(x + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = u2f(u[k]);
      } else {
        f32x4 a = reinterpret_cast<const f32x4*>(x + c)[0], b = reinterpret_cast<const f32x4*>(x + c)[1];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = a[k];
          v[k + 4] = b[k];
        }
      }
      float lm = -INFINITY;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if (c + k >= V_valid) v[k] = -INFINITY;
        lm = fmaxf(lm, v[k]);
        if (v[k] > best) {
          best = v[k];
          best_idx = c + k;
        }
      }
      float ls = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) ls += (v[k] == -INFINITY) ? 0.f : __expf(v[k] - lm);
      if (lm != -INFINITY) ms = ms_merge(ms, MaxSum{lm, ls});
    }
  } else {
    for (int c = threadIdx.x; c < V_valid; c += 256) {
      float v = ldf<T>(x + c);
      ms = ms_merge(ms, MaxSum{v, 1.f});
      if (v > best) {
        best = v;
        best_idx = c;
      }
    }
  }
  block_reduce_msa(ms, best, best_idx);
  const float lse = ms.m + __logf(ms.s);
  const long long lab = static_cast<long long>(labels[row]);
  const bool valid = lab != ignore_index && lab >= 0 && lab < V_valid;
  if (threadIdx.x == 0) {
    float loss = valid ? lse - ldf<T>(x + lab) : 0.f;
    if (row_loss) row_loss[row] = loss;
    if (metrics) ce_row_metrics(metrics, row_stats, row, loss, valid && best_idx == lab, valid);
  }
  if (!write_grad) return;
  __syncthreads();  // the label logit must be read before it is overwritten
  const float scale = valid ? grad_scale : 0.f;
  if (VEC) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      float v[8];
      if constexpr (sizeof(T) == 2) {
        u16x8 u = *reinterpret_cast<const u16x8*>(x + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = u2f(u[k]);
      } else {
        f32x4 a = reinterpret_cast<const f32x4*>(x + c)[0], b = reinterpret_cast<const f32x4*>(x + c)[1];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = a[k];
          v[k + 4] = b[k];
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float p = (c + k < V_valid) ? __expf(v[k] - lse) : 0.f;
        v[k] = (p - ((c + k) == lab ? 1.f : 0.f)) * scale;
      }
      if constexpr (sizeof(T) == 2) {
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = f2bf(v[k]);
        *reinterpret_cast<bf16x8*>(x + c) = o;
      } else {
        f32x4 a, b;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          a[k] = v[k];
          b[k] = v[k + 4];
        }
        reinterpret_cast<f32x4*>(x + c)[0] = a;
        reinterpret_cast<f32x4*>(x + c)[1] = b;
      }
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      float p = (c < V_valid) ? __expf(ldf<T>(x + c) - lse) : 0.f;
      stf<T>(x + c, (p - (c == lab ? 1.f : 0.f)) * scale);
    }
  }
}

// bf16 rows that fit in registers (V <= 2048 * NIT): the row is loaded ONCE
// (every chunk's load issued up front), reduced, and the gradient written
// from the same registers — one HBM read + one write per logit instead of
// the two reads of the streaming kernel above.  Since the whole row is in
// registers the reduction is three plain passes, ~12 VALU issues per logit
// (it was ~25 with a per-chunk online max/sum merge, a NaN-canonicalising
// fmaxf, a padding check and an argmax update per logit, and a label compare
// per gradient):
//   1. thread max with v_max3 (padding columns were set to -inf at load);
//   2. sum of exp2(v log2e - m log2e) — one FMA + one exp2 + one add — and,
//      only when metrics are requested, the first index of the maximum;
//   3. gradient p * scale (one FMA + exp2 + mul); the label's "- 1" is one
//      store by thread 0 after a barrier.
template <typename L, int NIT>
__global__ __launch_bounds__(256) void softmax_ce_reg_kernel(bf16* __restrict__ logits, const L* __restrict__ labels,
                                                             float* __restrict__ row_loss, float* __restrict__ metrics,
                                                             float* __restrict__ row_stats, int M, int V, int V_valid, float grad_scale,
                                                             int ignore_index, int write_grad) {
  constexpr float L2E = 1.4426950408889634f;
  const int row = blockIdx.x;
  bf16* x = logits + static_cast<size_t>(row) * V;
  const long long lab = static_cast<long long>(labels[row]);
  const bool valid = lab != ignore_index && lab >= 0 && lab < V_valid;
  // the label's logit, read before any thread overwrites the row with gradients
  const float lab_logit = (threadIdx.x == 0 && valid) ? u2f(reinterpret_cast<const unsigned short*>(x)[lab]) : 0.f;
  u16x8 u[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
    if (c < V) u[it] = *reinterpret_cast<const u16x8*>(x + c);
  }
  // padding columns (>= V_valid, only in the row's last chunks) become -inf
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
    if (c < V && c + 8 > V_valid) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (c + k >= V_valid) u[it][k] = 0xFF80;
    }
  }
  // ---- 1. thread max
  float t0 = -INFINITY, t1 = -INFINITY;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
    if (c < V) {
      float& t = (it & 1) ? t1 : t0;
#pragma unroll
      for (int k = 0; k < 8; k += 2) t = fmax3(t, u2f(u[it][k]), u2f(u[it][k + 1]));
    }
  }
  const float tm = fmax3(t0, t1, t1);
  // ---- 2. thread sum relative to the thread max (+ first index of the max)
  const float tmc = (tm == -INFINITY) ? 0.f : tm * L2E;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
    if (c < V) {
      float& sacc = (it & 1) ? s1 : s0;
#pragma unroll
      for (int k = 0; k < 8; ++k) sacc += fexp2(fmaf(u2f(u[it][k]), L2E, -tmc));
    }
  }
  int best_idx = 0;
  if (metrics) {
    best_idx = 0x7fffffff;
#pragma unroll
    for (int it = NIT - 1; it >= 0; --it) {
      const int c = (it * 256 + threadIdx.x) * 8;
      if (c < V) {
#pragma unroll
        for (int k = 7; k >= 0; --k) best_idx = (u2f(u[it][k]) == tm) ? c + k : best_idx;
      }
    }
  }
  MaxSum ms{tm, s0 + s1};
  float best = tm;
  block_reduce_msa(ms, best, best_idx);
  const float lse = ms.m + __logf(ms.s);
  if (threadIdx.x == 0) {
    float loss = valid ? lse - lab_logit : 0.f;
    if (row_loss) row_loss[row] = loss;
    if (metrics) ce_row_metrics(metrics, row_stats, row, loss, valid && best_idx == lab, valid);
  }
  if (!write_grad) return;
  // ---- 3. gradient softmax * scale, in place
  const float scale = valid ? grad_scale : 0.f;
  const float lsec = lse * L2E;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int c = (it * 256 + threadIdx.x) * 8;
    if (c < V) {
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = f2bf(fexp2(fmaf(u2f(u[it][k]), L2E, -lsec)) * scale);
      *reinterpret_cast<bf16x8*>(x + c) = o;
    }
  }
  // the label column: softmax - 1, written after every thread's row stores
  __syncthreads();
  if (threadIdx.x == 0 && valid) x[lab] = f2bf((fexp2(fmaf(lab_logit, L2E, -lsec)) - 1.f) * scale);
}

// Row softmax forward / backward (last dim).  One block per row.
template <typename T>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N) {
  const size_t base = static_cast<size_t>(blockIdx.x) * N;
  MaxSum ms{-INFINITY, 0.f};
  float best = 0.f;
  int bi = 0;
  for (int c = threadIdx.x; c < N; c += 256) ms = ms_merge(ms, MaxSum{ldf<T>(x + base + c), 1.f});
  block_reduce_msa(ms, best, bi);
  const float inv = 1.f / ms.s;
  for (int c = threadIdx.x; c < N; c += 256) stf<T>(y + base + c, __expf(ldf<T>(x + base + c) - ms.m) * inv);
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y,
                                                          T* __restrict__ dx, int N) {
  __shared__ float scratch[4];
  const size_t base = static_cast<size_t>(blockIdx.x) * N;
  float d = 0.f;
  for (int c = threadIdx.x; c < N; c += 256) d += ldf<T>(dy + base + c) * ldf<T>(y + base + c);
  d = block_sum<256>(d, scratch);
  for (int c = threadIdx.x; c < N; c += 256) {
    float yy = ldf<T>(y + base + c);
    stf<T>(dx + base + c, yy * (ldf<T>(dy + base + c) - d));
  }
}

void softmax_ce(int dtype, int label_bits, void* logits, const void* labels, float* row_loss, float* metrics,
                float* row_stats, int M, int V, int V_valid, float grad_scale, int ignore_index, int write_grad,
                hipStream_t st) {
  if (!metrics) row_stats = nullptr;
  const bool vec = (V % 8 == 0);
  dim3 grid(M), block(256);
#define FFK_CE(T, L, VEC)                                                                                   \
  hipLaunchKernelGGL((softmax_ce_kernel<T, L, VEC>), grid, block, 0, st, static_cast<T*>(logits),           \
                     static_cast<const L*>(labels), row_loss, metrics, row_stats, M, V, V_valid, grad_scale, ignore_index, \
                     write_grad)
  if (dtype == kBF16 && vec && V <= 2048 * 32) {
    // register-resident rows (one read + one write per logit)
#define FFK_CE_REG(L, NIT)                                                                                     \
  hipLaunchKernelGGL((softmax_ce_reg_kernel<L, NIT>), grid, block, 0, st, static_cast<bf16*>(logits),        \
                     static_cast<const L*>(labels), row_loss, metrics, row_stats, M, V, V_valid, grad_scale, ignore_index, \
                     write_grad)
    if (label_bits == 64) {
      if (V <= 2048 * 16) FFK_CE_REG(int64_t, 16);
      else FFK_CE_REG(int64_t, 32);
    } else {
      if (V <= 2048 * 16) FFK_CE_REG(int32_t, 16);
      else FFK_CE_REG(int32_t, 32);
    }
#undef FFK_CE_REG
  } else if (dtype == kBF16) {
    if (label_bits == 64) {
      if (vec) FFK_CE(bf16, int64_t, true);
      else FFK_CE(bf16, int64_t, false);
    } else {
      if (vec) FFK_CE(bf16, int32_t, true);
      else FFK_CE(bf16, int32_t, false);
    }
  } else if (dtype == kF32) {
    if (label_bits == 64) {
      if (vec) FFK_CE(float, int64_t, true);
      else FFK_CE(float, int64_t, false);
    } else {
      if (vec) FFK_CE(float, int32_t, true);
      else FFK_CE(float, int32_t, false);
    }
  } else {
    throw std::invalid_argument("softmax_ce: dtype");
  }
#undef FFK_CE
  FFK_LAUNCH_CHECK("softmax_ce");
  if (row_stats) {
    hipLaunchKernelGGL(ce_metrics_reduce_kernel, dim3(1), dim3(256), 0, st, row_stats, M, metrics);
    FFK_LAUNCH_CHECK("ce_metrics_reduce");
  }
}

void softmax_fwd(int dtype, const void* x, void* y, int M, int N, hipStream_t st) {
  if (dtype == kBF16)
    hipLaunchKernelGGL(softmax_fwd_kernel<bf16>, dim3(M), dim3(256), 0, st, static_cast<const bf16*>(x),
                       static_cast<bf16*>(y), N);
  else if (dtype == kF32)
    hipLaunchKernelGGL(softmax_fwd_kernel<float>, dim3(M), dim3(256), 0, st, static_cast<const float*>(x),
                       static_cast<float*>(y), N);
  else throw std::invalid_argument("softmax_fwd: dtype");
  FFK_LAUNCH_CHECK("softmax_fwd");
}

void softmax_bwd(int dtype, const void* dy, const void* y, void* dx, int M, int N, hipStream_t st) {
  if (dtype == kBF16)
    hipLaunchKernelGGL(softmax_bwd_kernel<bf16>, dim3(M), dim3(256), 0, st, static_cast<const bf16*>(dy),
                       static_cast<const bf16*>(y), static_cast<bf16*>(dx), N);
  else if (dtype == kF32)
    hipLaunchKernelGGL(softmax_bwd_kernel<float>, dim3(M), dim3(256), 0, st, static_cast<const float*>(dy),
                       static_cast<const float*>(y), static_cast<float*>(dx), N);
  else throw std::invalid_argument("softmax_bwd: dtype");
  FFK_LAUNCH_CHECK("softmax_bwd");
}

}  // namespace ffk
