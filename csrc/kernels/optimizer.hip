// Fused optimizer updates over flat parameter buffers (gfx950).
//
// Parity: lib/kernels/src/cuda/optimizer_kernel.cu — sgd_update (:20-41,
// PyTorch semantics: weight decay, momentum, Nesterov) and adam_update
// (:123-145, weight decay folded into the gradient, alpha_t bias correction
// precomputed on the host: lib/runtime/src/optimizer.cc:141-147).
// MI355X-first: all parameters live in ONE flat fp32 master buffer with one
// flat fp32 gradient buffer (DP all-reduce buckets are slices of it), so an
// optimizer step is a single launch over the whole model instead of one task
// per weight; the bf16 compute copy of the weights is written in the same
// pass (no separate cast launch).
#include "common.h"
#include "kernels.h"

namespace ffk {

template <typename GT>
__device__ __forceinline__ f32x4 load_grad4(const GT* g, int64_t i);
template <>
__device__ __forceinline__ f32x4 load_grad4<float>(const float* g, int64_t i) {
  return reinterpret_cast<const f32x4*>(g)[i];
}
template <>
__device__ __forceinline__ f32x4 load_grad4<bf16>(const bf16* g, int64_t i) {
  u16x4 u = reinterpret_cast<const u16x4*>(g)[i];
  return f32x4{u2f(u[0]), u2f(u[1]), u2f(u[2]), u2f(u[3])};
}

// Gradients are fp32 (atomically accumulated parameters) or bf16 (GEMM
// weight gradients written straight by the dW GEMM epilogue).
// 8 consecutive elements per thread per iteration: two 16-byte loads of each
// fp32 stream and one 16-byte load of a bf16 gradient, so a wave keeps ~2x the
// bytes in flight of the 4-wide form (the update is purely HBM-bound:
// 30 bytes / parameter).
template <typename GT>
__device__ __forceinline__ void load_grad8(const GT* g, int64_t i, f32x4& a, f32x4& b);
template <>
__device__ __forceinline__ void load_grad8<float>(const float* g, int64_t i, f32x4& a, f32x4& b) {
  a = reinterpret_cast<const f32x4*>(g)[2 * i];
  b = reinterpret_cast<const f32x4*>(g)[2 * i + 1];
}
template <>
__device__ __forceinline__ void load_grad8<bf16>(const bf16* g, int64_t i, f32x4& a, f32x4& b) {
  const u16x8 u = reinterpret_cast<const u16x8*>(g)[i];
  a = f32x4{u2f(u[0]), u2f(u[1]), u2f(u[2]), u2f(u[3])};
  b = f32x4{u2f(u[4]), u2f(u[5]), u2f(u[6]), u2f(u[7])};
}

template <typename GT>
__global__ __launch_bounds__(256) void adam8_kernel(float* __restrict__ w, const GT* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    bf16* __restrict__ w_bf16, int64_t n8, float lr, float beta1,
                                                    float beta2, float eps, float weight_decay, float bc1,
                                                    float bc2_sqrt, float grad_scale, int decoupled,
                                                    const float* __restrict__ hp) {
  if (hp) {  // device-resident {lr, step}: hipGraph replays see the current values
    lr = hp[0];
    bc1 = 1.f - __powf(beta1, hp[1]);
    bc2_sqrt = sqrtf(1.f - __powf(beta2, hp[1]));
  }
  const float inv_bc1 = 1.f / bc1, inv_bc2s = 1.f / bc2_sqrt;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n8; i += static_cast<int64_t>(gridDim.x) * 256) {
    f32x4 W[2], G[2], Mm[2], Vv[2];
    W[0] = reinterpret_cast<f32x4*>(w)[2 * i];
    W[1] = reinterpret_cast<f32x4*>(w)[2 * i + 1];
    load_grad8<GT>(g, i, G[0], G[1]);
    Mm[0] = reinterpret_cast<f32x4*>(m)[2 * i];
    Mm[1] = reinterpret_cast<f32x4*>(m)[2 * i + 1];
    Vv[0] = reinterpret_cast<f32x4*>(v)[2 * i];
    Vv[1] = reinterpret_cast<f32x4*>(v)[2 * i + 1];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float gg = G[h][k] * grad_scale;
        if (!decoupled) gg += weight_decay * W[h][k];
        Mm[h][k] = beta1 * Mm[h][k] + (1.f - beta1) * gg;
        Vv[h][k] = beta2 * Vv[h][k] + (1.f - beta2) * gg * gg;
        float upd = (Mm[h][k] * inv_bc1) / (sqrtf(Vv[h][k]) * inv_bc2s + eps);
        if (decoupled) upd += weight_decay * W[h][k];
        W[h][k] -= lr * upd;
      }
    reinterpret_cast<f32x4*>(w)[2 * i] = W[0];
    reinterpret_cast<f32x4*>(w)[2 * i + 1] = W[1];
    reinterpret_cast<f32x4*>(m)[2 * i] = Mm[0];
    reinterpret_cast<f32x4*>(m)[2 * i + 1] = Mm[1];
    reinterpret_cast<f32x4*>(v)[2 * i] = Vv[0];
    reinterpret_cast<f32x4*>(v)[2 * i + 1] = Vv[1];
    if (w_bf16) {
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[k] = f2bf(W[0][k]);
        o[4 + k] = f2bf(W[1][k]);
      }
      reinterpret_cast<bf16x8*>(w_bf16)[i] = o;
    }
  }
}

template <typename GT>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ w, const GT* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16* __restrict__ w_bf16, int64_t n4, float lr, float beta1,
                                                   float beta2, float eps, float weight_decay, float bc1,
                                                   float bc2_sqrt, float grad_scale, int decoupled,
                                                   const float* __restrict__ hp) {
  if (hp) {  // device-resident {lr, step}: hipGraph replays see the current values
    lr = hp[0];
    bc1 = 1.f - __powf(beta1, hp[1]);
    bc2_sqrt = sqrtf(1.f - __powf(beta2, hp[1]));
  }
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    f32x4 W = reinterpret_cast<f32x4*>(w)[i];
    f32x4 G = load_grad4<GT>(g, i);
    f32x4 Mm = reinterpret_cast<f32x4*>(m)[i];
    f32x4 Vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gg = G[k] * grad_scale;
      if (!decoupled) gg += weight_decay * W[k];
      Mm[k] = beta1 * Mm[k] + (1.f - beta1) * gg;
      Vv[k] = beta2 * Vv[k] + (1.f - beta2) * gg * gg;
      float upd = (Mm[k] / bc1) / (sqrtf(Vv[k]) / bc2_sqrt + eps);
      if (decoupled) upd += weight_decay * W[k];
      W[k] -= lr * upd;
    }
    reinterpret_cast<f32x4*>(w)[i] = W;
    reinterpret_cast<f32x4*>(m)[i] = Mm;
    reinterpret_cast<f32x4*>(v)[i] = Vv;
    if (w_bf16) {
      bf16x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = f2bf(W[k]);
      reinterpret_cast<bf16x4*>(w_bf16)[i] = o;
    }
  }
}

template <typename GT>
__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ w, const GT* __restrict__ g,
                                                  float* __restrict__ mom, bf16* __restrict__ w_bf16, int64_t n4,
                                                  float lr, float momentum, float weight_decay, int nesterov,
                                                  float grad_scale) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    f32x4 W = reinterpret_cast<f32x4*>(w)[i];
    f32x4 G = load_grad4<GT>(g, i);
    f32x4 Mo;
    if (mom) Mo = reinterpret_cast<f32x4*>(mom)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gg = G[k] * grad_scale + weight_decay * W[k];
      if (mom) {
        Mo[k] = momentum * Mo[k] + gg;
        gg = nesterov ? gg + momentum * Mo[k] : Mo[k];
      }
      W[k] -= lr * gg;
    }
    reinterpret_cast<f32x4*>(w)[i] = W;
    if (mom) reinterpret_cast<f32x4*>(mom)[i] = Mo;
    if (w_bf16) {
      bf16x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = f2bf(W[k]);
      reinterpret_cast<bf16x4*>(w_bf16)[i] = o;
    }
  }
}

// sum of squares of a flat fp32 buffer into out[0] (grad-norm clipping)
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, int64_t n4, float* out) {
  __shared__ float scratch[4];
  float s = 0.f;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    f32x4 v = reinterpret_cast<const f32x4*>(x)[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  s = block_sum<256>(s, scratch);
  if (threadIdx.x == 0) atomicAdd(out, s);
}


// ---------------------------------------------------------------------------
// Row-sparse SGD over embedding tables (plain SGD: untouched rows have zero
// gradient, so only the rows the step looked up change).  All tables of a
// flat go in one launch pair instead of ~11 framework kernels per table:
//   gather:  scratch[i] = master[r_i] - step * grad[r_i]       (reads only)
//   scatter: master[r_i] = scratch[i]; compute[r_i] = bf16(..); grad[r_i] = 0
// r_i = clamp(idx[i], 0, rows - 1).  A row looked up twice gets the same
// value written twice (both gathers saw the pre-update row), which is why the
// update is split across two launches: a single pass could read a row
// another thread already updated or whose gradient it already cleared.
template <typename GT, typename IT>
__device__ __forceinline__ void sparse_rows_phase(const SparseSgdTable& t, float* scratch, float step, int phase) {
  const int dim4 = t.dim >> 2;
  const int64_t items = t.n_idx * dim4;
  for (int64_t w = blockIdx.x * 256 + threadIdx.x; w < items; w += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t i = w / dim4;
    const int c = static_cast<int>(w - i * dim4) * 4;
    int64_t r = static_cast<int64_t>(static_cast<const IT*>(t.idx)[i]);
    r = r < 0 ? 0 : (r >= t.rows ? t.rows - 1 : r);
    const int64_t off = r * t.dim + c;
    f32x4* sv = reinterpret_cast<f32x4*>(scratch + t.scratch_off + i * t.dim + c);
    if (phase == 0) {
      f32x4 W = *reinterpret_cast<const f32x4*>(t.master + off);
      const f32x4 G = load_grad4<GT>(static_cast<const GT*>(t.grad) + off, 0);
#pragma unroll
      for (int k = 0; k < 4; ++k) W[k] -= step * G[k];
      *sv = W;
    } else {
      const f32x4 W = *sv;
      *reinterpret_cast<f32x4*>(t.master + off) = W;
      if (t.compute) {
        bf16x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = f2bf(W[k]);
        *reinterpret_cast<bf16x4*>(static_cast<bf16*>(t.compute) + off) = o;
      }
      if constexpr (sizeof(GT) == 4) *reinterpret_cast<f32x4*>(static_cast<float*>(t.grad) + off) = f32x4{};
      else *reinterpret_cast<u16x4*>(static_cast<bf16*>(t.grad) + off) = u16x4{};
    }
  }
}

__global__ __launch_bounds__(256) void sparse_sgd_kernel(SparseSgdArgs a, float* scratch, float step, int phase) {
  const SparseSgdTable& t = a.t[blockIdx.y];
  if (t.grad_bf16) {
    if (t.idx64) sparse_rows_phase<bf16, int64_t>(t, scratch, step, phase);
    else sparse_rows_phase<bf16, int32_t>(t, scratch, step, phase);
  } else {
    if (t.idx64) sparse_rows_phase<float, int64_t>(t, scratch, step, phase);
    else sparse_rows_phase<float, int32_t>(t, scratch, step, phase);
  }
}

static void need4(int64_t n, const char* w) {
  if (n % 4 != 0) throw std::invalid_argument(std::string(w) + ": flat buffer length must be a multiple of 4");
}

void adam_step(float* w, const void* g, int grad_dtype, float* m, float* v, void* w_bf16, int64_t n, float lr,
               float beta1, float beta2, float eps, float weight_decay, int step, float grad_scale, int decoupled,
               const float* hp, hipStream_t st) {
  need4(n, "adam");
  float bc1 = 1.f - powf(beta1, static_cast<float>(step));
  float bc2s = sqrtf(1.f - powf(beta2, static_cast<float>(step)));
  if (n % 8 == 0 && (reinterpret_cast<uintptr_t>(g) & 15) == 0 && (reinterpret_cast<uintptr_t>(w_bf16) & 15) == 0) {
    const int grid8 = grid_for(n / 8, 256, 256 * 16);
    if (grad_dtype == kBF16)
      hipLaunchKernelGGL(adam8_kernel<bf16>, dim3(grid8), dim3(256), 0, st, w, static_cast<const bf16*>(g), m, v,
                         static_cast<bf16*>(w_bf16), n / 8, lr, beta1, beta2, eps, weight_decay, bc1, bc2s,
                         grad_scale, decoupled, hp);
    else
      hipLaunchKernelGGL(adam8_kernel<float>, dim3(grid8), dim3(256), 0, st, w, static_cast<const float*>(g), m, v,
                         static_cast<bf16*>(w_bf16), n / 8, lr, beta1, beta2, eps, weight_decay, bc1, bc2s,
                         grad_scale, decoupled, hp);
    FFK_LAUNCH_CHECK("adam");
    return;
  }
  int grid = grid_for(n / 4, 256, 256 * 8);
  if (grad_dtype == kBF16)
    hipLaunchKernelGGL(adam_kernel<bf16>, dim3(grid), dim3(256), 0, st, w, static_cast<const bf16*>(g), m, v,
                       static_cast<bf16*>(w_bf16), n / 4, lr, beta1, beta2, eps, weight_decay, bc1, bc2s, grad_scale,
                       decoupled, hp);
  else
    hipLaunchKernelGGL(adam_kernel<float>, dim3(grid), dim3(256), 0, st, w, static_cast<const float*>(g), m, v,
                       static_cast<bf16*>(w_bf16), n / 4, lr, beta1, beta2, eps, weight_decay, bc1, bc2s, grad_scale,
                       decoupled, hp);
  FFK_LAUNCH_CHECK("adam");
}

void sgd_step(float* w, const void* g, int grad_dtype, float* mom, void* w_bf16, int64_t n, float lr,
              float momentum, float weight_decay, int nesterov, float grad_scale, hipStream_t st) {
  need4(n, "sgd");
  int grid = grid_for(n / 4, 256, 256 * 8);
  if (grad_dtype == kBF16)
    hipLaunchKernelGGL(sgd_kernel<bf16>, dim3(grid), dim3(256), 0, st, w, static_cast<const bf16*>(g), mom,
                       static_cast<bf16*>(w_bf16), n / 4, lr, momentum, weight_decay, nesterov, grad_scale);
  else
    hipLaunchKernelGGL(sgd_kernel<float>, dim3(grid), dim3(256), 0, st, w, static_cast<const float*>(g), mom,
                       static_cast<bf16*>(w_bf16), n / 4, lr, momentum, weight_decay, nesterov, grad_scale);
  FFK_LAUNCH_CHECK("sgd");
}


void sparse_sgd_rows(const SparseSgdArgs& a, float* scratch, float step, hipStream_t st) {
  if (a.nt <= 0) return;
  if (a.nt > kMaxSparseTables) throw std::invalid_argument("sparse_sgd: too many tables in one launch");
  int64_t most = 0;
  for (int i = 0; i < a.nt; ++i) {
    const SparseSgdTable& t = a.t[i];
    if (t.dim % 4 || t.rows <= 0) throw std::invalid_argument("sparse_sgd: row width must be a multiple of 4");
    most = std::max(most, t.n_idx * (t.dim / 4));
  }
  if (most == 0) return;
  const dim3 grid(static_cast<unsigned>(std::min<int64_t>((most + 255) / 256, 1024)), static_cast<unsigned>(a.nt));
  hipLaunchKernelGGL(sparse_sgd_kernel, grid, dim3(256), 0, st, a, scratch, step, 0);
  hipLaunchKernelGGL(sparse_sgd_kernel, grid, dim3(256), 0, st, a, scratch, step, 1);
  FFK_LAUNCH_CHECK("sparse_sgd");
}

void sum_squares(const float* x, int64_t n, float* out, hipStream_t st) {
  need4(n, "sum_squares");
  int grid = grid_for(n / 4, 256, 1024);
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid), dim3(256), 0, st, x, n / 4, out);
  FFK_LAUNCH_CHECK("sum_squares");
}

}  // namespace ffk
