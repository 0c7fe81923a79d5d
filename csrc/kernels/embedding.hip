// Embedding lookup (no aggregation / SUM / AVG bags) forward and backward.
//
// Parity: lib/kernels/src/cuda/embedding_kernels.cu (embed_forward_no_aggr,
// embed_forward_with_aggr, embed_backward_* with atomicAdd, :64-242).  Fixes
// the reference's AVG bug (the 1/L scale applied inside the accumulation
// loop, :106-113): here the bag is summed in fp32 and scaled once.
// CDNA4: each thread moves one 16-byte chunk (8 x bf16) of a row, rows are
// gathered whole; the backward scatter-adds fp32 rows with per-column atomics
// shaped as contiguous 256-byte wave segments (guide G12), into the flat fp32
// gradient buffer.
#include <cstdlib>

#include "common.h"
#include "kernels.h"

namespace ffk {

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* o) {
  if constexpr (sizeof(T) == 2) {
    u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = u2f(u[k]);
  } else {
    f32x4 a = reinterpret_cast<const f32x4*>(p)[0], b = reinterpret_cast<const f32x4*>(p)[1];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = a[k];
      o[k + 4] = b[k];
    }
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* p, const float* o) {
  if constexpr (sizeof(T) == 2) {
    bf16x8 v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = f2bf(o[k]);
    *reinterpret_cast<bf16x8*>(p) = v;
  } else {
    f32x4 a, b;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = o[k];
      b[k] = o[k + 4];
    }
    reinterpret_cast<f32x4*>(p)[0] = a;
    reinterpret_cast<f32x4*>(p)[1] = b;
  }
}

// out[b, :] = agg_{j<L} W[idx[b*L + j], :]   (L == 1 and mode 0 -> plain lookup)
template <typename T, typename I>
__global__ __launch_bounds__(256) void embed_fwd_kernel(const I* __restrict__ idx, const T* __restrict__ W,
                                                        T* __restrict__ out, int64_t B, int L, int D, int mode,
                                                        int64_t num_entries) {
  const int cpr = D / 8;
  const int64_t total = B * cpr;
  for (int64_t t = blockIdx.x * 256 + threadIdx.x; t < total; t += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t b = t / cpr;
    const int col = static_cast<int>(t % cpr) * 8;
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    for (int j = 0; j < L; ++j) {
      int64_t r = static_cast<int64_t>(idx[b * L + j]);
      if (r < 0 || r >= num_entries) continue;  // out-of-range ids contribute zeros
      float v[8];
      load8<T>(W + r * D + col, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
    if (mode == 2 && L > 0) {
      const float inv = 1.f / L;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] *= inv;
    }
    store8<T>(out + b * D + col, acc);
  }
}

// Scatter-add of output-row gradients into the table gradient.  For small,
// hot tables (position / segment embeddings: thousands of rows add into the
// same few table rows) the adds go to `copies` private replicas of the table
// gradient (row bj -> replica bj % copies), cutting same-address contention by
// `copies` (guide G12: one hot row is ~14x slower than spread rows); a second
// pass sums the replicas.
template <typename T, typename I>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const I* __restrict__ idx, const T* __restrict__ dout,
                                                        float* __restrict__ dW, int64_t B, int L, int D, int mode,
                                                        int64_t num_entries, int copies) {
  const int cpr = D / 8;
  const int64_t total = B * L * cpr;
  const float scale = (mode == 2 && L > 0) ? 1.f / L : 1.f;
  for (int64_t t = blockIdx.x * 256 + threadIdx.x; t < total; t += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t bj = t / cpr;
    const int col = static_cast<int>(t % cpr) * 8;
    const int64_t b = bj / L;
    int64_t r = static_cast<int64_t>(idx[bj]);
    if (r < 0 || r >= num_entries) continue;
    float v[8];
    load8<T>(dout + b * D + col, v);
    float* dst = dW + (static_cast<int64_t>(bj % copies) * num_entries + r) * D + col;
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(dst + k, v[k] * scale);
  }
}

// Same scatter-add, one wave per gradient row (D >= 64): lane l owns columns
// l, l+64, ... so every atomic instruction of the wave covers 256 contiguous
// bytes (two full cache lines) instead of 4-byte pieces of sixteen lines —
// the L2 atomic units see ~8x fewer requests.
template <typename T, typename I>
__global__ __launch_bounds__(256) void embed_bwd_wave_kernel(const I* __restrict__ idx, const T* __restrict__ dout,
                                                             float* __restrict__ dW, int64_t rows, int L, int D,
                                                             int mode, int64_t num_entries, int copies) {
  const int lane = threadIdx.x & 63;
  const float scale = (mode == 2 && L > 0) ? 1.f / L : 1.f;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * 4;
  for (int64_t bj = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); bj < rows; bj += nw) {
    const int64_t r = static_cast<int64_t>(idx[bj]);
    if (r < 0 || r >= num_entries) continue;
    const T* src = dout + (bj / L) * D;
    float* dst = dW + (static_cast<int64_t>(bj % copies) * num_entries + r) * D;
    int c = lane;
    for (; c + 7 * 64 < D; c += 8 * 64) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = static_cast<float>(src[c + u * 64]);
#pragma unroll
      for (int u = 0; u < 8; ++u) atomicAdd(dst + c + u * 64, v[u] * scale);
    }
    for (; c < D; c += 64) atomicAdd(dst + c, static_cast<float>(src[c]) * scale);
  }
}

// Tiny tables (token-type / segment embeddings: num_entries <= E <= 8, no
// bag): every lookup row lands in one of E table rows, so a scatter of fp32
// atomics is all same-address contention.  Instead: E masked column sums,
// laid out like colsum_act (elementwise.hip) — a block's 4 waves cover 512
// columns (8 per lane) of a slab of rows, 8 rows in flight per wave, the
// entry picked by predication (no dynamic register index); the waves' sums
// meet in LDS and each block adds E x 512 values with one atomic each.
template <typename T, typename I, int E>
__global__ __launch_bounds__(256) void embed_bwd_small_kernel(const I* __restrict__ idx, const T* __restrict__ dout,
                                                              float* __restrict__ dW, int64_t rows, int D,
                                                              int64_t num_entries) {
  __shared__ float red[4][E][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + lane * 8;
  const bool active = col < D;
  float acc[E][8];
#pragma unroll
  for (int q = 0; q < E; ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[q][k] = 0.f;
  const int64_t per = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = static_cast<int64_t>(blockIdx.y) * per;
  const int64_t r1 = r0 + per < rows ? r0 + per : rows;
  constexpr int U = 8;
  if (active) {
    for (int64_t r = r0 + wave; r < r1; r += 4 * U) {
      float v[U][8];
      int64_t e[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t rr = r + 4 * u;
        if (rr < r1) {
          e[u] = static_cast<int64_t>(idx[rr]);
          load8<T>(dout + rr * D + col, v[u]);
        } else {
          e[u] = -1;
#pragma unroll
          for (int k = 0; k < 8; ++k) v[u][k] = 0.f;
        }
      }
      // select, not multiply-by-mask: 0 * (inf or nan) of a row that belongs
      // to another entry would poison the sum
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < E; ++q)
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[q][k] += (e[u] == q) ? v[u][k] : 0.f;
    }
  }
#pragma unroll
  for (int q = 0; q < E; ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wave][q][lane * 8 + k] = acc[q][k];
  __syncthreads();
  for (int j = threadIdx.x; j < E * 512; j += 256) {
    const int q = j / 512, c = j % 512;
    const int cc = blockIdx.x * 512 + c;
    if (q < num_entries && cc < D)
      atomicAdd(dW + static_cast<int64_t>(q) * D + cc, red[0][q][c] + red[1][q][c] + red[2][q][c] + red[3][q][c]);
  }
}

// dW[i] += sum_c ws[c][i]   (i over num_entries*D, vectorised by 4)
__global__ __launch_bounds__(256) void embed_reduce_copies_kernel(const float* __restrict__ ws,
                                                                  float* __restrict__ dW, int64_t n4, int copies) {
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    f32x4 acc = reinterpret_cast<const f32x4*>(dW)[i];
    for (int c = 0; c < copies; ++c) acc += reinterpret_cast<const f32x4*>(ws)[c * n4 + i];
    reinterpret_cast<f32x4*>(dW)[i] = acc;
  }
}

void embedding_fwd(int dtype, int index_bits, const void* idx, const void* W, void* out, int64_t B, int L, int D,
                   int mode, int64_t num_entries, hipStream_t st) {
  if (D % 8 != 0) throw std::invalid_argument("embedding: dim must be a multiple of 8");
  int grid = grid_for(B * (D / 8), 256, 256 * 16);
#define FFK_EF(T, I)                                                                                         \
  hipLaunchKernelGGL((embed_fwd_kernel<T, I>), dim3(grid), dim3(256), 0, st, static_cast<const I*>(idx),     \
                     static_cast<const T*>(W), static_cast<T*>(out), B, L, D, mode, num_entries)
  if (dtype == kBF16) {
    if (index_bits == 64) FFK_EF(bf16, int64_t);
    else FFK_EF(bf16, int32_t);
  } else if (dtype == kF32) {
    if (index_bits == 64) FFK_EF(float, int64_t);
    else FFK_EF(float, int32_t);
  } else {
    throw std::invalid_argument("embedding: dtype");
  }
#undef FFK_EF
  FFK_LAUNCH_CHECK("embedding_fwd");
}

void embedding_bwd(int dtype, int index_bits, const void* idx, const void* dout, float* dW, int64_t B, int L, int D,
                   int mode, int64_t num_entries, float* workspace, int copies, hipStream_t st) {
  if (D % 8 != 0) throw std::invalid_argument("embedding: dim must be a multiple of 8");
  if (copies < 1) copies = 1;
  const char* se = getenv("FFK_EMB_SMALL");   // read per call: A/B and bisection switch
  if (num_entries <= 8 && L == 1 && mode == 0 && !(se && atoi(se) == 0)) {
    const int64_t rows = B;
    // ~1024 blocks in total, >= 64 rows per block (colsum_act's split)
    const int gx = (D + 511) / 512;
    const int gy = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((1024 + gx - 1) / gx, (rows + 63) / 64)));
    const dim3 grid(gx, gy);
#define FFK_ES(T, I, EE)                                                                                      \
  hipLaunchKernelGGL((embed_bwd_small_kernel<T, I, EE>), grid, dim3(256), 0, st,                              \
                     static_cast<const I*>(idx), static_cast<const T*>(dout), dW, rows, D, num_entries)
#define FFK_ES_E(T, I)                                                                                        \
  if (num_entries <= 2) FFK_ES(T, I, 2);                                                                      \
  else if (num_entries <= 4) FFK_ES(T, I, 4);                                                                 \
  else FFK_ES(T, I, 8)
    if (dtype == kBF16) {
      if (index_bits == 64) { FFK_ES_E(bf16, int64_t); }
      else { FFK_ES_E(bf16, int32_t); }
    } else if (dtype == kF32) {
      if (index_bits == 64) { FFK_ES_E(float, int64_t); }
      else { FFK_ES_E(float, int32_t); }
    } else {
      throw std::invalid_argument("embedding: dtype");
    }
#undef FFK_ES_E
#undef FFK_ES
    FFK_LAUNCH_CHECK("embedding_bwd_small");
    return;
  }
  if (copies > 1 && workspace == nullptr) throw std::invalid_argument("embedding_bwd: copies > 1 needs a workspace");
  float* target = copies > 1 ? workspace : dW;
  const bool wave = D >= 64;
  int grid = wave ? grid_for(B * L, 4, 256 * 16) : grid_for(B * L * (D / 8), 256, 256 * 16);
#define FFK_EB(T, I)                                                                                          \
  if (wave)                                                                                                   \
    hipLaunchKernelGGL((embed_bwd_wave_kernel<T, I>), dim3(grid), dim3(256), 0, st,                           \
                       static_cast<const I*>(idx), static_cast<const T*>(dout), target, B * L, L, D, mode,   \
                       num_entries, copies);                                                                  \
  else                                                                                                        \
    hipLaunchKernelGGL((embed_bwd_kernel<T, I>), dim3(grid), dim3(256), 0, st, static_cast<const I*>(idx),    \
                       static_cast<const T*>(dout), target, B, L, D, mode, num_entries, copies)
  if (dtype == kBF16) {
    if (index_bits == 64) FFK_EB(bf16, int64_t);
    else FFK_EB(bf16, int32_t);
  } else if (dtype == kF32) {
    if (index_bits == 64) FFK_EB(float, int64_t);
    else FFK_EB(float, int32_t);
  } else {
    throw std::invalid_argument("embedding: dtype");
  }
#undef FFK_EB
  FFK_LAUNCH_CHECK("embedding_bwd");
  if (copies > 1) {
    const int64_t n4 = num_entries * D / 4;
    hipLaunchKernelGGL(embed_reduce_copies_kernel, dim3(grid_for(n4, 256, 2048)), dim3(256), 0, st, workspace, dW,
                       n4, copies);
    FFK_LAUNCH_CHECK("embedding_bwd_reduce");
  }
}

}  // namespace ffk
