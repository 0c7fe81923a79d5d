// Shared device helpers for the gfx950 (CDNA4) kernel library.
//
// Conventions:
//  * wave64 everywhere (hard-coded 64, never warpSize);
//  * bf16 is moved as raw 16-bit words in 16-byte vectors (8 x bf16 per lane)
//    so every memory-bound kernel issues dwordx4 loads/stores;
//  * math is fp32; conversions go through __bf16 casts, which hipcc lowers to
//    v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN preserving);
//  * every launcher takes the HIP stream explicitly (the caller passes
//    torch.cuda.current_stream()), never allocates, never synchronises, so
//    launches can be captured into hipGraphs.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace ffk {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4t __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 x) { return static_cast<float>(x); }
__device__ __forceinline__ bf16 f2bf(float x) { return static_cast<bf16>(x); }
__device__ __forceinline__ float u2f(unsigned short u) { return __uint_as_float(static_cast<unsigned>(u) << 16); }
__device__ __forceinline__ unsigned short f2u(float x) {
  bf16 b = static_cast<bf16>(x);
  return __builtin_bit_cast(unsigned short, b);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `scratch` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += scratch[i];
  __syncthreads();
  return r;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, scratch[i]);
  __syncthreads();
  return r;
}

// bare v_exp_f32 (2^x): libm exp2f adds a denormal range fix-up (cmp +
// ldexp + 2 cndmask per element) that dominated the softmax VALU in attention
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

// max of three in ONE v_max3_f32.  fmaxf on values the compiler cannot prove
// canonical (MFMA accumulators) is lowered with a NaN-quieting v_max x,x per
// operand before the max itself: a 32-score tile max cost ~56 VALU issues
// instead of 16.  Scores here are never signalling NaNs.
__device__ __forceinline__ float fmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// tanh from one v_exp_f32 + one v_rcp_f32 (libm tanhf is ~10x the
// instructions and made the GELU backward VALU-bound); |err| < 1e-6 abs,
// saturates correctly at +-inf.
__device__ __forceinline__ float fast_tanh(float x) {
  return 1.f - __fdividef(2.f, __expf(2.f * x) + 1.f);
}
// tanh-approximated GELU in its sigmoid form: 0.5 (1 + tanh u) = s = 1 / (1 +
// 2^(-2 u log2 e)), u = k0 (x + k1 x^3): bare v_exp_f32 + v_rcp_f32 and a few
// FMAs per element (the GEMM epilogues apply it to 256 values per lane, where
// libm exp / divide fix-ups tripled the VALU work).  x -> -inf: 2^arg = inf,
// s = 0; x -> +inf: s = 1.
__device__ __forceinline__ float gelu_sig(float x, float x2) {
  constexpr float k1 = 0.044715f, c = -2.f * 0.7978845608028654f * 1.4426950408889634f;
  const float arg = x * __builtin_fmaf(c * k1, x2, c);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(arg));
}
__device__ __forceinline__ float gelu_tanh(float x) { return x * gelu_sig(x, x * x); }
// d/dx [x s(2u)] = s + x s (1 - s) 2 k0 (1 + 3 k1 x^2)
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  constexpr float k0x2 = 2.f * 0.7978845608028654f, k1x3 = 3.f * 0.044715f;
  const float x2 = x * x;
  const float s = gelu_sig(x, x2);
  const float w = x * __builtin_fmaf(k0x2 * k1x3, x2, k0x2);
  return __builtin_fmaf(w, s - s * s, s);
}

// Counter-based RNG (splitmix64 finaliser) for dropout: deterministic in
// (seed, offset, element index), so forward and backward regenerate the same
// mask without storing it and hipGraph replays stay reproducible.
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ULL * (idx + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  z ^= z >> 31;
  return static_cast<uint32_t>(z);
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t idx) {
  return (hash_u32(seed, idx) >> 8) * (1.0f / 16777216.0f);
}

inline void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

inline int grid_for(int64_t n, int per_block, int cap = 256 * 16) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

}  // namespace ffk

#define FFK_LAUNCH_CHECK(name) ::ffk::check(hipGetLastError(), name)
