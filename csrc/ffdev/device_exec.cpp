// GPU training backing of the legacy C API (ff/training_backing.h).
//
// Parity: the reference's C API (python/flexflow_c.cc:183-194, model
// compile / forward / backward / update) drives its GPU runtime; here the
// same entry points (csrc/ffi/flexflow_runtime_c.cc) drive this backing when a
// GPU is visible.  Design, single process / single GPU:
//  * every graph tensor and gradient lives in one device arena (256-B
//    aligned pieces); weights are initialised by the CPU backing's
//    initialisers (same values as a CPU run with the same seed) and uploaded;
//  * operators on the production kernel library (csrc/kernels, fp32 paths):
//    LINEAR, BATCHMATMUL and MULTIHEAD_ATTENTION on the exact-fp32 MFMA GEMM
//    (igemm32.hip: bias and the activation in its epilogue, the
//    pre-activation kept for backward; batched over heads x batch for the
//    attention scores), LAYERNORM (layernorm.hip), EMBEDDING (embedding.hip),
//    SOFTMAX (softmax.hip), CONCAT / SPLIT (tensorops.hip slice_copy), bias
//    gradients (elementwise.hip colsum_act), the last SOFTMAX fused with
//    sparse cross-entropy, MSE (tensorops.hip); small kernels below for the
//    shapes those kernels do not take (rows not a multiple of 8), DROPOUT
//    (the CPU backing's counter-hash mask, bit for bit), CONV2D / POOL2D /
//    BATCHNORM (NCHW, direct formulations), element-wise activations /
//    binaries / scalar ops / reshapes; a graph with any other operator stays
//    on the CPU backing (make_device_backing returns null);
//  * the host slots are mirrors: slot() copies a tensor out when the device
//    copy is newer and marks it written, and the next device step copies
//    written mirrors back -- the inline-mapping protocol of the reference's
//    regions, without Legion;
//  * SGD (momentum, Nesterov, L2) and Adam (L2 folded into the gradient, as
//    the CPU backing and the reference's adam_update) on the device.
// Everything runs on one HIP stream; metrics accumulate on the device and are
// read back when asked for.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "ff/local_exec.h"
#include "ff/training_backing.h"
#include "kernels.h"

namespace ff {
namespace {

#define FFD_CHECK(x)                                                                                  \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) throw FFError(std::string("device backing: ") + #x + ": " + hipGetErrorString(e_)); \
  } while (0)

// ----------------------------------------------------------------- kernels
constexpr int kDtF32 = 0;   // the kernel library's fp32 dtype code (csrc/kernels/common.h DType)

enum DAct : int { A_NONE = 0, A_RELU = 1, A_SIGMOID = 2, A_TANH = 3, A_GELU = 4, A_ELU = 5 };

__device__ __forceinline__ float d_act(int a, float x) {
  switch (a) {
    case A_RELU: return x > 0.f ? x : 0.f;
    case A_SIGMOID: return 1.f / (1.f + expf(-x));
    case A_TANH: return tanhf(x);
    case A_GELU: {
      const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
      return 0.5f * x * (1.f + tanhf(u));
    }
    case A_ELU: return x > 0.f ? x : expf(x) - 1.f;
    default: return x;
  }
}
__device__ __forceinline__ float d_act_grad(int a, float x) {
  switch (a) {
    case A_RELU: return x > 0.f ? 1.f : 0.f;
    case A_SIGMOID: {
      const float s = 1.f / (1.f + expf(-x));
      return s * (1.f - s);
    }
    case A_TANH: {
      const float t = tanhf(x);
      return 1.f - t * t;
    }
    case A_GELU: {
      const float k = 0.7978845608028654f;
      const float u = k * (x + 0.044715f * x * x * x);
      const float t = tanhf(u);
      return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
    }
    case A_ELU: return x > 0.f ? 1.f : expf(x);
    default: return 1.f;
  }
}

#define GRID_LOOP(i, n) for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < (n); i += 256ll * gridDim.x)

__global__ __launch_bounds__(256) void k_act(const float* x, float* y, int64_t n, int a) {
  GRID_LOOP(i, n) y[i] = d_act(a, x[i]);
}
// dx += dy * act'(x)   (x = the activation's input)
__global__ __launch_bounds__(256) void k_act_bwd(const float* dy, const float* x, float* dx, int64_t n, int a) {
  GRID_LOOP(i, n) dx[i] += dy[i] * d_act_grad(a, x[i]);
}
// g = dy * act'(pre)
__global__ __launch_bounds__(256) void k_act_grad(const float* dy, const float* pre, float* g, int64_t n, int a) {
  GRID_LOOP(i, n) g[i] = dy[i] * d_act_grad(a, pre[i]);
}
__global__ __launch_bounds__(256) void k_axpy(const float* x, float* y, int64_t n, float a) {
  GRID_LOOP(i, n) y[i] += a * x[i];
}
// db[j] += sum_r g[r, j]: one thread per column, rows strided
__global__ __launch_bounds__(256) void k_colsum(const float* g, float* db, int64_t rows, int64_t cols) {
  const int64_t j = blockIdx.x * 256ll + threadIdx.x;
  if (j >= cols) return;
  float s = 0.f;
  for (int64_t r = 0; r < rows; ++r) s += g[r * cols + j];
  db[j] += s;
}
// op: 0 add 1 sub 2 mul 3 div 4 max 5 min
__global__ __launch_bounds__(256) void k_binary(const float* a, const float* b, float* y, int64_t n, int op) {
  GRID_LOOP(i, n) {
    const float u = a[i], v = b[i];
    float r;
    switch (op) {
      case 0: r = u + v; break;
      case 1: r = u - v; break;
      case 2: r = u * v; break;
      case 3: r = u / v; break;
      case 4: r = fmaxf(u, v); break;
      default: r = fminf(u, v); break;
    }
    y[i] = r;
  }
}
__global__ __launch_bounds__(256) void k_binary_bwd(const float* g, const float* a, const float* b, float* da,
                                                    float* db, int64_t n, int op) {
  GRID_LOOP(i, n) {
    const float u = a[i], v = b[i], d = g[i];
    float ga = 0.f, gb = 0.f;
    switch (op) {
      case 0: ga = d; gb = d; break;
      case 1: ga = d; gb = -d; break;
      case 2: ga = d * v; gb = d * u; break;
      case 3: ga = d / v; gb = -d * u / (v * v); break;
      case 4: (u >= v ? ga : gb) = d; break;
      default: (u <= v ? ga : gb) = d; break;
    }
    if (da) da[i] += ga;
    if (db) db[i] += gb;
  }
}
// op: 0 *s 1 +s 2 -s 3 /s
__global__ __launch_bounds__(256) void k_scalar(const float* x, float* y, int64_t n, int op, float s) {
  GRID_LOOP(i, n) {
    const float u = x[i];
    y[i] = op == 0 ? u * s : op == 1 ? u + s : op == 2 ? u - s : u / s;
  }
}
// softmax over the last dim, one block per row
__global__ __launch_bounds__(256) void k_softmax(const float* x, float* y, int64_t cols) {
  __shared__ float red[256];
  const float* xr = x + blockIdx.x * cols;
  float* yr = y + blockIdx.x * cols;
  float m = -INFINITY;
  for (int64_t j = threadIdx.x; j < cols; j += 256) m = fmaxf(m, xr[j]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  m = red[0];
  __syncthreads();
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < cols; j += 256) s += expf(xr[j] - m);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float inv = 1.f / red[0];
  for (int64_t j = threadIdx.x; j < cols; j += 256) yr[j] = expf(xr[j] - m) * inv;
}
// dx += y * (dy - sum(dy * y)), one block per row
__global__ __launch_bounds__(256) void k_softmax_bwd(const float* dy, const float* y, float* dx, int64_t cols) {
  __shared__ float red[256];
  const int64_t base = blockIdx.x * cols;
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < cols; j += 256) s += dy[base + j] * y[base + j];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float dot = red[0];
  for (int64_t j = threadIdx.x; j < cols; j += 256) dx[base + j] += y[base + j] * (dy[base + j] - dot);
}
// fused softmax + cross-entropy on probabilities p (the softmax output):
// g[logits] += (p - onehot(y)) * scale; metrics {loss, correct, rows}
__global__ __launch_bounds__(256) void k_sparse_ce(const float* p, const int* labels, float* g, float* metrics,
                                                   int64_t rows, int64_t cols, float scale) {
  const int64_t r = blockIdx.x * 256ll + threadIdx.x;
  if (r >= rows) return;
  const float* pr = p + r * cols;
  const int y = labels[r];
  int am = 0;
  for (int64_t j = 1; j < cols; ++j)
    if (pr[j] > pr[am]) am = static_cast<int>(j);
  for (int64_t j = 0; j < cols; ++j) g[r * cols + j] += (pr[j] - (j == y ? 1.f : 0.f)) * scale;
  const float py = (y >= 0 && y < cols) ? pr[y] : 1.f;
  atomicAdd(metrics + 0, -logf(fmaxf(py, 1e-30f)));
  atomicAdd(metrics + 1, am == y ? 1.f : 0.f);
}
__global__ __launch_bounds__(256) void k_sgd(float* w, const float* g, float* buf, int64_t n, float lr, float mom,
                                             float wd, int nesterov) {
  GRID_LOOP(i, n) {
    float gg = g[i] + wd * w[i];
    if (buf) {
      buf[i] = mom * buf[i] + gg;
      gg = nesterov ? gg + mom * buf[i] : buf[i];
    }
    w[i] -= lr * gg;
  }
}
__global__ __launch_bounds__(256) void k_adam(float* w, const float* g, float* m, float* v, int64_t n, float lr,
                                              float b1, float b2, float eps, float wd, float bc1, float bc2) {
  GRID_LOOP(i, n) {
    const float gg = g[i] + wd * w[i];
    m[i] = b1 * m[i] + (1.f - b1) * gg;
    v[i] = b2 * v[i] + (1.f - b2) * gg * gg;
    w[i] -= lr * (m[i] / bc1) / (sqrtf(v[i] / bc2) + eps);
  }
}

// ---- conv2d / pool2d / batch norm, NCHW fp32 (the C API's small CNNs):
// direct formulations, one thread per output element (forward, dgrad), one
// block per weight element (wgrad) or channel (bias, batch norm).
struct CG {
  int N, C, H, W, O, OH, OW, KH, KW, SH, SW, PH, PW, G;
};
__global__ __launch_bounds__(256) void k_conv_fwd(const float* x, const float* w, const float* bias, float* y,
                                                  float* pre, CG g, int act) {
  const int64_t total = static_cast<int64_t>(g.N) * g.O * g.OH * g.OW;
  const int cpg = g.C / g.G, opg = g.O / g.G;
  GRID_LOOP(i, total) {
    const int ow = i % g.OW, oh = (i / g.OW) % g.OH, o = (i / (static_cast<int64_t>(g.OW) * g.OH)) % g.O;
    const int n = static_cast<int>(i / (static_cast<int64_t>(g.OW) * g.OH * g.O));
    const int grp = o / opg;
    float acc = bias ? bias[o] : 0.f;
    for (int ci = 0; ci < cpg; ++ci)
      for (int kh = 0; kh < g.KH; ++kh) {
        const int ih = oh * g.SH - g.PH + kh;
        if (ih < 0 || ih >= g.H) continue;
        for (int kw = 0; kw < g.KW; ++kw) {
          const int iw = ow * g.SW - g.PW + kw;
          if (iw < 0 || iw >= g.W) continue;
          acc = __builtin_fmaf(x[((static_cast<int64_t>(n) * g.C + grp * cpg + ci) * g.H + ih) * g.W + iw],
                               w[((static_cast<int64_t>(o) * cpg + ci) * g.KH + kh) * g.KW + kw], acc);
        }
      }
    if (pre) pre[i] = acc;
    y[i] = d_act(act, acc);
  }
}
// dx += sum over the outputs that read x[n, c, ih, iw]
__global__ __launch_bounds__(256) void k_conv_dgrad(const float* gy, const float* w, float* dx, CG g) {
  const int64_t total = static_cast<int64_t>(g.N) * g.C * g.H * g.W;
  const int cpg = g.C / g.G, opg = g.O / g.G;
  GRID_LOOP(i, total) {
    const int iw = i % g.W, ih = (i / g.W) % g.H, c = (i / (static_cast<int64_t>(g.W) * g.H)) % g.C;
    const int n = static_cast<int>(i / (static_cast<int64_t>(g.W) * g.H * g.C));
    const int grp = c / cpg, ci = c % cpg;
    float acc = 0.f;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int th = ih + g.PH - kh;
      if (th < 0 || th % g.SH) continue;
      const int oh = th / g.SH;
      if (oh >= g.OH) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int tw = iw + g.PW - kw;
        if (tw < 0 || tw % g.SW) continue;
        const int ow = tw / g.SW;
        if (ow >= g.OW) continue;
        for (int oo = 0; oo < opg; ++oo) {
          const int o = grp * opg + oo;
          acc = __builtin_fmaf(gy[((static_cast<int64_t>(n) * g.O + o) * g.OH + oh) * g.OW + ow],
                               w[((static_cast<int64_t>(o) * cpg + ci) * g.KH + kh) * g.KW + kw], acc);
        }
      }
    }
    dx[i] += acc;
  }
}
// dw[o, ci, kh, kw] += sum_{n, oh, ow} gy * x: one block per weight element
__global__ __launch_bounds__(256) void k_conv_wgrad(const float* gy, const float* x, float* dw, CG g) {
  __shared__ float red[256];
  const int cpg = g.C / g.G, opg = g.O / g.G;
  const int64_t wi = blockIdx.x;
  const int kw = wi % g.KW, kh = (wi / g.KW) % g.KH, ci = (wi / (g.KW * g.KH)) % cpg;
  const int o = static_cast<int>(wi / (static_cast<int64_t>(g.KW) * g.KH * cpg));
  const int c = (o / opg) * cpg + ci;
  const int64_t total = static_cast<int64_t>(g.N) * g.OH * g.OW;
  float acc = 0.f;
  for (int64_t t = threadIdx.x; t < total; t += 256) {
    const int ow = t % g.OW, oh = (t / g.OW) % g.OH, n = static_cast<int>(t / (static_cast<int64_t>(g.OW) * g.OH));
    const int ih = oh * g.SH - g.PH + kh, iw = ow * g.SW - g.PW + kw;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) continue;
    acc = __builtin_fmaf(gy[((static_cast<int64_t>(n) * g.O + o) * g.OH + oh) * g.OW + ow],
                         x[((static_cast<int64_t>(n) * g.C + c) * g.H + ih) * g.W + iw], acc);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (static_cast<int>(threadIdx.x) < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) dw[wi] += red[0];
}
// db[c] += sum over n and the S spatial positions of g[n, c, :] (one block per channel)
__global__ __launch_bounds__(256) void k_chan_sum(const float* gsrc, float* db, int N, int C, int64_t S) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  float acc = 0.f;
  for (int64_t t = threadIdx.x; t < static_cast<int64_t>(N) * S; t += 256) {
    const int64_t n = t / S, s = t % S;
    acc += gsrc[(n * C + c) * S + s];
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (static_cast<int>(threadIdx.x) < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) db[c] += red[0];
}
// pool: aux = argmax input index (max) or the window count (avg), as floats
__global__ __launch_bounds__(256) void k_pool_fwd(const float* x, float* y, float* pre, float* aux, CG g, int mx,
                                                  int act) {
  const int64_t total = static_cast<int64_t>(g.N) * g.C * g.OH * g.OW;
  GRID_LOOP(i, total) {
    const int ow = i % g.OW, oh = (i / g.OW) % g.OH;
    const int64_t nc = i / (static_cast<int64_t>(g.OW) * g.OH);
    float acc = mx ? -INFINITY : 0.f;
    int64_t best = -1;
    int cnt = 0;
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.SH - g.PH + kh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.SW - g.PW + kw;
        if (iw < 0 || iw >= g.W) continue;
        const int64_t xi = (nc * g.H + ih) * g.W + iw;
        const float v = x[xi];
        if (mx) {
          if (v > acc) acc = v, best = xi;
        } else {
          acc += v;
          ++cnt;
        }
      }
    }
    const float o = mx ? acc : acc / static_cast<float>(cnt > 0 ? cnt : 1);
    aux[i] = static_cast<float>(mx ? best : cnt);
    if (pre) pre[i] = o;
    y[i] = d_act(act, o);
  }
}
__global__ __launch_bounds__(256) void k_pool_bwd(const float* dy, const float* pre, const float* aux, float* dx,
                                                  CG g, int mx, int act) {
  const int64_t total = static_cast<int64_t>(g.N) * g.C * g.OH * g.OW;
  GRID_LOOP(i, total) {
    float gv = dy[i];
    if (pre) gv *= d_act_grad(act, pre[i]);
    if (mx) {
      const int64_t b = static_cast<int64_t>(aux[i]);
      if (b >= 0) atomicAdd(dx + b, gv);
      continue;
    }
    const int ow = i % g.OW, oh = (i / g.OW) % g.OH;
    const int64_t nc = i / (static_cast<int64_t>(g.OW) * g.OH);
    const float share = gv / fmaxf(1.f, aux[i]);
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.SH - g.PH + kh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.SW - g.PW + kw;
        if (iw < 0 || iw >= g.W) continue;
        atomicAdd(dx + (nc * g.H + ih) * g.W + iw, share);
      }
    }
  }
}
// batch norm over N and S per channel (one block per channel); aux = {mean, inv std}[C]
__global__ __launch_bounds__(256) void k_bn_fwd(const float* x, const float* gamma, const float* beta, float* y,
                                                float* aux, int N, int C, int64_t S, float eps, int relu) {
  __shared__ float red[256];
  const int c = blockIdx.x;
  const int64_t cnt = static_cast<int64_t>(N) * S;
  auto at = [&](int64_t t) { return (t / S * C + c) * S + t % S; };
  float s = 0.f;
  for (int64_t t = threadIdx.x; t < cnt; t += 256) s += x[at(t)];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (static_cast<int>(threadIdx.x) < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  const float mean = red[0] / static_cast<float>(cnt);
  __syncthreads();
  float v = 0.f;
  for (int64_t t = threadIdx.x; t < cnt; t += 256) {
    const float d = x[at(t)] - mean;
    v += d * d;
  }
  red[threadIdx.x] = v;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (static_cast<int>(threadIdx.x) < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  const float inv = 1.f / sqrtf(red[0] / static_cast<float>(cnt) + eps);
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  for (int64_t t = threadIdx.x; t < cnt; t += 256) {
    float o = (x[at(t)] - mean) * inv * gm + bt;
    if (relu && o < 0.f) o = 0.f;
    y[at(t)] = o;
  }
  if (threadIdx.x == 0) {
    aux[c] = mean;
    aux[C + c] = inv;
  }
}
__global__ __launch_bounds__(256) void k_bn_bwd(const float* dy, const float* x, const float* y, const float* gamma,
                                                const float* aux, float* dx, float* dgamma, float* dbeta, int N,
                                                int C, int64_t S, int relu) {
  __shared__ float ra[256], rb[256];
  const int c = blockIdx.x;
  const int64_t cnt = static_cast<int64_t>(N) * S;
  auto at = [&](int64_t t) { return (t / S * C + c) * S + t % S; };
  const float mean = aux[c], inv = aux[C + c];
  float sg = 0.f, sgx = 0.f;
  for (int64_t t = threadIdx.x; t < cnt; t += 256) {
    const int64_t i = at(t);
    float gv = dy[i];
    if (relu && y[i] <= 0.f) gv = 0.f;
    sg += gv;
    sgx += gv * (x[i] - mean) * inv;
  }
  ra[threadIdx.x] = sg;
  rb[threadIdx.x] = sgx;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (static_cast<int>(threadIdx.x) < k) {
      ra[threadIdx.x] += ra[threadIdx.x + k];
      rb[threadIdx.x] += rb[threadIdx.x + k];
    }
    __syncthreads();
  }
  sg = ra[0];
  sgx = rb[0];
  if (threadIdx.x == 0) {
    if (dgamma) dgamma[c] += sgx;
    if (dbeta) dbeta[c] += sg;
  }
  if (!dx) return;
  const float gm = gamma ? gamma[c] : 1.f, fc = static_cast<float>(cnt);
  for (int64_t t = threadIdx.x; t < cnt; t += 256) {
    const int64_t i = at(t);
    float gv = dy[i];
    if (relu && y[i] <= 0.f) gv = 0.f;
    const float xh = (x[i] - mean) * inv;
    dx[i] += gm * inv * (gv - sg / fc - xh * sgx / fc);
  }
}

// ---- dropout: the CPU backing's counter-hash mask (local_exec.cc hash_uniform), bit for bit
__device__ __forceinline__ float d_hash_uniform(uint64_t seed, uint64_t i) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + i + 0x632BE59BD9B4E019ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return static_cast<float>(z >> 40) * (1.0f / 16777216.0f);
}
// bwd = 0: y = mask(x) / (1 - p); bwd = 1: y += mask(x) / (1 - p)
__global__ __launch_bounds__(256) void k_dropout(const float* x, float* y, int64_t n, float p, uint64_t seed,
                                                 int bwd) {
  GRID_LOOP(i, n) {
    const float v = (p > 0.f && d_hash_uniform(seed, static_cast<uint64_t>(i)) < p) ? 0.f : x[i] / (1.f - p);
    if (bwd) y[i] += v;
    else y[i] = v;
  }
}
// float-carried indices -> int32 (the embedding kernels' index type)
__global__ __launch_bounds__(256) void k_f2i(const float* x, int* y, int64_t n) {
  GRID_LOOP(i, n) y[i] = static_cast<int>(x[i]);
}
// embedding for rows of D % 8 != 0 (embedding.hip takes 16-B rows)
__global__ __launch_bounds__(256) void k_embed_fwd(const int* idx, const float* W, float* y, int64_t B, int L,
                                                   int64_t D, float s) {
  GRID_LOOP(i, B * D) {
    const int64_t b = i / D, d = i % D;
    float acc = 0.f;
    for (int l = 0; l < L; ++l) acc += W[static_cast<int64_t>(idx[b * L + l]) * D + d];
    y[i] = s * acc;
  }
}
__global__ __launch_bounds__(256) void k_embed_bwd(const int* idx, const float* g, float* dW, int64_t B, int L,
                                                   int64_t D, float s) {
  GRID_LOOP(i, B * L * D) {
    const int64_t bl = i / D, d = i % D;
    atomicAdd(dW + static_cast<int64_t>(idx[bl]) * D + d, s * g[(bl / L) * D + d]);
  }
}
// layer norm over rows of N % 8 != 0 (layernorm.hip takes 16-B rows): one
// block per row; aux = {mean[R], rstd[R]}
__global__ __launch_bounds__(256) void k_ln_fwd(const float* x, const float* gamma, const float* beta, float* y,
                                                float* mean, float* rstd, int64_t N, float eps) {
  __shared__ float red[256];
  const float* xr = x + blockIdx.x * N;
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < N; j += 256) s += xr[j];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float mu = red[0] / static_cast<float>(N);
  __syncthreads();
  float v = 0.f;
  for (int64_t j = threadIdx.x; j < N; j += 256) v += (xr[j] - mu) * (xr[j] - mu);
  red[threadIdx.x] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float rs = 1.f / sqrtf(red[0] / static_cast<float>(N) + eps);
  for (int64_t j = threadIdx.x; j < N; j += 256) {
    float o = (xr[j] - mu) * rs;
    if (gamma) o = o * gamma[j] + (beta ? beta[j] : 0.f);
    y[blockIdx.x * N + j] = o;
  }
  if (threadIdx.x == 0) {
    mean[blockIdx.x] = mu;
    rstd[blockIdx.x] = rs;
  }
}
__global__ __launch_bounds__(256) void k_ln_bwd(const float* dy, const float* x, const float* gamma,
                                                const float* mean, const float* rstd, float* dx, float* dgamma,
                                                float* dbeta, int64_t N) {
  __shared__ float ra[256], rb[256];
  const int64_t r = blockIdx.x;
  const float mu = mean[r], rs = rstd[r];
  float s1 = 0.f, s2 = 0.f;
  for (int64_t j = threadIdx.x; j < N; j += 256) {
    const float xh = (x[r * N + j] - mu) * rs, g = dy[r * N + j];
    const float gg = g * (gamma ? gamma[j] : 1.f);
    s1 += gg;
    s2 += gg * xh;
    if (dgamma) atomicAdd(dgamma + j, g * xh);
    if (dbeta) atomicAdd(dbeta + j, g);
  }
  ra[threadIdx.x] = s1;
  rb[threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) {
      ra[threadIdx.x] += ra[threadIdx.x + o];
      rb[threadIdx.x] += rb[threadIdx.x + o];
    }
    __syncthreads();
  }
  if (!dx) return;
  const float m1 = ra[0] / static_cast<float>(N), m2 = rb[0] / static_cast<float>(N);
  for (int64_t j = threadIdx.x; j < N; j += 256) {
    const float xh = (x[r * N + j] - mu) * rs;
    const float gg = dy[r * N + j] * (gamma ? gamma[j] : 1.f);
    dx[r * N + j] += rs * (gg - m1 - xh * m2);
  }
}
// ---- multi-head attention helpers (op_attrs mha layout: weight [P, H], head
// h's column holds Wq [Eq, k] | Wk [Ek, k] | Wv [Ev, v] | Wo [v, E] row-major)
// Wd[h][p] = W[p][h] (to = 1: dW[p][h] += dWd[h][p])
__global__ __launch_bounds__(256) void k_head_major(const float* src, float* dst, int64_t P, int64_t H, int to) {
  GRID_LOOP(i, P * H) {
    const int64_t h = i / P, p = i % P;
    if (to) dst[p * H + h] += src[i];
    else dst[i] = src[p * H + h];
  }
}
// x[h][r][j] += bias[(off + j) * H + h] for r < R
__global__ __launch_bounds__(256) void k_head_bias(float* x, const float* bias, int64_t H, int64_t R, int64_t D,
                                                   int64_t off) {
  GRID_LOOP(i, H * R * D) {
    const int64_t j = i % D, h = i / (R * D);
    x[i] += bias[(off + j) * H + h];
  }
}
// dbias[(off + j) * H + h] += sum_r g[h][r][j]: one thread per (h, j)
__global__ __launch_bounds__(256) void k_head_bias_grad(const float* g, float* dbias, int64_t H, int64_t R,
                                                        int64_t D, int64_t off) {
  GRID_LOOP(i, H * D) {
    const int64_t h = i / D, j = i % D;
    const float* gh = g + h * R * D;
    float s = 0.f;
    for (int64_t r = 0; r < R; ++r) s += gh[r * D + j];
    dbias[(off + j) * H + h] += s;
  }
}
// scores -> probabilities in place, rows of Sk: scale, causal mask (query
// row q = row % Sq sees keys <= q), softmax; one block per row
__global__ __launch_bounds__(256) void k_attn_softmax(float* p, int64_t Sq, int64_t Sk, float scale, int causal) {
  __shared__ float red[256];
  float* r = p + blockIdx.x * Sk;
  const int64_t q = blockIdx.x % Sq;
  float m = -INFINITY;
  for (int64_t j = threadIdx.x; j < Sk; j += 256) {
    const float v = (causal && j > q) ? -INFINITY : r[j] * scale;
    r[j] = v;
    m = fmaxf(m, v);
  }
  red[threadIdx.x] = m;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + o]);
    __syncthreads();
  }
  m = red[0];
  __syncthreads();
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < Sk; j += 256) {
    const float e = r[j] == -INFINITY ? 0.f : expf(r[j] - m);
    r[j] = e;
    s += e;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float inv = 1.f / red[0];
  for (int64_t j = threadIdx.x; j < Sk; j += 256) r[j] *= inv;
}
// dS = P * (dP - rowsum(P * dP)) * scale, in place in dP
__global__ __launch_bounds__(256) void k_attn_softmax_bwd(const float* p, float* dp, int64_t Sk, float scale) {
  __shared__ float red[256];
  const float* pr = p + blockIdx.x * Sk;
  float* dr = dp + blockIdx.x * Sk;
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < Sk; j += 256) s += pr[j] * dr[j];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (static_cast<int>(threadIdx.x) < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  const float dot = red[0];
  for (int64_t j = threadIdx.x; j < Sk; j += 256) dr[j] = pr[j] * (dr[j] - dot) * scale;
}
// y[r][e] += b[e]
__global__ __launch_bounds__(256) void k_add_rows(float* y, const float* b, int64_t R, int64_t E) {
  GRID_LOOP(i, R * E) y[i] += b[i % E];
}

int grid_of(int64_t n) { return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096))); }

int dact_of(const std::string& s) {
  if (s == "relu") return A_RELU;
  if (s == "sigmoid") return A_SIGMOID;
  if (s == "tanh") return A_TANH;
  if (s == "gelu") return A_GELU;
  if (s == "elu") return A_ELU;
  return A_NONE;
}
int dact_of(OpType t) {
  switch (t) {
    case OpType::RELU: return A_RELU;
    case OpType::SIGMOID: return A_SIGMOID;
    case OpType::TANH: return A_TANH;
    case OpType::GELU: return A_GELU;
    case OpType::ELU: return A_ELU;
    default: return -1;
  }
}
// the igemm32 epilogue's activation codes (elementwise.hip Act)
int gemm_act(int a) { return a == A_RELU ? 1 : a == A_SIGMOID ? 2 : a == A_TANH ? 3 : a == A_GELU ? 4 : 0; }
int binary_of(OpType t) {
  switch (t) {
    case OpType::EW_ADD: return 0;
    case OpType::EW_SUB: return 1;
    case OpType::EW_MUL: return 2;
    case OpType::EW_DIV: return 3;
    case OpType::EW_MAX: return 4;
    case OpType::EW_MIN: return 5;
    default: return -1;
  }
}
int scalar_of(OpType t) {
  switch (t) {
    case OpType::SCALAR_MULTIPLY: return 0;
    case OpType::SCALAR_ADD: return 1;
    case OpType::SCALAR_SUB: return 2;
    case OpType::SCALAR_TRUE_DIV: return 3;
    default: return -1;
  }
}
bool is_view(OpType t) { return t == OpType::FLAT || t == OpType::RESHAPE; }

// why the device cannot run operator `t` (empty: it can)
std::string unsupported(const ComputationGraph& cg, int n) {
  const auto& node = cg.g.node(n);
  const OpType t = node.label.op.type;
  if (t == OpType::LINEAR) {
    const std::string a = node.label.op.s("activation");
    if (!a.empty() && a != "none" && dact_of(a) == A_NONE) return "LINEAR activation " + a;
    return "";
  }
  if (t == OpType::CONV2D || t == OpType::POOL2D) {
    const std::string a = node.label.op.s("activation");
    if (!a.empty() && a != "none" && dact_of(a) == A_NONE) return to_string(t) + " activation " + a;
    if (cg.shape(cg.layer_data_inputs(n)[0]).dims.size() != 4) return to_string(t) + " on a non-4-D tensor";
    if (t == OpType::POOL2D) {
      const std::string pt = node.label.op.s("pool_type");
      if (pt != "max" && pt != "avg") return "pool type " + pt;
    }
    return "";
  }
  if (t == OpType::BATCHNORM || t == OpType::BATCHMATMUL || t == OpType::CONCAT || t == OpType::SPLIT ||
      t == OpType::DROPOUT)
    return "";
  if (t == OpType::EMBEDDING) {
    const std::string a = node.label.op.s("aggr");
    if (a != "none" && a != "sum" && a != "avg") return "embedding aggregation " + a;
    return "";
  }
  if (t == OpType::LAYERNORM) {
    // the normalised axes must be the trailing ones (rows x N)
    const auto& d = cg.shape(cg.layer_data_inputs(n)[0]).dims;
    const int nd = static_cast<int>(d.size());
    std::vector<int> ax;
    for (auto a : node.label.op.ints("axes")) ax.push_back(static_cast<int>((a % nd + nd) % nd));
    std::sort(ax.begin(), ax.end());
    for (size_t i = 0; i < ax.size(); ++i)
      if (ax[i] != nd - static_cast<int>(ax.size()) + static_cast<int>(i)) return "layer norm over non-trailing axes";
    return "";
  }
  if (t == OpType::MULTIHEAD_ATTENTION) {
    const auto ins = cg.layer_data_inputs(n);
    if (ins.size() != 3 || cg.shape(ins[0]).dims.size() != 3) return "attention inputs";
    return "";
  }
  if (dact_of(t) >= 0 || binary_of(t) >= 0 || scalar_of(t) >= 0 || is_view(t) || t == OpType::SOFTMAX) {
    if (binary_of(t) >= 0) {
      auto ins = cg.layer_data_inputs(n);
      if (cg.shape(ins[0]).num_elements() != cg.shape(ins[1]).num_elements())
        return "broadcasting " + to_string(t);
    }
    return "";
  }
  return "operator " + to_string(t);
}

class DeviceTrainingBacking final : public TrainingBacking {
 public:
  DeviceTrainingBacking(const ComputationGraph& cg, LocalOptimizer opt, const std::string& loss, uint64_t seed,
                        int dev)
      : cg_(cg), host_(cg, std::move(opt), loss, seed), dev_(dev), seed_(seed) {
    FFD_CHECK(hipSetDevice(dev_));
    FFD_CHECK(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    // one arena: every value, gradient, pre-activation and optimizer buffer
    std::vector<std::pair<Key, int64_t>> want;
    for (int n : cg_.layers_in_topo_order()) {
      const auto& node = cg_.g.node(n);
      for (size_t i = 0; i < node.outputs.size(); ++i) {
        ValueRef v{n, static_cast<int>(i)};
        if (!host_.slot(v, false)) continue;
        want.push_back({Key{v, 0}, host_.slot(v, false)->numel()});
        if (host_.slot(v, true)) want.push_back({Key{v, 1}, host_.slot(v, true)->numel()});
      }
    }
    for (int n : host_.order()) {
      const auto& node = cg_.g.node(n);
      const OpType t = node.label.op.type;
      const int64_t ne = host_.slot({n, 0}, false)->numel();
      if ((t == OpType::LINEAR || t == OpType::CONV2D || t == OpType::POOL2D) &&
          dact_of(node.label.op.s("activation")) != A_NONE)
        want.push_back({Key{{n, 0}, 2}, ne});   // pre-activation
      if (t == OpType::POOL2D) want.push_back({Key{{n, 0}, 3}, ne});   // argmax / window counts
      if (t == OpType::BATCHNORM)
        want.push_back({Key{{n, 0}, 3}, 2 * host_.slot(cg_.layer_data_inputs(n)[0], false)->dims.at(1)});
      if (t == OpType::EMBEDDING)   // int32 copy of the float-carried indices
        want.push_back({Key{{n, 0}, 3}, host_.slot(cg_.layer_data_inputs(n)[0], false)->numel()});
      if (t == OpType::LAYERNORM) {
        const int64_t N = ln_cols(n), R = ne / std::max<int64_t>(N, 1);
        want.push_back({Key{{n, 0}, 3}, 2 * R});   // mean, rstd
        if (N % 8 == 0) want.push_back({Key{{n, 0}, 4}, 3 * int64_t(ffk::layernorm_bwd_grid(R, N)) * N});
      }
      if (t == OpType::MULTIHEAD_ATTENTION) {
        const MG g = mha_of(n);
        const int64_t q = g.H * g.B * g.Sq, k = g.H * g.B * g.Sk, pp = g.H * g.B * g.Sq * g.Sk;
        for (auto const& kv : std::vector<std::pair<int, int64_t>>{
                 {10, g.H * g.P}, {11, q * g.kd}, {12, k * g.kd}, {13, k * g.vd}, {14, pp}, {15, q * g.vd},
                 {16, g.H * g.P}, {17, q * g.vd}, {18, q * g.kd}, {19, k * g.kd}, {20, k * g.vd}, {21, pp}})
          want.push_back({Key{{n, 0}, kv.first}, kv.second});
      }
      tmp_elems_ = std::max(tmp_elems_, ne);
      if (t == OpType::LAYERNORM || t == OpType::SOFTMAX)
        tmp_elems_ = std::max(tmp_elems_, host_.slot(cg_.layer_data_inputs(n)[0], false)->numel());
    }
    const ValueRef out = host_.output();
    rows_ = 1;
    cols_ = 1;
    {
      const auto& d = host_.slot(out, false)->dims;
      cols_ = d.empty() ? 1 : d.back();
      rows_ = host_.slot(out, false)->numel() / std::max<int64_t>(cols_, 1);
    }
    int64_t total = 0;
    auto align = [](int64_t n) { return (n + 63) / 64 * 64; };   // 256 B
    for (auto const& w : want) total += align(w.second);
    total += align(tmp_elems_) * 2 + align(rows_) + 64;
    FFD_CHECK(hipMalloc(&arena_, static_cast<size_t>(std::max<int64_t>(total, 64)) * sizeof(float)));
    FFD_CHECK(hipMemsetAsync(arena_, 0, static_cast<size_t>(std::max<int64_t>(total, 64)) * sizeof(float), st_));
    int64_t off = 0;
    for (auto const& w : want) {
      buf_[w.first] = {arena_ + off, w.second};
      off += align(w.second);
    }
    tmp_ = arena_ + off;
    off += align(tmp_elems_);
    tmp2_ = arena_ + off;
    off += align(tmp_elems_);
    labels_ = reinterpret_cast<int*>(arena_ + off);
    off += align(rows_);
    metrics_d_ = arena_ + off;   // 8 floats
    // every value / gradient slot starts host-written: the first step uploads
    for (auto const& kv : buf_)
      if (kv.first.kind < 2) state_[kv.first] = HOST;
  }
  ~DeviceTrainingBacking() override {
    if (st_) (void)hipStreamSynchronize(st_);
    if (arena_) (void)hipFree(arena_);
    for (auto& kv : opt_state_) (void)hipFree(kv.second);
    if (st_) (void)hipStreamDestroy(st_);
  }

  HostTensor* slot(const ValueRef& v, bool grad) override {
    HostTensor* h = host_.slot(v, grad);
    if (!h) return nullptr;
    Key k{v, grad ? 1 : 0};
    auto it = state_.find(k);
    if (it != state_.end() && it->second == DEVICE) {
      const Buf& b = buf_.at(k);
      FFD_CHECK(hipMemcpyAsync(h->v.data(), b.p, b.n * sizeof(float), hipMemcpyDeviceToHost, st_));
      FFD_CHECK(hipStreamSynchronize(st_));
    }
    if (it != state_.end()) it->second = HOST;   // the caller may write through the pointer
    return h;
  }
  ValueRef output() const override { return host_.output(); }
  LocalOptimizer& optimizer() override { return host_.optimizer(); }

  void forward_layer(int n) override {
    push();
    fwd(n);
  }
  void forward() override {
    push();
    for (int n : host_.order()) fwd(n);
  }
  void backward(const std::vector<float>& labels) override;
  void update() override;
  const LocalMetrics& metrics() const override {
    float m[8];
    FFD_CHECK(hipMemcpyAsync(m, metrics_d_, sizeof(m), hipMemcpyDeviceToHost, st_));
    FFD_CHECK(hipStreamSynchronize(st_));
    metrics_.loss_sum = m[0];
    metrics_.correct = static_cast<int64_t>(std::llround(m[1]));
    metrics_.samples = samples_;
    return metrics_;
  }
  void reset_metrics() override {
    FFD_CHECK(hipMemsetAsync(metrics_d_, 0, 8 * sizeof(float), st_));
    samples_ = 0;
  }
  std::string device() const override { return "gpu:" + std::to_string(dev_); }

 private:
  struct Key {
    ValueRef v;
    int kind;  // 0 value, 1 gradient, 2 pre-activation, 3 operator aux (argmax, BN statistics)
    bool operator<(const Key& o) const { return v < o.v || (v == o.v && kind < o.kind); }
  };
  struct Buf {
    float* p = nullptr;
    int64_t n = 0;
  };
  enum Where { HOST, DEVICE, SYNCED };

  float* val(const ValueRef& v) { return buf_.at(Key{v, 0}).p; }
  float* grad(const ValueRef& v) {
    auto it = buf_.find(Key{v, 1});
    return it == buf_.end() ? nullptr : it->second.p;
  }
  int64_t numel(const ValueRef& v) const { return buf_.at(Key{v, 0}).n; }
  void mark(const ValueRef& v, int kind) { state_[Key{v, kind}] = DEVICE; }

  // host-written mirrors -> device
  void push() {
    for (auto& kv : state_) {
      if (kv.second != HOST) continue;
      const HostTensor* h = host_.slot(kv.first.v, kv.first.kind == 1);
      const Buf& b = buf_.at(kv.first);
      FFD_CHECK(hipMemcpyAsync(b.p, h->v.data(), b.n * sizeof(float), hipMemcpyHostToDevice, st_));
      kv.second = SYNCED;
    }
    FFD_CHECK(hipStreamSynchronize(st_));   // the host buffers may be rewritten after return
  }

  void fwd(int n);
  void bwd(int n);
  void mha_fwd(int n);
  void mha_bwd(int n);

  // multi-head attention geometry (local_exec.cc MhaGeom)
  struct MG {
    int64_t B, Sq, Sk, Eq, Ek, Ev, E, H, kd, vd, P;
    int64_t off_q() const { return 0; }
    int64_t off_k() const { return Eq * kd; }
    int64_t off_v() const { return Eq * kd + Ek * kd; }
    int64_t off_o() const { return Eq * kd + Ek * kd + Ev * vd; }
  };
  MG mha_of(int n) {
    const auto& op = cg_.g.node(n).label.op;
    const auto ins = cg_.layer_data_inputs(n);
    const auto& q = host_.slot(ins[0], false)->dims;
    MG g{};
    g.B = q[0];
    g.Sq = q[1];
    g.Eq = q[2];
    g.Sk = host_.slot(ins[1], false)->dims[1];
    g.Ek = host_.slot(ins[1], false)->dims[2];
    g.Ev = host_.slot(ins[2], false)->dims[2];
    g.E = op.i("embed_dim");
    g.H = op.i("num_heads");
    g.kd = op.i("kdim") > 0 ? op.i("kdim") : g.E / g.H;
    g.vd = op.i("vdim") > 0 ? op.i("vdim") : g.E / g.H;
    g.P = g.Eq * g.kd + g.Ek * g.kd + g.Ev * g.vd + g.vd * g.E;
    return g;
  }
  // layer norm: elements per normalised row (the trailing axes)
  int64_t ln_cols(int n) {
    const auto& op = cg_.g.node(n).label.op;
    const auto& d = host_.slot(cg_.layer_data_inputs(n)[0], false)->dims;
    const int nd = static_cast<int>(d.size());
    int64_t N = 1;
    for (auto a : op.ints("axes")) N *= d[(a % nd + nd) % nd];
    return N;
  }
  float* aux(int n, int kind) { return buf_.at(Key{{n, 0}, kind}).p; }
  uint64_t op_seed(int n) const {
    return seed_ * 7919ull + static_cast<uint64_t>(n) * 104729ull + static_cast<uint64_t>(step_);
  }

  const ComputationGraph& cg_;
  LocalTrainingBacking host_;
  int dev_;
  uint64_t seed_;
  hipStream_t st_ = nullptr;
  float* arena_ = nullptr;
  float *tmp_ = nullptr, *tmp2_ = nullptr, *metrics_d_ = nullptr;
  int* labels_ = nullptr;
  int64_t tmp_elems_ = 1, rows_ = 1, cols_ = 1, step_ = 0, samples_ = 0;
  std::map<Key, Buf> buf_;
  std::map<Key, Where> state_;
  std::map<std::pair<int, int>, float*> opt_state_;   // (weight node, 0: momentum / m, 1: v)
  mutable LocalMetrics metrics_;
};

CG conv_geom_of(const HostTensor& x, const HostTensor& y, const OpAttrs& op, bool pool) {
  CG g{};
  g.N = static_cast<int>(x.dims[0]);
  g.C = static_cast<int>(x.dims[1]);
  g.H = static_cast<int>(x.dims[2]);
  g.W = static_cast<int>(x.dims[3]);
  g.O = static_cast<int>(y.dims[1]);
  g.OH = static_cast<int>(y.dims[2]);
  g.OW = static_cast<int>(y.dims[3]);
  g.KH = static_cast<int>(op.i("kernel_h"));
  g.KW = static_cast<int>(op.i("kernel_w"));
  g.SH = static_cast<int>(op.i("stride_h"));
  g.SW = static_cast<int>(op.i("stride_w"));
  g.PH = static_cast<int>(op.i("padding_h"));
  g.PW = static_cast<int>(op.i("padding_w"));
  g.G = pool ? 1 : static_cast<int>(op.i("groups"));
  return g;
}

void DeviceTrainingBacking::fwd(int n) {
  const auto& node = cg_.g.node(n);
  const OpAttrs& op = node.label.op;
  const OpType t = op.type;
  const auto ins = cg_.layer_data_inputs(n);
  const ValueRef o{n, 0};
  float* y = val(o);
  const int64_t ne = numel(o);
  if (t == OpType::LINEAR) {
    const auto ws = cg_.layer_weights(n);
    const auto& wd = host_.slot(ws[0], false)->dims;
    const int64_t in = wd[0], outc = wd[1], rows = numel(ins[0]) / in;
    const int a = dact_of(op.s("activation"));
    float* pre = a != A_NONE ? buf_.at(Key{o, 2}).p : nullptr;
    ffk::gemm_f32(val(ins[0]), val(ws[0]), y, ws.size() > 1 ? val(ws[1]) : nullptr, pre, rows, outc, in, in, outc,
                  outc, false, false, gemm_act(a), 1.f, 0.f, 1, 1, st_);
  } else if (t == OpType::CONV2D || t == OpType::POOL2D) {
    const bool pool = t == OpType::POOL2D;
    const CG g = conv_geom_of(*host_.slot(ins[0], false), *host_.slot(o, false), op, pool);
    const int a = dact_of(op.s("activation"));
    float* pre = a != A_NONE ? buf_.at(Key{o, 2}).p : nullptr;
    if (pool) {
      hipLaunchKernelGGL(k_pool_fwd, dim3(grid_of(ne)), dim3(256), 0, st_, val(ins[0]), y, pre,
                         buf_.at(Key{o, 3}).p, g, op.s("pool_type") == "max" ? 1 : 0, a);
    } else {
      const auto ws = cg_.layer_weights(n);
      hipLaunchKernelGGL(k_conv_fwd, dim3(grid_of(ne)), dim3(256), 0, st_, val(ins[0]), val(ws[0]),
                         ws.size() > 1 ? val(ws[1]) : nullptr, y, pre, g, a);
    }
  } else if (t == OpType::BATCHNORM) {
    const auto& xd = host_.slot(ins[0], false)->dims;
    int64_t S = 1;
    for (size_t k = 2; k < xd.size(); ++k) S *= xd[k];
    const auto ws = cg_.layer_weights(n);
    hipLaunchKernelGGL(k_bn_fwd, dim3(static_cast<unsigned>(xd[1])), dim3(256), 0, st_, val(ins[0]),
                       ws.size() > 0 ? val(ws[0]) : nullptr, ws.size() > 1 ? val(ws[1]) : nullptr, y,
                       buf_.at(Key{o, 3}).p, static_cast<int>(xd[0]), static_cast<int>(xd[1]), S,
                       static_cast<float>(op.f("eps")), op.b("relu") ? 1 : 0);
  } else if (dact_of(t) >= 0) {
    hipLaunchKernelGGL(k_act, dim3(grid_of(ne)), dim3(256), 0, st_, val(ins[0]), y, ne, dact_of(t));
  } else if (binary_of(t) >= 0) {
    hipLaunchKernelGGL(k_binary, dim3(grid_of(ne)), dim3(256), 0, st_, val(ins[0]), val(ins[1]), y, ne,
                       binary_of(t));
  } else if (scalar_of(t) >= 0) {
    hipLaunchKernelGGL(k_scalar, dim3(grid_of(ne)), dim3(256), 0, st_, val(ins[0]), y, ne, scalar_of(t),
                       static_cast<float>(op.f("scalar")));
  } else if (is_view(t)) {
    FFD_CHECK(hipMemcpyAsync(y, val(ins[0]), ne * sizeof(float), hipMemcpyDeviceToDevice, st_));
  } else if (t == OpType::SOFTMAX) {
    const auto& d = host_.slot(o, false)->dims;
    const int64_t cols = d.empty() ? 1 : d.back();
    ffk::softmax_fwd(kDtF32, val(ins[0]), y, static_cast<int>(ne / cols), static_cast<int>(cols), st_);
  } else if (t == OpType::EMBEDDING) {
    const auto ws = cg_.layer_weights(n);
    const auto& wd = host_.slot(ws[0], false)->dims;   // [entries, D]
    const int64_t E = wd[0], D = wd[1], nidx = numel(ins[0]);
    const std::string aggr = op.s("aggr");
    const auto& id = host_.slot(ins[0], false)->dims;
    const int L = aggr == "none" ? 1 : static_cast<int>(id.back());
    int* idx = reinterpret_cast<int*>(aux(n, 3));
    hipLaunchKernelGGL(k_f2i, dim3(grid_of(nidx)), dim3(256), 0, st_, val(ins[0]), idx, nidx);
    if (D % 8 == 0)
      ffk::embedding_fwd(kDtF32, 32, idx, val(ws[0]), y, nidx / L, L, static_cast<int>(D),
                         aggr == "none" ? 0 : aggr == "sum" ? 1 : 2, E, st_);
    else
      hipLaunchKernelGGL(k_embed_fwd, dim3(grid_of(ne)), dim3(256), 0, st_, idx, val(ws[0]), y, nidx / L, L, D,
                         aggr == "avg" ? 1.f / static_cast<float>(L) : 1.f);
  } else if (t == OpType::LAYERNORM) {
    const auto ws = cg_.layer_weights(n);
    const int64_t N = ln_cols(n), R = ne / N;
    const float* gm = ws.size() > 0 ? val(ws[0]) : nullptr;
    const float* bt = ws.size() > 1 ? val(ws[1]) : nullptr;
    float* st = aux(n, 3);
    if (N % 8 == 0)
      ffk::layernorm_fwd(kDtF32, val(ins[0]), nullptr, nullptr, gm, bt, y, st, st + R, static_cast<int>(R),
                         static_cast<int>(N), static_cast<float>(op.f("eps")), st_);
    else
      hipLaunchKernelGGL(k_ln_fwd, dim3(static_cast<unsigned>(R)), dim3(256), 0, st_, val(ins[0]), gm, bt, y, st,
                         st + R, N, static_cast<float>(op.f("eps")));
  } else if (t == OpType::BATCHMATMUL) {
    const auto& a = host_.slot(ins[0], false)->dims;
    const int nd = static_cast<int>(a.size());
    const int64_t M = a[nd - 2], K = a[nd - 1], N = host_.slot(ins[1], false)->dims.back();
    const int64_t Bt = numel(ins[0]) / (M * K);
    ffk::gemm_f32(val(ins[0]), val(ins[1]), y, nullptr, nullptr, M, N, K, K, N, N, false, false, 0, 1.f, 0.f, 1, 1,
                  st_, static_cast<int>(Bt), M * K, K * N, M * N);
  } else if (t == OpType::CONCAT || t == OpType::SPLIT) {
    const bool cat = t == OpType::CONCAT;
    const auto& big = cat ? host_.slot(o, false)->dims : host_.slot(ins[0], false)->dims;
    const int nd = static_cast<int>(big.size());
    const int ax = static_cast<int>((op.i("axis") % nd + nd) % nd);
    int64_t outer = 1, inner = 1;
    for (int k = 0; k < ax; ++k) outer *= big[k];
    for (int k = ax + 1; k < nd; ++k) inner *= big[k];
    int64_t off = 0;
    const size_t pieces = cat ? ins.size() : node.outputs.size();
    for (size_t j = 0; j < pieces; ++j) {
      const ValueRef pv = cat ? ins[j] : ValueRef{n, static_cast<int>(j)};
      const int64_t len = host_.slot(pv, false)->dims[ax];
      if (cat) ffk::slice_copy(kDtF32, val(pv), y, outer, len, inner, big[ax], off, 0, 0, st_);
      else ffk::slice_copy(kDtF32, val(ins[0]), val(pv), outer, len, inner, big[ax], off, 1, 0, st_);
      if (!cat) mark(pv, 0);
      off += len;
    }
  } else if (t == OpType::DROPOUT) {
    hipLaunchKernelGGL(k_dropout, dim3(grid_of(ne)), dim3(256), 0, st_, val(ins[0]), y, ne,
                       static_cast<float>(op.f("rate")), op_seed(n), 0);
  } else if (t == OpType::MULTIHEAD_ATTENTION) {
    mha_fwd(n);
  } else {
    throw FFError("device backing: no device implementation for " + to_string(t));
  }
  FFD_CHECK(hipGetLastError());
  mark(o, 0);
}

// ---- multi-head attention (local_exec.cc mha_fwd / mha_bwd) on batched
// fp32 MFMA GEMMs: per-head projections over all B * S rows, scores and
// P @ V batched over heads x batch, the weight handled head-major (Wd[h][p])
void DeviceTrainingBacking::mha_fwd(int n) {
  const auto& op = cg_.g.node(n).label.op;
  const auto ins = cg_.layer_data_inputs(n);
  const auto ws = cg_.layer_weights(n);
  const MG g = mha_of(n);
  const ValueRef o{n, 0};
  float* y = val(o);
  float *Wd = aux(n, 10), *Q = aux(n, 11), *Kt = aux(n, 12), *V = aux(n, 13), *P = aux(n, 14), *O = aux(n, 15);
  const int64_t rq = g.B * g.Sq, rk = g.B * g.Sk;
  hipLaunchKernelGGL(k_head_major, dim3(grid_of(g.P * g.H)), dim3(256), 0, st_, val(ws[0]), Wd, g.P, g.H, 0);
  for (int64_t h = 0; h < g.H; ++h) {
    const float* Wh = Wd + h * g.P;
    ffk::gemm_f32(val(ins[0]), Wh + g.off_q(), Q + h * rq * g.kd, nullptr, nullptr, rq, g.kd, g.Eq, g.Eq, g.kd,
                  g.kd, false, false, 0, 1.f, 0.f, 1, 1, st_);
    ffk::gemm_f32(val(ins[1]), Wh + g.off_k(), Kt + h * rk * g.kd, nullptr, nullptr, rk, g.kd, g.Ek, g.Ek, g.kd,
                  g.kd, false, false, 0, 1.f, 0.f, 1, 1, st_);
    ffk::gemm_f32(val(ins[2]), Wh + g.off_v(), V + h * rk * g.vd, nullptr, nullptr, rk, g.vd, g.Ev, g.Ev, g.vd,
                  g.vd, false, false, 0, 1.f, 0.f, 1, 1, st_);
  }
  if (ws.size() > 1) {   // input bias [2k + v, H]
    hipLaunchKernelGGL(k_head_bias, dim3(grid_of(g.H * rq * g.kd)), dim3(256), 0, st_, Q, val(ws[1]), g.H, rq, g.kd,
                       int64_t(0));
    hipLaunchKernelGGL(k_head_bias, dim3(grid_of(g.H * rk * g.kd)), dim3(256), 0, st_, Kt, val(ws[1]), g.H, rk, g.kd,
                       g.kd);
    hipLaunchKernelGGL(k_head_bias, dim3(grid_of(g.H * rk * g.vd)), dim3(256), 0, st_, V, val(ws[1]), g.H, rk, g.vd,
                       2 * g.kd);
  }
  const int hb = static_cast<int>(g.H * g.B);
  ffk::gemm_f32(Q, Kt, P, nullptr, nullptr, g.Sq, g.Sk, g.kd, g.kd, g.kd, g.Sk, false, true, 0, 1.f, 0.f, 1, 1, st_,
                hb, g.Sq * g.kd, g.Sk * g.kd, g.Sq * g.Sk);
  hipLaunchKernelGGL(k_attn_softmax, dim3(static_cast<unsigned>(hb * g.Sq)), dim3(256), 0, st_, P, g.Sq, g.Sk,
                     1.f / std::sqrt(static_cast<float>(g.kd)), op.b("causal") ? 1 : 0);
  ffk::gemm_f32(P, V, O, nullptr, nullptr, g.Sq, g.vd, g.Sk, g.Sk, g.vd, g.vd, false, false, 0, 1.f, 0.f, 1, 1, st_,
                hb, g.Sq * g.Sk, g.Sk * g.vd, g.Sq * g.vd);
  for (int64_t h = 0; h < g.H; ++h)   // y = sum_h O_h Wo_h
    ffk::gemm_f32(O + h * rq * g.vd, Wd + h * g.P + g.off_o(), y, nullptr, nullptr, rq, g.E, g.vd, g.vd, g.E, g.E,
                  false, false, 0, 1.f, h == 0 ? 0.f : 1.f, 1, 1, st_);
  if (ws.size() > 2)
    hipLaunchKernelGGL(k_add_rows, dim3(grid_of(rq * g.E)), dim3(256), 0, st_, y, val(ws[2]), rq, g.E);
}

void DeviceTrainingBacking::mha_bwd(int n) {
  const auto ins = cg_.layer_data_inputs(n);
  const auto ws = cg_.layer_weights(n);
  const MG g = mha_of(n);
  const float* G = grad({n, 0});
  float *Wd = aux(n, 10), *Q = aux(n, 11), *Kt = aux(n, 12), *V = aux(n, 13), *P = aux(n, 14), *O = aux(n, 15);
  float *dWd = aux(n, 16), *dO = aux(n, 17), *dQ = aux(n, 18), *dK = aux(n, 19), *dV = aux(n, 20), *dP = aux(n, 21);
  const int64_t rq = g.B * g.Sq, rk = g.B * g.Sk;
  const int hb = static_cast<int>(g.H * g.B);
  if (ws.size() > 2)
    if (float* db = grad(ws[2])) {
      if (g.E % 8 == 0) ffk::colsum_act(kDtF32, G, nullptr, nullptr, db, rq, g.E, 0, 0.f, st_);
      else hipLaunchKernelGGL(k_colsum, dim3(static_cast<unsigned>((g.E + 255) / 256)), dim3(256), 0, st_, G, db,
                              rq, g.E);
    }
  for (int64_t h = 0; h < g.H; ++h) {
    // dWo_h = O_h^T G ; dO_h = G Wo_h^T
    ffk::gemm_f32(O + h * rq * g.vd, G, dWd + h * g.P + g.off_o(), nullptr, nullptr, g.vd, g.E, rq, g.vd, g.E, g.E,
                  true, false, 0, 1.f, 0.f, 1, 1, st_);
    ffk::gemm_f32(G, Wd + h * g.P + g.off_o(), dO + h * rq * g.vd, nullptr, nullptr, rq, g.vd, g.E, g.E, g.E, g.vd,
                  false, true, 0, 1.f, 0.f, 1, 1, st_);
  }
  // dP = dO V^T, dV = P^T dO, dS = softmax'(dP) * scale, dQ = dS K, dK = dS^T Q
  ffk::gemm_f32(dO, V, dP, nullptr, nullptr, g.Sq, g.Sk, g.vd, g.vd, g.vd, g.Sk, false, true, 0, 1.f, 0.f, 1, 1, st_,
                hb, g.Sq * g.vd, g.Sk * g.vd, g.Sq * g.Sk);
  ffk::gemm_f32(P, dO, dV, nullptr, nullptr, g.Sk, g.vd, g.Sq, g.Sk, g.vd, g.vd, true, false, 0, 1.f, 0.f, 1, 1, st_,
                hb, g.Sq * g.Sk, g.Sq * g.vd, g.Sk * g.vd);
  hipLaunchKernelGGL(k_attn_softmax_bwd, dim3(static_cast<unsigned>(hb * g.Sq)), dim3(256), 0, st_, P, dP, g.Sk,
                     1.f / std::sqrt(static_cast<float>(g.kd)));
  ffk::gemm_f32(dP, Kt, dQ, nullptr, nullptr, g.Sq, g.kd, g.Sk, g.Sk, g.kd, g.kd, false, false, 0, 1.f, 0.f, 1, 1,
                st_, hb, g.Sq * g.Sk, g.Sk * g.kd, g.Sq * g.kd);
  ffk::gemm_f32(dP, Q, dK, nullptr, nullptr, g.Sk, g.kd, g.Sq, g.Sk, g.kd, g.kd, true, false, 0, 1.f, 0.f, 1, 1, st_,
                hb, g.Sq * g.Sk, g.Sq * g.kd, g.Sk * g.kd);
  float *dxq = grad(ins[0]), *dxk = grad(ins[1]), *dxv = grad(ins[2]);
  for (int64_t h = 0; h < g.H; ++h) {
    float* dWh = dWd + h * g.P;
    const float* Wh = Wd + h * g.P;
    ffk::gemm_f32(val(ins[0]), dQ + h * rq * g.kd, dWh + g.off_q(), nullptr, nullptr, g.Eq, g.kd, rq, g.Eq, g.kd,
                  g.kd, true, false, 0, 1.f, 0.f, 1, 1, st_);
    ffk::gemm_f32(val(ins[1]), dK + h * rk * g.kd, dWh + g.off_k(), nullptr, nullptr, g.Ek, g.kd, rk, g.Ek, g.kd,
                  g.kd, true, false, 0, 1.f, 0.f, 1, 1, st_);
    ffk::gemm_f32(val(ins[2]), dV + h * rk * g.vd, dWh + g.off_v(), nullptr, nullptr, g.Ev, g.vd, rk, g.Ev, g.vd,
                  g.vd, true, false, 0, 1.f, 0.f, 1, 1, st_);
    if (dxq)
      ffk::gemm_f32(dQ + h * rq * g.kd, Wh + g.off_q(), dxq, nullptr, nullptr, rq, g.Eq, g.kd, g.kd, g.kd, g.Eq,
                    false, true, 0, 1.f, 1.f, 1, 1, st_);
    if (dxk)
      ffk::gemm_f32(dK + h * rk * g.kd, Wh + g.off_k(), dxk, nullptr, nullptr, rk, g.Ek, g.kd, g.kd, g.kd, g.Ek,
                    false, true, 0, 1.f, 1.f, 1, 1, st_);
    if (dxv)
      ffk::gemm_f32(dV + h * rk * g.vd, Wh + g.off_v(), dxv, nullptr, nullptr, rk, g.Ev, g.vd, g.vd, g.vd, g.Ev,
                    false, true, 0, 1.f, 1.f, 1, 1, st_);
  }
  if (ws.size() > 1)
    if (float* dbi = grad(ws[1])) {
      hipLaunchKernelGGL(k_head_bias_grad, dim3(grid_of(g.H * g.kd)), dim3(256), 0, st_, dQ, dbi, g.H, rq, g.kd,
                         int64_t(0));
      hipLaunchKernelGGL(k_head_bias_grad, dim3(grid_of(g.H * g.kd)), dim3(256), 0, st_, dK, dbi, g.H, rk, g.kd,
                         g.kd);
      hipLaunchKernelGGL(k_head_bias_grad, dim3(grid_of(g.H * g.vd)), dim3(256), 0, st_, dV, dbi, g.H, rk, g.vd,
                         2 * g.kd);
    }
  if (float* dW = grad(ws[0]))
    hipLaunchKernelGGL(k_head_major, dim3(grid_of(g.P * g.H)), dim3(256), 0, st_, dWd, dW, g.P, g.H, 1);
}

void DeviceTrainingBacking::bwd(int n) {
  const auto& node = cg_.g.node(n);
  const OpAttrs& op = node.label.op;
  const OpType t = op.type;
  const auto ins = cg_.layer_data_inputs(n);
  const ValueRef o{n, 0};
  if (t == OpType::SPLIT) {   // every output's gradient back into its slice of the input's
    float* dx = grad(ins[0]);
    if (!dx) return;
    const auto& big = host_.slot(ins[0], false)->dims;
    const int nd = static_cast<int>(big.size());
    const int ax = static_cast<int>((op.i("axis") % nd + nd) % nd);
    int64_t outer = 1, inner = 1;
    for (int k = 0; k < ax; ++k) outer *= big[k];
    for (int k = ax + 1; k < nd; ++k) inner *= big[k];
    int64_t off = 0;
    for (size_t j = 0; j < node.outputs.size(); ++j) {
      const ValueRef pv{n, static_cast<int>(j)};
      const int64_t len = host_.slot(pv, false)->dims[ax];
      if (const float* g = grad(pv)) ffk::slice_copy(kDtF32, g, dx, outer, len, inner, big[ax], off, 0, 1, st_);
      off += len;
    }
    FFD_CHECK(hipGetLastError());
    mark(ins[0], 1);
    return;
  }
  float* dy = grad(o);
  if (!dy) return;
  const int64_t ne = numel(o);
  if (t == OpType::LINEAR) {
    const auto ws = cg_.layer_weights(n);
    const auto& wd = host_.slot(ws[0], false)->dims;
    const int64_t in = wd[0], outc = wd[1], rows = numel(ins[0]) / in;
    const int a = dact_of(op.s("activation"));
    const float* g = dy;
    if (a != A_NONE) {
      hipLaunchKernelGGL(k_act_grad, dim3(grid_of(ne)), dim3(256), 0, st_, dy, buf_.at(Key{o, 2}).p, tmp_, ne, a);
      g = tmp_;
    }
    if (float* dw = grad(ws[0]))   // dW += x^T g
      ffk::gemm_f32(val(ins[0]), g, dw, nullptr, nullptr, in, outc, rows, in, outc, outc, true, false, 0, 1.f, 1.f, 1,
                    1, st_);
    if (ws.size() > 1)
      if (float* db = grad(ws[1])) {
        if (outc % 8 == 0) ffk::colsum_act(kDtF32, g, nullptr, nullptr, db, rows, outc, 0, 0.f, st_);
        else hipLaunchKernelGGL(k_colsum, dim3(static_cast<unsigned>((outc + 255) / 256)), dim3(256), 0, st_, g, db,
                                rows, outc);
      }
    if (float* dx = grad(ins[0]))   // dX += g W^T
      ffk::gemm_f32(g, val(ws[0]), dx, nullptr, nullptr, rows, in, outc, outc, outc, in, false, true, 0, 1.f, 1.f, 1,
                    1, st_);
  } else if (t == OpType::CONV2D) {
    const CG g = conv_geom_of(*host_.slot(ins[0], false), *host_.slot(o, false), op, false);
    const int a = dact_of(op.s("activation"));
    const float* gy = dy;
    if (a != A_NONE) {
      hipLaunchKernelGGL(k_act_grad, dim3(grid_of(ne)), dim3(256), 0, st_, dy, buf_.at(Key{o, 2}).p, tmp_, ne, a);
      gy = tmp_;
    }
    const auto ws = cg_.layer_weights(n);
    if (float* dw = grad(ws[0]))
      hipLaunchKernelGGL(k_conv_wgrad, dim3(static_cast<unsigned>(numel(ws[0]))), dim3(256), 0, st_, gy,
                         val(ins[0]), dw, g);
    if (ws.size() > 1)
      if (float* db = grad(ws[1]))
        hipLaunchKernelGGL(k_chan_sum, dim3(static_cast<unsigned>(g.O)), dim3(256), 0, st_, gy, db, g.N, g.O,
                           static_cast<int64_t>(g.OH) * g.OW);
    if (float* dx = grad(ins[0]))
      hipLaunchKernelGGL(k_conv_dgrad, dim3(grid_of(numel(ins[0]))), dim3(256), 0, st_, gy, val(ws[0]), dx, g);
  } else if (t == OpType::POOL2D) {
    const CG g = conv_geom_of(*host_.slot(ins[0], false), *host_.slot(o, false), op, true);
    const int a = dact_of(op.s("activation"));
    if (float* dx = grad(ins[0]))
      hipLaunchKernelGGL(k_pool_bwd, dim3(grid_of(ne)), dim3(256), 0, st_, dy,
                         a != A_NONE ? buf_.at(Key{o, 2}).p : nullptr, buf_.at(Key{o, 3}).p, dx, g,
                         op.s("pool_type") == "max" ? 1 : 0, a);
  } else if (t == OpType::BATCHNORM) {
    const auto& xd = host_.slot(ins[0], false)->dims;
    int64_t S = 1;
    for (size_t k = 2; k < xd.size(); ++k) S *= xd[k];
    const auto ws = cg_.layer_weights(n);
    hipLaunchKernelGGL(k_bn_bwd, dim3(static_cast<unsigned>(xd[1])), dim3(256), 0, st_, dy, val(ins[0]), val(o),
                       ws.size() > 0 ? val(ws[0]) : nullptr, buf_.at(Key{o, 3}).p, grad(ins[0]),
                       ws.size() > 0 ? grad(ws[0]) : nullptr, ws.size() > 1 ? grad(ws[1]) : nullptr,
                       static_cast<int>(xd[0]), static_cast<int>(xd[1]), S, op.b("relu") ? 1 : 0);
  } else if (dact_of(t) >= 0) {
    if (float* dx = grad(ins[0]))
      hipLaunchKernelGGL(k_act_bwd, dim3(grid_of(ne)), dim3(256), 0, st_, dy, val(ins[0]), dx, ne, dact_of(t));
  } else if (binary_of(t) >= 0) {
    hipLaunchKernelGGL(k_binary_bwd, dim3(grid_of(ne)), dim3(256), 0, st_, dy, val(ins[0]), val(ins[1]),
                       grad(ins[0]), grad(ins[1]), ne, binary_of(t));
  } else if (scalar_of(t) >= 0) {
    const int s = scalar_of(t);
    const float k = static_cast<float>(op.f("scalar"));
    if (float* dx = grad(ins[0]))
      hipLaunchKernelGGL(k_axpy, dim3(grid_of(ne)), dim3(256), 0, st_, dy, dx, ne,
                         s == 0 ? k : s == 3 ? 1.f / k : 1.f);
  } else if (is_view(t)) {
    if (float* dx = grad(ins[0])) hipLaunchKernelGGL(k_axpy, dim3(grid_of(ne)), dim3(256), 0, st_, dy, dx, ne, 1.f);
  } else if (t == OpType::SOFTMAX) {
    const auto& d = host_.slot(o, false)->dims;
    const int64_t cols = d.empty() ? 1 : d.back();
    if (float* dx = grad(ins[0])) {   // softmax.hip writes dx: through tmp, then accumulated
      ffk::softmax_bwd(kDtF32, dy, val(o), tmp_, static_cast<int>(ne / cols), static_cast<int>(cols), st_);
      hipLaunchKernelGGL(k_axpy, dim3(grid_of(ne)), dim3(256), 0, st_, tmp_, dx, ne, 1.f);
    }
  } else if (t == OpType::EMBEDDING) {
    const auto ws = cg_.layer_weights(n);
    if (float* dw = grad(ws[0])) {
      const auto& wd = host_.slot(ws[0], false)->dims;
      const int64_t E = wd[0], D = wd[1], nidx = numel(ins[0]);
      const std::string aggr = op.s("aggr");
      const int L = aggr == "none" ? 1 : static_cast<int>(host_.slot(ins[0], false)->dims.back());
      const int* idx = reinterpret_cast<const int*>(aux(n, 3));
      if (D % 8 == 0)
        ffk::embedding_bwd(kDtF32, 32, idx, dy, dw, nidx / L, L, static_cast<int>(D),
                           aggr == "none" ? 0 : aggr == "sum" ? 1 : 2, E, nullptr, 1, st_);
      else
        hipLaunchKernelGGL(k_embed_bwd, dim3(grid_of(nidx * D)), dim3(256), 0, st_, idx, dy, dw, nidx / L, L, D,
                           aggr == "avg" ? 1.f / static_cast<float>(L) : 1.f);
    }
  } else if (t == OpType::LAYERNORM) {
    const auto ws = cg_.layer_weights(n);
    const int64_t N = ln_cols(n), R = ne / N;
    const float* gm = ws.size() > 0 ? val(ws[0]) : nullptr;
    float* dg = ws.size() > 0 ? grad(ws[0]) : nullptr;
    float* dbt = ws.size() > 1 ? grad(ws[1]) : nullptr;
    const float* st = aux(n, 3);
    float* dx = grad(ins[0]);
    if (N % 8 == 0) {   // layernorm.hip writes dx: through tmp, then accumulated
      ffk::layernorm_bwd(kDtF32, dy, val(ins[0]), st, st + R, gm, tmp_, dg, dbt, aux(n, 4), static_cast<int>(R),
                         static_cast<int>(N), st_);
      if (dx) hipLaunchKernelGGL(k_axpy, dim3(grid_of(ne)), dim3(256), 0, st_, tmp_, dx, ne, 1.f);
    } else {
      hipLaunchKernelGGL(k_ln_bwd, dim3(static_cast<unsigned>(R)), dim3(256), 0, st_, dy, val(ins[0]), gm, st, st + R,
                         dx, dg, dbt, N);
    }
  } else if (t == OpType::BATCHMATMUL) {
    const auto& a = host_.slot(ins[0], false)->dims;
    const int nd = static_cast<int>(a.size());
    const int64_t M = a[nd - 2], K = a[nd - 1], N = host_.slot(ins[1], false)->dims.back();
    const int Bt = static_cast<int>(numel(ins[0]) / (M * K));
    if (float* da = grad(ins[0]))   // dA += G B^T
      ffk::gemm_f32(dy, val(ins[1]), da, nullptr, nullptr, M, K, N, N, N, K, false, true, 0, 1.f, 1.f, 1, 1, st_, Bt,
                    M * N, K * N, M * K);
    if (float* db = grad(ins[1]))   // dB += A^T G
      ffk::gemm_f32(val(ins[0]), dy, db, nullptr, nullptr, K, N, M, K, N, N, true, false, 0, 1.f, 1.f, 1, 1, st_, Bt,
                    M * K, M * N, K * N);
  } else if (t == OpType::CONCAT) {
    const auto& big = host_.slot(o, false)->dims;
    const int nd = static_cast<int>(big.size());
    const int ax = static_cast<int>((op.i("axis") % nd + nd) % nd);
    int64_t outer = 1, inner = 1;
    for (int k = 0; k < ax; ++k) outer *= big[k];
    for (int k = ax + 1; k < nd; ++k) inner *= big[k];
    int64_t off = 0;
    for (auto const& v : ins) {
      const int64_t len = host_.slot(v, false)->dims[ax];
      if (float* dx = grad(v)) ffk::slice_copy(kDtF32, dy, dx, outer, len, inner, big[ax], off, 1, 1, st_);
      off += len;
    }
  } else if (t == OpType::DROPOUT) {
    if (float* dx = grad(ins[0]))
      hipLaunchKernelGGL(k_dropout, dim3(grid_of(ne)), dim3(256), 0, st_, dy, dx, ne,
                         static_cast<float>(op.f("rate")), op_seed(n), 1);
  } else if (t == OpType::MULTIHEAD_ATTENTION) {
    mha_bwd(n);
  }
  FFD_CHECK(hipGetLastError());
  for (auto const& v : ins)
    if (grad(v)) mark(v, 1);
  for (auto const& v : cg_.layer_weights(n))
    if (grad(v)) mark(v, 1);
}

void DeviceTrainingBacking::backward(const std::vector<float>& labels) {
  push();
  for (auto const& kv : buf_)
    if (kv.first.kind == 1) FFD_CHECK(hipMemsetAsync(kv.second.p, 0, kv.second.n * sizeof(float), st_));
  const ValueRef out = host_.output();
  const std::string& loss = host_.loss();
  const float* p = val(out);
  samples_ += rows_;
  if (loss == "sparse_categorical_crossentropy") {
    if (static_cast<int64_t>(labels.size()) != rows_) throw FFError("device backing: label size mismatch");
    std::vector<int> li(labels.size());
    for (size_t i = 0; i < labels.size(); ++i) li[i] = static_cast<int>(labels[i]);
    FFD_CHECK(hipMemcpyAsync(labels_, li.data(), li.size() * sizeof(int), hipMemcpyHostToDevice, st_));
    // gradient w.r.t. the logits (the fused softmax's input)
    const ValueRef tgt = cg_.layer_data_inputs(out.node)[0];
    float* g = grad(tgt);
    hipLaunchKernelGGL(k_sparse_ce, dim3(static_cast<unsigned>((rows_ + 255) / 256)), dim3(256), 0, st_, p, labels_,
                       g ? g : tmp2_, metrics_d_, rows_, cols_, 1.f / static_cast<float>(rows_));
    FFD_CHECK(hipStreamSynchronize(st_));   // `li` leaves scope
    if (g) mark(tgt, 1);
  } else if (loss == "mean_squared_error" || loss == "mean_squared_error_avg_reduce") {
    if (static_cast<int64_t>(labels.size()) != numel(out)) throw FFError("device backing: label size mismatch");
    FFD_CHECK(hipMemcpyAsync(tmp2_, labels.data(), labels.size() * sizeof(float), hipMemcpyHostToDevice, st_));
    float* g = grad(out);
    // metrics block {loss, -, count, sq err, abs err}: slot 2 is not used here
    ffk::mse_loss_full(kDtF32, kDtF32, p, tmp2_, g ? tmp_ : nullptr, metrics_d_, numel(out),
                       2.f / static_cast<float>(rows_ * cols_), 1, cols_, 0, st_);
    if (g) {
      hipLaunchKernelGGL(k_axpy, dim3(grid_of(numel(out))), dim3(256), 0, st_, tmp_, g, numel(out), 1.f);
      mark(out, 1);
    }
    FFD_CHECK(hipStreamSynchronize(st_));   // `labels` may be freed by the caller
  } else {
    throw FFError("device backing: loss " + loss);
  }
  FFD_CHECK(hipGetLastError());
  const auto& ord = host_.order();
  for (auto it = ord.rbegin(); it != ord.rend(); ++it) {
    if (host_.fused_softmax_ce() && *it == out.node) continue;
    if (!host_.needs_grad({*it, 0})) continue;
    bwd(*it);
  }
}

void DeviceTrainingBacking::update() {
  push();
  ++step_;
  const LocalOptimizer& o = host_.optimizer();
  for (auto const& kv : buf_) {
    if (kv.first.kind != 1 || cg_.g.node(kv.first.v.node).label.op.type != OpType::WEIGHT) continue;
    const ValueRef v = kv.first.v;
    const int* l = &v.node;
    float* g = kv.second.p;
    float* w = val(v);
    const int64_t n = numel(v);
    auto state = [&](int which) {
      auto key = std::make_pair(*l, which);
      auto it = opt_state_.find(key);
      if (it != opt_state_.end()) return it->second;
      float* p = nullptr;
      FFD_CHECK(hipMalloc(&p, std::max<int64_t>(n, 1) * sizeof(float)));
      FFD_CHECK(hipMemsetAsync(p, 0, std::max<int64_t>(n, 1) * sizeof(float), st_));
      return opt_state_[key] = p;
    };
    if (o.kind == "adam") {
      const float bc1 = 1.f - static_cast<float>(std::pow(o.beta1, static_cast<double>(step_)));
      const float bc2 = 1.f - static_cast<float>(std::pow(o.beta2, static_cast<double>(step_)));
      hipLaunchKernelGGL(k_adam, dim3(grid_of(n)), dim3(256), 0, st_, w, g, state(0), state(1), n,
                         static_cast<float>(o.lr), static_cast<float>(o.beta1), static_cast<float>(o.beta2),
                         static_cast<float>(o.epsilon), static_cast<float>(o.weight_decay), bc1, bc2);
    } else {
      hipLaunchKernelGGL(k_sgd, dim3(grid_of(n)), dim3(256), 0, st_, w, g, o.momentum != 0.0 ? state(0) : nullptr, n,
                         static_cast<float>(o.lr), static_cast<float>(o.momentum),
                         static_cast<float>(o.weight_decay), o.nesterov ? 1 : 0);
    }
    FFD_CHECK(hipGetLastError());
    mark(v, 0);
  }
}

}  // namespace

std::unique_ptr<TrainingBacking> make_device_backing(const ComputationGraph& cg, LocalOptimizer opt,
                                                     const std::string& loss, uint64_t seed, std::string* why) {
  auto no = [&](const std::string& m) -> std::unique_ptr<TrainingBacking> {
    if (why) *why = m;
    return nullptr;
  };
  const char* want = std::getenv("FF_C_API_DEVICE");
  if (want && std::strcmp(want, "cpu") == 0) return no("FF_C_API_DEVICE=cpu");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
    (void)hipGetLastError();
    return no("no GPU visible");
  }
  for (int n : cg.layers_in_topo_order()) {
    const OpType t = cg.g.node(n).label.op.type;
    if (t == OpType::INPUT || t == OpType::WEIGHT) continue;
    const std::string u = unsupported(cg, n);
    if (!u.empty()) return no("no device implementation: " + u);
  }
  if (loss != "sparse_categorical_crossentropy" && loss != "mean_squared_error" &&
      loss != "mean_squared_error_avg_reduce")
    return no("loss " + loss + " runs on the CPU backing");
  // the fused softmax + CE needs the graph to end in SOFTMAX
  if (loss == "sparse_categorical_crossentropy") {
    int last = -1;
    for (int n : cg.layers_in_topo_order()) {
      const OpType t = cg.g.node(n).label.op.type;
      if (t != OpType::INPUT && t != OpType::WEIGHT) last = n;
    }
    if (last < 0 || cg.g.node(last).label.op.type != OpType::SOFTMAX)
      return no("cross-entropy without a final softmax");
  }
  int dev = 0;
  if (const char* d = std::getenv("FF_C_API_GPU")) dev = std::atoi(d);
  if (dev < 0 || dev >= count) dev = 0;
  return std::unique_ptr<TrainingBacking>(new DeviceTrainingBacking(cg, std::move(opt), loss, seed, dev));
}

}  // namespace ff
