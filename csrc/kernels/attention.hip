// Flash attention (forward + backward) for gfx950, bf16 in / fp32 accumulate.
//
// Parity: lib/kernels/src/cuda/ops/attention_kernels.cu, which calls cuDNN's
// monolithic cudnnMultiHeadAttnForward/BackwardData/BackwardWeights (:255,
// :292, :316) and materialises the whole attention matrix.  Here the score
// matrix never leaves the CU (blockwise online softmax), which is what makes
// the long-sequence configs of SURVEY.md §5.7 possible.
//
// CDNA4 design (see /opt/skills/guides/cdna_hip_programming.md §3, §5.5):
//  * MFMA v_mfma_f32_32x32x16_bf16; a workgroup = 4 waves, each wave owns 32
//    query rows (forward, dQ) or 32 key rows (dK/dV).
//  * "swapped" products: the forward computes S^T = K Q^T so every lane holds
//    scores of ONE query -> the row max / row sum are lane-local plus a single
//    exchange with lane^32; O^T = V^T P^T consumes the S^T accumulator
//    directly as the MFMA B operand (accumulator-as-operand, no LDS round
//    trip for P) and keeps the query on the lane, so the online-softmax
//    rescale is a per-lane scalar multiply.
//  * K/V tiles are staged global->registers->LDS with the next tile's loads
//    issued before the current tile's MFMAs (async-STAGE split, T14), double
//    buffered, one barrier per tile.
//  * LDS images are XOR-swizzled per row so ds_read_b128 row reads are
//    conflict-free; V^T (and K^T / Q^T / dO^T in the backward) operands come
//    from ds_read_b64_tr_b16 hardware-transposed reads of the same images.
//  * backward = dQ kernel (query block resident; also computes delta =
//    rowsum(dO*O) for its queries) then dK/dV kernel (key block resident,
//    loops over query tiles, key on the lane) -> no float atomics,
//    deterministic, no [N, N] buffers.
//
// Tensor addressing: every tensor is [B, S, H, D] with arbitrary strides for
// b / s / h and contiguous d, so the fused QKV projection output
// [B, S, 3, H, D] is consumed in place.  LSE is [B, H, S] fp32, log2 domain.
#include <cstdlib>

#include "kernels.h"
#include "mfma.h"

namespace ffk {

struct TensorView {
  const bf16* p;
  int64_t sb, ss, sh;  // element strides; d is contiguous
};

struct AttnParams {
  TensorView q, k, v, o, dout;
  bf16 *o_out, *dq, *dk, *dv;
  int64_t o_sb, o_ss, o_sh;                   // output strides (o_out)
  int64_t dq_sb, dq_ss, dq_sh, dk_sb, dk_ss, dk_sh, dv_sb, dv_ss, dv_sh;
  float* lse;    // [B, H, Sq] log2-domain
  float* delta;  // [B, H, Sq]
  float *dbq, *dbk, *dbv;  // optional [H*D] projection-bias gradients (column sums of dq / dk / dv)
  int64_t db_ld;           // > 0: dbq / dbk / dbv are per-32-row partial slabs with this row stride
  int B, H, Sq, Sk;
  float scale;       // softmax scale (1/sqrt(D) by default)
  float scale_log2;  // scale * log2(e)
  float inv_scale_log2;  // 1 / scale_log2 (no IEEE divide in the loops)
  int prio;          // raise wave priority around MFMA clusters (FFK_ATTN_PRIO; guide T5)
  int xcd;           // XCD-local head order of non-causal grids (FFK_ATTN_XCD, default on)
  int wide_store;    // 16-B output rows via permlane32_swap (FFK_ATTN_WIDE_STORE, default on)
};

// Store a wave's 32-row C^T tile (lane & 31 -> row, registers -> d) as rows
// of bf16, 16 bytes per store.  A lane holds 4 consecutive d of each 8-group
// (lane half h: d = 8 g + 4 h + e); v_permlane32_swap trades group 2p+1 of
// the lower half for group 2p of the upper half, so after the swap every
// lane holds 8 consecutive d (lower half: d 16p..16p+7 = its own group 2p
// and its partner's; upper half: 16p+8..16p+15) -- half the store
// instructions of the 8-byte form (the epilogue tail is store-issue bound,
// guide T21).  Every lane runs the swaps; `ok` guards only the stores.
template <int DT>
__device__ __forceinline__ void store_rows16(bf16* row, const f32x16 (&acc)[DT], float mul, int h, bool ok) {
  auto pk = [](float a, float b) -> unsigned {
    return static_cast<unsigned>(f2u(a)) | (static_cast<unsigned>(f2u(b)) << 16);
  };
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {
      const int ga = 2 * gp, gb = 2 * gp + 1;
      const unsigned xa0 = pk(acc[dt][4 * ga + 0] * mul, acc[dt][4 * ga + 1] * mul);
      const unsigned xa1 = pk(acc[dt][4 * ga + 2] * mul, acc[dt][4 * ga + 3] * mul);
      const unsigned yb0 = pk(acc[dt][4 * gb + 0] * mul, acc[dt][4 * gb + 1] * mul);
      const unsigned yb1 = pk(acc[dt][4 * gb + 2] * mul, acc[dt][4 * gb + 3] * mul);
      const auto s0 = __builtin_amdgcn_permlane32_swap(xa0, yb0, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(xa1, yb1, false, false);
      if (ok) {
        u32x4t v = {static_cast<unsigned>(s0[0]), static_cast<unsigned>(s1[0]), static_cast<unsigned>(s0[1]),
                    static_cast<unsigned>(s1[1])};
        *reinterpret_cast<u32x4t*>(row + dt * 32 + 16 * gp + 8 * h) = v;
      }
    }
}

// (head, block) of a non-causal workgroup, grid (blocks, B*H).  Dispatch puts
// linear id L = x + y * gridDim.x on XCD L % 8, so without a remap the
// blocks of one head (4 query blocks at S = 512) run on four XCDs and every
// XCD's L2 fetches that head's K / V.  The bijective remap (mfma.h) gives
// each XCD a contiguous range of linear ids, i.e. whole heads: a head's K / V
// come from HBM once and its other blocks hit in the XCD's L2.
__device__ __forceinline__ void attn_head_block(const AttnParams& P, int& bh, int& blk) {
  if (!P.xcd) {
    bh = blockIdx.y;
    blk = blockIdx.x;
    return;
  }
  const int W = gridDim.x * gridDim.y;
  const int r = xcd_remap(blockIdx.x + blockIdx.y * gridDim.x, W);
  bh = r / gridDim.x;
  blk = r % gridDim.x;
}

__device__ __forceinline__ void prio_hi(const AttnParams& P) {
  if (P.prio) __builtin_amdgcn_s_setprio(1);
}
__device__ __forceinline__ void prio_lo(const AttnParams& P) {
  if (P.prio) __builtin_amdgcn_s_setprio(0);
}

template <int D>
__device__ __forceinline__ int lds_off(int r, int c) {  // byte offset of chunk c of row r
  return img_off<D * 2>(r, c);
}
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const unsigned char* img, int row0, int dt, int lane) {
  return tr_frag_acc<D * 2>(img, row0, dt * 32, lane);
}

// Bias gradient of a projection: add the column sums of a wave's 32-row
// output tile (C^T accumulator: lane&31 -> row, registers -> d) times `mul`
// into db[d] — shuffles over the 32 rows of each lane half, then one fp32
// atomic per column (32 per lane half).  Rows outside the sequence must hold
// zeros (they do: masked rows contribute nothing to the accumulators).
template <int DT>
__device__ __forceinline__ void bias_colsum(const f32x16 (&acc)[DT], float mul, float* db, int lane) {
  const int h = lane >> 5;
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float v = acc[dt][r];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if ((lane & 31) == 0) atomicAdd(db + dt * 32 + 8 * (r >> 2) + 4 * h + (r & 3), v * mul);
    }
}

// Global [rows][D] tile -> registers (each thread `per` chunks of 16 B).
template <int D, int ROWS>
struct TileLoader {
  static constexpr int CHUNKS = ROWS * D / 8;
  static constexpr int PER = CHUNKS / 256;
  bf16x8 reg[PER];
  __device__ __forceinline__ void load(const TensorView& t, int b, int h, int row0, int nrows) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int r = c / (D / 8), ch = c % (D / 8);
      if (row0 + r < nrows) {
        reg[i] = *reinterpret_cast<const bf16x8*>(t.p + b * t.sb + static_cast<int64_t>(row0 + r) * t.ss +
                                                  h * t.sh + ch * 8);
      } else {
        reg[i] = bf16x8{};
      }
    }
  }
  __device__ __forceinline__ void store(unsigned char* img) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + 256 * i;
      const int r = c / (D / 8), ch = c % (D / 8);
      *reinterpret_cast<bf16x8*>(img + lds_off<D>(r, ch)) = reg[i];
    }
  }
};

// Bias-gradient partials of a wave's 32-row output tile, without atomics: the
// column sums over the 32 rows of each lane half as a reduce-scatter (each xor
// step halves the live values: 31 shuffles for D = 64 instead of 160), then
// one plain store per value into this wave's row of a partial slab (every
// (row block, column) is written by exactly one wave; the host sums the
// slab's rows).  Lane keeps k = (lane & 31) * NV / 32 + t, k = 16 dt + r.
// m ? a : b for m = all ones / zero, one v_bfi_b32
__device__ __forceinline__ float bfi_sel(unsigned m, float a, float b) {
  float r;
  asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(r) : "v"(m), "v"(a), "v"(b));
  return r;
}
template <int DT>
__device__ __forceinline__ void bias_partial(const f32x16 (&acc)[DT], float mul, float* row, int lane) {
  constexpr int NV = 16 * DT;
  float v[NV];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) v[dt * 16 + r] = acc[dt][r];
#pragma unroll
  for (int st = 0; st < 5; ++st) {
    const int o = 16 >> st, c = NV >> st;
    const unsigned m = (lane & o) ? ~0u : 0u;
#pragma unroll
    for (int i = 0; i < c / 2; ++i) {
      // bitwise selects in asm: as C selects hipcc turned the whole pass
      // into dynamically indexed array reads (cmp / cndmask chains over all
      // 32 values, 13k instructions, the kernels ran 2x slower)
      const float send = bfi_sel(m, v[i], v[i + c / 2]);
      const float keep = bfi_sel(m, v[i + c / 2], v[i]);
      v[i] = keep + __shfl_xor(send, o, 64);
    }
  }
  const int h = lane >> 5;
#pragma unroll
  for (int t = 0; t < NV / 32; ++t) {
    const int k = (lane & 31) * (NV / 32) + t, dt = k >> 4, r = k & 15;
    row[dt * 32 + 8 * (r >> 2) + 4 * h + (r & 3)] = v[t] * mul;
  }
}

// ===========================================================================
// Forward
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(AttnParams P) {
  constexpr int KS = D / 16;        // k-steps over the head dim
  constexpr int DT = D / 32;        // 32-wide output tiles over the head dim
  constexpr int KV = 64;            // keys per tile
  constexpr int TILE_BYTES = KV * D * 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[4 * TILE_BYTES];  // K0 V0 K1 V1

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  // causal: grid (B*H, q blocks) with the LAST (heaviest) query block of every
  // head dispatched first — longest-first order, so the kernel's tail is the
  // light blocks near the sequence start
  int bh = blockIdx.x, qb = gridDim.y - 1 - blockIdx.y;
  if (!CAUSAL) attn_head_block(P, bh, qb);
  const int b = bh / P.H, hh = bh % P.H;
  const int q_blk = qb * 128;
  const int qw = q_blk + wave * 32;
  const int q = qw + (lane & 31);
  const bool q_ok = q < P.Sq;

  // Q as the B operand of S^T = K Q^T: lane holds Q[q][16ks + 8h .. +8]
  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    qf[ks] = q_ok ? *reinterpret_cast<const bf16x8*>(P.q.p + b * P.q.sb + static_cast<int64_t>(q) * P.q.ss +
                                                     hh * P.q.sh + ks * 16 + 8 * h)
                  : bf16x8{};

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x16{};
  float m = -INFINITY, l = 0.f;

  int n_tiles = (P.Sk + KV - 1) / KV;
  if (CAUSAL) n_tiles = min(n_tiles, (q_blk + 128 + KV - 1) / KV);

  TileLoader<D, KV> kl, vl;
  kl.load(P.k, b, hh, 0, P.Sk);
  vl.load(P.v, b, hh, 0, P.Sk);
  kl.store(smem);
  vl.store(smem + TILE_BYTES);
  __syncthreads();

  for (int t = 0; t < n_tiles; ++t) {
    const int k0 = t * KV;
    const unsigned char* Kt = smem + (t & 1) * 2 * TILE_BYTES;
    const unsigned char* Vt = Kt + TILE_BYTES;
    const bool has_next = t + 1 < n_tiles;
    if (has_next) {  // issue next tile's HBM loads before this tile's MFMAs
      kl.load(P.k, b, hh, k0 + KV, P.Sk);
      vl.load(P.v, b, hh, k0 + KV, P.Sk);
    }
    const bool wave_active = !CAUSAL || (k0 <= qw + 31);
    if (wave_active) {
      // ---- S^T[key][q] for two 32-key tiles
      f32x16 s[2];
      prio_hi(P);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        s[kt] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          bf16x8 kf = lds_read16(Kt, lds_off<D>(kt * 32 + (lane & 31), 2 * ks + h));
          s[kt] = mfma32(kf, qf[ks], s[kt]);
        }
      }
      prio_lo(P);
      // ---- mask (only tiles that cross the sequence end or the causal
      // diagonal — a wave-uniform branch), tile max of the RAW scores: the
      // softmax scale is folded into one FMA per score inside exp2 below
      const bool need_mask = (k0 + KV > P.Sk) || (CAUSAL && k0 + KV - 1 > qw);
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (key >= P.Sk || (CAUSAL && key > q)) s[kt][r] = -INFINITY;
          }
      }
      // two independent v_max3 chains over the 32 scores (16 issues)
      float t0 = fmax3(s[0][0], s[0][1], s[0][2]);
      float t1 = fmax3(s[1][0], s[1][1], s[1][2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) {
        t0 = fmax3(t0, s[0][r], s[0][r + 1]);
        t1 = fmax3(t1, s[1][r], s[1][r + 1]);
      }
      float tmax = fmax3(fmax3(t0, s[0][15], s[1][15]), t1, t1);
      const float tother = __shfl_xor(tmax, 32, 64);
      tmax = fmax3(tmax, tother, tother);
      // ---- lazy rescale: the running max m only moves when some lane's
      // tile max exceeds it by more than 8 in the log2 domain (p <= 256 is
      // exact enough in fp32 and bf16-relative); a wave-uniform branch, so
      // the o *= alpha pass runs on a few early tiles instead of every tile
      if (__any(tmax > m + 8.f * P.inv_scale_log2)) {
        const float m_new = fmaxf(m, tmax);
        const float alpha = (m_new == -INFINITY) ? 1.f : fexp2((m - m_new) * P.scale_log2);
        m = m_new;
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      }
      const float mc = (m == -INFINITY) ? 0.f : m * P.scale_log2;
      float psum[2] = {0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = fexp2(fmaf(s[kt][r], P.scale_log2, -mc));
          s[kt][r] = pv;
          psum[kt] += pv;
        }
      l += psum[0] + psum[1];
      // ---- O^T[d][q] += V^T[d][key] P^T[key][q]
      prio_hi(P);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          bf16x8 pf = acc_to_frag(s[kt], st);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            bf16x8 vf = tr_frag<D>(Vt, kt * 32 + 16 * st, dt, lane);
            o[dt] = mfma32(vf, pf, o[dt]);
          }
        }
      prio_lo(P);
    }
    if (has_next) {
      unsigned char* nxt = smem + ((t + 1) & 1) * 2 * TILE_BYTES;
      kl.store(nxt);
      vl.store(nxt + TILE_BYTES);
    }
    __syncthreads();
  }

  // ---- epilogue: O = O^T / l, LSE
  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  bf16* orow = P.o_out + b * P.o_sb + static_cast<int64_t>(q) * P.o_ss + hh * P.o_sh;
  if (P.wide_store) {
    store_rows16<DT>(orow, o, inv, h, q_ok);
  } else if (q_ok) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][4 * g4 + e] * inv);
        *reinterpret_cast<bf16x4*>(orow + dt * 32 + 8 * g4 + 4 * h) = v;
      }
  }
  if (q_ok && h == 0)
    P.lse[static_cast<int64_t>(bh) * P.Sq + q] = (lt > 0.f) ? m * P.scale_log2 + log2f(lt) : -INFINITY;
}

// ===========================================================================
// Forward, software-pipelined across K/V tiles (FFK_ATTN_FWD_PIPE=1): the
// scores of tile t+1 (S MFMAs) are computed while tile t's softmax runs on
// the VALU, and tile t's P.V MFMAs follow, so inside ONE wave the matrix cores
// and the VALU work on different tiles instead of waiting for each other
// (guide "sm-split"; with one barrier per tile the two waves of a SIMD run in
// phase, so the overlap has to come from within the wave).  K leads V by one
// tile in the LDS ring: during iteration t a buffer holds {K(t+1), V(t)}.
template <int D, bool CAUSAL>
__global__ __launch_bounds__(256, 2) void attn_fwd_pipe_kernel(AttnParams P) {
  constexpr int KS = D / 16, DT = D / 32, KV = 64;
  constexpr int TILE_BYTES = KV * D * 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[4 * TILE_BYTES];  // [K V] x 2

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  int bh = blockIdx.x, qb = gridDim.y - 1 - blockIdx.y;
  if (!CAUSAL) attn_head_block(P, bh, qb);
  const int b = bh / P.H, hh = bh % P.H;
  const int q_blk = qb * 128;
  const int qw = q_blk + wave * 32;
  const int q = qw + (lane & 31);
  const bool q_ok = q < P.Sq;

  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
    qf[ks] = q_ok ? *reinterpret_cast<const bf16x8*>(P.q.p + b * P.q.sb + static_cast<int64_t>(q) * P.q.ss +
                                                     hh * P.q.sh + ks * 16 + 8 * h)
                  : bf16x8{};

  f32x16 o[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt] = f32x16{};
  float m = -INFINITY, l = 0.f;

  int n_tiles = (P.Sk + KV - 1) / KV;
  if (CAUSAL) n_tiles = min(n_tiles, (q_blk + 128 + KV - 1) / KV);
  auto active = [&](int t) { return t < n_tiles && (!CAUSAL || t * KV <= qw + 31); };

  auto scores = [&](const unsigned char* Kt, f32x16 (&s)[2]) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
      s[kt] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
        s[kt] = mfma32(lds_read16(Kt, lds_off<D>(kt * 32 + (lane & 31), 2 * ks + h)), qf[ks], s[kt]);
    }
  };

  TileLoader<D, KV> kl, vl;
  // prologue: K(0) -> buffer 1's K slot (free until iteration 0 ends), K(1) and
  // V(0) -> buffer 0
  kl.load(P.k, b, hh, 0, P.Sk);
  kl.store(smem + 2 * TILE_BYTES);
  if (n_tiles > 1) kl.load(P.k, b, hh, KV, P.Sk);
  vl.load(P.v, b, hh, 0, P.Sk);
  if (n_tiles > 1) kl.store(smem);
  vl.store(smem + TILE_BYTES);
  __syncthreads();
  f32x16 sa[2], sb[2];
  if (active(0)) scores(smem + 2 * TILE_BYTES, sa);
  __syncthreads();   // every wave read K(0) before iteration 0 restages buffer 1

  // one tile: softmax(t) on `sc` (+ S(t+1) into `sn` from the current buffer),
  // then O += V(t)^T P(t)
  auto step = [&](int t, f32x16 (&sc)[2], f32x16 (&sn)[2]) {
    const int k0 = t * KV;
    const unsigned char* buf = smem + (t & 1) * 2 * TILE_BYTES;
    const unsigned char* Kn = buf;                 // K(t+1)
    const unsigned char* Vt = buf + TILE_BYTES;    // V(t)
    const bool more_k = t + 2 < n_tiles, more_v = t + 1 < n_tiles;
    if (more_k) kl.load(P.k, b, hh, k0 + 2 * KV, P.Sk);
    if (more_v) vl.load(P.v, b, hh, k0 + KV, P.Sk);
    const bool act = active(t);
    // S(t+1): independent of this tile's softmax — the scheduler interleaves
    // its MFMAs with the VALU work below
    if (active(t + 1)) scores(Kn, sn);
    if (act) {
      const bool need_mask = (k0 + KV > P.Sk) || (CAUSAL && k0 + KV - 1 > qw);
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (key >= P.Sk || (CAUSAL && key > q)) sc[kt][r] = -INFINITY;
          }
      }
      float t0 = fmax3(sc[0][0], sc[0][1], sc[0][2]);
      float t1 = fmax3(sc[1][0], sc[1][1], sc[1][2]);
#pragma unroll
      for (int r = 3; r < 15; r += 2) {
        t0 = fmax3(t0, sc[0][r], sc[0][r + 1]);
        t1 = fmax3(t1, sc[1][r], sc[1][r + 1]);
      }
      float tmax = fmax3(fmax3(t0, sc[0][15], sc[1][15]), t1, t1);
      const float tother = __shfl_xor(tmax, 32, 64);
      tmax = fmax3(tmax, tother, tother);
      if (__any(tmax > m + 8.f * P.inv_scale_log2)) {
        const float m_new = fmaxf(m, tmax);
        const float alpha = (m_new == -INFINITY) ? 1.f : fexp2((m - m_new) * P.scale_log2);
        m = m_new;
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      }
      const float mc = (m == -INFINITY) ? 0.f : m * P.scale_log2;
      float psum[2] = {0.f, 0.f};
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float pv = fexp2(fmaf(sc[kt][r], P.scale_log2, -mc));
          sc[kt][r] = pv;
          psum[kt] += pv;
        }
      l += psum[0] + psum[1];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const bf16x8 pf = acc_to_frag(sc[kt], st);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] = mfma32(tr_frag<D>(Vt, kt * 32 + 16 * st, dt, lane), pf, o[dt]);
        }
    }
    unsigned char* nb = smem + ((t + 1) & 1) * 2 * TILE_BYTES;
    if (more_k) kl.store(nb);
    if (more_v) vl.store(nb + TILE_BYTES);
    __syncthreads();
  };

  int t = 0;
  for (; t + 1 < n_tiles; t += 2) {
    step(t, sa, sb);
    step(t + 1, sb, sa);
  }
  if (t < n_tiles) step(t, sa, sb);

  const float lt = l + __shfl_xor(l, 32, 64);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
  if (q_ok) {
    bf16* orow = P.o_out + b * P.o_sb + static_cast<int64_t>(q) * P.o_ss + hh * P.o_sh;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][4 * g4 + e] * inv);
        *reinterpret_cast<bf16x4*>(orow + dt * 32 + 8 * g4 + 4 * h) = v;
      }
    if (h == 0) P.lse[static_cast<int64_t>(bh) * P.Sq + q] = (lt > 0.f) ? m * P.scale_log2 + log2f(lt) : -INFINITY;
  }
}

// ===========================================================================
// Backward preprocessing: delta[b,h,q] = sum_d dO[q][d] * O[q][d]
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(AttnParams P) {
  constexpr int TPR = D / 8;  // threads per row
  const int64_t rows = static_cast<int64_t>(P.B) * P.H * P.Sq;
  const int64_t row = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) / TPR;
  const int c = threadIdx.x % TPR;
  float acc = 0.f;
  if (row < rows) {
    const int q = static_cast<int>(row % P.Sq);
    const int bh = static_cast<int>(row / P.Sq);
    const int b = bh / P.H, hh = bh % P.H;
    u16x8 a = *reinterpret_cast<const u16x8*>(P.o.p + b * P.o.sb + static_cast<int64_t>(q) * P.o.ss +
                                              hh * P.o.sh + c * 8);
    u16x8 d = *reinterpret_cast<const u16x8*>(P.dout.p + b * P.dout.sb + static_cast<int64_t>(q) * P.dout.ss +
                                              hh * P.dout.sh + c * 8);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += u2f(a[k]) * u2f(d[k]);
  }
#pragma unroll
  for (int o = TPR / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (row < rows && c == 0) P.delta[row] = acc;
}

// ===========================================================================
// dQ: query block resident (4 waves x 32 rows), loop over 64-key tiles.
//   S^T = K Q^T ; P^T = exp2(S^T*c - lse) ; dP^T = V dO^T ;
//   dS^T = P^T (dP^T - delta) ; dQ^T += K^T dS^T ; dQ = scale * dQ
// D = 64: 3 waves per SIMD (168 VGPRs) non-causal; causal needs the mask
// registers on top and spilled at 168 — a scratch reload inside the loop is a
// VMEM op, and its vmcnt wait drained the next K / V tile's prefetch every
// iteration — so the causal form runs 2 waves per SIMD without spills
// FUSED_DELTA: delta = rowsum(dO * O) of the block's own queries is computed
// here from the dO fragments already in registers (plus one 16-B O load per
// fragment) and written out for the dK / dV kernel, which then runs AFTER
// this one — the separate delta pass (a full re-read of dO and O) goes away.
template <int D, bool CAUSAL, bool FUSED_DELTA = false>
__global__ __launch_bounds__(256, (D == 64 ? (CAUSAL ? 2 : 3) : 1)) void attn_bwd_dq_kernel(AttnParams P) {
  constexpr int KS = D / 16, DT = D / 32, KV = 64;
  constexpr int TILE_BYTES = KV * D * 2;
  __shared__ __attribute__((aligned(16))) unsigned char smem[4 * TILE_BYTES];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  int bh = blockIdx.x, qb = gridDim.y - 1 - blockIdx.y;   // causal: longest-first (fwd)
  if (!CAUSAL) attn_head_block(P, bh, qb);
  const int b = bh / P.H, hh = bh % P.H;
  const int q_blk = qb * 128;
  const int qw = q_blk + wave * 32;
  const int q = qw + (lane & 31);
  const bool q_ok = q < P.Sq;

  bf16x8 qf[KS], df[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = q_ok ? *reinterpret_cast<const bf16x8*>(P.q.p + b * P.q.sb + static_cast<int64_t>(q) * P.q.ss +
                                                     hh * P.q.sh + ks * 16 + 8 * h)
                  : bf16x8{};
    df[ks] = q_ok ? *reinterpret_cast<const bf16x8*>(P.dout.p + b * P.dout.sb +
                                                     static_cast<int64_t>(q) * P.dout.ss + hh * P.dout.sh +
                                                     ks * 16 + 8 * h)
                  : bf16x8{};
  }
  const float lse = q_ok ? P.lse[static_cast<int64_t>(bh) * P.Sq + q] : 0.f;
  float dlt;
  if constexpr (FUSED_DELTA) {
    // lane (q, h) holds d = 16 ks + 8 h .. +8 of dO row q: a partial dot over
    // those, then the other half from lane ^ 32
    float part = 0.f;
    if (q_ok) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const bf16x8 of = *reinterpret_cast<const bf16x8*>(P.o.p + b * P.o.sb + static_cast<int64_t>(q) * P.o.ss +
                                                           hh * P.o.sh + ks * 16 + 8 * h);
#pragma unroll
        for (int e = 0; e < 8; ++e) part += bf2f(of[e]) * bf2f(df[ks][e]);
      }
    }
    dlt = part + __shfl_xor(part, 32, 64);
    if (q_ok && h == 0) P.delta[static_cast<int64_t>(bh) * P.Sq + q] = dlt;
  } else {
    dlt = q_ok ? P.delta[static_cast<int64_t>(bh) * P.Sq + q] : 0.f;
  }

  f32x16 dq[DT];
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt] = f32x16{};

  int n_tiles = (P.Sk + KV - 1) / KV;
  if (CAUSAL) n_tiles = min(n_tiles, (q_blk + 128 + KV - 1) / KV);

  TileLoader<D, KV> kl, vl;
  kl.load(P.k, b, hh, 0, P.Sk);
  vl.load(P.v, b, hh, 0, P.Sk);
  kl.store(smem);
  vl.store(smem + TILE_BYTES);
  __syncthreads();

  for (int t = 0; t < n_tiles; ++t) {
    const int k0 = t * KV;
    const unsigned char* Kt = smem + (t & 1) * 2 * TILE_BYTES;
    const unsigned char* Vt = Kt + TILE_BYTES;
    const bool has_next = t + 1 < n_tiles;
    if (has_next) {
      kl.load(P.k, b, hh, k0 + KV, P.Sk);
      vl.load(P.v, b, hh, k0 + KV, P.Sk);
    }
    const bool wave_active = !CAUSAL || (k0 <= qw + 31);
    const bool need_mask = (k0 + KV > P.Sk) || (CAUSAL && k0 + KV - 1 > qw) || (qw + 31 >= P.Sq);
    if (wave_active) {
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        f32x16 s = f32x16{}, dp = f32x16{};
        prio_hi(P);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const int off = lds_off<D>(kt * 32 + (lane & 31), 2 * ks + h);
          s = mfma32(lds_read16(Kt, off), qf[ks], s);
          dp = mfma32(lds_read16(Vt, off), df[ks], dp);
        }
        prio_lo(P);
        if (need_mask) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            float pv = fexp2(s[r] * P.scale_log2 - lse);
            if (key >= P.Sk || (CAUSAL && key > q) || !q_ok) pv = 0.f;
            s[r] = pv * (dp[r] - dlt);  // dS^T
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) s[r] = fexp2(s[r] * P.scale_log2 - lse) * (dp[r] - dlt);
        }
        prio_hi(P);
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          bf16x8 sf = acc_to_frag(s, st);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) dq[dt] = mfma32(tr_frag<D>(Kt, kt * 32 + 16 * st, dt, lane), sf, dq[dt]);
        }
        prio_lo(P);
      }
    }
    if (has_next) {
      unsigned char* nxt = smem + ((t + 1) & 1) * 2 * TILE_BYTES;
      kl.store(nxt);
      vl.store(nxt + TILE_BYTES);
    }
    __syncthreads();
  }
  if (P.dbq && P.db_ld) {
    if (qw < P.Sq)  // waves wholly past the sequence own no slab row
      bias_partial<DT>(dq, P.scale, P.dbq + (static_cast<int64_t>(b) * ((P.Sq + 31) / 32) + qw / 32) * P.db_ld + hh * D,
                     lane);
  } else if (P.dbq) {
    bias_colsum<DT>(dq, P.scale, P.dbq + hh * D, lane);
  }
  bf16* row = P.dq + b * P.dq_sb + static_cast<int64_t>(q) * P.dq_ss + hh * P.dq_sh;
  if (P.wide_store) {
    store_rows16<DT>(row, dq, P.scale, h, q_ok);
  } else if (q_ok) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        bf16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = f2bf(dq[dt][4 * g4 + e] * P.scale);
        *reinterpret_cast<bf16x4*>(row + dt * 32 + 8 * g4 + 4 * h) = v;
      }
  }
}

// ===========================================================================
// dK / dV: key block resident (4 waves x NKT*32 keys), loop over 64-query tiles.
//   S = Q K^T (key on lane) ; P = exp2(S*c - lse[q]) ; dP = dO V^T ;
//   dS = P (dP - delta[q]) ; dV^T += dO^T P ; dK^T += Q^T dS ; dK = scale*dK
// NKT = 2 (64 keys per wave): every Q / dO fragment read from LDS feeds two
// key subtiles, halving LDS traffic per MFMA; slower in practice (register
// pressure -> 1 wave/SIMD), kept behind FFK_ATTN_BWD_NKT=2 for experiments.
template <int D, bool CAUSAL, int NKT, bool PF = false>
__global__ __launch_bounds__(256, (D == 64 && NKT == 1 ? 2 : 1)) void attn_bwd_dkdv_kernel(AttnParams P) {
  static_assert(!PF || NKT == 1, "PF prefetch is written for one key subtile per wave");
  constexpr int KS = D / 16, DT = D / 32, QT = 64, KW = 32 * NKT;
  constexpr int TILE_BYTES = QT * D * 2;
  constexpr int STAGE = 2 * TILE_BYTES + 2 * QT * 4;  // Q, dO, lse, delta
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * STAGE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5;
  // causal: heads fastest, key block 0 (the most query tiles) first — longest first
  int bh = blockIdx.x, kb = blockIdx.y;
  if (!CAUSAL) attn_head_block(P, bh, kb);
  const int b = bh / P.H, hh = bh % P.H;
  const int k_blk = kb * (4 * KW);
  const int kw = k_blk + wave * KW;

  // K, V rows as B operands (lane holds row `key`, d = 16ks + 8h ..)
  bf16x8 kf[NKT][KS], vf[NKT][KS];
  int key[NKT];
  bool k_ok[NKT];
#pragma unroll
  for (int j = 0; j < NKT; ++j) {
    key[j] = kw + 32 * j + (lane & 31);
    k_ok[j] = key[j] < P.Sk;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[j][ks] = k_ok[j] ? *reinterpret_cast<const bf16x8*>(P.k.p + b * P.k.sb +
                                                             static_cast<int64_t>(key[j]) * P.k.ss + hh * P.k.sh +
                                                             ks * 16 + 8 * h)
                          : bf16x8{};
      vf[j][ks] = k_ok[j] ? *reinterpret_cast<const bf16x8*>(P.v.p + b * P.v.sb +
                                                             static_cast<int64_t>(key[j]) * P.v.ss + hh * P.v.sh +
                                                             ks * 16 + 8 * h)
                          : bf16x8{};
    }
  }
  f32x16 dk[NKT][DT], dv[NKT][DT];
#pragma unroll
  for (int j = 0; j < NKT; ++j)
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) dk[j][dt] = dv[j][dt] = f32x16{};

  const int n_q_tiles = (P.Sq + QT - 1) / QT;
  const int t0 = CAUSAL ? (k_blk / QT) : 0;

  TileLoader<D, QT> ql, dl;
  // row constants of a query tile, pre-shaped to seed the S and dP
  // accumulators (guide: "row constants as the initial accumulator"):
  // S' = Q K^T - lse / c, dP' = dO V^T - delta, so p = exp2(c S') and
  // dS = p dP' need no subtraction.  Fetched into registers with the tile's
  // Q / dO loads (a whole tile ahead) and parked in LDS after the compute:
  // loading them at the park point exposed one global-load latency per tile
  // to all four waves through the barrier that follows.
  // The raw values are kept until the park point and only then shaped: any
  // arithmetic on them at the fetch makes the compiler wait for the load
  // there, and vmcnt retires in order, so that wait would also drain the
  // Q / dO tile loads issued just before.
  float nls = 0.f, nds = 0.f;
  bool nok = false;
  auto fetch_scalars = [&](int q0) {
    const int qq = q0 + threadIdx.x;
    nok = threadIdx.x < QT && qq < P.Sq;
    if (nok) {
      nls = P.lse[static_cast<int64_t>(bh) * P.Sq + qq];
      nds = P.delta[static_cast<int64_t>(bh) * P.Sq + qq];
    }
  };
  auto park_scalars = [&](unsigned char* stage) {
    float* ls = reinterpret_cast<float*>(stage + 2 * TILE_BYTES);
    if (threadIdx.x < QT) {
      ls[threadIdx.x] = nok ? -nls * P.inv_scale_log2 : -INFINITY;
      ls[QT + threadIdx.x] = nok ? -nds : 0.f;
    }
  };
  // unconditional (rows past Sq load as zeros without touching memory): with
  // an `if (t0 < n_q_tiles)` around it the compiler kept a CFG path from the
  // K / V fragment loads above into the loop that skipped this block's
  // vmcnt(0), so the first MFMA of EVERY iteration waited on vmcnt — and
  // vmcnt retires in order, so that wait drained the next tile's prefetch
  // right after issuing it (one exposed global-load latency per tile)
  ql.load(P.q, b, hh, t0 * QT, P.Sq);
  dl.load(P.dout, b, hh, t0 * QT, P.Sq);
  fetch_scalars(t0 * QT);
  ql.store(smem);
  dl.store(smem + TILE_BYTES);
  park_scalars(smem);
  __syncthreads();

  for (int t = t0; t < n_q_tiles; ++t) {
    const int q0 = t * QT;
    unsigned char* stage = smem + ((t - t0) & 1) * STAGE;
    const unsigned char* Qt = stage;
    const unsigned char* Dt = stage + TILE_BYTES;
    const float* ls = reinterpret_cast<const float*>(stage + 2 * TILE_BYTES);
    const float* ds = ls + QT;
    const bool has_next = t + 1 < n_q_tiles;
    if (has_next) {
      ql.load(P.q, b, hh, q0 + QT, P.Sq);
      dl.load(P.dout, b, hh, q0 + QT, P.Sq);
      fetch_scalars(q0 + QT);
    }
    const bool wave_active = !CAUSAL || (q0 + QT - 1 >= kw);
    const bool need_mask = (q0 + QT > P.Sq) || (CAUSAL && q0 < kw + KW - 1) || (kw + KW - 1 >= P.Sk);
    if (wave_active) {
#pragma unroll
      for (int qt = 0; qt < 2; ++qt) {
        f32x16 s[NKT], dp[NKT];
        // PF: every LDS fragment of this 32-query subtile is requested before
        // the MFMAs that consume it — the row fragments of S / dP ahead of
        // the first product, the transposed fragments of dV / dK under the
        // S / dP products and the exp2 pass — instead of one read pair per
        // MFMA pair, each waiting out the LDS latency (FFK_ATTN_BWD_PF)
        [[maybe_unused]] bf16x8 qa_pf[PF ? KS : 1], da_pf[PF ? KS : 1];
        [[maybe_unused]] bf16x8 tda_pf[PF ? 2 : 1][PF ? DT : 1], tqa_pf[PF ? 2 : 1][PF ? DT : 1];
        if constexpr (PF) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const int off = lds_off<D>(qt * 32 + (lane & 31), 2 * ks + h);
            qa_pf[ks] = lds_read16(Qt, off);
            da_pf[ks] = lds_read16(Dt, off);
          }
        }
#pragma unroll
        for (int j = 0; j < NKT; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ql_ = qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            s[j][r] = ls[ql_];
            dp[j][r] = ds[ql_];
          }
        prio_hi(P);
        if constexpr (PF) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            s[0] = mfma32(qa_pf[ks], kf[0][ks], s[0]);
            dp[0] = mfma32(da_pf[ks], vf[0][ks], dp[0]);
          }
#pragma unroll
          for (int st = 0; st < 2; ++st)
#pragma unroll
            for (int dt = 0; dt < DT; ++dt) {
              tda_pf[st][dt] = tr_frag<D>(Dt, qt * 32 + 16 * st, dt, lane);
              tqa_pf[st][dt] = tr_frag<D>(Qt, qt * 32 + 16 * st, dt, lane);
            }
        } else {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            const int off = lds_off<D>(qt * 32 + (lane & 31), 2 * ks + h);
            const bf16x8 qa = lds_read16(Qt, off), da = lds_read16(Dt, off);
#pragma unroll
            for (int j = 0; j < NKT; ++j) {
              s[j] = mfma32(qa, kf[j][ks], s[j]);
              dp[j] = mfma32(da, vf[j][ks], dp[j]);
            }
          }
        }
        prio_lo(P);
#pragma unroll
        for (int j = 0; j < NKT; ++j) {
          if (need_mask) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const int qq = q0 + qt * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
              float pv = fexp2(s[j][r] * P.scale_log2);
              if (qq >= P.Sq || (CAUSAL && key[j] > qq) || !k_ok[j]) pv = 0.f;
              s[j][r] = pv;
              dp[j][r] = pv * dp[j][r];
            }
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              const float pv = fexp2(s[j][r] * P.scale_log2);
              s[j][r] = pv;
              dp[j][r] = pv * dp[j][r];
            }
          }
        }
        prio_hi(P);
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          bf16x8 pf[NKT], sf[NKT];
#pragma unroll
          for (int j = 0; j < NKT; ++j) {
            pf[j] = acc_to_frag(s[j], st);
            sf[j] = acc_to_frag(dp[j], st);
          }
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) {
            bf16x8 da, qa;
            if constexpr (PF) {
              da = tda_pf[st][dt];
              qa = tqa_pf[st][dt];
            } else {
              da = tr_frag<D>(Dt, qt * 32 + 16 * st, dt, lane);
              qa = tr_frag<D>(Qt, qt * 32 + 16 * st, dt, lane);
            }
#pragma unroll
            for (int j = 0; j < NKT; ++j) {
              dv[j][dt] = mfma32(da, pf[j], dv[j][dt]);
              dk[j][dt] = mfma32(qa, sf[j], dk[j][dt]);
            }
          }
        }
        prio_lo(P);
      }
    }
    if (has_next) {
      unsigned char* nxt = smem + ((t + 1 - t0) & 1) * STAGE;
      ql.store(nxt);
      dl.store(nxt + TILE_BYTES);
      park_scalars(nxt);
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < NKT; ++j) {
    if (P.db_ld) {
      if (kw + 32 * j >= P.Sk) continue;
      const int64_t roff = (static_cast<int64_t>(b) * ((P.Sk + 31) / 32) + (kw + 32 * j) / 32) * P.db_ld + hh * D;
      if (P.dbk) bias_partial<DT>(dk[j], P.scale, P.dbk + roff, lane);
      if (P.dbv) bias_partial<DT>(dv[j], 1.f, P.dbv + roff, lane);
    } else {
      if (P.dbk) bias_colsum<DT>(dk[j], P.scale, P.dbk + hh * D, lane);
      if (P.dbv) bias_colsum<DT>(dv[j], 1.f, P.dbv + hh * D, lane);
    }
  }
#pragma unroll
  for (int j = 0; j < NKT; ++j) {
    bf16* krow = P.dk + b * P.dk_sb + static_cast<int64_t>(key[j]) * P.dk_ss + hh * P.dk_sh;
    bf16* vrow = P.dv + b * P.dv_sb + static_cast<int64_t>(key[j]) * P.dv_ss + hh * P.dv_sh;
    if (P.wide_store) {   // every lane swaps; k_ok guards the stores
      store_rows16<DT>(krow, dk[j], P.scale, h, k_ok[j]);
      store_rows16<DT>(vrow, dv[j], 1.f, h, k_ok[j]);
      continue;
    }
    if (!k_ok[j]) continue;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        bf16x4 a, c;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          a[e] = f2bf(dk[j][dt][4 * g4 + e] * P.scale);
          c[e] = f2bf(dv[j][dt][4 * g4 + e]);
        }
        *reinterpret_cast<bf16x4*>(krow + dt * 32 + 8 * g4 + 4 * h) = a;
        *reinterpret_cast<bf16x4*>(vrow + dt * 32 + 8 * g4 + 4 * h) = c;
      }
  }
}

// ===========================================================================
static AttnParams make_params(const AttnTensors& t, int B, int H, int Sq, int Sk, int D, float scale) {
  AttnParams P{};
  auto tv = [](const AttnTensors::T& x) {
    return TensorView{static_cast<const bf16*>(x.p), x.sb, x.ss, x.sh};
  };
  P.q = tv(t.q);
  P.k = tv(t.k);
  P.v = tv(t.v);
  P.o = tv(t.o);
  P.dout = tv(t.dout);
  P.o_out = static_cast<bf16*>(const_cast<void*>(t.o.p));
  P.o_sb = t.o.sb; P.o_ss = t.o.ss; P.o_sh = t.o.sh;
  P.dq = static_cast<bf16*>(const_cast<void*>(t.dq.p));
  P.dq_sb = t.dq.sb; P.dq_ss = t.dq.ss; P.dq_sh = t.dq.sh;
  P.dk = static_cast<bf16*>(const_cast<void*>(t.dk.p));
  P.dk_sb = t.dk.sb; P.dk_ss = t.dk.ss; P.dk_sh = t.dk.sh;
  P.dv = static_cast<bf16*>(const_cast<void*>(t.dv.p));
  P.dv_sb = t.dv.sb; P.dv_ss = t.dv.ss; P.dv_sh = t.dv.sh;
  P.lse = t.lse;
  P.delta = t.delta;
  P.dbq = t.dbq;
  P.dbk = t.dbk;
  P.dbv = t.dbv;
  P.db_ld = t.db_ld;
  P.B = B; P.H = H; P.Sq = Sq; P.Sk = Sk;
  P.scale = scale;
  P.scale_log2 = scale * 1.4426950408889634f;
  P.inv_scale_log2 = 1.f / P.scale_log2;
  // default: on for D = 128 (forward -7 %, backward -1 %), off for D = 64
  // where it measured neutral (profiles/ab_attn_prio_r2.txt)
  static const int prio = [] {
    const char* e = getenv("FFK_ATTN_PRIO");
    return e ? atoi(e) : -1;
  }();
  P.prio = prio >= 0 ? prio : (D == 128 ? 1 : 0);
  // read per call: tools/attn_time.py --xcd-ab switches it inside one process
  const char* xe = getenv("FFK_ATTN_XCD");
  P.xcd = xe ? atoi(xe) : 1;
  const char* we = getenv("FFK_ATTN_WIDE_STORE");
  P.wide_store = we ? atoi(we) : 1;
  return P;
}

void attention_fwd(const AttnTensors& t, int B, int H, int Sq, int Sk, int D, float scale, bool causal,
                   hipStream_t st) {
  AttnParams P = make_params(t, B, H, Sq, Sk, D, scale);
  const unsigned nq = static_cast<unsigned>((Sq + 127) / 128), nbh = static_cast<unsigned>(B * H);
  dim3 grid = causal ? dim3(nbh, nq) : dim3(nq, nbh), block(256);
  // read per call (not cached): the A/B tests switch it inside one process.
  // Opt-in: 2 waves / SIMD (226 VGPRs) against the default's 3, and slower at
  // both bench shapes (BERT 0.145 vs 0.118 ms, GPT causal 0.253 vs 0.212 ms,
  // profiles/r4/attn_pipe_ab_r4.jsonl): the third wave hides more than the
  // in-wave overlap gains
  const char* pe = getenv("FFK_ATTN_FWD_PIPE");
  const int pipe = pe ? atoi(pe) : 0;
  if (pipe && D == 64) {
    if (causal) hipLaunchKernelGGL((attn_fwd_pipe_kernel<64, true>), grid, block, 0, st, P);
    else hipLaunchKernelGGL((attn_fwd_pipe_kernel<64, false>), grid, block, 0, st, P);
    FFK_LAUNCH_CHECK("attention_fwd");
    return;
  }
  if (D == 64) {
    if (causal) hipLaunchKernelGGL((attn_fwd_kernel<64, true>), grid, block, 0, st, P);
    else hipLaunchKernelGGL((attn_fwd_kernel<64, false>), grid, block, 0, st, P);
  } else if (D == 128) {
    if (causal) hipLaunchKernelGGL((attn_fwd_kernel<128, true>), grid, block, 0, st, P);
    else hipLaunchKernelGGL((attn_fwd_kernel<128, false>), grid, block, 0, st, P);
  } else {
    throw std::invalid_argument("attention: head dim must be 64 or 128");
  }
  FFK_LAUNCH_CHECK("attention_fwd");
}

template <int D, bool CAUSAL>
static void launch_dkdv(int nkt, dim3 grid, dim3 block, hipStream_t st, const AttnParams& P) {
  if constexpr (D == 64) {
    if (nkt == 2) {
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, CAUSAL, 2>), grid, block, 0, st, P);
      return;
    }
  }
  // default on: GPT causal shape 0.341 -> 0.333 ms, BERT within noise
  // (profiles/ab_attn_bwd_pf_r3.txt); FFK_ATTN_BWD_PF=0 for the per-pair reads
  static const int pf = [] {
    const char* e = getenv("FFK_ATTN_BWD_PF");
    return e ? atoi(e) : 1;
  }();
  if (pf && D == 64) {  // at D = 128 (one wave / SIMD) the prefetch registers spill
    hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, CAUSAL, 1, D == 64>), grid, block, 0, st, P);
    return;
  }
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, CAUSAL, 1>), grid, block, 0, st, P);
}

void attention_bwd(const AttnTensors& t, int B, int H, int Sq, int Sk, int D, float scale, bool causal,
                   hipStream_t st) {
  AttnParams P = make_params(t, B, H, Sq, Sk, D, scale);
  const int64_t rows = static_cast<int64_t>(B) * H * Sq;
  const int tpr = D / 8;
  dim3 gd(static_cast<unsigned>((rows * tpr + 255) / 256));
  static const int nkt_env = [] {
    const char* e = getenv("FFK_ATTN_BWD_NKT");
    return e ? atoi(e) : 0;
  }();
  // NKT = 2 (64 keys per wave) halves LDS reads per MFMA but needs ~500
  // registers (1 wave/SIMD, spills when causal): measured 0.24 vs 0.21 ms
  // (BERT shape) and 0.92 vs 0.56 ms (GPT causal) — opt-in only.
  const int nkt = D == 64 && nkt_env == 2 ? 2 : 1;
  const unsigned nq = static_cast<unsigned>((Sq + 127) / 128), nbh = static_cast<unsigned>(B * H);
  const unsigned nk = static_cast<unsigned>((Sk + 128 * nkt - 1) / (128 * nkt));
  dim3 gq = causal ? dim3(nbh, nq) : dim3(nq, nbh), gk = causal ? dim3(nbh, nk) : dim3(nk, nbh), block(256);
  // read per call: the A/B tool switches it inside one process
  const char* fde = getenv("FFK_ATTN_BWD_FUSED_DELTA");
  const bool fused_delta = fde ? atoi(fde) != 0 : true;
#define FFK_ATTN_BWD(DD, CC)                                                          \
  if (fused_delta) {                                                                  \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, CC, true>), gq, block, 0, st, P);      \
    launch_dkdv<DD, CC>(nkt, gk, block, st, P);                                       \
  } else {                                                                            \
    hipLaunchKernelGGL((attn_bwd_delta_kernel<DD>), gd, block, 0, st, P);             \
    launch_dkdv<DD, CC>(nkt, gk, block, st, P);                                       \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<DD, CC>), gq, block, 0, st, P);            \
  }
  if (D == 64) {
    if (causal) { FFK_ATTN_BWD(64, true); }
    else { FFK_ATTN_BWD(64, false); }
  } else if (D == 128) {
    if (causal) { FFK_ATTN_BWD(128, true); }
    else { FFK_ATTN_BWD(128, false); }
  } else {
    throw std::invalid_argument("attention: head dim must be 64 or 128");
  }
#undef FFK_ATTN_BWD
  FFK_LAUNCH_CHECK("attention_bwd");
}

}  // namespace ffk
