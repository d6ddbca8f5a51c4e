// Fused cross-entropy forward + logits-gradient.
//
// nanoGPT: F.cross_entropy(logits.view(-1, V), targets.view(-1), ignore_index=-1)
// over logits [N, V] (V = 50304 for GPT-2: 1.2 GB of bf16 logits per 124M
// micro-step).  One 256-thread block per row:
//   pass 1: online (max, sum-exp) over the row with 16-byte loads,
//           block-combined through LDS;
//   pass 2: re-read the row (L2/Infinity-Cache resident) and overwrite it IN
//           PLACE with softmax - onehot(target) in bf16 (the unnormalised
//           dL/dlogits; the 1/n_valid * grad_out factor is applied later on the
//           small [N, C] side of the lm_head GEMMs).
// row_loss[r] = logsumexp - logit[target] (0 for ignored rows, whose gradient
// row is zeroed).  The [N, V] fp32 softmax never exists.
//
// For V <= 256 x 8 x kRegChunks (GPT-2's 50304) the row is held in registers
// (xent_reg_kernel): every thread issues all its 16-byte loads at once (deep
// memory parallelism), the reductions and the gradient come from registers, and
// HBM sees exactly one read and one write of the logits (the streaming kernel
// re-reads the row and depends on it still being in L2).
#include "common.h"

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  if (m2 > m) {
    s = s * __expf(m - m2) + s2;
    m = m2;
  } else {
    s = s + s2 * __expf(m2 - m);
  }
}

template <bool VEC, bool H = false>
__global__ __launch_bounds__(kBlock) void xent_kernel(bf16_t* __restrict__ logits, const int64_t* __restrict__ targets,
                                                     float* __restrict__ row_loss, int V, int ld, int write_grad) {
  const int row = blockIdx.x;
  bf16_t* lr = logits + (int64_t)row * ld;
  const int64_t tgt = targets[row];
  float m = -INFINITY, s = 0.0f;
  if (VEC) {
    const int nv = ld / 8;
    for (int i = threadIdx.x; i < nv; i += kBlock) {
      float f[8];
      load8e<H>(lr + i * 8, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = i * 8 + j < V ? f[j] : -INFINITY;
      float bm = f[0];
#pragma unroll
      for (int j = 1; j < 8; ++j) bm = fmaxf(bm, f[j]);
      if (bm == -INFINITY) continue;  // a chunk of padding columns only
      float bs = 0.0f;
#pragma unroll
      for (int j = 0; j < 8; ++j) bs += __expf(f[j] - bm);
      online_merge(m, s, bm, bs);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += kBlock) online_merge(m, s, e2f<H>(lr[i]), 1.0f);
  }
  // wave reduce of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64);
    const float s2 = __shfl_xor(s, o, 64);
    if (m2 != -INFINITY) online_merge(m, s, m2, s2);
  }
  __shared__ float sm[kBlock / 64], ss[kBlock / 64];
  __shared__ float tgt_logit;
  if ((threadIdx.x & 63) == 0) {
    sm[threadIdx.x >> 6] = m;
    ss[threadIdx.x >> 6] = s;
  }
  if (threadIdx.x == 0) tgt_logit = (tgt >= 0 && tgt < V) ? e2f<H>(lr[tgt]) : 0.0f;
  __syncthreads();
  float M = sm[0], S = ss[0];
#pragma unroll
  for (int w = 1; w < kBlock / 64; ++w) online_merge(M, S, sm[w], ss[w]);
  const float lse = M + __logf(S);
  const bool valid = tgt >= 0 && tgt < V;
  if (threadIdx.x == 0) row_loss[row] = valid ? lse - tgt_logit : 0.0f;
  if (!write_grad) return;
  const float invS = 1.0f / S;
  if (VEC) {
    const int nv = ld / 8;
    for (int i = threadIdx.x; i < nv; i += kBlock) {
      float f[8];
      load8e<H>(lr + i * 8, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = i * 8 + j;
        float p = valid && col < V ? __expf(f[j] - M) * invS : 0.0f;
        if (valid && col == tgt) p -= 1.0f;
        f[j] = p;
      }
      store8e<H>(lr + i * 8, f);
    }
  } else {
    for (int i = threadIdx.x; i < V; i += kBlock) {
      float p = valid ? __expf(e2f<H>(lr[i]) - M) * invS : 0.0f;
      if (valid && i == tgt) p -= 1.0f;
      lr[i] = f2e<H>(p);
    }
  }
}

// Register-resident variants: RB threads per row, RC 16-byte chunks per thread
// (rows up to RB * 8 * RC logits).  Fewer chunks per thread = fewer VGPRs = more
// rows in flight per CU: the load phase of one row overlaps the exp / store phase
// of the others (a 256 x 25 block is VGPR-limited to 2 rows per CU).
constexpr int kRegChunks = 25;  // 256 threads: rows up to 51200 bf16 logits

template <int RB>
__device__ __forceinline__ float block_reduce_max(float v, float* red) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < RB / 64; ++w) r = fmaxf(r, red[w]);
  return r;
}

template <int RB>
__device__ __forceinline__ float block_reduce_sum(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
#pragma unroll
  for (int w = 1; w < RB / 64; ++w) r += red[w];
  return r;
}

typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));

// NT bit 0: nontemporal logit loads, bit 1: nontemporal gradient stores + packed
// v_cvt_pk_bf16_f32 conversion (the logits are streamed exactly once each way)
template <int RB, int RC, int NT = 0, bool H = false>
__global__ __launch_bounds__(RB) void xent_reg_kernel(bf16_t* __restrict__ logits,
                                                     const int64_t* __restrict__ targets,
                                                     float* __restrict__ row_loss, int V, int ld,
                                                     int write_grad) {
  constexpr int kBlock = RB;
  constexpr int kRegChunks = RC;
  const int row = blockIdx.x;
  bf16_t* lr = logits + (int64_t)row * ld;
  const int64_t tgt = targets[row];
  const bool valid = tgt >= 0 && tgt < V;
  const int nv = ld / 8;
  const bool pad = V != ld;  // vocabulary padding columns (>= V) take no part
  __shared__ float red[kBlock / 64];
  // all loads first (clamped index, no branch around a load), then compute
  uint4 r[kRegChunks];
#pragma unroll
  for (int c = 0; c < kRegChunks; ++c) {
    const int i = min((int)threadIdx.x + c * kBlock, nv - 1);
    if constexpr (NT & 1) {
      const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(lr + (int64_t)i * 8));
      r[c] = make_uint4(v.x, v.y, v.z, v.w);
    } else {
      r[c] = *reinterpret_cast<const uint4*>(lr + (int64_t)i * 8);
    }
  }
  const float tgt_logit = valid ? e2f<H>(lr[tgt]) : 0.0f;
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < kRegChunks; ++c) {
    if ((int)threadIdx.x + c * kBlock < nv) {
      const uint32_t w4[4] = {r[c].x, r[c].y, r[c].z, r[c].w};
      const int col = ((int)threadIdx.x + c * kBlock) * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float lo = !pad || col + 2 * q < V ? lo2f<H>(w4[q]) : -INFINITY;
        const float hi = !pad || col + 2 * q + 1 < V ? hi2f<H>(w4[q]) : -INFINITY;
        m = fmaxf(m, fmaxf(lo, hi));
      }
    }
  }
  const float M = block_reduce_max<RB>(m, red);
  float s = 0.0f;
#pragma unroll
  for (int c = 0; c < kRegChunks; ++c) {
    if ((int)threadIdx.x + c * kBlock < nv) {
      const uint32_t w4[4] = {r[c].x, r[c].y, r[c].z, r[c].w};
      const int col = ((int)threadIdx.x + c * kBlock) * 8;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float e0 = __expf(lo2f<H>(w4[q]) - M), e1 = __expf(hi2f<H>(w4[q]) - M);
        s += (!pad || col + 2 * q < V ? e0 : 0.0f) + (!pad || col + 2 * q + 1 < V ? e1 : 0.0f);
      }
    }
  }
  const float S = block_reduce_sum<RB>(s, red);
  if (threadIdx.x == 0) row_loss[row] = valid ? M + __logf(S) - tgt_logit : 0.0f;
  if (!write_grad) return;
  const float invS = 1.0f / S;
#pragma unroll
  for (int c = 0; c < kRegChunks; ++c) {
    const int i = (int)threadIdx.x + c * kBlock;
    if (i < nv) {
      const uint32_t w4[4] = {r[c].x, r[c].y, r[c].z, r[c].w};
      float f[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f[2 * q] = valid && (!pad || i * 8 + 2 * q < V) ? __expf(lo2f<H>(w4[q]) - M) * invS : 0.0f;
        f[2 * q + 1] = valid && (!pad || i * 8 + 2 * q + 1 < V) ? __expf(hi2f<H>(w4[q]) - M) * invS : 0.0f;
      }
      if (valid && (tgt >> 3) == i) f[tgt & 7] -= 1.0f;
      if constexpr (NT & 2) {
        u32x4_t v;
        v.x = pk2<H>(f[0], f[1]);
        v.y = pk2<H>(f[2], f[3]);
        v.z = pk2<H>(f[4], f[5]);
        v.w = pk2<H>(f[6], f[7]);
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(lr + (int64_t)i * 8));
      } else {
        store8e<H>(lr + (int64_t)i * 8, f);
      }
    }
  }
}

}  // namespace

// write_grad bits 8..15 select the register-resident geometry (A/B timing,
// scripts/membound_ab.py at 122880 x 50304: 1024 x 7 4.55 ms = 5.4 TB/s,
// 512 x 13 4.59 ms, 256 x 25 4.86 ms): 0 = default (1024 x 7, nontemporal loads and
// stores), 1 = 256 x 25, 2 = 512 x 13, 3 / 4 / 5 = 1024 x 7 with nontemporal loads + stores /
// stores / loads, 6 = 1024 x 7 plain.  Nontemporal loads + stores: 4618 -> 4348 us
// (5.35 -> 5.69 TB/s, bitwise-identical output); stores alone 4557, loads alone 4641.
// Rows are `ld` apart; columns >= V (vocabulary padding, ld > V) are excluded and get a
// zero gradient.  Since round 4 this separate pass serves deterministic mode and the shapes
// the fused path (xent_fused.hip) does not take.
namespace {
template <bool H>
hipError_t xent_entry(void* logits, const void* targets, void* row_loss, int N, int V, int ld, int write_grad,
                      hipStream_t s) {
  const int variant = (write_grad >> 8) & 0xff;
  write_grad &= 0xff;
  if (ld < V) return hipErrorInvalidValue;
  bf16_t* lg = (bf16_t*)logits;
  const int64_t* tg = (const int64_t*)targets;
  float* rl = (float*)row_loss;
  const bool vec = ld % 8 == 0;
  if (vec && variant >= 3 && variant <= 5 && ld <= 1024 * 8 * 7) {
    // 3: nontemporal loads + stores, 4: nontemporal stores, 5: nontemporal loads
    if (variant == 3) xent_reg_kernel<1024, 7, 3, H><<<N, 1024, 0, s>>>(lg, tg, rl, V, ld, write_grad);
    else if (variant == 4) xent_reg_kernel<1024, 7, 2, H><<<N, 1024, 0, s>>>(lg, tg, rl, V, ld, write_grad);
    else xent_reg_kernel<1024, 7, 1, H><<<N, 1024, 0, s>>>(lg, tg, rl, V, ld, write_grad);
  } else if (vec && variant == 1 && ld <= 256 * 8 * 25)
    xent_reg_kernel<256, 25, 0, H><<<N, 256, 0, s>>>(lg, tg, rl, V, ld, write_grad);
  else if (vec && variant == 2 && ld <= 512 * 8 * 13)
    xent_reg_kernel<512, 13, 0, H><<<N, 512, 0, s>>>(lg, tg, rl, V, ld, write_grad);
  else if (vec && (variant == 6 || (int64_t)N * ld * 2 < NSA_NT_MIN_BYTES) && ld <= 1024 * 8 * 7)
    xent_reg_kernel<1024, 7, 0, H><<<N, 1024, 0, s>>>(lg, tg, rl, V, ld, write_grad);
  else if (vec && ld <= 1024 * 8 * 7)  // default: nontemporal loads + stores
    xent_reg_kernel<1024, 7, 3, H><<<N, 1024, 0, s>>>(lg, tg, rl, V, ld, write_grad);
  else if (vec)
    xent_kernel<true, H><<<N, kBlock, 0, s>>>(lg, tg, rl, V, ld, write_grad);
  else
    xent_kernel<false, H><<<N, kBlock, 0, s>>>(lg, tg, rl, V, ld, write_grad);
  return hipGetLastError();
}
}  // namespace

NSA_API hipError_t nsa_xent_fwd(void* logits, const void* targets, void* row_loss, int N, int V, int ld,
                                int write_grad, hipStream_t s) {
  return xent_entry<false>(logits, targets, row_loss, N, V, ld, write_grad, s);
}
// fp16 logits (dtype float16: autocast's fp16 logits, the softmax and loss in fp32)
NSA_API hipError_t nsa_xent_fwd_h(void* logits, const void* targets, void* row_loss, int N, int V, int ld,
                                  int write_grad, hipStream_t s) {
  return xent_entry<true>(logits, targets, row_loss, N, V, ld, write_grad, s);
}
