// Memory-bound elementwise kernels: exact-erf GELU fwd/bwd, hash dropout,
// fp32 -> bf16 cast.  16-byte vector access per lane (8 bf16); each thread keeps
// kUnroll independent 16-byte loads in flight (all loads of an iteration are
// issued before any math), which lifted GELU from ~4.4 to HBM-rate; grid-strided
// over 256 CUs x 8 blocks (cdna_hip_programming.md Guideline 11).
//
// nanoGPT MLP uses nn.GELU() — the exact erf form, not the tanh approximation
// (SURVEY.md §2.3 U-M3, K4).
#include "common.h"

#include <stdlib.h>

namespace {

constexpr int kBlock = 256;
#ifndef NSA_EW_UNROLL
#define NSA_EW_UNROLL 4  // loads in flight per thread (A/B at 377M elements: 2 / 4 / 8 -> GELU bwd 426 / 399 / 414 us)
#endif
constexpr int kUnroll = NSA_EW_UNROLL;

// Grid cap: 2048 blocks = 8 per CU x 4 waves fill every wave slot (fastest alone).
// NSA_EW_MAX_BLOCKS lowers it (an A/B knob: room for another stream's workgroups; the
// training step itself runs on one compute stream).
inline int64_t ew_grid_cap() {
  static int64_t cap = [] {
    const char* e = getenv("NSA_EW_MAX_BLOCKS");
    const long v = e ? atol(e) : 0;
    return (int64_t)(v > 0 ? v : 2048);
  }();
  return cap;
}

inline int grid_for(int64_t n_vec) {
  int64_t g = (n_vec + kBlock * kUnroll - 1) / (kBlock * kUnroll);
  if (g > ew_grid_cap()) g = ew_grid_cap();
  if (g < 1) g = 1;
  return (int)g;
}

#ifdef NSA_GELU_PROBE_COPY  // A/B probe only (build_variant): data movement without the erf math
__device__ __forceinline__ float gelu_f(float x) { return x; }
__device__ __forceinline__ float gelu_grad(float x) { return x; }
#else
__device__ __forceinline__ float gelu_f(float x) { return nsa_gelu(x); }
__device__ __forceinline__ float gelu_grad(float x) { return nsa_gelu_grad(x); }
#endif

typedef unsigned ew_u32x4 __attribute__((ext_vector_type(4)));
// NT: nontemporal 16-byte loads / stores (each byte is streamed exactly once)
template <bool NT>
__device__ __forceinline__ uint4 ld16(const bf16_t* p) {
  if constexpr (NT) {
    const ew_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const ew_u32x4*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    return *reinterpret_cast<const uint4*>(p);
  }
}
template <bool NT, bool H = false>
__device__ __forceinline__ void st8(bf16_t* p, const float (&f)[8]) {
  if constexpr (NT) {
    ew_u32x4 v;
    v.x = pk2<H>(f[0], f[1]);
    v.y = pk2<H>(f[2], f[3]);
    v.z = pk2<H>(f[4], f[5]);
    v.w = pk2<H>(f[6], f[7]);
    __builtin_nontemporal_store(v, reinterpret_cast<ew_u32x4*>(p));
  } else {
    store8e<H>(p, f);
  }
}

// H (every kernel below): the 16-bit tensors are fp16 instead of bf16
template <bool NT = false, bool H = false>
__global__ __launch_bounds__(kBlock) void gelu_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         int64_t n) {
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * kBlock * kUnroll;
  for (int64_t i0 = (int64_t)blockIdx.x * kBlock * kUnroll + threadIdx.x; i0 < nv; i0 += stride) {
    uint4 u[kUnroll];
#pragma unroll
    for (int r = 0; r < kUnroll; ++r) {
      const int64_t i = min(i0 + (int64_t)r * kBlock, nv - 1);
      u[r] = ld16<NT>(x + i * 8);
    }
#pragma unroll
    for (int r = 0; r < kUnroll; ++r) {
      const int64_t i = i0 + (int64_t)r * kBlock;
      if (i < nv) {
        float f[8];
        unpack8e<H>(u[r], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = gelu_f(f[j]);
        st8<NT, H>(y + i * 8, f);
      }
    }
  }
  // scalar tail
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    y[i] = f2e<H>(gelu_f(e2f<H>(x[i])));
}

template <bool NT = false, bool H = false>
__global__ __launch_bounds__(kBlock) void gelu_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                         bf16_t* __restrict__ dx, int64_t n) {
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * kBlock * kUnroll;
  for (int64_t i0 = (int64_t)blockIdx.x * kBlock * kUnroll + threadIdx.x; i0 < nv; i0 += stride) {
    uint4 ug[kUnroll], ux[kUnroll];
#pragma unroll
    for (int r = 0; r < kUnroll; ++r) {
      const int64_t i = min(i0 + (int64_t)r * kBlock, nv - 1);
      ug[r] = ld16<NT>(dy + i * 8);
      ux[r] = ld16<NT>(x + i * 8);
    }
#pragma unroll
    for (int r = 0; r < kUnroll; ++r) {
      const int64_t i = i0 + (int64_t)r * kBlock;
      if (i < nv) {
        float g[8], f[8];
        unpack8e<H>(ug[r], g);
        unpack8e<H>(ux[r], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = g[j] * gelu_grad(f[j]);
        st8<NT, H>(dx + i * 8, f);
      }
    }
  }
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    dx[i] = f2e<H>(e2f<H>(dy[i]) * gelu_grad(e2f<H>(x[i])));
}

template <bool H = false>
__global__ __launch_bounds__(kBlock) void dropout_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                        int64_t n, uint32_t thresh, float scale, uint64_t salt) {
  const uint64_t seed = nsa_seed(salt);
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kBlock) {
    float f[8];
    load8e<H>(x + i * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = nsa_keep(seed, (uint64_t)(i * 8 + j), thresh) ? f[j] * scale : 0.0f;
    store8e<H>(y + i * 8, f);
  }
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    y[i] = f2e<H>(nsa_keep(seed, (uint64_t)i, thresh) ? e2f<H>(x[i]) * scale : 0.0f);
}

template <bool H = false>
__global__ __launch_bounds__(kBlock) void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                              int64_t n) {
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kBlock) {
    const float4 a = reinterpret_cast<const float4*>(x)[2 * i];
    const float4 b = reinterpret_cast<const float4*>(x)[2 * i + 1];
    float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    store8e<H>(y + i * 8, f);
  }
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    y[i] = f2e<H>(x[i]);
}

// dst[C][R] = src[R][C]^T for bf16 (R, C multiples of 64): the cached K-contiguous
// weight transposes of the input-gradient GEMMs, rebuilt once per optimizer step.
// One wave per 64 x 64 region as 8 x 8 blocks of 8 x 8 elements: lane (lx, ly)
// loads block (ly, lx) as eight 16-B row pieces (lanes lx = 0..7 read one 128-B
// line), transposes it in registers with v_perm_b32, and stores eight 16-B column
// pieces (lanes ly = 0..7 write one 128-B line of the destination row).
// torch's generic transpose copy ran the 50304 x 768 lm_head weight at 0.39 TB/s.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                            int R, int C) {
  const int lane = threadIdx.x & 63;
  const int64_t region = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int rc = C / 64;
  if (region >= (int64_t)(R / 64) * rc) return;
  const int r0 = (int)(region / rc) * 64, c0 = (int)(region % rc) * 64;
  const int lx = lane & 7, ly = lane >> 3;
  const int br = r0 + 8 * ly, bc = c0 + 8 * lx;
  uint4 in[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) in[i] = *reinterpret_cast<const uint4*>(src + (int64_t)(br + i) * C + bc);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    // column j of the block: element j of rows 0..7 = 16-bit half (j & 1) of dword j >> 1
    const uint32_t sel = (j & 1) ? 0x07060302u : 0x05040100u;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t lo = reinterpret_cast<const uint32_t*>(&in[2 * k])[j >> 1];
      const uint32_t hi = reinterpret_cast<const uint32_t*>(&in[2 * k + 1])[j >> 1];
      w[k] = __builtin_amdgcn_perm(hi, lo, sel);
    }
    *reinterpret_cast<uint4*>(dst + (int64_t)(bc + j) * R + br) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// out[i] += sum over s = 0 .. S-1 (in that order) of ws[s * n + i]: the fixed-order
// reduction of split-K weight-gradient partials (deterministic mode)
__global__ __launch_bounds__(kBlock) void splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                              int64_t n, int splits) {
  const int64_t nv = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kBlock) {
    float4 acc = reinterpret_cast<const float4*>(ws)[i];
    for (int sp = 1; sp < splits; ++sp) {
      const float4 v = reinterpret_cast<const float4*>(ws + (int64_t)sp * n)[i];
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    float4 o = reinterpret_cast<float4*>(out)[i];
    o.x += acc.x;
    o.y += acc.y;
    o.z += acc.z;
    o.w += acc.w;
    reinterpret_cast<float4*>(out)[i] = o;
  }
  for (int64_t i = nv * 4 + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    float acc = ws[i];
    for (int sp = 1; sp < splits; ++sp) acc += ws[(int64_t)sp * n + i];
    out[i] += acc;
  }
}

// y[i] *= s[0]  (16-bit tensor scaled by a device scalar; no host sync)
template <bool H = false>
__global__ __launch_bounds__(kBlock) void scale_bf16_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                           const float* __restrict__ s, int64_t n) {
  const float sc = s[0];
  const int64_t nv = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nv; i += (int64_t)gridDim.x * kBlock) {
    float f[8];
    load8e<H>(x + i * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] *= sc;
    store8e<H>(y + i * 8, f);
  }
  for (int64_t i = nv * 8 + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock)
    y[i] = f2e<H>(e2f<H>(x[i]) * sc);
}

}  // namespace

// nontemporal loads / stores in the GELU passes (default; NSA_EW_NT=0 turns them off, read
// once, nsa_ew_set_nt for A/B runs).  scripts/membound_ab.py at 122880 x 3072: fwd 282.7 -> 278.3 us,
// bwd 428.4 -> 410.9 us (5.29 -> 5.51 TB/s)
// resolved once from NSA_EW_NT (0 = plain loads / stores); nsa_ew_set_nt switches it (A/B)
static int& ew_nt_flag() {
  static int f = [] {
    const char* e = getenv("NSA_EW_NT");
    return !(e && e[0] == '0') ? 1 : 0;
  }();
  return f;
}
static bool ew_nt() { return ew_nt_flag() != 0; }

// set the streaming-store policy of the elementwise kernels (on < 0: keep); returns the old one
NSA_API int nsa_ew_set_nt(int on) {
  const int prev = ew_nt_flag();
  if (on >= 0) ew_nt_flag() = on ? 1 : 0;
  return prev;
}

template <bool H>
static hipError_t gelu_fwd_entry(const void* x, void* y, int64_t n, hipStream_t s) {
  if (ew_nt() && n * 2 >= NSA_NT_MIN_BYTES)
    gelu_fwd_kernel<true, H><<<grid_for(n / 8), kBlock, 0, s>>>((const bf16_t*)x, (bf16_t*)y, n);
  else
    gelu_fwd_kernel<false, H><<<grid_for(n / 8), kBlock, 0, s>>>((const bf16_t*)x, (bf16_t*)y, n);
  NSA_LAUNCH_CHECK();
}
template <bool H>
static hipError_t gelu_bwd_entry(const void* dy, const void* x, void* dx, int64_t n, hipStream_t s) {
  if (ew_nt() && n * 2 >= NSA_NT_MIN_BYTES)
    gelu_bwd_kernel<true, H><<<grid_for(n / 8), kBlock, 0, s>>>((const bf16_t*)dy, (const bf16_t*)x, (bf16_t*)dx, n);
  else
    gelu_bwd_kernel<false, H><<<grid_for(n / 8), kBlock, 0, s>>>((const bf16_t*)dy, (const bf16_t*)x, (bf16_t*)dx,
                                                                  n);
  NSA_LAUNCH_CHECK();
}
NSA_API hipError_t nsa_gelu_fwd(const void* x, void* y, int64_t n, hipStream_t s) {
  return gelu_fwd_entry<false>(x, y, n, s);
}
NSA_API hipError_t nsa_gelu_bwd(const void* dy, const void* x, void* dx, int64_t n, hipStream_t s) {
  return gelu_bwd_entry<false>(dy, x, dx, n, s);
}
NSA_API hipError_t nsa_gelu_fwd_h(const void* x, void* y, int64_t n, hipStream_t s) {
  return gelu_fwd_entry<true>(x, y, n, s);
}
NSA_API hipError_t nsa_gelu_bwd_h(const void* dy, const void* x, void* dx, int64_t n, hipStream_t s) {
  return gelu_bwd_entry<true>(dy, x, dx, n, s);
}

NSA_DEFINE_RNG_ADVANCE(nsa_rng_advance_ew)
NSA_API hipError_t nsa_rng_advance_emb(hipStream_t s);
NSA_API hipError_t nsa_rng_advance_attn(hipStream_t s);
NSA_API hipError_t nsa_rng_advance_emb_set(uint64_t v, hipStream_t s);
NSA_API hipError_t nsa_rng_advance_attn_set(uint64_t v, hipStream_t s);
NSA_API hipError_t nsa_rng_advance_attn_h(hipStream_t s);  // the fp16 attention build's counter
NSA_API hipError_t nsa_rng_advance_attn_h_set(uint64_t v, hipStream_t s);
NSA_API hipError_t nsa_rng_advance_ln(hipStream_t s);  // the LayerNorm's fused branch dropout
NSA_API hipError_t nsa_rng_advance_ln_set(uint64_t v, hipStream_t s);

// set every translation unit's dropout step counter (start of a run)
NSA_API hipError_t nsa_rng_set(uint64_t v, hipStream_t s) {
  hipError_t e = nsa_rng_advance_ew_set(v, s);
  if (e == hipSuccess) e = nsa_rng_advance_emb_set(v, s);
  if (e == hipSuccess) e = nsa_rng_advance_attn_set(v, s);
  if (e == hipSuccess) e = nsa_rng_advance_attn_h_set(v, s);
  if (e == hipSuccess) e = nsa_rng_advance_ln_set(v, s);
  return e;
}

// one micro-step's dropout counter bump in every translation unit (see common.h)
NSA_API hipError_t nsa_rng_advance(hipStream_t s) {
  hipError_t e = nsa_rng_advance_ew(s);
  if (e == hipSuccess) e = nsa_rng_advance_emb(s);
  if (e == hipSuccess) e = nsa_rng_advance_attn(s);
  if (e == hipSuccess) e = nsa_rng_advance_attn_h(s);
  if (e == hipSuccess) e = nsa_rng_advance_ln(s);
  return e;
}

NSA_API hipError_t nsa_dropout(const void* x, void* y, int64_t n, float p, uint64_t seed, hipStream_t s) {
  const float scale = p < 1.0f ? 1.0f / (1.0f - p) : 0.0f;
  dropout_kernel<false><<<grid_for(n / 8), kBlock, 0, s>>>((const bf16_t*)x, (bf16_t*)y, n, nsa_drop_thresh(p), scale,
                                                           seed);
  NSA_LAUNCH_CHECK();
}
NSA_API hipError_t nsa_dropout_h(const void* x, void* y, int64_t n, float p, uint64_t seed, hipStream_t s) {
  const float scale = p < 1.0f ? 1.0f / (1.0f - p) : 0.0f;
  dropout_kernel<true><<<grid_for(n / 8), kBlock, 0, s>>>((const bf16_t*)x, (bf16_t*)y, n, nsa_drop_thresh(p), scale,
                                                          seed);
  NSA_LAUNCH_CHECK();
}

NSA_API hipError_t nsa_splitk_reduce(const void* ws, void* out, int64_t n, int splits, hipStream_t s) {
  splitk_reduce_kernel<<<grid_for(n / 4 + 1), kBlock, 0, s>>>((const float*)ws, (float*)out, n, splits);
  return hipGetLastError();
}

NSA_API hipError_t nsa_transpose_bf16(const void* src, void* dst, int R, int C, hipStream_t s) {
  if (R % 64 || C % 64) return hipErrorInvalidValue;
  const int64_t regions = (int64_t)(R / 64) * (C / 64);
  transpose_bf16_kernel<<<(unsigned)((regions + 3) / 4), 256, 0, s>>>((const bf16_t*)src, (bf16_t*)dst, R, C);
  return hipGetLastError();
}

NSA_API hipError_t nsa_cast_f32_bf16(const void* x, void* y, int64_t n, hipStream_t s) {
  cast_f32_bf16_kernel<false><<<grid_for(n / 8), kBlock, 0, s>>>((const float*)x, (bf16_t*)y, n);
  NSA_LAUNCH_CHECK();
}
NSA_API hipError_t nsa_cast_f32_bf16_h(const void* x, void* y, int64_t n, hipStream_t s) {  // fp32 -> fp16
  cast_f32_bf16_kernel<true><<<grid_for(n / 8), kBlock, 0, s>>>((const float*)x, (bf16_t*)y, n);
  NSA_LAUNCH_CHECK();
}

NSA_API hipError_t nsa_scale_rows_bf16(const void* x, void* y, const void* scale, int64_t n, hipStream_t s) {
  scale_bf16_kernel<false><<<grid_for(n / 8), kBlock, 0, s>>>((const bf16_t*)x, (bf16_t*)y, (const float*)scale, n);
  NSA_LAUNCH_CHECK();
}
NSA_API hipError_t nsa_scale_rows_bf16_h(const void* x, void* y, const void* scale, int64_t n, hipStream_t s) {
  scale_bf16_kernel<true><<<grid_for(n / 8), kBlock, 0, s>>>((const bf16_t*)x, (bf16_t*)y, (const float*)scale, n);
  NSA_LAUNCH_CHECK();
}
