// Shared helpers for the gfx950 (MI355X / CDNA4) kernel library.
//
// Conventions used by every kernel in this directory:
//  * bf16 tensors are stored as raw 16-bit words (bf16_t) and moved in 16-byte
//    vectors (8 elements per lane) — hipcc does not vectorise scalar bf16 loads
//    (cdna_hip_programming.md Guideline 13);
//  * math is fp32; f32 -> bf16 uses the compiler cast, which lowers to
//    v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN-preserving);
//  * waves are 64 lanes; block sizes are multiples of 64;
//  * every launch takes the caller's hipStream_t and returns hipError_t.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define NSA_API extern "C" __attribute__((visibility("default")))

#define NSA_LAUNCH_CHECK() \
  do {                     \
    return hipGetLastError(); \
  } while (0)

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

// 8 x bf16 in one 16-byte vector
struct __attribute__((aligned(16))) bf16v8 {
  bf16_t v[8];
};

__device__ __forceinline__ void unpack8(uint4 u, float (&f)[8]) {
  f[0] = __uint_as_float(u.x << 16);
  f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16);
  f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16);
  f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16);
  f[7] = __uint_as_float(u.w & 0xffff0000u);
}

__device__ __forceinline__ void load8(const bf16_t* p, float (&f)[8]) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  f[0] = __uint_as_float(u.x << 16);
  f[1] = __uint_as_float(u.x & 0xffff0000u);
  f[2] = __uint_as_float(u.y << 16);
  f[3] = __uint_as_float(u.y & 0xffff0000u);
  f[4] = __uint_as_float(u.z << 16);
  f[5] = __uint_as_float(u.z & 0xffff0000u);
  f[6] = __uint_as_float(u.w << 16);
  f[7] = __uint_as_float(u.w & 0xffff0000u);
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

__device__ __forceinline__ void store8(bf16_t* p, const float (&f)[8]) {
  uint4 u;
  u.x = pack2(f[0], f[1]);
  u.y = pack2(f[2], f[3]);
  u.z = pack2(f[4], f[5]);
  u.w = pack2(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = u;
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

// Counter-based dropout RNG: keep(seed, i) is a pure function of (seed, index),
// so backward regenerates the forward mask without storing it.
__device__ __forceinline__ uint32_t nsa_hash(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

__device__ __forceinline__ bool nsa_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
  return nsa_hash(seed, idx) >= thresh;
}

// Graph-safe dropout RNG.  The host passes each dropout call site a salt (drawn from
// torch's CPU generator, so activation checkpointing replays it); kernels mix in a
// device-side step counter that nsa_rng_advance() bumps once per micro-step from
// inside the stream.  A captured HIP graph bakes the salts but replays the counter
// increment, so every replayed micro-step draws fresh masks, and forward / backward
// / recompute of one micro-step see the same counter.  Each translation unit has
// its own copy of the counter (no relocatable device code); nsa_rng_advance bumps
// all of them in lockstep.
static __device__ uint64_t nsa_rng_step = 0;

__device__ __forceinline__ uint64_t nsa_seed(uint64_t salt) {
  return salt ^ (nsa_rng_step * 0xD1B54A32D192ED03ull);
}

// NAME(stream) bumps this TU's counter; NAME##_set(value, stream) sets it (a new run
// restarts its dropout stream at 0, independent of earlier runs in the process)
#define NSA_DEFINE_RNG_ADVANCE(NAME)                                                       \
  __global__ void NAME##_kernel() { nsa_rng_step += 1; }                                   \
  __global__ void NAME##_set_kernel(uint64_t v) { nsa_rng_step = v; }                      \
  NSA_API hipError_t NAME(hipStream_t s) {                                                 \
    NAME##_kernel<<<1, 1, 0, s>>>();                                                        \
    return hipGetLastError();                                                              \
  }                                                                                        \
  NSA_API hipError_t NAME##_set(uint64_t v, hipStream_t s) {                               \
    NAME##_set_kernel<<<1, 1, 0, s>>>(v);                                                   \
    return hipGetLastError();                                                              \
  }

static inline uint32_t nsa_drop_thresh(float p) {
  double t = (double)p * 4294967296.0;
  if (t >= 4294967295.0) return 0xffffffffu;
  if (t <= 0.0) return 0u;
  return (uint32_t)t;
}

// GELU (exact-erf form of nn.GELU) with a fast erf: Abramowitz & Stegun 7.1.26
// (|error| < 1.5e-7, far below one bf16 ulp), sharing one exp between erf and
// the normal pdf:  with z = x/sqrt(2), exp(-z^2) = exp(-x^2/2) = sqrt(2 pi) pdf(x).
__device__ __forceinline__ void nsa_gelu_cdf_pdf(float x, float& cdf, float& pdf) {
  const float z = fabsf(x) * 0.70710678118654752f;
  // v_rcp_f32 (1 ulp) — __frcp_rn lowers to a full IEEE division sequence here
  // (v_div_scale x2 / v_div_fmas / v_div_fixup), which made the GELU forward VALU-bound
  const float t = __builtin_amdgcn_rcpf(1.0f + 0.3275911f * z);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float e = __expf(-z * z);
  const float erf_abs = 1.0f - poly * e;
  const float erf_z = x < 0.0f ? -erf_abs : erf_abs;
  cdf = 0.5f * (1.0f + erf_z);
  pdf = e * 0.39894228040143268f;
}

__device__ __forceinline__ float nsa_gelu(float x) {
  float c, p;
  nsa_gelu_cdf_pdf(x, c, p);
  return x * c;
}

__device__ __forceinline__ float nsa_gelu_grad(float x) {
  float c, p;
  nsa_gelu_cdf_pdf(x, c, p);
  return c + x * p;
}

// The same GELU on two values at once: the non-transcendental arithmetic as packed-f32
// VALU (v_pk_fma_f32 / v_pk_mul_f32, two lanes' worth per instruction), v_rcp_f32 and
// v_exp_f32 per element.  For the GEMM epilogues, where one wave per SIMD runs the GELU of
// a 256 x 256 tile with no MFMA beside it.
typedef float nsa_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void nsa_gelu_cdf_pdf2(nsa_f32x2 x, nsa_f32x2& cdf, nsa_f32x2& pdf) {
  const nsa_f32x2 z = nsa_f32x2{fabsf(x.x), fabsf(x.y)} * 0.70710678118654752f;
  const nsa_f32x2 d = 1.0f + 0.3275911f * z;
  const nsa_f32x2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  const nsa_f32x2 poly =
      t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const nsa_f32x2 y = z * z * -1.4426950408889634f;  // exp(-z^2) = 2^(-z^2 log2 e)
  const nsa_f32x2 e = {__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
  const nsa_f32x2 erf_abs = 1.0f - poly * e;
  const nsa_f32x2 erf_z = {__builtin_copysignf(erf_abs.x, x.x), __builtin_copysignf(erf_abs.y, x.y)};
  cdf = 0.5f + 0.5f * erf_z;
  pdf = e * 0.39894228040143268f;
}
__device__ __forceinline__ nsa_f32x2 nsa_gelu2(nsa_f32x2 x) {
  nsa_f32x2 c, p;
  nsa_gelu_cdf_pdf2(x, c, p);
  return x * c;
}
__device__ __forceinline__ nsa_f32x2 nsa_gelu_grad2(nsa_f32x2 x) {
  nsa_f32x2 c, p;
  nsa_gelu_cdf_pdf2(x, c, p);
  return c + x * p;
}
// gelu(x) and gelu'(x) from one erf / pdf evaluation (the c_fc GELU epilogue stores gelu'(u)
// for the backward instead of u: see gemm_nt4.hip Q_EPI_GELU)
__device__ __forceinline__ void nsa_gelu_and_grad2(nsa_f32x2 x, nsa_f32x2& g, nsa_f32x2& gp) {
  nsa_f32x2 c, p;
  nsa_gelu_cdf_pdf2(x, c, p);
  g = x * c;
  gp = c + x * p;
}

// fp16 pairs (gelu'(u) is stored as fp16: 2^-11 relative rounding, 4x finer than bf16)
typedef _Float16 nsa_f16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t nsa_pk_f16(float a, float b) {  // v_cvt_pk_f16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((nsa_f32x2{a, b}), nsa_f16x2));
}
__device__ __forceinline__ nsa_f32x2 nsa_unpk_f16(uint32_t u) {
  return __builtin_convertvector(__builtin_bit_cast(nsa_f16x2, u), nsa_f32x2);
}
__device__ __forceinline__ float nsa_h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t nsa_f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

// ---------------------------------------------------------------------------------------
// 16-bit element types.  The training kernels take a compile-time H: false = bf16 (the
// default compute dtype), true = fp16 (nanoGPT's dtype='float16' with a dynamic loss scale).
// Both are stored as raw 16-bit words (bf16_t) and moved in the same vectors; only the
// conversions and the MFMA opcode differ (gfx950's fp16 MFMAs run at the bf16 rate).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <bool H>
__device__ __forceinline__ float e2f(uint16_t v) {
  if constexpr (H) return (float)__builtin_bit_cast(_Float16, v);
  else return __uint_as_float(((uint32_t)v) << 16);
}
template <bool H>
__device__ __forceinline__ uint16_t f2e(float f) {
  if constexpr (H) return __builtin_bit_cast(uint16_t, (_Float16)f);
  else return f2bf(f);
}
// the low / high element of a packed pair
template <bool H>
__device__ __forceinline__ float lo2f(uint32_t w) {
  if constexpr (H) return (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xffffu));
  else return __uint_as_float(w << 16);
}
template <bool H>
__device__ __forceinline__ float hi2f(uint32_t w) {
  if constexpr (H) return (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
  else return __uint_as_float(w & 0xffff0000u);
}
// two f32 -> one dword of two elements (v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32, RNE)
template <bool H>
__device__ __forceinline__ uint32_t pk2(float lo, float hi) {
  typedef float f2_t __attribute__((ext_vector_type(2)));
  if constexpr (H) {
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2_t{lo, hi}), h2_t));
  } else {
    typedef __bf16 b2_t __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2_t{lo, hi}), b2_t));
  }
}
template <bool H>
__device__ __forceinline__ void unpack8e(uint4 u, float (&f)[8]) {
  f[0] = lo2f<H>(u.x);
  f[1] = hi2f<H>(u.x);
  f[2] = lo2f<H>(u.y);
  f[3] = hi2f<H>(u.y);
  f[4] = lo2f<H>(u.z);
  f[5] = hi2f<H>(u.z);
  f[6] = lo2f<H>(u.w);
  f[7] = hi2f<H>(u.w);
}
template <bool H>
__device__ __forceinline__ void load8e(const bf16_t* p, float (&f)[8]) {
  unpack8e<H>(*reinterpret_cast<const uint4*>(p), f);
}
template <bool H>
__device__ __forceinline__ void store8e(bf16_t* p, const float (&f)[8]) {
  uint4 u;
  u.x = pk2<H>(f[0], f[1]);
  u.y = pk2<H>(f[2], f[3]);
  u.z = pk2<H>(f[4], f[5]);
  u.w = pk2<H>(f[6], f[7]);
  *reinterpret_cast<uint4*>(p) = u;
}
// one scalar f32 -> element (the value a cast to the element type gives)
template <bool H>
__device__ __forceinline__ __bf16 f2frag(float f) {
  return __builtin_bit_cast(__bf16, f2e<H>(f));
}
// MFMAs on 8-element fragments held in bf16x8 containers (the bits of either type)
template <bool H>
__device__ __forceinline__ f32x16 mfma32e(bf16x8 a, bf16x8 b, f32x16 c) {
  if constexpr (H)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <bool H>
__device__ __forceinline__ f32x4 mfma16e(bf16x8 a, bf16x8 b, f32x4 c) {
  if constexpr (H)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
                                                  0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// Nontemporal streams only pay for tensors larger than the 256 MB Infinity Cache: a smaller
// one can stay cache-resident for its next reader (shakespeare_char config, 25 MB LayerNorm
// rows: 4.78 ms/iter with nontemporal streams everywhere, 4.72-4.76 gated).  Streams of at
// least this many bytes use them.
#ifndef NSA_NT_MIN_BYTES
#define NSA_NT_MIN_BYTES (256LL << 20)
#endif

