// Cross-entropy fused into the tied lm_head GEMMs (SURVEY.md §2.7 K8 + K10; nanoGPT
// F.cross_entropy(logits, targets, ignore_index=-1) with a mean over the valid rows).
//
// The logits [M, V] are never stored.  With c_r = the target logit of row r (computed here
// first, a gather-dot), the forward GEMM's epilogue (gemm_nt4.hip, EPI_XENT) writes
// E = exp(logit - c_r) in bf16 plus per-half-tile row sums; then
//   S_r = sum_v E[r, v] = exp(lse_r - c_r)   ->   loss_r = log S_r,  softmax = E / S_r.
// Backward, with g = upstream gradient / valid rows:
//   dX = g (E · W / S - W[t])                  (gemm_nt4 EPI_XDX: fp32 subtraction, one rounding)
//   dW = E^T · (g x / S) - g sum_{r: t_r = v} x_r   (the four-wave weight-grad GEMM on E, then
//        nsa_xent_dw_fix: the onehot part as fp32 atomics, with the bf16 rounding of the
//        target entry's product taken back out, so p_t - 1 keeps fp32 precision).
// Rows whose S leaves [0.5, 1e30] (a per-token loss beyond ~69 nats, or a target logit far
// from the GEMM's) are recomputed exactly by nsa_xent_fixup (normally none: the kernel exits).
#include "common.h"
#include "segsum.h"

namespace {

// c_r = x_r · W[t_r] (fp32 from bf16), t32_r = t_r (or -1 when ignored / out of range): one
// wave per row, 16-byte loads
// H: fp16 x / W / E (dtype float16); shift: added to c (fp16 E range, see nsa_gemm_nt4_xent_h)
template <bool H>
__global__ __launch_bounds__(256) void xent_tlogit_kernel(const bf16_t* __restrict__ x, int ldx,
                                                          const bf16_t* __restrict__ W, int ldw,
                                                          const int64_t* __restrict__ tgt, float* __restrict__ crow,
                                                          int* __restrict__ t32, int M, int C, int V, float shift) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const int64_t t = tgt[row];
  const bool valid = t >= 0 && t < V;
  float s = 0.0f;
  if (valid) {
    const bf16_t* xr = x + (int64_t)row * ldx;
    const bf16_t* wr = W + t * ldw;
    for (int c = lane * 8; c < C; c += 512) {
      float a[8], b[8];
      load8e<H>(xr + c, a);
      load8e<H>(wr + c, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) s = __builtin_fmaf(a[j], b[j], s);
    }
    s = wave_sum(s);
  }
  if (lane == 0) {
    crow[row] = s + shift;
    t32[row] = valid ? (int)t : -1;
  }
}

// S_r = sum of the GEMM epilogue's partials; loss_r = log S_r, invS_r = 1 / S_r (0 and 0 for
// an ignored row); rows outside [0.5, 1e30] go on the fix-up list (ignored rows above 1e30 too)
// [lo, hi]: the range of S kept (bf16 E: [0.5, 1e30]; fp16 E, shifted: [0.5 e^-shift, 6e4]);
// loss = log S + shift
__global__ __launch_bounds__(256) void xent_combine_kernel(const float* __restrict__ part, int slots,
                                                           const int* __restrict__ t32, float* __restrict__ loss,
                                                           float* __restrict__ invS, int* __restrict__ nfix,
                                                           int* __restrict__ fixlist, int M, float lo, float hi,
                                                           float shift) {
  const int row = blockIdx.x * 256 + threadIdx.x;
  if (row >= M) return;
  // 8 independent loads in flight per thread (the slot loop was one dependent chain of
  // ~400 load-adds per row at GPT-2's 394 slots: 154 us for 194 MB)
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 8 <= slots; k += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += part[(int64_t)(k + u) * M + row];
  }
  for (; k < slots; ++k) acc[0] += part[(int64_t)k * M + row];
  const float S = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  if (t32[row] < 0) {
    loss[row] = 0.0f;
    invS[row] = 0.0f;
    // an ignored row is scaled by 0 in both backward GEMMs, which an overflowed E (inf, with
    // the shift c = 0: any logit above ~88) would turn into NaN: the fix-up zeroes its E row
    if (!(S <= hi)) fixlist[atomicAdd(nfix, 1)] = row;
    return;
  }
  if (!(S >= lo && S <= hi)) {  // also catches NaN / inf
    fixlist[atomicAdd(nfix, 1)] = row;
    loss[row] = 0.0f;
    invS[row] = 0.0f;
    return;
  }
  loss[row] = __logf(S) + shift;
  invS[row] = 1.0f / S;
}

// Exact recompute of a flagged row: logits l_v = x_r · W_v (fp32), m = max, E = exp(l - m),
// S = sum E, loss = m + log S - l_t (a flagged ignored row: E = 0).  One workgroup per listed row (grid-stride over the
// device-side count: with no flagged row every workgroup exits at once).
// Grid of the fix-up: every workgroup reads the device count and exits when it has no row, so
// an empty list costs one short launch whatever the grid.  1024 (4 per CU, 33 KB of LDS each)
// rather than round 5's 64: fp16 E flags every row whose largest logit passes its target's
// by ~11 nats, a share that grows as a model trains, and each flagged row costs two V x C
// passes (profiles/r6_xent_f16_cliff.md)
#ifndef NSA_XENT_FIX_GRID
#define NSA_XENT_FIX_GRID 1024
#endif
template <bool H>
__global__ __launch_bounds__(256) void xent_fixup_kernel(const bf16_t* __restrict__ x, int ldx,
                                                         const bf16_t* __restrict__ W, int ldw, bf16_t* __restrict__ E,
                                                         int lde, const int* __restrict__ t32,
                                                         const int* __restrict__ nfix, const int* __restrict__ fixlist,
                                                         float* __restrict__ loss, float* __restrict__ invS, int C,
                                                         int V, int Vpad) {
  __shared__ float xs[8192];
  __shared__ float red[2][4];
  const int n = *nfix;
  for (int f = blockIdx.x; f < n; f += gridDim.x) {
    const int row = fixlist[f];
    __syncthreads();
    if (t32[row] < 0) {  // ignored row (workgroup-uniform): E = 0, loss and 1/S stay 0
      for (int v = threadIdx.x * 8; v < Vpad; v += 256 * 8)
        *reinterpret_cast<uint4*>(E + (int64_t)row * lde + v) = make_uint4(0u, 0u, 0u, 0u);
      continue;
    }
    for (int c = threadIdx.x; c < C; c += 256) xs[c] = e2f<H>(x[(int64_t)row * ldx + c]);
    __syncthreads();
    auto logit = [&](int v) {
      const bf16_t* wr = W + (int64_t)v * ldw;
      float s = 0.0f;
      for (int c = 0; c < C; c += 8) {
        float b[8];
        load8e<H>(wr + c, b);
#pragma unroll
        for (int j = 0; j < 8; ++j) s = __builtin_fmaf(xs[c + j], b[j], s);
      }
      return s;
    };
    float m = -INFINITY;
    for (int v = threadIdx.x; v < V; v += 256) m = fmaxf(m, logit(v));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[0][threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
    float s = 0.0f;
    for (int v = threadIdx.x; v < Vpad; v += 256) {
      const float e = v < V ? __expf(logit(v) - m) : 0.0f;
      E[(int64_t)row * lde + v] = f2e<H>(e);
      s += e;
    }
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[1][threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float S = red[1][0] + red[1][1] + red[1][2] + red[1][3];
      loss[row] = m + __logf(S) - logit(t32[row]);
      invS[row] = 1.0f / S;
    }
  }
}

// Backward prologue, per row: coefficient pair {g / S, g} (0, 0 ignored), the row W[t] gathered
// for the dX epilogue, and xs = bf16(x g / S) for the weight-gradient GEMM
template <bool H>
__global__ __launch_bounds__(256) void xent_bwd_prep_kernel(const bf16_t* __restrict__ x, int ldx,
                                                            const bf16_t* __restrict__ W, int ldw,
                                                            const int* __restrict__ t32, const float* __restrict__ invS,
                                                            const float* __restrict__ gsc, float* __restrict__ coef,
                                                            bf16_t* __restrict__ wrows, bf16_t* __restrict__ xs, int M,
                                                            int C) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const float g = *gsc;
  const int t = t32[row];
  const float sc = g * invS[row];
  if (lane == 0) {
    coef[2 * row] = sc;
    coef[2 * row + 1] = t < 0 ? 0.0f : g;
  }
  const bf16_t* wr = W + (int64_t)(t < 0 ? 0 : t) * ldw;
  const bf16_t* xr = x + (int64_t)row * ldx;
  for (int c = lane * 8; c < C; c += 512) {
    *reinterpret_cast<uint4*>(wrows + (int64_t)row * C + c) = *reinterpret_cast<const uint4*>(wr + c);
    float a[8];
    load8e<H>(xr + c, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] *= sc;
    store8e<H>(xs + (int64_t)row * C + c, a);
  }
}

// The onehot part of dW, per valid row r with target t:  gW[t] += E[r,t] (s x_r - bf16(s x_r))
// - g x_r  (s = g / S): subtracts g x_r and takes back the rounding the GEMM's bf16 operand
// put on the target entry's product.  fp32 atomics, one wave per row.
template <bool H>
__global__ __launch_bounds__(256) void xent_dw_fix_kernel(const bf16_t* __restrict__ x, int ldx,
                                                          const bf16_t* __restrict__ E, int lde,
                                                          const int* __restrict__ t32, const float* __restrict__ invS,
                                                          const float* __restrict__ gsc, float* __restrict__ gW,
                                                          int ldg, int M, int C) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= M) return;
  const int t = t32[row];
  if (t < 0) return;
  const float g = *gsc;
  const float s = g * invS[row];
  const float et = e2f<H>(E[(int64_t)row * lde + t]);
  const bf16_t* xr = x + (int64_t)row * ldx;
  float* gr = gW + (int64_t)t * ldg;
  // one column per lane per step: every atomic wave-instruction covers 256 contiguous
  // bytes of the target row (the full atomic rate; 8 columns per lane spread one
  // instruction over 2 KB and ran ~9x slower: 2.56 ms per micro-step at 122880 rows)
  for (int c = lane; c < C; c += 64) {
    const float a = e2f<H>(xr[c]);
    const float p = s * a;
    const float pr = e2f<H>(f2e<H>(p));
    atomicAdd(gr + c, et * (p - pr) - g * a);
  }
}

// The same onehot term without atomics: the valid rows stably sorted by target (segsum.h;
// the fp32 atomics above contend on the few rows of a small vocabulary and run at the chip's
// atomic rate on GPT-2's)
template <bool H>
struct XentFixRow {
  const bf16_t* x;
  int ldx;
  const bf16_t* E;
  int lde;
  const int* t32;
  const float* invS;
  const float* gsc;
  // t = the row's target (the destination id): no dependent load of t32
  __device__ __forceinline__ void load(int64_t row, int64_t t, int c, float (&f)[8]) const {
    const float g = *gsc;
    const float s = g * invS[row];
    const float et = e2f<H>(E[row * lde + t]);
    float a[8];
    load8e<H>(x + row * ldx + c, a);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float p = s * a[j];
      f[j] = et * (p - e2f<H>(f2e<H>(p))) - g * a[j];
    }
  }
};

}  // namespace

namespace {
template <bool H>
hipError_t tlogit_entry(const void* x, int ldx, const void* W, int ldw, const void* tgt, void* crow, void* t32, int M,
                        int C, int V, float shift, hipStream_t s) {
  if (C % 8 || ldx % 8 || ldw % 8) return hipErrorInvalidValue;
  xent_tlogit_kernel<H><<<(M + 3) / 4, 256, 0, s>>>((const bf16_t*)x, ldx, (const bf16_t*)W, ldw,
                                                    (const int64_t*)tgt, (float*)crow, (int*)t32, M, C, V, shift);
  return hipGetLastError();
}
template <bool H>
hipError_t fixup_entry(const void* x, int ldx, const void* W, int ldw, void* E, int lde, const void* t32,
                       const void* nfix, const void* fixlist, void* loss, void* invS, int C, int V, int Vpad,
                       hipStream_t s) {
  if (C > 8192 || C % 8 || ldw % 8 || Vpad % 8 || lde % 8) return hipErrorInvalidValue;
  xent_fixup_kernel<H><<<NSA_XENT_FIX_GRID, 256, 0, s>>>((const bf16_t*)x, ldx, (const bf16_t*)W, ldw, (bf16_t*)E, lde,
                                          (const int*)t32, (const int*)nfix, (const int*)fixlist, (float*)loss,
                                          (float*)invS, C, V, Vpad);
  return hipGetLastError();
}
template <bool H>
hipError_t bwd_prep_entry(const void* x, int ldx, const void* W, int ldw, const void* t32, const void* invS,
                          const void* gsc, void* coef, void* wrows, void* xs, int M, int C, hipStream_t s) {
  if (C % 8 || ldx % 8 || ldw % 8) return hipErrorInvalidValue;
  xent_bwd_prep_kernel<H><<<(M + 3) / 4, 256, 0, s>>>((const bf16_t*)x, ldx, (const bf16_t*)W, ldw, (const int*)t32,
                                                      (const float*)invS, (const float*)gsc, (float*)coef,
                                                      (bf16_t*)wrows, (bf16_t*)xs, M, C);
  return hipGetLastError();
}
template <bool H>
hipError_t dw_fix_entry(const void* x, int ldx, const void* E, int lde, const void* t32, const void* invS,
                        const void* gsc, void* gW, int ldg, int M, int C, hipStream_t s) {
  xent_dw_fix_kernel<H><<<(M + 3) / 4, 256, 0, s>>>((const bf16_t*)x, ldx, (const bf16_t*)E, lde, (const int*)t32,
                                                    (const float*)invS, (const float*)gsc, (float*)gW, ldg, M, C);
  return hipGetLastError();
}
template <bool H>
hipError_t dw_fix_sorted_entry(const void* x, int ldx, const void* E, int lde, const void* t32, const void* invS,
                               const void* gsc, const void* ids, const void* order, const void* seg, void* part,
                               void* gW, int ldg, int M, int C, int V, hipStream_t s) {
  if (C % 8 || ldx % 8) return hipErrorInvalidValue;
  const XentFixRow<H> f{(const bf16_t*)x, ldx, (const bf16_t*)E, lde, (const int*)t32, (const float*)invS,
                        (const float*)gsc};
  return seg_scatter_add<int, XentFixRow<H>>((const int*)ids, (const int64_t*)order, (const int64_t*)seg,
                                             (float*)part, f, (float*)gW, ldg, M, V, C, s);
}
}  // namespace

// the onehot dW term for a small vocabulary (V x C fp32 <= 128 KB): LDS-privatised
// scatter-add over the unsorted targets (segsum.h seg_lds_kernel)
NSA_API hipError_t nsa_xent_dw_fix_lds(const void* x, int ldx, const void* E, int lde, const void* t32,
                                       const void* invS, const void* gsc, void* part, void* gW, int ldg, int M, int C, int V,
                                       hipStream_t s) {
  if (C % 8 || ldx % 8) return hipErrorInvalidValue;
  const XentFixRow<false> f{(const bf16_t*)x, ldx, (const bf16_t*)E, lde, (const int*)t32, (const float*)invS,
                            (const float*)gsc};
  return seg_scatter_add_lds<int, XentFixRow<false>>((const int*)t32, f, (float*)part, (float*)gW, ldg, M, V, C, s);
}
NSA_API hipError_t nsa_xent_dw_fix_lds_h(const void* x, int ldx, const void* E, int lde, const void* t32,
                                         const void* invS, const void* gsc, void* part, void* gW, int ldg, int M, int C, int V,
                                         hipStream_t s) {
  if (C % 8 || ldx % 8) return hipErrorInvalidValue;
  const XentFixRow<true> f{(const bf16_t*)x, ldx, (const bf16_t*)E, lde, (const int*)t32, (const float*)invS,
                           (const float*)gsc};
  return seg_scatter_add_lds<int, XentFixRow<true>>((const int*)t32, f, (float*)part, (float*)gW, ldg, M, V, C, s);
}

// the onehot dW term, atomic-free: ids = t32 stably sorted (int32), order = their rows,
// seg[V + 1] = segment starts, part = [2 * ceil(M / 16), C] fp32 workspace (segsum.h)
NSA_API hipError_t nsa_xent_dw_fix_sorted(const void* x, int ldx, const void* E, int lde, const void* t32,
                                          const void* invS, const void* gsc, const void* ids, const void* order,
                                          const void* seg, void* part, void* gW, int ldg, int M, int C, int V,
                                          hipStream_t s) {
  return dw_fix_sorted_entry<false>(x, ldx, E, lde, t32, invS, gsc, ids, order, seg, part, gW, ldg, M, C, V, s);
}
NSA_API hipError_t nsa_xent_dw_fix_sorted_h(const void* x, int ldx, const void* E, int lde, const void* t32,
                                            const void* invS, const void* gsc, const void* ids, const void* order,
                                            const void* seg, void* part, void* gW, int ldg, int M, int C, int V,
                                            hipStream_t s) {
  return dw_fix_sorted_entry<true>(x, ldx, E, lde, t32, invS, gsc, ids, order, seg, part, gW, ldg, M, C, V, s);
}

// c = the target logit (+ shift; 0 for bf16 E), t32 = the target or -1 (ignored / out of range)
NSA_API hipError_t nsa_xent_tlogit(const void* x, int ldx, const void* W, int ldw, const void* tgt, void* crow,
                                   void* t32, int M, int C, int V, float shift, hipStream_t s) {
  return tlogit_entry<false>(x, ldx, W, ldw, tgt, crow, t32, M, C, V, shift, s);
}
NSA_API hipError_t nsa_xent_tlogit_h(const void* x, int ldx, const void* W, int ldw, const void* tgt, void* crow,
                                     void* t32, int M, int C, int V, float shift, hipStream_t s) {
  return tlogit_entry<true>(x, ldx, W, ldw, tgt, crow, t32, M, C, V, shift, s);
}

// nfix must be zeroed by the caller before this launch (it is a stream-ordered counter).
// Rows with S outside [lo, hi] go on the fix-up list; loss = log S + shift.
NSA_API hipError_t nsa_xent_combine(const void* part, int slots, const void* t32, void* loss, void* invS, void* nfix,
                                    void* fixlist, int M, float lo, float hi, float shift, hipStream_t s) {
  xent_combine_kernel<<<(M + 255) / 256, 256, 0, s>>>((const float*)part, slots, (const int*)t32, (float*)loss,
                                                      (float*)invS, (int*)nfix, (int*)fixlist, M, lo, hi, shift);
  return hipGetLastError();
}

NSA_API hipError_t nsa_xent_fixup(const void* x, int ldx, const void* W, int ldw, void* E, int lde, const void* t32,
                                  const void* nfix, const void* fixlist, void* loss, void* invS, int C, int V,
                                  int Vpad, hipStream_t s) {
  return fixup_entry<false>(x, ldx, W, ldw, E, lde, t32, nfix, fixlist, loss, invS, C, V, Vpad, s);
}
NSA_API hipError_t nsa_xent_fixup_h(const void* x, int ldx, const void* W, int ldw, void* E, int lde, const void* t32,
                                    const void* nfix, const void* fixlist, void* loss, void* invS, int C, int V,
                                    int Vpad, hipStream_t s) {
  return fixup_entry<true>(x, ldx, W, ldw, E, lde, t32, nfix, fixlist, loss, invS, C, V, Vpad, s);
}

NSA_API hipError_t nsa_xent_bwd_prep(const void* x, int ldx, const void* W, int ldw, const void* t32,
                                     const void* invS, const void* gsc, void* coef, void* wrows, void* xs, int M,
                                     int C, hipStream_t s) {
  return bwd_prep_entry<false>(x, ldx, W, ldw, t32, invS, gsc, coef, wrows, xs, M, C, s);
}
NSA_API hipError_t nsa_xent_bwd_prep_h(const void* x, int ldx, const void* W, int ldw, const void* t32,
                                       const void* invS, const void* gsc, void* coef, void* wrows, void* xs, int M,
                                       int C, hipStream_t s) {
  return bwd_prep_entry<true>(x, ldx, W, ldw, t32, invS, gsc, coef, wrows, xs, M, C, s);
}

NSA_API hipError_t nsa_xent_dw_fix(const void* x, int ldx, const void* E, int lde, const void* t32, const void* invS,
                                   const void* gsc, void* gW, int ldg, int M, int C, hipStream_t s) {
  if (C % 8 || ldx % 8) return hipErrorInvalidValue;
  return dw_fix_entry<false>(x, ldx, E, lde, t32, invS, gsc, gW, ldg, M, C, s);
}
NSA_API hipError_t nsa_xent_dw_fix_h(const void* x, int ldx, const void* E, int lde, const void* t32,
                                     const void* invS, const void* gsc, void* gW, int ldg, int M, int C,
                                     hipStream_t s) {
  if (C % 8 || ldx % 8) return hipErrorInvalidValue;
  return dw_fix_entry<true>(x, ldx, E, lde, t32, invS, gsc, gW, ldg, M, C, s);
}
