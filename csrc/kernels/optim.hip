// Fused flat AdamW + global gradient-norm clipping.
//
// One optimizer step over ALL parameters is three launches, independent of
// the tensor count (torch's multi-tensor path chunks per tensor list):
//   nsa_sumsq_partial : per-block sum of squares of the flat fp32 grad
//   nsa_clip_coef     : one block -> global norm + combined grad multiplier
//   nsa_adamw_step    : one HBM-bound pass, 16 B/lane vectors:
//                       reads p,g,m,v (16 B/elt), writes p,m,v (12 B) + bf16 p (2 B)
// Everything stays on the device (no host sync), so the step is capturable.
//
// Math = torch.optim.AdamW (decoupled weight decay):
//   p *= 1 - lr*wd ; m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g^2
//   p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
// where g = grad * coef and coef = grad_scale * min(1, max_norm/(norm+1e-6)).
//
// fp16 training (--dtype=float16) passes the dynamic loss scale's device
// state `ls` (optim/loss_scale.py LS_* slots) to all three kernels, so GradScaler's
// unscale / inf check / skip / scale update happen on the device with no host sync:
//   sumsq   : squares of grad * pre / ls[SCALE] (the UNSCALED gradient: finite scaled
//             gradients cannot overflow the sum) + a separate count of non-finite elements
//   clip    : found_inf = any non-finite element or a non-finite sum; coef = 0 then, the
//             scale backs off / grows by GradScaler's policy, the device step counter
//             advances only on a good step
//   adamw   : returns at once on a found_inf step; bias corrections from the device step
#include "common.h"

namespace {

constexpr int kBlock = 256;
// dynamic loss-scale state slots (float32), mirrored in optim/loss_scale.py
enum { LS_SCALE = 0, LS_TRACKER = 1, LS_FOUND = 2, LS_SKIPPED = 3, LS_STEP = 4 };

template <bool H = false>  // H: the compute shadow is fp16 (dtype float16)
__global__ __launch_bounds__(kBlock) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      bf16_t* __restrict__ pb, const uint8_t* __restrict__ wd_mask,
                                                      int64_t n4, float lr, float b1, float b2, float eps, float wd,
                                                      float step_size, float inv_bc2_sqrt,
                                                      const float* __restrict__ coef_ptr,
                                                      const float* __restrict__ ls) {
  if (ls != nullptr) {
    if (ls[LS_FOUND] != 0.0f) return;  // GradScaler: skip the step (wave-uniform)
    const float t = ls[LS_STEP];        // good steps so far, this one included
    step_size = lr / (1.0f - powf(b1, t));
    inv_bc2_sqrt = 1.0f / sqrtf(1.0f - powf(b2, t));
  }
  const float coef = coef_ptr[0];
  const float decay = 1.0f - lr * wd;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock) {
    float4 pp = reinterpret_cast<float4*>(p)[i];
    const float4 gg = reinterpret_cast<const float4*>(g)[i];
    float4 mm = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    const float d = wd_mask[(i * 4) >> 6] ? decay : 1.0f;  // 64-element chunks never straddle params
    float* pa = &pp.x;
    const float* ga = &gg.x;
    float* ma = &mm.x;
    float* va = &vv.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = ga[j] * coef;
      ma[j] = b1 * ma[j] + (1.0f - b1) * gj;
      va[j] = b2 * va[j] + (1.0f - b2) * gj * gj;
      const float denom = sqrtf(va[j]) * inv_bc2_sqrt + eps;
      pa[j] = pa[j] * d - step_size * ma[j] / denom;
    }
    reinterpret_cast<float4*>(p)[i] = pp;
    reinterpret_cast<float4*>(m)[i] = mm;
    reinterpret_cast<float4*>(v)[i] = vv;
    if (pb) {
      uint2 o;
      o.x = pk2<H>(pp.x, pp.y);
      o.y = pk2<H>(pp.z, pp.w);
      reinterpret_cast<uint2*>(pb)[i] = o;
    }
  }
}

// partial[b] = sum of (g * pre)^2 over block b's elements; with a loss scale, also
// partial[nblocks + b] = the number of non-finite elements (pre is then divided by the scale)
__global__ __launch_bounds__(kBlock) void sumsq_partial_kernel(const float* __restrict__ g, int64_t n4,
                                                              float* __restrict__ partial, float pre,
                                                              const float* __restrict__ ls) {
  if (ls != nullptr) pre /= ls[LS_SCALE];
  float acc = 0.0f;
  float bad = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock) {
    const float4 x = reinterpret_cast<const float4*>(g)[i];
    const float a = x.x * pre, b = x.y * pre, c = x.z * pre, d = x.w * pre;
    acc += a * a + b * b + c * c + d * d;
    if (ls != nullptr)
      bad += (float)(!__builtin_isfinite(x.x)) + (float)(!__builtin_isfinite(x.y)) +
             (float)(!__builtin_isfinite(x.z)) + (float)(!__builtin_isfinite(x.w));
  }
  acc = wave_sum(acc);
  if (ls != nullptr) bad = wave_sum(bad);
  __shared__ float red[2][kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = acc;
    red[1][threadIdx.x >> 6] = bad;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.0f, nb = 0.0f;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) {
      s += red[0][w];
      nb += red[1][w];
    }
    partial[blockIdx.x] = s;
    if (ls != nullptr) partial[gridDim.x + blockIdx.x] = nb;
  }
}

// norm = sqrt(sum of the partials) (already multiplied by the gradient scale in the
// sumsq pass); coef = scale * min(1, max_norm / (norm + 1e-6)), scale divided by the loss
// scale when one is given; then the loss-scale update (GradScaler's policy)
__global__ __launch_bounds__(1024) void clip_coef_kernel(const float* __restrict__ partial, int nparts, float scale,
                                                        float max_norm, float* __restrict__ norm_out,
                                                        float* __restrict__ coef_out, float* __restrict__ ls,
                                                        float growth, float backoff, float interval) {
  double acc = 0.0, bad = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 1024) {
    acc += (double)partial[i];
    if (ls != nullptr) bad += (double)partial[nparts + i];
  }
  __shared__ double red[2][1024];
  red[0][threadIdx.x] = acc;
  red[1][threadIdx.x] = bad;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float norm = (float)sqrt(red[0][0]);
    float c = 1.0f;
    if (max_norm > 0.0f) {
      c = max_norm / (norm + 1e-6f);
      if (c > 1.0f) c = 1.0f;
    }
    if (ls == nullptr) {
      norm_out[0] = norm;
      coef_out[0] = scale * c;
      return;
    }
    const bool found = red[1][0] > 0.0 || !__builtin_isfinite(norm);
    norm_out[0] = found ? __builtin_inff() : norm;
    coef_out[0] = found ? 0.0f : scale / ls[LS_SCALE] * c;
    ls[LS_FOUND] = found ? 1.0f : 0.0f;
    if (found) {
      ls[LS_SCALE] *= backoff;
      ls[LS_TRACKER] = 0.0f;
      ls[LS_SKIPPED] += 1.0f;
    } else {
      ls[LS_STEP] += 1.0f;
      ls[LS_TRACKER] += 1.0f;
      if (ls[LS_TRACKER] >= interval) {
        ls[LS_SCALE] *= growth;
        ls[LS_TRACKER] = 0.0f;
      }
    }
  }
}

// out[c] += sum_r partial[r][c]   (LayerNorm dW/db second-stage reduction)
// grid = (ceil(C/64), splits): each block sums its slice of rows for 64 columns
// (4 waves x strided rows, lane = column, coalesced 256-B rows), folds the 4
// waves in LDS and adds into the fp32 gradient with one atomic per column —
// `splits`-way contention per address only.
__global__ __launch_bounds__(kBlock) void colsum_kernel(const float* __restrict__ partial, float* __restrict__ out,
                                                       int rows, int C, int rows_per_split) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * rows_per_split;
  const int r1 = min(rows, r0 + rows_per_split);
  float acc = 0.0f;
  if (c < C) {
#pragma unroll 4
    for (int r = r0 + w; r < r1; r += 4) acc += partial[(int64_t)r * C + c];
  }
  __shared__ float red[4][64];
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < C) atomicAdd(out + c, red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}

// Bias gradient, first stage: partial[b][c] = sum over row slice b of dy[r][c] (bf16 in, fp32
// sums).  Block = 4 row lanes x 64 column chunks of 8 (16-byte loads); the 4 row lanes fold
// in LDS.  The second stage is colsum_kernel (nsa_colsum_accum[_ordered]) into the gradient.
template <bool H = false>  // H: dy is fp16
__global__ __launch_bounds__(kBlock) void colsum_bf16_kernel(const bf16_t* __restrict__ dy, int ld, int rows, int C,
                                                            int rows_per_block, float* __restrict__ partial) {
  const int cx = threadIdx.x & 63, ry = threadIdx.x >> 6;
  const int c = (blockIdx.x * 64 + cx) * 8;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    for (int r = r0 + ry; r < r1; r += 4) {
      float f[8];
      load8e<H>(dy + (int64_t)r * ld + c, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += f[j];
    }
  }
  __shared__ float red[4][64 * 8 + 4];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[ry][cx * 8 + j] = acc[j];
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 8; i += kBlock) {
    const int cc = blockIdx.x * 64 * 8 + i;
    if (cc < C) partial[(int64_t)blockIdx.y * C + cc] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

}  // namespace

// partial [nblk][C] (fp32) = column sums of dy [rows][C] (bf16, leading dim ld) over nblk row slices
NSA_API hipError_t nsa_colsum_bf16_partial(const void* dy, int ld, int rows, int C, void* partial, int nblk,
                                           hipStream_t s) {
  if (C % 8 || ld % 8 || nblk < 1) return hipErrorInvalidValue;
  dim3 grid((C / 8 + 63) / 64, nblk);
  colsum_bf16_kernel<false><<<grid, kBlock, 0, s>>>((const bf16_t*)dy, ld, rows, C, (rows + nblk - 1) / nblk,
                                                    (float*)partial);
  NSA_LAUNCH_CHECK();
}
NSA_API hipError_t nsa_colsum_bf16_partial_h(const void* dy, int ld, int rows, int C, void* partial, int nblk,
                                             hipStream_t s) {
  if (C % 8 || ld % 8 || nblk < 1) return hipErrorInvalidValue;
  dim3 grid((C / 8 + 63) / 64, nblk);
  colsum_bf16_kernel<true><<<grid, kBlock, 0, s>>>((const bf16_t*)dy, ld, rows, C, (rows + nblk - 1) / nblk,
                                                   (float*)partial);
  NSA_LAUNCH_CHECK();
}

template <bool H>
static hipError_t adamw_entry(void* p, const void* g, void* m, void* v, void* p_bf16, const void* wd_mask, int64_t n,
                              float lr, float beta1, float beta2, float eps, float wd, float bc1, float bc2_sqrt,
                              const void* coef, const void* ls, hipStream_t s) {
  if (n % 4 != 0) return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  int64_t grid = (n4 + kBlock - 1) / kBlock;
  if (grid > 4096) grid = 4096;
  adamw_kernel<H><<<(int)grid, kBlock, 0, s>>>((float*)p, (const float*)g, (float*)m, (float*)v, (bf16_t*)p_bf16,
                                            (const uint8_t*)wd_mask, n4, lr, beta1, beta2, eps, wd, lr / bc1,
                                            1.0f / bc2_sqrt, (const float*)coef, (const float*)ls);
  NSA_LAUNCH_CHECK();
}
NSA_API hipError_t nsa_adamw_step(void* p, const void* g, void* m, void* v, void* p_bf16, const void* wd_mask,
                                  int64_t n, float lr, float beta1, float beta2, float eps, float wd, float bc1,
                                  float bc2_sqrt, const void* coef, const void* ls, hipStream_t s) {
  return adamw_entry<false>(p, g, m, v, p_bf16, wd_mask, n, lr, beta1, beta2, eps, wd, bc1, bc2_sqrt, coef, ls, s);
}
// the same with an fp16 compute shadow
NSA_API hipError_t nsa_adamw_step_h(void* p, const void* g, void* m, void* v, void* p_f16, const void* wd_mask,
                                    int64_t n, float lr, float beta1, float beta2, float eps, float wd, float bc1,
                                    float bc2_sqrt, const void* coef, const void* ls, hipStream_t s) {
  return adamw_entry<true>(p, g, m, v, p_f16, wd_mask, n, lr, beta1, beta2, eps, wd, bc1, bc2_sqrt, coef, ls, s);
}

// partial holds nblocks floats, 2 * nblocks with a loss scale (ls != null)
NSA_API hipError_t nsa_sumsq_partial(const void* g, int64_t n, void* partial, int nblocks, float pre, const void* ls,
                                     hipStream_t s) {
  if (n % 4 != 0) return hipErrorInvalidValue;
  sumsq_partial_kernel<<<nblocks, kBlock, 0, s>>>((const float*)g, n / 4, (float*)partial, pre, (const float*)ls);
  NSA_LAUNCH_CHECK();
}

NSA_API hipError_t nsa_clip_coef(const void* partial, int nparts, float scale, float max_norm, void* norm_out,
                                 void* coef_out, void* ls, float growth, float backoff, float interval,
                                 hipStream_t s) {
  clip_coef_kernel<<<1, 1024, 0, s>>>((const float*)partial, nparts, scale, max_norm, (float*)norm_out,
                                      (float*)coef_out, (float*)ls, growth, backoff, interval);
  NSA_LAUNCH_CHECK();
}

NSA_API hipError_t nsa_colsum_accum(const void* partial, void* out, int rows, int C, hipStream_t s) {
  int splits = rows / 32;
  if (splits < 1) splits = 1;
  if (splits > 32) splits = 32;
  const int rps = (rows + splits - 1) / splits;
  dim3 grid((C + 63) / 64, splits);
  colsum_kernel<<<grid, kBlock, 0, s>>>((const float*)partial, (float*)out, rows, C, rps);
  NSA_LAUNCH_CHECK();
}

// deterministic mode: one row range per column block, so each column's single atomic
// add lands on the flat gradient in a fixed order (bitwise reproducible)
NSA_API hipError_t nsa_colsum_accum_ordered(const void* partial, void* out, int rows, int C, hipStream_t s) {
  dim3 grid((C + 63) / 64, 1);
  colsum_kernel<<<grid, kBlock, 0, s>>>((const float*)partial, (float*)out, rows, C, rows);
  NSA_LAUNCH_CHECK();
}
