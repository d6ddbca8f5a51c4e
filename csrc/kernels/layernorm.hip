// LayerNorm forward/backward, bf16 I/O, fp32 statistics (SURVEY.md §2.7 K3;
// nanoGPT LayerNorm: F.layer_norm(x, w.shape, w, b, 1e-5), optional bias).
//
// Layout: one 64-lane wave owns one row; lane l holds columns
// (k*64 + l)*8 .. +8 for k < NK, so a row of C <= 512*NK bf16 values lives in
// registers (NK*8 floats per lane) and is read from HBM exactly once.
// 4 waves (rows) per 256-thread block -> N/4 blocks (3072 for GPT-2 124M),
// far more than the 256 CUs.
//
// Backward: dx = rstd * (dy*w - mean(dy*w) - xhat * mean(dy*w*xhat)) per row;
// dw = sum_rows dy*xhat, db = sum_rows dy are accumulated per lane in
// registers across the rows a block visits, reduced across the block's 4
// waves in LDS and written as one partial row per block; nsa_colsum_accum then
// reduces the partial rows (split over row ranges, fp32 atomics) into the flat
// gradient buffer.  Backward rows are software-pipelined (next row's loads in
// flight while the current row is reduced).
#include "common.h"

namespace {

template <int NK>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                    bf16_t* __restrict__ sum_out, const bf16_t* __restrict__ w,
                                                    const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                    float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                    int N, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const bf16_t* xr = x + (int64_t)row * C;
  float v[NK][8];
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
      load8(xr + c, v[k]);
      if (res) {  // fused residual add: s = x + res, written out (bf16) and normalised
        float rv[8];
        load8(res + (int64_t)row * C + c, rv);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = bf2f(f2bf(v[k][j] + rv[j]));
        store8(sum_out + (int64_t)row * C + c, v[k]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[k][j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[k][j] = 0.0f;
    }
  }
  const float mean = wave_sum(s) / (float)C;
  float ss = 0.0f;
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = v[k][j] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / (float)C + eps);
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
      float wf[8], bfv[8], o[8];
      load8(w + c, wf);
      if (b) {
        load8(b + c, bfv);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) bfv[j] = 0.0f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[k][j] - mean) * rstd * wf[j] + bfv[j];
      store8(y + (int64_t)row * C + c, o);
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <int NK>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                    const bf16_t* __restrict__ w, const float* __restrict__ mean_in,
                                                    const float* __restrict__ rstd_in, const bf16_t* __restrict__ dres,
                                                    bf16_t* __restrict__ dx,
                                                    float* __restrict__ dw_part, float* __restrict__ db_part, int N,
                                                    int C) {
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][C]
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  float wf[NK][8];
  float dwa[NK][8], dba[NK][8];
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    const int c = (k * 64 + lane) * 8;
    if (c < C) {
      load8(w + c, wf[k]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) wf[k][j] = 0.0f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dwa[k][j] = 0.0f;
      dba[k][j] = 0.0f;
    }
  }
  // Rows are software-pipelined: the next row's x / dy / dres vectors are loaded
  // (as raw 16-byte words) while the current row is reduced and written, so each
  // row costs one overlapped memory round trip instead of two dependent ones.
  const int row_step = gridDim.x * 4;
  int row = blockIdx.x * 4 + wv;
  uint4 nx[NK], nd[NK], nr[NK];
#define NSA_LNB_LOAD(R)                                                                  \
  _Pragma("unroll") for (int k = 0; k < NK; ++k) {                                       \
    const int c = min((k * 64 + lane) * 8, C - 8);                                       \
    const int64_t off = (int64_t)min((R), N - 1) * C + c;                                \
    nx[k] = *reinterpret_cast<const uint4*>(x + off);                                    \
    nd[k] = *reinterpret_cast<const uint4*>(dy + off);                                   \
    if (dres) nr[k] = *reinterpret_cast<const uint4*>(dres + off);                       \
  }
  NSA_LNB_LOAD(row)
  for (; row < N; row += row_step) {
    const float mean = mean_in[row];
    const float rstd = rstd_in[row];
    uint4 cx[NK], cd[NK], cr[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      cx[k] = nx[k];
      cd[k] = nd[k];
      cr[k] = nr[k];
    }
    NSA_LNB_LOAD(row + row_step)
    float xh[NK][8], g[NK][8];
    float s1 = 0.0f, s2 = 0.0f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < C) {
        float xv[8], dv[8];
        unpack8(cx[k], xv);
        unpack8(cd[k], dv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[k][j] = (xv[j] - mean) * rstd;
          g[k][j] = dv[j] * wf[k][j];
          s1 += g[k][j];
          s2 += g[k][j] * xh[k][j];
          dwa[k][j] += dv[j] * xh[k][j];
          dba[k][j] += dv[j];
        }
      }
    }
    const float m1 = wave_sum(s1) / (float)C;
    const float m2 = wave_sum(s2) / (float)C;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < C) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = rstd * (g[k][j] - m1 - xh[k][j] * m2);
        if (dres) {  // gradient arriving through the residual path of the fused add
          float rv[8];
          unpack8(cr[k], rv);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += rv[j];
        }
        store8(dx + (int64_t)row * C + c, o);
      }
    }
  }
#undef NSA_LNB_LOAD
  // block reduction of the per-lane dw/db partials (4 waves -> 1 row)
  for (int pass = 0; pass < 2; ++pass) {
    float* dst = pass == 0 ? dw_part : db_part;
    if (dst == nullptr) continue;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int c = (k * 64 + lane) * 8;
      if (c < C) {
#pragma unroll
        for (int j = 0; j < 8; ++j) red[wv * C + c + j] = pass == 0 ? dwa[k][j] : dba[k][j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256)
      dst[(int64_t)blockIdx.x * C + c] = red[c] + red[C + c] + red[2 * C + c] + red[3 * C + c];
    __syncthreads();
  }
}

template <int NK>
hipError_t launch_fwd(const void* x, const void* res, void* sum_out, const void* w, const void* b, void* y,
                      void* mean, void* rstd, int N, int C, float eps, hipStream_t s) {
  ln_fwd_kernel<NK><<<(N + 3) / 4, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)res, (bf16_t*)sum_out,
                                                (const bf16_t*)w, (const bf16_t*)b, (bf16_t*)y, (float*)mean,
                                                (float*)rstd, N, C, eps);
  return hipGetLastError();
}

template <int NK>
hipError_t launch_bwd(const void* dy, const void* x, const void* w, const void* mean, const void* rstd,
                      const void* dres, void* dx, void* dw_part, void* db_part, int N, int C, int nblk,
                      hipStream_t s) {
  ln_bwd_kernel<NK><<<nblk, 256, 4 * C * sizeof(float), s>>>(
      (const bf16_t*)dy, (const bf16_t*)x, (const bf16_t*)w, (const float*)mean, (const float*)rstd,
      (const bf16_t*)dres, (bf16_t*)dx,
      (float*)dw_part, (float*)db_part, N, C);
  return hipGetLastError();
}

}  // namespace

#define NSA_NK_SWITCH(NK_EXPR, CALL)                      \
  switch (NK_EXPR) {                                        \
    case 1: { constexpr int K_ = 1; return CALL; }          \
    case 2: { constexpr int K_ = 2; return CALL; }          \
    case 3: { constexpr int K_ = 3; return CALL; }          \
    case 4: { constexpr int K_ = 4; return CALL; }          \
    case 5:                                                 \
    case 6: { constexpr int K_ = 6; return CALL; }          \
    case 7:                                                 \
    case 8: { constexpr int K_ = 8; return CALL; }          \
    default:                                                \
      if ((NK_EXPR) <= 16) { constexpr int K_ = 16; return CALL; } \
      return hipErrorInvalidValue;                          \
  }

// y = LN(x [+ res]) ; with res != NULL also writes sum_out = x + res (bf16)
NSA_API hipError_t nsa_layernorm_fwd(const void* x, const void* res, void* sum_out, const void* w, const void* b,
                                     void* y, void* mean, void* rstd, int N, int C, float eps, hipStream_t s) {
  if (C % 8 != 0) return hipErrorInvalidValue;
  NSA_NK_SWITCH((C + 511) / 512, launch_fwd<K_>(x, res, sum_out, w, b, y, mean, rstd, N, C, eps, s));
}

// dx = LN'(dy) [+ dres]; per-block dw/db partial rows for nsa_colsum_accum
NSA_API hipError_t nsa_layernorm_bwd(const void* dy, const void* x, const void* w, const void* mean,
                                     const void* rstd, const void* dres, void* dx, void* dw_part, void* db_part,
                                     int N, int C, int nblk, hipStream_t s) {
  if (C % 8 != 0 || C > 8192) return hipErrorInvalidValue;
  NSA_NK_SWITCH((C + 511) / 512, launch_bwd<K_>(dy, x, w, mean, rstd, dres, dx, dw_part, db_part, N, C, nblk, s));
}
