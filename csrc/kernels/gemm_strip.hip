// Column-strip "NT" GEMM: C[:, 0:NS] = A[M, K] · B[NS, K]^T (+ bias), NS <= 64, for the last
// columns of a GEMM whose N is a multiple of the persistent kernel's 256-wide tile plus a
// small remainder: GPT-2 1.5B's n_embd = 1600 = 6 x 256 + 64.  The four-wave kernel
// (gemm_nt4.hip) runs the first 1536 columns (1440 tiles at M = 61440, 5.6 CU rounds) and
// this kernel the 64-column strip, instead of a seventh column tile shifted back over
// columns it already covered (1680 tiles, 6.6 rounds): the tile the persistent kernel
// would spend on 64 new columns computes 256.
//
// The strip reads every row of A for 64 outputs: 2·64 flops per 2-byte element, so it is
// bound by the A stream (61440 x 1600 bf16 = 197 MB; 8 TB/s HBM peak), not by MFMAs.  The
// geometry serves that stream: each wave owns 64 rows x NS columns (4 x NS/16 accumulators
// of v_mfma_f32_16x16x32_bf16) and free-runs over K with no LDS and no barrier -- A and B
// fragments go from global memory straight into registers in the MFMA operand layout
// (lane l: row / column l & 15, k 8 (l >> 4) .. + 7 of a 32-deep step: 16 contiguous bytes
// of a K-contiguous row), a ring of NSA_STRIP_D k-steps in flight (B, 64 x K, is re-read
// per wave from L2).  A first form (16 rows per wave, B staged through LDS behind a barrier
// per 64-deep K-tile, A two K-tiles ahead) ran at 1.7 TB/s: every K-tile waited on the B
// loads and the barrier.  Shape rules: NS % 16 == 0, NS <= 64, K % 32 == 0.
#include "common.h"

namespace {

constexpr int ST_ROWS = 64;  // rows per wave (4 A fragments)
#ifndef NSA_STRIP_D
#define NSA_STRIP_D 4  // 32-deep k-steps in flight per wave
#endif
constexpr int ST_D = NSA_STRIP_D;

template <bool H, bool BIAS, int NF>
__global__ __launch_bounds__(256) void gemm_strip_kernel(const bf16_t* __restrict__ A, int lda,
                                                         const bf16_t* __restrict__ B, int ldb, bf16_t* __restrict__ C,
                                                         int ldc, const bf16_t* __restrict__ bias, int M, int NS,
                                                         int K) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * ST_ROWS;
  if (row0 >= M) return;  // wave-uniform: no barriers in this kernel
  const int kq = (lane >> 4) * 8;
  const bf16_t* ap[4];
  const bf16_t* bp[NF];
#pragma unroll
  for (int i = 0; i < 4; ++i) ap[i] = A + (int64_t)min(row0 + 16 * i + (lane & 15), M - 1) * lda + kq;
#pragma unroll
  for (int j = 0; j < NF; ++j) bp[j] = B + (int64_t)(16 * j + (lane & 15)) * ldb + kq;
  const int nks = K / 32;
  // ring of ST_D k-steps: slot u holds k-step ks + u's 4 A and NF B fragments
  bf16x8 fa[ST_D][4], fb[ST_D][NF];
#pragma unroll
  for (int u = 0; u < ST_D; ++u) {
    const int k = min(u, nks - 1) * 32;
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[u][i] = *reinterpret_cast<const bf16x8*>(ap[i] + k);
#pragma unroll
    for (int j = 0; j < NF; ++j) fb[u][j] = *reinterpret_cast<const bf16x8*>(bp[j] + k);
  }
  f32x4 acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < nks; ks += ST_D) {
#pragma unroll
    for (int u = 0; u < ST_D; ++u) {
      if (ks + u < nks) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < NF; ++j) acc[i][j] = mfma16e<H>(fa[u][i], fb[u][j], acc[i][j]);
        if (ks + u + ST_D < nks) {
          const int k = (ks + u + ST_D) * 32;
#pragma unroll
          for (int i = 0; i < 4; ++i) fa[u][i] = *reinterpret_cast<const bf16x8*>(ap[i] + k);
#pragma unroll
          for (int j = 0; j < NF; ++j) fb[u][j] = *reinterpret_cast<const bf16x8*>(bp[j] + k);
        }
      }
    }
  }
  // lane l holds rows 4 (l >> 4) + e of column l & 15 of each 16 x 16 block
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int col = 16 * j + (lane & 15);
    const float bv = BIAS ? e2f<H>(bias[col]) : 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = row0 + 16 * i + 4 * (lane >> 4) + e;
        if (r < M) C[(int64_t)r * ldc + col] = f2e<H>(acc[i][j][e] + bv);
      }
    }
  }
}

template <bool H>
hipError_t strip_entry(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias, int M,
                       int NS, int K, hipStream_t s) {
  if (M < 1 || NS < 16 || NS > 64 || NS % 16 || K < 32 || K % 32 || lda % 8 || ldb % 8 ||
      (uintptr_t)A % 16 || (uintptr_t)B % 16)
    return hipErrorInvalidValue;
  const int grid = (M + 4 * ST_ROWS - 1) / (4 * ST_ROWS);
#define NSA_STRIP_GO(NF_)                                                                                     \
  if (bias)                                                                                                    \
    gemm_strip_kernel<H, true, NF_><<<grid, 256, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)B, ldb,        \
                                                         (bf16_t*)C, ldc, (const bf16_t*)bias, M, NS, K);     \
  else                                                                                                         \
    gemm_strip_kernel<H, false, NF_><<<grid, 256, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)B, ldb,       \
                                                          (bf16_t*)C, ldc, nullptr, M, NS, K)
  switch (NS / 16) {
    case 1: NSA_STRIP_GO(1); break;
    case 2: NSA_STRIP_GO(2); break;
    case 3: NSA_STRIP_GO(3); break;
    default: NSA_STRIP_GO(4); break;
  }
#undef NSA_STRIP_GO
  return hipGetLastError();
}

}  // namespace

// C[:, 0:NS] (row stride ldc) = A[M, K] · B[NS, K]^T (+ bias[NS]); bf16 (or fp16: _h)
NSA_API hipError_t nsa_gemm_strip(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                                  int M, int NS, int K, hipStream_t s) {
  return strip_entry<false>(A, lda, B, ldb, C, ldc, bias, M, NS, K, s);
}
NSA_API hipError_t nsa_gemm_strip_h(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* bias,
                                    int M, int NS, int K, hipStream_t s) {
  return strip_entry<true>(A, lda, B, ldb, C, ldc, bias, M, NS, K, s);
}
