// Bounds-checked bf16 "NT" GEMM for the shapes the persistent four-wave kernel (gemm_nt4.hip)
// does not take: M or N below one 256 x 256 tile (tiny models, short prefills, test
// configs), K not a multiple of 64, odd N.  C[M,N] = A[M,K] · B[N,K]^T, fp32 accumulate, the
// same epilogues as gemm_nt4.hip (bf16 / + bias, gelu'(u) + gelu(u), acc * U).
//
// Geometry: 64 x 64 output tile per 256-thread workgroup, 4 waves as 2 x 2 of 32 x 32 (2 x 2
// accumulators of v_mfma_f32_16x16x32_bf16), 32-deep K steps staged through LDS with
// 16-byte loads (rows beyond M / N and k beyond K are zero-filled, so K % 8 == 0 is the only
// shape rule).  Register-staged and single-buffered: these shapes are launch- or
// latency-bound, not MFMA-bound, and the kernel exists so that no GEMM of the training step
// needs a vendor library whatever the model shape.
#include "common.h"

namespace {

constexpr int S_BM = 64, S_BN = 64, S_BK = 32;
constexpr int S_LD = S_BK + 8;  // LDS row pitch in bf16 (80 B: the 16-B fragment reads of a
                                // lane group land on distinct bank groups)

enum { S_EPI_BF16 = 0, S_EPI_GELU = 1, S_EPI_DGELU = 2 };

template <int EPI, bool BIAS, bool H = false>
__global__ __launch_bounds__(256) void gemm_small_kernel(const bf16_t* __restrict__ A, int lda,
                                                         const bf16_t* __restrict__ B, int ldb, bf16_t* __restrict__ C,
                                                         bf16_t* __restrict__ C2, int ldc,
                                                         const bf16_t* __restrict__ U, const bf16_t* __restrict__ bias,
                                                         int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) bf16_t sA[S_BM * S_LD];
  __shared__ __attribute__((aligned(16))) bf16_t sB[S_BN * S_LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * S_BM, n0 = blockIdx.x * S_BN;
  // staging: thread t copies 16-B chunk (t & 3) of row t >> 2 of each operand tile
  const int lr = tid >> 2, lc = (tid & 3) * 8;
  const bool arow = m0 + lr < M, brow = n0 + lr < N;
  const bf16_t* ap = A + (int64_t)(arow ? m0 + lr : 0) * lda + lc;
  const bf16_t* bp = B + (int64_t)(brow ? n0 + lr : 0) * ldb + lc;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint4 zero = make_uint4(0, 0, 0, 0);
  for (int k0 = 0; k0 < K; k0 += S_BK) {
    const bool kin = k0 + lc < K;
    const uint4 va = (arow && kin) ? *reinterpret_cast<const uint4*>(ap + k0) : zero;
    const uint4 vb = (brow && kin) ? *reinterpret_cast<const uint4*>(bp + k0) : zero;
    __syncthreads();  // the previous step's fragment reads are done
    *reinterpret_cast<uint4*>(sA + lr * S_LD + lc) = va;
    *reinterpret_cast<uint4*>(sB + lr * S_LD + lc) = vb;
    __syncthreads();
    // fragments: lane l holds row (l & 15), k = 8 (l >> 4) .. + 7 of each 16-row block
    bf16x8 fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      fa[i] = *reinterpret_cast<const bf16x8*>(sA + (wm * 32 + i * 16 + (lane & 15)) * S_LD + 8 * (lane >> 4));
      fb[i] = *reinterpret_cast<const bf16x8*>(sB + (wn * 32 + i * 16 + (lane & 15)) * S_LD + 8 * (lane >> 4));
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma16e<H>(fa[i], fb[j], acc[i][j]);
  }
  // C/D layout: lane l holds rows 4 (l >> 4) + e, column l & 15 of each 16 x 16 block
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn * 32 + j * 16 + (lane & 15);
      if (col >= N) continue;
      const float bcol = BIAS ? e2f<H>(bias[col]) : 0.0f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + e;
        if (row >= M) continue;
        const int64_t o = (int64_t)row * ldc + col;
        float v = acc[i][j][e] + bcol;
        if constexpr (EPI == S_EPI_DGELU) v = e2f<H>(f2e<H>(v)) * nsa_h2f(U[o]);  // U = gelu'(u), fp16
        const bf16_t vb = f2e<H>(v);
        if constexpr (EPI == S_EPI_GELU) {  // C <- gelu'(u) (fp16), C2 <- gelu(u)
          const float uf = e2f<H>(vb);
          C[o] = nsa_f2h(nsa_gelu_grad(uf));
          C2[o] = f2e<H>(nsa_gelu(uf));
        } else {
          C[o] = vb;
        }
      }
    }
  }
}

}  // namespace

// Same contract as nsa_gemm_nt4 (epi 0 bf16, 1 gelu'(u) (fp16) / gelu(u) into C / C2, 2 acc * U with
// U = gelu'(u) in fp16;
// optional bias[N]) for any M, N >= 1 and K % 8 == 0 (lda, ldb % 8 == 0, 16-B aligned rows).
namespace {
template <bool H>
hipError_t gemm_small_entry(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* C2,
                            const void* U, const void* bias, int M, int N, int K, hipStream_t s) {
  if (M < 1 || N < 1 || K < 1 || K % 8 || lda % 8 || ldb % 8 || lda < K || ldb < K || ldc < N ||
      (uintptr_t)A % 16 || (uintptr_t)B % 16)
    return hipErrorInvalidValue;
  if ((epi == S_EPI_GELU && !C2) || (epi == S_EPI_DGELU && (!U || bias))) return hipErrorInvalidValue;
  const dim3 grid((N + S_BN - 1) / S_BN, (M + S_BM - 1) / S_BM);
  const bf16_t *a = (const bf16_t*)A, *b = (const bf16_t*)B, *u = (const bf16_t*)U, *bi = (const bf16_t*)bias;
  bf16_t *c = (bf16_t*)C, *c2 = (bf16_t*)C2;
#define SMALL(E, BI) gemm_small_kernel<E, BI, H><<<grid, 256, 0, s>>>(a, lda, b, ldb, c, c2, ldc, u, bi, M, N, K)
  switch (epi) {
    case S_EPI_BF16:
      if (bias) SMALL(S_EPI_BF16, true);
      else SMALL(S_EPI_BF16, false);
      break;
    case S_EPI_GELU:
      if (bias) SMALL(S_EPI_GELU, true);
      else SMALL(S_EPI_GELU, false);
      break;
    case S_EPI_DGELU: SMALL(S_EPI_DGELU, false); break;
    default: return hipErrorInvalidValue;
  }
#undef SMALL
  return hipGetLastError();
}
}  // namespace

NSA_API hipError_t nsa_gemm_small(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* C2,
                                  const void* U, const void* bias, int M, int N, int K, hipStream_t s) {
  return gemm_small_entry<false>(epi, A, lda, B, ldb, C, ldc, C2, U, bias, M, N, K, s);
}
// fp16 operands / outputs
NSA_API hipError_t nsa_gemm_small_h(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                                    void* C2, const void* U, const void* bias, int M, int N, int K, hipStream_t s) {
  return gemm_small_entry<true>(epi, A, lda, B, ldb, C, ldc, C2, U, bias, M, N, K, s);
}
