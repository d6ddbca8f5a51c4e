// bf16 MFMA weight-gradient GEMM for gfx950 (dW = dY^T · X for
// every nn.Linear), split over the token dimension with the fp32 result added straight
// into the flat fp32 gradient buffer:
//
//   C[M,N] += A[M,K] · B[K,N]   with A stored [K][M] (dY, tokens x out-features) and
//                               B stored [K][N] (X, tokens x in-features), fp32 accumulate,
//                               v_mfma_f32_16x16x32_bf16 on ds_read_b64_tr_b16 fragments.
//
// (The forward and input-gradient GEMMs are gemm_nt4.hip / gemm_small.hip.)
//
// Structure (cdna_hip_programming.md §5): 256x256 block tile, 8 waves as 2 (M) x 4 (N),
// each wave 128x64 = 8x4 16x16 accumulators.  K is split over blockIdx.z; split z owns
// 64-deep K blocks [z*n/S, (z+1)*n/S) (any split count).  Operands are staged by LDS-DMA
// (global_load_lds_dwordx4 from inline asm; hipcc would drain vmcnt(0) before every
// ds_read around the builtin) with counted `s_waitcnt vmcnt` across raw barriers
// (never 0 in the loop).  Because the DMA destination is lane-linear, the XOR swizzle of
// the LDS images is applied to the per-lane global source address (rule 21).
// Epilogue: each wave re-shapes its accumulators through LDS so that every fp32 atomic
// (or plain store, deterministic mode) wave instruction covers one contiguous 256-B row
// — the full-rate shape of MI355X_MICROARCH.md "Global float atomics".
// Block ids are remapped so that the blocks sharing an XCD (b % 8) walk neighbouring
// tiles (T1, bijective form).
//
// Role: the weight-gradient kernel for the shapes the four-wave kernel (gemm_wg4.hip) does not
// take (an output side below 256: tiny models, test configs) -- it accepts M, N >= 8.
// "ring64": 64-deep LDS-DMA slots (every DMA row a whole 128-B line), two slots, each
// multiplied as two 32-deep sub-slices with the next sub-slice's fragments read under the
// current one's MFMAs.  The round-1/2 variants that lost to it or to gemm_wg4.hip ("ring",
// "phase", register-staged, 5-slot / pipelined rings, persistent p8, 4-wave 128x128 and
// 2-workgroup-per-CU geometries) are in git history; measurements in docs/performance.md.
#include "common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int WAVES_M = 2, WAVES_N = 4;
constexpr int WTM = BM / WAVES_M;  // 128
constexpr int WTN = BN / WAVES_N;  // 64
constexpr int FM = WTM / 16;       // 8
constexpr int FN = WTN / 16;       // 4
constexpr int EP_LD = 68;                                   // epilogue row pitch (fp32), +4 breaks bank aliasing
constexpr int EP_BYTES = (NTHREADS / 64) * 64 * EP_LD * 4;  // 136 KiB

// EPI_STORE_F32: split z stores its fp32 partial tile to C + z * M * ldc (plain stores;
// the deterministic weight-gradient path sums the splits in a fixed order afterwards)
enum Epi : int { EPI_ATOMIC_F32 = 1, EPI_STORE_F32 = 4 };

// row-contiguous image [64][W]: 2W-byte rows, chunk' = chunk ^ 2*g(row), g = (r&3) | ((r>>3)&1)<<2
template <int W>
__device__ __forceinline__ int rimg(int row, int chunk) {
  const int g = (row & 3) | (((row >> 3) & 1) << 2);
  return row * (W * 2) + ((chunk ^ (2 * g)) << 4);
}

__device__ __forceinline__ s16x4 lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}

// operand fragment of 16 rows (or columns) x 32 k for the 16x16x32 MFMA from a [K][W]
// image: lane l: element j = X[r0 + (l & 15)][k = 32*kk + 8*(l >> 4) + j]
template <int W>
__device__ __forceinline__ bf16x8 load_frag(const char* tile, int r0, int kk, int lane) {
  const int ig = lane & 15;
  const int q = ig >> 2, p = ig & 3;
  const int krow = 32 * kk + 8 * (lane >> 4) + q;
  const int col = r0 + 4 * p;
  const int off = (col & 7) * 2;
  const s16x4 a = lds_tr(tile + rimg<W>(krow, col >> 3) + off);
  const s16x4 b = lds_tr(tile + rimg<W>(krow + 4, col >> 3) + off);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  float* C;  // fp32 [M][ldc] (atomic epilogue) or [splits][M][ldc] (partials)
  int M, N, K;
  int lda, ldb, ldc;
  int tiles_m, tiles_n;
};

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// fp32 epilogue: re-shape through LDS so each atomic / store wave-instruction covers one
// contiguous 256-B row
template <int EPI>
__device__ __forceinline__ void wgrad_epilogue(const GemmArgs& g, f32x4 (&acc)[FM][FN], char* smem, int m0, int n0,
                                               int wm, int wn, int lane, int wave, int mlo = 0, int nlo = 0) {
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);
  __syncthreads();
  float* ep = reinterpret_cast<float*>(smem) + wave * 64 * EP_LD;
  float* Cz = g.C;
  if constexpr (EPI == EPI_STORE_F32) Cz += (int64_t)blockIdx.z * g.M * g.ldc;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int ii = 0; ii < FM / 2; ++ii) {
      const int i = half * (FM / 2) + ii;
#pragma unroll
      for (int j = 0; j < FN; ++j)
        *reinterpret_cast<float4*>(ep + (16 * ii + lrow) * EP_LD + 16 * j + lcol) =
            make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int row_base = m0 + wm * WTM + half * 64;
    const int col = n0 + wn * WTN + lane;
    if (col < g.N && col >= nlo) {
      for (int rr = 0; rr < 64; ++rr) {
        const int row = row_base + rr;
        if (row < g.M && row >= mlo) {
          if constexpr (EPI == EPI_STORE_F32)
            Cz[(int64_t)row * g.ldc + col] = ep[rr * EP_LD + lane];
          else
            atomicAdd(Cz + (int64_t)row * g.ldc + col, ep[rr * EP_LD + lane]);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// per-lane global source of one 16-byte DMA piece of a [K][W] image row (swizzled chunk)
__device__ __forceinline__ const bf16_t* tn_src(const bf16_t* base, int ld, int k0, int row, int pc, int lim, int c0) {
  const int gg = (row & 3) | (((row >> 3) & 1) << 2);
  const int c = pc ^ (2 * gg);
  return base + (int64_t)(k0 + row) * ld + min(c0 + c * 8, lim - 8);
}

// ---------------------------------------------------------------------------
// Variant 7 ("ring64"): LDS-DMA slots 64 deep in K (every DMA row a whole 128-B line;
// the 32-deep ring fetches 64-B half-lines), two 64 KiB slots, each multiplied as two
// 32-deep sub-slices with the fragment pipeline (reads of the next sub-slice under the
// MFMAs of the current one: A in place, B double-buffered):
//   phase A: MFMA(k, 0) | read (k, 1)           (same slot, no barrier)
//   wait own DMA of slot k+1 + lgkmcnt(0), barrier, DMA slot k+2 -> slot k's buffer
//   phase B: MFMA(k, 1) | read (k+1, 0)
// Slot k's buffer is free at that barrier: its (k,0) reads completed before phase A's
// MFMAs and its (k,1) reads before the barrier, in every wave.
// ---------------------------------------------------------------------------
constexpr int R64_SLOT_A = BM * 64 * 2;   // 32 KiB
constexpr int R64_SLOT = 2 * R64_SLOT_A;  // A + B
constexpr int R64_SMEM = 2 * R64_SLOT > EP_BYTES ? 2 * R64_SLOT : EP_BYTES;
static_assert(R64_SMEM <= 163840, "LDS budget");

template <int EPI, bool H = false>
__global__ __launch_bounds__(NTHREADS, 2) void wgrad_ring64_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[R64_SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int nwg = g.tiles_m * g.tiles_n;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int tm = bid / g.tiles_n, tn = bid % g.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nkb = g.K / 64, kb0 = (int)blockIdx.z * nkb / (int)gridDim.z;
  const int k_begin = kb0 * 64;
  const int nk = ((int)blockIdx.z + 1) * nkb / (int)gridDim.z - kb0;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  // per thread and slot: 4 DMA pieces of A and 4 of B (32 KiB each / 512 lanes / 16 B)
  auto issue = [&](int s) {
    const int k0 = k_begin + s * 64;
    const uint32_t slot = lds0 + (uint32_t)((s & 1) * R64_SLOT);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = j * NTHREADS + tid;
      const uint32_t wbase = (uint32_t)((j * NTHREADS + wave * 64) * 16);
      const int row = e >> 5, pc = e & 31;
      glds16(tn_src(g.A, g.lda, k0, row, pc, g.M, m0), __builtin_amdgcn_readfirstlane(slot + wbase));
      glds16(tn_src(g.B, g.ldb, k0, row, pc, g.N, n0), __builtin_amdgcn_readfirstlane(slot + R64_SLOT_A + wbase));
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue(0);
  if (nk > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  bf16x8 af[FM], b0[FN], b1[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) b0[j] = load_frag<BN>(smem + R64_SLOT_A, wn * WTN + 16 * j, 0, lane);
#pragma unroll
  for (int i = 0; i < FM; ++i) af[i] = load_frag<BM>(smem, wm * WTM + 16 * i, 0, lane);

#define NSA_R64_PHASE(BC, BNX, TA, TB, KKN)                                                     \
  __builtin_amdgcn_s_setprio(1);                                                              \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) {                                            \
    _Pragma("unroll") for (int j = 0; j < FN; ++j)                                            \
      acc[i][j] = mfma16e<H>(BC[j], af[i], acc[i][j]);                                        \
    af[i] = load_frag<BM>((TA), wm * WTM + 16 * i, (KKN), lane);                              \
    if (i < FN) BNX[i] = load_frag<BN>((TB), wn * WTN + 16 * i, (KKN), lane);                 \
  }                                                                                           \
  __builtin_amdgcn_s_setprio(0);

  for (int k = 0; k < nk; ++k) {
    const char* ta = smem + (k & 1) * R64_SLOT;
    const char* tn = smem + ((k + 1) & 1) * R64_SLOT;  // next slot (garbage reads past the end: discarded)
    NSA_R64_PHASE(b0, b1, ta, ta + R64_SLOT_A, 1)
    if (k + 1 < nk) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (k + 2 < nk) issue(k + 2);
    NSA_R64_PHASE(b1, b0, tn, tn + R64_SLOT_A, 0)
  }
#undef NSA_R64_PHASE
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wgrad_epilogue<EPI>(g, acc, smem, m0, n0, wm, wn, lane, wave);
}


}  // namespace

// C (fp32) [M, N] (+)= A^T B with A stored [K][M], B stored [K][N] (leading dims lda / ldb),
// K split over `splits` workgroups per output tile.
// epi: 1 = fp32 atomic add into C, 4 = split z stores its fp32 partial into C + z*M*ldc
// (bits 8..15, the round-2 variant selector, are ignored).
namespace {
template <bool H>
hipError_t gemm_ring64_entry(int layout, int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                             void* C2, const void* U, int M, int N, int K, int splits, hipStream_t s) {
  (void)C2;
  (void)U;
  epi &= 0xff;
  if (layout != 2 || (epi != EPI_ATOMIC_F32 && epi != EPI_STORE_F32)) return hipErrorInvalidValue;
  if (K % BK != 0 || splits < 1 || splits > K / BK || M < 8 || N < 8 || M % 8 || N % 8) return hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (float*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.tiles_m = (M + BM - 1) / BM;
  a.tiles_n = (N + BN - 1) / BN;
  const dim3 grid(a.tiles_m * a.tiles_n, 1, splits);
  if (epi == EPI_ATOMIC_F32) wgrad_ring64_kernel<EPI_ATOMIC_F32, H><<<grid, NTHREADS, 0, s>>>(a);
  else wgrad_ring64_kernel<EPI_STORE_F32, H><<<grid, NTHREADS, 0, s>>>(a);
  return hipGetLastError();
}
}  // namespace

NSA_API hipError_t nsa_gemm(int layout, int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                            void* C2, const void* U, int M, int N, int K, int splits, hipStream_t s) {
  return gemm_ring64_entry<false>(layout, epi, A, lda, B, ldb, C, ldc, C2, U, M, N, K, splits, s);
}
// fp16 A / B
NSA_API hipError_t nsa_gemm_h(int layout, int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                              void* C2, const void* U, int M, int N, int K, int splits, hipStream_t s) {
  return gemm_ring64_entry<true>(layout, epi, A, lda, B, ldb, C, ldc, C2, U, M, N, K, splits, s);
}
