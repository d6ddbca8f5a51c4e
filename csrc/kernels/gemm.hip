// bf16 MFMA GEMM for gfx950 with the layouts and epilogues of GPT training
// (every nn.Linear forward, input-grad and weight-grad).
//
//   C[M,N] (+)= A[M,K] · B[K,N]     fp32 accumulate, v_mfma_f32_16x16x32_bf16
//
// Operand storage (row-major torch tensors; `lda`/`ldb` are row strides):
//   A_K = true : A stored [M][K]   (forward X, input-grad dY)       -> ds_read_b128 fragments
//   A_K = false: A stored [K][M]   (weight-grad dY^T: dY is [M][N]) -> ds_read_b64_tr_b16 fragments
//   B_K = true : B stored [N][K]   (forward W: nn.Linear weight)    -> ds_read_b128
//   B_K = false: B stored [K][N]   (input-grad W, weight-grad X)    -> ds_read_b64_tr_b16
// so   forward      Y  = X · W^T     is <A_K=1, B_K=1>
//      input grad   dX = dY · W      is <A_K=1, B_K=0>
//      weight grad  dW = dY^T · X    is <A_K=0, B_K=0>, split over K (=tokens) with an
//                   fp32 atomic-add epilogue straight into the flat fp32 gradient buffer.
//
// Structure (cdna_hip_programming.md §5): 256x256 block tile, BK = 64, 8 waves as
// 2 (M) x 4 (N), each wave 128x64 = 8x4 16x16 accumulators (128 AGPR/VGPR).
// Tiles are staged global -> registers -> LDS (T14 split: loads for tile k+1 are
// issued before the MFMAs of tile k and written to the other LDS buffer after
// them; one barrier per K step).  LDS images are XOR-swizzled per 16-byte chunk
// (scripts/lds_swizzle_check.py: conflict-free for the b128 and tr16 patterns).
// The epilogue goes through LDS so that every global store / atomic wave
// instruction covers whole contiguous rows (256 B of fp32 for the atomics — the
// full-rate shape of MI355X_MICROARCH.md "Global float atomics").
// Block ids are remapped so that the blocks sharing an XCD (b % 8) walk
// neighbouring tiles (T1, bijective form).
#include "common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHREADS = 512;
constexpr int WAVES_M = 2, WAVES_N = 4;
constexpr int WTM = BM / WAVES_M;  // 128
constexpr int WTN = BN / WAVES_N;  // 64
constexpr int FM = WTM / 16;       // 8
constexpr int FN = WTN / 16;       // 4
constexpr int TILE_A_BYTES = BM * BK * 2;
constexpr int TILE_B_BYTES = BN * BK * 2;
constexpr int STAGE_BYTES = TILE_A_BYTES + TILE_B_BYTES;  // 64 KiB
constexpr int LDS_BYTES = 2 * STAGE_BYTES;                // 128 KiB
constexpr int EP_LD = 68;                                 // epilogue row pitch (fp32), +4 breaks bank aliasing
constexpr int EP_BYTES = (NTHREADS / 64) * 64 * EP_LD * 4;  // 136 KiB
constexpr int SMEM_BYTES = LDS_BYTES > EP_BYTES ? LDS_BYTES : EP_BYTES;

// EPI_STORE_F32: split z stores its fp32 partial tile to C + z * M * ldc (plain stores;
// the deterministic weight-gradient path sums the splits in a fixed order afterwards)
enum Epi : int { EPI_STORE_BF16 = 0, EPI_ATOMIC_F32 = 1, EPI_GELU = 2, EPI_DGELU = 3, EPI_STORE_F32 = 4 };

// ---- swizzled LDS addressing -------------------------------------------------
// K-contiguous image [rows][64]: 128-B rows, chunk' = chunk ^ ((row >> 1) & 7)
__device__ __forceinline__ int kimg(int row, int chunk) { return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4); }
// row-contiguous image [64][W]: 2W-byte rows, chunk' = chunk ^ 2*g(row), g = (r&3) | ((r>>3)&1)<<2
template <int W>
__device__ __forceinline__ int rimg(int row, int chunk) {
  const int g = (row & 3) | (((row >> 3) & 1) << 2);
  return row * (W * 2) + ((chunk ^ (2 * g)) << 4);
}

__device__ __forceinline__ bf16x8 as_frag(uint4 u) { return __builtin_bit_cast(bf16x8, u); }

__device__ __forceinline__ s16x4 lds_tr(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}

// operand fragment of 16 rows (or columns) x 32 k for the 16x16x32 MFMA
// lane l: element j = X[r0 + (l & 15)][k = 32*kk + 8*(l >> 4) + j]
template <bool KCONTIG, int W>
__device__ __forceinline__ bf16x8 load_frag(const char* tile, int r0, int kk, int lane) {
  if constexpr (KCONTIG) {
    return as_frag(*reinterpret_cast<const uint4*>(tile + kimg(r0 + (lane & 15), 4 * kk + (lane >> 4))));
  } else {
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
}

__device__ __forceinline__ float gelu_f(float x) { return nsa_gelu(x); }
__device__ __forceinline__ float gelu_grad(float x) { return nsa_gelu_grad(x); }

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;          // bf16 [M][ldc] or fp32 [M][ldc] (atomic epilogue)
  bf16_t* C2;       // EPI_GELU: gelu(acc) output (C holds the pre-activation)
  const bf16_t* U;  // EPI_DGELU: pre-activation whose gelu' scales acc
  int M, N, K;
  int lda, ldb, ldc;
  int k_per_split;  // unused by the kernels (kept for layout); splits cover 64-deep K blocks unevenly
  int tiles_m, tiles_n;
};

template <bool A_K, bool B_K, int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;

  // XCD-aware, bijective block -> tile remap (blocks b, b+8, ... share an XCD)
  const int nwg = g.tiles_m * g.tiles_n;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int tm = bid / g.tiles_n, tn = bid % g.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // split z owns K blocks [z*nkb/S, (z+1)*nkb/S): any split count, no K % (64*S) rule
  const int nkb = g.K / 64, kb0 = (int)blockIdx.z * nkb / (int)gridDim.z;
  const int k_begin = kb0 * 64;
  const int nk = (((int)blockIdx.z + 1) * nkb / (int)gridDim.z - kb0) * (64 / BK);

  // ---- global -> register staging: 4 x 16 B of A and 4 x 16 B of B per thread
  // (plain code, no lambdas: a by-reference capture of ra/rb sends them to scratch)
  uint4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
#define NSA_LOAD_A(c, dst, k0)                                                                   \
  {                                                                                              \
    const int e = tid + NTHREADS * (c);                                                          \
    if constexpr (A_K) {                                                                         \
      const int m = min(m0 + (e >> 3), g.M - 1);                                                 \
      dst = *reinterpret_cast<const uint4*>(g.A + (int64_t)m * g.lda + (k0) + (e & 7) * 8);      \
    } else {                                                                                     \
      const int m = min(m0 + (e & 31) * 8, g.M - 8);                                             \
      dst = *reinterpret_cast<const uint4*>(g.A + (int64_t)((k0) + (e >> 5)) * g.lda + m);       \
    }                                                                                            \
  }
#define NSA_LOAD_B(c, dst, k0)                                                                   \
  {                                                                                              \
    const int e = tid + NTHREADS * (c);                                                          \
    if constexpr (B_K) {                                                                         \
      const int n = min(n0 + (e >> 3), g.N - 1);                                                 \
      dst = *reinterpret_cast<const uint4*>(g.B + (int64_t)n * g.ldb + (k0) + (e & 7) * 8);      \
    } else {                                                                                     \
      const int n = min(n0 + (e & 31) * 8, g.N - 8);                                             \
      dst = *reinterpret_cast<const uint4*>(g.B + (int64_t)((k0) + (e >> 5)) * g.ldb + n);       \
    }                                                                                            \
  }
#define NSA_STORE_A(c, src, ta)                                                                  \
  {                                                                                              \
    const int e = tid + NTHREADS * (c);                                                          \
    if constexpr (A_K) *reinterpret_cast<uint4*>((ta) + kimg(e >> 3, e & 7)) = src;              \
    else *reinterpret_cast<uint4*>((ta) + rimg<BM>(e >> 5, e & 31)) = src;                       \
  }
#define NSA_STORE_B(c, src, tb)                                                                  \
  {                                                                                              \
    const int e = tid + NTHREADS * (c);                                                          \
    if constexpr (B_K) *reinterpret_cast<uint4*>((tb) + kimg(e >> 3, e & 7)) = src;              \
    else *reinterpret_cast<uint4*>((tb) + rimg<BN>(e >> 5, e & 31)) = src;                       \
  }
#define NSA_STAGE_LOAD(k0)                                                                       \
  {                                                                                              \
    NSA_LOAD_A(0, ra0, k0) NSA_LOAD_A(1, ra1, k0) NSA_LOAD_A(2, ra2, k0) NSA_LOAD_A(3, ra3, k0)  \
    NSA_LOAD_B(0, rb0, k0) NSA_LOAD_B(1, rb1, k0) NSA_LOAD_B(2, rb2, k0) NSA_LOAD_B(3, rb3, k0)  \
  }
#define NSA_STAGE_WRITE(buf)                                                                     \
  {                                                                                              \
    char* ta_ = smem + (buf) * STAGE_BYTES;                                                      \
    char* tb_ = ta_ + TILE_A_BYTES;                                                              \
    NSA_STORE_A(0, ra0, ta_) NSA_STORE_A(1, ra1, ta_) NSA_STORE_A(2, ra2, ta_) NSA_STORE_A(3, ra3, ta_) \
    NSA_STORE_B(0, rb0, tb_) NSA_STORE_B(1, rb1, tb_) NSA_STORE_B(2, rb2, tb_) NSA_STORE_B(3, rb3, tb_) \
  }

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  NSA_STAGE_LOAD(k_begin)
  NSA_STAGE_WRITE(0)
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) NSA_STAGE_LOAD(k_begin + (kt + 1) * BK)
    const char* ta = smem + cur * STAGE_BYTES;
    const char* tb = ta + TILE_A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = load_frag<A_K, BM>(ta, wm * WTM + 16 * i, kk, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = load_frag<B_K, BN>(tb, wn * WTN + 16 * j, kk, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) NSA_STAGE_WRITE(cur ^ 1)
    __syncthreads();
  }

  // ---- epilogue through LDS: per wave a private [64 rows][64 + 4 pad] fp32 region,
  // the 128-row wave tile in two halves of 64 rows.
  float* ep = reinterpret_cast<float*>(smem) + wave * 64 * EP_LD;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int ii = 0; ii < FM / 2; ++ii) {
      const int i = half * (FM / 2) + ii;
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) ep[(16 * ii + 4 * (lane >> 4) + e) * EP_LD + 16 * j + (lane & 15)] = acc[i][j][e];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int row_base = m0 + wm * WTM + half * 64;
    const int col_base = n0 + wn * WTN;
    if constexpr (EPI == EPI_ATOMIC_F32 || EPI == EPI_STORE_F32) {
      // one wave instruction = one 64-float (256 B) contiguous row segment
      float* C = reinterpret_cast<float*>(g.C);
      if constexpr (EPI == EPI_STORE_F32) C += (int64_t)blockIdx.z * g.M * g.ldc;
      const int col = col_base + lane;
      if (col < g.N) {
        for (int rr = 0; rr < 64; ++rr) {
          const int row = row_base + rr;
          if (row < g.M) {
            if constexpr (EPI == EPI_STORE_F32)
              C[(int64_t)row * g.ldc + col] = ep[rr * EP_LD + lane];
            else
              atomicAdd(C + (int64_t)row * g.ldc + col, ep[rr * EP_LD + lane]);
          }
        }
      }
    } else {
      // 16 lanes x 4 columns per row, 4 rows per wave instruction, 8-byte bf16 stores
      bf16_t* C = reinterpret_cast<bf16_t*>(g.C);
      const int c4 = (lane & 15) * 4;
      const int col = col_base + c4;
      for (int rr = lane >> 4; rr < 64; rr += 4) {
        const int row = row_base + rr;
        if (row < g.M && col < g.N) {
          const float4 v = *reinterpret_cast<const float4*>(ep + rr * EP_LD + c4);
          float o[4] = {v.x, v.y, v.z, v.w};
          const int64_t off = (int64_t)row * g.ldc + col;
          if constexpr (EPI == EPI_DGELU) {
            const uint2 u = *reinterpret_cast<const uint2*>(g.U + off);
            o[0] *= gelu_grad(__uint_as_float(u.x << 16));
            o[1] *= gelu_grad(__uint_as_float(u.x & 0xffff0000u));
            o[2] *= gelu_grad(__uint_as_float(u.y << 16));
            o[3] *= gelu_grad(__uint_as_float(u.y & 0xffff0000u));
          }
          uint2 w;
          w.x = pack2(o[0], o[1]);
          w.y = pack2(o[2], o[3]);
          *reinterpret_cast<uint2*>(C + off) = w;
          if constexpr (EPI == EPI_GELU) {
            // gelu of the bf16-rounded pre-activation, exactly what a separate kernel would see
            uint2 gv;
            gv.x = pack2(gelu_f(__uint_as_float(w.x << 16)), gelu_f(__uint_as_float(w.x & 0xffff0000u)));
            gv.y = pack2(gelu_f(__uint_as_float(w.y << 16)), gelu_f(__uint_as_float(w.y & 0xffff0000u)));
            *reinterpret_cast<uint2*>(g.C2 + off) = gv;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// ---------------------------------------------------------------------------
// Variant 1 ("ring"): same 256x256 tile / 8 waves / 2x4 wave grid, but K is
// staged in 32-deep slices by LDS-DMA (global_load_lds_dwordx4, no VGPRs) into a
// 4-slot LDS ring with TWO slices in flight: slice k+2 is issued while slice k
// is multiplied, and each wave waits only for slice k with a counted
// `s_waitcnt vmcnt(8)` folded into the raw `s_barrier` (never vmcnt(0) in the
// loop — cdna_hip_programming.md §5 "Pipelining across barriers", T3/T4).
// The DMA is issued from inline asm: with the builtin, hipcc sees a pending LDS
// write and drains vmcnt(0) before every ds_read.  Because the DMA destination is
// lane-linear, the XOR swizzle is applied to the per-lane GLOBAL source address
// (rule 21): image row r, physical chunk p holds logical chunk p ^ h(r).
// WAR: slice k+3 reuses the slot of slice k-2 (5 slots), whose last reads
// finished before every wave passed the barrier of iteration k-1.
// The MFMA operands are swapped (C^T = B^T A^T) so each lane's accumulator holds
// 4 consecutive output COLUMNS of one row: bf16 results are stored straight from
// registers as 8-byte pieces (no LDS round trip); only the fp32 atomic epilogue
// re-shapes through LDS into whole 256-B rows.
// ---------------------------------------------------------------------------
constexpr int RBK = 32;
constexpr int RSLOT_A = BM * RBK * 2;          // 16 KiB
constexpr int RSLOT_BYTES = 2 * RSLOT_A;       // A + B
template <int SLOTS>
struct RingGeo {
  static constexpr int BYTES = SLOTS * RSLOT_BYTES;
  static constexpr int SMEM = BYTES > EP_BYTES ? BYTES : EP_BYTES;
  static_assert(SMEM <= 163840, "LDS budget");
};

// K-contiguous [256][32] image: 64-B rows, chunk' = chunk ^ (((row >> 3) & 1) << 1)
__device__ __forceinline__ int kimg32(int row, int chunk) {
  return row * 64 + ((chunk ^ (((row >> 3) & 1) << 1)) << 4);
}

__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

template <bool KCONTIG>
__device__ __forceinline__ bf16x8 ring_frag(const char* tile, int r0, int lane) {
  if constexpr (KCONTIG) {
    return as_frag(*reinterpret_cast<const uint4*>(tile + kimg32(r0 + (lane & 15), lane >> 4)));
  } else {
    return load_frag<false, 256>(tile, r0, 0, lane);
  }
}

// Epilogue shared by the ring kernels.  fp32 atomics (and the non-DIRECT bf16
// variants) re-shape through LDS so that each wave instruction covers whole
// contiguous rows; DIRECT stores each lane's 4 consecutive columns from registers.
template <int EPI, bool DIRECT>
__device__ __forceinline__ void ring_epilogue(const GemmArgs& g, f32x4 (&acc)[FM][FN], char* smem, int m0, int n0,
                                              int wm, int wn, int lane, int wave) {
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);
  if constexpr (EPI == EPI_ATOMIC_F32 || EPI == EPI_STORE_F32 || !DIRECT) {
    // re-shape through LDS so each atomic wave-instruction covers one 256-B row
    __syncthreads();
    float* ep = reinterpret_cast<float*>(smem) + wave * 64 * EP_LD;
    float* C = reinterpret_cast<float*>(g.C);
    (void)C;
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
      if constexpr (EPI == EPI_ATOMIC_F32 || EPI == EPI_STORE_F32) {
        float* Cz = C;
        if constexpr (EPI == EPI_STORE_F32) Cz += (int64_t)blockIdx.z * g.M * g.ldc;
        const int col = n0 + wn * WTN + lane;
        if (col < g.N) {
          for (int rr = 0; rr < 64; ++rr) {
            const int row = row_base + rr;
            if (row < g.M) {
              if constexpr (EPI == EPI_STORE_F32)
                Cz[(int64_t)row * g.ldc + col] = ep[rr * EP_LD + lane];
              else
                atomicAdd(Cz + (int64_t)row * g.ldc + col, ep[rr * EP_LD + lane]);
            }
          }
        }
      } else {
        // 16 lanes x 4 columns = one 64-column row, 4 rows per wave instruction
        bf16_t* Cb = reinterpret_cast<bf16_t*>(g.C);
        const int c4 = (lane & 15) * 4;
        const int col = n0 + wn * WTN + c4;
        for (int rr = lane >> 4; rr < 64; rr += 4) {
          const int row = row_base + rr;
          if (row < g.M && col < g.N) {
            const float4 v = *reinterpret_cast<const float4*>(ep + rr * EP_LD + c4);
            float o[4] = {v.x, v.y, v.z, v.w};
            const int64_t off = (int64_t)row * g.ldc + col;
            if constexpr (EPI == EPI_DGELU) {
              const uint2 u = *reinterpret_cast<const uint2*>(g.U + off);
              o[0] *= gelu_grad(__uint_as_float(u.x << 16));
              o[1] *= gelu_grad(__uint_as_float(u.x & 0xffff0000u));
              o[2] *= gelu_grad(__uint_as_float(u.y << 16));
              o[3] *= gelu_grad(__uint_as_float(u.y & 0xffff0000u));
            }
            uint2 w;
            w.x = pack2(o[0], o[1]);
            w.y = pack2(o[2], o[3]);
            *reinterpret_cast<uint2*>(Cb + off) = w;
            if constexpr (EPI == EPI_GELU) {
              uint2 gv;
              gv.x = pack2(gelu_f(__uint_as_float(w.x << 16)), gelu_f(__uint_as_float(w.x & 0xffff0000u)));
              gv.y = pack2(gelu_f(__uint_as_float(w.y << 16)), gelu_f(__uint_as_float(w.y & 0xffff0000u)));
              *reinterpret_cast<uint2*>(g.C2 + off) = gv;
            }
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
  } else {
    bf16_t* C = reinterpret_cast<bf16_t*>(g.C);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = m0 + wm * WTM + 16 * i + lrow;
      if (row >= g.M) continue;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = n0 + wn * WTN + 16 * j + lcol;
        if (col >= g.N) continue;
        float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        const int64_t off = (int64_t)row * g.ldc + col;
        if constexpr (EPI == EPI_DGELU) {
          const uint2 u = *reinterpret_cast<const uint2*>(g.U + off);
          o[0] *= gelu_grad(__uint_as_float(u.x << 16));
          o[1] *= gelu_grad(__uint_as_float(u.x & 0xffff0000u));
          o[2] *= gelu_grad(__uint_as_float(u.y << 16));
          o[3] *= gelu_grad(__uint_as_float(u.y & 0xffff0000u));
        }
        uint2 w;
        w.x = pack2(o[0], o[1]);
        w.y = pack2(o[2], o[3]);
        *reinterpret_cast<uint2*>(C + off) = w;
        if constexpr (EPI == EPI_GELU) {
          uint2 gv;
          gv.x = pack2(gelu_f(__uint_as_float(w.x << 16)), gelu_f(__uint_as_float(w.x & 0xffff0000u)));
          gv.y = pack2(gelu_f(__uint_as_float(w.y << 16)), gelu_f(__uint_as_float(w.y & 0xffff0000u)));
          *reinterpret_cast<uint2*>(g.C2 + off) = gv;
        }
      }
    }
  }
}

// PIPE = true ("pipelined ring", variants 5/6): besides the slice DMA, the MFMA
// operand fragments are software-pipelined too.  Iteration k multiplies slice k
// from registers while it reads slice k+1's fragments out of LDS, interleaved with
// the MFMAs: A fragments are reloaded in place right after their last use, B
// fragments are double-buffered (named sets, unrolled by 2: no dynamic register
// indexing).  PMC counters of the plain ring showed every wave stalling on LDS
// reads right after each barrier (SQ_WAIT_INST_LDS ~5x hipBLASLt's); here the read
// latency hides under the MFMAs of the previous slice.  Slot reuse: the DMA of
// slice k+RSLOTS goes into slice k's slot, whose fragment reads every wave finished
// (lgkmcnt(0) folded into the barrier) before the barrier of iteration k.
template <bool A_K, bool B_K, int EPI, int RSLOTS, bool DIRECT, bool PIPE = false>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_ring_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[RingGeo<RSLOTS>::SMEM];
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
  const int nk = (((int)blockIdx.z + 1) * nkb / (int)gridDim.z - kb0) * (64 / RBK);
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  // per thread and slice: 2 DMA pieces of A and 2 of B (16 KiB each / 512 lanes / 16 B)
  auto issue = [&](int s) {
    const int k0 = k_begin + s * RBK;
    const uint32_t slot = lds0 + (uint32_t)((s % RSLOTS) * RSLOT_BYTES);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int e = j * NTHREADS + tid;  // 16-byte piece index == LDS byte offset / 16
      const uint32_t wbase = (uint32_t)((j * NTHREADS + wave * 64) * 16);
      const bf16_t* srcA;
      const bf16_t* srcB;
      if constexpr (A_K) {
        const int row = e >> 2, pc = e & 3;
        const int c = pc ^ (((row >> 3) & 1) << 1);
        srcA = g.A + (int64_t)min(m0 + row, g.M - 1) * g.lda + k0 + c * 8;
      } else {
        const int row = e >> 5, pc = e & 31;
        const int gg = (row & 3) | (((row >> 3) & 1) << 2);
        const int c = pc ^ (2 * gg);
        srcA = g.A + (int64_t)(k0 + row) * g.lda + min(m0 + c * 8, g.M - 8);
      }
      if constexpr (B_K) {
        const int row = e >> 2, pc = e & 3;
        const int c = pc ^ (((row >> 3) & 1) << 1);
        srcB = g.B + (int64_t)min(n0 + row, g.N - 1) * g.ldb + k0 + c * 8;
      } else {
        const int row = e >> 5, pc = e & 31;
        const int gg = (row & 3) | (((row >> 3) & 1) << 2);
        const int c = pc ^ (2 * gg);
        srcB = g.B + (int64_t)(k0 + row) * g.ldb + min(n0 + c * 8, g.N - 8);
      }
      glds16(srcA, __builtin_amdgcn_readfirstlane(slot + wbase));
      glds16(srcB, __builtin_amdgcn_readfirstlane(slot + RSLOT_A + wbase));
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if constexpr (PIPE) {
    // prologue: slices 0 .. RSLOTS-1 in flight, slice 0's fragments into registers
#pragma unroll
    for (int a = 0; a < RSLOTS; ++a)
      if (nk > a) issue(a);
    {
      const int younger0 = min(RSLOTS - 1, nk - 1);
      if (younger0 >= 3) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
      else if (younger0 == 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      else if (younger0 == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    bf16x8 af[FM], b0[FN], b1[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) b0[j] = ring_frag<B_K>(smem + RSLOT_A, wn * WTN + 16 * j, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = ring_frag<A_K>(smem, wm * WTM + 16 * i, lane);

// one pipelined iteration: wait for slice K+1 (own DMA) and every wave's reads of
// slice K, barrier, refill slice K's slot with slice K+RSLOTS, then MFMAs of slice K
// (registers BC / af) interleaved with the reads of slice K+1 (into af / BNX).
// Reads past the last slice hit a valid slot and are discarded (pad, don't branch).
#define NSA_PIPE_ITER(KK, BC, BNX)                                                              \
  {                                                                                           \
    const int k_ = (KK);                                                                      \
    const int younger = min(k_ + RSLOTS - 1, nk - 1) - (k_ + 1);                              \
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");  \
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");              \
    if (k_ + RSLOTS < nk) issue(k_ + RSLOTS);                                                 \
    const char* ta_ = smem + ((k_ + 1) % RSLOTS) * RSLOT_BYTES;                               \
    const char* tb_ = ta_ + RSLOT_A;                                                          \
    __builtin_amdgcn_s_setprio(1);                                                            \
    _Pragma("unroll") for (int i = 0; i < FM; ++i) {                                          \
      _Pragma("unroll") for (int j = 0; j < FN; ++j)                                          \
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(BC[j], af[i], acc[i][j], 0, 0, 0); \
      af[i] = ring_frag<A_K>(ta_, wm * WTM + 16 * i, lane);                                   \
      if (i < FN) BNX[i] = ring_frag<B_K>(tb_, wn * WTN + 16 * i, lane);                      \
    }                                                                                         \
    __builtin_amdgcn_s_setprio(0);                                                            \
  }

    for (int k = 0; k < nk; k += 2) {
      NSA_PIPE_ITER(k, b0, b1)
      if (k + 1 < nk) NSA_PIPE_ITER(k + 1, b1, b0)
    }
#undef NSA_PIPE_ITER
  } else {
  constexpr int AHEAD = RSLOTS - 2;  // slices in flight beyond the one being multiplied
    // prologue: slices 0 .. AHEAD-1; the loop issues slice k + AHEAD at iteration k
  #pragma unroll
    for (int a = 0; a < AHEAD; ++a)
      if (nk > a) issue(a);
    for (int k = 0; k < nk; ++k) {
      // wait for slice k; the younger slices (up to AHEAD, 4 DMA pieces each) may stay in flight
      const int younger = min(AHEAD, nk - 1 - k);
      if (k + AHEAD < nk) issue(k + AHEAD);
      if constexpr (AHEAD == 3) {
        if (younger == 3) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
        else if (younger == 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        if (younger == 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
        else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
      }
      const char* ta = smem + (k % RSLOTS) * RSLOT_BYTES;
      const char* tb = ta + RSLOT_A;
      bf16x8 af[FM], bfr[FN];
  #pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = ring_frag<B_K>(tb, wn * WTN + 16 * j, lane);
  #pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = ring_frag<A_K>(ta, wm * WTM + 16 * i, lane);
      __builtin_amdgcn_s_setprio(1);
  #pragma unroll
      for (int i = 0; i < FM; ++i)
  #pragma unroll
        for (int j = 0; j < FN; ++j)  // swapped operands: acc[i][j][e] = C[16i + (l&15)][16j + 4(l>>4) + e]
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ring_epilogue<EPI, DIRECT>(g, acc, smem, m0, n0, wm, wn, lane, wave);
}


// ---------------------------------------------------------------------------
// Variants 7/8 ("ring64"): LDS-DMA slots 64 deep in K, so every DMA row of a
// K-contiguous operand is a whole 128-B line (the 32-deep ring fetches 64-B
// half-lines: twice the TA work, measured as the NT forward's deficit), laid out
// as the register-staged kernel's images (kimg / rimg<256>, swizzle applied to
// the per-lane global source).  Two 64 KiB slots; each slot is multiplied as two
// 32-deep sub-slices with the fragment pipeline (reads of the next sub-slice
// under the MFMAs of the current one: A in place, B double-buffered):
//   phase A: MFMA(k, 0) | read (k, 1)           (same slot, no barrier)
//   wait own DMA of slot k+1 + lgkmcnt(0), barrier, DMA slot k+2 -> slot k's buffer
//   phase B: MFMA(k, 1) | read (k+1, 0)
// Slot k's buffer is free at that barrier: its (k,0) reads completed before phase
// A's MFMAs and its (k,1) reads before the barrier, in every wave.
// ---------------------------------------------------------------------------
constexpr int R64_SLOT_A = BM * 64 * 2;   // 32 KiB
constexpr int R64_SLOT = 2 * R64_SLOT_A;  // A + B
constexpr int R64_SMEM = 2 * R64_SLOT > EP_BYTES ? 2 * R64_SLOT : EP_BYTES;

template <bool A_K, bool B_K, int EPI, bool DIRECT>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_ring64_kernel(GemmArgs g) {
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
      const bf16_t* srcA;
      const bf16_t* srcB;
      if constexpr (A_K) {
        const int row = e >> 3, c = (e & 7) ^ ((row >> 1) & 7);
        srcA = g.A + (int64_t)min(m0 + row, g.M - 1) * g.lda + k0 + c * 8;
      } else {
        const int row = e >> 5;
        const int gg = (row & 3) | (((row >> 3) & 1) << 2);
        const int c = (e & 31) ^ (2 * gg);
        srcA = g.A + (int64_t)(k0 + row) * g.lda + min(m0 + c * 8, g.M - 8);
      }
      if constexpr (B_K) {
        const int row = e >> 3, c = (e & 7) ^ ((row >> 1) & 7);
        srcB = g.B + (int64_t)min(n0 + row, g.N - 1) * g.ldb + k0 + c * 8;
      } else {
        const int row = e >> 5;
        const int gg = (row & 3) | (((row >> 3) & 1) << 2);
        const int c = (e & 31) ^ (2 * gg);
        srcB = g.B + (int64_t)(k0 + row) * g.ldb + min(n0 + c * 8, g.N - 8);
      }
      glds16(srcA, __builtin_amdgcn_readfirstlane(slot + wbase));
      glds16(srcB, __builtin_amdgcn_readfirstlane(slot + R64_SLOT_A + wbase));
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
  for (int j = 0; j < FN; ++j) b0[j] = load_frag<B_K, BN>(smem + R64_SLOT_A, wn * WTN + 16 * j, 0, lane);
#pragma unroll
  for (int i = 0; i < FM; ++i) af[i] = load_frag<A_K, BM>(smem, wm * WTM + 16 * i, 0, lane);

#define NSA_R64_PHASE(BC, BNX, TA, TB, KKN)                                                     \
  __builtin_amdgcn_s_setprio(1);                                                              \
  _Pragma("unroll") for (int i = 0; i < FM; ++i) {                                            \
    _Pragma("unroll") for (int j = 0; j < FN; ++j)                                            \
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(BC[j], af[i], acc[i][j], 0, 0, 0);   \
    af[i] = load_frag<A_K, BM>((TA), wm * WTM + 16 * i, (KKN), lane);                         \
    if (i < FN) BNX[i] = load_frag<B_K, BN>((TB), wn * WTN + 16 * i, (KKN), lane);            \
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
  ring_epilogue<EPI, DIRECT>(g, acc, smem, m0, n0, wm, wn, lane, wave);
}

// ---------------------------------------------------------------------------
// Variant 11 ("w4"): the ring64 pipeline with 4 waves (one per SIMD) that each own
// a 128x128 quarter of the 256x256 tile (8x8 accumulators = 256 registers, which
// the compiler keeps in AGPRs: nothing but the MFMAs touches them in the loop).
// Per 64-deep K-tile the 8-wave layout (128x64 per wave) reads
// 8 x (128 + 64) x 128 B = 192 KiB of fragments from LDS; 4 x (128 + 128) x 128 B
// = 128 KiB here, for the same 64 KiB of DMA writes and the same MFMA count, which
// is what bounds the transposed-read weight-gradient layout (every fragment a pair
// of ds_read_b64_tr_b16).  Slot protocol, swizzles and DMA geometry as ring64,
// with 8 DMA pieces per thread and operand per slot instead of 4.
// ---------------------------------------------------------------------------
constexpr int W4_THREADS = 256;
constexpr int W4_WT = 128;            // wave tile (both dims)
constexpr int W4_F = W4_WT / 16;      // 8 fragments per dim

// MFMA with its accumulator tied to one AGPR tuple (in/out operand).  With all 256
// AGPRs holding loop-carried accumulators, the builtin's untied form lets the
// register allocator pick a different destination and rotate the tuples back with
// ~256 v_accvgpr moves per iteration.  The hazards the compiler does not see through
// the asm are covered by the caller: chains start with mfma_first (no VALU
// initialisation to wait for) and wait states precede the epilogue's reads; operand VGPRs come straight
// from LDS reads (lgkmcnt waits are inserted for asm operands as for any use).
__device__ __forceinline__ void mfma_tied(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// first product of a chain: accumulator operand = inline constant 0 (no VALU init)
__device__ __forceinline__ void mfma_first(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}

// FM_ x FN_ accumulators of 16x16 per wave (wave tile 16 FM_ x 16 FN_), 2 x 2 waves
template <int EPI, int FM_ = W4_F, int FN_ = W4_F>
__device__ __forceinline__ void w4_epilogue(const GemmArgs& g, f32x4 (&acc)[FM_][FN_], char* smem, int m0, int n0,
                                            int wm, int wn, int lane, int wave) {
  constexpr int WM_ = 16 * FM_, WN_ = 16 * FN_;
  const int lrow = lane & 15, lcol = 4 * (lane >> 4);
  if constexpr (EPI == EPI_ATOMIC_F32 || EPI == EPI_STORE_F32) {
    // re-shape each 64x64 quarter of the wave tile through LDS: one 256-B row per
    // atomic / store wave-instruction
    __syncthreads();
    float* ep = reinterpret_cast<float*>(smem) + wave * 64 * EP_LD;
    float* Cz = reinterpret_cast<float*>(g.C);
    if constexpr (EPI == EPI_STORE_F32) Cz += (int64_t)blockIdx.z * g.M * g.ldc;
#pragma unroll
    for (int q = 0; q < (FM_ / 4) * (FN_ / 4); ++q) {
      const int hm = q / (FN_ / 4), hn = q % (FN_ / 4);
#pragma unroll
      for (int ii = 0; ii < 4; ++ii)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const f32x4 v = acc[hm * 4 + ii][hn * 4 + jj];
          *reinterpret_cast<float4*>(ep + (16 * ii + lrow) * EP_LD + 16 * jj + lcol) = make_float4(v[0], v[1], v[2], v[3]);
        }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int row_base = m0 + wm * WM_ + hm * 64;
      const int col = n0 + wn * WN_ + hn * 64 + lane;
      if (col < g.N) {
        for (int rr = 0; rr < 64; ++rr) {
          const int row = row_base + rr;
          if (row < g.M) {
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
  } else {
    bf16_t* C = reinterpret_cast<bf16_t*>(g.C);
#pragma unroll
    for (int i = 0; i < FM_; ++i) {
      const int row = m0 + wm * WM_ + 16 * i + lrow;
      if (row >= g.M) continue;
#pragma unroll
      for (int j = 0; j < FN_; ++j) {
        const int col = n0 + wn * WN_ + 16 * j + lcol;
        if (col >= g.N) continue;
        float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        const int64_t off = (int64_t)row * g.ldc + col;
        if constexpr (EPI == EPI_DGELU) {
          const uint2 u = *reinterpret_cast<const uint2*>(g.U + off);
          o[0] *= gelu_grad(__uint_as_float(u.x << 16));
          o[1] *= gelu_grad(__uint_as_float(u.x & 0xffff0000u));
          o[2] *= gelu_grad(__uint_as_float(u.y << 16));
          o[3] *= gelu_grad(__uint_as_float(u.y & 0xffff0000u));
        }
        uint2 w;
        w.x = pack2(o[0], o[1]);
        w.y = pack2(o[2], o[3]);
        *reinterpret_cast<uint2*>(C + off) = w;
        if constexpr (EPI == EPI_GELU) {
          uint2 gv;
          gv.x = pack2(gelu_f(__uint_as_float(w.x << 16)), gelu_f(__uint_as_float(w.x & 0xffff0000u)));
          gv.y = pack2(gelu_f(__uint_as_float(w.y << 16)), gelu_f(__uint_as_float(w.y & 0xffff0000u)));
          *reinterpret_cast<uint2*>(g.C2 + off) = gv;
        }
      }
    }
  }
}

template <bool A_K, bool B_K, int EPI>
__global__ __launch_bounds__(W4_THREADS, 1) void gemm_w4_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[2 * R64_SLOT];  // 128 KiB (epilogue: 4 x 17 KiB)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
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

  // per thread and slot: 8 DMA pieces of A and 8 of B (32 KiB each / 256 lanes / 16 B)
  auto issue = [&](int s) {
    const int k0 = k_begin + s * 64;
    const uint32_t slot = lds0 + (uint32_t)((s & 1) * R64_SLOT);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = j * W4_THREADS + tid;
      const uint32_t wbase = (uint32_t)((j * W4_THREADS + wave * 64) * 16);
      const bf16_t* srcA;
      const bf16_t* srcB;
      if constexpr (A_K) {
        const int row = e >> 3, c = (e & 7) ^ ((row >> 1) & 7);
        srcA = g.A + (int64_t)min(m0 + row, g.M - 1) * g.lda + k0 + c * 8;
      } else {
        const int row = e >> 5;
        const int gg = (row & 3) | (((row >> 3) & 1) << 2);
        const int c = (e & 31) ^ (2 * gg);
        srcA = g.A + (int64_t)(k0 + row) * g.lda + min(m0 + c * 8, g.M - 8);
      }
      if constexpr (B_K) {
        const int row = e >> 3, c = (e & 7) ^ ((row >> 1) & 7);
        srcB = g.B + (int64_t)min(n0 + row, g.N - 1) * g.ldb + k0 + c * 8;
      } else {
        const int row = e >> 5;
        const int gg = (row & 3) | (((row >> 3) & 1) << 2);
        const int c = (e & 31) ^ (2 * gg);
        srcB = g.B + (int64_t)(k0 + row) * g.ldb + min(n0 + c * 8, g.N - 8);
      }
      glds16(srcA, __builtin_amdgcn_readfirstlane(slot + wbase));
      glds16(srcB, __builtin_amdgcn_readfirstlane(slot + R64_SLOT_A + wbase));
    }
  };

  f32x4 acc[W4_F][W4_F];  // first written by the zero-accumulator MFMAs of K-tile 0

  issue(0);
  if (nk > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  bf16x8 af[W4_F], b0[W4_F], b1[W4_F];
#pragma unroll
  for (int j = 0; j < W4_F; ++j) b0[j] = load_frag<B_K, BN>(smem + R64_SLOT_A, wn * W4_WT + 16 * j, 0, lane);
#pragma unroll
  for (int i = 0; i < W4_F; ++i) af[i] = load_frag<A_K, BM>(smem, wm * W4_WT + 16 * i, 0, lane);

#define NSA_W4_PHASE(BC, BNX, TA, TB, KKN, FIRST)                                              \
  __builtin_amdgcn_s_setprio(1);                                                             \
  _Pragma("unroll") for (int i = 0; i < W4_F; ++i) {                                         \
    _Pragma("unroll") for (int j = 0; j < W4_F; ++j) {                                       \
      if (FIRST)                                                                             \
        mfma_first(acc[i][j], BC[j], af[i]);                                                 \
      else                                                                                   \
        mfma_tied(acc[i][j], BC[j], af[i]);                                                  \
    }                                                                                        \
    if (i < W4_F / 2) { /* B early: the next phase's first row needs all of them */           \
      BNX[2 * i] = load_frag<B_K, BN>((TB), wn * W4_WT + 32 * i, (KKN), lane);                 \
      BNX[2 * i + 1] = load_frag<B_K, BN>((TB), wn * W4_WT + 32 * i + 16, (KKN), lane);        \
    }                                                                                        \
    af[i] = load_frag<A_K, BM>((TA), wm * W4_WT + 16 * i, (KKN), lane);                      \
  }                                                                                          \
  __builtin_amdgcn_s_setprio(0);

  // the loop body is branch-free (its last two iterations are peeled): a branch
  // between the MFMA phases makes the register allocator copy the 256 loop-carried
  // AGPR accumulators at the loop header
#define NSA_W4_STEP(K, WAIT, ISS, FIRST)                                                       \
  {                                                                                          \
    const char* ta = smem + ((K) & 1) * R64_SLOT;                                            \
    const char* tn = smem + (((K) + 1) & 1) * R64_SLOT; /* past the end: discarded reads */  \
    NSA_W4_PHASE(b0, b1, ta, ta + R64_SLOT_A, 1, FIRST)                                      \
    if (WAIT) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");      \
    if (ISS) issue((K) + 2);                                                                 \
    NSA_W4_PHASE(b1, b0, tn, tn + R64_SLOT_A, 0, false)                                      \
  }
  if (nk == 1) {
    NSA_W4_STEP(0, false, false, true)
  } else if (nk == 2) {
    NSA_W4_STEP(0, true, false, true)
    NSA_W4_STEP(1, false, false, false)
  } else {
    NSA_W4_STEP(0, true, true, true)
    int k = 1;
    for (; k + 2 < nk; ++k) NSA_W4_STEP(k, true, true, false)
    NSA_W4_STEP(k, true, false, false)
    NSA_W4_STEP(k + 1, false, false, false)
  }
#undef NSA_W4_STEP
#undef NSA_W4_PHASE
  // last MFMA results -> VALU / LDS reads of the accumulators: 18 wait states cover the
  // 8-pass MFMA's write latency
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  w4_epilogue<EPI>(g, acc, smem, m0, n0, wm, wn, lane, wave);
}

// ---------------------------------------------------------------------------
// Variants 9/10 ("p8": phase-paired, persistent).  cdna_hip_programming.md §5's
// 256² 8-phase structure, re-derived for the GPT layouts (A K-contiguous:
// forward NT and input-grad NN):
//  * a K-tile (64 deep, 64 KiB: A image [256][64] kimg + B image) is computed in
//    4 PHASES of 16 MFMAs, one 64x32 output quadrant (qm, qn) per phase, in the
//    order (0,0) (0,1) (1,1) (1,0); fragments are read from LDS at the head of
//    the phase that uses them: p0 A[qm0]+B[qn0], p1 B[qn1], p2 A[qm1], p3 none
//    (B[qn0] kept in a second register set);
//  * each K-tile is staged as 4 HALF-TILES of 16 KiB (2 LDS-DMA per thread), one
//    per phase, issued 6 phases ahead in the order  A0 B0 B1 A1  where A0/A1 are
//    the rows of quadrant qm = 0/1 and B0/B1 the columns of qn = 0/1 (K-contiguous
//    B) or the k rows 0-31/32-63 (B stored [K][N]) — every DMA row a whole line.
//    A half-tile's slot was last read 2+ phases before its refill is issued
//    (A0 <- p0, B0 <- p0 / p1, B1 <- p1, A1 <- p2), and every phase ends its DMA
//    issue with a counted vmcnt that retires the half-tile issued 4 phases
//    earlier (3 stay in flight); a half-tile is read >= 1 phase after that wait;
//  * 8 waves = 2 groups (wm = 0/1, one wave of each per SIMD) staggered by one
//    barrier: each phase is [reads + DMA + vmcnt | barrier | 16 MFMA | barrier],
//    so one group's LDS reads run beside the other group's MFMAs on every SIMD
//    (MI355X_MICROARCH.md "Two waves per SIMD"); raw s_barrier only (a
//    __syncthreads would drain the DMA with vmcnt(0));
//  * persistent: grid = min(tiles, 256); the next tile's first 6 half-tiles are
//    issued before this tile's epilogue, which stores straight from registers,
//    so the K-loop prologue hides under the stores.  Tiles are walked in a
//    grouped order (GM row-blocks x all columns) inside each XCD's contiguous
//    share (bijective remap: blocks b, b+8, ... share an XCD).
// Measured (scripts/gemm_ab.py, M = 122880, random operands, profiles/r1_gemm_p8_probes.md):
// the structure alone (NSA_P8_PROBE_NODMA) runs 1650 TF/s at K = 3072, but with
// the LDS-DMA staging it is ~1000 TF/s (hipBLASLt 1300); not waiting on vmcnt
// (NSA_P8_PROBE_NOWAIT) or L2-resident operands (NSA_P8_PROBE_L2) recover <5 %,
// one DMA piece per phase instead of two (NSA_P8_PIECES=1) ~8 %: the cost is
// the DMA's presence in the read segments, not its latency or HBM traffic.
// Kept as an autotuner candidate / experiment, not selected by default.
// ---------------------------------------------------------------------------
#ifndef NSA_P8_DMA_POS
#define NSA_P8_DMA_POS 0  // where a phase issues its DMA: 0 after its LDS reads, 1 before them, 2 in its MFMAs
#endif
#ifndef NSA_P8_PIECES
#define NSA_P8_PIECES 2  // DMA pieces per wave and half-tile (1 = timing probe, half the bytes)
#endif
constexpr int P8_HALF = 16384;               // bytes per half-tile
constexpr int P8_BUF = 4 * P8_HALF;          // one K-tile: A image (32 KiB) + B image (32 KiB)
constexpr int P8_SMEM = 2 * P8_BUF;          // 128 KiB
constexpr int P8_GM = 4;                     // grouped tile order: row-blocks per group

__device__ __forceinline__ void p8_wait(int inflight) {
#ifdef NSA_P8_PROBE_NOWAIT
  if (inflight > 0) return;  // timing probe: only the drains at the end of a tile wait
#endif
  // vmcnt = 2 DMA instructions per half-tile still allowed in flight
  if (inflight >= 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (inflight == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (inflight == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (inflight == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void p8_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <bool B_K, int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void gemm_p8_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[P8_SMEM];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int nk = g.K / 64;
  const int nh = 4 * nk;  // half-tiles per output tile
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  // DMA geometry of the 4 half-tile kinds (2 pieces of 1 KiB per wave each),
  // computed per issue (wave-uniform bases + lane bits: no live registers).
  // A (kimg [256][64], 128-B rows): half qh = rows (r >> 6 & 1) == qh, piece pc
  // (16 per half) = 8 rows.  B K-contiguous: half qh = rows wn*64 + qh*32 + [0,32).
  // B [K][N] (rimg<256>, 512-B rows): half kh = k rows kh*32 + [0,32), 2 rows/piece.
  const int tiles = g.tiles_m * g.tiles_n;
  const int G = gridDim.x;
  auto tile_of = [&](int seq, int& m0, int& n0) {
    // bijective XCD remap of the virtual grid [0, tiles), then grouped order
    const int xcd = seq % 8, q = tiles / 8, r = tiles % 8;
    const int t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + seq / 8;
    const int grp = t / (P8_GM * g.tiles_n);
    const int first = grp * P8_GM;
    const int gm = min(P8_GM, g.tiles_m - first);
    const int in = t - grp * P8_GM * g.tiles_n;
    m0 = (first + in % gm) * BM;
    n0 = (in / gm) * BN;
  };

  // issue half-tile h (= 4 * ktile + kind) of the tile at (m0, n0)
  auto issue = [&](int h, int m0, int n0) {
    const int kt = h >> 2, kind = h & 3;
#ifdef NSA_P8_PROBE_L2
    const int k0 = 0;  // timing probe: every K-tile re-reads the first one (L2-resident operands)
#else
    const int k0 = kt * 64;
#endif
    const uint32_t buf = lds0 + (uint32_t)((kt & 1) * P8_BUF);
#ifdef NSA_P8_PROBE_NODMA
    return;  // timing probe: no staging at all (wrong results)
#endif
    if (kind == 0 || kind == 3) {
      const int qh = kind == 3;
#pragma unroll
      for (int j = 0; j < NSA_P8_PIECES; ++j) {
        const int pc = wave * 2 + j;
        const int rb = (pc >> 3) * 128 + qh * 64 + (pc & 7) * 8;  // wave-uniform
        const int row = rb + (lane >> 3);
        const int col = ((lane & 7) ^ ((row >> 1) & 7)) * 8;
        const bf16_t* src = g.A + (int64_t)min(m0 + row, g.M - 1) * g.lda + k0 + col;
        glds16(src, __builtin_amdgcn_readfirstlane(buf + (uint32_t)(rb * 128)));
      }
    } else {
      const int qh = kind == 2;
#pragma unroll
      for (int j = 0; j < NSA_P8_PIECES; ++j) {
        const int pc = wave * 2 + j;
        const bf16_t* src;
        uint32_t off;
        if constexpr (B_K) {
          const int rb = (pc >> 2) * 64 + qh * 32 + (pc & 3) * 8;
          const int row = rb + (lane >> 3);
          const int col = ((lane & 7) ^ ((row >> 1) & 7)) * 8;
          src = g.B + (int64_t)min(n0 + row, g.N - 1) * g.ldb + k0 + col;
          off = (uint32_t)(rb * 128);
        } else {
          const int kb = qh * 32 + pc * 2;
          const int krow = kb + (lane >> 5);
          const int gg = (krow & 3) | (((krow >> 3) & 1) << 2);
          const int col = ((lane & 31) ^ (2 * gg)) * 8;
          src = g.B + (int64_t)(k0 + krow) * g.ldb + min(n0 + col, g.N - 8);
          off = (uint32_t)(kb * 512);
        }
        glds16(src, __builtin_amdgcn_readfirstlane(buf + 2 * P8_HALF + off));
      }
    }
  };
  auto prologue = [&](int m0, int n0) {
    const int pre = min(6, nh);
    for (int h = 0; h < pre; ++h) issue(h, m0, n0);
  };

  int seq = blockIdx.x;
  if (seq >= tiles) return;
  int m0, n0;
  tile_of(seq, m0, n0);
  prologue(m0, n0);

  while (true) {
    // K-tile 0 resident (half-tiles 0..3); 4 and 5 may stay in flight
    p8_wait(min(6, nh) - 4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    p8_barrier();
    if (wm == 1) p8_barrier();  // stagger: group 1 runs one barrier behind group 0

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 af[4][2], b0f[2][2], b1f[2][2];

    for (int kt = 0; kt < nk; ++kt) {
      const char* ta = smem + (kt & 1) * P8_BUF;
      const char* tb = ta + 2 * P8_HALF;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int P = 4 * kt + p;
#if NSA_P8_DMA_POS == 1
        if (P + 6 < nh) issue(P + 6, m0, n0);  // probe: DMA ahead of the fragment reads
#endif
        // ---- LDS reads of this phase's fragments
        if (p == 0 || p == 2) {
          const int qm = p >> 1;
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
              af[i][kk] = load_frag<true, BM>(ta, wm * WTM + qm * 64 + 16 * i, kk, lane);
        }
        if (p == 0) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) b0f[j][kk] = load_frag<B_K, BN>(tb, wn * WTN + 16 * j, kk, lane);
        }
        if (p == 1) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
              b1f[j][kk] = load_frag<B_K, BN>(tb, wn * WTN + 32 + 16 * j, kk, lane);
        }
        // ---- DMA of half-tile P + 6, then retire what phase P + 1 reads: half-tile
        // P + 2 (issued 4 phases ago; 3 stay in flight) — or P + 3 when B is stored
        // [K][N]: its k-halves are kinds 1 and 2 and phase 0 reads both
#if NSA_P8_DMA_POS == 0
        if (P + 6 < nh) issue(P + 6, m0, n0);
        if constexpr (B_K)
          p8_wait(min(4, max(0, nh - P - 3)));
        else
          p8_wait(min(3, max(0, nh - P - 4)));
#elif NSA_P8_DMA_POS == 1
        if constexpr (B_K)
          p8_wait(min(4, max(0, nh - P - 3)));
        else
          p8_wait(min(3, max(0, nh - P - 4)));
#else
        // probe: this phase's DMA is issued inside its MFMA cluster (below), so it is
        // not yet among the younger operations here
        if constexpr (B_K)
          p8_wait(min(3, max(0, nh - P - 3)));
        else
          p8_wait(min(2, max(0, nh - P - 4)));
#endif
        p8_barrier();
        // ---- 16 MFMAs of quadrant (qm, qn): (0,0) (0,1) (1,1) (1,0)
        __builtin_amdgcn_s_setprio(1);
        {
          const int qm = p >> 1;
          const bool q1 = (p == 1 || p == 2);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
              for (int kk = 0; kk < 2; ++kk) {
                const bf16x8 bb = q1 ? b1f[j][kk] : b0f[j][kk];
                acc[qm * 4 + i][(q1 ? 2 : 0) + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                    bb, af[i][kk], acc[qm * 4 + i][(q1 ? 2 : 0) + j], 0, 0, 0);
#if NSA_P8_DMA_POS == 2
                if (i == 0 && j == 1 && kk == 1 && P + 6 < nh) issue(P + 6, m0, n0);
#endif
              }
        }
        __builtin_amdgcn_s_setprio(0);
        p8_barrier();
      }
    }
    if (wm == 0) p8_barrier();  // close the stagger: both groups at the same barrier count
    // every wave's reads of both buffers are complete: the next tile may refill them
    const int nseq = seq + G;
    int nm0 = 0, nn0 = 0;
    const bool more = nseq < tiles;
    if (more) {
      tile_of(nseq, nm0, nn0);
      prologue(nm0, nn0);
    }
    ring_epilogue<EPI, true>(g, acc, smem, m0, n0, wm, wn, lane, wave);
    if (!more) break;
    // stores and the prologue DMA share vmcnt: retire everything before the loop's wait
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    seq = nseq;
    m0 = nm0;
    n0 = nn0;
  }
}

// ---------------------------------------------------------------------------
// Variants 12/13 ("w4 ring", weight-gradient layout only: A and B stored [K][rows]):
// the w4 wave geometry fed by an NS-slot ring of 32-deep slices (NS = 4 / 5, 32 KiB
// each), one slice per MFMA phase.  Top of phase j: wait for this wave's DMA of slice
// j+1 (slices up to j+NS-2 may stay in flight), barrier, DMA slice j+NS-1 into the
// slot of slice j-1 (read in phase j-2, consumed by phase j-1's MFMAs, so every wave
// is done with it); then 64 MFMAs on slice j (registers) | fragment reads of slice j+1.
// No lgkmcnt(0) at the barrier, and the DMA lead is NS-2 phases (2048 / 3072 MFMA
// cycles) instead of the 2-slot ring's one 64-deep K step.
// ---------------------------------------------------------------------------
constexpr int W4R_SLICE = 32;

template <int N>
__device__ __forceinline__ void vm_wait_n() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Generalised to a 2 x 2 wave grid of 16 FM_ x 16 FN_ wave tiles (block tile
// 32 FM_ x 32 FN_): variants 12 / 13 are FM_ = FN_ = 8 (one 256x256 workgroup per CU,
// one wave per SIMD); variants 14-16 use 64- or 128-row wave tiles and small enough
// rings that 2-3 independent workgroups share a CU, so one workgroup's barrier and
// DMA waits run beside another's MFMAs (the flash dK/dV kernel's k1w4 geometry).
template <int EPI, int NS, int FM_, int FN_, int MINW>
__global__ __launch_bounds__(W4_THREADS, MINW) void gemm_w4r_kernel(GemmArgs g) {
  constexpr int BM_ = 32 * FM_, BN_ = 32 * FN_;
  constexpr int OPER_A = W4R_SLICE * BM_ * 2, OPER_B = W4R_SLICE * BN_ * 2;
  constexpr int SLOT = OPER_A + OPER_B;
  constexpr int PA = OPER_A / 16 / W4_THREADS, PB = OPER_B / 16 / W4_THREADS;  // DMA pieces per thread
  constexpr int PIECES = PA + PB;
  constexpr int EPI_BYTES = 4 * 64 * EP_LD * 4;  // epilogue: one 64x64 fp32 staging tile per wave
  constexpr int SMEM = NS * SLOT > EPI_BYTES ? NS * SLOT : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  static_assert(SMEM <= 163840, "LDS budget");
  static_assert(PA >= 1 && PB >= 1 && FM_ % 4 == 0 && FN_ % 4 == 0, "geometry");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = g.tiles_m * g.tiles_n;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int tm = bid / g.tiles_n, tn = bid % g.tiles_n;
  const int m0 = tm * BM_, n0 = tn * BN_;
  // splits own whole 64-deep blocks (as every other variant); slices are 32 deep
  const int nkb = g.K / 64, kb0 = (int)blockIdx.z * nkb / (int)gridDim.z;
  const int k_begin = kb0 * 64;
  const int ns = 2 * (((int)blockIdx.z + 1) * nkb / (int)gridDim.z - kb0);  // slices
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  // slice s -> slot: [32][BM_] and [32][BN_] rimg images, PA + PB DMA pieces per thread
  auto issue = [&](int s, int slot_idx) {
    const int k0 = k_begin + s * W4R_SLICE;
    const uint32_t slot = lds0 + (uint32_t)(slot_idx * SLOT);
#pragma unroll
    for (int j = 0; j < PA; ++j) {
      const int e = j * W4_THREADS + tid;
      const uint32_t wbase = (uint32_t)((j * W4_THREADS + wave * 64) * 16);
      const int row = e / (BM_ / 8);
      const int gg = (row & 3) | (((row >> 3) & 1) << 2);
      const int c = (e % (BM_ / 8)) ^ (2 * gg);
      glds16(g.A + (int64_t)(k0 + row) * g.lda + min(m0 + c * 8, g.M - 8),
             __builtin_amdgcn_readfirstlane(slot + wbase));
    }
#pragma unroll
    for (int j = 0; j < PB; ++j) {
      const int e = j * W4_THREADS + tid;
      const uint32_t wbase = (uint32_t)((j * W4_THREADS + wave * 64) * 16);
      const int row = e / (BN_ / 8);
      const int gg = (row & 3) | (((row >> 3) & 1) << 2);
      const int c = (e % (BN_ / 8)) ^ (2 * gg);
      glds16(g.B + (int64_t)(k0 + row) * g.ldb + min(n0 + c * 8, g.N - 8),
             __builtin_amdgcn_readfirstlane(slot + OPER_A + wbase));
    }
  };
  // wait until at most `n` younger slices' DMA are in flight
  auto wait_slices = [&](int n) {
    if (n >= 3) vm_wait_n<3 * PIECES>();
    else if (n == 2) vm_wait_n<2 * PIECES>();
    else if (n == 1) vm_wait_n<PIECES>();
    else vm_wait_n<0>();
  };

  f32x4 acc[FM_][FN_];  // first written by the zero-accumulator MFMAs of slice 0
  const int pre = min(NS - 1, ns);
  for (int s = 0; s < pre; ++s) issue(s, s);
  wait_slices(pre - 1);
  asm volatile("s_barrier" ::: "memory");
  bf16x8 af[FM_], b0[FN_], b1[FN_];
#pragma unroll
  for (int j = 0; j < FN_; ++j) b0[j] = load_frag<false, BN_>(smem + OPER_A, wn * 16 * FN_ + 16 * j, 0, lane);
#pragma unroll
  for (int i = 0; i < FM_; ++i) af[i] = load_frag<false, BM_>(smem, wm * 16 * FM_ + 16 * i, 0, lane);

  // B fragments of the next slice are read in the first FN_/2 rows (two per row), A
  // fragments in place after their row's MFMAs
#define NSA_W4R_PHASE(BC, BNX, TA, FIRST)                                                       \
  __builtin_amdgcn_s_setprio(1);                                                             \
  _Pragma("unroll") for (int i = 0; i < FM_; ++i) {                                          \
    _Pragma("unroll") for (int j = 0; j < FN_; ++j) {                                        \
      if (FIRST)                                                                             \
        mfma_first(acc[i][j], BC[j], af[i]);                                                 \
      else                                                                                   \
        mfma_tied(acc[i][j], BC[j], af[i]);                                                  \
    }                                                                                        \
    if (i < FN_ / 2) {                                                                       \
      BNX[2 * i] = load_frag<false, BN_>((TA) + OPER_A, wn * 16 * FN_ + 32 * i, 0, lane);      \
      BNX[2 * i + 1] = load_frag<false, BN_>((TA) + OPER_A, wn * 16 * FN_ + 32 * i + 16, 0, lane); \
    }                                                                                        \
    af[i] = load_frag<false, BM_>((TA), wm * 16 * FM_ + 16 * i, 0, lane);                    \
  }                                                                                          \
  __builtin_amdgcn_s_setprio(0);

  // phase j: top-of-phase wait + barrier + refill, then MFMA(j) | read(j+1).  The slot
  // of slice j+1 and the refill slot are tracked incrementally (no % NS per phase).
  int rd = 1 % NS;   // slot of slice j+1
  int wr = NS - 1;   // slot of slice j+NS-1 (= slot of slice j-1)
#define NSA_W4R_TOP(J)                                                                         \
  {                                                                                          \
    wait_slices(max(0, min(ns - (J) - 2, NS - 3))); /* slice J+1 landed */                   \
    asm volatile("s_barrier" ::: "memory");                                                  \
    if ((J) + NS - 1 < ns) issue((J) + NS - 1, wr);                                          \
  }
#define NSA_W4R_ADV()                        \
  {                                          \
    rd = rd + 1 == NS ? 0 : rd + 1;          \
    wr = wr + 1 == NS ? 0 : wr + 1;          \
  }
  {
    NSA_W4R_TOP(0)
    const char* ta = smem + rd * SLOT;
    NSA_W4R_PHASE(b0, b1, ta, true)
    NSA_W4R_ADV()
  }
  int j = 1;
  for (; j + 1 < ns; j += 2) {
    {
      NSA_W4R_TOP(j)
      const char* ta = smem + rd * SLOT;
      NSA_W4R_PHASE(b1, b0, ta, false)
      NSA_W4R_ADV()
    }
    {
      NSA_W4R_TOP(j + 1)
      const char* ta = smem + rd * SLOT;
      NSA_W4R_PHASE(b0, b1, ta, false)
      NSA_W4R_ADV()
    }
  }
  if (j < ns) {
    NSA_W4R_TOP(j)
    const char* ta = smem + rd * SLOT;  // slice ns: garbage reads, discarded
    NSA_W4R_PHASE(b1, b0, ta, false)
  }
#undef NSA_W4R_TOP
#undef NSA_W4R_ADV
#undef NSA_W4R_PHASE
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  w4_epilogue<EPI, FM_, FN_>(g, acc, smem, m0, n0, wm, wn, lane, wave);
}

template <bool A_K, bool B_K, int EPI>
hipError_t launch(const GemmArgs& a0, int splits, int variant, hipStream_t s) {
  GemmArgs a = a0;
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  a.k_per_split = a.K / splits;
  dim3 grid(a.tiles_m * a.tiles_n, 1, splits);
  if constexpr (A_K && EPI != EPI_ATOMIC_F32 && EPI != EPI_STORE_F32) {
    if (variant == 9 || variant == 10) {
      if (splits != 1) return hipErrorInvalidValue;
      const int tiles = a.tiles_m * a.tiles_n;
      const int g = variant == 9 ? (tiles < 256 ? tiles : 256) : tiles;
      gemm_p8_kernel<B_K, EPI><<<dim3(g), NTHREADS, 0, s>>>(a);
      return hipGetLastError();
    }
  }
  if (variant == 9 || variant == 10) variant = 7;  // TN (weight grad): the ring64 kernel
  if constexpr (!A_K && !B_K) {
    if (variant >= 12 && variant <= 16) {
      // 12/13: 256x256 tiles, 4 / 5 slots; 14: 256x128, 3 slots (2 workgroups/CU);
      // 15 / 16: 128x128, 4 / 3 slots (2/CU: the 70 KiB epilogue staging bounds it)
      const int bm = variant <= 14 ? 256 : 128, bn = variant <= 13 ? 256 : 128;
      a.tiles_m = (a.M + bm - 1) / bm;
      a.tiles_n = (a.N + bn - 1) / bn;
      const dim3 gr(a.tiles_m * a.tiles_n, 1, splits);
      if (variant == 12) gemm_w4r_kernel<EPI, 4, 8, 8, 1><<<gr, W4_THREADS, 0, s>>>(a);
      else if (variant == 13) gemm_w4r_kernel<EPI, 5, 8, 8, 1><<<gr, W4_THREADS, 0, s>>>(a);
      else if (variant == 14) gemm_w4r_kernel<EPI, 3, 8, 4, 2><<<gr, W4_THREADS, 0, s>>>(a);
      else if (variant == 15) gemm_w4r_kernel<EPI, 4, 4, 4, 2><<<gr, W4_THREADS, 0, s>>>(a);
      else gemm_w4r_kernel<EPI, 3, 4, 4, 2><<<gr, W4_THREADS, 0, s>>>(a);
      return hipGetLastError();
    }
  }
  if (variant >= 11 && variant <= 16) {  // other layouts: the 4-wave 256x256 kernel
    gemm_w4_kernel<A_K, B_K, EPI><<<grid, W4_THREADS, 0, s>>>(a);
    return hipGetLastError();
  }
  if (variant == 1)
    gemm_ring_kernel<A_K, B_K, EPI, 4, false><<<grid, NTHREADS, 0, s>>>(a);
  else if (variant == 2)
    gemm_ring_kernel<A_K, B_K, EPI, 5, false><<<grid, NTHREADS, 0, s>>>(a);
  else if (variant == 3)
    gemm_ring_kernel<A_K, B_K, EPI, 4, true><<<grid, NTHREADS, 0, s>>>(a);
  else if (variant == 4)
    gemm_ring_kernel<A_K, B_K, EPI, 5, true><<<grid, NTHREADS, 0, s>>>(a);
  else if (variant == 5)
    gemm_ring_kernel<A_K, B_K, EPI, 4, false, true><<<grid, NTHREADS, 0, s>>>(a);
  else if (variant == 6)
    gemm_ring_kernel<A_K, B_K, EPI, 4, true, true><<<grid, NTHREADS, 0, s>>>(a);
  else if (variant == 7)
    gemm_ring64_kernel<A_K, B_K, EPI, false><<<grid, NTHREADS, 0, s>>>(a);
  else if (variant == 8)
    gemm_ring64_kernel<A_K, B_K, EPI, true><<<grid, NTHREADS, 0, s>>>(a);
  else
    gemm_kernel<A_K, B_K, EPI><<<grid, NTHREADS, 0, s>>>(a);
  return hipGetLastError();
}

}  // namespace

// layout: 0 = NT (A [M][K], B [N][K]: forward), 1 = NN (A [M][K], B [K][N]: input grad),
//         2 = TN (A stored [K][M], B [K][N]: weight grad)
// epi: 0 store bf16, 1 fp32 atomic add into C, 2 store pre-activation + gelu into C2,
//      3 store acc * gelu'(U), 4 fp32 store of split z's partial into C + z*M*ldc
// bits 8..15 of `epi` select the pipeline: 0 = register-staged BK=64 double buffer,
// 1..4 = LDS-DMA ring (BK=32 slices): 1 = 4 slots (2 in flight) + LDS epilogue,
// 2 = 5 slots + LDS epilogue, 3 = 4 slots + direct stores, 4 = 5 slots + direct stores,
// 5/6 = pipelined ring (fragments of slice k+1 read under slice k's MFMAs), LDS / direct epilogue,
// 7/8 = ring64 (64-deep slots, whole-line DMA rows, pipelined sub-slices), LDS / direct epilogue
// (fragment double-buffering across slices was tried: 256 registers + 468 B/lane of
// scratch at 2 waves/SIMD, so it is not kept)
NSA_API hipError_t nsa_gemm(int layout, int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                            void* C2, const void* U, int M, int N, int K, int splits, hipStream_t s) {
  const int variant = (epi >> 8) & 0xff;
  epi &= 0xff;
  if (K % BK != 0 || splits < 1 || splits > K / BK || M < 8 || N < 8 || M % 8 || N % 8) return hipErrorInvalidValue;
  if (layout == 2 && M % 8) return hipErrorInvalidValue;
  if (epi != EPI_ATOMIC_F32 && epi != EPI_STORE_F32 && splits != 1) return hipErrorInvalidValue;
  GemmArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = C;
  a.C2 = (bf16_t*)C2;
  a.U = (const bf16_t*)U;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
#define NSA_GEMM_CASE(L, AK, BKc)                                                       \
  if (layout == L) {                                                                   \
    switch (epi) {                                                                     \
      case EPI_STORE_BF16: return launch<AK, BKc, EPI_STORE_BF16>(a, splits, variant, s);       \
      case EPI_ATOMIC_F32: return launch<AK, BKc, EPI_ATOMIC_F32>(a, splits, variant, s);       \
      case EPI_STORE_F32: return launch<AK, BKc, EPI_STORE_F32>(a, splits, variant, s);         \
      case EPI_GELU: return launch<AK, BKc, EPI_GELU>(a, splits, variant, s);                   \
      case EPI_DGELU: return launch<AK, BKc, EPI_DGELU>(a, splits, variant, s);                 \
      default: return hipErrorInvalidValue;                                            \
    }                                                                                  \
  }
  NSA_GEMM_CASE(0, true, true)
  NSA_GEMM_CASE(1, true, false)
  NSA_GEMM_CASE(2, false, false)
#undef NSA_GEMM_CASE
  return hipErrorInvalidValue;
}
