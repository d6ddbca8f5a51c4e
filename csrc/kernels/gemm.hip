// bf16 MFMA weight-gradient GEMM for gfx950 (dW = dY^T · X for
// every nn.Linear), split over the token dimension with the fp32 result added straight
// into the flat fp32 gradient buffer:
//
//   C[M,N] += A[M,K] · B[K,N]   with A stored [K][M] (dY, tokens x out-features) and
//                               B stored [K][N] (X, tokens x in-features), fp32 accumulate,
//                               v_mfma_f32_16x16x32_bf16 on ds_read_b64_tr_b16 fragments.
//
// (The forward and input-gradient GEMMs are the persistent NT kernel in gemm_nt.hip.)
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
// Variants (the per-shape tuner times both, ops/gemm_tune.py::wgrad_acc):
//   1 = "ring":   32-deep K slices in a 4-slot LDS ring, two slices in flight;
//   7 = "ring64": 64-deep slots (every DMA row a whole 128-B line), two slots, each
//                 multiplied as two 32-deep sub-slices with the next sub-slice's fragments
//                 read under the current one's MFMAs;
//   9 = "phase":  the NT kernel's 4-phase staggered schedule (see below).
// Rejected variants (register-staged, 5-slot / pipelined rings, persistent p8, 4-wave
// 128x128 and 2-workgroup-per-CU geometries) and their measurements are recorded in
// docs/performance.md.
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
// Variant 1 ("ring"): K staged in 32-deep slices by LDS-DMA into a 4-slot LDS ring with
// TWO slices in flight: slice k+2 is issued while slice k is multiplied, and each wave
// waits only for slice k with a counted `s_waitcnt vmcnt(N)` folded into the raw
// `s_barrier`.  WAR: slice k+2 reuses the slot of slice k-2, whose reads every wave
// finished before passing the barrier of iteration k-1.  MFMA operands are swapped
// (C^T = B^T A^T) so each lane's accumulator holds 4 consecutive output columns of a row.
// ---------------------------------------------------------------------------
constexpr int RBK = 32;
constexpr int RSLOT_A = BM * RBK * 2;     // 16 KiB
constexpr int RSLOT_BYTES = 2 * RSLOT_A;  // A + B
constexpr int RSLOTS = 4;
constexpr int RING_SMEM = RSLOTS * RSLOT_BYTES > EP_BYTES ? RSLOTS * RSLOT_BYTES : EP_BYTES;
static_assert(RING_SMEM <= 163840, "LDS budget");

template <int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void wgrad_ring_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[RING_SMEM];
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
      const int row = e >> 5, pc = e & 31;
      glds16(tn_src(g.A, g.lda, k0, row, pc, g.M, m0), __builtin_amdgcn_readfirstlane(slot + wbase));
      glds16(tn_src(g.B, g.ldb, k0, row, pc, g.N, n0), __builtin_amdgcn_readfirstlane(slot + RSLOT_A + wbase));
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int AHEAD = RSLOTS - 2;  // slices in flight beyond the one being multiplied
#pragma unroll
  for (int a = 0; a < AHEAD; ++a)
    if (nk > a) issue(a);
  for (int k = 0; k < nk; ++k) {
    // wait for slice k; the younger slices (up to AHEAD, 4 DMA pieces each) may stay in flight
    const int younger = min(AHEAD, nk - 1 - k);
    if (k + AHEAD < nk) issue(k + AHEAD);
    if (younger == 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    const char* ta = smem + (k % RSLOTS) * RSLOT_BYTES;
    const char* tb = ta + RSLOT_A;
    bf16x8 af[FM], bfr[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) bfr[j] = load_frag<256>(tb, wn * WTN + 16 * j, 0, lane);
#pragma unroll
    for (int i = 0; i < FM; ++i) af[i] = load_frag<256>(ta, wm * WTM + 16 * i, 0, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j)  // swapped operands: acc[i][j][e] = C[16i + (l&15)][16j + 4(l>>4) + e]
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  wgrad_epilogue<EPI>(g, acc, smem, m0, n0, wm, wn, lane, wave);
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

template <int EPI>
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
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(BC[j], af[i], acc[i][j], 0, 0, 0);   \
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


// ---------------------------------------------------------------------------
// Variant 9 ("phase"): the persistent NT kernel's main loop (gemm_nt.hip) on the
// weight-gradient layout — one 64-deep K-tile (64 KiB) consumed in 4 phases of 16 MFMAs,
// one 64x32 quadrant per phase, the two wave groups one raw barrier apart (one group's
// LDS reads beside the other's MFMAs), LDS-DMA of one 16-KiB half-tile per phase issued
// 6 phases ahead with per-lane source offsets computed once and one M0 write per piece
// pair, counted vmcnt(8) in every phase.  Differences from NT: operands are stored [K][rows]
// so a half-tile is a [64 k][128] image (256-B rows, rimg<128> swizzle: conflict-free for the
// ds_read_b64_tr_b16 fragment reads — scripts/lds_swizzle_check.py) holding the rows of one
// quadrant half (A: m with (m >> 6) & 1 == h; B: n with (n >> 5) & 1 == h); one work item
// (tile, K split) per workgroup; fp32 atomic / partial-store epilogue through LDS.
// ---------------------------------------------------------------------------
constexpr int PH_HALF = 16384;             // [64][128] bf16
constexpr int PH_BUF = 4 * PH_HALF;        // A0 A1 B0 B1
constexpr int PH_SMEM = 2 * PH_BUF > EP_BYTES ? 2 * PH_BUF : EP_BYTES;
static_assert(PH_SMEM <= 163840, "LDS budget");

__device__ __forceinline__ void dma16x2_tn(const char* sbase, uint32_t voff0, uint32_t voff1m, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %3\n\tglobal_load_lds_dwordx4 %1, %3 offset:1024"
               :
               : "v"(voff0), "v"(voff1m), "s"(lds), "s"(sbase)
               : "memory");
}

__device__ __forceinline__ void ph_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int EPI>
__global__ __launch_bounds__(NTHREADS, 2) void wgrad_phase_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[PH_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int nwg = g.tiles_m * g.tiles_n;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, r = nwg % 8;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  }
  const int tm = bid / g.tiles_n, tn = bid % g.tiles_n;
  const int mlo = tm * BM, nlo = tn * BN;
  const int m0 = min(mlo, g.M - BM), n0 = min(nlo, g.N - BN);  // tail tiles shifted back inside
  const int nkb = g.K / 64, kb0 = (int)blockIdx.z * nkb / (int)gridDim.z;
  const int nk = ((int)blockIdx.z + 1) * nkb / (int)gridDim.z - kb0;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  // per-lane DMA offsets (bytes from the K-tile's first row at column m0 / n0): piece pc =
  // 2 wave + j = k rows 4 pc .. 4 pc + 3 of a half; lane l: k row 4 pc + l / 16, physical
  // chunk l % 16 holding logical chunk c = p ^ 2 g(row) = image columns 8 c .. 8 c + 7
  uint32_t voA[2], voB[2], voA1m[2], voB1m[2], ldA[2], ldB[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = 2 * wave + j;
      const int kr = 4 * pc + (lane >> 4);
      const int gg = (kr & 3) | (((kr >> 3) & 1) << 2);
      const int c = (lane & 15) ^ (2 * gg);
      const int ma = (c >> 3) * 128 + h * 64 + (c & 7) * 8;  // A half h: m with (m >> 6) & 1 == h
      const int nb = (c >> 2) * 64 + h * 32 + (c & 3) * 8;   // B half h: n with (n >> 5) & 1 == h
      const uint32_t oa = (uint32_t)((kr * g.lda + ma) * 2), ob = (uint32_t)((kr * g.ldb + nb) * 2);
      if (j == 0) {
        voA[h] = oa;
        voB[h] = ob;
        ldA[h] = lds0 + (uint32_t)(h * PH_HALF + pc * 1024);
        ldB[h] = lds0 + (uint32_t)(2 * PH_HALF + h * PH_HALF + pc * 1024);
      } else {
        voA1m[h] = oa - 1024u;
        voB1m[h] = ob - 1024u;
      }
    }
  }
  // B half image columns: n = (nh >> 5) * 64 + h * 32 + (nh & 31), so wave wn's columns
  // wn*64 + qn*32 + [0, 32) are nh = wn*32 + [0, 32) of half qn (A: mh = wm*64 + [0, 64))
  const char* abase = reinterpret_cast<const char*>(g.A + (int64_t)kb0 * 64 * g.lda + m0);
  const char* bbase = reinterpret_cast<const char*>(g.B + (int64_t)kb0 * 64 * g.ldb + n0);
  const int64_t astep = (int64_t)64 * g.lda * 2, bstep = (int64_t)64 * g.ldb * 2;
  // half-tile kinds: 0 = A half 0, 1 = B half 0, 2 = B half 1, 3 = A half 1
  auto issue_half = [&](int kt, int kind) {
    const uint32_t buf = (uint32_t)((kt & 1) * PH_BUF);
    if (kind == 0 || kind == 3) {
      const int h = kind == 3;
      dma16x2_tn(abase + kt * astep, voA[h], voA1m[h], ldA[h] + buf);
    } else {
      const int h = kind == 2;
      dma16x2_tn(bbase + kt * bstep, voB[h], voB1m[h], ldB[h] + buf);
    }
  };
  issue_half(0, 0);
  issue_half(0, 1);
  issue_half(0, 2);
  issue_half(0, 3);
  if (nk > 1) {
    issue_half(1, 0);
    issue_half(1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  ph_barrier();
  if (wm == 1) ph_barrier();  // stagger: group 1 runs one barrier behind group 0

  f32x4 acc[FM][FN];
  bf16x8 af[4][2], b0f[2][2], b1f[2][2];

#define PH_PHASE(P, FIRST)                                                                      \
  {                                                                                            \
    const char* base_ = smem + (kt & 1) * PH_BUF;                                              \
    if (P == 0 || P == 2) {                                                                    \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        af[i][kk] = load_frag<128>(base_ + (P >> 1) * PH_HALF, wm * 64 + 16 * i, kk, lane);    \
    }                                                                                          \
    if (P == 0 || P == 1) {                                                                    \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) {                                       \
        const bf16x8 f_ = load_frag<128>(base_ + 2 * PH_HALF + P * PH_HALF, wn * 32 + 16 * j, kk, lane); \
        if (P == 0) b0f[j][kk] = f_;                                                           \
        else b1f[j][kk] = f_;                                                                  \
      }                                                                                        \
    }                                                                                          \
    {                                                                                          \
      /* half-tile P+6: p0 B1(kt+1), p1 A1(kt+1), p2 A0(kt+2), p3 B0(kt+2) */                  \
      const int it_ = kt + (P < 2 ? 1 : 2);                                                    \
      if (it_ < nk) {                                                                          \
        issue_half(it_, P == 0 ? 2 : P == 1 ? 3 : P == 2 ? 0 : 1);                             \
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                                      \
      } else {                                                                                 \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                      \
      }                                                                                        \
    }                                                                                          \
    ph_barrier();                                                                              \
    __builtin_amdgcn_s_setprio(1);                                                             \
    {                                                                                          \
      constexpr int qm = (P == 2 || P == 3), qn = (P == 1 || P == 2);                          \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                            \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) {                                       \
        const bf16x8 bb_ = qn ? b1f[j][kk] : b0f[j][kk];                                       \
        f32x4& a_ = acc[qm * 4 + i][qn * 2 + j];                                               \
        a_ = __builtin_amdgcn_mfma_f32_16x16x32_bf16(                                          \
            bb_, af[i][kk], ((FIRST) && kk == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : a_, 0, 0, 0);  \
      }                                                                                        \
    }                                                                                          \
    __builtin_amdgcn_s_setprio(0);                                                             \
    ph_barrier();                                                                              \
  }
  {
    const int kt = 0;
    PH_PHASE(0, true)
    PH_PHASE(1, true)
    PH_PHASE(2, true)
    PH_PHASE(3, true)
  }
  for (int kt = 1; kt < nk; ++kt) {
    PH_PHASE(0, false)
    PH_PHASE(1, false)
    PH_PHASE(2, false)
    PH_PHASE(3, false)
  }
#undef PH_PHASE
  if (wm == 0) ph_barrier();  // close the stagger
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  wgrad_epilogue<EPI>(g, acc, smem, m0, n0, wm, wn, lane, wave, mlo, nlo);
}

}  // namespace

// C (fp32) [M, N] (+)= A^T B with A stored [K][M], B stored [K][N] (leading dims lda / ldb),
// K split over `splits` workgroups per output tile.
// epi: 1 = fp32 atomic add into C, 4 = split z stores its fp32 partial into C + z*M*ldc;
// bits 8..15 of `epi` select the variant: 1 = ring, 7 = ring64 (default), 9 = phase
// (M, N >= 256; falls back to ring64 otherwise).
NSA_API hipError_t nsa_gemm(int layout, int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                            void* C2, const void* U, int M, int N, int K, int splits, hipStream_t s) {
  (void)C2;
  (void)U;
  int variant = (epi >> 8) & 0xff;
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
  if (variant == 9 && M >= BM && N >= BN && lda % 8 == 0 && ldb % 8 == 0 &&
      (int64_t)64 * lda * 2 < (1ll << 31) && (int64_t)64 * ldb * 2 < (1ll << 31)) {
    if (epi == EPI_ATOMIC_F32) wgrad_phase_kernel<EPI_ATOMIC_F32><<<grid, NTHREADS, 0, s>>>(a);
    else wgrad_phase_kernel<EPI_STORE_F32><<<grid, NTHREADS, 0, s>>>(a);
  } else if (variant == 1) {
    if (epi == EPI_ATOMIC_F32) wgrad_ring_kernel<EPI_ATOMIC_F32><<<grid, NTHREADS, 0, s>>>(a);
    else wgrad_ring_kernel<EPI_STORE_F32><<<grid, NTHREADS, 0, s>>>(a);
  } else {
    if (epi == EPI_ATOMIC_F32) wgrad_ring64_kernel<EPI_ATOMIC_F32><<<grid, NTHREADS, 0, s>>>(a);
    else wgrad_ring64_kernel<EPI_STORE_F32><<<grid, NTHREADS, 0, s>>>(a);
  }
  return hipGetLastError();
}
