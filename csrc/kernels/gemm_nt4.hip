// Four-wave NT GEMM for gfx950 with a software-pipelined MFMA stream (A/B candidate
// beside gemm_nt.hip):  C[M,N] = A[M,K] · B[N,K]^T, bf16 in, fp32 accumulate, bf16 out.
//
// Why a second NT kernel: PMC at the K = 50304 lm_head input-grad shape
// (profiles/r3_gemm_pmc.md) puts gemm_nt.hip's 8-wave, barrier-paced phase structure at
// 73 % MFMA-busy cycles with waves parked on s_waitcnt / s_barrier 32 % of their
// cycles; hipBLASLt's 4-wave 256x256 solution reaches 90 % with 4 % of its cycles
// waiting.  This kernel is that shape of pipeline written directly:
//  * 256x256 tile, 4 waves (one per SIMD) of 128x128 = 8x8 accumulators of
//    v_mfma_f32_16x16x32_bf16 held in 256 AGPRs (tied asm operands);
//  * a 64-deep K-tile is two 32-deep k-steps of 64 MFMAs each; the 16 fragments of
//    the next k-step (8 of B, then 8 of A, ds_read_b128) are read during the first half
//    of the current one into the other register set (2 x 64 VGPRs), so an MFMA never
//    waits for LDS;
//  * operands arrive by LDS-DMA (global_load_lds_dwordx4, 16 one-KiB pieces per wave
//    per K-tile, XOR swizzle in the source address) into two 64-KiB buffers; the pieces
//    of K-tile t+2 are issued one per four MFMAs during the second k-step of K-tile t,
//    right after the tile's ONE barrier, which is also what frees K-tile t's buffer;
//  * every memory op is inline asm with hand-placed s_waitcnt (the compiler sees no
//    memory traffic in the loop and inserts no waits of its own).
// Layout conventions (swizzles, fragment maps, accumulator order) follow gemm_nt.hip.
#include "common.h"

namespace {

constexpr int T4_BM = 256, T4_BN = 256, T4_BK = 64;
constexpr int T4_THREADS = 256;
constexpr int T4_IMG = T4_BM * T4_BK * 2;  // 32 KiB: one operand's K-tile image [256][64] bf16, 128-B rows
constexpr int T4_BUF = 2 * T4_IMG;         // A image then B image
constexpr int T4_SMEM = 2 * T4_BUF;        // 128 KiB
#ifndef NT4_DMA_EARLY
#define NT4_DMA_EARLY 0  // 1: DMA pieces one per 2 MFMAs in the first half of k-step 1 (measured slower);
                         // 0: one per 4 MFMAs over the whole step
#endif
#ifndef NT4_REGSTAGE
#define NT4_REGSTAGE 0  // 1: operands through VGPRs (global_load + ds_write): measured 26 % slower, and the
                        // staging registers cross the loop back-edge (a compiler copy can read them
                        // before their loads land: wrong results seen) -- A/B only
#endif
#ifndef NT4_PROBE_NODMA
#define NT4_PROBE_NODMA 0  // timing probe: no DMA after the prologue (stale operands, wrong results)
#endif
#ifndef NT4_RD_SPREAD
#define NT4_RD_SPREAD 0  // next-step fragment reads one per 4 MFMAs over the whole step (0: per 2, first half)
#endif

struct Nt4Args {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  int M, N, K;
  int lda, ldb, ldc;
  int tiles_m, tiles_n;
};

__device__ __forceinline__ void mfma_acc(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
__device__ __forceinline__ void mfma_zero(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(b), "v"(a));
}
template <int OFF>
__device__ __forceinline__ void lds_rd(bf16x8& dst, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(dst) : "v"(addr), "n"(OFF) : "memory");
}
// one 1-KiB DMA piece: lane l's 16 bytes from sbase + voff land at lds + 16 l
__device__ __forceinline__ void dma16(const char* sbase, uint32_t voff, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

typedef uint32_t t4_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void gload16(t4_u32x4& dst, const char* sbase, uint32_t voff) {
  asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(dst) : "v"(voff), "s"(sbase) : "memory");
}
__device__ __forceinline__ void lds_wr16(uint32_t addr, const t4_u32x4& v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// The last MFMAs' results, then the wave's 128x128 bf16 quarter staged through its own
// 32 KiB of LDS (the operand buffers are free after the barrier) and stored as whole
// 256-B row segments (16 lanes per row, 4 rows per instruction).
__device__ __forceinline__ void nt4_epilogue(const Nt4Args& g, const f32x4 (&acc)[8][8], char* smem, int wave, int lane,
                                             int wm, int wn, int m0, int n0, int mlo, int nlo) {
  __syncthreads();
  char* stage = smem + wave * 32768;
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 tv = acc[i][j];
      const int row = 16 * i + r;                   // 0..127
      const int col = 16 * j + 4 * q;               // 0..127, 4 consecutive
      const int chunk = (col >> 3) ^ (row & 15);    // 16-byte chunk of the 256-B row, swizzled
      *reinterpret_cast<uint2*>(stage + row * 256 + chunk * 16 + (col & 4) * 2) =
          make_uint2(pack2(tv[0], tv[1]), pack2(tv[2], tv[3]));
    }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const bool full = (m0 == mlo) & (n0 == nlo);
#pragma unroll
  for (int s = 0; s < 32; ++s) {
    const int row = 4 * s + (lane >> 4);  // 0..127
    const int c = lane & 15;              // 16-byte chunk
    const uint4 val = *reinterpret_cast<const uint4*>(stage + row * 256 + ((c ^ (row & 15)) << 4));
    const int grow = m0 + wm * 128 + row, gcol = n0 + wn * 128 + 8 * c;
    if (!full && (grow < mlo || gcol < nlo)) continue;
    *reinterpret_cast<uint4*>(g.C + (int64_t)grow * g.ldc + gcol) = val;
  }
}

}  // namespace

// One output tile per workgroup (grid = tiles, XCD-grouped order), tail tiles shifted
// back inside the matrix (M, N >= 256, K % 128 == 0: an even number of K-tiles).
__global__ __launch_bounds__(T4_THREADS, 1) void gemm_nt4_kernel(Nt4Args g) {
  __shared__ __attribute__((aligned(16))) char smem[T4_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nk = g.K / T4_BK;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  const int tiles = g.tiles_m * g.tiles_n;
  int v = blockIdx.x;
  {
    const int G = gridDim.x, x = v % 8, q = G / 8, r = G % 8;
    v = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + v / 8;
  }
  if (v >= tiles) return;
  // row-major over the tile grid: a row panel of A is shared by the XCD's consecutive tiles
  const int tm = v / g.tiles_n, tn = v % g.tiles_n;
  const int mlo = tm * T4_BM, nlo = tn * T4_BN;
  const int m0 = min(mlo, g.M - T4_BM), n0 = min(nlo, g.N - T4_BN);

  // ---- DMA: wave w copies pieces w + 4q (q = 0..7) of each image: rows 32q + 8w + lane/8.
  // Image row r, physical chunk p holds logical chunk p ^ ((r >> 1) & 7); for these rows
  // (r >> 1) & 7 = (4w + lane/16) & 7, the same for every q.
  const int prow = 8 * wave + (lane >> 3);
  const int pch = (lane & 7) ^ ((4 * wave + (lane >> 4)) & 7);
  const uint32_t voA = (uint32_t)(prow * g.lda * 2 + pch * 16);
  const uint32_t voB = (uint32_t)(prow * g.ldb * 2 + pch * 16);
  const char* a_tile = reinterpret_cast<const char*>(g.A + (int64_t)m0 * g.lda);
  const char* b_tile = reinterpret_cast<const char*>(g.B + (int64_t)n0 * g.ldb);
  const int64_t a_q = (int64_t)32 * g.lda * 2, b_q = (int64_t)32 * g.ldb * 2;  // bytes per q step
  // pieces of K-tile kt into buffer buf: A pieces then B pieces, one call per piece
  auto dma_piece = [&](int kt, int buf, int pc) {
    const uint32_t img = lds0 + (uint32_t)(buf * T4_BUF + (pc >= 8 ? T4_IMG : 0));
    const int q = pc & 7;
    const uint32_t dst = img + (uint32_t)((wave + 4 * q) * 1024);
    if (pc < 8) dma16(a_tile + q * a_q + (int64_t)kt * 128, voA, dst);
    else dma16(b_tile + q * b_q + (int64_t)kt * 128, voB, dst);
  };

  // register staging (NT4_REGSTAGE): the same 16 pieces per wave and K-tile, loaded with
  // global_load_dwordx4 (same swizzled source addresses) and written lane-linear with
  // ds_write_b128 to where the DMA would have put them
  t4_u32x4 stg[16];
  const uint32_t wr0 = lds0 + (uint32_t)(wave * 1024 + 16 * lane);
  auto load_piece = [&](int kt, int pc) {
    const int q = pc & 7;
    if (pc < 8) gload16(stg[pc], a_tile + q * a_q + (int64_t)kt * 128, voA);
    else gload16(stg[pc], b_tile + q * b_q + (int64_t)kt * 128, voB);
  };
  auto write_piece = [&](int buf, int pc) {
    const int q = pc & 7;
    lds_wr16(wr0 + (uint32_t)(buf * T4_BUF + (pc >= 8 ? T4_IMG : 0) + 4096 * q), stg[pc]);
  };

  // ---- fragment addresses: rows wm*128 + 16 i + (lane & 15) (A) / wn*128 + 16 j + ... (B),
  // logical chunk 4 kk + (lane >> 4); i / j and the buffer go in the immediate offset
  // (A rows of one buffer span 32 KiB: i * 2048 + buf * 65536 would overflow the 16-bit
  // offset, so each buffer has its own base)
  const int sw = (lane >> 1) & 7;
  uint32_t adA[2][2], adB[2][2];  // [buf][kk]
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ch = ((4 * kk + (lane >> 4)) ^ sw) << 4;
      adA[b][kk] = lds0 + (uint32_t)(b * T4_BUF + (wm * 128 + (lane & 15)) * 128 + ch);
      adB[b][kk] = lds0 + (uint32_t)(b * T4_BUF + T4_IMG + (wn * 128 + (lane & 15)) * 128 + ch);
    }

  f32x4 acc[8][8];
  bf16x8 xa[8], xb[8], ya[8], yb[8];  // register sets X (k-step 0) and Y (k-step 1)

  // prologue: K-tiles 0 and 1 into the buffers (K-tile 2 left in the staging registers
  // when register-staged), wait for 0, read X of K-tile 0
  if constexpr (NT4_REGSTAGE) {
#pragma unroll
    for (int kt = 0; kt < 2; ++kt) {
#pragma unroll
      for (int pc = 0; pc < 16; ++pc) load_piece(kt, pc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int pc = 0; pc < 16; ++pc) write_piece(kt, pc);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int pc = 0; pc < 16; ++pc) load_piece(min(2, nk - 1), pc);
  } else {
#pragma unroll
    for (int pc = 0; pc < 16; ++pc) dma_piece(0, 0, pc);
#pragma unroll
    for (int pc = 0; pc < 16; ++pc) dma_piece(1, 1, pc);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
#define NT4_READ_SET(SA, SB, BUF, KK)                                                   \
  {                                                                                     \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) lds_rd<0>(SB[j], adB[BUF][KK] + 2048 * j); \
    _Pragma("unroll") for (int i = 0; i < 8; ++i) lds_rd<0>(SA[i], adA[BUF][KK] + 2048 * i); \
  }
  NT4_READ_SET(xa, xb, 0, 0)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // One k-step: 64 MFMAs on set (CA, CB); during the first 32, read the 16 fragments of
  // the next k-step (buffer NBUF, kk NKK) into (NA, NB) when READ; during all 64, issue the
  // DMA pieces of K-tile DKT into buffer DBUF (one per 4 MFMAs) when DMA.
#define NT4_STEP(CA, CB, NA, NB, NBUF, NKK, READ, DMA, DKT, DBUF, ZERO)                         \
  {                                                                                            \
    constexpr bool RD_ = READ, DM_ = DMA, Z_ = ZERO;                                           \
    _Pragma("unroll") for (int m = 0; m < 64; ++m) {                                           \
      const int i_ = m >> 3, j_ = m & 7;                                                       \
      if constexpr (Z_) mfma_zero(acc[i_][j_], CB[j_], CA[i_]);                                \
      else mfma_acc(acc[i_][j_], CB[j_], CA[i_]);                                              \
      if (RD_ && (NT4_RD_SPREAD ? (m & 3) == 0 : ((m & 1) == 0 && m < 32))) {                  \
        const int r_ = NT4_RD_SPREAD ? (m >> 2) : (m >> 1);                                    \
        if (r_ < 8) lds_rd<0>(NB[r_], adB[NBUF][NKK] + 2048 * r_);                            \
        else lds_rd<0>(NA[r_ - 8], adA[NBUF][NKK] + 2048 * (r_ - 8));                         \
      }                                                                                        \
      if constexpr (NT4_REGSTAGE) {                                                            \
        /* first half: write the staged K-tile (DKT) into DBUF; second half: load K-tile */     \
        /* DKT + 1 into the staging registers (a write reads its registers long before) */     \
        if (DM_ && !NT4_PROBE_NODMA && (m & 1) == 1) {                                          \
          if (m < 32) write_piece((DBUF), m >> 1);                                              \
          else load_piece(min((DKT) + 1, nk - 1), (m - 32) >> 1);                               \
        }                                                                                      \
      } else if (DM_ && !NT4_PROBE_NODMA && (NT4_DMA_EARLY ? ((m & 1) == 1 && m < 32) : (m & 3) == 1)) { \
        dma_piece((DKT), (DBUF), NT4_DMA_EARLY ? (m >> 1) : (m >> 2));                          \
      }                                                                                        \
    }                                                                                          \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                        \
  }

  // K-tile t in buffer B_ = t & 1: k-step 0 on X (reading Y = its second half), the
  // tile's one barrier (after it K-tile t+1 has landed and buffer B_ is free), k-step 1 on
  // Y (reading X = K-tile t+1's first half, DMA of K-tile t+2 into B_).  Past the end the
  // DMA re-fetches the last K-tile into a buffer nobody reads again and the reads fetch
  // unused fragments, so the loop body has no branch (a branch between MFMA steps makes
  // the register allocator copy the 256 loop-carried accumulators).
#define NT4_KTILE(B_, KT)                                                                      \
  {                                                                                            \
    NT4_STEP(xa, xb, ya, yb, B_, 1, true, false, 0, 0, false)                                  \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                          \
    __builtin_amdgcn_s_barrier();                                                              \
    NT4_STEP(ya, yb, xa, xb, (B_ ^ 1), 0, true, true, min((KT) + 2, nk - 1), B_, false)       \
  }

  // nk is even (host check), so the K-tile pairs below cover it exactly
  for (int t = 0; t < nk; t += 2) {
    NT4_KTILE(0, t)
    NT4_KTILE(1, t + 1)
  }
#undef NT4_KTILE
#undef NT4_STEP
#undef NT4_READ_SET

  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");  // re-fetches past the end
  nt4_epilogue(g, acc, smem, wave, lane, wm, wn, m0, n0, mlo, nlo);
}

// NT4_STAGED variant: the same wave geometry and MFMA stream, operands in FOUR 32-KiB
// slots of one 32-deep k-step each (A [256][32] + B [256][32], 64-B rows).  Each k-step
// opens with a counted wait + barrier (k-step s+1 landed, the slot of s-1 free); the DMA of
// k-step s+3 (8 pieces per wave) is spread one per 8 MFMAs over k-step s, so the operand
// stream has no bursts and two k-steps of lead.  64-B rows: physical chunk = chunk ^
// g((row >> 2) & 3) with g = {0, 2, 3, 1}, conflict-free for ds_read_b128's lane groups.
constexpr int T4S_SLOT = 2 * T4_BM * 32 * 2;  // 32 KiB
__device__ __forceinline__ int t4s_g(int b) { return (0x1320 >> (4 * b)) & 3; }  // {0, 2, 3, 1}

__global__ __launch_bounds__(T4_THREADS, 1) void gemm_nt4s_kernel(Nt4Args g) {
  __shared__ __attribute__((aligned(16))) char smem[4 * T4S_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ns = g.K / 32;  // k-steps, a multiple of 4 (host check)
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));
  const int tiles = g.tiles_m * g.tiles_n;
  int v = blockIdx.x;
  {
    const int G = gridDim.x, x = v % 8, q = G / 8, r = G % 8;
    v = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + v / 8;
  }
  if (v >= tiles) return;
  const int tm = v / g.tiles_n, tn = v % g.tiles_n;
  const int mlo = tm * T4_BM, nlo = tn * T4_BN;
  const int m0 = min(mlo, g.M - T4_BM), n0 = min(nlo, g.N - T4_BN);

  // DMA: a piece = 16 rows x 64 B; wave w copies pieces w + 4q (q = 0..3) of A and of B:
  // rows 64q + 16w + lane/4, physical chunk lane % 4 <- logical chunk (lane % 4) ^ g(row>>2 & 3)
  // with (row >> 2) & 3 = (lane >> 4) for these rows (64q + 16w is a multiple of 16)
  const int prow = 16 * wave + (lane >> 2);
  const int pch = (lane & 3) ^ t4s_g(lane >> 4);
  const uint32_t voA = (uint32_t)(prow * g.lda * 2 + pch * 16);
  const uint32_t voB = (uint32_t)(prow * g.ldb * 2 + pch * 16);
  const char* a_tile = reinterpret_cast<const char*>(g.A + (int64_t)m0 * g.lda);
  const char* b_tile = reinterpret_cast<const char*>(g.B + (int64_t)n0 * g.ldb);
  const int64_t a_q = (int64_t)64 * g.lda * 2, b_q = (int64_t)64 * g.ldb * 2;
  auto dma_piece = [&](int ks, int slot, int pc) {  // pc 0..7: A q = pc, B q = pc - 4
    const int q = pc & 3;
    const uint32_t dst = lds0 + (uint32_t)(slot * T4S_SLOT + (pc >= 4 ? T4S_SLOT / 2 : 0) + (wave + 4 * q) * 1024);
    if (pc < 4) dma16(a_tile + q * a_q + (int64_t)ks * 64, voA, dst);
    else dma16(b_tile + q * b_q + (int64_t)ks * 64, voB, dst);
  };
  // fragments: row wm*128 + 16 i + (lane & 15), logical chunk lane >> 4 of the 64-B row
  const int rphys = ((lane >> 4) ^ t4s_g((lane >> 2) & 3)) << 4;
  const uint32_t adA = lds0 + (uint32_t)((wm * 128 + (lane & 15)) * 64 + rphys);
  const uint32_t adB = lds0 + (uint32_t)(T4S_SLOT / 2 + (wn * 128 + (lane & 15)) * 64 + rphys);

  f32x4 acc[8][8];
  bf16x8 xa[8], xb[8], ya[8], yb[8];
#pragma unroll
  for (int st = 0; st < 3; ++st)
#pragma unroll
    for (int pc = 0; pc < 8; ++pc) dma_piece(min(st, ns - 1), st, pc);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // k-step 0
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int j = 0; j < 8; ++j) lds_rd<0>(xb[j], adB + 1024 * j);
#pragma unroll
  for (int i = 0; i < 8; ++i) lds_rd<0>(xa[i], adA + 1024 * i);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");

  // k-step S (slot S & 3) on (CA, CB): wait for k-step S+1 (8 younger pieces may fly),
  // barrier, 64 MFMAs; reads of k-step S+1 (slot (S+1) & 3) one per 2 MFMAs in the first
  // half; DMA of k-step S+3 into slot (S+3) & 3 (= the slot of S-1) one per 8 MFMAs.
#define NT4S_STEP(SL, CA, CB, NA, NB, S)                                                       \
  {                                                                                            \
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                                          \
    __builtin_amdgcn_s_barrier();                                                              \
    const int dks_ = min((S) + 3, ns - 1);                                                     \
    _Pragma("unroll") for (int m = 0; m < 64; ++m) {                                           \
      const int i_ = m >> 3, j_ = m & 7;                                                       \
      mfma_acc(acc[i_][j_], CB[j_], CA[i_]);                                                   \
      if ((m & 1) == 0 && m < 32) {                                                            \
        const int r_ = m >> 1;                                                                 \
        constexpr uint32_t nso_ = (uint32_t)((((SL) + 1) & 3) * T4S_SLOT);                     \
        if (r_ < 8) lds_rd<0>(NB[r_], adB + nso_ + 1024 * r_);                                \
        else lds_rd<0>(NA[r_ - 8], adA + nso_ + 1024 * (r_ - 8));                             \
      }                                                                                        \
      if ((m & 7) == 3) dma_piece(dks_, ((SL) + 3) & 3, m >> 3);                              \
    }                                                                                          \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                        \
  }
  for (int s0 = 0; s0 < ns; s0 += 4) {
    NT4S_STEP(0, xa, xb, ya, yb, s0)
    NT4S_STEP(1, ya, yb, xa, xb, s0 + 1)
    NT4S_STEP(2, xa, xb, ya, yb, s0 + 2)
    NT4S_STEP(3, ya, yb, xa, xb, s0 + 3)
  }
#undef NT4S_STEP
  asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
  nt4_epilogue(g, acc, smem, wave, lane, wm, wn, m0, n0, mlo, nlo);
}

NSA_API hipError_t nsa_gemm_nt4(const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M, int N, int K,
                                hipStream_t s) {
  if (M < T4_BM || N < T4_BN || K < 2 * T4_BK || K % (2 * T4_BK) != 0 || lda % 8 || ldb % 8 || ldc % 8 || lda < K ||
      ldb < K || ldc < N)
    return hipErrorInvalidValue;
  if ((int64_t)T4_BM * lda * 2 >= (1ll << 31) || (int64_t)T4_BN * ldb * 2 >= (1ll << 31)) return hipErrorInvalidValue;
  Nt4Args a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.tiles_m = (M + T4_BM - 1) / T4_BM;
  a.tiles_n = (N + T4_BN - 1) / T4_BN;
#ifndef NT4_STAGED
#define NT4_STAGED 1  // 0: two 64-KiB buffers, one barrier per K-tile (gemm_nt4_kernel)
#endif
  if (NT4_STAGED)
    gemm_nt4s_kernel<<<dim3(a.tiles_m * a.tiles_n), T4_THREADS, 0, s>>>(a);
  else
    gemm_nt4_kernel<<<dim3(a.tiles_m * a.tiles_n), T4_THREADS, 0, s>>>(a);
  return hipGetLastError();
}
