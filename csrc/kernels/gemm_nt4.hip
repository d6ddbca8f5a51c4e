// Persistent four-wave bf16 "NT" GEMM for gfx950: C[M,N] = A[M,K] · B[N,K]^T (both operands
// K-contiguous, fp32 accumulate), with fused epilogues (bf16 store (+ bias), gelu'(u) (fp16)
// + gelu(u) for the c_fc forward, acc * U with U = gelu'(u) for the mlp.c_proj input grad,
// and the cross-entropy pair XENT / XDX for the tied lm_head).
//
// Why four waves: round 3's eight-wave NT kernel (128x64 per wave, since removed) read
// 24 fragments (24 KiB) per wave per 64-deep K-tile for 64 MFMAs; with 8 waves that is
// 192 KiB of ds_read_b128 plus 64 KiB of LDS-DMA writes per CU per K-tile, against
// 2048 MFMA cycles per SIMD — the LDS array runs near its 256 B/clk (PMC:
// SQ_LDS_CMD_FIFO_FULL 60M at the lm_head dX shape, profiles/r3_gemm_pmc.md).  Here a wave
// owns 128x128 (8x8 accumulators of v_mfma_f32_16x16x32_bf16 = 256 AGPRs) and reads 32
// fragments per 128 MFMAs: 128 KiB of reads per CU per K-tile, a third less.
//
// Schedule of one 64-deep K-tile (two 32-deep k-steps, 128 MFMAs per wave, one wave per
// SIMD; the numbers are MFMA slots n = 0..127, k-step 0 = n < 64; ER / DS / VMS / RS below):
//   n  0-15   read the 16 k-step-1 fragments of this buffer, one per MFMA
//   n 17/18   lgkmcnt(0) (the wait names every fragment), barrier: the buffer is free
//   n 19-109  LDS-DMA of K-tile t+2 into this buffer, one 1-KiB piece per 6 MFMAs
//   n 92/93   vmcnt(10) + barrier: K-tile t+1 (issued one K-tile ago) has landed
//   n 94-124  read K-tile t+1's 16 k-step-0 fragments (other buffer), one per 2 MFMAs
//   n 127     lgkmcnt(0)
// so DMA has about one K-tile (~2048 MFMA cycles) to land, two 64-KiB buffers suffice, and
// no MFMA waits on LDS.  LDS-DMA is buffer_load_dwordx4 ... lds with the tile row base in
// the buffer resource (advanced 128 B per K-tile), the piece's row offset in an SGPR
// soffset and one per-lane VGPR offset (XOR swizzle of the 16-B chunk in the source
// address, cdna_hip_programming.md rule 21); four pieces share one M0 write through the
// instruction offset: no VALU and one SALU per piece.  (Shaped after hipBLASLt's gfx950
// MT256x256x64 solution for these layouts, read with llvm-objdump; measured alternatives
// — three barriers per K-tile, M0 per piece, denser DMA, compiler-placed LDS waits, an
// LDS-re-shaped epilogue, start-time staggering — are in docs/performance.md.)
//
// The MFMA's first operand is the A fragment, so a lane holds rows 4 (l >> 4) + e (e = 0..3)
// of output column l & 15 of each 16x16 tile.  B rows are staged in a permuted order: image
// row 16 j + r of a wave's half holds output column 8 r + j, so for one (i, e) a lane's
// accumulators of the 8 fragments j are 8 CONSECUTIVE columns and one store instruction
// writes 4 rows x 256 contiguous bytes straight from the accumulators (no LDS round trip).
//
// Persistent: grid = #CUs, tiles walked in an XCD-grouped order (tile groups of row blocks
// x every column, each XCD's workgroups on neighbouring tiles); the DMA
// cursor runs straight on into the next tile, so the next tile's first two K-tiles load
// while this tile's epilogue stores.  Tail tiles are shifted back inside the matrix and
// store only their not-yet-covered rows / columns: M, N >= 256, N % 8 == 0, K % 64 == 0.
#include <cstdlib>
#include <utility>

#include "common.h"

namespace {

constexpr int Q_BM = 256, Q_BN = 256, Q_BK = 64;
constexpr int Q_THR = 256;
constexpr int Q_IMG = Q_BM * Q_BK * 2;  // 32 KiB: one operand's [256][64] bf16 K-tile image
constexpr int Q_BUF = 2 * Q_IMG;        // A image, then B image
constexpr int Q_SMEM = 2 * Q_BUF;       // 128 KiB, two buffers

#ifndef NSA_NT4_DS
#define NSA_NT4_DS 6  // MFMAs between LDS-DMA pieces
#endif
#ifndef NSA_NT4_VMS
#define NSA_NT4_VMS 92  // slot of the wait for the previous K-tile's pieces
#endif
#ifndef NSA_NT4_ER
#define NSA_NT4_ER 1  // MFMAs between the k-step-1 fragment reads at the K-tile head
#endif
#ifndef NSA_NT4_RS
#define NSA_NT4_RS 2  // MFMAs between the next K-tile's fragment reads
#endif

enum { Q_EPI_BF16 = 0, Q_EPI_GELU = 1, Q_EPI_DGELU = 2, Q_EPI_XENT = 3, Q_EPI_XDX = 4 };

// Overlapped epilogue (OVL, plain bf16 / fp16 outputs without bias): each tile's stores ride in the next
// tile's first two K-tiles instead of stalling the MFMA pipe between tiles.  In the first
// K-tile, k-step 0 runs fragment row by fragment row; each accumulator tile is copied out just
// before the MFMA that restarts it, rows 0-3 go out as 256-byte row stores after their eighth
// MFMA, rows 4-7 are held packed (64 VGPRs) and stored in the second K-tile (OVL2): 16 stores
// per K-tile rather than 32, which the per-CU write path drains under the MFMAs.  Measured
// (profiles/r6_nt4_ovl.md, same process): c_attn 333.8 -> 314.5 us, attn.c_proj 138.5 ->
// 135.2, c_attn.dx 336.4 -> 329.9, mlp.c_proj / c_fc.dx -1.2 / -1.7 %; all 32 stores in the
// first K-tile (OVL1) had gained only at K = 3072.  Needs two K-tiles (K >= 128).
constexpr int Q_OVL_MIN_K = 2 * 64;
#ifndef NSA_NT4_OVL2
#define NSA_NT4_OVL2 1  // 0 (A/B builds only): all 32 stores in the first K-tile (OVL1)
#endif

// GELU epilogue lookup table (built on the host by ops/gemm.py gelu_table with torch's exact-erf
// GELU): entry i = gelu(u) as bf16 | gelu'(u) as fp16 << 16 for the bf16 u with bit pattern
// (14208 + i % 2560) | (i >= 2560) << 15, i.e. every bf16 with 2^-16 <= |u| < 16.  The
// epilogue stages it in LDS beside the operand buffers and looks each u up (one ds_read_b32
// instead of an erf, an exp and a reciprocal); a row of 8 values per lane with any u outside
// the table (zero, |u| < 2^-16, |u| >= 16, inf / NaN) takes the arithmetic path for the
// whole wave.
constexpr int Q_GTAB_LO = 14208, Q_GTAB_N = 2560, Q_GTAB_BYTES = 2 * Q_GTAB_N * 4;
#ifndef NSA_NT4_GTAB
#define NSA_NT4_GTAB 1  // 0 (A/B builds only): the arithmetic GELU for every row
#endif
#ifndef NSA_NT4_XLANE
#define NSA_NT4_XLANE 1  // 1: the XDX and fp16 GELU' epilogues re-derive the lane id (q_lane_now)
#endif
#ifndef NSA_NT4_DDEF
#define NSA_NT4_DDEF 1  // 0 (A/B builds only): the GELU' epilogue stores all its rows itself
#endif
#ifndef NSA_NT4_XDEF
#define NSA_NT4_XDEF 1  // 0 (A/B builds only): the XENT epilogue stores all its rows itself
#endif
#ifndef NSA_NT4_GROW
#define NSA_NT4_GROW 1  // 0 (A/B builds only): the lookups row by row (one ballot and LDS round trip per row)
#endif

// pieces a K-tile has issued when it waits for the previous K-tile's
constexpr int Q_D0 = 15 * NSA_NT4_ER + 4;  // slot of the first piece
constexpr int Q_ISS = (NSA_NT4_VMS - Q_D0) / NSA_NT4_DS + 1 < 16 ? (NSA_NT4_VMS - Q_D0) / NSA_NT4_DS + 1 : 16;
// vector-memory operations one wave's epilogue of a full tile can leave outstanding (an
// upper bound: its stores, plus loads the compiler has not yet waited for)
template <int EPI>
constexpr int q_epi_vm() {
  return EPI == Q_EPI_BF16 ? 32 : EPI == Q_EPI_XENT ? 48 : 64;
}

typedef int q_i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t q_u32x4 __attribute__((ext_vector_type(4)));

struct Nt4Args {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;
  bf16_t* C2;
  const bf16_t* U;     // DGELU: gelu'(u) (fp16); GELU: the 5120-entry lookup table (see Q_GTAB)
  const bf16_t* bias;  // BIAS: bias[N] added before the store (and before GELU)
  // fused cross-entropy (see nsa_gemm_nt4_xent / _xdx below)
  const float* rowf;   // XENT: per-row shift c (the target logit); XDX: per-row pairs {g / S, g or 0}
  float* part;         // XENT: per-(column half-tile, row) partial sums of exp(logit - c)
  int nvalid;
  int M, N, K;
  int lda, ldb, ldc;
  int tiles_m, tiles_n, tiles;
  int gm;
};

template <int I>
using QI = std::integral_constant<int, I>;
template <class F, int... Is>
__device__ __forceinline__ void q_for(F&& f, std::integer_sequence<int, Is...>) {
  (f(QI<Is>{}), ...);
}

// H: fp16 operands (v_mfma_f32_16x16x32_f16, the same cycles); the fragments are raw bits
template <bool H>
__device__ __forceinline__ void q_mfma(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (H) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// first k-step of an output tile: the accumulator starts from 0 (no zeroing pass)
template <bool H>
__device__ __forceinline__ void q_mfma0(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (H) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(a), "v"(b));
}
// the overlapped epilogue's first-k-step MFMA: C = 0 like q_mfma0, but the accumulator operand
// is tied ("+a"), so the restarted tile lands in the same AGPRs and the previous tile's values
// are copied out (v_accvgpr_read) before it, not kept alive in other registers
template <bool H>
__device__ __forceinline__ void q_mfma0t(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  if constexpr (H) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "+a"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "+a"(acc) : "v"(a), "v"(b));
}
// a 16-byte row store pinned between the MFMAs (asm volatile statements keep their order):
// buffer resource over the previous tile (num_records 0 before the first tile: dropped),
// lane offset + row offset.  The leading nop covers an SGPR operand fresh from a VALU write
// (hipcc restores spilled SGPRs with v_readlane right before the asm, and pads nothing for an
// asm reader: without it the store took a stale row offset); the trailing one keeps the next
// instruction off its data registers until the store has read them
template <bool NT>
__device__ __forceinline__ void q_st16b(q_i32x4 rsrc, uint32_t voff, uint32_t soff, q_u32x4 v) {
  if constexpr (NT)
    asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, %3 offen nt\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rsrc),
                 "s"(soff)
                 : "memory");
  else
    asm volatile("s_nop 4\n\tbuffer_store_dwordx4 %0, %1, %2, %3 offen\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(rsrc),
                 "s"(soff)
                 : "memory");
}
// copy-out of one accumulator tile (four AGPRs) into VGPRs, pinned between the MFMAs
__device__ __forceinline__ void q_acc_rd(float (&t)[4], const f32x4& a) {
  asm volatile(
      "v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\t"
      "v_accvgpr_read_b32 %2, %6\n\tv_accvgpr_read_b32 %3, %7"
      : "=v"(t[0]), "=v"(t[1]), "=v"(t[2]), "=v"(t[3])
      : "a"(a[0]), "a"(a[1]), "a"(a[2]), "a"(a[3]));
}
// the next accumulator tile's copy-out packed with the previous one's values (lo = t, hi = a):
// w[e] = {t[e], a[e]} as bf16x2 (H: fp16x2; both RNE, the instructions pk2 compiles to)
template <bool H>
__device__ __forceinline__ void q_acc_rdpk(uint32_t (&w)[4], const float (&t)[4], const f32x4& a) {
  float x0, x1, x2, x3;
#define Q_RDPK(CVT)                                                                                              \
  asm volatile("v_accvgpr_read_b32 %4, %12\n\tv_accvgpr_read_b32 %5, %13\n\t"                                \
               "v_accvgpr_read_b32 %6, %14\n\tv_accvgpr_read_b32 %7, %15\n\t" CVT " %0, %8, %4\n\t" CVT        \
               " %1, %9, %5\n\t" CVT " %2, %10, %6\n\t" CVT " %3, %11, %7"                                      \
               : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3]), "=&v"(x0), "=&v"(x1), "=&v"(x2), "=&v"(x3) \
               : "v"(t[0]), "v"(t[1]), "v"(t[2]), "v"(t[3]), "a"(a[0]), "a"(a[1]), "a"(a[2]), "a"(a[3]))
  if constexpr (H) Q_RDPK("v_cvt_pk_f16_f32");
  else Q_RDPK("v_cvt_pk_bf16_f32");
#undef Q_RDPK
}
template <int OFF>
__device__ __forceinline__ void q_rd(bf16x8& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "n"(OFF));
}
// wait for every outstanding LDS read; the fragments it covers are named so the compiler
// cannot touch them before the data has landed (cdna_hip_programming.md "What hipcc does not do")
__device__ __forceinline__ void q_wait16(bf16x8 (&f)[8], bf16x8 (&h)[8]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]),
                 "+v"(h[0]), "+v"(h[1]), "+v"(h[2]), "+v"(h[3]), "+v"(h[4]), "+v"(h[5]), "+v"(h[6]), "+v"(h[7]));
}
__device__ __forceinline__ void q_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void q_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// one 1-KiB LDS-DMA piece: lane l's 16 bytes from rsrc.base + soff + voff + OFF land at
// M0 + OFF + 16 l.  Pieces go in groups of four consecutive KiB of LDS: the group's first
// piece (OFF = 0) writes M0, the other three reuse it with the instruction offset (which
// applies to the LDS and the global address alike; their soff carries -OFF), so a group
// costs one M0 write instead of four.  Nothing else in the kernel touches M0 between the
// pieces of a group (checked in the ISA: no other m0 writes).
template <int OFF>
__device__ __forceinline__ void q_dma(uint32_t lds, uint32_t voff, q_i32x4 rsrc, uint32_t soff) {
  if constexpr (OFF == 0) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(lds), "v"(voff),
                 "s"(rsrc), "s"(soff)
                 : "memory");
  } else {
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen offset:%3 lds" ::"v"(voff), "s"(rsrc), "s"(soff), "n"(OFF)
                 : "memory");
  }
}

#ifndef NSA_NT4_GLDS
#define NSA_NT4_GLDS 1  // 1: global_load_lds_dwordx4 (SGPR base + per-piece VGPR offset) instead of buffer_load ... lds
#endif
template <int OFF>
__device__ __forceinline__ void q_dmag(uint32_t lds, uint32_t voff, const void* sbase) {
  if constexpr (OFF == 0) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds), "v"(voff), "s"(sbase)
                 : "memory");
  } else {
    asm volatile("global_load_lds_dwordx4 %0, %1 offset:%2" ::"v"(voff), "s"(sbase), "n"(OFF) : "memory");
  }
}

__device__ __forceinline__ void q_tile_coords(const Nt4Args& g, int seq, int& m0, int& n0, int& mlo, int& nlo) {
  const int per = g.gm * g.tiles_n;
  const int grp = seq / per;
  const int first = grp * g.gm;
  const int gm = min(g.gm, g.tiles_m - first);
  const int in = seq - grp * per;
  mlo = (first + in % gm) * Q_BM;
  nlo = (in / gm) * Q_BN;
  m0 = min(mlo, g.M - Q_BM);
  n0 = min(nlo, g.N - Q_BN);
}

constexpr int Q_GRP = 3072;  // largest instruction offset inside an M0 group of DMA pieces

// raw buffer resource over [base, base + bytes): gfx9 word 3 = 0x00020000 (32-bit data format)
__device__ __forceinline__ q_i32x4 q_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  q_i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32) & 0xffff);
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

// DMA cursor: the K-tile whose pieces the current K-tile's slots issue (two ahead)
struct QCur {
  q_i32x4 ra, rb;
  int seq, k;
  bool valid;
};

__device__ __forceinline__ void q_cur_tile(const Nt4Args& g, QCur& c, int seq) {
  c.seq = seq;
  c.k = 0;
  c.valid = seq < g.tiles;
  if (c.valid) {
    int m0, n0, mlo, nlo;
    q_tile_coords(g, seq, m0, n0, mlo, nlo);
    // the resource base sits Q_GRP bytes below the tile's first row (every soffset carries
    // +Q_GRP), so the soffsets of a piece group never go negative
    c.ra = q_rsrc(reinterpret_cast<const char*>(g.A + (int64_t)m0 * g.lda) - Q_GRP, (uint32_t)(Q_BM * g.lda * 2 + Q_GRP));
    c.rb = q_rsrc(reinterpret_cast<const char*>(g.B + (int64_t)n0 * g.ldb) - Q_GRP, (uint32_t)(Q_BN * g.ldb * 2 + Q_GRP));
  } else {
    // past the last tile the slots still issue their pieces (no branches in the K-tile
    // body, vmcnt counts stay fixed): an empty range makes every load out of bounds, so
    // nothing is fetched and the never-read buffer receives zeros
    // (GLDS: no range check, so the base stays a real tile-0 address, lowered like the rest)
    c.ra = q_rsrc(reinterpret_cast<const char*>(g.A) - Q_GRP, 0);
    c.rb = q_rsrc(reinterpret_cast<const char*>(g.B) - Q_GRP, 0);
  }
}
__device__ __forceinline__ void q_add_base(q_i32x4& r, int bytes) {
  uint64_t b = ((uint64_t)(uint32_t)r.y << 32) | (uint32_t)r.x;
  b += (uint64_t)bytes;
  r.x = (int)(uint32_t)b;
  r.y = (int)(uint32_t)(b >> 32);
  r.z -= bytes;
}
__device__ __forceinline__ void q_cur_next(const Nt4Args& g, QCur& c, int nk, int G) {
  if (!c.valid) return;
  if (++c.k == nk) {
    q_cur_tile(g, c, c.seq + G);
  } else {
    q_add_base(c.ra, 2 * Q_BK);
    q_add_base(c.rb, 2 * Q_BK);
  }
}

// The wait for the previous K-tile's pieces.  vmcnt counts in issue order, so in the first
// K-tile after a full tile's epilogue that epilogue's stores (and U loads) are younger than
// the awaited pieces and may stay outstanding: the count grows by q_epi_vm (capped: when it
// would exceed the 6-bit field the epilogue has already drained down to the cap).
template <int ISS, int EPI>
__device__ __forceinline__ void q_vmw(bool after_epi) {
  constexpr int W = ISS == 0 ? 0 : (ISS + q_epi_vm<EPI>() < 63 ? ISS + q_epi_vm<EPI>() : 63);
  if (after_epi) q_vmwait<W>();
  else q_vmwait<ISS>();
}

// two f32 -> one dword of two bf16 (one v_cvt_pk_bf16_f32, RNE)
typedef __bf16 q_bf16x2 __attribute__((ext_vector_type(2)));
typedef float q_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t q_pk(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((q_f32x2){a, b}, q_bf16x2));
}

template <bool NT>
__device__ __forceinline__ void q_st16(bf16_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  if constexpr (NT) {
    __builtin_nontemporal_store(q_u32x4{a, b, c, d}, reinterpret_cast<q_u32x4*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = make_uint4(a, b, c, d);
  }
}

// sum over the 16 lanes of a DPP row (lanes 16 q .. 16 q + 15); every lane gets the total
__device__ __forceinline__ float q_rowsum16(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false));
  return v;
}

// Epilogue straight from the accumulators: for fragment row i and element e, lane l holds
// row 16 i + 4 (l >> 4) + e of the wave's 128 rows, columns 8 (l & 15) + 0..7 (fragments
// j = 0..7), so the 16 lanes of a quarter-wave write one row's 256 contiguous bytes.
//
// Fused cross-entropy (nanoGPT F.cross_entropy over the tied lm_head):
//  XENT (logits GEMM): E = exp(acc - c_row) in bf16 instead of the logits (columns >= nvalid,
//       the vocabulary padding, give 0), and the row sums of the fp32 E over the wave's 128
//       columns into part[2 tile_n + wn][row] (plain stores, one writer per slot: no atomics);
//  XDX  (dX = dlogits · W): out = g (acc / S_row - W[t_row]) in fp32 before the one rounding,
//       i.e. (softmax - onehot) · W without a dlogits tensor (ignored rows: 1/S = 0, no W row).
// The lane id, re-derived where it is used: opaque to the compiler, so the lane-derived row and
// column offsets are not kept live across the K-loop (the XDX epilogue spilled two of them).
__device__ __forceinline__ int q_lane_now() {
  int l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

template <int EPI, bool NT, bool BIAS, bool NOSTORE = false, bool H = false, bool DEFER = false>
__device__ __forceinline__ void q_epilogue(const Nt4Args& g, const f32x4 (&acc)[8][8], int seq, int wm, int wn,
                                           int lane, const char* tab, uint32_t (&defer)[4][4][4]) {
  int m0, n0, mlo, nlo;
  q_tile_coords(g, seq, m0, n0, mlo, nlo);
  const bool full = (m0 == mlo) & (n0 == nlo);
  if constexpr ((EPI == Q_EPI_XDX || (EPI == Q_EPI_DGELU && H)) && NSA_NT4_XLANE) lane = q_lane_now();
  const int r = lane & 15, q = lane >> 4;
  const int col = n0 + wn * 128 + 8 * r;
  const int row0 = m0 + wm * 128 + 4 * q;
  float bv[8];
  if constexpr (BIAS) load8e<H>(g.bias + col, bv);
  // EPI_DGELU: the U pieces of two fragment rows are in flight at a time
  q_u32x4 uv[2][4];
  auto load_u = [&](int i, q_u32x4 (&dst)[4]) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = row0 + 16 * i + e;  // in bounds: tiles lie inside the matrix
      dst[e] = __builtin_nontemporal_load(reinterpret_cast<const q_u32x4*>(g.U + (int64_t)row * g.ldc + col));
    }
  };
  if constexpr (EPI == Q_EPI_DGELU) {
    load_u(0, uv[0]);
    load_u(1, uv[1]);
  }
  // EPI_XENT: the shift c of the lane's 32 rows (log2 units), the vocabulary-padding edge
  constexpr float kLog2e = 1.4426950408889634f;
  f32x4 crow[8];
  if constexpr (EPI == Q_EPI_XENT) {
#pragma unroll
    for (int i = 0; i < 8; ++i) crow[i] = *reinterpret_cast<const f32x4*>(g.rowf + row0 + 16 * i) * kLog2e;
  }
  const bool edge = EPI == Q_EPI_XENT && n0 + wn * 128 + 128 > g.nvalid;
  const int tn = nlo / Q_BN;  // column tile index
  // EPI_XDX: per fragment row the 4 rows' coefficient pairs {g / S, g or 0}, two rows ahead
  // (with the gathered W rows, which ride in U like the GELU' epilogue's pre-activations)
  f32x4 xc[2][2];
  auto load_c = [&](int i, f32x4 (&dst)[2]) {
    const f32x4* p = reinterpret_cast<const f32x4*>(g.rowf + 2 * (row0 + 16 * i));
    dst[0] = p[0];
    dst[1] = p[1];
  };
  if constexpr (EPI == Q_EPI_XDX) {
    load_u(0, uv[0]);
    load_u(1, uv[1]);
    load_c(0, xc[0]);
    load_c(1, xc[1]);
  }
  // one base pointer per lane; a store's row offset (16 i + e) rows is wave-uniform
  bf16_t* const cb = g.C + (int64_t)row0 * g.ldc + col;
  bf16_t* const cb2 = EPI == Q_EPI_GELU ? g.C2 + (int64_t)row0 * g.ldc + col : nullptr;
  if constexpr (EPI == Q_EPI_DGELU && NSA_NT4_GROW) {
    // acc * gelu'(u) one fragment row at a time, with the U rows two fragment rows ahead
    // loaded BEFORE this row's stores: vmcnt completes in order, so a U load issued after a
    // row's stores made the next-but-one row wait for those stores' acknowledgements
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t w[4][4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t b = pk2<H>(acc[i][2 * h][e], acc[i][2 * h + 1][e]);
          const nsa_f32x2 a = nsa_f32x2{lo2f<H>(b), hi2f<H>(b)} * nsa_unpk_f16(uv[i & 1][e][h]);
          w[e][h] = pk2<H>(a.x, a.y);
        }
      if (i + 2 < 8) load_u(i + 2, uv[i & 1]);
      if (DEFER && i >= 4) {  // DDEF: rows 4-7 go out from the next tile's first K-tile
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int h = 0; h < 4; ++h) defer[i - 4][e][h] = w[e][h];
        continue;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool skip = !full && (row0 + 16 * i + e < mlo || col < nlo);
        if (skip) continue;
        const int64_t off = (int64_t)(16 * i + e) * g.ldc;
        if constexpr (NOSTORE) asm volatile("" ::"v"(w[e][0]), "v"(w[e][1]), "v"(w[e][2]), "v"(w[e][3]));
        else q_st16<NT>(cb + off, w[e][0], w[e][1], w[e][2], w[e][3]);
      }
    }
    return;
  }
  if constexpr (EPI == Q_EPI_GELU && !H && !BIAS && NSA_NT4_GTAB && NSA_NT4_GROW) {
    // GELU by lookup, one fragment row (4 output rows, 32 values per lane) at a time: one
    // ballot for the group and its 32 table reads in flight together, instead of a branch
    // and a dependent LDS round trip per output row (not with a bias: 44 B of spills)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      uint32_t w[4][4], ia[4][4], ib[4][4];
      bool oob = false;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          float v0 = acc[i][2 * h][e], v1 = acc[i][2 * h + 1][e];
          if constexpr (BIAS) {
            v0 += bv[2 * h];
            v1 += bv[2 * h + 1];
          }
          const uint32_t b = q_pk(v0, v1);
          w[e][h] = b;
          const uint32_t t0 = (b & 0x7fffu) - (uint32_t)Q_GTAB_LO, t1 = ((b >> 16) & 0x7fffu) - (uint32_t)Q_GTAB_LO;
          oob |= (t0 >= (uint32_t)Q_GTAB_N) | (t1 >= (uint32_t)Q_GTAB_N);
          ia[e][h] = 4u * (t0 + ((b >> 15) & 1u) * (uint32_t)Q_GTAB_N);
          ib[e][h] = 4u * (t1 + (b >> 31) * (uint32_t)Q_GTAB_N);
        }
      }
      uint32_t gg[4][4], gp[4][4];
      if (__builtin_amdgcn_ballot_w64(oob) == 0) {
        uint32_t ea[4][4], eb[4][4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            ea[e][h] = *reinterpret_cast<const uint32_t*>(tab + ia[e][h]);
            eb[e][h] = *reinterpret_cast<const uint32_t*>(tab + ib[e][h]);
          }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            gg[e][h] = __builtin_amdgcn_perm(eb[e][h], ea[e][h], 0x05040100u);  // the two gelu(u) halves
            gp[e][h] = __builtin_amdgcn_perm(eb[e][h], ea[e][h], 0x07060302u);  // the two gelu'(u) halves
          }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            nsa_f32x2 gv, dv;
            nsa_gelu_and_grad2(nsa_f32x2{lo2f<false>(w[e][h]), hi2f<false>(w[e][h])}, gv, dv);
            gg[e][h] = q_pk(gv.x, gv.y);
            gp[e][h] = nsa_pk_f16(dv.x, dv.y);
          }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool skip = !full && (row0 + 16 * i + e < mlo || col < nlo);
        if (skip) continue;
        const int64_t off = (int64_t)(16 * i + e) * g.ldc;
        if constexpr (NOSTORE) {
          asm volatile("" ::"v"(gp[e][0]), "v"(gp[e][1]), "v"(gp[e][2]), "v"(gp[e][3]), "v"(gg[e][0]), "v"(gg[e][1]),
                       "v"(gg[e][2]), "v"(gg[e][3]));
        } else {
          q_st16<NT>(cb + off, gp[e][0], gp[e][1], gp[e][2], gp[e][3]);
          q_st16<NT>(cb2 + off, gg[e][0], gg[e][1], gg[e][2], gg[e][3]);
        }
      }
    }
    return;
  }
  {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float rs[4];  // XENT: the 4 rows' partial sums
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool skip = !full && (row0 + 16 * i + e < mlo || col < nlo);
        const int64_t off = (int64_t)(16 * i + e) * g.ldc;
        if constexpr (EPI == Q_EPI_XENT) {
          // no early exit here: every lane takes part in the row reduction
          const float c = crow[i][e];
          uint32_t w[4];
          float s = 0.0f, mx = 0.0f;
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            float e0 = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i][2 * h][e], kLog2e, -c));
            float e1 = __builtin_amdgcn_exp2f(__builtin_fmaf(acc[i][2 * h + 1][e], kLog2e, -c));
            if (edge) {
              e0 = col + 2 * h < g.nvalid ? e0 : 0.0f;
              e1 = col + 2 * h + 1 < g.nvalid ? e1 : 0.0f;
            }
            w[h] = H ? pk2<true>(e0, e1) : q_pk(e0, e1);
            s += e0 + e1;
            if constexpr (H) mx = __builtin_fmaxf(mx, __builtin_fmaxf(e0, e1));
          }
          // fp16 E saturates at 65504 (a logit ~11 nats above the row's target): such a row's
          // sum is made inf, so nsa_xent_combine sends it to the exact fix-up
          if constexpr (H) s = mx > 65504.0f ? __builtin_inff() : s;
          rs[e] = q_rowsum16(col < nlo ? 0.0f : s);
          if (DEFER && i >= 4) {
            // XDEF: fragment rows 4-7 go out from the next tile's first K-tile (every row:
            // rows another tile also covers get the same bits)
#pragma unroll
            for (int h = 0; h < 4; ++h) defer[i - 4][e][h] = w[h];
          } else if (!skip) {
            if constexpr (NOSTORE) asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
            else q_st16<NT>(cb + off, w[0], w[1], w[2], w[3]);
          }
          continue;
        }
        if (skip) continue;
        uint32_t w[4];
        if constexpr (EPI == Q_EPI_XDX) {
          const float sc = xc[i & 1][e >> 1][2 * (e & 1)];
          const float gw = xc[i & 1][e >> 1][2 * (e & 1) + 1];
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const uint32_t wr = uv[i & 1][e][h];
            const float v0 = __builtin_fmaf(sc, acc[i][2 * h][e], -gw * lo2f<H>(wr));
            const float v1 = __builtin_fmaf(sc, acc[i][2 * h + 1][e], -gw * hi2f<H>(wr));
            w[h] = H ? pk2<true>(v0, v1) : q_pk(v0, v1);
          }
        } else if constexpr (BIAS) {
#pragma unroll
          for (int h = 0; h < 4; ++h)
            w[h] = pk2<H>(acc[i][2 * h][e] + bv[2 * h], acc[i][2 * h + 1][e] + bv[2 * h + 1]);
        } else {
#pragma unroll
          for (int h = 0; h < 4; ++h) w[h] = pk2<H>(acc[i][2 * h][e], acc[i][2 * h + 1][e]);
        }
        if constexpr (EPI == Q_EPI_DGELU) {
          // U holds gelu'(u) as fp16 pairs (written by the forward's GELU epilogue)
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const nsa_f32x2 a = nsa_f32x2{lo2f<H>(w[h]), hi2f<H>(w[h])} * nsa_unpk_f16(uv[i & 1][e][h]);
            w[h] = pk2<H>(a.x, a.y);
          }
        }
        if constexpr (EPI == Q_EPI_GELU) {
          // u = w (bf16, as the reference's autocast c_fc output): C <- gelu'(u) as fp16 (the
          // backward's only use of u, so its GELU' epilogue is one multiply), C2 <- gelu(u)
          uint32_t gg[4], gp[4];
          uint32_t ia[4], ib[4];
          bool oob = false;
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const uint32_t b = w[h];
            const uint32_t t0 = (b & 0x7fffu) - (uint32_t)Q_GTAB_LO, t1 = ((b >> 16) & 0x7fffu) - (uint32_t)Q_GTAB_LO;
            oob |= (t0 >= (uint32_t)Q_GTAB_N) | (t1 >= (uint32_t)Q_GTAB_N);
            ia[h] = 4u * (t0 + ((b >> 15) & 1u) * (uint32_t)Q_GTAB_N);
            ib[h] = 4u * (t1 + (b >> 31) * (uint32_t)Q_GTAB_N);
          }
          // the table is indexed by bf16 bit patterns: fp16 outputs take the arithmetic path
          if (NSA_NT4_GTAB && !H && __builtin_amdgcn_ballot_w64(oob) == 0) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              const uint32_t ea = *reinterpret_cast<const uint32_t*>(tab + ia[h]);
              const uint32_t eb = *reinterpret_cast<const uint32_t*>(tab + ib[h]);
              gg[h] = __builtin_amdgcn_perm(eb, ea, 0x05040100u);  // the two gelu(u) halves
              gp[h] = __builtin_amdgcn_perm(eb, ea, 0x07060302u);  // the two gelu'(u) halves
            }
          } else {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              nsa_f32x2 gv, dv;
              nsa_gelu_and_grad2(nsa_f32x2{lo2f<H>(w[h]), hi2f<H>(w[h])}, gv, dv);
              gg[h] = pk2<H>(gv.x, gv.y);
              gp[h] = nsa_pk_f16(dv.x, dv.y);
            }
          }
          if constexpr (NOSTORE) {
            asm volatile("" ::"v"(gp[0]), "v"(gp[1]), "v"(gp[2]), "v"(gp[3]), "v"(gg[0]), "v"(gg[1]), "v"(gg[2]),
                         "v"(gg[3]));
          } else {
            q_st16<NT>(cb + off, gp[0], gp[1], gp[2], gp[3]);
            q_st16<NT>(cb2 + off, gg[0], gg[1], gg[2], gg[3]);
          }
        } else if constexpr (NOSTORE) {
          asm volatile("" ::"v"(w[0]), "v"(w[1]), "v"(w[2]), "v"(w[3]));
        } else {
          q_st16<NT>(cb + off, w[0], w[1], w[2], w[3]);
        }
      }
      if constexpr (EPI == Q_EPI_XENT) {
        // lanes r = 0..3 of each row group write the 4 rows' sums (one slot per wave column half)
        const int row = row0 + 16 * i + r;
        const float v = r == 0 ? rs[0] : r == 1 ? rs[1] : r == 2 ? rs[2] : rs[3];
        if (r < 4 && row >= mlo && !NOSTORE) g.part[(int64_t)(2 * tn + wn) * g.M + row] = v;
      }
      if constexpr (EPI == Q_EPI_DGELU || EPI == Q_EPI_XDX) {
        if (i + 2 < 8) load_u(i + 2, uv[i & 1]);
      }
      if constexpr (EPI == Q_EPI_XDX) {
        if (i + 2 < 8) load_c(i + 2, xc[i & 1]);
      }
    }
  }
}

}  // namespace

// PROBE (timing only, wrong results; compiled in only with -DNSA_PROBES, i.e. a
// build_variant library): 1 = no DMA after the prologue, 2 = no wait for the previous
// K-tile's pieces, 3 = no barriers in the K-loop, 4 = no epilogue at all, 5 = epilogue
// arithmetic without its stores
template <int EPI, bool NT, int PROBE, bool BIAS = false, bool H = false, bool OVLE = false>
__global__ __launch_bounds__(Q_THR, 1) void gemm_nt4_kernel(Nt4Args g) {
  static_assert(!OVLE || (EPI == Q_EPI_BF16 && !BIAS && PROBE == 0), "OVL: plain 16-bit outputs only");
  __shared__ __attribute__((aligned(16))) char smem[Q_SMEM + (EPI == Q_EPI_GELU && !H ? Q_GTAB_BYTES : 0)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int G = gridDim.x;
  const int nk = g.K / Q_BK;
  // GELU: the lookup table first (LDS address 0: an index is its own LDS address), then the
  // operand buffers
  constexpr int QT = EPI == Q_EPI_GELU && !H ? Q_GTAB_BYTES : 0;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem + QT));

  // XCD-aware virtual block id: blocks b, b+8, ... share an XCD and get consecutive ids
  int v = blockIdx.x;
  {
    const int x = v % 8, qq = G / 8, rr = G % 8;
    v = (x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq) + v / 8;
  }
  if (v >= g.tiles) return;
  if constexpr (EPI == Q_EPI_GELU && !H) {  // the GELU table into LDS (before any operand DMA is in flight)
    const uint4* src = reinterpret_cast<const uint4*>(g.U);
    uint4* dst = reinterpret_cast<uint4*>(smem);
    for (int k = threadIdx.x; k < Q_GTAB_BYTES / 16; k += Q_THR) dst[k] = src[k];
  }

  // ---- DMA geometry.  Wave w copies pieces P = 8 w + p (p = 0..7) of each image: image rows
  // 8 P + i, i = lane >> 3, physical 16-B chunk lane & 7, which holds logical chunk
  // (lane & 7) ^ s(row), s(r) = (r >> 1) & 7 = (4 (p & 1) + (i >> 1)) & 7.
  // A: image row = tile row.  B: image row q = 128 h + 16 j + r holds tile column
  // 128 h + 8 r + j (see the header): for a piece, 128 (w >> 1) + 64 (p & 1) + 4 (w & 1)
  // + (p >> 1) + 8 i.
  const int li = lane >> 3, lc = lane & 7;
  uint32_t voA[2], voB[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t ch = (uint32_t)((lc ^ ((4 * h + (li >> 1)) & 7)) << 4);
    voA[h] = (uint32_t)(li * g.lda * 2) + ch;
    voB[h] = (uint32_t)(8 * li * g.ldb * 2) + ch;
  }
  // per-piece row offsets, less the instruction offset of the piece in its M0 group, plus the
  // Q_GRP the resource base was lowered by (so never negative)
  uint32_t soA[8], soB[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    soA[p] = (uint32_t)__builtin_amdgcn_readfirstlane((64 * wave + 8 * p) * g.lda * 2 + Q_GRP - (p & 3) * 1024);
    soB[p] = (uint32_t)__builtin_amdgcn_readfirstlane(
        (128 * (wave >> 1) + 64 * (p & 1) + 4 * (wave & 1) + (p >> 1)) * g.ldb * 2 + Q_GRP - (p & 3) * 1024);
  }
  const uint32_t dmaA0 = lds0 + (uint32_t)(wave * 8 * 1024);          // + buffer + p * 1 KiB
  const uint32_t dmaB0 = lds0 + (uint32_t)(Q_IMG + wave * 8 * 1024);

  // ---- fragment read bases (buffer 0): A rows wm*128 + 16 i + (lane & 15), B image rows
  // wn*128 + 16 j + (lane & 15), logical chunk 4 kk + (lane >> 4)
  const int sw = ((lane & 15) >> 1) & 7;
  uint32_t rA[2], rB[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const uint32_t ch = (uint32_t)(((4 * kk + (lane >> 4)) ^ sw) << 4);
    rA[kk] = lds0 + (uint32_t)((wm * 128 + (lane & 15)) * 128) + ch;
    rB[kk] = lds0 + (uint32_t)(Q_IMG + (wn * 128 + (lane & 15)) * 128) + ch;
  }

  // piece P of K-tile cursor c into buffer buf (the pieces of an M0 group are issued in order)
  // GLDS: per-piece VGPR offsets (row offset folded in), the tile base as an SGPR pair.  (The
  // plain-epilogue instantiations spill a few of these: 2 x 6 VGPRs, reloaded behind a
  // vmcnt(0) at the epilogue head.  Adding voff + soff at each issue instead (no spills)
  // measured 2.8 ms/step slower: the 16 adds per K-tile cost more than the drain.)
  uint32_t vpA[NSA_NT4_GLDS ? 8 : 1], vpB[NSA_NT4_GLDS ? 8 : 1];
  if constexpr (NSA_NT4_GLDS) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      vpA[p] = voA[p & 1] + soA[p];
      vpB[p] = voB[p & 1] + soB[p];
    }
  }
  auto sbase = [](const q_i32x4& r) {
    return reinterpret_cast<const void*>(((uint64_t)(uint32_t)r.y << 32) | (uint32_t)r.x);
  };
  auto issue_a = [&](const QCur& c, uint32_t buf, auto P) {
    constexpr int p = decltype(P)::value;
    if constexpr (NSA_NT4_GLDS)
      q_dmag<(p & 3) * 1024>(dmaA0 + buf + (uint32_t)((p & 4) * 1024), vpA[p], sbase(c.ra));
    else
      q_dma<(p & 3) * 1024>(dmaA0 + buf + (uint32_t)((p & 4) * 1024), voA[p & 1], c.ra, soA[p]);
  };
  auto issue_b = [&](const QCur& c, uint32_t buf, auto P) {
    constexpr int p = decltype(P)::value;
    if constexpr (NSA_NT4_GLDS)
      q_dmag<(p & 3) * 1024>(dmaB0 + buf + (uint32_t)((p & 4) * 1024), vpB[p], sbase(c.rb));
    else
      q_dma<(p & 3) * 1024>(dmaB0 + buf + (uint32_t)((p & 4) * 1024), voB[p & 1], c.rb, soB[p]);
  };

  // ---- prologue: K-tiles 0 and 1 of this workgroup's sequence into buffers 0 / 1
  QCur c;
  q_cur_tile(g, c, v);
  q_for([&](auto P) { issue_a(c, 0, P); }, std::make_integer_sequence<int, 8>{});
  q_for([&](auto P) { issue_b(c, 0, P); }, std::make_integer_sequence<int, 8>{});
  q_cur_next(g, c, nk, G);
  q_for([&](auto P) { issue_a(c, Q_BUF, P); }, std::make_integer_sequence<int, 8>{});
  q_for([&](auto P) { issue_b(c, Q_BUF, P); }, std::make_integer_sequence<int, 8>{});
  q_vmwait<16>();
  q_cur_next(g, c, nk, G);  // c = the K-tile the first loop iteration's slots issue (two ahead)
  q_barrier();

  f32x4 acc[8][8];
  bf16x8 a0[8], b0[8], a1[8], b1[8];
  q_for([&](auto I) {
    constexpr int n = decltype(I)::value;
    q_rd<n * 2048>(a0[n], rA[0]);
    q_rd<n * 2048>(b0[n], rB[0]);
  }, std::make_integer_sequence<int, 8>{});
  q_wait16(a0, b0);

  uint32_t buf = 0;  // LDS buffer of the K-tile being multiplied (byte offset 0 / Q_BUF)
  int seq = v;
  bool pend = false;  // the previous tile's epilogue left its vector-memory ops in flight
  // one 64-deep K-tile; FIRST: the tile's first, whose k-step 0 starts the accumulators at 0
  // OVL: the previous tile's accumulators leave fragment row by fragment row (i outer in
  // k-step 0): each is read out just before the MFMA that restarts it, and a row's four
  // 256-byte row stores go out after its eighth MFMA (pcb: the previous tile's base pointer)
  float ovt[4];
  uint32_t ovw[4][4];
  uint32_t ovd[4][4][4];  // OVL2: fragment rows 4-7, [i - 4][e][h], stored by the next K-tile
  q_i32x4 prs = q_rsrc(g.C, 0);  // the previous tile (none yet: every store out of range)
  const uint32_t pvo = (uint32_t)(((wm * 128 + 4 * (lane >> 4)) * g.ldc + wn * 128 + 8 * (lane & 15)) * 2);
  auto ktile = [&](auto FIRST_, auto OVL_, auto DEF_) {
    constexpr bool FIRST = decltype(FIRST_)::value;
    constexpr bool OVL = decltype(OVL_)::value;
    constexpr bool DEF = decltype(DEF_)::value;  // OVL2: this K-tile stores the deferred rows
    static_assert(!OVL || FIRST, "the overlapped epilogue rides in a tile's first K-tile");
    static_assert(!DEF || !FIRST || ((EPI == Q_EPI_XENT || EPI == Q_EPI_DGELU) && !OVL),
                  "OVL2's deferred rows go out in a tile's second K-tile");
    constexpr bool OV2 = OVL && NSA_NT4_OVL2;
    constexpr bool dv = PROBE != 1;
    const uint32_t nb = buf ^ (uint32_t)Q_BUF;
    q_for([&](auto I) {
      constexpr int n = decltype(I)::value;
      constexpr int kk = n >> 6;
      constexpr int j = OVL && kk == 0 ? n & 7 : (n >> 3) & 7;
      constexpr int i = OVL && kk == 0 ? (n >> 3) & 7 : n & 7;
      if constexpr (kk == 0) {
        if constexpr (OVL) {
          // the copy-out is itself pinned (volatile asm), so hipcc cannot hoist the 256
          // copies ahead of the K-tile; odd j packs with the even j before it (bf16 pairs of
          // adjacent columns, as one 16-byte row store wants them)
          if constexpr (j % 2 == 0) q_acc_rd(ovt, acc[i][j]);
          else q_acc_rdpk<H>(ovw[j >> 1], ovt, acc[i][j]);
          q_mfma0t<H>(acc[i][j], a0[i], b0[j]);
        } else if constexpr (FIRST) {
          q_mfma0<H>(acc[i][j], a0[i], b0[j]);
        } else {
          q_mfma<H>(acc[i][j], a0[i], b0[j]);
        }
        if constexpr (OVL && n == 63) {
          // the A fragments stay allocated to the end of k-step 0: no copy-out temporary may
          // take an A fragment's registers while an MFMA that reads them is still in flight
          asm volatile("" ::"v"(a0[0]), "v"(a0[1]), "v"(a0[2]), "v"(a0[3]), "v"(a0[4]), "v"(a0[5]), "v"(a0[6]),
                       "v"(a0[7]));
        }
        if constexpr (OVL && j == 7) {
          if constexpr (OV2 && i >= 4) {
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
              for (int h = 0; h < 4; ++h) ovd[i - 4][e][h] = ovw[h][e];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              q_st16b<NT>(prs, pvo, (uint32_t)((16 * i + e) * g.ldc * 2),
                          q_u32x4{ovw[0][e], ovw[1][e], ovw[2][e], ovw[3][e]});
          }
        }
      } else {
        q_mfma<H>(acc[i][j], a1[i], b1[j]);
      }
      if constexpr (DEF && n < 16) {
        constexpr int di = n >> 2, de = n & 3;
        q_st16b<NT>(prs, pvo, (uint32_t)((16 * (4 + di) + de) * g.ldc * 2),
                    q_u32x4{ovd[di][de][0], ovd[di][de][1], ovd[di][de][2], ovd[di][de][3]});
      }
      // two barriers per K-tile: both k-step-1 image reads first, then all 16 pieces of
      // K-tile t+2 spread one per DS MFMAs, then K-tile t+1's k-step-0 fragments
      constexpr int ER = NSA_NT4_ER;  // MFMAs between the k-step-1 fragment reads
      if constexpr (n <= 15 * ER && n % ER == 0) {
        constexpr int s = n / ER;
        if constexpr (s < 8) q_rd<s * 2048>(a1[s], rA[1] + buf);
        else q_rd<(s - 8) * 2048>(b1[s - 8], rB[1] + buf);
      }
      if constexpr (n == 15 * ER + 2) q_wait16(a1, b1);
      if constexpr (n == 15 * ER + 3 && PROBE != 3) q_barrier();
      constexpr int D0 = 15 * ER + 4, DS = NSA_NT4_DS, VMS = NSA_NT4_VMS;
      static_assert(D0 + 15 * DS <= 127 && VMS + 2 + 15 * NSA_NT4_RS <= 127, "every piece and read fits the K-tile");
      if constexpr (n >= D0 && (n - D0) % DS == 0 && (n - D0) / DS < 16) {
        constexpr int pc = (n - D0) / DS;
        if constexpr (dv) {
          if constexpr (pc < 8) issue_a(c, buf, QI<pc>{});
          else issue_b(c, buf, QI<pc - 8>{});
        }
      }
      constexpr int issued = (VMS - D0) / DS + 1 < 16 ? (VMS - D0) / DS + 1 : 16;
      if constexpr (n == VMS && PROBE != 2) {
        // every store an OVL2 K-tile issued before this wait is younger than the pieces it waits
        // for; XDEF (XENT's first K-tile): the previous epilogue left 32 operations and this
        // K-tile's 16 deferred stores, 48 = q_epi_vm<XENT> (a tail tile's epilogue drained)
        if constexpr ((EPI == Q_EPI_XENT || EPI == Q_EPI_DGELU) && DEF) q_vmw<dv ? issued : 0, EPI>(pend);
        else if constexpr (OV2 || DEF) q_vmwait<(dv ? issued : 0) + 16>();
        else q_vmw<dv ? issued : 0, EPI>(FIRST && (pend || OVL));
      }
      if constexpr (n == VMS + 1 && PROBE != 3) q_barrier();
      if constexpr (n >= VMS + 2 && n < VMS + 2 + 16 * NSA_NT4_RS && (n - VMS - 2) % NSA_NT4_RS == 0) {
        constexpr int s = (n - VMS - 2) / NSA_NT4_RS;
        if constexpr (s < 8) q_rd<s * 2048>(b0[s], rB[0] + nb);
        else q_rd<(s - 8) * 2048>(a0[s - 8], rA[0] + nb);
      }
      if constexpr (n == 127) q_wait16(a0, b0);
    }, std::make_integer_sequence<int, 128>{});
    buf = nb;
    q_cur_next(g, c, nk, G);
  };
  if constexpr (OVLE) {
    // every tile's first K-tile stores the previous tile (the first tile's copy-out reads these
    // zeros and its stores are dropped).  Tail tiles store all of their rows and columns: the
    // ones another tile also covers get the same bits twice (same operands, same K order).
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    int last;
    while (true) {
      ktile(std::true_type{}, std::true_type{}, std::false_type{});
      if constexpr (NSA_NT4_OVL2) {
        ktile(std::false_type{}, std::false_type{}, std::true_type{});  // nk >= 2 (host check)
        for (int kt = 2; kt < nk; ++kt) ktile(std::false_type{}, std::false_type{}, std::false_type{});
      } else {
        for (int kt = 1; kt < nk; ++kt) ktile(std::false_type{}, std::false_type{}, std::false_type{});
      }
      last = seq;
      seq += G;
      if (seq >= g.tiles) break;
      int m0, n0, mlo, nlo;
      q_tile_coords(g, last, m0, n0, mlo, nlo);
      prs = q_rsrc(g.C + (int64_t)m0 * g.ldc + n0, 0x7fffffffu);
    }
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    q_epilogue<EPI, NT, BIAS, false, H>(g, acc, last, wm, wn, lane, smem, ovd);
    q_vmwait<0>();
    return;
  }
  // XDEF (XENT) / DDEF (GELU'): the epilogue leaves fragment rows 4-7 (16 row stores) to the
  // next tile's first K-tile, where the write path drains them under the MFMAs
  constexpr bool XDEF = PROBE == 0 && ((EPI == Q_EPI_XENT && NSA_NT4_XDEF) ||
                                       (EPI == Q_EPI_DGELU && !H && NSA_NT4_GROW && NSA_NT4_DDEF));
  while (true) {
    if constexpr (XDEF) ktile(std::true_type{}, std::false_type{}, std::true_type{});
    else ktile(std::true_type{}, std::false_type{}, std::false_type{});
    for (int kt = 1; kt < nk; ++kt) ktile(std::false_type{}, std::false_type{}, std::false_type{});
    // MFMA results -> VALU reads: let the last MFMAs drain (hazard not tracked through asm)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    if constexpr (PROBE != 4) {
      q_epilogue<EPI, NT, BIAS, PROBE == 5, H, XDEF>(g, acc, seq, wm, wn, lane, smem, ovd);
      if constexpr (XDEF) {
        int m0, n0, mlo, nlo;
        q_tile_coords(g, seq, m0, n0, mlo, nlo);
        prs = q_rsrc(g.C + (int64_t)m0 * g.ldc + n0, 0x7fffffffu);  // the next tile's first K-tile stores rows 4-7
      }
      int m0, n0, mlo, nlo;
      q_tile_coords(g, seq, m0, n0, mlo, nlo);
      if ((m0 == mlo) & (n0 == nlo)) {
        // every store was issued: the next tile's first wait counts them
        if constexpr (q_epi_vm<EPI>() + Q_ISS > 63) q_vmwait<63 - Q_ISS>();
        pend = true;
      } else {
        q_vmwait<0>();  // a tail tile skips masked stores: drain instead of counting
        pend = false;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) asm volatile("" ::"a"(acc[i][j]));
    }
    seq += G;
    if (seq >= g.tiles) break;
  }
  if constexpr (XDEF) {  // the last tile's deferred rows
#pragma unroll
    for (int di = 0; di < 4; ++di)
#pragma unroll
      for (int de = 0; de < 4; ++de)
        q_st16b<NT>(prs, pvo, (uint32_t)((16 * (4 + di) + de) * g.ldc * 2),
                    q_u32x4{ovd[di][de][0], ovd[di][de][1], ovd[di][de][2], ovd[di][de][3]});
  }
  q_vmwait<0>();
}

namespace {

hipError_t nt4_check(const Nt4Args& a, int grid) {
  if (a.M < Q_BM || a.N < Q_BN || a.K < Q_BK || a.K % Q_BK != 0 || a.N % 8 || a.lda % 8 || a.ldb % 8 || a.ldc % 8 ||
      a.lda < a.K || a.ldb < a.K || a.ldc < a.N || grid < 1)
    return hipErrorInvalidValue;
  if ((int64_t)Q_BM * a.lda * 2 + Q_GRP >= (1ll << 31) || (int64_t)Q_BN * a.ldb * 2 + Q_GRP >= (1ll << 31))
    return hipErrorInvalidValue;
  return hipSuccess;
}

void nt4_geometry(Nt4Args& a, int gmsel) {
  a.tiles_m = (a.M + Q_BM - 1) / Q_BM;
  a.tiles_n = (a.N + Q_BN - 1) / Q_BN;
  a.tiles = a.tiles_m * a.tiles_n;
  // tile groups (q_cur_tile): 4 row blocks x every column for the N <= 1024 outputs (c_attn /
  // c_fc dX, attn.c_proj, mlp.c_proj: 0.2-2.3 % faster than 1), rows for N <= 4096, 8 beyond
  a.gm = gmsel ? gmsel : (a.tiles_n <= 4 ? 4 : a.tiles_n <= 16 ? 1 : 8);
}

template <int E, bool B, bool H = false>
void nt4_launch(const Nt4Args& a, dim3 gr, bool nt, int probe, hipStream_t s, bool ovl = false) {
  if constexpr (E == Q_EPI_BF16 && !B) {
    if (ovl && probe == 0) {
      if (nt) gemm_nt4_kernel<E, true, 0, false, H, true><<<gr, Q_THR, 0, s>>>(a);
      else gemm_nt4_kernel<E, false, 0, false, H, true><<<gr, Q_THR, 0, s>>>(a);
      return;
    }
  }
#ifdef NSA_PROBES
  switch (probe) {
    case 1: gemm_nt4_kernel<E, true, 1, B, H><<<gr, Q_THR, 0, s>>>(a); return;
    case 2: gemm_nt4_kernel<E, true, 2, B, H><<<gr, Q_THR, 0, s>>>(a); return;
    case 3: gemm_nt4_kernel<E, true, 3, B, H><<<gr, Q_THR, 0, s>>>(a); return;
    case 4: gemm_nt4_kernel<E, true, 4, B, H><<<gr, Q_THR, 0, s>>>(a); return;
    case 5: gemm_nt4_kernel<E, true, 5, B, H><<<gr, Q_THR, 0, s>>>(a); return;
    default: break;
  }
#else
  (void)probe;
#endif
  if (nt) gemm_nt4_kernel<E, true, 0, B, H><<<gr, Q_THR, 0, s>>>(a);
  else gemm_nt4_kernel<E, false, 0, B, H><<<gr, Q_THR, 0, s>>>(a);
}

bool nt4_store_nt(int stp, int64_t out_bytes) { return stp == 1 || (stp == 0 && out_bytes >= NSA_NT_MIN_BYTES); }

}  // namespace

// C = A · B^T (bf16) with an optional bias[N] (bf16) added to every row.
// epi: 0 bf16, 1 gelu'(u) (fp16) / gelu(u) into C / C2, 2 acc * U (U = gelu'(u), fp16); bits 8-11 timing probe (-DNSA_PROBES
// builds only; 1 no DMA, 4 no stores, ...); bits 12-13 store policy: 0 nontemporal above the
// Infinity Cache, 1 always, 2 never; bits 14-15 overlapped epilogue (plain bf16 without bias):
// 0 from K = Q_OVL_MIN_K, 1 always, 2 never; bits 16-23 row-blocks per tile group, 0 = automatic.
// grid = persistent workgroups.
namespace {
template <bool H>
hipError_t gemm_nt4_entry(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* C2,
                          const void* U, const void* bias, int M, int N, int K, int grid, hipStream_t s) {
  const int stp = (epi >> 12) & 0x3;
  const int probe = (epi >> 8) & 0xf;
  const int gmsel = (epi >> 16) & 0xff;
  const int ovp = (epi >> 14) & 0x3;  // overlapped epilogue: 0 automatic (K >= Q_OVL_MIN_K), 1 always, 2 never
  epi &= 0xff;
  Nt4Args a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.C2 = (bf16_t*)C2;
  a.U = (const bf16_t*)U;
  a.bias = (const bf16_t*)bias;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  if (nt4_check(a, grid) != hipSuccess) return hipErrorInvalidValue;
  if ((epi == Q_EPI_GELU && (!C2 || (!U && !H) || (uintptr_t)U % 16)) || (epi == Q_EPI_DGELU && (!U || bias)) ||
      (bias && (uintptr_t)bias % 16))
    return hipErrorInvalidValue;
  nt4_geometry(a, gmsel);
  const bool nt = nt4_store_nt(stp, (int64_t)M * N * 2 * (epi == Q_EPI_GELU ? 2 : 1));
  const dim3 gr(grid < a.tiles ? grid : a.tiles);
  switch (epi) {
    case Q_EPI_BF16:
      if (bias) nt4_launch<Q_EPI_BF16, true, H>(a, gr, nt, probe, s);
      else nt4_launch<Q_EPI_BF16, false, H>(a, gr, nt, probe, s,
                                            (ovp == 1 || (ovp == 0 && K >= Q_OVL_MIN_K)) && (!NSA_NT4_OVL2 || K >= 2 * Q_BK));
      break;
    case Q_EPI_GELU:
      if (bias) nt4_launch<Q_EPI_GELU, true, H>(a, gr, nt, probe, s);
      else nt4_launch<Q_EPI_GELU, false, H>(a, gr, nt, probe, s);
      break;
    case Q_EPI_DGELU: nt4_launch<Q_EPI_DGELU, false, H>(a, gr, nt, probe, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
}  // namespace

NSA_API hipError_t nsa_gemm_nt4(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* C2,
                                const void* U, const void* bias, int M, int N, int K, int grid, hipStream_t s) {
  return gemm_nt4_entry<false>(epi, A, lda, B, ldb, C, ldc, C2, U, bias, M, N, K, grid, s);
}
// fp16 operands and outputs (gelu'(u) stays fp16; the GELU epilogue computes instead of
// looking up, U may be null there)
NSA_API hipError_t nsa_gemm_nt4_h(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* C2,
                                  const void* U, const void* bias, int M, int N, int K, int grid, hipStream_t s) {
  return gemm_nt4_entry<true>(epi, A, lda, B, ldb, C, ldc, C2, U, bias, M, N, K, grid, s);
}

// Fused cross-entropy, forward: E = exp(A · B^T - c[row]) (bf16, [M, N] at ldc; columns >=
// nvalid give 0) and part[2 (column tile) + (column half)][row] = the fp32 row sums of E over
// that half tile (2 * ceil(N / 256) slots of M floats).  c = the target logit of the row
// (computed before this GEMM), so sum_j E = exp(loss_row) >= ~1: no overflow short of a
// per-token loss of ~80 nats (nsa_xent_combine flags such rows for an exact recompute).
namespace {
template <bool H>
hipError_t nt4_xent_entry(const void* A, int lda, const void* B, int ldb, void* E, int ldc, const void* crow,
                          void* part, int M, int N, int nvalid, int K, int grid, hipStream_t s) {
  Nt4Args a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)E;
  a.rowf = (const float*)crow;
  a.part = (float*)part;
  a.nvalid = nvalid;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  if (nt4_check(a, grid) != hipSuccess || nvalid < 1 || nvalid > N || M % 4 || !crow || !part)
    return hipErrorInvalidValue;
  nt4_geometry(a, 0);
  const dim3 gr(grid < a.tiles ? grid : a.tiles);
  int probe = 0;
#ifdef NSA_PROBES
  // timing probes of the XENT GEMM (probe builds only; see gemm_nt4_kernel): 4 no epilogue,
  // 5 epilogue arithmetic without its stores
  if (const char* e = getenv("NSA_PROBE_XENT")) probe = atoi(e);
#endif
  nt4_launch<Q_EPI_XENT, false, H>(a, gr, nt4_store_nt(0, (int64_t)M * N * 2), probe, s);
  return hipGetLastError();
}
}  // namespace
NSA_API hipError_t nsa_gemm_nt4_xent(const void* A, int lda, const void* B, int ldb, void* E, int ldc,
                                     const void* crow, void* part, int M, int N, int nvalid, int K, int grid,
                                     hipStream_t s) {
  return nt4_xent_entry<false>(A, lda, B, ldb, E, ldc, crow, part, M, N, nvalid, K, grid, s);
}
// fp16 operands and E = exp(logit - target logit) in fp16: entries far below the target sit in
// fp16's subnormal range (absolute precision 2^-24, as autocast's fp16 dlogits), and a row
// whose largest logit passes its target's by more than ~11 nats (an E entry above 65504)
// returns an inf row sum, which nsa_xent_combine sends to the exact fix-up.
NSA_API hipError_t nsa_gemm_nt4_xent_h(const void* A, int lda, const void* B, int ldb, void* E, int ldc,
                                       const void* crow, void* part, int M, int N, int nvalid, int K, int grid,
                                       hipStream_t s) {
  return nt4_xent_entry<true>(A, lda, B, ldb, E, ldc, crow, part, M, N, nvalid, K, grid, s);
}

// Fused cross-entropy, input gradient: C = cs[row] * (A · B^T) - cw[row] * U with A = E [M, K]
// (the forward's exp), B = W^T [N, K] (K = the padded vocabulary), U [M, N] (ld ldc) = the
// rows W[target] gathered by nsa_xent_bwd_prep, and rowc [M][2] = {cs, cw} = {g / S, g} (0, 0
// for an ignored row): g (softmax - onehot) · W with the subtraction in fp32.
namespace {
template <bool H>
hipError_t nt4_xdx_entry(const void* A, int lda, const void* B, int ldb, void* C, int ldc, const void* U,
                         const void* rowc, int M, int N, int K, int grid, hipStream_t s) {
  Nt4Args a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.U = (const bf16_t*)U;
  a.rowf = (const float*)rowc;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  if (nt4_check(a, grid) != hipSuccess || M % 4 || !U || !rowc) return hipErrorInvalidValue;
  nt4_geometry(a, 0);
  const dim3 gr(grid < a.tiles ? grid : a.tiles);
  nt4_launch<Q_EPI_XDX, false, H>(a, gr, nt4_store_nt(0, (int64_t)M * N * 2), 0, s);
  return hipGetLastError();
}
}  // namespace
NSA_API hipError_t nsa_gemm_nt4_xdx(const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                                    const void* U, const void* rowc, int M, int N, int K, int grid, hipStream_t s) {
  return nt4_xdx_entry<false>(A, lda, B, ldb, C, ldc, U, rowc, M, N, K, grid, s);
}
NSA_API hipError_t nsa_gemm_nt4_xdx_h(const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                                      const void* U, const void* rowc, int M, int N, int K, int grid, hipStream_t s) {
  return nt4_xdx_entry<true>(A, lda, B, ldb, C, ldc, U, rowc, M, N, K, grid, s);
}
