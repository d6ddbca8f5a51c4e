// Persistent bf16 "NT" GEMM for gfx950 — the forward and input-gradient GEMMs of
// GPT training, with the MLP activation fused in the epilogue:
//
//   C[M,N] = A[M,K] · B[N,K]^T        (both operands K-contiguous, fp32 accumulate)
//     forward     Y  = X · W^T          A = X  [M][K],  B = W   [N][K]  (nn.Linear weight)
//     input grad  dX = dY · W           A = dY [M][N],  B = W^T [K][N]  (cached transpose)
//   epilogues: bf16 store | u + gelu(u) (c_fc forward) | acc * gelu'(U) (mlp.c_proj dX)
//
// Design (cdna_hip_programming.md §5 "256² 8-phase template", re-derived here):
//  * 256x256 output tile per workgroup, 8 waves as 2 (M) x 4 (N), each wave 128x64 =
//    8x4 accumulators of v_mfma_f32_16x16x32_bf16 (swapped operands: a lane holds 4
//    consecutive output columns of one row);
//  * one 64-deep K-tile (A image [256][64] + B image [256][64], 64 KiB, two buffers) is
//    consumed in 4 PHASES of 16 MFMAs, one 64x32 quadrant (qm, qn) per phase in the
//    order (0,0) (0,1) (1,1) (1,0): fragments are read at the head of the phase that
//    first needs them (p0: A[qm0], p1: B[qn1], p2: A[qm1]), and phase 3 reads the NEXT
//    K-tile's B[qn0] (8 / 4 / 8 / 4 fragment reads per phase);
//  * staging is LDS-DMA only (global_load_lds_dwordx4, no VGPR round trip): each
//    K-tile is 4 half-tiles of 16 KiB (A rows of quadrant 0 / 1, B columns of quadrant
//    0 / 1), two 1-KiB pieces per wave each, one half-tile per phase, issued in the order
//    B0 A0 B1 A1 5-6 phases ahead of its first read.  Every per-lane source offset is computed ONCE per kernel
//    (the XOR swizzle lives in the source address, rule 21); per K-tile only two SGPR
//    base pointers advance, and both pieces of a wave share one M0 write, so a DMA costs
//    no VALU work.  Each phase retires what is four half-tiles old with `s_waitcnt
//    vmcnt(8)` (never 0 in the loop) and a buffer is read one phase after that wait
//    (RAW); a half-tile region is refilled >= 2 phases after its last read (WAR);
//  * the two wave groups (wm = 0 / 1, one wave of each on every SIMD) run one raw
//    s_barrier apart, so each phase is [LDS reads + DMA | barrier | 16 MFMA | barrier]
//    and one group's reads run beside the other group's MFMAs on every SIMD;
//  * persistent: grid = #CUs, tiles walked in an XCD-grouped order; the DMA stream runs
//    straight on into the next tile (its first 6 half-tiles are in flight during this
//    tile's last K-tile);
//  * epilogue through a wave-private LDS slice into whole-row 16-byte stores (see
//    store_tile_lds), nontemporal for outputs larger than the Infinity Cache;
//  * ragged edges without per-lane masks: a tail tile is shifted back inside the
//    matrix (m0 = min(m0, M - 256)) and only its not-yet-covered rows / columns are
//    stored, so M, N >= 256 and K % 64 == 0 are the only shape rules.
//
// Measured on MI355X (scripts/gemm_nt_ab.py, M = 122880, uniform random operands,
// interleaved with hipBLASLt in one process; docs/performance.md has the table): the
// epilogue decides the K = 768 shapes — the accumulator-order stores (16 rows x 64 B per
// instruction) cost ~30 % of those GEMMs, whole-row stores through LDS and nontemporal
// stores most of it back; the main loop runs ~73 % MFMA-busy (PMC) at K = 50304.
#include "common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHR = 512;
constexpr int IMG = BM * BK * 2;          // 32 KiB: one operand's K-tile image [256][64] bf16, 128-B rows
constexpr int BUF = 2 * IMG;              // A image then B image
constexpr int EPI_LDS = 2 * BUF;          // epilogue staging: 4 KiB per wave after the two buffers
constexpr int SMEM = 2 * BUF + 8 * 4096;  // 160 KiB
static_assert(SMEM <= 163840, "LDS budget");
#ifndef NSA_NT_DEF
#define NSA_NT_DEF 4  // epilogue rounds (of 4) deferred into the next tile's first K-tile
#endif
#ifndef NSA_NT_VMW
#define NSA_NT_VMW 8  // steady-state DMA wait: vmcnt(VMW) keeps VMW / 2 half-tiles in flight (A/B probe)
#endif
#ifndef NSA_NT_RPP
#define NSA_NT_RPP 4  // deferred rounds stored per phase
#endif

enum { EPI_BF16 = 0, EPI_GELU = 1, EPI_DGELU = 2 };

struct NtArgs {
  const bf16_t* A;
  const bf16_t* B;
  bf16_t* C;         // [M][ldc]
  bf16_t* C2;        // EPI_GELU: gelu(C)
  const bf16_t* U;   // EPI_DGELU: pre-activation, [M][ldc]
  int M, N, K;
  int lda, ldb, ldc;
  int tiles_m, tiles_n, tiles;
  int gm;  // grouped tile order: row-blocks per group
};

// LDS-DMA of a wave's two 1-KiB pieces of a half-tile: lane l's 16 bytes from sbase + voff
// land at lds + 16 l.  Piece 1 lands 1 KiB after piece 0 in LDS, and the instruction offset
// (applied to the LDS destination AND the global address) provides that 1 KiB, so its
// per-lane source offset carries -1024.  One M0 write for both.  M0 is not preserved:
// nothing else in this kernel uses it (checked in the .s).
__device__ __forceinline__ void dma16x2(const char* sbase, uint32_t voff0, uint32_t voff1m, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %3\n\tglobal_load_lds_dwordx4 %1, %3 offset:1024"
               :
               : "v"(voff0), "v"(voff1m), "s"(lds), "s"(sbase)
               : "memory");
}

template <int N>
__device__ __forceinline__ void vm_wait_imm() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ bf16x8 rd16(const char* p) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
}

// tile sequence number -> (row, col) origin, grouped g.gm row-blocks x all columns; tail
// tiles are shifted back inside the matrix (lo = first row / column this tile owns)
__device__ __forceinline__ void tile_coords(const NtArgs& g, int seq, int& m0, int& n0, int& mlo, int& nlo) {
  const int per = g.gm * g.tiles_n;
  const int grp = seq / per;
  const int first = grp * g.gm;
  const int gm = min(g.gm, g.tiles_m - first);
  const int in = seq - grp * per;
  mlo = (first + in % gm) * BM;
  nlo = (in / gm) * BN;
  m0 = min(mlo, g.M - BM);
  n0 = min(nlo, g.N - BN);
}

// DMA cursor: the K-tile a phase's half-tile belongs to (scalar state)
struct Cur {
  const char* a;  // A + m0 * lda + k * 64 (bytes)
  const char* b;
  uint32_t buf;   // LDS buffer byte offset of this K-tile (global K-tile parity)
  int k, seq;
  bool valid;
};

__device__ __forceinline__ void cur_set_tile(const NtArgs& g, Cur& c, int seq) {
  c.seq = seq;
  c.k = 0;
  c.valid = seq < g.tiles;
  if (c.valid) {
    int m0, n0, mlo, nlo;
    tile_coords(g, seq, m0, n0, mlo, nlo);
    c.a = reinterpret_cast<const char*>(g.A + (int64_t)m0 * g.lda);
    c.b = reinterpret_cast<const char*>(g.B + (int64_t)n0 * g.ldb);
  }
}

__device__ __forceinline__ void cur_next(const NtArgs& g, Cur& c, int nk, int G) {
  c.buf ^= (uint32_t)BUF;
  if (!c.valid) return;
  if (++c.k == nk) {
    cur_set_tile(g, c, c.seq + G);
  } else {
    c.a += 2 * BK;
    c.b += 2 * BK;
  }
}

typedef uint32_t nt_u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ void st16(bf16_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  if constexpr (NT) {
    __builtin_nontemporal_store(nt_u32x4{a, b, c, d}, reinterpret_cast<nt_u32x4*>(p));
  } else {
    *reinterpret_cast<uint4*>(p) = make_uint4(a, b, c, d);
  }
}

// Epilogue through a wave-private 4-KiB LDS slice (the 32 KiB after the two K-tile buffers,
// which no DMA touches, so it needs no barrier against the next tile's staging).  In the
// accumulator layout consecutive lanes hold different rows, so a store straight from the
// registers writes 16 rows x 64 B per instruction with no two adjacent lanes contiguous;
// re-shaped through LDS, each store instruction writes 8 whole 128-byte row segments (lane
// l: row l / 8, 16-byte chunk l % 8).  Four rounds of 32 rows x 64 columns per wave.  Image:
// row r at 128 r, 16-byte chunk c at (c ^ (r & 7)) * 16 (writes 2-way, reads conflict-free).
// EPI_DGELU: the U pieces of two rounds are in flight at a time (the first two before the
// first round), so their latency runs under the LDS re-shaping and the other round's stores.
template <int EPI, bool NT>
__device__ __forceinline__ void store_tile_lds(const NtArgs& g, const f32x4 (&acc)[8][4], char* stage, int m0, int n0,
                                               int mlo, int nlo, int wm, int wn, int lane) {
  const bool full = (m0 == mlo) & (n0 == nlo);
  const int r = lane & 15, q = lane >> 4;
  const int rr = lane >> 3, cc = lane & 7;  // read / store lane map
  const int col = n0 + wn * 64 + 8 * cc;
  nt_u32x4 uv[2][4];  // U of rounds rd and rd + 1 (two rounds in flight)
  auto load_u = [&](int rd, nt_u32x4 (&dst)[4]) {
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int grow = m0 + wm * 128 + 32 * rd + 8 * s2 + rr;  // in bounds: tiles lie inside the matrix
      dst[s2] = __builtin_nontemporal_load(reinterpret_cast<const nt_u32x4*>(g.U + (int64_t)grow * g.ldc + col));
    }
  };
  if constexpr (EPI == EPI_DGELU) {
    load_u(0, uv[0]);
    load_u(1, uv[1]);
  }
#pragma unroll
  for (int rd = 0; rd < 4; ++rd) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
      const int row = 16 * i2 + r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 t = acc[2 * rd + i2][j];
        const int chunk = (2 * j + (q >> 1)) ^ (row & 7);
        *reinterpret_cast<uint2*>(stage + row * 128 + chunk * 16 + (q & 1) * 8) =
            make_uint2(pack2(t[0], t[1]), pack2(t[2], t[3]));
      }
    }
    uint4 v[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int row = 8 * s2 + rr;
      v[s2] = *reinterpret_cast<const uint4*>(stage + row * 128 + ((cc ^ (row & 7)) << 4));
    }
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int grow = m0 + wm * 128 + 32 * rd + 8 * s2 + rr;
      if (!full && (grow < mlo || col < nlo)) continue;
      const int64_t off = (int64_t)grow * g.ldc + col;
      uint32_t w[4] = {v[s2].x, v[s2].y, v[s2].z, v[s2].w};
      if constexpr (EPI == EPI_DGELU) {
        const nt_u32x4 ur = uv[rd & 1][s2];
        const uint32_t uu[4] = {ur[0], ur[1], ur[2], ur[3]};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a0 = __uint_as_float(w[e] << 16) * nsa_gelu_grad(__uint_as_float(uu[e] << 16));
          const float a1 = __uint_as_float(w[e] & 0xffff0000u) * nsa_gelu_grad(__uint_as_float(uu[e] & 0xffff0000u));
          w[e] = pack2(a0, a1);
        }
      }
      st16<NT>(g.C + off, w[0], w[1], w[2], w[3]);
      if constexpr (EPI == EPI_GELU) {
        // gelu of the bf16-rounded pre-activation: what a separate GELU kernel would see
        uint32_t gg[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          gg[e] = pack2(nsa_gelu(__uint_as_float(w[e] << 16)), nsa_gelu(__uint_as_float(w[e] & 0xffff0000u)));
        st16<NT>(g.C2 + off, gg[0], gg[1], gg[2], gg[3]);
      }
    }
    if constexpr (EPI == EPI_DGELU) {
      if (rd + 2 < 4) load_u(rd + 2, uv[rd & 1]);
    }
  }
}

// One round of a wave's output rows (32 rows x 64 columns): 4 (EPI_GELU: 8) stores.
template <int EPI, bool NT>
__device__ __forceinline__ void issue_round(const NtArgs& g, const uint4 (&v)[4], int m0, int n0, int wm, int wn,
                                            int lane, int rd) {
  const int rr = lane >> 3, cc = lane & 7;
  const int col = n0 + wn * 64 + 8 * cc;
#pragma unroll
  for (int s2 = 0; s2 < 4; ++s2) {
    const int grow = m0 + wm * 128 + 32 * rd + 8 * s2 + rr;
    const int64_t off = (int64_t)grow * g.ldc + col;
    st16<NT>(g.C + off, v[s2].x, v[s2].y, v[s2].z, v[s2].w);
    if constexpr (EPI == EPI_GELU) {
      const uint32_t w[4] = {v[s2].x, v[s2].y, v[s2].z, v[s2].w};
      uint32_t gg[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        gg[e] = pack2(nsa_gelu(__uint_as_float(w[e] << 16)), nsa_gelu(__uint_as_float(w[e] & 0xffff0000u)));
      st16<NT>(g.C2 + off, gg[0], gg[1], gg[2], gg[3]);
    }
  }
}

// Deferred epilogue: the same LDS re-shaping as store_tile_lds (and the GELU' product) for
// a full tile, but the last DEF rounds' whole-row pieces stay in registers (16 VGPRs per
// round) and go out in phase 0 of the next tile's first K-tile (issue_round), under that
// tile's MFMAs.
template <int EPI, bool NT, int DEF>
__device__ __forceinline__ void stage_tile(const NtArgs& g, const f32x4 (&acc)[8][4], char* stage, int m0, int n0,
                                           int wm, int wn, int lane, uint4 (&pst)[DEF][4]) {
  const int r = lane & 15, q = lane >> 4;
  const int rr = lane >> 3, cc = lane & 7;
  const int col = n0 + wn * 64 + 8 * cc;
  nt_u32x4 uv[2][4];
  auto load_u = [&](int rd, nt_u32x4 (&dst)[4]) {
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int grow = m0 + wm * 128 + 32 * rd + 8 * s2 + rr;
      dst[s2] = __builtin_nontemporal_load(reinterpret_cast<const nt_u32x4*>(g.U + (int64_t)grow * g.ldc + col));
    }
  };
  if constexpr (EPI == EPI_DGELU) {
    load_u(0, uv[0]);
    load_u(1, uv[1]);
  }
#pragma unroll
  for (int rd = 0; rd < 4; ++rd) {
#pragma unroll
    for (int i2 = 0; i2 < 2; ++i2) {
      const int row = 16 * i2 + r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 t = acc[2 * rd + i2][j];
        const int chunk = (2 * j + (q >> 1)) ^ (row & 7);
        *reinterpret_cast<uint2*>(stage + row * 128 + chunk * 16 + (q & 1) * 8) =
            make_uint2(pack2(t[0], t[1]), pack2(t[2], t[3]));
      }
    }
    uint4 v[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      const int row = 8 * s2 + rr;
      v[s2] = *reinterpret_cast<const uint4*>(stage + row * 128 + ((cc ^ (row & 7)) << 4));
    }
    if constexpr (EPI == EPI_DGELU) {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const nt_u32x4 ur = uv[rd & 1][s2];
        uint32_t w[4] = {v[s2].x, v[s2].y, v[s2].z, v[s2].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a0 = __uint_as_float(w[e] << 16) * nsa_gelu_grad(__uint_as_float(ur[e] << 16));
          const float a1 = __uint_as_float(w[e] & 0xffff0000u) * nsa_gelu_grad(__uint_as_float(ur[e] & 0xffff0000u));
          w[e] = pack2(a0, a1);
        }
        v[s2] = make_uint4(w[0], w[1], w[2], w[3]);
      }
      if (rd + 2 < 4) load_u(rd + 2, uv[rd & 1]);
    }
    if (rd < 4 - DEF) {
      issue_round<EPI, NT>(g, v, m0, n0, wm, wn, lane, rd);
    } else {
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) pst[rd - (4 - DEF)][s2] = v[s2];
    }
  }
}

}  // namespace

// NT: nontemporal epilogue stores.  PROBE: 1 = no DMA after the prologue (stale LDS, wrong
// results), 2 = synchronous epilogue (no deferred stores; A/B, correct), 4 = no epilogue
// stores (wrong).
template <int EPI, bool NT, int PROBE, bool BAL>
__global__ __launch_bounds__(NTHR, 2) void gemm_nt_kernel(NtArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x;
  const int nk = g.K / BK;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  // XCD-aware virtual block id: blocks b, b+8, ... share an XCD and get consecutive ids
  int v = blockIdx.x;
  {
    const int x = v % 8, q = G / 8, r = G % 8;
    v = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + v / 8;
  }
  if (v >= g.tiles) return;

  // ---- per-lane DMA source offsets (bytes from the K-tile's row base), fixed for the kernel.
  // Half h of A = rows {r : (r >> 6) & 1 == h}; piece pc = 2 wave + j covers 8 rows.
  // Half h of B = columns {c : (c >> 5) & 1 == h}.  Image row r, physical 16-B chunk p
  // holds logical chunk p ^ ((r >> 1) & 7).
  uint32_t voA[2], voB[2], voA1m[2], voB1m[2];  // [half]: piece 0, piece 1 - 1024
  uint32_t ldA[2], ldB[2];                      // [half]: LDS address of piece 0
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = 2 * wave + j;
      const int rbA = (pc >> 3) * 128 + h * 64 + (pc & 7) * 8;
      const int rbB = (pc >> 2) * 64 + h * 32 + (pc & 3) * 8;
      const int ra = rbA + (lane >> 3), rb = rbB + (lane >> 3);
      const uint32_t oa = (uint32_t)(ra * g.lda * 2 + (((lane & 7) ^ ((ra >> 1) & 7)) << 4));
      const uint32_t ob = (uint32_t)(rb * g.ldb * 2 + (((lane & 7) ^ ((rb >> 1) & 7)) << 4));
      if (j == 0) {
        voA[h] = oa;
        voB[h] = ob;
        ldA[h] = lds0 + (uint32_t)(rbA * 128);
        ldB[h] = lds0 + (uint32_t)(IMG + rbB * 128);
      } else {  // rows 8 apart in the image = 1 KiB after piece 0 in LDS (dma16x2)
        voA1m[h] = oa - 1024u;
        voB1m[h] = ob - 1024u;
      }
    }
  }

  // ---- fragment read offsets: row wm*128 + 16 i + (lane & 15) (A) / wn*64 + ... (B),
  // logical chunk 4 kk + (lane >> 4)
  const int sw = (lane >> 1) & 7;
  int offA[2], offB[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int ch = ((4 * kk + (lane >> 4)) ^ sw) << 4;
    offA[kk] = (wm * 128 + (lane & 15)) * 128 + ch;
    offB[kk] = IMG + (wn * 64 + (lane & 15)) * 128 + ch;
  }

  // half-tile kinds: 0 = A half 0, 1 = B half 0, 2 = B half 1, 3 = A half 1
  auto issue_half = [&](const Cur& c, int kind) {
    if (kind == 0 || kind == 3) {
      const int h = kind == 3;
      dma16x2(c.a, voA[h], voA1m[h], ldA[h] + c.buf);
    } else {
      const int h = kind == 2;
      dma16x2(c.b, voB[h], voB1m[h], ldB[h] + c.buf);
    }
  };

  // ---- DMA stream: c1 = the K-tile after the one being multiplied, c2 = the one after that.
  // Prologue: K-tile 0 (all four half-tiles) and K-tile 1's A0 / B0.
  Cur c1, c2;
  c1.buf = 0;
  cur_set_tile(g, c1, v);
  // stream order per K-tile: B0, A0, B1, A1 (BAL) / A0, B0, B1, A1
  issue_half(c1, BAL ? 1 : 0);
  issue_half(c1, BAL ? 0 : 1);
  issue_half(c1, 2);
  issue_half(c1, 3);
  c2 = c1;
  cur_next(g, c2, nk, G);
  if (c2.valid) {
    issue_half(c2, BAL ? 1 : 0);
    issue_half(c2, BAL ? 0 : 1);
    vm_wait_imm<NSA_NT_VMW>();
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  uint32_t bufc = 0;  // the multiplied K-tile's buffer
  c1 = c2;
  cur_next(g, c2, nk, G);
  raw_barrier();
  if (wm == 1) raw_barrier();  // stagger: group 1 runs one barrier behind group 0

  int seq = v;
  // pend: the previous tile stored its first 4 - DEF rounds at its end and staged the last
  // DEF in pst; they go out RPP per phase at the head of this tile's first K-tile, after
  // the phase's DMA (registers: the accumulators of the later quadrants are not live yet
  // there).  vmcnt is in order, so a wait counts every store issued after the half-tile it
  // retires (SR stores per round): in K-tile 0 the 4 - DEF stored at the tile end plus the
  // deferred ones issued so far, in K-tile 1 the deferred ones issued from phase P on.
  constexpr int SR = EPI == EPI_GELU ? 8 : 4;
  constexpr int DEF = NSA_NT_DEF, RPP = NSA_NT_RPP;
  static_assert(DEF >= 1 && DEF <= 4 && RPP >= 1 && 8 + 4 * SR < 64, "deferred-store accounting");
  bool pend = false;
  int pm0 = 0, pn0 = 0;
  uint4 pst[DEF][4];
  f32x4 acc[8][4];
  bf16x8 af[4][2], b0f[2][2], b1f[2][2], b0n[2][2];
  // B0 of K-tile 0 (retired with A0 by the prologue's wait); afterwards each K-tile's
  // phase 3 reads the NEXT K-tile's B0, so the read load per phase is 8 / 4 / 8 / 4
  // fragments instead of 12 / 4 / 8 / 0
  if constexpr (BAL) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) b0f[j][kk] = rd16(smem + offB[kk] + (16 * j) * 128);
  }

// one phase: P = 0..3, FIRST = first K-tile of an output tile (kk = 0 MFMAs start from 0),
// KT = 1 / 2 / 0: the tile's first / second / any later K-tile (deferred-store accounting).
// [LDS reads | DMA of half-tile P+6 + counted wait retiring what phase P+1 reads | barrier |
//  16 MFMAs | barrier]
#define NT_PHASE(P, FIRST, KT)                                                                    \
  {                                                                                            \
    const char* base_ = smem + bufc;                                                           \
    if (P == 0 || P == 2) {                                                                    \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        af[i][kk] = rd16(base_ + offA[kk] + ((P >> 1) * 64 + 16 * i) * 128);                   \
    }                                                                                          \
    if (!BAL && P == 0) {                                                                      \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        b0f[j][kk] = rd16(base_ + offB[kk] + (16 * j) * 128);                                  \
    }                                                                                          \
    if (BAL && P == 3) { /* the next K-tile's B0 (other buffer): b0n -> b0f after the MFMAs */ \
      const char* nb_ = smem + (bufc ^ (uint32_t)BUF);                                         \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        b0n[j][kk] = rd16(nb_ + offB[kk] + (16 * j) * 128);                                    \
    }                                                                                          \
    if (P == 1) {                                                                              \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        b1f[j][kk] = rd16(base_ + offB[kk] + (32 + 16 * j) * 128);                             \
    }                                                                                          \
    {                                                                                          \
      const Cur& cc_ = (P < 2) ? c1 : c2;                                                      \
      if (cc_.valid && PROBE != 1)                                                             \
        issue_half(cc_, P == 0 ? 2 : P == 1 ? 3 : P == 2 ? (BAL ? 1 : 0) : (BAL ? 0 : 1));       \
      if (KT == 1 && RPP * P < DEF && pend) {                                                  \
        _Pragma("unroll") for (int d_ = RPP * P; d_ < DEF && d_ < RPP * (P + 1); ++d_)          \
          issue_round<EPI, NT>(g, pst[d_], pm0, pn0, wm, wn, lane, 4 - DEF + d_);              \
      }                                                                                        \
      if (cc_.valid) {                                                                         \
        if ((KT == 1 || (KT == 2 && RPP * P < DEF)) && pend) {                                 \
          vm_wait_imm<NSA_NT_VMW + (KT == 1 ? (4 - DEF) * SR + SR * (DEF < RPP * (P + 1) ? DEF : RPP * (P + 1)) \
                                   : SR * (DEF > RPP * P ? DEF - RPP * P : 0))>();              \
        } else {                                                                               \
          vm_wait_imm<NSA_NT_VMW>();                                                          \
        }                                                                                      \
      } else {                                                                                 \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                      \
      }                                                                                        \
    }                                                                                          \
    raw_barrier();                                                                             \
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
    if (BAL && P == 3) {                                                                       \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk) b0f[j][kk] = b0n[j][kk];                \
    }                                                                                          \
    raw_barrier();                                                                             \
  }
#define NT_KTILE(FIRST, KT)          \
  {                                  \
    constexpr int KT_ = KT;          \
    NT_PHASE(0, FIRST, KT_)          \
    NT_PHASE(1, FIRST, KT_)          \
    NT_PHASE(2, FIRST, KT_)          \
    NT_PHASE(3, FIRST, KT_)          \
    bufc ^= (uint32_t)BUF;           \
    c1 = c2;                         \
    cur_next(g, c2, nk, G);          \
  }

  while (true) {
    NT_KTILE(true, 1)
    if (nk > 1) {
      NT_KTILE(false, 2)
      pend = false;
      for (int t = 2; t < nk; ++t) NT_KTILE(false, 0)
    }
    int m0, n0, mlo, nlo;
    tile_coords(g, seq, m0, n0, mlo, nlo);
    if constexpr (PROBE != 4) {
      // defer when another tile follows and spans >= 2 K-tiles, and no store is masked
      // off (the wait counts above assume every store of a round is issued)
      if (PROBE != 1 && PROBE != 2 && nk > 1 && seq + G < g.tiles && (m0 == mlo) & (n0 == nlo)) {
        stage_tile<EPI, NT, DEF>(g, acc, smem + EPI_LDS + wave * 4096, m0, n0, wm, wn, lane, pst);
        pend = true;
        pm0 = m0;
        pn0 = n0;
      } else {
        store_tile_lds<EPI, NT>(g, acc, smem + EPI_LDS + wave * 4096, m0, n0, mlo, nlo, wm, wn, lane);
        // redefine pst on this path too: otherwise the previous tile's staged values flow
        // round the loop here and stay allocated through every K-tile (spills)
#pragma unroll
        for (int d = 0; d < DEF; ++d)
#pragma unroll
          for (int s2 = 0; s2 < 4; ++s2) pst[d][s2] = make_uint4(0, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    }
    seq += G;
    if (seq >= g.tiles) break;
  }
#undef NT_KTILE
#undef NT_PHASE
  if (wm == 0) raw_barrier();  // close the stagger: both groups end at the same barrier count
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// epi: 0 = bf16 store, 1 = u + gelu(u) into C / C2, 2 = acc * gelu'(U).
// bits 8-11: probe (1 no DMA, 4 no stores: timing only; 2 no post-epilogue window).  bits 12-13: epilogue
// store policy (0 = nontemporal when the output exceeds the 256 MiB Infinity Cache,
// 1 = always, 2 = never); bit 14: phase-3 B0 prefetch off (A/B); bits 16-23: row-blocks
// per tile group (0 = automatic).  grid = persistent workgroup count (#CUs).
NSA_API hipError_t nsa_gemm_nt(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* C2,
                               const void* U, int M, int N, int K, int grid, hipStream_t s) {
  const int epi_full = epi;
  const int probe = (epi >> 8) & 0xf;
  const int stp = (epi >> 12) & 0x3;
  const bool bal = !((epi >> 14) & 1);
  epi &= 0xff;
  if (M < BM || N < BN || K < BK || K % BK != 0 || lda % 8 || ldb % 8 || ldc % 8 || lda < K || ldb < K ||
      ldc < N || grid < 1)
    return hipErrorInvalidValue;
  if ((int64_t)BM * lda * 2 >= (1ll << 31) || (int64_t)BN * ldb * 2 >= (1ll << 31)) return hipErrorInvalidValue;
  if ((epi == EPI_GELU && !C2) || (epi == EPI_DGELU && !U)) return hipErrorInvalidValue;
  NtArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (bf16_t*)C;
  a.C2 = (bf16_t*)C2;
  a.U = (const bf16_t*)U;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.tiles_m = (M + BM - 1) / BM;
  a.tiles_n = (N + BN - 1) / BN;
  a.tiles = a.tiles_m * a.tiles_n;
  // Tile order.  The 32 workgroups of an XCD take 32 consecutive tiles.  Narrow outputs
  // (<= 16 column tiles: every GPT-2 linear but the lm_head) go row-major, so a row panel of
  // A — streamed from HBM when K is large — is read by all its column tiles on one XCD at
  // the same time; wide outputs (the lm_head's 197 column tiles) in groups of 8 row-blocks.
  const int gmsel = (epi_full >> 16) & 0xff;
  a.gm = gmsel ? gmsel : (a.tiles_n <= 16 ? 1 : 8);
  const int64_t out_bytes = (int64_t)M * N * 2 * (epi == EPI_GELU ? 2 : 1);
  const bool nt = stp == 1 || (stp == 0 && out_bytes >= NSA_NT_MIN_BYTES);
  const dim3 gr(grid < a.tiles ? grid : a.tiles);
#define NT_LAUNCH(E)                                                          \
  if (probe == 1) gemm_nt_kernel<E, true, 1, true><<<gr, NTHR, 0, s>>>(a);    \
  else if (probe == 2) gemm_nt_kernel<E, true, 2, true><<<gr, NTHR, 0, s>>>(a); \
  else if (probe == 4) gemm_nt_kernel<E, true, 4, true><<<gr, NTHR, 0, s>>>(a); \
  else if (!bal) gemm_nt_kernel<E, true, 0, false><<<gr, NTHR, 0, s>>>(a);    \
  else if (nt) gemm_nt_kernel<E, true, 0, true><<<gr, NTHR, 0, s>>>(a);       \
  else gemm_nt_kernel<E, false, 0, true><<<gr, NTHR, 0, s>>>(a);
  switch (epi) {
    case EPI_BF16: NT_LAUNCH(EPI_BF16) break;
    case EPI_GELU: NT_LAUNCH(EPI_GELU) break;
    case EPI_DGELU: NT_LAUNCH(EPI_DGELU) break;
    default: return hipErrorInvalidValue;
  }
#undef NT_LAUNCH
  return hipGetLastError();
}
