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
//    8x4 accumulators of v_mfma_f32_16x16x32_bf16 (swapped operands, so a lane holds
//    4 consecutive output columns of one row: 8-byte stores straight from registers);
//  * one 64-deep K-tile (A image [256][64] + B image [256][64], 64 KiB, two buffers) is
//    consumed in 4 PHASES of 16 MFMAs, one 64x32 quadrant (qm, qn) per phase in the
//    order (0,0) (0,1) (1,1) (1,0): fragments are read at the head of the phase that
//    first needs them (p0: A[qm0] + B[qn0], p1: B[qn1], p2: A[qm1], p3: none);
//  * staging is LDS-DMA only (global_load_lds_dwordx4, no VGPR round trip): each
//    K-tile is 4 half-tiles of 16 KiB (A rows of quadrant 0 / 1, B columns of quadrant
//    0 / 1), two 1-KiB pieces per wave each, one half-tile per phase, issued 6 phases
//    ahead of its first read.  Every per-lane source offset is computed ONCE per kernel
//    (the XOR swizzle lives in the source address, rule 21); per K-tile only two SGPR
//    base pointers advance, so a DMA costs no VALU work.  Each phase retires what is
//    four half-tiles old with `s_waitcnt vmcnt(8)` (never 0 in the loop) and a buffer is
//    read one phase after that wait (RAW); a half-tile region is refilled >= 2 phases
//    after its last read (WAR);
//  * the two wave groups (wm = 0 / 1, one wave of each on every SIMD) run one raw
//    s_barrier apart, so each phase is [LDS reads + DMA | barrier | 16 MFMA | barrier]
//    and one group's reads run beside the other group's MFMAs on every SIMD;
//  * persistent: grid = #CUs, tiles walked in an XCD-grouped order; the DMA stream runs
//    straight on into the next tile (its first 6 half-tiles are in flight during this
//    tile's last K-tile), and the epilogue's stores drain under the next tile's MFMAs;
//  * ragged edges without per-lane masks: a tail tile is shifted back inside the
//    matrix (m0 = min(m0, M - 256)) and only its not-yet-covered rows / columns are
//    stored, so M, N >= 256 and K % 64 == 0 are the only shape rules.
#include "common.h"

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int NTHR = 512;
constexpr int IMG = BM * BK * 2;  // 32 KiB: one operand's K-tile image [256][64] bf16, 128-B rows
constexpr int BUF = 2 * IMG;      // A image then B image
constexpr int SMEM = 2 * BUF;     // two K-tile buffers: 128 KiB
constexpr int GM = 8;             // grouped tile order: row-blocks per group

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
};

// LDS-DMA of one 1-KiB piece: lane l's 16 bytes from sbase + voff land at lds + 16 l
__device__ __forceinline__ void dma16(const char* sbase, uint32_t voff, uint32_t lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

// Both 1-KiB pieces of a wave's half-tile share one M0 write: piece 1 lands 1 KiB after
// piece 0 in LDS, and the instruction offset (applied to the LDS destination AND the
// global address) provides that 1 KiB, so its per-lane source offset carries -1024.
// M0 is not preserved: nothing else in these kernels uses it (checked in the .s).
__device__ __forceinline__ void dma16x2(const char* sbase, uint32_t voff0, uint32_t voff1m, uint32_t lds) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %3\n\tglobal_load_lds_dwordx4 %1, %3 offset:1024"
               :
               : "v"(voff0), "v"(voff1m), "s"(lds), "s"(sbase)
               : "memory");
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

__device__ __forceinline__ bf16x8 rd16(const char* p) {
  return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p));
}

// tile sequence number -> (row, col) origin, grouped GM row-blocks x all columns; tail
// tiles are shifted back inside the matrix (lo = first row / column this tile owns)
__device__ __forceinline__ void tile_coords(const NtArgs& g, int seq, int& m0, int& n0, int& mlo, int& nlo) {
  const int per = GM * g.tiles_n;
  const int grp = seq / per;
  const int first = grp * GM;
  const int gm = min(GM, g.tiles_m - first);
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

// Store one 64x32 quadrant (qm, qn) of a wave's 128x64 accumulator tile.  Lane
// (r = lane & 15, q = lane >> 4) holds C[16 i + r][16 j + 4 q + e]; v_permlane16_swap on the
// packed accumulator pair (j, j+1) gives every lane 8 consecutive columns (q even: tile j,
// q odd: tile j+1; columns 8 (q >> 1) ..), so a quadrant leaves in 4 dwordx4 stores (64
// contiguous bytes per row) instead of 8 dwordx2 (the store tail is issue-bound,
// cdna_hip_programming.md T21).
template <int EPI, bool LANE_ROWMAJOR = false>
__device__ __forceinline__ void store_quad(const NtArgs& g, const f32x4 (&acc)[8][4], int qm, int qn, int m0, int n0,
                                           int mlo, int nlo, int wm, int wn, int lane) {
  const int q = lane >> 4;
  const bool full = (m0 == mlo) & (n0 == nlo);  // wave-uniform: no row / column masks
  const int col = LANE_ROWMAJOR ? n0 + wn * 64 + 32 * qn + 8 * (lane & 3)
                                : n0 + wn * 64 + 32 * qn + 16 * (q & 1) + 8 * (q >> 1);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = m0 + wm * 128 + 16 * (qm * 4 + i) + (LANE_ROWMAJOR ? (lane >> 2) : (lane & 15));
    const f32x4 t0 = acc[qm * 4 + i][qn * 2], t1 = acc[qm * 4 + i][qn * 2 + 1];
    const auto sl = __builtin_amdgcn_permlane16_swap(pack2(t0[0], t0[1]), pack2(t1[0], t1[1]), false, false);
    const auto sh = __builtin_amdgcn_permlane16_swap(pack2(t0[2], t0[3]), pack2(t1[2], t1[3]), false, false);
    uint32_t w[4] = {sl[0], sh[0], sl[1], sh[1]};
    if (!full && (row < mlo || col < nlo)) continue;
    const int64_t off = (int64_t)row * g.ldc + col;
    if constexpr (EPI == EPI_DGELU) {
      const uint4 u = *reinterpret_cast<const uint4*>(g.U + off);
      const uint32_t uu[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a0 = __uint_as_float(w[e] << 16) * nsa_gelu_grad(__uint_as_float(uu[e] << 16));
        const float a1 = __uint_as_float(w[e] & 0xffff0000u) * nsa_gelu_grad(__uint_as_float(uu[e] & 0xffff0000u));
        w[e] = pack2(a0, a1);
      }
    }
    *reinterpret_cast<uint4*>(g.C + off) = make_uint4(w[0], w[1], w[2], w[3]);
    if constexpr (EPI == EPI_GELU) {
      // gelu of the bf16-rounded pre-activation: what a separate GELU kernel would see
      uint32_t gg[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        gg[e] = pack2(nsa_gelu(__uint_as_float(w[e] << 16)), nsa_gelu(__uint_as_float(w[e] & 0xffff0000u)));
      *reinterpret_cast<uint4*>(g.C2 + off) = make_uint4(gg[0], gg[1], gg[2], gg[3]);
    }
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform n (multiples of 4 up to 60; larger waits for 60)
__device__ __forceinline__ void vm_wait_dyn(int n) {
  if (n >= 60) asm volatile("s_waitcnt vmcnt(60)" ::: "memory");
  else if (n >= 56) asm volatile("s_waitcnt vmcnt(56)" ::: "memory");
  else if (n >= 52) asm volatile("s_waitcnt vmcnt(52)" ::: "memory");
  else if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else if (n >= 44) asm volatile("s_waitcnt vmcnt(44)" ::: "memory");
  else if (n >= 40) asm volatile("s_waitcnt vmcnt(40)" ::: "memory");
  else if (n >= 36) asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
  else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if (n >= 28) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
  else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

// PROBE (timing only, wrong results): 1 = no DMA after the prologue, 2 = no vmcnt waits in
// the loop, 3 = only one of the two pieces per phase, 4 = no epilogue stores (VAR 1), 5 =
// PROBE 1 with VAR 1, 6 / 7 = workgroup start times staggered (VAR 1 / 0), 8 = epilogue
// stores with row-major lane order (data misplaced; coalescing probe).
// VAR 0: the epilogue of tile i is spread over the first K-tile of tile i+1 (quadrant p
// leaves in phase p's LDS-read segment, right before phase p's MFMAs overwrite it), so the
// stores interleave with the MFMAs of the other wave group instead of stalling it in one
// burst; VAR 1: the whole epilogue between the tiles.  (EPI_DGELU always uses VAR 1: its U
// loads would stall a spread epilogue phase by phase.)
template <int EPI, int PROBE, int VAR>
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
  if constexpr (PROBE == 6) {
    // probe: desynchronise the workgroups' tile boundaries (epilogue store bursts)
    for (int d = 0; d < (v & 7); ++d) __builtin_amdgcn_s_sleep(80);
  }

  // ---- per-lane DMA source offsets (bytes from the K-tile's row base), fixed for the kernel.
  // Half h of A = rows {r : (r >> 6) & 1 == h}; piece pc = 2 wave + j covers 8 rows.
  // Half h of B = columns {c : (c >> 5) & 1 == h}.  Image row r, physical 16-B chunk p
  // holds logical chunk p ^ ((r >> 1) & 7).
  constexpr bool NODMA = PROBE == 1;
  uint32_t voA[2][2], voB[2][2];
  uint32_t ldA[2][2], ldB[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pc = 2 * wave + j;
      const int rbA = (pc >> 3) * 128 + h * 64 + (pc & 7) * 8;
      const int rbB = (pc >> 2) * 64 + h * 32 + (pc & 3) * 8;
      const int ra = rbA + (lane >> 3), rb = rbB + (lane >> 3);
      voA[h][j] = (uint32_t)(ra * g.lda * 2 + (((lane & 7) ^ ((ra >> 1) & 7)) << 4));
      voB[h][j] = (uint32_t)(rb * g.ldb * 2 + (((lane & 7) ^ ((rb >> 1) & 7)) << 4));
      ldA[h][j] = lds0 + (uint32_t)(rbA * 128);
      ldB[h][j] = lds0 + (uint32_t)(IMG + rbB * 128);
    }
  // pieces 0 / 1 of a half are rows 8 apart in the image: 1 KiB apart in LDS (dma16x2)
  const uint32_t voA1m[2] = {voA[0][1] - 1024u, voA[1][1] - 1024u};
  const uint32_t voB1m[2] = {voB[0][1] - 1024u, voB[1][1] - 1024u};

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

  // ---- DMA stream: c1 = the K-tile after the one being multiplied, c2 = the one after that
  Cur c1, c2;
  c1.buf = 0;
  cur_set_tile(g, c1, v);
  // kind: 0 = A half 0, 1 = B half 0, 2 = B half 1, 3 = A half 1; piece j = 0 / 1.  NODMA
  // (timing probe): only the prologue stages anything, later K-tiles re-read stale LDS
  auto issue_piece = [&](const Cur& c, int kind, int j, bool prologue) {
    if (!NODMA || prologue) {
      if (kind == 0 || kind == 3) {
        const int h = kind == 3;
        dma16(c.a, voA[h][j], ldA[h][j] + c.buf);
      } else {
        const int h = kind == 2;
        dma16(c.b, voB[h][j], ldB[h][j] + c.buf);
      }
    }
  };
  // prologue: K-tile 0 (all four half-tiles) and K-tile 1's A0 / B0
#pragma unroll
  for (int kind = 0; kind < 4; ++kind) {
    issue_piece(c1, kind, 0, true);
    issue_piece(c1, kind, 1, true);
  }
  c2 = c1;
  cur_next(g, c2, nk, G);
  bool more = c2.valid;
  if (more) {
    issue_piece(c2, 0, 0, true);
    issue_piece(c2, 0, 1, true);
    issue_piece(c2, 1, 0, true);
    issue_piece(c2, 1, 1, true);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  // the multiplied K-tile's buffer; c1 <- K-tile 1, c2 <- K-tile 2
  uint32_t bufc = 0;
  c1 = c2;
  cur_next(g, c2, nk, G);
  raw_barrier();
  if (wm == 1) raw_barrier();  // stagger: group 1 runs one barrier behind group 0

  constexpr bool SPREAD = VAR == 0 && EPI != EPI_DGELU;
  constexpr int SPQ = EPI == EPI_GELU ? 8 : 4;  // VMEM stores per spread quadrant
  int seq = v;
  bool has_prev = false;  // a finished tile's accumulators wait to be stored (SPREAD)
  int pm0 = 0, pn0 = 0, pmlo = 0, pnlo = 0;
  int w1 = 0, w2 = 0, w3 = 0;  // stores issued in the previous 3 phases (vmcnt accounting)
  f32x4 acc[8][4];
  bf16x8 af[4][2], b0f[2][2], b1f[2][2];

// LDS fragment reads of phase P
#define NT_READS(P)                                                                             \
  {                                                                                            \
    const char* base_ = smem + bufc;                                                           \
    if (P == 0 || P == 2) {                                                                    \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        af[i][kk] = rd16(base_ + offA[kk] + ((P >> 1) * 64 + 16 * i) * 128);                   \
    }                                                                                          \
    if (P == 0) {                                                                              \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        b0f[j][kk] = rd16(base_ + offB[kk] + (16 * j) * 128);                                  \
    }                                                                                          \
    if (P == 1) {                                                                              \
      _Pragma("unroll") for (int j = 0; j < 2; ++j)                                            \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        b1f[j][kk] = rd16(base_ + offB[kk] + (32 + 16 * j) * 128);                             \
    }                                                                                          \
  }
// DMA of phase P (half-tile P+6 of the stream) + the counted wait retiring what phase P+1 reads
#define NT_DMA_WAIT(P)                                                                          \
  {                                                                                            \
    const Cur& cc_ = (P < 2) ? c1 : c2;                                                        \
    constexpr int kind_ = P == 0 ? 2 : P == 1 ? 3 : P == 2 ? 0 : 1;                            \
    if (cc_.valid) {                                                                           \
      if constexpr (PROBE == 1) {                                                              \
      } else if constexpr (PROBE == 3) {                                                       \
        issue_piece(cc_, kind_, 0, false);                                                     \
      } else if constexpr (VAR == 1) {                                                         \
        issue_piece(cc_, kind_, 0, false);                                                     \
        issue_piece(cc_, kind_, 1, false);                                                     \
      } else if constexpr (kind_ == 0 || kind_ == 3) {                                         \
        constexpr int h_ = kind_ == 3;                                                         \
        dma16x2(cc_.a, voA[h_][0], voA1m[h_], ldA[h_][0] + cc_.buf);                           \
      } else {                                                                                 \
        constexpr int h_ = kind_ == 2;                                                         \
        dma16x2(cc_.b, voB[h_][0], voB1m[h_], ldB[h_][0] + cc_.buf);                           \
      }                                                                                        \
      if constexpr (PROBE == 2) {                                                              \
      } else if constexpr (PROBE == 3) {                                                       \
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");                                      \
      } else if constexpr (SPREAD) {                                                           \
        vm_wait_dyn(8 + st_ + w1 + w2 + w3);                                                   \
      } else {                                                                                 \
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                                      \
      }                                                                                        \
    } else {                                                                                   \
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                        \
    }                                                                                          \
  }
// one phase: P = 0..3, FIRST = first K-tile of an output tile (kk = 0 MFMAs start from 0)
#define NT_PHASE(P, FIRST)                                                                      \
  {                                                                                            \
    int st_ = 0;                                                                               \
    if constexpr (SPREAD && (FIRST)) {                                                         \
      if (has_prev) {                                                                          \
        store_quad<EPI>(g, acc, P == 2 || P == 3, P == 1 || P == 2, pm0, pn0, pmlo, pnlo, wm, wn, lane); \
        st_ = SPQ;                                                                             \
      }                                                                                        \
    }                                                                                          \
    NT_READS(P)                                                                                \
    NT_DMA_WAIT(P)                                                                             \
    w3 = w2;                                                                                   \
    w2 = w1;                                                                                   \
    w1 = st_;                                                                                  \
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
    raw_barrier();                                                                             \
  }
#define NT_KTILE(FIRST)              \
  {                                  \
    NT_PHASE(0, FIRST)               \
    NT_PHASE(1, FIRST)               \
    NT_PHASE(2, FIRST)               \
    NT_PHASE(3, FIRST)               \
    bufc ^= (uint32_t)BUF;           \
    c1 = c2;                         \
    cur_next(g, c2, nk, G);          \
  }

  while (true) {
    NT_KTILE(true)
    for (int t = 1; t < nk; ++t) NT_KTILE(false)

    int m0, n0, mlo, nlo;
    tile_coords(g, seq, m0, n0, mlo, nlo);
    if constexpr (SPREAD) {
      has_prev = true;
      pm0 = m0;
      pn0 = n0;
      pmlo = mlo;
      pnlo = nlo;
    } else if constexpr (PROBE != 4) {
#pragma unroll
      for (int qd = 0; qd < 4; ++qd)
        store_quad<EPI, PROBE == 8>(g, acc, qd >> 1, qd & 1, m0, n0, mlo, nlo, wm, wn, lane);
    } else {
      // probe: keep the accumulators live without storing them
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("" ::"v"(acc[i][j]));
    }
    seq += G;
    if (seq >= g.tiles) break;
  }
  if constexpr (SPREAD) {  // the last tile's epilogue has no next tile to hide under
#pragma unroll
    for (int qd = 0; qd < 4; ++qd) store_quad<EPI>(g, acc, qd >> 1, qd & 1, pm0, pn0, pmlo, pnlo, wm, wn, lane);
  }
#undef NT_KTILE
#undef NT_PHASE
#undef NT_READS
#undef NT_DMA_WAIT
  if (wm == 0) raw_barrier();  // close the stagger: both groups end at the same barrier count
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// epi: 0 = bf16 store, 1 = u + gelu(u) into C / C2, 2 = acc * gelu'(U); bits 8-11: timing
// probe (see the kernel; wrong results); bits 12-15: variant.  grid = persistent workgroup count (#CUs).
NSA_API hipError_t nsa_gemm_nt(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* C2,
                               const void* U, int M, int N, int K, int grid, hipStream_t s) {
  const int probe = (epi >> 8) & 0xf;
  const int var = (epi >> 12) & 0xf;
  epi &= 0xff;
  if (M < BM || N < BN || K < BK || K % BK != 0 || lda % 8 || ldb % 8 || ldc % 4 || lda < K || ldb < K ||
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
  const dim3 gr(grid < a.tiles ? grid : a.tiles);
#define NT_LAUNCH(E)                                                        \
  if (probe == 1) gemm_nt_kernel<E, 1, 0><<<gr, NTHR, 0, s>>>(a);           \
  else if (probe == 2) gemm_nt_kernel<E, 2, 0><<<gr, NTHR, 0, s>>>(a);      \
  else if (probe == 3) gemm_nt_kernel<E, 3, 0><<<gr, NTHR, 0, s>>>(a);      \
  else if (probe == 4) gemm_nt_kernel<E, 4, 1><<<gr, NTHR, 0, s>>>(a);      \
  else if (probe == 5) gemm_nt_kernel<E, 1, 1><<<gr, NTHR, 0, s>>>(a);      \
  else if (probe == 6) gemm_nt_kernel<E, 6, 1><<<gr, NTHR, 0, s>>>(a);      \
  else if (probe == 7) gemm_nt_kernel<E, 6, 0><<<gr, NTHR, 0, s>>>(a);      \
  else if (probe == 8) gemm_nt_kernel<E, 8, 1><<<gr, NTHR, 0, s>>>(a);      \
  else if (var == 1) gemm_nt_kernel<E, 0, 1><<<gr, NTHR, 0, s>>>(a);        \
  else gemm_nt_kernel<E, 0, 0><<<gr, NTHR, 0, s>>>(a);
  switch (epi) {
    case EPI_BF16: NT_LAUNCH(EPI_BF16) break;
    case EPI_GELU: NT_LAUNCH(EPI_GELU) break;
    case EPI_DGELU: NT_LAUNCH(EPI_DGELU) break;
    default: return hipErrorInvalidValue;
  }
#undef NT_LAUNCH
  return hipGetLastError();
}
