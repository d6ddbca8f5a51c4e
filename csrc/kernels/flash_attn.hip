// Causal flash attention forward + backward for gfx950.
//
// nanoGPT's CausalSelfAttention calls
//   F.scaled_dot_product_attention(q, k, v, dropout_p, is_causal=True)
// on q,k,v split out of the packed c_attn output.  Our kernels read the packed
// activation qkv[B, T, 3C] (q | k | v, head h at columns h*D) directly and write
// y[B, T, C] / dqkv[B, T, 3C] directly, so there are no transposes or splits
// around the kernel at all.
//
// Matrix work is v_mfma_f32_32x32x16_bf16 on 64-lane waves.  Layout choices
// (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"):
//
// forward, per wave = 32 queries, per KV tile = 64 keys (2 sub-blocks of 32):
//   S^T[key][q] = K · Q^T         A = K   (LDS, ds_read_b128), B = Q^T (registers)
//     -> the query is the MFMA column = the lane: running max / sum / rescale
//        are lane-local (+ one xor-32 exchange), no LDS round trip.
//   O^T[d][q] += V^T · P^T        A = V^T (LDS, ds_read_b64_tr_b16 transposed
//        read of the row-major V tile), B = P^T straight from the S^T
//        accumulator registers (bf16-converted, permuted k order).
// backward: a dK/dV kernel (per wave = 32 keys, loop over query blocks) and a separate
// dQ kernel (per wave = 32 queries, loop over key tiles), so dQ is written once, in bf16,
// with no atomics and no fp32 accumulator:
//   S = Q·K^T, dP = dO·V^T        key on the lane; K, V fragments live in registers
//   dV^T += dO^T · P,  dK^T += Q^T · dS      accumulators as B operands, A by tr reads
//   dQ^T += K^T · dS^T            (dQ kernel) the query on the lane, recomputing S and dP
// Kernel variants are chosen once per process (FlashConfig below), not per launch.
//
// LDS images are XOR-swizzled per 16-byte chunk with a bit-reversed row key:
//   phys_chunk = chunk ^ bitrev((row / rows_per_bank_row) mod chunks_per_row)
// which is conflict-free both for the 16-row ds_read_b128 groups and for the
// 4-row x 4-chunk blocks of ds_read_b64_tr_b16 (checked for D = 32, 64, 128).
//
// Built with -fno-slp-vectorize (nanosandbox_amd/build.py FILE_FLAGS): hipcc's SLP pass packed
// adjacent f32 multiplies / adds of the softmax (score scaling, row sums, dS) into v_pk_mul_f32
// / v_pk_add_f32, which cost more issue cycles beside MFMAs than two scalar ops
// (MI355X_MICROARCH.md 'price of one filler': 1 v_pk_fma_f32 +22 cycles vs 2 v_fma_f32); the
// fast-tile score scaling is written as scalar multiplies for the same reason.
//
// Softmax uses exp2 with log2(e)/sqrt(D) folded into one multiplier; the LSE
// (natural log) is saved per query for the backward recompute of P.
// Dropout (char config, p = 0.2) uses the counter-based hash of common.h on
// (b*H+h, q, k), so the backward regenerates the mask.
#include "common.h"

#include <type_traits>

// Element type.  This file is compiled twice: as is (bf16) and by flash_attn_f16.hip with
// NSA_FA_F16 = 1 (fp16 Q/K/V/O/dO/dQKV and fp16 P / dS operands, nanoGPT's dtype='float16';
// v_mfma_f32_32x32x16_f16 runs at the bf16 rate).  The fp16 build's entry points carry an
// _h suffix and share the bf16 build's kernel selection (FlashConfig).
#ifndef NSA_FA_F16
#define NSA_FA_F16 0
#endif
#if NSA_FA_F16
#define NSA_FA_SYM(name) name##_h
#else
#define NSA_FA_SYM(name) name
#endif
constexpr bool kFaH = NSA_FA_F16 != 0;

namespace {

// one f32 -> an operand-fragment element; a fragment element -> f32
__device__ __forceinline__ __bf16 fa_elt(float v) { return f2frag<kFaH>(v); }
__device__ __forceinline__ float fa_f(__bf16 v) { return e2f<kFaH>(__builtin_bit_cast(uint16_t, v)); }

constexpr float kLog2e = 1.4426950408889634f;
#ifndef ATTN_ORDER_DEFAULT
#define ATTN_ORDER_DEFAULT 0
#endif

template <int D>
struct Geo {
  static constexpr int CPR = D / 8;                         // 16-byte chunks per row
  static constexpr int RPB = CPR >= 16 ? 1 : 16 / CPR;      // rows per 256-byte bank row
  static constexpr int BITS = CPR == 4 ? 2 : CPR == 8 ? 3 : 4;
};

template <int BITS>
__device__ __forceinline__ int bitrev(int k) {
  if constexpr (BITS == 2) return ((k & 1) << 1) | ((k >> 1) & 1);
  else if constexpr (BITS == 3) return ((k & 1) << 2) | (k & 2) | ((k >> 2) & 1);
  else return (int)(__builtin_bitreverse32((uint32_t)k) >> 28);
}

// byte offset of (row, chunk) inside a swizzled [rows][D] bf16 tile
template <int D>
__device__ __forceinline__ int swz(int row, int chunk) {
  using G = Geo<D>;
  const int key = bitrev<G::BITS>((row / G::RPB) & (G::CPR - 1));
  return row * (D * 2) + ((chunk ^ key) << 4);
}

__device__ __forceinline__ uint4 lds_b128(const char* base, int off) {
  return *reinterpret_cast<const uint4*>(base + off);
}

__device__ __forceinline__ s16x4 lds_tr(const char* base, int off) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(base + off));
}

__device__ __forceinline__ bf16x8 cat_tr(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}

__device__ __forceinline__ bf16x8 as_frag(uint4 u) { return __builtin_bit_cast(bf16x8, u); }

__device__ __forceinline__ f32x16 mfma(bf16x8 a, bf16x8 b, f32x16 c) { return mfma32e<kFaH>(a, b, c); }

// Workgroup -> (b*H + h, tile) order; tile 0 is a kernel's heaviest (longest causal
// range), launched first.
//  order 0: tile-major with (b, h) fastest: every (b, h)'s heaviest tile before any
//           lighter one, chip-wide.
//  order 1 (XCD-grouped): the dispatcher places workgroup v on XCD v % 8, so XCD x is
//           given a contiguous range of (b, h) and walks all tiles of one (b, h) back to
//           back, heaviest first.  The K/V (forward, dQ) or Q/dO (dK/dV) rows those tiles
//           all stream then come from that XCD's L2 while they are in flight together,
//           instead of once per tile from HBM (with tile-major order the 8 tiles of a
//           (b, h) are B*H workgroups apart and never co-resident).
__device__ __forceinline__ void attn_order(int n_tiles, int BH, int order, int& bh, int& t) {
  const int v = blockIdx.x;
  if (order == 0) {
    t = v / BH;
    bh = v % BH;
    return;
  }
  if (order == 2) {  // (b, h)-major: the tiles of one (b, h) are consecutive workgroups
    bh = v / n_tiles;
    t = v % n_tiles;
    return;
  }
  const int total = n_tiles * BH;
  const int xcd = v % 8, q = total / 8, r = total % 8;
  const int u = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + v / 8;
  bh = u / n_tiles;
  t = u % n_tiles;
}

// Kernel selection, resolved once (first launch) from the environment and changed only
// through nsa_flash_set_variant (tests / A/B scripts):
//   fwd   NSA_FLASH_FWD = auto (default) | v1 | v5: D = 64 forward kernel; auto = v5 without
//         dropout once the grid has >= 4096 workgroups, else v1 (fwd_launch); v5 = 64 queries
//         per wave, two K/V tiles per barrier, fast tiles (no running max while scores stay in
//         range); v1 = 32 queries per wave, exact online softmax, dropout
//   bwd   NSA_FLASH_BWD = v3 (default) | v2 | v1: D = 64 backward; v3 = v2 with the dK/dV
//         kernel taking two query slices per barrier; v1 = the generic kernels
//         (software-pipelining the dQ tile's / the dK/dV slice pair's MFMAs under each
//         other's VALU with sched_group_barrier measured no gain / a spilling kernel:
//         docs/performance.md, round 5)
//   order NSA_ATTN_ORDER = 0 (default) | 1: workgroup order (attn_order)
enum { FWD_AUTO = 0, FWD_V1 = 1, FWD_V5 = 5 };
enum { BWD_V1 = 1, BWD_V2 = 2, BWD_V3 = 3 };
struct FlashConfig {
  int fwd, bwd, order;
};
}  // namespace
// one selection for both element types: the fp16 build uses the bf16 build's record
NSA_API void* nsa_flash_config_ptr();
namespace {
#if NSA_FA_F16
FlashConfig& flash_config() { return *static_cast<FlashConfig*>(nsa_flash_config_ptr()); }
#else
FlashConfig& flash_config() {
  static FlashConfig c = [] {
    FlashConfig d{FWD_AUTO, BWD_V3, ATTN_ORDER_DEFAULT};
    if (const char* e = getenv("NSA_FLASH_FWD"))
      d.fwd = (e[0] == 'v' && (e[1] == '1' || e[1] == '5')) ? e[1] - '0' : FWD_AUTO;
    if (const char* e = getenv("NSA_FLASH_BWD"))
      d.bwd = (e[0] == 'v' && e[1] >= '1' && e[1] <= '3') ? e[1] - '0' : BWD_V3;
    if (const char* e = getenv("NSA_ATTN_ORDER")) d.order = (e[0] >= '0' && e[0] <= '2') ? e[0] - '0' : 0;
    return d;
  }();
  return c;
}
#endif
int attn_order_env() { return flash_config().order; }

// accumulator register i of a 32x32 tile holds row (i&3) + 8*(i>>2) + 4*h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Transposed-read address for an MFMA operand whose 8 elements are 4+4 consecutive
// rows of a row-major tile:  first read rows r0+0..3, second read rows r1+0..3;
// the lane's column is col_base + (lane & 31) where col_base is this 32-column tile.
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const char* tile, int r0, int r1, int col_base, int lane) {
  const int g = lane >> 4, ig = lane & 15;
  const int q = ig >> 2, p = ig & 3;
  const int col = col_base + 16 * (g & 1) + 4 * p;
  const int chunk = col >> 3, half = (col >> 2) & 1;
  const s16x4 a = lds_tr(tile, swz<D>(r0 + q, chunk) + half * 8);
  const s16x4 b = lds_tr(tile, swz<D>(r1 + q, chunk) + half * 8);
  return cat_tr(a, b);
}

// tr-read fragment for a tile with a different row width W (elements) than D
template <int W>
__device__ __forceinline__ bf16x8 tr_frag_w(const char* tile, int r0, int r1, int col_base, int lane) {
  return tr_frag<W>(tile, r0, r1, col_base, lane);
}

// global -> LDS DMA of 16 bytes per lane (lane l writes lds_dst + 16 l); M0 saved and
// restored around it.  Volatile asm: the compiler keeps it where it is written (it
// neither sinks it towards a later use nor counts it in its own vmcnt bookkeeping).
// glds16s: wave-uniform 64-bit base in SGPRs + a 32-bit per-lane byte offset (one VGPR
// per address instead of two).
// NSA_FA_M0KEEP=0 (default): M0 is written, not saved and restored — nothing else in these
// kernels reads M0 (checked in the ISA: every m0 access is one of these statements), and
// the save / restore pair cost two SALU per piece.
#ifndef NSA_FA_M0KEEP
#define NSA_FA_M0KEEP 0
#endif
__device__ __forceinline__ void glds16s(uint32_t voff, const void* sbase, uint32_t lds_dst) {
  if constexpr (NSA_FA_M0KEEP) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(sbase), "s"(lds_dst)
                 : "memory");
  } else {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(lds_dst)
                 : "memory");
  }
}
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  if constexpr (NSA_FA_M0KEEP) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds_dst)
                 : "memory");
  } else {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(lds_dst) : "memory");
  }
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (0 .. 15)
__device__ __forceinline__ void vm_wait(int n) {
#define NSA_VMW(N) \
  case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
  switch (n) {
    NSA_VMW(0) NSA_VMW(1) NSA_VMW(2) NSA_VMW(3) NSA_VMW(4) NSA_VMW(5) NSA_VMW(6) NSA_VMW(7)
    NSA_VMW(8) NSA_VMW(9) NSA_VMW(10) NSA_VMW(11) NSA_VMW(12) NSA_VMW(13) NSA_VMW(14)
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
#undef NSA_VMW
}

// =============================================================================
// forward
// =============================================================================
// Deferred rescale (cdna_hip_programming.md T13): a lane keeps its running max
// until a tile's max exceeds it by more than kDeferLog2 (log2 units), so the
// O-wide rescale runs only on the (rare, after the first tiles) tiles where some
// lane's max grows that much.  P is then bounded by 2^kDeferLog2 = 256, which the
// fp32 accumulators absorb; l and the saved LSE stay exact (both relative to m).
constexpr float kDeferLog2 = 8.0f;

// sum / max with the other half-wave (lane ^ 32) through one v_permlane32_swap:
// the swap returns {own value for lanes < 32 | partner's for lanes >= 32,
// partner's for lanes < 32 | own for lanes >= 32}, so combining both halves of
// the pair gives the pair's reduction on every lane.
__device__ __forceinline__ float half_swap_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float half_swap_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

// Dropout parameters of one launch (char config); unused by the DROP=false build.
struct DropArgs {
  uint32_t thresh;
  float scale;
  uint64_t seed;
  int bh, T;
};

// One 64-key tile for one wave (32 queries): S^T = K·Q^T, online softmax, O^T += V^T·P^T.
// MASK: the tile straddles this wave's causal diagonal (exactly one tile per wave).
template <int D, bool MASK, bool DROP>
__device__ __forceinline__ void fwd_tile(const char* kt, const char* vt, const bf16x8 (&qf)[D / 16],
                                         f32x16 (&o)[D / 32], float& m_i, float& l_i, int kv0, int qpos, int h,
                                         int r, int lane, float scale_log2, const DropArgs& dr) {
  constexpr int NKS = D / 16;
  constexpr int NDT = D / 32;
  f32x16 st[2];
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    st[sb] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 kf = as_frag(lds_b128(kt, swz<D>(32 * sb + r, 2 * ks + h)));
      st[sb] = mfma(kf, qf[ks], st[sb]);
    }
  }
  float mt = -INFINITY;
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (MASK) {
        if (kv0 + 32 * sb + acc_row(i, h) > qpos) st[sb][i] = -INFINITY;
      }
      mt = fmaxf(mt, st[sb][i]);
    }
  }
  mt = half_swap_max(mt);
  const bool grow = (mt - m_i) * scale_log2 > kDeferLog2;
  if (__builtin_amdgcn_ballot_w64(grow)) {  // wave-uniform: rescale only when some lane's max moved
    const float m_new = grow ? mt : m_i;
    const float alpha = fast_exp2((m_i - m_new) * scale_log2);
    l_i *= alpha;
    m_i = m_new;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[dt] *= alpha;
  }
  const float mc = m_i * scale_log2;
  float rs = 0.0f;
  bf16x8 pf[2][2];
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float p = fast_exp2(st[sb][i] * scale_log2 - mc);
      rs += p;
      if constexpr (DROP) {
        const int kpos = kv0 + 32 * sb + acc_row(i, h);
        const uint64_t id = ((uint64_t)dr.bh * dr.T + (uint64_t)qpos) * (uint64_t)dr.T + (uint64_t)kpos;
        p = nsa_keep(dr.seed, id, dr.thresh) ? p * dr.scale : 0.0f;
      }
      pf[sb][i >> 3][i & 7] = fa_elt(p);
    }
  }
  l_i += half_swap_sum(rs);
  // O^T += V^T · P^T
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r0 = 32 * sb + 16 * s + 4 * h;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 vf = tr_frag<D>(vt, r0, r0 + 8, 32 * dt, lane);
        o[dt] = mfma(vf, pf[sb][s], o[dt]);
      }
    }
  }
}

// K/V tile staging through registers (T14 split: issue before compute, write after)
#define NSA_FWD_STAGE_LOAD(J)                                                                   \
  _Pragma("unroll") for (int c = 0; c < CHUNKS_PER_THREAD; ++c) {                               \
    const int e = tid + 256 * c;                                                                \
    const int row = e / CPR, ch = e % CPR;                                                      \
    int key = (J) * BN + row;                                                                   \
    key = key < T ? key : T - 1;                                                                \
    kst[c] = *reinterpret_cast<const uint4*>(kbase + (int64_t)key * row_stride + ch * 8);       \
    vst[c] = *reinterpret_cast<const uint4*>(vbase + (int64_t)key * row_stride + ch * 8);       \
  }
#define NSA_FWD_STAGE_WRITE(BUF)                                                                \
  _Pragma("unroll") for (int c = 0; c < CHUNKS_PER_THREAD; ++c) {                               \
    const int e = tid + 256 * c;                                                                \
    const int row = e / CPR, ch = e % CPR;                                                      \
    *reinterpret_cast<uint4*>(smem + (BUF) * TILE_BYTES + swz<D>(row, ch)) = kst[c];            \
    *reinterpret_cast<uint4*>(smem + (2 + (BUF)) * TILE_BYTES + swz<D>(row, ch)) = vst[c];      \
  }

// workgroup = 4 waves x 32 queries; K/V tiles of 64 keys double-buffered in LDS
// (32 KB at D = 64, so LDS admits 4 workgroups per CU; VGPRs set the occupancy).
// DMA (D = 64): the next K/V tile is fetched by LDS-DMA into the idle buffer at the top
// of the iteration.  The register-staged form (DMA = false, other head dims) is what the
// T14 split intends, but hipcc sinks the staging loads out of the loop head into the
// latch, right before their LDS writes (the tile compute sits in branches), so every
// tile waited out a full global-memory round trip.
template <int D, bool DROP, bool DMA = false>
__global__ __launch_bounds__(256, (D <= 64 && !DROP) ? (DMA ? 4 : 3) : 2) void flash_fwd_kernel(
    const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out, float* __restrict__ lse_out, int B, int T, int H,
    float scale_log2, uint32_t drop_thresh, float drop_scale, uint64_t seed, int order) {
  constexpr int BN = 64;
  constexpr int TILE_BYTES = BN * D * 2;
  constexpr int CPR = D / 8;
  constexpr int CHUNKS_PER_THREAD = BN * CPR / 256;  // 16-byte chunks of one K (or V) tile per thread
  constexpr int NKS = D / 16;                       // k-steps over the head dim
  constexpr int NDT = D / 32;                       // 32-wide output tiles over the head dim
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // K[2], V[2]

  const int C = H * D;
  const int64_t row_stride = 3 * (int64_t)C;
  const int BH = B * H;
  const int n_qt = (T + 127) / 128;
  int bh, qt;
  attn_order(n_qt, BH, order, bh, qt);
  qt = n_qt - 1 - qt;  // heaviest (longest causal) tiles first
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int q0 = qt * 128;
  const int q0w = q0 + 32 * w;
  const int qpos = q0w + r;
  const bf16_t* base = qkv + (int64_t)b * T * row_stride;
  const bf16_t* qbase = base + hh * D;
  const bf16_t* kbase = base + C + hh * D;
  const bf16_t* vbase = base + 2 * C + hh * D;
  const DropArgs dr{drop_thresh, drop_scale, nsa_seed(seed), bh, T};

  // Q^T fragments (B operand): lane holds Q[qpos][16ks + 8h .. +8]
  bf16x8 qf[NKS];
  {
    const int qc = qpos < T ? qpos : T - 1;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      qf[ks] = as_frag(*reinterpret_cast<const uint4*>(qbase + (int64_t)qc * row_stride + 16 * ks + 8 * h));
  }

  f32x16 o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = f32x16{};
  float m_i = -1e30f, l_i = 0.0f;

  const int kv_end = min(T, q0 + 128);
  const int n_tiles = (kv_end + BN - 1) / BN;

  if constexpr (DMA) {
    static_assert(D == 64, "DMA tile geometry is for D = 64");
    // tile j -> buffer: wave w fills rows 16w .. 16w+15 of K and V (2 x 1 KiB pieces
    // each); lane l lands at 16 l of its piece, i.e. row 16w + 8i + (l >> 3), physical
    // chunk l & 7, so it fetches logical chunk (l & 7) ^ key(row)
    const uint32_t lds0 =
        __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));
    const int prow = 16 * w + (lane >> 3);
    const int pch0 = (lane & 7) ^ bitrev<3>((prow >> 1) & 7);
    const int pch1 = (lane & 7) ^ bitrev<3>(((prow + 8) >> 1) & 7);
    // per-lane byte offsets from the tile's first key row (a batch's qkv slice is
    // T x 3C x 2 bytes, far below 4 GiB); the tile base lives in SGPRs
    const uint32_t koff0 = (uint32_t)((prow * (int)row_stride + pch0 * 8) * 2);
    const uint32_t koff8 = (uint32_t)(((prow + 8) * (int)row_stride + pch1 * 8) * 2);
    auto issue = [&](int jt, int buf) {
      const bf16_t* kt_base = kbase + (int64_t)jt * BN * row_stride;
      uint32_t o0 = koff0, o8 = koff8;
      if (jt * BN + BN > T) {  // ragged last tile: clamp rows to T - 1 (wave-uniform branch)
        const int r0 = min(jt * BN + prow, T - 1) - jt * BN, r8 = min(jt * BN + prow + 8, T - 1) - jt * BN;
        o0 = (uint32_t)((r0 * (int)row_stride + pch0 * 8) * 2);
        o8 = (uint32_t)((r8 * (int)row_stride + pch1 * 8) * 2);
      }
      const uint32_t kb = lds0 + (uint32_t)(buf * TILE_BYTES + 16 * w * 128);
      const uint32_t vb = kb + 2 * TILE_BYTES;
      glds16s(o0, kt_base, __builtin_amdgcn_readfirstlane(kb));
      glds16s(o8, kt_base, __builtin_amdgcn_readfirstlane(kb + 1024));
      glds16s(o0, kt_base + C, __builtin_amdgcn_readfirstlane(vb));
      glds16s(o8, kt_base + C, __builtin_amdgcn_readfirstlane(vb + 1024));
    };
    asm volatile("" ::"v"(qf[0]), "v"(qf[1]), "v"(qf[2]), "v"(qf[3]));  // Q landed before the DMA
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int j = 0; j < n_tiles; ++j) {
      const int cur = j & 1;
      const int kv0 = j * BN;
      // the idle buffer held tile j-1, which every wave finished at the last barrier
      // (the final iteration re-fetches its own tile there: harmless, branch-free)
      issue(min(j + 1, n_tiles - 1), cur ^ 1);
      const char* kt = smem + cur * TILE_BYTES;
      const char* vt = smem + (2 + cur) * TILE_BYTES;
      if (kv0 + BN - 1 <= q0w)  // wave-uniform: whole tile visible to every query of the wave
        fwd_tile<D, false, DROP>(kt, vt, qf, o, m_i, l_i, kv0, qpos, h, r, lane, scale_log2, dr);
      else if (kv0 <= q0w + 31)  // the wave's diagonal tile
        fwd_tile<D, true, DROP>(kt, vt, qf, o, m_i, l_i, kv0, qpos, h, r, lane, scale_log2, dr);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    uint4 kst[CHUNKS_PER_THREAD], vst[CHUNKS_PER_THREAD];
    NSA_FWD_STAGE_LOAD(0)
    NSA_FWD_STAGE_WRITE(0)
    __syncthreads();

    for (int j = 0; j < n_tiles; ++j) {
      const int cur = j & 1;
      const int kv0 = j * BN;
      // unconditional staging (the last iteration re-stages its own tile into the idle
      // buffer): conditional register staging makes hipcc keep kst/vst in scratch
      { NSA_FWD_STAGE_LOAD(min(j + 1, n_tiles - 1)) }
      const char* kt = smem + cur * TILE_BYTES;
      const char* vt = smem + (2 + cur) * TILE_BYTES;
      if (kv0 + BN - 1 <= q0w)  // wave-uniform: whole tile visible to every query of the wave
        fwd_tile<D, false, DROP>(kt, vt, qf, o, m_i, l_i, kv0, qpos, h, r, lane, scale_log2, dr);
      else if (kv0 <= q0w + 31)  // the wave's diagonal tile
        fwd_tile<D, true, DROP>(kt, vt, qf, o, m_i, l_i, kv0, qpos, h, r, lane, scale_log2, dr);
      { NSA_FWD_STAGE_WRITE(cur ^ 1) }
      __syncthreads();
    }
  }

  // epilogue: O = O^T / l ; lane owns query qpos, registers hold d
  if (qpos < T) {
    const float inv_l = 1.0f / l_i;
    bf16_t* orow = out + ((int64_t)b * T + qpos) * C + hh * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 u;
        u.x = pk2<kFaH>(o[dt][4 * g + 0] * inv_l, o[dt][4 * g + 1] * inv_l);
        u.y = pk2<kFaH>(o[dt][4 * g + 2] * inv_l, o[dt][4 * g + 3] * inv_l);
        *reinterpret_cast<uint2*>(orow + d) = u;
      }
    }
    if (h == 0) lse_out[(int64_t)bh * T + qpos] = (m_i * scale_log2 + __log2f(l_i)) * 0.6931471805599453f;
  }
}
#undef NSA_FWD_STAGE_LOAD
#undef NSA_FWD_STAGE_WRITE

// =============================================================================
// forward v3 (D = 64): one wave = 64 queries as two independent 32-query blocks
// against the same K/V tile.  v1 gives a wave one dependency chain per tile
// (S MFMAs -> row max -> exp -> P·V MFMAs) and leaves the overlap to the other
// waves of the SIMD; the PMC trace shows the waves parked on that chain (42 %
// of wave cycles in s_waitcnt, ≈21 % MFMA busy).  Two blocks per wave give the
// scheduler a second chain inside the wave (block A's softmax VALU beside block
// B's S MFMAs, A's P·V beside B's exp) and halve the LDS reads per MFMA (each K
// fragment and each transposed V fragment feeds two MFMAs).  Workgroup = 4 waves
// = 256 queries; K/V tiles of 64 keys by LDS-DMA, double-buffered (32 KB).
// =============================================================================
template <bool MASK, bool DROP>
__device__ __forceinline__ void fwd_tile2(const char* kt, const char* vt, const bf16x8 (&qf)[2][4],
                                          f32x16 (&o)[2][2], float (&m_i)[2], float (&l_i)[2], int kv0, int qposA,
                                          int h, int r, int lane, float scale_log2, const DropArgs& dr) {
  constexpr int D = 64;
  f32x16 st[2][2];  // [block][key sub-block]
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    st[0][sb] = f32x16{};
    st[1][sb] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 kf = as_frag(lds_b128(kt, swz<D>(32 * sb + r, 2 * ks + h)));
      st[0][sb] = mfma(kf, qf[0][ks], st[0][sb]);
      st[1][sb] = mfma(kf, qf[1][ks], st[1][sb]);
    }
  }
  float mt[2];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    mt[blk] = -INFINITY;
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if constexpr (MASK) {
          if (kv0 + 32 * sb + acc_row(i, h) > qposA + 32 * blk) st[blk][sb][i] = -INFINITY;
        }
        mt[blk] = fmaxf(mt[blk], st[blk][sb][i]);
      }
    }
    mt[blk] = half_swap_max(mt[blk]);
  }
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const bool grow = (mt[blk] - m_i[blk]) * scale_log2 > kDeferLog2;
    if (__builtin_amdgcn_ballot_w64(grow)) {
      const float m_new = grow ? mt[blk] : m_i[blk];
      const float alpha = fast_exp2((m_i[blk] - m_new) * scale_log2);
      l_i[blk] *= alpha;
      m_i[blk] = m_new;
      o[blk][0] *= alpha;
      o[blk][1] *= alpha;
    }
  }
  bf16x8 pf[2][2][2];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const float mc = m_i[blk] * scale_log2;
    float rs = 0.0f;
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float p = fast_exp2(st[blk][sb][i] * scale_log2 - mc);
        rs += p;
        if constexpr (DROP) {
          const int kpos = kv0 + 32 * sb + acc_row(i, h);
          const uint64_t id =
              ((uint64_t)dr.bh * dr.T + (uint64_t)(qposA + 32 * blk)) * (uint64_t)dr.T + (uint64_t)kpos;
          p = nsa_keep(dr.seed, id, dr.thresh) ? p * dr.scale : 0.0f;
        }
        pf[blk][sb][i >> 3][i & 7] = fa_elt(p);
      }
    }
    l_i[blk] += half_swap_sum(rs);
  }
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r0 = 32 * sb + 16 * s + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const bf16x8 vf = tr_frag<D>(vt, r0, r0 + 8, 32 * dt, lane);
        o[0][dt] = mfma(vf, pf[0][sb][s], o[0][dt]);
        o[1][dt] = mfma(vf, pf[1][sb][s], o[1][dt]);
      }
    }
  }
}

// =============================================================================
// forward v5 (D = 64): v4's geometry (64 queries per wave as two 32-query blocks, two
// K/V tiles per barrier) with the softmax's per-element instruction count cut in half.
//
// Scores are taken in log2 units, S' = c q·k with c = scale*log2(e) (Q pre-scaled when it is
// loaded, or one packed multiply per score pair: NSA_FWD5_QSCALE below).  The max subtraction is then not needed for
// correctness, only for range: O and l are sums of 2^(S' - m) for ANY per-query m, and
// O / l does not depend on m.  While every score of a wave's queries stays within fp32 /
// bf16 range the kernel runs with m = 0 ("fast" tiles): p = exp2(S') straight from the
// accumulator -- no row max (34 v_max3 + exchanges), no subtract / fma per element, no
// rescale test.  Per tile and lane: 64 v_exp_f32, 32 v_cvt_pk_bf16_f32, the row sum and
// one range test, against v4's ~315 VALU.  The range test is exact: a tile whose row sum
// exceeds 2^64 (or is not finite), or a query whose running l would stay below 2^-60, is
// redone by v4's exact tile (row max, deferred rescale) and the wave stays on exact tiles
// from then on, so extreme logits cost speed, never accuracy.
//
// NSA_FWD5_ROWSUM 0 (default): row sums as fp32 adds of p; 1: v_dot2_f32_bf16 over the bf16
// pairs the P·V MFMAs consume (half the instructions, and l sums exactly the P that
// multiplies V, but a v_dot2 beside MFMAs costs ~10 cycles of issue: MI355X_MICROARCH.md).
// Back-to-back on one box, each against v4 in its own process: v5/v4 0.946 with f32 adds vs
// 0.972-0.979 with v_dot2 (profiles/r5_ab_v5*.log).
// =============================================================================
//
// NSA_FWD5_QSCALE 1: Q pre-scaled as above; 0: Q as loaded and the fast tiles multiply each
// score pair by scale*log2(e) with one v_pk_mul_f32 (32 more VALU per tile, but the scores
// are exactly v4's: the bf16 rounding of q*c costs up to a few % of p once single products
// q_d k_d reach tens of log2 units, e.g. the test suite's +-100 logits).
#ifndef NSA_FWD5_ROWSUM
#define NSA_FWD5_ROWSUM 0
#endif
#ifndef NSA_FWD5_QSCALE
#define NSA_FWD5_QSCALE 0
#endif

template <bool MASK>
__device__ __forceinline__ bool fwd_tile5(const char* kt, const char* vt, const bf16x8 (&qf)[2][4], f32x16 (&o)[2][2],
                                          float (&l_i)[2], int kv0, int qposA, int h, int r, int lane,
                                          float scale_log2) {
  constexpr int D = 64;
  f32x16 st[2][2];  // [block][key sub-block]
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    st[0][sb] = f32x16{};
    st[1][sb] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 kf = as_frag(lds_b128(kt, swz<D>(32 * sb + r, 2 * ks + h)));
      st[0][sb] = mfma(kf, qf[0][ks], st[0][sb]);
      st[1][sb] = mfma(kf, qf[1][ks], st[1][sb]);
    }
  }
  bf16x8 pf[2][2][2];
  float rs[2];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    float acc[2] = {0.0f, 0.0f};  // one chain per key sub-block
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      if constexpr (!NSA_FWD5_QSCALE) {
#pragma unroll
        for (int i = 0; i < 16; ++i) st[blk][sb][i] *= scale_log2;  // scalar v_mul_f32 (see NSA_FA_NOSLP)
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float s = st[blk][sb][i];
        if constexpr (MASK) {
          if (kv0 + 32 * sb + acc_row(i, h) > qposA + 32 * blk) s = -INFINITY;
        }
        const float p = fast_exp2(s);
        if constexpr (NSA_FWD5_ROWSUM == 0) acc[sb] += p;
        pf[blk][sb][i >> 3][i & 7] = fa_elt(p);
      }
      if constexpr (NSA_FWD5_ROWSUM == 1) {
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if constexpr (kFaH) {
            typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
            const f16x8 hv = __builtin_bit_cast(f16x8, pf[blk][sb][s]);
            const f16x2_t one = __builtin_bit_cast(f16x2_t, 0x3C003C00u);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[sb] = __builtin_amdgcn_fdot2(f16x2_t{hv[2 * e], hv[2 * e + 1]}, one, acc[sb], false);
          } else {
            typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
            const bf16x2_t one = __builtin_bit_cast(bf16x2_t, 0x3F803F80u);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[sb] = __builtin_amdgcn_fdot2_f32_bf16(bf16x2_t{pf[blk][sb][s][2 * e], pf[blk][sb][s][2 * e + 1]},
                                                        one, acc[sb], false);
          }
        }
      }
    }
    rs[blk] = half_swap_sum(acc[0] + acc[1]);
  }
  const float lA = l_i[0] + rs[0], lB = l_i[1] + rs[1];
  // NaN-safe: a non-finite sum fails every comparison.  bf16 P holds any fp32 value; fp16 P
  // only up to 65504 and keeps 2^-11 relative precision down to 2^-14, hence its tighter range
  const float hi = kFaH ? 0x1p15f : 0x1p64f, lo = kFaH ? 0x1p-8f : 0x1p-60f;
  const bool ok = rs[0] <= hi && rs[1] <= hi && lA >= lo && lB >= lo;
  if (__builtin_amdgcn_ballot_w64(!ok)) return false;  // wave-uniform: redo this tile exactly
  l_i[0] = lA;
  l_i[1] = lB;
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r0 = 32 * sb + 16 * s + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
        const bf16x8 vf = tr_frag<D>(vt, r0, r0 + 8, 32 * dt, lane);
        o[0][dt] = mfma(vf, pf[0][sb][s], o[0][dt]);
        o[1][dt] = mfma(vf, pf[1][sb][s], o[1][dt]);
      }
    }
  }
  return true;
}

// Hand-over from fast tiles (m = 0) to exact tiles: O and l so far are sums of 2^(S'),
// relative to m = 0.  The exact tiles' deferred rescale only ever RAISES m, so the hand-over
// first moves each query to m' = log2(l) (O and l times 2^-m', l becomes ~1): a tile whose
// scores underflowed (all far below the earlier ones) then adds ~0, one that overflowed
// raises m from there.  A query with nothing accumulated yet (l = 0) gets m = -inf-like, so
// its first exact tile sets the max.  m_i is in the exact tiles' units (raw scores, times
// their multiplier sl).
__device__ __forceinline__ void fwd5_to_exact(f32x16 (&o)[2][2], float (&m_i)[2], float (&l_i)[2], float sl) {
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    if (l_i[blk] > 0.0f) {
      const float mp = __log2f(l_i[blk]);
      const float f = fast_exp2(-mp);
      l_i[blk] *= f;
      o[blk][0] *= f;
      o[blk][1] *= f;
      m_i[blk] = mp / sl;
    } else {
      m_i[blk] = -1e30f;
    }
  }
}

// Workgroup = 4 waves x 64 queries, 4-slot K/V ring filled by LDS-DMA, two tiles per
// barrier (round 4's v4 schedule, whose exact pair tile fwd_tile2 is v5's fallback).
// No dropout (dropout runs v1).
// Probe build only (-DNSA_PROBE_SKIP_TILE=1, build_variant): skip key tile 1 of every
// workgroup -- wrong output, used to show the test suite catches a dropped causal tile.
#ifndef NSA_PROBE_SKIP_TILE
#define NSA_PROBE_SKIP_TILE 0
#endif
#ifndef NSA_PROBE_KV_SHARED
#define NSA_PROBE_KV_SHARED 0  // probe build: every (b, h) reads (0, 0)'s K/V (wrong output; traffic probe)
#endif
__global__ __launch_bounds__(256, 2) void flash_fwd5_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                            float* __restrict__ lse_out, int B, int T, int H,
                                                            float scale_log2, int order) {
  constexpr int D = 64;
  constexpr int BN = 64;
  constexpr int NS = 4;
  constexpr int TILE_BYTES = BN * D * 2;
  __shared__ __attribute__((aligned(16))) char smem[2 * NS * TILE_BYTES];  // K[NS], V[NS]

  const int C = H * D;
  const int64_t row_stride = 3 * (int64_t)C;
  const int BH = B * H;
  const int n_qt = (T + 255) / 256;
  int bh, qt;
  attn_order(n_qt, BH, order, bh, qt);
  qt = n_qt - 1 - qt;  // heaviest (longest causal) tiles first
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int q0 = qt * 256;
  const int q0w = q0 + 64 * w;
  const int qposA = q0w + r;
  const bf16_t* base = qkv + (int64_t)b * T * row_stride;
  const bf16_t* qbase = base + hh * D;
  const bf16_t* kbase = NSA_PROBE_KV_SHARED ? qkv + C : base + C + hh * D;

  // Q fragments, pre-scaled by scale * log2(e) (scores come out of the MFMA in log2 units)
  bf16x8 qf[2][4];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int qp = qposA + 32 * blk;
    const int qc = qp < T ? qp : T - 1;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const bf16x8 raw = as_frag(*reinterpret_cast<const uint4*>(qbase + (int64_t)qc * row_stride + 16 * ks + 8 * h));
#pragma unroll
      for (int e = 0; e < 8; ++e) qf[blk][ks][e] = NSA_FWD5_QSCALE ? fa_elt(fa_f(raw[e]) * scale_log2) : raw[e];
    }
  }
  f32x16 o[2][2];
  float m_i[2], l_i[2];
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    o[blk][0] = f32x16{};
    o[blk][1] = f32x16{};
    m_i[blk] = 0.0f;  // fast tiles: m = 0 (exact tiles take over from there)
    l_i[blk] = 0.0f;
  }
  bool fast = true;  // wave-uniform

  const int kv_end = min(T, q0 + 256);
  const int n_tiles = (kv_end + BN - 1) / BN;
  const uint32_t lds0 =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));
  const int prow = 16 * w + (lane >> 3);
  const int pch0 = (lane & 7) ^ bitrev<3>((prow >> 1) & 7);
  const int pch1 = (lane & 7) ^ bitrev<3>(((prow + 8) >> 1) & 7);
  const uint32_t koff0 = (uint32_t)((prow * (int)row_stride + pch0 * 8) * 2);
  const uint32_t koff8 = (uint32_t)(((prow + 8) * (int)row_stride + pch1 * 8) * 2);
  auto issue = [&](int jt, int buf) {
    const bf16_t* kt_base = kbase + (int64_t)jt * BN * row_stride;
    uint32_t o0 = koff0, o8 = koff8;
    if (jt * BN + BN > T) {
      const int r0 = min(jt * BN + prow, T - 1) - jt * BN, r8 = min(jt * BN + prow + 8, T - 1) - jt * BN;
      o0 = (uint32_t)((r0 * (int)row_stride + pch0 * 8) * 2);
      o8 = (uint32_t)((r8 * (int)row_stride + pch1 * 8) * 2);
    }
    const uint32_t kb = lds0 + (uint32_t)(buf * TILE_BYTES + 16 * w * 128);
    const uint32_t vb = kb + NS * TILE_BYTES;
    glds16s(o0, kt_base, __builtin_amdgcn_readfirstlane(kb));
    glds16s(o8, kt_base, __builtin_amdgcn_readfirstlane(kb + 1024));
    glds16s(o0, kt_base + C, __builtin_amdgcn_readfirstlane(vb));
    glds16s(o8, kt_base + C, __builtin_amdgcn_readfirstlane(vb + 1024));
  };
  asm volatile("" ::"v"(qf[0][0]), "v"(qf[0][1]), "v"(qf[0][2]), "v"(qf[0][3]), "v"(qf[1][0]), "v"(qf[1][1]),
               "v"(qf[1][2]), "v"(qf[1][3]));  // Q landed before the DMA
  const DropArgs dr{0u, 1.0f, 0ull, bh, T};
  const float sl_exact = NSA_FWD5_QSCALE ? 1.0f : scale_log2;  // the exact tiles' score multiplier
  issue(0, 0);
  issue(min(1, n_tiles - 1), 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int j = 0; j < n_tiles; j += 2) {
    issue(min(j + 2, n_tiles - 1), (j + 2) % 4);
    issue(min(j + 3, n_tiles - 1), (j + 3) % 4);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int jj = j + u;
      if (NSA_PROBE_SKIP_TILE && jj == 1) continue;  // test-suite probe: one causal tile dropped
      if (jj < n_tiles) {
        const int kv0 = jj * BN;
        const char* kt = smem + (jj % 4) * TILE_BYTES;
        const char* vt = smem + (4 + jj % 4) * TILE_BYTES;
        if (kv0 + BN - 1 <= q0w) {
          if (!(fast && fwd_tile5<false>(kt, vt, qf, o, l_i, kv0, qposA, h, r, lane, scale_log2))) {
            if (fast) fwd5_to_exact(o, m_i, l_i, sl_exact);
            fast = false;
            fwd_tile2<false, false>(kt, vt, qf, o, m_i, l_i, kv0, qposA, h, r, lane, sl_exact, dr);
          }
        } else if (kv0 <= q0w + 63) {
          if (!(fast && fwd_tile5<true>(kt, vt, qf, o, l_i, kv0, qposA, h, r, lane, scale_log2))) {
            if (fast) fwd5_to_exact(o, m_i, l_i, sl_exact);
            fast = false;
            fwd_tile2<true, false>(kt, vt, qf, o, m_i, l_i, kv0, qposA, h, r, lane, sl_exact, dr);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int blk = 0; blk < 2; ++blk) {
    const int qp = qposA + 32 * blk;
    if (qp < T) {
      const float inv_l = 1.0f / l_i[blk];
      bf16_t* orow = out + ((int64_t)b * T + qp) * C + hh * D;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = 32 * dt + 8 * g + 4 * h;
          uint2 u;
          u.x = pk2<kFaH>(o[blk][dt][4 * g + 0] * inv_l, o[blk][dt][4 * g + 1] * inv_l);
          u.y = pk2<kFaH>(o[blk][dt][4 * g + 2] * inv_l, o[blk][dt][4 * g + 3] * inv_l);
          *reinterpret_cast<uint2*>(orow + d) = u;
        }
      }
      if (h == 0) lse_out[(int64_t)bh * T + qp] = (m_i[blk] * sl_exact + __log2f(l_i[blk])) * 0.6931471805599453f;
    }
  }
}

// =============================================================================
// backward preprocessing (generic path), one pass over [B, T, C]:
//   delta[b, h, t] = rowsum(dO * O)  (fp32)
// =============================================================================
template <int D>
__global__ __launch_bounds__(256) void flash_bwd_pre_kernel(const bf16_t* __restrict__ o,
                                                           const bf16_t* __restrict__ dout,
                                                           float* __restrict__ delta, int B, int T, int H) {
  constexpr int LPR = D / 8;  // lanes per (b, t, h) row, 8 elements each
  const int C = H * D;
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t row = gid / LPR;  // row = (b*T + t)*H + h  -> contiguous [B, T, C] walk
  const int sub = gid % LPR;
  if (row >= (int64_t)B * T * H) return;
  const int hh = row % H;
  const int64_t bt = row / H;
  const int t = bt % T, b = bt / T;
  const int64_t off = bt * C + hh * D + sub * 8;
  float a[8], g[8];
  load8e<kFaH>(o + off, a);
  load8e<kFaH>(dout + off, g);
  float s = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += a[j] * g[j];
#pragma unroll
  for (int k = LPR / 2; k > 0; k >>= 1) s += __shfl_xor(s, k, 64);
  if (sub == 0) delta[((int64_t)b * H + hh) * T + t] = s;
}

// =============================================================================
// backward dK/dV kernel (generic path): one workgroup = KB keys (KB/32 waves x 32) of
// one (b, h); KB = 256 keys (8 waves) for D = 64, 128 (4 waves) for D = 32 / 128.
// =============================================================================
template <int D>
struct BwdGeo {
  static constexpr int KB = D == 64 ? 256 : 128;
  static constexpr int NW = KB / 32;
};

// P and dS of one 32-query half for this lane's key -> bf16 MFMA fragments (i order).
template <bool MASK, bool DROP>
__device__ __forceinline__ void bwd_probs(const f32x16& sacc, const f32x16& dpacc, const float* lse2_s,
                                          const float* delta_s, int qrow0, int qbase_pos, int kpos, int h,
                                          float scale_log2, const DropArgs& dr, bf16x8 (&pfr)[2],
                                          bf16x8 (&dsfr)[2]) {
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 l4 = *reinterpret_cast<const float4*>(lse2_s + qrow0 + 8 * g + 4 * h);
    const float4 d4 = *reinterpret_cast<const float4*>(delta_s + qrow0 + 8 * g + 4 * h);
    const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
    const float dlv[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 4 * g + e;
      const int q = qbase_pos + 8 * g + 4 * h + e;
      float p = fast_exp2(sacc[i] * scale_log2 - lv[e]);
      if constexpr (MASK) {
        if (kpos > q || q >= dr.T) p = 0.0f;
      }
      float dp = dpacc[i];
      float pd = p;
      if constexpr (DROP) {
        const uint64_t id = ((uint64_t)dr.bh * dr.T + (uint64_t)q) * (uint64_t)dr.T + (uint64_t)kpos;
        const bool keep = nsa_keep(dr.seed, id, dr.thresh);
        pd = keep ? p * dr.scale : 0.0f;
        dp = keep ? dp * dr.scale : 0.0f;
      }
      pfr[i >> 3][i & 7] = fa_elt(pd);
      dsfr[i >> 3][i & 7] = fa_elt(p * (dp - dlv[e]));
    }
  }
}

#define NSA_BWD_STAGE_LOAD(QBI)                                                          \
  _Pragma("unroll") for (int c = 0; c < QCH; ++c) {                                      \
    const int e = tid + NT * c;                                                          \
    const int row = e / CPR, ch = e % CPR;                                               \
    int q = (QBI) * QB + row;                                                            \
    q = q < T ? q : T - 1;                                                               \
    qst[c] = *reinterpret_cast<const uint4*>(qbase + (int64_t)q * row_stride + ch * 8);  \
    dost[c] = *reinterpret_cast<const uint4*>(dobase + (int64_t)q * C + ch * 8);         \
  }                                                                                      \
  {                                                                                      \
    int q = (QBI) * QB + (tid & (QB - 1));                                               \
    q = q < T ? q : T - 1;                                                               \
    lst = lse_bh[q] * kLog2e;                                                            \
    dst = delta_bh[q];                                                                   \
  }
#define NSA_BWD_STAGE_WRITE(BUF)                                                         \
  _Pragma("unroll") for (int c = 0; c < QCH; ++c) {                                      \
    const int e = tid + NT * c;                                                          \
    const int row = e / CPR, ch = e % CPR;                                               \
    *reinterpret_cast<uint4*>(qs_lds + (BUF) * QT_BYTES + swz<D>(row, ch)) = qst[c];     \
    *reinterpret_cast<uint4*>(do_lds + (BUF) * QT_BYTES + swz<D>(row, ch)) = dost[c];    \
  }                                                                                      \
  if (tid < QB) {                                                                        \
    ld_lds[(BUF) * QB + tid] = lst;                                                      \
    ld_lds[2 * QB + (BUF) * QB + tid] = dst;                                             \
  }

// dK / dV only: flash_bwd_dq_kernel forms dQ per query tile (two workgroups per CU).
template <int D, bool DROP>
__global__ __launch_bounds__(BwdGeo<D>::NW * 64, 2) void flash_bwd_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dqkv, int B, int T, int H, float scale, float scale_log2,
    uint32_t drop_thresh, float drop_scale, uint64_t seed) {
  using G = BwdGeo<D>;
  constexpr int QB = 64, KB = G::KB, NT = G::NW * 64;  // QB: queries per staged block (128 measured slower)
  constexpr int CPR = D / 8;
  constexpr int NKS = D / 16;
  constexpr int NDT = D / 32;
  constexpr int QT_BYTES = QB * D * 2;
  constexpr int QCH = QB * CPR / NT;  // 16-byte chunks per thread per Q (or dO) tile
  static_assert(QCH >= 1 && QB * CPR == QCH * NT, "Q tile staging must divide evenly");
  __shared__ __attribute__((aligned(16))) char smem[4 * QT_BYTES + 4 * QB * 4];
  char* const qs_lds = smem;                                               // Q[2]
  char* const do_lds = smem + 2 * QT_BYTES;                                // dO[2]
  float* const ld_lds = reinterpret_cast<float*>(smem + 4 * QT_BYTES);     // lse2[2][QB], delta[2][QB]

  const int C = H * D;
  const int64_t row_stride = 3 * (int64_t)C;
  const int BH = B * H;
  const int kb = blockIdx.x / BH;  // key blocks near 0 see the most queries: launched first
  const int bh = blockIdx.x % BH;
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int k0 = kb * KB;
  const int kw0 = k0 + 32 * w;
  const int kpos = kw0 + r;  // this lane's key (S / dP / dK / dV column)
  const bf16_t* base = qkv + (int64_t)b * T * row_stride;
  const bf16_t* qbase = base + hh * D;
  const bf16_t* kbase = base + C + hh * D;
  const bf16_t* vbase = base + 2 * C + hh * D;
  const bf16_t* dobase = dout + (int64_t)b * T * C + hh * D;
  const float* lse_bh = lse + (int64_t)bh * T;
  const float* delta_bh = delta + (int64_t)bh * T;
  const DropArgs dr{drop_thresh, drop_scale, nsa_seed(seed), bh, T};

  // K^T / V^T fragments for S = Q·K^T and dP = dO·V^T (B operands): K[kpos][16ks+8h..]
  bf16x8 kf[NKS], vf[NKS];
  {
    const int kc = kpos < T ? kpos : T - 1;
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      kf[ks] = as_frag(*reinterpret_cast<const uint4*>(kbase + (int64_t)kc * row_stride + 16 * ks + 8 * h));
      vf[ks] = as_frag(*reinterpret_cast<const uint4*>(vbase + (int64_t)kc * row_stride + 16 * ks + 8 * h));
    }
  }
  f32x16 dk[NDT], dv[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) {
    dk[dt] = f32x16{};
    dv[dt] = f32x16{};
  }

  const int qb_first = k0 / QB;
  const int n_qb = (T + QB - 1) / QB;

  // delta = rowsum(dO * O) comes precomputed (flash_bwd_pre_kernel): forming it while
  // staging re-read O once per key block, inside the loop (measured 1154 -> 1335 us)
  uint4 qst[QCH], dost[QCH];
  float lst, dst;
  NSA_BWD_STAGE_LOAD(qb_first)
  NSA_BWD_STAGE_WRITE(0)
  __syncthreads();

  for (int qb = qb_first; qb < n_qb; ++qb) {
    const int cur = (qb - qb_first) & 1;
    const char* qt = qs_lds + cur * QT_BYTES;
    const char* dot = do_lds + cur * QT_BYTES;
    const float* lse2_s = ld_lds + cur * QB;
    const float* delta_s = ld_lds + 2 * QB + cur * QB;
    // unconditional (clamped) staging keeps qst/dost in registers (see forward)
    { NSA_BWD_STAGE_LOAD(min(qb + 1, n_qb - 1)) }

#pragma unroll
    for (int qs = 0; qs < QB / 32; ++qs) {
      const int qbase_pos = qb * QB + qs * 32;
      // S = Q · K^T  (rows = queries in registers, column = this lane's key)
      f32x16 sacc = f32x16{};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 qa = as_frag(lds_b128(qt, swz<D>(qs * 32 + r, 2 * ks + h)));
        sacc = mfma(qa, kf[ks], sacc);
      }
      f32x16 dpacc = f32x16{};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const bf16x8 da = as_frag(lds_b128(dot, swz<D>(qs * 32 + r, 2 * ks + h)));
        dpacc = mfma(da, vf[ks], dpacc);
      }
      bf16x8 pfr[2], dsfr[2];
      // wave-uniform: some (query, key) pair of this 32 x 32 block is masked / out of range
      if (qbase_pos < kw0 + 31 || qbase_pos + 32 > T)
        bwd_probs<true, DROP>(sacc, dpacc, lse2_s, delta_s, qs * 32, qbase_pos, kpos, h, scale_log2, dr, pfr, dsfr);
      else
        bwd_probs<false, DROP>(sacc, dpacc, lse2_s, delta_s, qs * 32, qbase_pos, kpos, h, scale_log2, dr, pfr,
                               dsfr);
      // dV^T += dO^T · P  and  dK^T += Q^T · dS   (accumulators as B operands)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int r0 = qs * 32 + 16 * s + 4 * h;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) {
          const bf16x8 doa = tr_frag<D>(dot, r0, r0 + 8, 32 * dt, lane);
          dv[dt] = mfma(doa, pfr[s], dv[dt]);
          const bf16x8 qa = tr_frag<D>(qt, r0, r0 + 8, 32 * dt, lane);
          dk[dt] = mfma(qa, dsfr[s], dk[dt]);
        }
      }
    }
    // buffer cur^1 was last read in the previous iteration, which ended in a barrier
    { NSA_BWD_STAGE_WRITE(cur ^ 1) }
    __syncthreads();
  }

  // epilogue: dK = scale * dK^T^T, dV = dV^T^T  -> dqkv[:, :, C + ...] and [2C + ...]
  if (kpos < T) {
    bf16_t* krow = dqkv + ((int64_t)b * T + kpos) * row_stride + C + hh * D;
    bf16_t* vrow = krow + C;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 uk, uv;
        uk.x = pk2<kFaH>(dk[dt][4 * g + 0] * scale, dk[dt][4 * g + 1] * scale);
        uk.y = pk2<kFaH>(dk[dt][4 * g + 2] * scale, dk[dt][4 * g + 3] * scale);
        uv.x = pk2<kFaH>(dv[dt][4 * g + 0], dv[dt][4 * g + 1]);
        uv.y = pk2<kFaH>(dv[dt][4 * g + 2], dv[dt][4 * g + 3]);
        *reinterpret_cast<uint2*>(krow + d) = uk;
        *reinterpret_cast<uint2*>(vrow + d) = uv;
      }
    }
  }
}
#undef NSA_BWD_STAGE_LOAD
#undef NSA_BWD_STAGE_WRITE

// =============================================================================
// dQ kernel (split mode): one workgroup = 4 waves x 32 queries of one (b, h), the
// forward kernel's structure with the LSE known up front (no online max / rescale):
//   S^T  = K · Q^T,  dP^T = V · dO^T     A = K / V rows from LDS, B = Q^T / dO^T registers
//   dS^T = P^T ∘ (dP^T − delta),  P^T = exp2(S^T · scale·log2e − lse·log2e)   (lane = query)
//   dQ^T += K^T · dS^T                  A = K^T by transposed LDS reads, B = dS^T straight
//                                       from the accumulator registers (bf16)
// dQ is written once, in bf16, into dqkv[:, :, 0:C]: no atomics, no fp32 accumulator.
// =============================================================================
template <int D, bool MASK, bool DROP>
__device__ __forceinline__ void dq_tile(const char* kt, const char* vt, const bf16x8 (&qf)[D / 16],
                                        const bf16x8 (&gf)[D / 16], f32x16 (&dq)[D / 32], float lse2, float dlt,
                                        int kv0, int qpos, int h, int r, int lane, float scale_log2,
                                        const DropArgs& dr) {
  constexpr int NKS = D / 16;
  constexpr int NDT = D / 32;
  // one 32-key half at a time: S/dP accumulators and dS fragments of a single half are
  // live at once (register pressure sets this kernel's occupancy)
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    f32x16 st = f32x16{}, pt = f32x16{};
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 kf = as_frag(lds_b128(kt, swz<D>(32 * sb + r, 2 * ks + h)));
      st = mfma(kf, qf[ks], st);
    }
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 vf = as_frag(lds_b128(vt, swz<D>(32 * sb + r, 2 * ks + h)));
      pt = mfma(vf, gf[ks], pt);
    }
    bf16x8 dsf[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kpos = kv0 + 32 * sb + acc_row(i, h);
      float p = fast_exp2(st[i] * scale_log2 - lse2);
      if constexpr (MASK) {
        if (kpos > qpos) p = 0.0f;
      }
      float dp = pt[i];
      if constexpr (DROP) {
        const uint64_t id = ((uint64_t)dr.bh * dr.T + (uint64_t)qpos) * (uint64_t)dr.T + (uint64_t)kpos;
        dp = nsa_keep(dr.seed, id, dr.thresh) ? dp * dr.scale : 0.0f;
      }
      dsf[i >> 3][i & 7] = fa_elt(p * (dp - dlt));
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r0 = 32 * sb + 16 * s + 4 * h;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const bf16x8 kf = tr_frag<D>(kt, r0, r0 + 8, 32 * dt, lane);
        dq[dt] = mfma(kf, dsf[s], dq[dt]);
      }
    }
  }
}

#ifndef NSA_DQK_OCC
#define NSA_DQK_OCC 3  // waves per SIMD (A/B at B120: 2 -> 1312 us, 3 -> 1262 us, 4 spills -> 1452 us)
#endif
template <int D, bool DROP>
__global__ __launch_bounds__(256, NSA_DQK_OCC) void flash_bwd_dq_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ delta, bf16_t* __restrict__ dqkv, int B, int T, int H, float scale,
    float scale_log2, uint32_t drop_thresh, float drop_scale, uint64_t seed, float delta_sign) {
  constexpr int BN = 64;
  constexpr int TILE_BYTES = BN * D * 2;
  constexpr int CPR = D / 8;
  constexpr int CHUNKS_PER_THREAD = BN * CPR / 256;
  constexpr int NKS = D / 16;
  constexpr int NDT = D / 32;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];  // K[2], V[2]

  const int C = H * D;
  const int64_t row_stride = 3 * (int64_t)C;
  const int BH = B * H;
  const int n_qt = (T + 127) / 128;
  const int qt = n_qt - 1 - (int)(blockIdx.x / BH);  // heaviest (longest causal) tiles first
  const int bh = blockIdx.x % BH;
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int q0 = qt * 128;
  const int q0w = q0 + 32 * w;
  const int qpos = q0w + r;
  const bf16_t* base = qkv + (int64_t)b * T * row_stride;
  const bf16_t* kbase = base + C + hh * D;
  const bf16_t* vbase = base + 2 * C + hh * D;
  const DropArgs dr{drop_thresh, drop_scale, nsa_seed(seed), bh, T};

  // Q^T and dO^T fragments (B operands): lane holds row qpos, d = 16ks + 8h .. +8
  bf16x8 qf[NKS], gf[NKS];
  const int qc = qpos < T ? qpos : T - 1;
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    qf[ks] = as_frag(*reinterpret_cast<const uint4*>(base + (int64_t)qc * row_stride + hh * D + 16 * ks + 8 * h));
    gf[ks] = as_frag(*reinterpret_cast<const uint4*>(dout + ((int64_t)b * T + qc) * C + hh * D + 16 * ks + 8 * h));
  }
  const float lse2 = lse[(int64_t)bh * T + qc] * kLog2e;
  const float dlt = delta_sign * delta[(int64_t)bh * T + qc];  // v2 workspaces hold -delta

  f32x16 dq[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) dq[dt] = f32x16{};

  const int kv_end = min(T, q0 + 128);
  const int n_tiles = (kv_end + BN - 1) / BN;

  uint4 kst[CHUNKS_PER_THREAD], vst[CHUNKS_PER_THREAD];
#define NSA_DQ_STAGE_LOAD(J)                                                                    \
  _Pragma("unroll") for (int c = 0; c < CHUNKS_PER_THREAD; ++c) {                               \
    const int e = tid + 256 * c;                                                                \
    const int row = e / CPR, ch = e % CPR;                                                      \
    int key = (J) * BN + row;                                                                   \
    key = key < T ? key : T - 1;                                                                \
    kst[c] = *reinterpret_cast<const uint4*>(kbase + (int64_t)key * row_stride + ch * 8);       \
    vst[c] = *reinterpret_cast<const uint4*>(vbase + (int64_t)key * row_stride + ch * 8);       \
  }
#define NSA_DQ_STAGE_WRITE(BUF)                                                                 \
  _Pragma("unroll") for (int c = 0; c < CHUNKS_PER_THREAD; ++c) {                               \
    const int e = tid + 256 * c;                                                                \
    const int row = e / CPR, ch = e % CPR;                                                      \
    *reinterpret_cast<uint4*>(smem + (BUF) * TILE_BYTES + swz<D>(row, ch)) = kst[c];            \
    *reinterpret_cast<uint4*>(smem + (2 + (BUF)) * TILE_BYTES + swz<D>(row, ch)) = vst[c];      \
  }
  NSA_DQ_STAGE_LOAD(0)
  NSA_DQ_STAGE_WRITE(0)
  __syncthreads();

  for (int j = 0; j < n_tiles; ++j) {
    const int cur = j & 1;
    const int kv0 = j * BN;
    { NSA_DQ_STAGE_LOAD(min(j + 1, n_tiles - 1)) }
    const char* kt = smem + cur * TILE_BYTES;
    const char* vt = smem + (2 + cur) * TILE_BYTES;
    if (kv0 + BN - 1 <= q0w)  // wave-uniform: whole tile visible to every query of the wave
      dq_tile<D, false, DROP>(kt, vt, qf, gf, dq, lse2, dlt, kv0, qpos, h, r, lane, scale_log2, dr);
    else if (kv0 <= q0w + 31)  // the wave's diagonal tile
      dq_tile<D, true, DROP>(kt, vt, qf, gf, dq, lse2, dlt, kv0, qpos, h, r, lane, scale_log2, dr);
    { NSA_DQ_STAGE_WRITE(cur ^ 1) }
    __syncthreads();
  }
#undef NSA_DQ_STAGE_LOAD
#undef NSA_DQ_STAGE_WRITE

  // epilogue: dQ = scale · dQ^T^T -> dqkv[b, qpos, hh*D + d]; lane owns query qpos
  if (qpos < T) {
    bf16_t* qrow = dqkv + ((int64_t)b * T + qpos) * row_stride + hh * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 u;
        u.x = pk2<kFaH>(dq[dt][4 * g + 0] * scale, dq[dt][4 * g + 1] * scale);
        u.y = pk2<kFaH>(dq[dt][4 * g + 2] * scale, dq[dt][4 * g + 3] * scale);
        *reinterpret_cast<uint2*>(qrow + d) = u;
      }
    }
  }
}

// =============================================================================
// Backward v2 (D = 64, the GPT-2 head size): dK/dV kernel, templated on
//   NKB = 32-key blocks per wave (1 or 2) and NW = waves per workgroup (4 or 8).
//
// Wave w owns keys kw = k0 + 32*NKB*w as NKB 32-key blocks whose dK^T / dV^T
// accumulators stay resident while the workgroup sweeps 32-query slices.  With
// NKB = 2 each slice's Q / dO row fragments (ds_read_b128) and Q^T / dO^T transposed
// fragments (ds_read_b64_tr_b16) feed both key blocks (24 LDS reads per 32 MFMAs).
//
// Query slices (Q and dO [32][64] tiles, XOR-swizzled as swz<64>, plus a per-wave
// copy of the slice's row constants) arrive by LDS-DMA into a 2-slot ring, one
// slice ahead: slice j+1 is issued right after the barrier that opens slice j, into
// the slot slice j-1 used (every wave retired its reads of it -- lgkmcnt(0) -- before
// that barrier).  Each wave waits only for its own pieces of slice j with vmcnt(0)
// before the barrier (slice j+1 is not yet issued then); raw s_barrier (a
// __syncthreads would add a fence).  The slice loop is unrolled by the ring parity,
// so every LDS address is a per-lane base + an immediate offset.
//
// Row constants come in as the accumulators' initial values (cdna_hip_programming.md
// App. B "row constants as the initial accumulator"): S' = Q·K^T - lse/scale and
// dP' = dO·V^T - delta leave the MFMA chains ready, so P = exp2(c·S') and
// dS = P·dP' cost one multiply each.  P and dS are packed to bf16 pairwise
// (one v_cvt_pk_bf16_f32 per two elements).
// =============================================================================
constexpr int V2_QT = 32 * 64 * 2;  // one [32][64] bf16 tile

template <int NW>
struct V2Geo {
  static constexpr int SLOT = 2 * V2_QT + NW * 256;  // Q, dO, NW x (32 -lse/scale + 32 -delta)
  static constexpr int PIECES = NW == 4 ? 3 : 2;     // LDS-DMA instructions per wave per slice
};

__device__ __forceinline__ void glds4(const void* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// two f32 -> one dword of two bf16 (v_cvt_pk_bf16_f32, RNE)
__device__ __forceinline__ uint32_t cvt2(float a, float b) { return pk2<kFaH>(a, b); }

// 16 accumulator values -> the two bf16x8 operand fragments (k-steps 0 and 1)
__device__ __forceinline__ void pack16(const float (&v)[16], bf16x8 (&f)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    uint4 u;
    u.x = cvt2(v[8 * s + 0], v[8 * s + 1]);
    u.y = cvt2(v[8 * s + 2], v[8 * s + 3]);
    u.z = cvt2(v[8 * s + 4], v[8 * s + 5]);
    u.w = cvt2(v[8 * s + 6], v[8 * s + 7]);
    f[s] = __builtin_bit_cast(bf16x8, u);
  }
}

// f32x16 of a per-query row constant for this lane's accumulator rows acc_row(i, h)
__device__ __forceinline__ f32x16 row_consts(const float* v, int h) {
  f32x16 a;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const float4 x = *reinterpret_cast<const float4*>(v + 8 * g + 4 * h);
    a[4 * g + 0] = x.x;
    a[4 * g + 1] = x.y;
    a[4 * g + 2] = x.z;
    a[4 * g + 3] = x.w;
  }
  return a;
}

// Ring-slot dispatch: calls f(std::integral_constant<int, k>) for k = j % NS, so the
// slot's LDS offsets are compile-time (immediates) inside every branch-free body.
template <int K, int NS, typename F>
__device__ __forceinline__ void slot_dispatch(int k, F& f) {
  if constexpr (K + 1 < NS) {
    if (k == K)
      f(std::integral_constant<int, K>{});
    else
      slot_dispatch<K + 1, NS>(k, f);
  } else {
    f(std::integral_constant<int, K>{});
  }
}


// one 32-query slice for one wave: S, dP for its NKB key blocks, P / dS, then dV^T, dK^T.
// ld = this wave's copy of the slice's row constants: [0, 32) -lse/scale, [32, 64) -delta.
template <int NKB, bool MASK, bool DROP>
__device__ __forceinline__ void dkdv_slice(const char* qt, const char* dot, const float* ld,
                                           const bf16x8 (&kf)[NKB][4], const bf16x8 (&vf)[NKB][4],
                                           f32x16 (&dk)[NKB][2], f32x16 (&dv)[NKB][2], int q0, int kw, int h,
                                           int r, int lane, float scale_log2, const DropArgs& dr) {
  constexpr int D = 64;
  bf16x8 qa[4], da[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qa[ks] = as_frag(lds_b128(qt, swz<D>(r, 2 * ks + h)));
    da[ks] = as_frag(lds_b128(dot, swz<D>(r, 2 * ks + h)));
  }
  f32x16 sacc[NKB], pacc[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    sacc[kb] = row_consts(ld, h);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) sacc[kb] = mfma(qa[ks], kf[kb][ks], sacc[kb]);
  }
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    pacc[kb] = DROP ? f32x16{} : row_consts(ld + 32, h);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) pacc[kb] = mfma(da[ks], vf[kb][ks], pacc[kb]);
  }
  bf16x8 pfr[NKB][2], dsfr[NKB][2];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    const int key = kw + 32 * kb + r;
    f32x16 nd;
    if constexpr (DROP) nd = row_consts(ld + 32, h);
    float pv[16], dsv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float p = fast_exp2(sacc[kb][i] * scale_log2);
      if constexpr (MASK) p = key > q0 + acc_row(i, h) ? 0.0f : p;
      if constexpr (DROP) {
        const int q = q0 + acc_row(i, h);
        const uint64_t id = ((uint64_t)dr.bh * dr.T + (uint64_t)q) * (uint64_t)dr.T + (uint64_t)key;
        const bool keep = nsa_keep(dr.seed, id, dr.thresh);
        pv[i] = keep ? p * dr.scale : 0.0f;
        dsv[i] = p * ((keep ? pacc[kb][i] * dr.scale : 0.0f) + nd[i]);
      } else {
        pv[i] = p;
        dsv[i] = p * pacc[kb][i];
      }
    }
    pack16(pv, pfr[kb]);
    pack16(dsv, dsfr[kb]);
  }
  // dV^T += dO^T · P,  dK^T += Q^T · dS   (each transposed fragment feeds every key block)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int r0 = 16 * s + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      const bf16x8 doa = tr_frag<D>(dot, r0, r0 + 8, 32 * dt, lane);
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) dv[kb][dt] = mfma(doa, pfr[kb][s], dv[kb][dt]);
      const bf16x8 qta = tr_frag<D>(qt, r0, r0 + 8, 32 * dt, lane);
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) dk[kb][dt] = mfma(qta, dsfr[kb][s], dk[kb][dt]);
    }
  }
}

#ifndef NSA_DKDV_NS
#define NSA_DKDV_NS 4  // LDS ring slots of the v2 dK/dV kernel (NS - 1 slices in flight)
#endif

template <int NKB, int NW, bool DROP, int G = 1>
__global__ __launch_bounds__(NW * 64, NKB == 2 ? 1 : (NW == 8 ? 1 : 2)) void flash_bwd_dkdv2_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const float* __restrict__ nls,
    const float* __restrict__ nd, bf16_t* __restrict__ dqkv, int B, int T, int H, float scale,
    float scale_log2, uint32_t drop_thresh, float drop_scale, uint64_t seed, int order) {
  constexpr int D = 64;
  constexpr int KPW = 32 * NKB;       // keys per wave
  constexpr int KWG = KPW * NW;       // keys per workgroup
  constexpr int SLOT = V2Geo<NW>::SLOT;
  // G > 1: G slices per barrier in a 2G-slot ring (G computed while the next G land)
  constexpr int NS = G > 1 ? 2 * G : NSA_DKDV_NS, LA = NS - 1;
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int C = H * D;
  const int64_t row_stride = 3 * (int64_t)C;
  const int BH = B * H;
  int bh, kbw;  // key blocks near 0 see the most queries: launched first
  attn_order((T + KWG - 1) / KWG, BH, order, bh, kbw);
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int k0 = kbw * KWG;
  const int kw = k0 + KPW * w;
  const bf16_t* base = qkv + (int64_t)b * T * row_stride;
  const bf16_t* qbase = base + hh * D;
  const bf16_t* kbase = base + C + hh * D;
  const bf16_t* vbase = base + 2 * C + hh * D;
  const bf16_t* dobase = dout + (int64_t)b * T * C + hh * D;
  const float* nls_bh = nls + (int64_t)bh * T;
  const float* nd_bh = nd + (int64_t)bh * T;
  const DropArgs dr{drop_thresh, drop_scale, nsa_seed(seed), bh, T};
  const uint32_t lds0 =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  const int s_first = k0 / 32;
  const int n_mine = T / 32 - s_first;  // query slices this workgroup visits

  // slice s -> ring slot: the [32][64] Q and dO tiles are 4 + 4 pieces of 8 rows x 128 B
  // (with 4 waves each wave copies one of each, with 8 waves one of the two); the
  // swz<64> image is lane-linear, so the XOR goes on the per-lane source chunk.  Each
  // wave also copies the slice's row constants for itself: lanes 0-31 -lse/scale,
  // 32-63 -delta.
  const int piece = NW == 4 ? w : (w & 3);
  const int prow = 8 * piece + (lane >> 3);
  const int pch = (lane & 7) ^ bitrev<3>((prow >> 1) & 7);
  const bf16_t* qsrc = qbase + (int64_t)prow * row_stride + pch * 8;  // + slice * 32 rows
  const bf16_t* dosrc = dobase + (int64_t)prow * C + pch * 8;
  const float* csrc = (h == 0 ? nls_bh : nd_bh) + r;
  auto issue = [&](int s, int slot) {
    const uint32_t sb = lds0 + (uint32_t)(slot * SLOT);
    if (NW == 4 || w < 4) glds16(qsrc + (int64_t)s * 32 * row_stride, sb + (uint32_t)(8 * piece * 128));
    if (NW == 4 || w >= 4) glds16(dosrc + (int64_t)s * 32 * C, sb + (uint32_t)(V2_QT + 8 * piece * 128));
    glds4(csrc + s * 32, sb + (uint32_t)(2 * V2_QT + w * 256));
  };

  for (int j = 0; j < (G > 1 ? G : LA) && j < n_mine; ++j) issue(s_first + j, j);

  // K^T / V^T fragments (B operands of S = Q·K^T, dP = dO·V^T): K[key][16ks + 8h ..]
  bf16x8 kf[NKB][4], vf[NKB][4];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    int kc = kw + 32 * kb + r;
    kc = kc < T ? kc : T - 1;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      kf[kb][ks] = as_frag(*reinterpret_cast<const uint4*>(kbase + (int64_t)kc * row_stride + 16 * ks + 8 * h));
      vf[kb][ks] = as_frag(*reinterpret_cast<const uint4*>(vbase + (int64_t)kc * row_stride + 16 * ks + 8 * h));
    }
  }
  // Retire the fragment loads HERE, in hipcc's own bookkeeping: an asm use of every
  // fragment makes it wait for them now.  Otherwise its wait for a fragment's first
  // use lands inside the slice loop and (blind to the asm LDS-DMA) drains the ring's
  // in-flight slice with vmcnt(0) every iteration.
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
    asm volatile("" ::"v"(kf[kb][0]), "v"(kf[kb][1]), "v"(kf[kb][2]), "v"(kf[kb][3]), "v"(vf[kb][0]),
                 "v"(vf[kb][1]), "v"(vf[kb][2]), "v"(vf[kb][3]));
  f32x16 dk[NKB][2], dv[NKB][2];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
      dk[kb][dt] = f32x16{};
      dv[kb][dt] = f32x16{};
    }

  // Open slice j (ring slot j % NS): this wave's pieces of it have landed (slices
  // j+1 .. j+LA-1 may stay in flight) and its LDS reads of slice j-1 are retired; the
  // barrier makes every wave's pieces visible and frees slice j-1's slot for slice j+LA.
  auto open_slice = [&](int j) {
    vm_wait(V2Geo<NW>::PIECES * min(LA - 1, n_mine - 1 - j));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (j + LA < n_mine) issue(s_first + j + LA, (j + LA) % NS);
  };
  auto slice_full = [&](int j) {
    auto f = [&](auto slot) {
      const char* qt = smem + decltype(slot)::value * SLOT;
      dkdv_slice<NKB, false, DROP>(qt, qt + V2_QT, reinterpret_cast<const float*>(qt + 2 * V2_QT) + w * 64, kf,
                                   vf, dk, dv, (s_first + j) * 32, kw, h, r, lane, scale_log2, dr);
    };
    slot_dispatch<0, NS>(j % NS, f);
  };
  auto slice_diag = [&](int j) {
    auto f = [&](auto slot) {
      const char* qt = smem + decltype(slot)::value * SLOT;
      dkdv_slice<NKB, true, DROP>(qt, qt + V2_QT, reinterpret_cast<const float*>(qt + 2 * V2_QT) + w * 64, kf,
                                  vf, dk, dv, (s_first + j) * 32, kw, h, r, lane, scale_log2, dr);
    };
    slot_dispatch<0, NS>(j % NS, f);
  };

  // Three loops with branch-free bodies: slices wholly before this wave's keys (no
  // work), the slices on its diagonal (masked), the rest.  Every wave runs n_mine
  // iterations in all: same barrier count.
  const int j_diag = min(NKB * w, n_mine);
  const int j_full = min(NKB * w + NKB, n_mine);
  if constexpr (G > 1) {
    // G slices per barrier: group (j .. j + G - 1) runs while slices j + G .. j + 2G - 1 fly
    // into the slots of the previous group (freed by the barrier that opens this one)
    for (int j = 0; j < n_mine; j += G) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#pragma unroll
      for (int u = 0; u < G; ++u)
        if (j + G + u < n_mine) issue(s_first + j + G + u, (j + G + u) % NS);
#pragma unroll
      for (int u = 0; u < G; ++u) {
        const int jj = j + u;
        if (jj >= j_full) {
          if (jj < n_mine) slice_full(jj);
        } else if (jj >= j_diag) {
          slice_diag(jj);
        }
      }
    }
  } else {
    int j = 0;
    for (; j < j_diag; ++j) open_slice(j);
    for (; j < j_full; ++j) {
      open_slice(j);
      slice_diag(j);
    }
    for (; j < n_mine; ++j) {
      open_slice(j);
      slice_full(j);
    }
  }

  // epilogue: dK = scale * (dK^T)^T, dV = (dV^T)^T -> dqkv[:, :, C + ...] and [2C + ...]
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    const int kpos = kw + 32 * kb + r;
    if (kpos < T) {
      bf16_t* krow = dqkv + ((int64_t)b * T + kpos) * row_stride + C + hh * D;
      bf16_t* vrow = krow + C;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int d = 32 * dt + 8 * g + 4 * h;
          uint2 uk, uv;
          uk.x = cvt2(dk[kb][dt][4 * g + 0] * scale, dk[kb][dt][4 * g + 1] * scale);
          uk.y = cvt2(dk[kb][dt][4 * g + 2] * scale, dk[kb][dt][4 * g + 3] * scale);
          uv.x = cvt2(dv[kb][dt][4 * g + 0], dv[kb][dt][4 * g + 1]);
          uv.y = cvt2(dv[kb][dt][4 * g + 2], dv[kb][dt][4 * g + 3]);
          *reinterpret_cast<uint2*>(krow + d) = uk;
          *reinterpret_cast<uint2*>(vrow + d) = uv;
        }
      }
    }
  }
}

// =============================================================================
// dQ kernel v2 (D = 64): one workgroup = 4 waves x 32 queries of one (b, h), the
// query on the lane (swapped products, as the forward):
//   S^T  = K · Q^T,  dP^T = V · dO^T     A = K / V rows (ds_read_b128), B = Q^T / dO^T
//                                        fragments held in registers for the whole loop
//   dS^T = P^T · dP'^T,  P^T = exp2(c·S^T - lse·log2e),  dP'^T = dP^T - delta
//   dQ^T += K^T · dS^T                   A = K^T (ds_read_b64_tr_b16), B = dS^T packed
//                                        straight from the accumulator registers
// lse·log2e and delta are per-lane scalars here; -delta enters as a constant
// initial-accumulator tile (C operand), so dS costs one multiply per element and P
// is never converted to bf16 (only dS feeds an MFMA).  64-key K / V tiles arrive by
// LDS-DMA into a 2-slot ring one tile ahead (4 pieces per wave per tile); the tile
// loop is unrolled by ring parity (immediate LDS offsets) and split into branch-free
// loops: fully visible tiles, the wave's one diagonal tile, trailing tiles past it.
// dQ is written once, in bf16: no atomics, no fp32 accumulator.
// =============================================================================
constexpr int DQ2_T = 64 * 64 * 2;  // one [64][64] bf16 tile
#ifndef NSA_DQ2_NS
#define NSA_DQ2_NS 4  // LDS ring slots of the v2 dQ kernel (NS - 1 tiles in flight)
#endif
#ifndef NSA_DQ2_OCC
#define NSA_DQ2_OCC 2  // waves per SIMD the v2 dQ kernel is compiled for
#endif

template <bool MASK, bool DROP>
__device__ __forceinline__ void dq2_tile(const char* kt, const char* vt, const bf16x8 (&qf)[4],
                                         const bf16x8 (&gf)[4], const f32x16& ndt, f32x16 (&dq)[2], float lse2,
                                         int kv0, int qpos, int h, int r, int lane, float scale_log2,
                                         const DropArgs& dr) {
  constexpr int D = 64;
  f32x16 st[2], pt[2];
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    st[sb] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) st[sb] = mfma(as_frag(lds_b128(kt, swz<D>(32 * sb + r, 2 * ks + h))), qf[ks], st[sb]);
  }
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    pt[sb] = DROP ? f32x16{} : ndt;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) pt[sb] = mfma(as_frag(lds_b128(vt, swz<D>(32 * sb + r, 2 * ks + h))), gf[ks], pt[sb]);
  }
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    float dsv[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kpos = kv0 + 32 * sb + acc_row(i, h);
      float p = fast_exp2(st[sb][i] * scale_log2 - lse2);
      if constexpr (MASK) p = kpos > qpos ? 0.0f : p;
      if constexpr (DROP) {
        const uint64_t id = ((uint64_t)dr.bh * dr.T + (uint64_t)qpos) * (uint64_t)dr.T + (uint64_t)kpos;
        dsv[i] = p * ((nsa_keep(dr.seed, id, dr.thresh) ? pt[sb][i] * dr.scale : 0.0f) + ndt[i]);
      } else {
        dsv[i] = p * pt[sb][i];
      }
    }
    bf16x8 dsf[2];
    pack16(dsv, dsf);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int r0 = 32 * sb + 16 * s + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 2; ++dt) dq[dt] = mfma(tr_frag<D>(kt, r0, r0 + 8, 32 * dt, lane), dsf[s], dq[dt]);
    }
  }
}


template <bool DROP>
__global__ __launch_bounds__(256, NSA_DQ2_OCC) void flash_bwd_dq2_kernel(
    const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ dout, const bf16_t* __restrict__ o,
    const float* __restrict__ lse, float* __restrict__ nls, float* __restrict__ nd, bf16_t* __restrict__ dqkv, int B,
    int T, int H, float scale, float scale_log2, uint32_t drop_thresh, float drop_scale, uint64_t seed, int order) {
  constexpr int D = 64;
  constexpr int SLOT = 2 * DQ2_T;  // K, V
  constexpr int NS = NSA_DQ2_NS, LA = NS - 1;
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];
  const int C = H * D;
  const int64_t row_stride = 3 * (int64_t)C;
  const int BH = B * H;
  const int n_qt = (T + 127) / 128;
  int bh, qt;
  attn_order(n_qt, BH, order, bh, qt);
  qt = n_qt - 1 - qt;  // heaviest (longest causal) tiles first
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int q0w = qt * 128 + 32 * w;
  const int qpos = q0w + r;
  const int qc = qpos < T ? qpos : T - 1;
  const bf16_t* base = qkv + (int64_t)b * T * row_stride;
  const DropArgs dr{drop_thresh, drop_scale, nsa_seed(seed), bh, T};
  const uint32_t lds0 =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  // K / V tile j -> ring slot: 8 + 8 pieces of 8 rows x 128 B, wave w copies K rows and
  // V rows 16w .. 16w+15 (two pieces each), XOR swizzle on the per-lane source chunk
  const int prow = 16 * w + (lane >> 3);
  const int pch0 = (lane & 7) ^ bitrev<3>((prow >> 1) & 7);        // piece 0: row prow
  const int pch1 = (lane & 7) ^ bitrev<3>(((prow + 8) >> 1) & 7);  // piece 1: row prow + 8
  const bf16_t* krow = base + C + hh * D + (int64_t)prow * row_stride;
  const int kv_end = min(T, qt * 128 + 128);
  const int n_tiles = (kv_end + 63) / 64;
  auto issue = [&](int j, int slot) {
    const uint32_t sb = lds0 + (uint32_t)(slot * SLOT) + (uint32_t)(16 * w * 128);
    const int64_t o = (int64_t)j * 64 * row_stride;
    int64_t o0 = 0, o8 = 8 * row_stride;
    if (j * 64 + 64 > T) {  // last, partial tile: rows past T re-read row T-1 (their keys are masked)
      const int k = j * 64 + prow;
      o0 = (int64_t)(min(k, T - 1) - k) * row_stride;
      o8 = (int64_t)(min(k + 8, T - 1) - k) * row_stride;
    }
    const bf16_t* k0 = krow + o + o0 + pch0 * 8;
    const bf16_t* k8 = krow + o + o8 + pch1 * 8;
    glds16(k0, sb);
    glds16(k8, sb + 1024);
    glds16(k0 + C, sb + DQ2_T);
    glds16(k8 + C, sb + DQ2_T + 1024);
  };
  for (int j = 0; j < LA && j < n_tiles; ++j) issue(j, j);

  // Q^T and dO^T fragments (B operands): lane holds row qpos, d = 16ks + 8h .. +8
  bf16x8 qf[4], gf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = as_frag(*reinterpret_cast<const uint4*>(base + (int64_t)qc * row_stride + hh * D + 16 * ks + 8 * h));
    gf[ks] = as_frag(*reinterpret_cast<const uint4*>(dout + ((int64_t)b * T + qc) * C + hh * D + 16 * ks + 8 * h));
  }
  // lse·log2e = -nls·c (nls = -lse/scale), and the -delta tile
  // this kernel runs first and forms the row constants itself: delta = rowsum(dO * O)
  // from the dO fragments it holds anyway plus the matching O pieces (the two lane
  // halves hold d = 8h + 16ks .. +8), written out for the dK/dV kernel as -delta and
  // -lse/scale (no separate preprocessing pass over O and dO)
  float dpart = 0.0f;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    float fo[8], fg[8];
    load8e<kFaH>(o + ((int64_t)b * T + qc) * C + hh * D + 16 * ks + 8 * h, fo);
    unpack8e<kFaH>(__builtin_bit_cast(uint4, gf[ks]), fg);
#pragma unroll
    for (int e = 0; e < 8; ++e) dpart += fo[e] * fg[e];
  }
  const float ndl = -half_swap_sum(dpart);
  const float lse_q = lse[(int64_t)bh * T + qc];
  const float lse2 = lse_q * kLog2e;
  if (h == 0 && qpos < T) {
    nd[(int64_t)bh * T + qpos] = ndl;
    nls[(int64_t)bh * T + qpos] = -lse_q / scale;
  }
  asm volatile("" ::"v"(qf[0]), "v"(qf[1]), "v"(qf[2]), "v"(qf[3]), "v"(gf[0]), "v"(gf[1]), "v"(gf[2]),
               "v"(gf[3]), "v"(lse2), "v"(ndl));  // retire these loads before the ring loop (see dK/dV)
  f32x16 ndt;
#pragma unroll
  for (int i = 0; i < 16; ++i) ndt[i] = ndl;
  f32x16 dq[2];
  dq[0] = f32x16{};
  dq[1] = f32x16{};

  auto open_tile = [&](int j) {
    vm_wait(4 * min(LA - 1, n_tiles - 1 - j));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (j + LA < n_tiles) issue(j + LA, (j + LA) % NS);
  };
  auto tile_full = [&](int j) {
    auto f = [&](auto slot) {
      const char* kt = smem + decltype(slot)::value * SLOT;
      dq2_tile<false, DROP>(kt, kt + DQ2_T, qf, gf, ndt, dq, lse2, 64 * j, qpos, h, r, lane, scale_log2, dr);
    };
    slot_dispatch<0, NS>(j % NS, f);
  };
  auto tile_diag = [&](int j) {
    auto f = [&](auto slot) {
      const char* kt = smem + decltype(slot)::value * SLOT;
      dq2_tile<true, DROP>(kt, kt + DQ2_T, qf, gf, ndt, dq, lse2, 64 * j, qpos, h, r, lane, scale_log2, dr);
    };
    slot_dispatch<0, NS>(j % NS, f);
  };

  // tiles [0, m) are visible to every query of the wave; tile m holds its diagonal;
  // later tiles (at most one) are all masked
  const int m = min(q0w / 64, n_tiles);
  int j = 0;
  for (; j < m; ++j) {
    open_tile(j);
    tile_full(j);
  }
  if (j < n_tiles) {
    open_tile(j);
    tile_diag(j);
    ++j;
  }
  for (; j < n_tiles; ++j) open_tile(j);

  // epilogue: dQ = scale · (dQ^T)^T -> dqkv[b, qpos, hh*D + d]; lane owns query qpos
  if (qpos < T) {
    bf16_t* qrow = dqkv + ((int64_t)b * T + qpos) * row_stride + hh * D;
#pragma unroll
    for (int dt = 0; dt < 2; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = 32 * dt + 8 * g + 4 * h;
        uint2 u;
        u.x = cvt2(dq[dt][4 * g + 0] * scale, dq[dt][4 * g + 1] * scale);
        u.y = cvt2(dq[dt][4 * g + 2] * scale, dq[dt][4 * g + 3] * scale);
        *reinterpret_cast<uint2*>(qrow + d) = u;
      }
    }
  }
}

template <int D>
hipError_t fwd_launch(const void* qkv, void* out, void* lse, int B, int T, int H, float scale, float p,
                      uint64_t seed, hipStream_t s) {
  const int n_qt = (T + 127) / 128;
  const uint32_t th = p > 0.0f ? nsa_drop_thresh(p) : 0u;
  const float dscale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const int order = attn_order_env();
  if constexpr (D == 64) {
    // v5 (64 queries per wave as two 32-query blocks, 4-slot K/V ring, two tiles per barrier,
    // no running max while the scores stay in range) by default without dropout once the grid
    // has >= 4096 workgroups: B120 T1024 H12 (5760 workgroups) 333 us vs v1's 377 -- v5 halves
    // the K/V re-reads, which pays once qkv (566 MB) no longer sits in the 256 MB Infinity
    // Cache (B60: v1 159 vs the 64-query form's 188 us); with dropout v1 (the per-element hash
    // doubles the 64-query chain: 109 vs 158 us at B16).  fp16 runs v5 with the fast tiles'
    // row sums bounded to [2^-8, 2^15] (P <= 65504).  Round 6 removed the variants that lost
    // their A/Bs: v3 / v4 (v5's geometry with exact tiles; v4 338.1 vs v5 333.3 us,
    // profiles/r5_ab_fwd45.log), v6 (v1's geometry with fast tiles, 375.4 vs 343.5,
    // profiles/r5_ab_v6.log) and a one-wave-per-SIMD pipelined v7 (556 vs 341 us,
    // docs/performance.md round 6).
    const int n_qt5 = (T + 255) / 256;
    const int sel = flash_config().fwd;
    if (!th && (sel == FWD_V5 || (sel == FWD_AUTO && (int64_t)n_qt5 * B * H >= 4096))) {
      flash_fwd5_kernel<<<n_qt5 * B * H, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)out, (float*)lse, B, T, H,
                                                      scale * kLog2e, order);
      return hipGetLastError();
    }
    // v1 with LDS-DMA K/V staging
    if (th)
      flash_fwd_kernel<D, true, true><<<n_qt * B * H, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)out, (float*)lse, B,
                                                                   T, H, scale * kLog2e, th, dscale, seed, order);
    else
      flash_fwd_kernel<D, false, true><<<n_qt * B * H, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)out, (float*)lse,
                                                                    B, T, H, scale * kLog2e, th, dscale, seed, order);
    return hipGetLastError();
  }
  // D = 32 / 128: register-staged v1
  if (th)
    flash_fwd_kernel<D, true><<<n_qt * B * H, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)out, (float*)lse, B, T, H,
                                                           scale * kLog2e, th, dscale, seed, order);
  else
    flash_fwd_kernel<D, false><<<n_qt * B * H, 256, 0, s>>>((const bf16_t*)qkv, (bf16_t*)out, (float*)lse, B, T, H,
                                                            scale * kLog2e, th, dscale, seed, order);
  return hipGetLastError();
}

// generic backward (any D, any T): delta pre-pass -> dK/dV kernel -> dQ kernel.
// ws[0] = delta [B, H, T].
template <int D>
hipError_t bwd_launch(const void* qkv, const void* o, const void* dout, const void* lse, void* delta, void* dqkv,
                      int B, int T, int H, float scale, float p, uint64_t seed, hipStream_t s) {
  const int64_t threads = (int64_t)B * T * H * (D / 8);
  flash_bwd_pre_kernel<D><<<(unsigned)((threads + 255) / 256), 256, 0, s>>>((const bf16_t*)o, (const bf16_t*)dout,
                                                                             (float*)delta, B, T, H);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint32_t th = p > 0.0f ? nsa_drop_thresh(p) : 0u;
  const float dscale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const int n_kb = (T + BwdGeo<D>::KB - 1) / BwdGeo<D>::KB;
  const dim3 grid(n_kb * B * H), block(BwdGeo<D>::NW * 64);
#define NSA_BWD_ARGS                                                                                        \
  (const bf16_t*)qkv, (const bf16_t*)dout, (const float*)lse, (const float*)delta, (bf16_t*)dqkv, B, T, H, \
      scale, scale * kLog2e, th, dscale, seed
  if (th) flash_bwd_kernel<D, true><<<grid, block, 0, s>>>(NSA_BWD_ARGS);
  else flash_bwd_kernel<D, false><<<grid, block, 0, s>>>(NSA_BWD_ARGS);
#undef NSA_BWD_ARGS
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int n_qt = (T + 127) / 128;
  if (th)
    flash_bwd_dq_kernel<D, true><<<n_qt * B * H, 256, 0, s>>>(
        (const bf16_t*)qkv, (const bf16_t*)dout, (const float*)lse, (const float*)delta, (bf16_t*)dqkv, B, T, H,
        scale, scale * kLog2e, th, dscale, seed, 1.0f);
  else
    flash_bwd_dq_kernel<D, false><<<n_qt * B * H, 256, 0, s>>>(
        (const bf16_t*)qkv, (const bf16_t*)dout, (const float*)lse, (const float*)delta, (bf16_t*)dqkv, B, T, H,
        scale, scale * kLog2e, th, dscale, seed, 1.0f);
  return hipGetLastError();
}

// v2 backward (D = 64, T % 32 == 0): the dQ v2 kernel (which also forms the row
// constants -delta, -lse/scale) -> the dK/dV v2 kernel, 1 key block per wave, 4 waves
// (two independent workgroups per CU).  ws = 2 x [B, H, T] fp32.  A/B at B120 T1024 H12
// (whole backward): v1 1307, 2 key blocks per wave 1304, 8 waves 1203, this 1189 us.
hipError_t bwd2_launch64(const void* qkv, const void* o, const void* dout, const void* lse, void* ws, void* dqkv,
                         int B, int T, int H, float scale, float p, uint64_t seed, hipStream_t s) {
  float* nd = (float*)ws;
  float* nls = nd + (int64_t)B * H * T;
  const uint32_t th = p > 0.0f ? nsa_drop_thresh(p) : 0u;
  const float dscale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const int n_qt = (T + 127) / 128;
  const int order = attn_order_env();
  if (th)
    flash_bwd_dq2_kernel<true><<<n_qt * B * H, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)dout,
                                                            (const bf16_t*)o, (const float*)lse, nls, nd, (bf16_t*)dqkv,
                                                            B, T, H, scale, scale * kLog2e, th, dscale, seed, order);
  else
    flash_bwd_dq2_kernel<false><<<n_qt * B * H, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)dout,
                                                             (const bf16_t*)o, (const float*)lse, nls, nd,
                                                             (bf16_t*)dqkv, B, T, H, scale, scale * kLog2e, th, dscale,
                                                             seed, order);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int n_kb = (T + 127) / 128;
  // two query slices per barrier (v3, default): B120 T1024 H12 whole backward 1151 vs 1181 us
  // (profiles/r4_attn_ab_pair.log; the same change in the dQ kernel measured 1152)
  // (three slices per barrier in a 6-slot ring measured 1171 vs 1141 us: profiles/r4_attn_ab_dkdv_g3.log)
  if (flash_config().bwd == BWD_V3 && !th)
    flash_bwd_dkdv2_kernel<1, 4, false, 2><<<n_kb * B * H, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)dout,
                                                                          nls, nd, (bf16_t*)dqkv, B, T, H, scale,
                                                                          scale * kLog2e, th, dscale, seed, order);
  else if (th)
    flash_bwd_dkdv2_kernel<1, 4, true><<<n_kb * B * H, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)dout, nls, nd,
                                                                   (bf16_t*)dqkv, B, T, H, scale, scale * kLog2e, th,
                                                                   dscale, seed, order);
  else
    flash_bwd_dkdv2_kernel<1, 4, false><<<n_kb * B * H, 256, 0, s>>>((const bf16_t*)qkv, (const bf16_t*)dout, nls,
                                                                    nd, (bf16_t*)dqkv, B, T, H, scale, scale * kLog2e,
                                                                    th, dscale, seed, order);
  return hipGetLastError();
}

}  // namespace

// Backward with a 2 x [B, H, T] fp32 workspace.  D = 64 with T % 32 == 0 runs the v2
// kernels (unless the bwd variant is v1); every other shape the generic backward with
// ws[0] as delta.
NSA_API hipError_t NSA_FA_SYM(nsa_flash_bwd2)(const void* qkv, const void* o, const void* dout, const void* lse, void* ws,
                                  void* dqkv, int B, int T, int H, int D, float scale, float p, uint64_t seed,
                                  hipStream_t s) {
  if (D == 64 && T % 32 == 0 && flash_config().bwd >= BWD_V2)
    return bwd2_launch64(qkv, o, dout, lse, ws, dqkv, B, T, H, scale, p, seed, s);
  switch (D) {
    case 32: return bwd_launch<32>(qkv, o, dout, lse, ws, dqkv, B, T, H, scale, p, seed, s);
    case 64: return bwd_launch<64>(qkv, o, dout, lse, ws, dqkv, B, T, H, scale, p, seed, s);
    case 128: return bwd_launch<128>(qkv, o, dout, lse, ws, dqkv, B, T, H, scale, p, seed, s);
    default: return hipErrorInvalidValue;
  }
}

#define NSA_FA_RNG(NAME) NSA_DEFINE_RNG_ADVANCE(NAME)
NSA_FA_RNG(NSA_FA_SYM(nsa_rng_advance_attn))


NSA_API hipError_t NSA_FA_SYM(nsa_flash_fwd)(const void* qkv, void* out, void* lse, int B, int T, int H, int D, float scale,
                                 float p, uint64_t seed, hipStream_t s) {
  switch (D) {
    case 32: return fwd_launch<32>(qkv, out, lse, B, T, H, scale, p, seed, s);
    case 64: return fwd_launch<64>(qkv, out, lse, B, T, H, scale, p, seed, s);
    case 128: return fwd_launch<128>(qkv, out, lse, B, T, H, scale, p, seed, s);
    default: return hipErrorInvalidValue;
  }
}

#if !NSA_FA_F16
NSA_API void* nsa_flash_config_ptr() { return &flash_config(); }

// Kernel selection (see FlashConfig): fwd 0 auto / 1 v1 / 5 v5, bwd 1 v1 / 2 v2 / 3 v3, order 0 / 1 / 2; a negative value keeps the current setting.  Returns the previous selection as
// fwd | bwd << 4 | order << 8.
NSA_API int nsa_flash_set_variant(int fwd, int bwd, int order) {
  FlashConfig& c = flash_config();
  const int prev = c.fwd | (c.bwd << 4) | (c.order << 8);
  if (fwd == FWD_AUTO || fwd == FWD_V1 || fwd == FWD_V5) c.fwd = fwd;
  if (bwd >= BWD_V1 && bwd <= BWD_V3) c.bwd = bwd;
  if (order >= 0 && order <= 2) c.order = order;
  return prev;
}
#endif  // !NSA_FA_F16
