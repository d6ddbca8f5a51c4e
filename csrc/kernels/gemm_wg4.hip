// Four-wave bf16 weight-gradient GEMM for gfx950 (dW = dY^T · X), the
// main loop of gemm_nt4.hip on operands stored token-major:
//
//   C[M,N] (+)= A[K,M]^T · B[K,N]   A = dY [tokens][out] (lda), B = X [tokens][in] (ldb),
//                                   C fp32 [out][in] (the flat gradient), K = tokens,
//                                   split S ways (split z owns K-tiles
//                                   [z n / S, (z+1) n / S), any split count)
//
// Per workgroup one 256x256 output tile, 4 waves of 128x128 (8x8 accumulators of
// v_mfma_f32_16x16x32_bf16 in AGPRs, tied asm operands).  A K-tile is 64 tokens: two images
// [64][256] bf16 (512-B rows) staged by LDS-DMA (buffer_load_dwordx4 ... lds, one M0 write
// per group of four 1-KiB pieces, piece = 2 token rows) into two buffers; the MFMA fragments
// (16 rows/columns x 32 tokens) are read transposed with ds_read_b64_tr_b16, two per
// fragment.  Image chunk swizzle: 16-B chunk c of row r at c ^ 2 g(r), g = (r & 3) |
// ((r >> 3) & 1) << 2 (the eight rows of a transposed read's lane groups in eight distinct
// 32-B bank groups; the same image as gemm.hip's rimg).  Schedule per K-tile (MFMA slots):
//   n 0-31   the k-step-1 fragments (32 transposed reads, this buffer)
//   n 33/34  wait, barrier (this buffer is free)
//   n 35-125 LDS-DMA of K-tile t+2 into this buffer, one piece per 6 MFMAs
//   n 92/93  vmcnt, barrier (K-tile t+1 has landed)
//   n 94-125 K-tile t+1's k-step-0 fragments (32 reads, other buffer)
// MFMA operands are swapped (B fragment first) so a lane holds 4 consecutive output columns
// of a row: the epilogue re-shapes 64-row halves through LDS into whole 256-B rows, one fp32
// atomic (or plain store for the deterministic partials) per lane per row and half.
#include <utility>

#include "common.h"

namespace {

constexpr int W_BM = 256, W_BN = 256, W_BK = 64;
constexpr int W_THR = 256;
constexpr int W_IMG = W_BK * 256 * 2;  // 32 KiB: [64 tokens][256] bf16
constexpr int W_SMEM = 4 * W_IMG;      // A0 A1 B0 B1
constexpr int W_GRP = 3072;            // largest instruction offset inside an M0 group of pieces

enum : int { W_EPI_ATOMIC = 1, W_EPI_STORE = 4 };

typedef int w_i32x4 __attribute__((ext_vector_type(4)));

struct Wg4Args {
  const bf16_t* A;
  const bf16_t* B;
  float* C;
  float* gb;  // BG: gb[m] += sum over the split's tokens of A[k][m] (the bias gradient)
  int M, N, K;
  int lda, ldb, ldc;
  int tiles_m, tiles_n, splits;
};

template <int I>
struct WI {
  static constexpr int value = I;
};
template <class F, int... Is>
__device__ __forceinline__ void w_for_impl(F&& f, std::integer_sequence<int, Is...>) {
  (f(WI<Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void w_for(F&& f) {
  w_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <bool H>
__device__ __forceinline__ void w_mfma(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  if constexpr (H) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
  else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a));
}
template <bool H>
__device__ __forceinline__ void w_mfma0(f32x4& acc, const bf16x8& b, const bf16x8& a) {
  if constexpr (H) asm volatile("v_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "=a"(acc) : "v"(b), "v"(a));
  else asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(acc) : "v"(b), "v"(a));
}
__device__ __forceinline__ void w_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void w_vmwait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int OFF>
__device__ __forceinline__ void w_dma(uint32_t lds, uint32_t voff, w_i32x4 rsrc, uint32_t soff) {
  if constexpr (OFF == 0) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds" ::"s"(lds), "v"(voff),
                 "s"(rsrc), "s"(soff)
                 : "memory");
  } else {
    asm volatile("buffer_load_dwordx4 %0, %1, %2 offen offset:%3 lds" ::"v"(voff), "s"(rsrc), "s"(soff), "n"(OFF)
                 : "memory");
  }
}
#ifndef NSA_WG4_GLDS
#define NSA_WG4_GLDS 0  // 1: global_load_lds_dwordx4 with an SGPR base + per-piece VGPR offsets (measured 1-3 % slower here)
#endif
template <int OFF>
__device__ __forceinline__ void w_dmag(uint32_t lds, uint32_t voff, const void* sbase) {
  if constexpr (OFF == 0) {
    asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2" ::"s"(lds), "v"(voff), "s"(sbase)
                 : "memory");
  } else {
    asm volatile("global_load_lds_dwordx4 %0, %1 offset:%2" ::"v"(voff), "s"(sbase), "n"(OFF) : "memory");
  }
}
__device__ __forceinline__ w_i32x4 w_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  w_i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32) & 0xffff);
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}
__device__ __forceinline__ void w_add_base(w_i32x4& r, uint32_t bytes) {
  uint64_t b = ((uint64_t)(uint32_t)r.y << 32) | (uint32_t)r.x;
  b += bytes;
  r.x = (int)(uint32_t)b;
  r.y = (int)(uint32_t)(b >> 32);
}
// transposed fragment half: lane l gets 4 consecutive tokens of column (l & 15)
__device__ __forceinline__ s16x4 w_tr(uint32_t addr) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(uintptr_t)addr);
}
__device__ __forceinline__ bf16x8 w_cat(s16x4 a, s16x4 b) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v = __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ int w_g(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

}  // namespace

// sum of a fragment's 8 bf16 values into an f32 (v_dot2c_f32_bf16 against a literal 1.0 pair)
// (fp16: v_dot2_f32_f16 against 1.0 pairs)
template <bool H>
__device__ __forceinline__ float w_sum8(const bf16x8& a, float acc) {
  if constexpr (H) {
    typedef _Float16 w_f16x2 __attribute__((ext_vector_type(2)));
    const f16x8 h = __builtin_bit_cast(f16x8, a);
    const w_f16x2 one = __builtin_bit_cast(w_f16x2, 0x3C003C00u);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_fdot2(w_f16x2{h[2 * e], h[2 * e + 1]}, one, acc, false);
  } else {
    typedef __bf16 w_bf16x2 __attribute__((ext_vector_type(2)));
    const w_bf16x2 one = __builtin_bit_cast(w_bf16x2, 0x3F803F80u);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc = __builtin_amdgcn_fdot2_f32_bf16(w_bf16x2{a[2 * e], a[2 * e + 1]}, one, acc, false);
  }
  return acc;
}

// BG: the bias gradient (column sums of dY over the tokens) from the dY fragments the MFMAs
// read anyway -- no second pass over dY (the separate column-sum kernel read the whole dY
// again: 14.8 ms/step at GPT-2 124M with biases).  The work is spread so that no workgroup
// carries much of it: K-tile kt of a split is summed by the tiles of column block
// kt % tiles_n only, and of the two waves that read the same A fragments, wave wn takes the
// fragments i with i % 2 == wn (4 v_dot2c per fragment, in MFMA gaps).  Each wave ends
// with one atomic add per column it summed.  (All sums in the first column block's wn = 0
// waves measured +16-18 % on that kernel: the slowest workgroup sets a one-round grid.)
template <int EPI, bool BG = false, bool H = false>
__global__ __launch_bounds__(W_THR, 1) void wgrad4_kernel(Wg4Args g) {
  __shared__ __attribute__((aligned(16))) char smem[W_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char*)smem));

  // work item u = (split z, tile v), one block each on a 1-D grid.  Blocks b, b+8, ... share
  // an XCD; the remap gives an XCD consecutive items u, i.e. every tile of one or a few
  // splits, so the token slices of dY and X that those tiles share are read from HBM once
  // and then hit in that XCD's L2 (the 768 x 768 dW, 9 tiles x 28 splits: 3x less HBM).
  const int tiles = g.tiles_m * g.tiles_n;
  int u = blockIdx.x;
  {
    const int G = gridDim.x, x = u % 8, qq = G / 8, rr = G % 8;
    u = (x < rr ? x * (qq + 1) : rr * (qq + 1) + (x - rr) * qq) + u / 8;
  }
  if (u >= tiles * g.splits) return;
  const int v = u % tiles, z = u / tiles;
  const int tm = v / g.tiles_n, tn = v % g.tiles_n;
  const int mlo = tm * W_BM, nlo = tn * W_BN;
  const int m0 = min(mlo, g.M - W_BM), n0 = min(nlo, g.N - W_BN);
  const int nkt = g.K / W_BK;
  const int kt0 = (int)((int64_t)z * nkt / g.splits), kt1 = (int)((int64_t)(z + 1) * nkt / g.splits);
  const int nk = kt1 - kt0;

  // ---- DMA geometry: wave w copies pieces P = 8 w + p of each image = token rows
  // 16 w + 2 p + h (h = lane >> 5), physical chunk lane & 31 holding logical chunk
  // (lane & 31) ^ 2 g(row); g depends on (p & 1, p >> 2, h) only.
  const int h = lane >> 5, lc = lane & 31;
  uint32_t voA[4], voB[4];
#pragma unroll
  for (int pp = 0; pp < 4; ++pp) {
    const int p = (pp & 1) | ((pp >> 1) << 2);  // representative piece of the class
    const int row = 2 * p + h;
    const uint32_t ch = (uint32_t)((lc ^ (2 * w_g(row))) << 4);
    voA[pp] = (uint32_t)(h * g.lda * 2) + ch;
    voB[pp] = (uint32_t)(h * g.ldb * 2) + ch;
  }
  uint32_t soA[8], soB[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    soA[p] = (uint32_t)__builtin_amdgcn_readfirstlane((16 * wave + 2 * p) * g.lda * 2 + W_GRP - (p & 3) * 1024);
    soB[p] = (uint32_t)__builtin_amdgcn_readfirstlane((16 * wave + 2 * p) * g.ldb * 2 + W_GRP - (p & 3) * 1024);
  }
  // LDS: A buffers at 0 / W_IMG, B buffers at 2 W_IMG / 3 W_IMG (buffer = XOR W_IMG)
  const uint32_t dmaA = lds0 + (uint32_t)(wave * 8 * 1024);
  const uint32_t dmaB = lds0 + (uint32_t)(2 * W_IMG + wave * 8 * 1024);

  // buffer resources: token row kt0 * 64 of the tile's columns, lowered by W_GRP
  const uint32_t stepA = (uint32_t)(W_BK * g.lda * 2), stepB = (uint32_t)(W_BK * g.ldb * 2);
  w_i32x4 ra = w_rsrc(reinterpret_cast<const char*>(g.A + (int64_t)kt0 * W_BK * g.lda + m0) - W_GRP, 0xffffffffu);
  w_i32x4 rb = w_rsrc(reinterpret_cast<const char*>(g.B + (int64_t)kt0 * W_BK * g.ldb + n0) - W_GRP, 0xffffffffu);
  int kd = 0;  // K-tile index (within the split) of the cursor
  auto cur_next = [&]() {
    if (++kd >= nk) {
      // past the split's last K-tile: buffer_load gets an empty range (loads nothing); the
      // global_load_lds form re-reads the split's last K-tile into a buffer nobody reads
      ra.z = 0;
      rb.z = 0;
    } else {
      w_add_base(ra, stepA);
      w_add_base(rb, stepB);
    }
  };
  uint32_t vpA[NSA_WG4_GLDS ? 8 : 1], vpB[NSA_WG4_GLDS ? 8 : 1];
  if constexpr (NSA_WG4_GLDS) {
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      vpA[p] = voA[(p & 1) | ((p >> 2) << 1)] + soA[p];
      vpB[p] = voB[(p & 1) | ((p >> 2) << 1)] + soB[p];
    }
  }
  auto sbase = [](const w_i32x4& r) {
    return reinterpret_cast<const void*>(((uint64_t)(uint32_t)r.y << 32) | (uint32_t)r.x);
  };
  auto issue_a = [&](uint32_t buf, auto P) {
    constexpr int p = decltype(P)::value;
    if constexpr (NSA_WG4_GLDS)
      w_dmag<(p & 3) * 1024>(dmaA + buf + (uint32_t)((p & 4) * 1024), vpA[p], sbase(ra));
    else
      w_dma<(p & 3) * 1024>(dmaA + buf + (uint32_t)((p & 4) * 1024), voA[(p & 1) | ((p >> 2) << 1)], ra, soA[p]);
  };
  auto issue_b = [&](uint32_t buf, auto P) {
    constexpr int p = decltype(P)::value;
    if constexpr (NSA_WG4_GLDS)
      w_dmag<(p & 3) * 1024>(dmaB + buf + (uint32_t)((p & 4) * 1024), vpB[p], sbase(rb));
    else
      w_dma<(p & 3) * 1024>(dmaB + buf + (uint32_t)((p & 4) * 1024), voB[(p & 1) | ((p >> 2) << 1)], rb, soB[p]);
  };

  // ---- fragment read addresses (buffer 0, k-step 0, first half): fragment f covers columns
  // 16 f of the wave's 128; lane (q, p) = (l & 15) >> 2, l & 3 reads token row
  // 8 (l >> 4) + q, columns 16 f + 4 p: chunk 2 f' + (p >> 1) with f' the image column block.
  // k-step 1 = +32 rows (16 KiB), second half = +4 rows (2 KiB): g is unchanged by both.
  const int ig = lane & 15, fq = ig >> 2, fp = ig & 3;
  const int krow = 8 * (lane >> 4) + fq;
  const int gk = w_g(krow);
  uint32_t rdA[8], rdB[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    const int fa = wm * 8 + f, fb = wn * 8 + f;  // 16-column blocks of the 256-wide image
    rdA[f] = lds0 + (uint32_t)(krow * 512 + (((2 * fa + (fp >> 1)) ^ (2 * gk)) << 4) + (fp & 1) * 8);
    rdB[f] = lds0 + (uint32_t)(2 * W_IMG + krow * 512 + (((2 * fb + (fp >> 1)) ^ (2 * gk)) << 4) + (fp & 1) * 8);
  }

  // ---- prologue: K-tiles 0 and 1 into buffers 0 / 1
  w_for<8>([&](auto P) { issue_a(0, P); });
  w_for<8>([&](auto P) { issue_b(0, P); });
  cur_next();
  w_for<8>([&](auto P) { issue_a(W_IMG, P); });
  w_for<8>([&](auto P) { issue_b(W_IMG, P); });
  w_vmwait<16>();
  cur_next();
  w_barrier();

  f32x4 acc[8][8];
  bf16x8 a0[8], b0[8], a1[8], b1[8];
#pragma unroll
  for (int f = 0; f < 8; ++f) {
    a0[f] = w_cat(w_tr(rdA[f]), w_tr(rdA[f] + 2048));
    b0[f] = w_cat(w_tr(rdB[f]), w_tr(rdB[f] + 2048));
  }

  float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int kc = kt0;  // BG: global index of the K-tile being multiplied
  uint32_t buf = 0;
  auto ktile = [&](auto FIRST_) {
    constexpr bool FIRST = decltype(FIRST_)::value;
    const bool do_bg = BG && kc % g.tiles_n == tn;  // wave-uniform
    w_for<128>([&](auto I) {
      constexpr int n = decltype(I)::value;
      constexpr int kk = n >> 6, j = (n >> 3) & 7, i = n & 7;
      if constexpr (kk == 0) {
        if constexpr (FIRST) w_mfma0<H>(acc[i][j], b0[j], a0[i]);
        else w_mfma<H>(acc[i][j], b0[j], a0[i]);
      } else {
        w_mfma<H>(acc[i][j], b1[j], a1[i]);
      }
      if constexpr (BG && j == 1) {  // the fragment the previous slot's MFMA read
        if (do_bg && (i & 1) == wn) bsum[i] = w_sum8<H>(kk == 0 ? a0[i] : a1[i], bsum[i]);
      }
      // k-step 1 fragments of this buffer, one transposed read per MFMA
      if constexpr (n < 32) {
        constexpr int f = (n >> 1) & 7, hf = n & 1;
        if constexpr (n < 16) {
          if constexpr (hf == 0) a1[f] = w_cat(w_tr(rdA[f] + 16384), w_tr(rdA[f] + 16384 + 2048));
        } else {
          if constexpr (hf == 0) b1[f] = w_cat(w_tr(rdB[f] + 16384), w_tr(rdB[f] + 16384 + 2048));
        }
      }
      if constexpr (n == 33) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this buffer's reads done
      if constexpr (n == 34) w_barrier();
      constexpr int D0 = 35, DS = 6;
      if constexpr (n >= D0 && (n - D0) % DS == 0 && (n - D0) / DS < 16) {
        constexpr int pc = (n - D0) / DS;
        if constexpr (pc < 8) issue_a(buf, WI<pc>{});
        else issue_b(buf, WI<pc - 8>{});
      }
      if constexpr (n == 62) {
#pragma unroll
        for (int f = 0; f < 8; ++f) {
          rdA[f] ^= (uint32_t)W_IMG;
          rdB[f] ^= (uint32_t)W_IMG;
        }
      }
      if constexpr (n == 92) w_vmwait<(92 - D0) / DS + 1>();
      if constexpr (n == 93) w_barrier();
      if constexpr (n >= 94 && n < 126 && ((n - 94) & 1) == 0) {
        constexpr int f = ((n - 94) >> 1) & 7;
        if constexpr (n < 110) b0[f] = w_cat(w_tr(rdB[f]), w_tr(rdB[f] + 2048));
        else a0[f] = w_cat(w_tr(rdA[f]), w_tr(rdA[f] + 2048));
      }
    });
    buf ^= (uint32_t)W_IMG;
    cur_next();
    ++kc;
  };
  ktile(WI<1>{});
  for (int kt = 1; kt < nk; ++kt) ktile(WI<0>{});
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  if constexpr (BG) {
    const int first = kt0 + ((tn - kt0 % g.tiles_n) + g.tiles_n) % g.tiles_n;  // first kt >= kt0 with kt % tiles_n == tn
    if (first < kt1) {  // this workgroup summed at least one K-tile
      // lanes l, l ^ 16, l ^ 32, l ^ 48 hold the same column's token groups
#pragma unroll
      for (int f = 0; f < 8; ++f) {
        if ((f & 1) != wn) continue;
        float v = bsum[f];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        const int m = m0 + wm * 128 + 16 * f + (lane & 15);
        if (lane < 16 && m >= mlo) atomicAdd(g.gb + m, v);
      }
    }
  }
  w_barrier();  // every wave is done with the K-tile buffers: the epilogue reuses them

  // ---- epilogue: two halves of 64 rows per wave through a wave-private 32-KiB slice
  // [64][128] fp32 (512-B rows, 16-B unit u of row r at u ^ (r & 7)); lane l holds row
  // 16 i + (l & 15), columns 16 j + 4 (l >> 4) + 0..3
  char* ep = smem + wave * 32768;
  const int er = lane & 15, eq = lane >> 4;
  float* Cz = g.C;
  if constexpr (EPI == W_EPI_STORE) Cz += (int64_t)z * g.M * g.ldc;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int ii = 0; ii < 4; ++ii) {
      const int i = 4 * half + ii;
      const int row = 16 * ii + er;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int u = 4 * j + eq;
        *reinterpret_cast<f32x4*>(ep + row * 512 + ((u ^ (row & 7)) << 4)) = acc[i][j];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int col0 = n0 + wn * 128;
    // the K-splits of one tile add into the same rows: each split walks them from its own
    // starting row, so concurrent atomics of different splits hit different lines
    const int rot = (z * 23) & 63;
#pragma unroll 4
    for (int r2 = 0; r2 < 64; ++r2) {
      const int rr = (r2 + rot) & 63;
      const int grow = m0 + wm * 128 + 64 * half + rr;
#pragma unroll
      for (int c2 = 0; c2 < 2; ++c2) {
        const int c = 64 * c2 + lane;
        const float val = *reinterpret_cast<const float*>(ep + rr * 512 + ((((c >> 2) ^ (rr & 7))) << 4) + (c & 3) * 4);
        if (grow >= mlo && col0 + c >= nlo) {
          if constexpr (EPI == W_EPI_STORE)
            Cz[(int64_t)grow * g.ldc + col0 + c] = val;
          else
            atomicAdd(Cz + (int64_t)grow * g.ldc + col0 + c, val);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// C (fp32) [M, N] (+)= A^T B, A stored [K][M], B stored [K][N]; K split over `splits`.
// epi: 1 = fp32 atomic add into C, 4 = split z stores its partial into C + z*M*ldc.
// M, N >= 256, M % 8 == N % 8 == 0, K % 64 == 0, splits <= K / 64.
// gb (optional, epi 1 only): the bias gradient gb[m] += sum_k A[k][m], fused (see BG).
// (the _h entry points take fp16 A / B)
namespace {
template <bool H>
hipError_t wgrad4_entry(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* gb, int M,
                        int N, int K, int splits, hipStream_t s) {
  if (gb && epi != W_EPI_ATOMIC) return hipErrorInvalidValue;
  if ((epi != W_EPI_ATOMIC && epi != W_EPI_STORE) || M < W_BM || N < W_BN || M % 8 || N % 8 || K % W_BK ||
      splits < 1 || splits > K / W_BK || lda % 8 || ldb % 8 || lda < M || ldb < N || ldc < N)
    return hipErrorInvalidValue;
  if ((int64_t)W_BK * lda * 2 + W_GRP >= (1ll << 31) || (int64_t)W_BK * ldb * 2 + W_GRP >= (1ll << 31))
    return hipErrorInvalidValue;
  Wg4Args a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = (float*)C;
  a.M = M;
  a.N = N;
  a.K = K;
  a.lda = lda;
  a.ldb = ldb;
  a.ldc = ldc;
  a.tiles_m = (M + W_BM - 1) / W_BM;
  a.tiles_n = (N + W_BN - 1) / W_BN;
  a.splits = splits;
  const dim3 grid(a.tiles_m * a.tiles_n * splits);
  a.gb = (float*)gb;
  if (gb) wgrad4_kernel<W_EPI_ATOMIC, true, H><<<grid, W_THR, 0, s>>>(a);
  else if (epi == W_EPI_ATOMIC) wgrad4_kernel<W_EPI_ATOMIC, false, H><<<grid, W_THR, 0, s>>>(a);
  else wgrad4_kernel<W_EPI_STORE, false, H><<<grid, W_THR, 0, s>>>(a);
  return hipGetLastError();
}
}  // namespace

NSA_API hipError_t nsa_gemm_wgrad4b(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, void* gb,
                                    int M, int N, int K, int splits, hipStream_t s) {
  return wgrad4_entry<false>(epi, A, lda, B, ldb, C, ldc, gb, M, N, K, splits, s);
}
NSA_API hipError_t nsa_gemm_wgrad4(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M,
                                   int N, int K, int splits, hipStream_t s) {
  return wgrad4_entry<false>(epi, A, lda, B, ldb, C, ldc, nullptr, M, N, K, splits, s);
}
NSA_API hipError_t nsa_gemm_wgrad4b_h(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                                      void* gb, int M, int N, int K, int splits, hipStream_t s) {
  return wgrad4_entry<true>(epi, A, lda, B, ldb, C, ldc, gb, M, N, K, splits, s);
}
NSA_API hipError_t nsa_gemm_wgrad4_h(int epi, const void* A, int lda, const void* B, int ldb, void* C, int ldc, int M,
                                     int N, int K, int splits, hipStream_t s) {
  return wgrad4_entry<true>(epi, A, lda, B, ldb, C, ldc, nullptr, M, N, K, splits, s);
}
