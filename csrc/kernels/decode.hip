// Incremental decoding (serving path): KV-cache append and single-query attention
// over the cache for gfx950.  nanoGPT's generate() re-runs the whole context for
// every new token (reference sample.py -> model.generate, SURVEY.md §2.3 U-M11 /
// U-S1); runtime/decode.py keeps per-layer K/V caches instead and replays one
// token's forward as a HIP graph, so the position of the token being decoded lives
// in device memory (`pos`) and every kernel here reads it there: nothing in the
// captured step depends on a host value that changes between tokens.
//
// Cache layout: K and V as [B, H, Tmax, D] bf16, one 128-byte row per key at D = 64
// (a wave reads 64 consecutive rows = 8 KiB contiguous for the scores, and one
// 128-byte row per key for the weighted V sum).
//
// Attention (flash-decoding): the cache is split into 256-key chunks; workgroup
// (b*H + h, s) scores its chunk's keys (one key per thread, q in LDS), forms the
// chunk-local softmax (max m, sum l) and the chunk's weighted V sum o, and writes
// (m, l, o[64]) to a workspace; a combine kernel rescales the chunks to the global
// max.  Chunks past `pos` write an empty partial (m = -inf) and exit, so the grid is
// fixed by Tmax (graph-safe) while the work follows the live context length.
#include "common.h"

#include <math.h>
#include <stdlib.h>

#include <algorithm>

namespace {

constexpr int DA_D = 64;        // head dim of the decode-attention kernel
constexpr int DA_CHUNK = 256;   // keys per workgroup (one per thread)
constexpr int DA_PO = 4;          // o[] offset in a partial: 16-byte aligned for vector reads
constexpr int DA_PART = DA_PO + DA_D;  // m, l, (pad), o[64]

__global__ __launch_bounds__(256) void kv_append_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ kc,
                                                        bf16_t* __restrict__ vc, const int64_t* __restrict__ pos_dev,
                                                        int pos0, int B, int S, int H, int D, int Tmax) {
  // one thread per 16-byte chunk of a K or V row: index = (((b*S + s)*2 + kv)*H + h)*cpr + c
  const int cpr = D / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t total = (int64_t)B * S * 2 * H * cpr;
  if (i >= total) return;
  const int c = (int)(i % cpr);
  int64_t r = i / cpr;
  const int hh = (int)(r % H);
  r /= H;
  const int kv = (int)(r & 1);
  r >>= 1;
  const int s = (int)(r % S);
  const int b = (int)(r / S);
  const int p = (pos_dev ? (int)*pos_dev : pos0) + s;
  if (p < 0 || p >= Tmax) return;
  const int C = H * D;
  const bf16_t* src = qkv + ((int64_t)b * S + s) * 3 * C + (1 + kv) * C + hh * D + c * 8;
  bf16_t* dst = (kv ? vc : kc) + (((int64_t)b * H + hh) * Tmax + p) * D + c * 8;
  *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(src);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// grid (B*H, n_split), 256 threads
// append: also store the new token's K / V rows at position pos (kc_w / vc_w alias
// kc / vc; separate non-restrict pointers for the one write)
__global__ __launch_bounds__(256) void decode_attn_partial_kernel(const bf16_t* __restrict__ qkv,
                                                                  const bf16_t* __restrict__ kc,
                                                                  const bf16_t* __restrict__ vc, bf16_t* kc_w,
                                                                  bf16_t* vc_w, const int64_t* __restrict__ pos_dev,
                                                                  float* __restrict__ ws, int H, int Tmax,
                                                                  float scale_log2, int append) {
  __shared__ float qs[DA_D];
  __shared__ float ps[DA_CHUNK];
  __shared__ float red[2][4];
  __shared__ float os[4][DA_D];
  const int bh = blockIdx.x, s = blockIdx.y, n_split = gridDim.y;
  const int b = bh / H, hh = bh % H;
  const int C = H * DA_D;
  const int pos = (int)*pos_dev;  // the query's own position = the newest key
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float* part = ws + ((int64_t)bh * n_split + s) * DA_PART;
  const int k0 = s * DA_CHUNK;
  if (k0 > pos) {  // chunk beyond the live context: empty partial
    if (tid < DA_PART) part[tid] = tid == 0 ? -INFINITY : 0.0f;
    return;
  }
  const bf16_t* qrow = qkv + (int64_t)b * 3 * C + hh * DA_D;  // q | k | v of the new token
  if (tid < DA_D) qs[tid] = bf2f(qrow[tid]);
  if (append && pos < k0 + DA_CHUNK && tid < 2 * (DA_D / 8)) {
    // this chunk holds position pos: store the new token's K / V rows for later steps
    // (this kernel itself takes them straight from qkv, so no write->read ordering)
    const int c = tid & 7, kv = tid >> 3;
    *reinterpret_cast<uint4*>((kv ? vc_w : kc_w) + ((int64_t)bh * Tmax + pos) * DA_D + 8 * c) =
        *reinterpret_cast<const uint4*>(qrow + (1 + kv) * C + 8 * c);
  }
  __syncthreads();
  const int key = k0 + tid;
  const bool live = key <= pos;
  float sc = -INFINITY;
  if (live) {
    const bf16_t* krow = key == pos ? qrow + C : kc + ((int64_t)bh * Tmax + key) * DA_D;
    float acc = 0.0f;
#pragma unroll
    for (int c = 0; c < DA_D / 8; ++c) {
      float kf[8];
      load8(krow + 8 * c, kf);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc = fmaf(qs[8 * c + j], kf[j], acc);
    }
    sc = acc * scale_log2;
  }
  float m = wave_max(sc);
  if (lane == 0) red[0][w] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  const float p = live ? exp2f(sc - m) : 0.0f;
  const float lw = wave_sum(p);
  if (lane == 0) red[1][w] = lw;
  ps[tid] = p;
  __syncthreads();
  // weighted V sum: thread (key group kg = tid / 8: keys k0 + 8 kg .. +7; dims 8 dg .. +7)
  // issues its 8 16-byte row loads together (one 2-byte load per key and lane in a
  // 64-long dependent loop was the kernel's latency chain).  Keys past pos read the row
  // at pos (finite) and carry p = 0; the new token's row comes from qkv when appending
  // (this launch is what writes it to the cache).
  const int kg = tid >> 3, dg = tid & 7;
  float o[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = 0.0f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int kk = min(k0 + 8 * kg + j, pos);
    const bf16_t* vr = (append && kk == pos) ? qrow + 2 * C : vc + ((int64_t)bh * Tmax + kk) * DA_D;
    float vf[8];
    load8(vr + 8 * dg, vf);
    const float pj = ps[8 * kg + j];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = fmaf(pj, vf[e], o[e]);
  }
#pragma unroll
  for (int off = 8; off < 64; off <<= 1)  // the wave's 8 key groups (lane bits 3..5)
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += __shfl_xor(o[e], off, 64);
  if (lane < 8)
#pragma unroll
    for (int e = 0; e < 8; ++e) os[w][8 * lane + e] = o[e];
  __syncthreads();
  if (tid < DA_D) part[DA_PO + tid] = os[0][tid] + os[1][tid] + os[2][tid] + os[3][tid];
  if (tid == 0) {
    part[0] = m;
    part[1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// grid B*H, 64 threads: out[b, h*64 + d] = sum_s 2^(m_s - M) o_s[d] / sum_s 2^(m_s - M) l_s
__global__ __launch_bounds__(64) void decode_attn_combine_kernel(const float* __restrict__ ws,
                                                                 bf16_t* __restrict__ out, int H, int n_split) {
  const int bh = blockIdx.x, d = threadIdx.x;
  const int b = bh / H, hh = bh % H;
  const float* part = ws + (int64_t)bh * n_split * DA_PART;
  float M = -INFINITY;
  for (int s = 0; s < n_split; ++s) M = fmaxf(M, part[s * DA_PART]);
  float L = 0.0f, o = 0.0f;
  for (int s = 0; s < n_split; ++s) {
    const float f = exp2f(part[s * DA_PART] - M);  // empty chunks: 2^-inf = 0
    L = fmaf(f, part[s * DA_PART + 1], L);
    o = fmaf(f, part[s * DA_PART + DA_PO + d], o);
  }
  out[(int64_t)b * H * DA_D + hh * DA_D + d] = f2bf(o / L);
}

// ---------------------------------------------------------------------------
// Sampling (nanoGPT sample.py: logits / temperature, keep the top_k, softmax,
// multinomial) for one row per workgroup, fully on the device so the decode graph can
// feed the sampled token back without a host round trip (torch's topk / multinomial
// chain is ~20 launches and its segmented sort is not graph-replay safe here).
// Each of the 1024 threads keeps up to 52 logits of the row in registers as
// order-preserving uint32 keys (element j * 1024 + t: coalesced loads).
// Top-k path (top_k <= 1024, the serving case):
//  1. one wave finds a key lo0 with k .. 2k of the 1024 per-thread maxima >= it: the
//     row's k-th largest key is >= lo0 (k distinct elements are), so every top-k
//     element is among the keys >= lo0, and those live only in threads whose maximum
//     is >= lo0: typically ~k .. 2k keys;
//  2. the candidates are compacted into LDS in (thread, j) order (deterministic);
//  3. the exact k-th largest key thr among them (one wave; a block-wide 16-ary search
//     beyond 1024 candidates); the wave then forms w_i = exp2((l_i - M) log2(e) / T)
//     for the candidates >= thr (ties kept, as torch's `logits < v[:, [-1]]` mask),
//     scans them and picks the first whose running sum exceeds u = uniform * sum w
//     (uniform from the counter hash of (salt, row, position)).
// Bisection counts are ballots + scalar popcounts (no shuffles) and stop early (at
// exactly k entries >= mid for the exact select, inside the k .. 2k window for lo0).
// Otherwise (no top-k, k > 1024, or > 4096 candidates): bisection over all keys with
// block reductions and a block-wide scan (the single-CU VALU cost of 32 passes over
// 50k keys made this ~70 us per row; the top-k path is a few us).
// The chosen id is written to tok[b] and gen[b, *pos].
// ---------------------------------------------------------------------------
constexpr int SMP_THREADS = 1024;
constexpr int SMP_CAP = 4096;  // top-k candidates compacted into LDS

__device__ __forceinline__ uint32_t fkey(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_val(uint32_t k) {  // inverse of fkey
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

template <typename T>
__device__ __forceinline__ T block_reduce(T v, T* red, bool is_max) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const T o = __shfl_xor(v, off, 64);
    v = is_max ? (o > v ? o : v) : v + o;
  }
  __syncthreads();  // red[] may still be read from the previous reduction
  if (lane == 0) red[w] = v;
  __syncthreads();
  T r = red[0];
  for (int i = 1; i < SMP_THREADS / 64; ++i) r = is_max ? (red[i] > r ? red[i] : r) : r + red[i];
  return r;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// k-th largest selection: the largest K in [lo, hi] with #{i : a[i] >= K} >= k (the
// k-th largest of a[] when count(a >= lo) >= k and count(a >= hi + 1) < k).  Counts
// come from ballots (v_cmp into a lane mask + a scalar popcount: no cross-lane
// shuffles), so a bisection step of one wave over 16 values per lane is ~40
// instructions with lo / hi in scalar registers.  a[] is zero-padded to a multiple of
// 256 entries (key 0 is below every threshold tried, which is >= lo + 1).

// 16 entries per lane of a[0..npad) (npad <= 1024): entries 256 j + 4 lane .. +3
__device__ __forceinline__ void load16_lds(const uint32_t* a, int npad, int lane, uint32_t (&v)[16]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = 256 * j + 4 * lane;
    const uint4 q = i < npad ? *reinterpret_cast<const uint4*>(a + i) : make_uint4(0, 0, 0, 0);
    v[4 * j] = q.x;
    v[4 * j + 1] = q.y;
    v[4 * j + 2] = q.z;
    v[4 * j + 3] = q.w;
  }
}

__device__ __forceinline__ uint32_t count16(const uint32_t (&v)[16], uint32_t th) {
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) c += (uint32_t)__popcll(__ballot(v[j] >= th));
  return c;
}

// one wave, up to 1024 entries held as v[16] per lane, no barriers.  Exact k-th largest
// by bisection that stops as soon as exactly k entries are >= mid (the answer is then
// the smallest of them): ~log2(n) + a few steps instead of 32.
__device__ uint32_t wave_kth16(const uint32_t (&v)[16], int k, uint32_t lo, uint32_t hi) {
  lo = __builtin_amdgcn_readfirstlane(lo);
  hi = __builtin_amdgcn_readfirstlane(hi);
  while (lo < hi) {
    const uint32_t mid = lo + (uint32_t)(((uint64_t)hi - lo + 1) / 2);
    const uint32_t c = count16(v, mid);
    if (c == (uint32_t)k) {
      uint32_t m = 0xffffffffu;
#pragma unroll
      for (int j = 0; j < 16; ++j) m = min(m, v[j] >= mid ? v[j] : 0xffffffffu);
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, off, 64));
      return __builtin_amdgcn_readfirstlane(m);
    }
    if (c > (uint32_t)k)
      lo = mid;
    else
      hi = mid - 1;
  }
  return lo;
}

// one wave: some K >= lo with k <= count(v >= K) <= kcap (or the exact k-th largest when
// no such K is met), for a lower bound that only has to keep the candidate set small
__device__ uint32_t wave_bound16(const uint32_t (&v)[16], int k, int kcap, uint32_t lo, uint32_t hi) {
  lo = __builtin_amdgcn_readfirstlane(lo);
  hi = __builtin_amdgcn_readfirstlane(hi);
  while (lo < hi) {
    const uint32_t mid = lo + (uint32_t)(((uint64_t)hi - lo + 1) / 2);
    const uint32_t c = count16(v, mid);
    if (c >= (uint32_t)k) {
      lo = mid;
      if (c <= (uint32_t)kcap) break;
    } else {
      hi = mid - 1;
    }
  }
  return lo;
}

// the whole 1024-thread block, up to 4096 entries in LDS: 16-ary search, per round wave
// w counts the entries >= the (w + 1)-th of 15 interior thresholds, one barrier, every
// wave narrows [lo, hi] to the bracket (8 rounds over the 32-bit key space); cnt[]
// holds 32 words of LDS (two alternating rounds)
__device__ uint32_t block_kth_largest(const uint32_t* a, int npad, int k, uint32_t lo, uint32_t hi, uint32_t* cnt) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  lo = __builtin_amdgcn_readfirstlane(lo);
  hi = __builtin_amdgcn_readfirstlane(hi);
  int round = 0;
  while (lo < hi) {
    const uint64_t span = (uint64_t)hi - lo + 1;
    uint32_t* cr = cnt + 16 * (round & 1);
    if (w < 15) {
      const uint64_t th = (uint64_t)lo + (span * (uint64_t)(w + 1) + 15) / 16;
      uint32_t c = 0;
      if (th <= hi) {
        const uint32_t t32 = (uint32_t)th;
        for (int i = 4 * lane; i < npad; i += 256) {  // uniform trip count (npad % 256 == 0)
          const uint4 q = *reinterpret_cast<const uint4*>(a + i);
          c += (uint32_t)(__popcll(__ballot(q.x >= t32)) + __popcll(__ballot(q.y >= t32)) +
                          __popcll(__ballot(q.z >= t32)) + __popcll(__ballot(q.w >= t32)));
        }
      }
      if (lane == 0) cr[w] = c;  // 0 above hi: never chosen (count(>= hi + 1) < k)
    }
    __syncthreads();  // the other half of cnt[] was last read before this barrier
    int best = 0;  // threshold 0 is lo itself
#pragma unroll
    for (int i = 1; i < 16; ++i)
      if (cr[i - 1] >= (uint32_t)k) best = i;
    best = __builtin_amdgcn_readfirstlane(best);
    const uint32_t nlo = best == 0 ? lo : (uint32_t)((uint64_t)lo + (span * (uint64_t)best + 15) / 16);
    const uint32_t nhi = best == 15 ? hi : (uint32_t)((uint64_t)lo + (span * (uint64_t)(best + 1) + 15) / 16 - 1);
    lo = nlo;
    hi = nhi;
    ++round;
  }
  __syncthreads();  // cnt[] free for the next call
  return lo;
}

#ifdef NSA_SMP_TIMING  // phase timestamps of row 0 (experiment builds only)
__device__ uint64_t g_smp_ticks[8];
#define SMP_TICK(i) \
  if (b == 0 && t == 0) g_smp_ticks[i] = wall_clock64()
#else
#define SMP_TICK(i)
#endif

constexpr int SMP_MAXC = 52;  // logits per thread kept in registers (V <= 53248: the GPT-2 vocab is 50304)

template <bool VEC4>
__global__ __launch_bounds__(SMP_THREADS) void sample_topk_kernel(const float* __restrict__ logits, int V, int ld,
                                                                  float scale_log2, int top_k, uint64_t salt,
                                                                  const uint64_t* __restrict__ salt_dev,
                                                                  const int64_t* __restrict__ pos,
                                                                  int64_t* __restrict__ tok, int64_t* __restrict__ gen,
                                                                  int gen_ld) {
  __shared__ uint32_t redu[SMP_THREADS / 64];
  __shared__ float scan[SMP_THREADS];
  __shared__ __attribute__((aligned(16))) uint32_t tmx[SMP_THREADS];
  __shared__ __attribute__((aligned(16))) uint32_t ck[SMP_CAP];
  __shared__ int ci[SMP_CAP];
  __shared__ uint32_t cnt16[32];
  __shared__ uint32_t lo_sh;
  __shared__ uint32_t wtot[SMP_THREADS / 64];
  const int b = blockIdx.x, t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float* row = logits + (int64_t)b * ld;
  // element j * 1024 + t stays in registers as an order-preserving key (key 0 = padding,
  // below every real key)
  uint32_t key[SMP_MAXC];
  if (VEC4) {  // element 4 * (j * 1024 + t) + e: 13 coalesced 16-byte loads per thread
    const float4* row4 = reinterpret_cast<const float4*>(row);
    const int V4 = V / 4;
#pragma unroll
    for (int j = 0; j < SMP_MAXC / 4; ++j) {
      const int i4 = j * SMP_THREADS + t;
      // unconditional clamped loads, all in flight together, and an AND mask rather than
      // a select (a select on a loaded value is turned into a branch around the load)
      const float4 v = row4[min(i4, V4 - 1)];
      const uint32_t live = (uint32_t)((i4 - V4) >> 31);  // all ones for i4 < V4
      key[4 * j + 0] = fkey(v.x) & live;
      key[4 * j + 1] = fkey(v.y) & live;
      key[4 * j + 2] = fkey(v.z) & live;
      key[4 * j + 3] = fkey(v.w) & live;
    }
  } else {  // element j * 1024 + t
#pragma unroll
    for (int j = 0; j < SMP_MAXC; ++j) {
      const int i = j * SMP_THREADS + t;
      const float v = row[min(i, V - 1)];
      key[j] = fkey(v) & (uint32_t)((i - V) >> 31);
    }
  }
  // key 0 is padding: every real key is > 0 (fkey sets the top bit or inverts a negative)
  uint32_t kmax = 0, kmin = 0xffffffffu;
#pragma unroll
  for (int j = 0; j < SMP_MAXC; ++j) {
    kmax = max(kmax, key[j]);
    kmin = min(kmin, key[j] ? key[j] : 0xffffffffu);
  }
  SMP_TICK(0);
  const uint32_t tmax = kmax;
  kmax = block_reduce<uint32_t>(kmax, redu, true);
  SMP_TICK(1);
  const float m = key_val(kmax);
  const int p = (int)*pos;
  // the device salt (when given) is read at run time, so a captured sampling graph draws a
  // fresh stream whenever the caller rewrites it (one per generate call)
  const uint64_t sl = salt ^ (salt_dev ? *salt_dev : 0ull);
  const uint32_t hsh = nsa_hash(nsa_seed(sl), (uint64_t)b * 0x9E3779B97F4A7C15ull + (uint64_t)p);
  const float unif = (float)(hsh >> 8) * (1.0f / 16777216.0f);

  if (top_k > 0 && top_k < V && top_k <= SMP_THREADS) {
    tmx[t] = tmax;
    __syncthreads();
    if (w == 0) {
      uint32_t v[16];
      load16_lds(tmx, SMP_THREADS, lane, v);
      // any K with k <= #(thread maxima >= K) bounds the row's k-th largest from below;
      // up to 2k maxima above it keep the candidate set small
      const uint32_t r = wave_bound16(v, top_k, 2 * top_k, 0u, kmax);
      if (lane == 0) lo_sh = r;
    }
    __syncthreads();
    const uint32_t lo0 = lo_sh;
    SMP_TICK(2);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < SMP_MAXC; ++j) c += key[j] >= lo0 ? 1u : 0u;
    uint32_t incl = c;  // inclusive prefix over the wave's lanes
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    if (lane == 63) wtot[w] = incl;
    __syncthreads();
    uint32_t woff = 0, n = 0;
    for (int i = 0; i < SMP_THREADS / 64; ++i) {
      woff += i < w ? wtot[i] : 0u;
      n += wtot[i];
    }
    if (n <= (uint32_t)SMP_CAP) {  // block-uniform
      uint32_t q = woff + incl - c;
      int tt = t;
      asm volatile("" : "+v"(tt));  // opaque: the element ids below are recomputed, not kept live from the loads
#pragma unroll
      for (int j = 0; j < SMP_MAXC; ++j)
        if (key[j] >= lo0) {
          ck[q] = key[j];
          ci[q] = VEC4 ? 4 * ((j >> 2) * SMP_THREADS + tt) + (j & 3) : j * SMP_THREADS + tt;
          ++q;
        }
      for (int i = (int)n + t; i < (((int)n + 255) & ~255); i += SMP_THREADS) ck[i] = 0u;  // zero padding
      __syncthreads();
      SMP_TICK(3);
      const int npad = ((int)n + 255) & ~255;
      uint32_t thr = 0;
      if (npad > 1024)
        thr = block_kth_largest(ck, npad, top_k, lo0, kmax, cnt16);
      SMP_TICK(4);
      if (w == 0) {
        if (npad <= 1024) {
          uint32_t v[16];
          load16_lds(ck, npad, lane, v);
          thr = wave_kth16(v, top_k, lo0, kmax);
        }
        const int per = ((int)n + 63) / 64, c0 = min((int)n, lane * per), c1 = min((int)n, c0 + per);
        float sum = 0.0f;
        for (int i = c0; i < c1; ++i)
          if (ck[i] >= thr) sum += exp2f((key_val(ck[i]) - m) * scale_log2);
        float run = sum;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const float o = __shfl_up(run, off, 64);
          if (lane >= off) run += o;
        }
        float before = __shfl_up(run, 1, 64);
        if (lane == 0) before = 0.0f;
        const float total = __shfl(run, 63, 64);
        const float u = unif * total;
        if ((u >= before && u < run) || (lane == 63 && u >= total)) {
          int pick = -1;
          float acc = before;
          for (int i = c0; i < c1; ++i) {
            if (ck[i] >= thr) {
              acc += exp2f((key_val(ck[i]) - m) * scale_log2);
              pick = ci[i];
              if (acc > u) break;
            }
          }
          for (int i = (int)n - 1; pick < 0 && i >= 0; --i)  // u >= total on an empty last chunk
            if (ck[i] >= thr) pick = ci[i];
          tok[b] = pick;
          gen[(int64_t)b * gen_ld + p] = pick;
        }
        SMP_TICK(5);
      }
      return;
    }
  }

  uint32_t thr = 1;  // keep every real key
  if (top_k > 0 && top_k < V) {
    // exact k-th largest key by bisection over [key(min), key(max)]: the largest K with
    // count(key >= K) >= k; counts from registers, one block reduction per step
    uint32_t lo = ~block_reduce<uint32_t>(~kmin, redu, true), hi = kmax;
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo + 1) / 2;
      uint32_t c = 0;
#pragma unroll
      for (int j = 0; j < SMP_MAXC; ++j) c += key[j] >= mid ? 1u : 0u;
      if (block_reduce<uint32_t>(c, redu, false) >= (uint32_t)top_k)
        lo = mid;
      else
        hi = mid - 1;
    }
    thr = lo;  // the k-th largest key (ties with it are kept)
  }
  float part = 0.0f;
#pragma unroll
  for (int j = 0; j < SMP_MAXC; ++j)
    if (key[j] >= thr) part += exp2f((key_val(key[j]) - m) * scale_log2);
  scan[t] = part;
  __syncthreads();
  // inclusive scan of the per-thread sums (Hillis-Steele over 1024 entries)
  for (int off = 1; off < SMP_THREADS; off <<= 1) {
    const float v = t >= off ? scan[t - off] : 0.0f;
    __syncthreads();
    scan[t] += v;
    __syncthreads();
  }
  const float total = scan[SMP_THREADS - 1];
  const float u = unif * total;
  const float before = t > 0 ? scan[t - 1] : 0.0f;
  // exactly one thread owns the crossing (u in [before, scan[t])); u >= total (rounding)
  // falls to the last thread
  const bool mine = (u >= before && u < scan[t]) || (t == SMP_THREADS - 1 && u >= total);
  if (mine) {
    int pick = -1, tt = t;
    asm volatile("" : "+v"(tt));
    float acc = before;
    bool done = false;
#pragma unroll
    for (int j = 0; j < SMP_MAXC; ++j) {
      if (!done && key[j] >= thr) {
        acc += exp2f((key_val(key[j]) - m) * scale_log2);
        pick = VEC4 ? 4 * ((j >> 2) * SMP_THREADS + tt) + (j & 3) : j * SMP_THREADS + tt;
        done = acc > u;
      }
    }
    if (pick < 0) {  // no kept element in this thread (u >= total on the last one): any kept one
      for (int i = V - 1; i >= 0; --i)
        if (fkey(row[i]) >= thr) {
          pick = i;
          break;
        }
    }
    tok[b] = pick;
    gen[(int64_t)b * gen_ld + p] = pick;
  }
}

// ---------------------------------------------------------------------------
// Decode linear: y[m, n] = act(sum_k x[m, k] W[n, k] + b[n]) for M <= 8 rows (the
// decode batch), bf16 in / out, fp32 accumulation.  At these M every nn.Linear is a
// weight stream: one kernel with the bias (and GELU) in its epilogue replaces the
// library GEMM plus the bias-broadcast copy `addmm` issues, two launches per linear.
// Workgroup = 8 output columns; its 4 waves split K (16-byte pieces: chunk
// g = (it * 4 + wave) * 64 + lane covers k = 8g .. 8g+7), each lane keeps 8 x M partial
// dot products, a butterfly (halve-and-exchange) shuffle reduction leaves each lane
// with one (column, row) total over the wave, and the 4 waves meet in LDS.
// ---------------------------------------------------------------------------
template <int M, int V>
__device__ __forceinline__ float wave_reduce_multi(float (&v)[V], int lane, int& index) {
  // V values per lane -> lane holds the wave-wide sum of value `index`
  int cnt = V;
  index = 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    if (cnt > 1) {
      const bool upper = (lane & off) != 0;
      const int h = cnt / 2;
#pragma unroll
      for (int i = 0; i < V / 2; ++i) {
        if (i < h) {
          const float send = upper ? v[i] : v[i + h];
          const float keep = upper ? v[i + h] : v[i];
          v[i] = keep + __shfl_xor(send, off, 64);
        }
      }
      if (upper) index += h;
      cnt = h;
    } else {
      v[0] += __shfl_xor(v[0], off, 64);
    }
  }
  return v[0];
}

template <int M, int ACT, bool OUTF, int NC = 8>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ W,
                                                   const bf16_t* __restrict__ bias, void* __restrict__ y, int rows,
                                                   int N, int K) {
  constexpr int V = NC * M;
  __shared__ float red[4][V];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.x * NC;
  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.0f;
  const int nchunk = K / 8;
#pragma unroll 4
  for (int g = w * 64 + lane; g < nchunk; g += 256) {
    const int k = 8 * g;
    float xf[M][8];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (m < rows) load8(x + (int64_t)m * K + k, xf[m]);
      else
#pragma unroll
        for (int j = 0; j < 8; ++j) xf[m][j] = 0.0f;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float wf[8];
      load8(W + (int64_t)min(n0 + c, N - 1) * K + k, wf);
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c * M + m] = fmaf(xf[m][j], wf[j], acc[c * M + m]);
    }
  }
  int idx;
  const float v = wave_reduce_multi<M, V>(acc, lane, idx);
  // lanes below the last split's offset hold duplicates: the first of each group writes
  constexpr int DUP = 64 / V;  // lanes per value
  if ((lane & (DUP - 1)) == 0) red[w][idx] = v;
  __syncthreads();
  if (tid < V) {
    const int c = tid / M, m = tid % M, n = n0 + c;
    if (m < rows && n < N) {
      float o = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      if (bias) o += bf2f(bias[n]);
      if (ACT == 1) o = nsa_gelu(o);
      if constexpr (OUTF)
        reinterpret_cast<float*>(y)[(int64_t)m * N + n] = o;
      else
        reinterpret_cast<bf16_t*>(y)[(int64_t)m * N + n] = f2bf(o);
    }
  }
}

// Single-row decode linear with its input's producer in the prologue: every workgroup
// builds the row x[K] (bf16-rounded, in LDS) itself, then streams its NC weight rows:
//   PRO_LN     s = res + branch (fp32; written to res_out by workgroup 0), x = LN(s)
//   PRO_EMB_LN s = wte[*tok] + wpe[*pos] (written to res_out by workgroup 0), x = LN(s)
//   PRO_ATTN   x = the flash-decoding combine of the attention partials (ws, H heads)
//   y = act(x W^T + bias)
// The recomputation is cheap (K <= 8192 values, L2-resident) and removes the separate
// add+LayerNorm / combine / embedding launch per linear: at batch 1 each launch costs a
// few microseconds of fixed overhead against ~1-10 us of weight streaming.  The first
// K piece of the weights is loaded before the prologue, so its latency overlaps it.
// res_out must not alias res.
enum { PRO_LN = 0, PRO_ATTN = 1, PRO_EMB_LN = 2 };

struct RowPro {
  const float* res;
  const bf16_t* branch;
  float* res_out;
  const bf16_t* lw;
  const bf16_t* lb;
  float eps;
  const float* ws;
  int n_split;
  const int64_t* tok;
  const int64_t* pos;
  const bf16_t* wte;
  const bf16_t* wpe;
  int64_t* pos_inc;  // PRO_LN: incremented by one thread after the row (the decode step's position)
};

template <int PRO, int ACT, bool OUTF, int NC>
__global__ __launch_bounds__(256) void gemv_row_kernel(const RowPro a, const bf16_t* __restrict__ W,
                                                       const bf16_t* __restrict__ bias, void* __restrict__ y, int N,
                                                       int K) {
  extern __shared__ float hs[];  // [K] input row
  __shared__ float red[4][NC];
  __shared__ float stat[2][4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nchunk = K / 8, g0 = w * 64 + lane;
  const int nblk = (N + NC - 1) / NC;
  int cb = blockIdx.x;  // column blocks cb, cb + gridDim.x, ...: the prologue runs once per workgroup
  uint4 wp[NC];  // first K piece of the next block's weight rows, in flight ahead of use
  if (g0 < nchunk) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      wp[c] = *reinterpret_cast<const uint4*>(W + (int64_t)min(cb * NC + c, N - 1) * K + 8 * g0);
  }
  // Prologue.  K <= 2048 (every GPT-2 width): thread g owns x[8g .. 8g+7] and issues all
  // of its loads at once (16-byte vectors), so the row costs one memory round trip and
  // two block reductions; wider rows loop.
  const bool vec = K <= 2048;
  const int g8 = 8 * tid;
  const bool own = vec && g8 < K;
  if constexpr (PRO == PRO_ATTN) {
    const int H = K / DA_D, ns = a.n_split;
    float* fs = hs + K;  // [H][ns] chunk weights 2^(m_s - M) / L
    for (int h = tid; h < H; h += 256) {
      const float* part = a.ws + (int64_t)h * ns * DA_PART;
      float M = -INFINITY;
#pragma unroll 4
      for (int sp = 0; sp < ns; ++sp) M = fmaxf(M, part[sp * DA_PART]);
      float L = 0.0f;
#pragma unroll 4
      for (int sp = 0; sp < ns; ++sp) L = fmaf(exp2f(part[sp * DA_PART] - M), part[sp * DA_PART + 1], L);
      const float inv = 1.0f / L;
      for (int sp = 0; sp < ns; ++sp) fs[h * ns + sp] = exp2f(part[sp * DA_PART] - M) * inv;  // empty: 0
    }
    __syncthreads();
    for (int k0 = g8; k0 < K; k0 += 8 * 256) {  // 8 dims of one head per thread and pass
      const int h = k0 / DA_D;
      const float* o = a.ws + (int64_t)h * ns * DA_PART + DA_PO + (k0 % DA_D);
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int sp = 0; sp < ns; ++sp) {
        const float f = fs[h * ns + sp];
        const float4 u0 = *reinterpret_cast<const float4*>(o + sp * DA_PART);
        const float4 u1 = *reinterpret_cast<const float4*>(o + sp * DA_PART + 4);
        acc[0] = fmaf(f, u0.x, acc[0]);
        acc[1] = fmaf(f, u0.y, acc[1]);
        acc[2] = fmaf(f, u0.z, acc[2]);
        acc[3] = fmaf(f, u0.w, acc[3]);
        acc[4] = fmaf(f, u1.x, acc[4]);
        acc[5] = fmaf(f, u1.y, acc[5]);
        acc[6] = fmaf(f, u1.z, acc[6]);
        acc[7] = fmaf(f, u1.w, acc[7]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) hs[k0 + e] = bf2f(f2bf(acc[e]));  // the bf16 attention output
    }
  } else {
    const bool write_s = PRO == PRO_EMB_LN || a.branch != nullptr;
    int64_t te = 0, pe = 0;
    if constexpr (PRO == PRO_EMB_LN) {
      te = *a.tok;
      pe = *a.pos;
    }
    float xv[8], lwv[8], lbv[8];
    float sum = 0.0f;
    if (vec) {
#pragma unroll
      for (int e = 0; e < 8; ++e) xv[e] = lwv[e] = lbv[e] = 0.0f;
      if (own) {
        if constexpr (PRO == PRO_EMB_LN) {
          float e0[8], e1[8];
          load8(a.wte + te * K + g8, e0);
          load8(a.wpe + pe * K + g8, e1);
#pragma unroll
          for (int e = 0; e < 8; ++e) xv[e] = e0[e] + e1[e];
        } else {
          const float4 r0 = *reinterpret_cast<const float4*>(a.res + g8);
          const float4 r1 = *reinterpret_cast<const float4*>(a.res + g8 + 4);
          xv[0] = r0.x; xv[1] = r0.y; xv[2] = r0.z; xv[3] = r0.w;
          xv[4] = r1.x; xv[5] = r1.y; xv[6] = r1.z; xv[7] = r1.w;
          if (a.branch) {
            float bv[8];
            load8(a.branch + g8, bv);
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[e] += bv[e];
          }
        }
        load8(a.lw + g8, lwv);
        if (a.lb) load8(a.lb + g8, lbv);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) sum += xv[e];
    } else {
      for (int k = tid; k < K; k += 256) {
        float v;
        if constexpr (PRO == PRO_EMB_LN) {
          v = bf2f(a.wte[te * K + k]) + bf2f(a.wpe[pe * K + k]);
        } else {
          v = a.res[k];
          if (a.branch) v += bf2f(a.branch[k]);
        }
        hs[k] = v;
        sum += v;
      }
    }
    sum = wave_sum(sum);
    if (lane == 0) stat[0][w] = sum;
    __syncthreads();
    const float mean = (stat[0][0] + stat[0][1] + stat[0][2] + stat[0][3]) / (float)K;
    float sq = 0.0f;
    if (vec) {
      if (own)
#pragma unroll
        for (int e = 0; e < 8; ++e) sq = fmaf(xv[e] - mean, xv[e] - mean, sq);
    } else {
      for (int k = tid; k < K; k += 256) {
        const float d = hs[k] - mean;
        sq = fmaf(d, d, sq);
      }
    }
    sq = wave_sum(sq);
    if (lane == 0) stat[1][w] = sq;
    __syncthreads();
    const float rstd = rsqrtf((stat[1][0] + stat[1][1] + stat[1][2] + stat[1][3]) / (float)K + a.eps);
    if (vec) {
      if (own) {
        if (blockIdx.x == 0 && write_s) {
          *reinterpret_cast<float4*>(a.res_out + g8) = make_float4(xv[0], xv[1], xv[2], xv[3]);
          *reinterpret_cast<float4*>(a.res_out + g8 + 4) = make_float4(xv[4], xv[5], xv[6], xv[7]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) hs[g8 + e] = bf2f(f2bf((xv[e] - mean) * rstd * lwv[e] + lbv[e]));
      }
    } else {
      for (int k = tid; k < K; k += 256) {
        const float sv = hs[k];
        if (blockIdx.x == 0 && write_s) a.res_out[k] = sv;
        float h = (sv - mean) * rstd * bf2f(a.lw[k]);
        if (a.lb) h += bf2f(a.lb[k]);
        hs[k] = bf2f(f2bf(h));  // the bf16 activation the LayerNorm kernel would hand the GEMM
      }
    }
  }
  __syncthreads();
  for (; cb < nblk; cb += gridDim.x) {
    const int n0 = cb * NC;
    float acc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = 0.0f;
    if (g0 < nchunk) {
      float xf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) xf[j] = hs[8 * g0 + j];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        float wf[8];
        unpack8(wp[c], wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c] = fmaf(xf[j], wf[j], acc[c]);
      }
    }
    for (int g = g0 + 256; g < nchunk; g += 256) {
      const int k = 8 * g;
      float xf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) xf[j] = hs[k + j];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        float wf[8];
        load8(W + (int64_t)min(n0 + c, N - 1) * K + k, wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c] = fmaf(xf[j], wf[j], acc[c]);
      }
    }
    const int nb = cb + gridDim.x;
    if (nb < nblk && g0 < nchunk) {  // next block's first piece: in flight during the reduction
#pragma unroll
      for (int c = 0; c < NC; ++c)
        wp[c] = *reinterpret_cast<const uint4*>(W + (int64_t)min(nb * NC + c, N - 1) * K + 8 * g0);
    }
    int idx;
    const float v = wave_reduce_multi<1, NC>(acc, lane, idx);
    if ((lane & (64 / NC - 1)) == 0) red[w][idx] = v;
    __syncthreads();
    if (tid < NC) {
      const int n = n0 + tid;
      if (n < N) {
        float o = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
        if (bias) o += bf2f(bias[n]);
        if (ACT == 1) o = nsa_gelu(o);
        if constexpr (OUTF)
          reinterpret_cast<float*>(y)[n] = o;
        else
          reinterpret_cast<bf16_t*>(y)[n] = f2bf(o);
      }
    }
    __syncthreads();  // red[] is rewritten by the next block
  }
  if constexpr (PRO == PRO_LN)
    if (a.pos_inc && blockIdx.x == 0 && tid == 0) *a.pos_inc += 1;
}

// NSA_GEMV_GRID: workgroup cap of the single-row GEMVs (default 1024: 4 per CU);
// NSA_GEMV_NC: output columns per workgroup block (2, 4, 8 or 16)
int gemv_row_grid() {
  static const int g = [] {
    const char* e = getenv("NSA_GEMV_GRID");
    return e ? std::max(1, atoi(e)) : 1024;
  }();
  return g;
}
int env_nc(const char* name) {  // 0: unset
  const char* e = getenv(name);
  const int v = e ? atoi(e) : 0;
  return v == 2 || v == 4 || v == 8 || v == 16 ? v : 0;
}
int gemv_row_nc() {  // default 4: measured per-token decode (graph) 124M 0.372 / 1.5B 2.065 ms at 8, 0.336 / 1.901 at 4
  static const int n = env_nc("NSA_GEMV_NC");
  return n ? n : 4;
}

// NSA_GEMV1_NC: columns per workgroup of the plain one-row GEMV (default 2: the narrow
// MLP down-projection, N = C, gets C / 2 workgroups; 4 / 8 measured 1-3% slower per token)
int gemv1_nc(int N) {
  static const int n = env_nc("NSA_GEMV1_NC");
  (void)N;
  return n ? n : 2;
}

template <int PRO>
hipError_t launch_gemv_row(const RowPro& a, const void* W, const void* bias, void* y, int N, int K, int act,
                           int out_f32, hipStream_t s) {
  // the row, plus the chunk weights of the attention combine
  const size_t lds = (size_t)(K + (PRO == PRO_ATTN ? (K / DA_D) * a.n_split : 0)) * sizeof(float);
  const bf16_t* w = (const bf16_t*)W;
  const bf16_t* b = (const bf16_t*)bias;
  // at most gemv_row_grid() workgroups, each looping over column blocks (the vocabulary
  // head: ~6 blocks per workgroup instead of one prologue per 8 columns)
  const int nc = gemv_row_nc();
  const int nblk = (N + nc - 1) / nc;
  const unsigned grid = (unsigned)std::min(nblk, gemv_row_grid());
#define NSA_ROW(NC_)                                                                      \
  do {                                                                                    \
    if (act)                                                                              \
      gemv_row_kernel<PRO, 1, false, NC_><<<grid, 256, lds, s>>>(a, w, b, y, N, K);      \
    else if (out_f32)                                                                     \
      gemv_row_kernel<PRO, 0, true, NC_><<<grid, 256, lds, s>>>(a, w, b, y, N, K);       \
    else                                                                                  \
      gemv_row_kernel<PRO, 0, false, NC_><<<grid, 256, lds, s>>>(a, w, b, y, N, K);      \
  } while (0)
  if (nc == 16)
    NSA_ROW(16);
  else if (nc == 4)
    NSA_ROW(4);
  else if (nc == 2)
    NSA_ROW(2);
  else
    NSA_ROW(8);
#undef NSA_ROW
  return hipGetLastError();
}

}  // namespace

// K/V rows of qkv [B, S, 3C] -> caches [B, H, Tmax, D] at positions p0 .. p0+S-1 where
// p0 = *pos (int64 device scalar) or, with pos == NULL, the host value pos0.
NSA_API hipError_t nsa_kv_append(const void* qkv, void* kc, void* vc, const void* pos, int pos0, int B, int S, int H,
                                 int D, int Tmax, hipStream_t s) {
  if (D % 8 || B < 1 || S < 1) return hipErrorInvalidValue;
  const int64_t total = (int64_t)B * S * 2 * H * (D / 8);
  kv_append_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(
      (const bf16_t*)qkv, (bf16_t*)kc, (bf16_t*)vc, (const int64_t*)pos, pos0, B, S, H, D, Tmax);
  return hipGetLastError();
}

// Single-query causal attention of the newest token (position *pos) over the caches.
// qkv: [B, 1, 3C] (q | k | v); out: [B, C] bf16; ws: B*H*ceil(Tmax/256)*68 fp32.
// append != 0: the new token's K / V are taken from qkv and stored at *pos (fused
// kv_append); otherwise the caches must already hold position *pos.  out == NULL leaves
// the partials in ws for nsa_gemv_attn.
NSA_API hipError_t nsa_decode_attn(const void* qkv, void* kc, void* vc, const void* pos, void* ws, void* out, int B,
                                   int H, int D, int Tmax, float scale, int append, hipStream_t s) {
  if (D != DA_D || B < 1 || H < 1 || Tmax < 1) return hipErrorInvalidValue;
  const int n_split = (Tmax + DA_CHUNK - 1) / DA_CHUNK;
  decode_attn_partial_kernel<<<dim3(B * H, n_split), 256, 0, s>>>(
      (const bf16_t*)qkv, (const bf16_t*)kc, (const bf16_t*)vc, (bf16_t*)kc, (bf16_t*)vc, (const int64_t*)pos,
      (float*)ws, H, Tmax, scale * 1.4426950408889634f, append);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || !out) return e;  // out == NULL: the consumer combines (nsa_gemv_attn)
  decode_attn_combine_kernel<<<B * H, 64, 0, s>>>((const float*)ws, (bf16_t*)out, H, n_split);
  return hipGetLastError();
}

// Top-k / temperature sampling of logits [B, V] (fp32, row stride ld) on the device:
// writes tok[b] and gen[b * gen_ld + *pos].  top_k <= 0 keeps every logit.  The uniform is a
// counter hash of (salt ^ *salt_dev, row, position); salt_dev may be NULL.
NSA_API hipError_t nsa_sample_topk(const void* logits, int B, int V, int ld, float temperature, int top_k,
                                   uint64_t salt, const void* salt_dev, const void* pos, void* tok, void* gen,
                                   int gen_ld, hipStream_t s) {
  if (B < 1 || V < 1 || V > SMP_THREADS * SMP_MAXC || !(temperature > 0.0f)) return hipErrorInvalidValue;
  const bool vec4 = V % 4 == 0 && ld % 4 == 0 && ((uintptr_t)logits & 15) == 0;
  if (vec4)
    sample_topk_kernel<true><<<B, SMP_THREADS, 0, s>>>((const float*)logits, V, ld, 1.4426950408889634f / temperature,
                                                       top_k, salt, (const uint64_t*)salt_dev, (const int64_t*)pos,
                                                       (int64_t*)tok, (int64_t*)gen, gen_ld);
  else
    sample_topk_kernel<false><<<B, SMP_THREADS, 0, s>>>((const float*)logits, V, ld, 1.4426950408889634f / temperature,
                                                        top_k, salt, (const uint64_t*)salt_dev, (const int64_t*)pos,
                                                        (int64_t*)tok, (int64_t*)gen, gen_ld);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Decode linear for a batch of 2 .. 64 rows on the matrix cores ("skinny GEMM").
// The vector GEMV keeps 8 x M fp32 partial dot products per lane and reduces them by
// shuffles, so its VALU cost grows with M; in round 2, from 2 rows on, the then-used
// library GEMM beat it while running at a few % of the MFMA rate (GPT-2 1.5B batch 8
// decoded at 4.2 ms/token against 1.9 at batch 1; no library GEMM is on this path any
// more: M > SKINNY_MAX_ROWS goes to our small-tile / NT kernels).  Here the weight is
// streamed once through v_mfma_f32_16x16x32_bf16 with the roles swapped:
//   Y^T[n, m] = W[n, k] · X^T[k, m]      A = 16 weight rows (lane l: row n0 + (l & 15),
//                                         16 contiguous bytes of it), B = X^T (lane l:
//                                         batch row m = l & 15 of a 16-row group),
// so every lane's weight load is a 16-byte piece of one weight row, and MT 16-row
// groups of X share each weight fragment.  Workgroup = 16 output columns; its NW = 4 waves
// take interleaved 32-wide K units (8 in flight per wave), then meet in
// LDS; the epilogue adds the bias, applies exact-erf GELU and stores Y[m, n] for m < M.
// Rows past M read row M - 1 (valid memory) and are never stored.
// ---------------------------------------------------------------------------
template <int MT, int ACT, bool OUTF, int NW = 4>
__global__ __launch_bounds__(NW * 64) void skinny_gemm_kernel(const bf16_t* __restrict__ x,
                                                              const bf16_t* __restrict__ W,
                                                              const bf16_t* __restrict__ bias, void* __restrict__ yv,
                                                              int M, int N, int K) {
  __shared__ float red[NW][MT][4][64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.x * 16;
  const int g = lane >> 4, c = lane & 15;
  const bf16_t* wrow = W + (int64_t)(n0 + c) * K + 8 * g;
  const bf16_t* xrow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) xrow[t] = x + (int64_t)min(16 * t + c, M - 1) * K + 8 * g;
  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{};
  const int U = K / 32;  // 32-wide K units; wave w takes units w, w + NW, w + 2 NW, ...
  // UN units per wave in flight; units past the end re-read the last unit with a zero
  // weight fragment (branch-free, so every load of an iteration issues before any wait)
  constexpr int UN = 8;
  for (int u0 = w; u0 < U; u0 += NW * UN) {
    uint4 a[UN], b[UN][MT];
#pragma unroll
    for (int j = 0; j < UN; ++j) {
      const int uu = u0 + NW * j;
      const int uc = uu < U ? uu : U - 1;
      a[j] = *reinterpret_cast<const uint4*>(wrow + 32 * uc);
      if (uu >= U) a[j] = uint4{0u, 0u, 0u, 0u};
#pragma unroll
      for (int t = 0; t < MT; ++t) b[j][t] = *reinterpret_cast<const uint4*>(xrow[t] + 32 * uc);
    }
#pragma unroll
    for (int j = 0; j < UN; ++j)
#pragma unroll
      for (int t = 0; t < MT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[j]),
                                                         __builtin_bit_cast(bf16x8, b[j][t]), acc[t], 0, 0, 0);
  }
  // C layout: lane l holds column m = l & 15 of the 16-row group, rows n = 4 (l >> 4) + i
#pragma unroll
  for (int t = 0; t < MT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[w][t][i][lane] = acc[t][i];
  __syncthreads();
  // 16 columns x 16 MT batch rows: thread e -> (m, n) with n fastest (coalesced stores)
  for (int e = tid; e < 16 * 16 * MT; e += NW * 64) {
    const int n = e & 15, m = e >> 4;
    if (m >= M) break;
    const int t = m >> 4, mc = m & 15;
    const int i = n & 3, ln = 16 * (n >> 2) + mc;
    float v = 0.0f;
#pragma unroll
    for (int q = 0; q < NW; ++q) v += red[q][t][i][ln];
    if (bias) v += bf2f(bias[n0 + n]);
    if constexpr (ACT == 1) v = nsa_gelu(v);
    if constexpr (OUTF)
      reinterpret_cast<float*>(yv)[(int64_t)m * N + n0 + n] = v;
    else
      reinterpret_cast<bf16_t*>(yv)[(int64_t)m * N + n0 + n] = f2bf(v);
  }
}

// y[rows, N] = act(x[rows, K] W[N, K]^T + b) for 2 <= rows <= 64 (N % 16 == 0, K % 32 == 0)
NSA_API hipError_t nsa_skinny_gemm(const void* x, const void* W, const void* bias, void* y, int rows, int N, int K,
                                   int act, int out_f32, hipStream_t s) {
  if (rows < 1 || rows > 64 || N % 16 || K % 32 || N < 16 || K < 32 || (act && out_f32)) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)(N / 16);
#define NSA_SKINNY(MT)                                                                                            \
  do {                                                                                                            \
    if (act)                                                                                                      \
      skinny_gemm_kernel<MT, 1, false><<<grid, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias, \
                                                            y, rows, N, K);                                       \
    else if (out_f32)                                                                                             \
      skinny_gemm_kernel<MT, 0, true><<<grid, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias,  \
                                                           y, rows, N, K);                                        \
    else                                                                                                          \
      skinny_gemm_kernel<MT, 0, false><<<grid, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias, \
                                                            y, rows, N, K);                                       \
  } while (0)
  // NW = 16 waves per workgroup (1024 threads) measured slower in the decode graph: GPT-2
  // 124M / 1.5B batch 8 0.733 / 3.84 ms/token vs 0.532 / 3.34 with NW = 4
  if (rows <= 16) NSA_SKINNY(1);
  else if (rows <= 32) NSA_SKINNY(2);
  else NSA_SKINNY(4);
#undef NSA_SKINNY
  return hipGetLastError();
}

// Skinny GEMM with the residual add + LayerNorm in the prologue (decode batches of
// 2..16 rows, the batch counterpart of gemv_row_kernel<PRO_LN>): every workgroup forms
// s = res + branch and x = LN(s) for all rows itself (wave w: rows w, w + 4, ...; a row of
// K <= 2048 lives in 32 registers per lane, two-pass mean / variance as nanoGPT's fp32
// LayerNorm), stores x as bf16 in LDS ([16][K + 8], padded rows) and reads the MFMA B
// fragments from there; workgroup 0 writes s (fp32).  The first round of weight loads is
// issued before the prologue and each round prefetches the next, so the weight stream
// overlaps the LayerNorm.  Removes the separate add+LayerNorm launch per linear.
__device__ __forceinline__ float sk_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int ACT, bool OUTF>
__global__ __launch_bounds__(256) void skinny_ln_gemm_kernel(const float* __restrict__ res,
                                                             const bf16_t* __restrict__ branch,
                                                             float* __restrict__ s_out, const bf16_t* __restrict__ lw,
                                                             const bf16_t* __restrict__ lb, float eps,
                                                             const bf16_t* __restrict__ W,
                                                             const bf16_t* __restrict__ bias, void* __restrict__ yv,
                                                             int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) bf16_t xs[];  // [16][K + 8]
  __shared__ float red[4][4][64];
  const int KP = K + 8;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.x * 16;
  const int g = lane >> 4, c = lane & 15;
  const bf16_t* wrow = W + (int64_t)(n0 + c) * K + 8 * g;
  const int U = K / 32;
  constexpr int UN = 8;
  uint4 a[UN];
  auto load_a = [&](int u0, uint4 (&dst)[UN]) {
#pragma unroll
    for (int j = 0; j < UN; ++j) {
      const int uu = u0 + 4 * j;
      dst[j] = *reinterpret_cast<const uint4*>(wrow + 32 * (uu < U ? uu : U - 1));
      if (uu >= U) dst[j] = uint4{0u, 0u, 0u, 0u};
    }
  };
  load_a(w, a);
  // prologue: LayerNorm of the M batch rows into LDS; rows M..15 are zeroed (they only feed
  // output columns m >= M, which are never stored)
  for (int m = M + w; m < 16; m += 4)
    for (int k = 8 * lane; k < K; k += 512) *reinterpret_cast<uint4*>(xs + m * KP + k) = uint4{0u, 0u, 0u, 0u};
  for (int m = w; m < M; m += 4) {
    const int mm = m;
    float v[4][8];
    float sum = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = (q * 64 + lane) * 8;
      if (k < K) {
        const float4 r0 = *reinterpret_cast<const float4*>(res + (int64_t)mm * K + k);
        const float4 r1 = *reinterpret_cast<const float4*>(res + (int64_t)mm * K + k + 4);
        v[q][0] = r0.x; v[q][1] = r0.y; v[q][2] = r0.z; v[q][3] = r0.w;
        v[q][4] = r1.x; v[q][5] = r1.y; v[q][6] = r1.z; v[q][7] = r1.w;
        if (branch) {
          float bv[8];
          load8(branch + (int64_t)mm * K + k, bv);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[q][e] += bv[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) sum += v[q][e];
      }
    }
    const float mean = sk_wave_sum(sum) / (float)K;
    float sq = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if ((q * 64 + lane) * 8 < K)
#pragma unroll
        for (int e = 0; e < 8; ++e) sq = fmaf(v[q][e] - mean, v[q][e] - mean, sq);
    const float rstd = rsqrtf(sk_wave_sum(sq) / (float)K + eps);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = (q * 64 + lane) * 8;
      if (k < K) {
        float wv[8], bv[8], o[8];
        load8(lw + k, wv);
        if (lb) {
          load8(lb + k, bv);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) bv[e] = 0.0f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (v[q][e] - mean) * rstd * wv[e] + bv[e];
        store8(xs + m * KP + k, o);
        if (blockIdx.x == 0 && s_out && m < M) {
          float* sp = s_out + (int64_t)m * K + k;
          *reinterpret_cast<float4*>(sp) = make_float4(v[q][0], v[q][1], v[q][2], v[q][3]);
          *reinterpret_cast<float4*>(sp + 4) = make_float4(v[q][4], v[q][5], v[q][6], v[q][7]);
        }
      }
    }
  }
  __syncthreads();
  f32x4 acc = f32x4{};
  for (int u0 = w; u0 < U; u0 += 4 * UN) {
    uint4 b[UN];
#pragma unroll
    for (int j = 0; j < UN; ++j) {
      const int uu = u0 + 4 * j;
      b[j] = *reinterpret_cast<const uint4*>(xs + c * KP + 32 * (uu < U ? uu : U - 1) + 8 * g);
    }
    uint4 an[UN];
    const bool more = u0 + 4 * UN < U;  // wave-uniform
    if (more) load_a(u0 + 4 * UN, an);
#pragma unroll
    for (int j = 0; j < UN; ++j)
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a[j]), __builtin_bit_cast(bf16x8, b[j]),
                                                    acc, 0, 0, 0);
    if (more) {
#pragma unroll
      for (int j = 0; j < UN; ++j) a[j] = an[j];
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[w][i][lane] = acc[i];
  __syncthreads();
  {
    const int e = tid, n = e & 15, m = e >> 4;
    if (m < M) {
      const int i = n & 3, ln = 16 * (n >> 2) + m;
      float o = red[0][i][ln] + red[1][i][ln] + red[2][i][ln] + red[3][i][ln];
      if (bias) o += bf2f(bias[n0 + n]);
      if constexpr (ACT == 1) o = nsa_gelu(o);
      if constexpr (OUTF)
        reinterpret_cast<float*>(yv)[(int64_t)m * N + n0 + n] = o;
      else
        reinterpret_cast<bf16_t*>(yv)[(int64_t)m * N + n0 + n] = f2bf(o);
    }
  }
}

// (s, y) for 2..16 decode rows: s = res + branch (fp32, branch bf16 or NULL: s_out unused),
// y = act(LN(s) W^T + b); N % 16 == 0, K % 32 == 0, K <= 1920 (LDS image [16][K + 8] bf16)
NSA_API hipError_t nsa_skinny_ln_gemm(const void* res, const void* branch, void* s_out, const void* lw,
                                      const void* lb, float eps, const void* W, const void* bias, void* y, int rows,
                                      int N, int K, int act, int out_f32, hipStream_t s) {
  if (rows < 1 || rows > 16 || N % 16 || K % 32 || N < 16 || K < 32 || K > 1920 || (act && out_f32) ||
      (branch && !s_out))
    return hipErrorInvalidValue;
  const unsigned grid = (unsigned)(N / 16);
  const size_t lds = (size_t)16 * (K + 8) * sizeof(bf16_t);
#define NSA_SKLN(A, F)                                                                                    \
  skinny_ln_gemm_kernel<A, F><<<grid, 256, lds, s>>>((const float*)res, (const bf16_t*)branch, (float*)s_out, \
                                                     (const bf16_t*)lw, (const bf16_t*)lb, eps, (const bf16_t*)W, \
                                                     (const bf16_t*)bias, y, rows, N, K)
  if (act) NSA_SKLN(1, false);
  else if (out_f32) NSA_SKLN(0, true);
  else NSA_SKLN(0, false);
#undef NSA_SKLN
  return hipGetLastError();
}

// Decode-batch linear y[rows, N] = act(x[rows, K] W[N, K]^T + b), rows <= 8, K % 8 == 0;
// act: 0 none, 1 exact-erf GELU; out_f32: y is fp32 (e.g. logits) instead of bf16.
// bias may be NULL.
NSA_API hipError_t nsa_gemv(const void* x, const void* W, const void* bias, void* y, int rows, int N, int K, int act,
                            int out_f32, hipStream_t s) {
  if (rows < 1 || rows > 8 || K % 8 || N < 1 || (act && out_f32)) return hipErrorInvalidValue;
  const unsigned grid = (unsigned)((N + 7) / 8);
#define NSA_GEMV(MR)                                                                                        \
  do {                                                                                                      \
    if (act)                                                                                                \
      gemv_kernel<MR, 1, false><<<grid, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias, \
                                                     y, rows, N, K);                                        \
    else if (out_f32)                                                                                       \
      gemv_kernel<MR, 0, true><<<grid, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias,  \
                                                    y, rows, N, K);                                         \
    else                                                                                                    \
      gemv_kernel<MR, 0, false><<<grid, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias, \
                                                     y, rows, N, K);                                        \
  } while (0)
  if (rows == 1) {
    // one row: NC columns per workgroup (narrow outputs need more, smaller workgroups to
    // keep enough weight bytes in flight)
    const int nc = gemv1_nc(N);
    const unsigned g1 = (unsigned)((N + nc - 1) / nc);
#define NSA_GEMV1(NC_)                                                                                       \
  do {                                                                                                       \
    if (act)                                                                                                 \
      gemv_kernel<1, 1, false, NC_><<<g1, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias, \
                                                       y, 1, N, K);                                          \
    else if (out_f32)                                                                                        \
      gemv_kernel<1, 0, true, NC_><<<g1, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias,  \
                                                      y, 1, N, K);                                           \
    else                                                                                                     \
      gemv_kernel<1, 0, false, NC_><<<g1, 256, 0, s>>>((const bf16_t*)x, (const bf16_t*)W, (const bf16_t*)bias, \
                                                       y, 1, N, K);                                          \
  } while (0)
    if (nc == 2) NSA_GEMV1(2);
    else if (nc == 4) NSA_GEMV1(4);
    else NSA_GEMV1(8);
#undef NSA_GEMV1
  } else if (rows == 2) NSA_GEMV(2);
  else if (rows <= 4) NSA_GEMV(4);
  else NSA_GEMV(8);
#undef NSA_GEMV
  return hipGetLastError();
}

// One decode row: res_out = res + branch (if branch), h = LN(res [+ branch]) with (lw, lb),
// y = act(h W^T + bias) (fp32 y with out_f32).  K % 8 == 0, K <= 8192; res_out must not
// alias res.  pos_inc (may be NULL): an int64 the kernel increments once (the decode
// position, advanced by the step's last kernel instead of a separate add launch).
NSA_API hipError_t nsa_gemv_ln(const void* res, const void* branch, void* res_out, const void* lw, const void* lb,
                               const void* W, const void* bias, void* y, int N, int K, float eps, int act,
                               int out_f32, void* pos_inc, hipStream_t s) {
  if (K % 8 || K > 8192 || N < 1 || (act && out_f32) || (branch && (!res_out || res_out == res)))
    return hipErrorInvalidValue;
  RowPro a{};
  a.res = (const float*)res;
  a.branch = (const bf16_t*)branch;
  a.res_out = (float*)res_out;
  a.lw = (const bf16_t*)lw;
  a.lb = (const bf16_t*)lb;
  a.eps = eps;
  a.pos_inc = (int64_t*)pos_inc;
  return launch_gemv_row<PRO_LN>(a, W, bias, y, N, K, act, out_f32, s);
}

// First decode linear of a single-row step: res_out = wte[*tok] + wpe[*pos] (fp32, the
// residual stream), y = act(LN(res_out) W^T + bias).
NSA_API hipError_t nsa_gemv_emb_ln(const void* tok, const void* pos, const void* wte, const void* wpe, void* res_out,
                                   const void* lw, const void* lb, const void* W, const void* bias, void* y, int N,
                                   int K, float eps, int act, int out_f32, hipStream_t s) {
  if (K % 8 || K > 8192 || N < 1 || (act && out_f32) || !res_out) return hipErrorInvalidValue;
  RowPro a{};
  a.res_out = (float*)res_out;
  a.lw = (const bf16_t*)lw;
  a.lb = (const bf16_t*)lb;
  a.eps = eps;
  a.tok = (const int64_t*)tok;
  a.pos = (const int64_t*)pos;
  a.wte = (const bf16_t*)wte;
  a.wpe = (const bf16_t*)wpe;
  return launch_gemv_row<PRO_EMB_LN>(a, W, bias, y, N, K, act, out_f32, s);
}

// Single-row linear over the attention output: x = combine of the decode-attention
// partials ws (nsa_decode_attn with out == NULL, batch 1), K = H * 64.
NSA_API hipError_t nsa_gemv_attn(const void* ws, int n_split, const void* W, const void* bias, void* y, int N, int K,
                                 int act, int out_f32, hipStream_t s) {
  if (K % DA_D || K > 8192 || N < 1 || n_split < 1 || (K / DA_D) * n_split > 16384 || (act && out_f32))
    return hipErrorInvalidValue;
  RowPro a{};
  a.ws = (const float*)ws;
  a.n_split = n_split;
  return launch_gemv_row<PRO_ATTN>(a, W, bias, y, N, K, act, out_f32, s);
}

#ifdef NSA_SMP_TIMING
NSA_API hipError_t nsa_smp_ticks(uint64_t* host) { return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_smp_ticks), sizeof(uint64_t) * 8); }
#endif
