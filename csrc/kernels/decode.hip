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

namespace {

constexpr int DA_D = 64;        // head dim of the decode-attention kernel
constexpr int DA_CHUNK = 256;   // keys per workgroup (one per thread)
constexpr int DA_PART = 2 + DA_D;  // m, l, o[64]

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
  // weighted V sum: wave w covers keys k0 + 64w .. +63, lane = output dim
  const int kw0 = k0 + 64 * w;
  const int kend = min(64, pos - kw0 + 1);          // live keys of this wave (may be <= 0)
  const bool new_here = append && pos < kw0 + 64 && kend > 0;  // the new token is its last live key
  const bf16_t* vrow = vc + ((int64_t)bh * Tmax + kw0) * DA_D + lane;
  float o = 0.0f;
  for (int j = 0; j < kend - (new_here ? 1 : 0); ++j) o = fmaf(ps[64 * w + j], bf2f(vrow[(int64_t)j * DA_D]), o);
  if (new_here) o = fmaf(ps[64 * w + kend - 1], bf2f(qrow[2 * C + lane]), o);  // its V row from qkv
  os[w][lane] = o;
  __syncthreads();
  if (tid < DA_D) part[2 + tid] = os[0][tid] + os[1][tid] + os[2][tid] + os[3][tid];
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
    o = fmaf(f, part[s * DA_PART + 2 + d], o);
  }
  out[(int64_t)b * H * DA_D + hh * DA_D + d] = f2bf(o / L);
}

// ---------------------------------------------------------------------------
// Sampling (nanoGPT sample.py: logits / temperature, keep the top_k, softmax,
// multinomial) for one row per workgroup, fully on the device so the decode graph can
// feed the sampled token back without a host round trip (torch's topk / multinomial
// chain is ~20 launches and its segmented sort is not graph-replay safe here).
//  1. row max M;
//  2. top-k threshold: bisection over the order-preserving uint32 image of the logits
//     (held in registers: a 1024-thread workgroup keeps up to 52 per thread), the
//     k-th largest key K; ties with it are kept, as with torch's `logits < v[:, [-1]]`
//     mask (an LDS-atomic radix select measured 156 us at V = 50304: one hot bin per
//     digit pass serialises the atomics);
//  3. w_i = exp2((l_i - M) * log2(e) / temperature) for kept i, S = sum w_i;
//  4. u = uniform * S from the counter hash (salt, b, position), and the first index
//     whose running sum of w exceeds u (per-thread contiguous chunks + an LDS scan).
// The chosen id is written to tok[b] and gen[b, *pos].
// ---------------------------------------------------------------------------
constexpr int SMP_THREADS = 1024;

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

constexpr int SMP_MAXC = 52;  // logits per thread kept in registers (V <= 53248: the GPT-2 vocab is 50304)

__global__ __launch_bounds__(SMP_THREADS) void sample_topk_kernel(const float* __restrict__ logits, int V, int ld,
                                                                  float scale_log2, int top_k, uint64_t salt,
                                                                  const int64_t* __restrict__ pos,
                                                                  int64_t* __restrict__ tok, int64_t* __restrict__ gen,
                                                                  int gen_ld) {
  __shared__ uint32_t redu[SMP_THREADS / 64];
  __shared__ float scan[SMP_THREADS];
  const int b = blockIdx.x, t = threadIdx.x;
  const float* row = logits + (int64_t)b * ld;
  const int chunk = (V + SMP_THREADS - 1) / SMP_THREADS;
  const int i0 = min(V, t * chunk), n = min(V, i0 + chunk) - i0;
  // the thread's contiguous chunk stays in registers (as order-preserving keys; key 0 =
  // padding, below every real key) for every pass below
  uint32_t key[SMP_MAXC];
  uint32_t kmax = 0, kmin = 0xffffffffu;
#pragma unroll
  for (int j = 0; j < SMP_MAXC; ++j) {
    key[j] = j < n ? fkey(row[i0 + j]) : 0u;
    if (j < n) {
      kmax = max(kmax, key[j]);
      kmin = min(kmin, key[j]);
    }
  }
  kmax = block_reduce<uint32_t>(kmax, redu, true);
  const float m = key_val(kmax);
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
  const int p = (int)*pos;
  const uint32_t h = nsa_hash(nsa_seed(salt), (uint64_t)b * 0x9E3779B97F4A7C15ull + (uint64_t)p);
  const float u = (float)(h >> 8) * (1.0f / 16777216.0f) * total;
  const float before = t > 0 ? scan[t - 1] : 0.0f;
  // exactly one thread owns the crossing (u in [before, scan[t])); u >= total (rounding)
  // falls to the last thread with mass
  const bool mine = (u >= before && u < scan[t]) || (t == SMP_THREADS - 1 && u >= total);
  if (mine) {
    int pick = -1;
    float acc = before;
    bool done = false;
#pragma unroll
    for (int j = 0; j < SMP_MAXC; ++j) {
      if (!done && key[j] >= thr) {
        acc += exp2f((key_val(key[j]) - m) * scale_log2);
        pick = i0 + j;
        done = acc > u;
      }
    }
    if (pick < 0) {  // no kept element in this chunk (u >= total on the last thread): last kept overall
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

template <int M, int ACT, bool OUTF>
__global__ __launch_bounds__(256) void gemv_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ W,
                                                   const bf16_t* __restrict__ bias, void* __restrict__ y, int rows,
                                                   int N, int K) {
  constexpr int NC = 8, V = NC * M;
  __shared__ float red[4][V];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n0 = blockIdx.x * NC;
  float acc[V];
#pragma unroll
  for (int i = 0; i < V; ++i) acc[i] = 0.0f;
  const int nchunk = K / 8;
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
// qkv: [B, 1, 3C] (q | k | v); out: [B, C] bf16; ws: B*H*ceil(Tmax/256)*66 fp32.
// append != 0: the new token's K / V are taken from qkv and stored at *pos (fused
// kv_append); otherwise the caches must already hold position *pos.
NSA_API hipError_t nsa_decode_attn(const void* qkv, void* kc, void* vc, const void* pos, void* ws, void* out, int B,
                                   int H, int D, int Tmax, float scale, int append, hipStream_t s) {
  if (D != DA_D || B < 1 || H < 1 || Tmax < 1) return hipErrorInvalidValue;
  const int n_split = (Tmax + DA_CHUNK - 1) / DA_CHUNK;
  decode_attn_partial_kernel<<<dim3(B * H, n_split), 256, 0, s>>>(
      (const bf16_t*)qkv, (const bf16_t*)kc, (const bf16_t*)vc, (bf16_t*)kc, (bf16_t*)vc, (const int64_t*)pos,
      (float*)ws, H, Tmax, scale * 1.4426950408889634f, append);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  decode_attn_combine_kernel<<<B * H, 64, 0, s>>>((const float*)ws, (bf16_t*)out, H, n_split);
  return hipGetLastError();
}

// Top-k / temperature sampling of logits [B, V] (fp32, row stride ld) on the device:
// writes tok[b] and gen[b * gen_ld + *pos].  top_k <= 0 keeps every logit.
NSA_API hipError_t nsa_sample_topk(const void* logits, int B, int V, int ld, float temperature, int top_k,
                                   uint64_t salt, const void* pos, void* tok, void* gen, int gen_ld, hipStream_t s) {
  if (B < 1 || V < 1 || V > SMP_THREADS * SMP_MAXC || !(temperature > 0.0f)) return hipErrorInvalidValue;
  sample_topk_kernel<<<B, SMP_THREADS, 0, s>>>((const float*)logits, V, ld, 1.4426950408889634f / temperature, top_k,
                                               salt, (const int64_t*)pos, (int64_t*)tok, (int64_t*)gen, gen_ld);
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
  if (rows == 1) NSA_GEMV(1);
  else if (rows == 2) NSA_GEMV(2);
  else if (rows <= 4) NSA_GEMV(4);
  else NSA_GEMV(8);
#undef NSA_GEMV
  return hipGetLastError();
}
