// Token + position embedding forward/backward (SURVEY.md §2.7 K11/K12;
// nanoGPT: x = drop(wte(idx) + wpe(arange(T)))).
//
// forward : one wave per token row; 16-byte gathers of the wte row and the wpe
//           row, fp32 add, optional hash dropout, bf16 store.
// backward: dwte — the tied wte/lm_head gradient lives in the fp32 flat
//           gradient buffer; each wave stages its token's dx row in LDS and
//           issues fp32 atomics so that every wave-instruction covers 256
//           contiguous bytes (the full-rate atomic shape, MI355X_MICROARCH.md
//           "Global float atomics").  B*T*C*4 bytes of atomics per micro-step
//           (38 MB for GPT-2 124M) ≈ 30 us at the ~1.3 TB/s chip atomic rate.
//           dwpe — owned per (t, column-octet): the thread sums over the batch
//           and read-modify-writes the flat buffer, no atomics.
//
// The output (the residual stream) and its gradient are bf16 or fp32 (XT): fp32 is
// nanoGPT's autocast contract (the embedding sum stays fp32), bf16 is opt-in.
#include "common.h"

namespace {

__device__ __forceinline__ void ld8(const bf16_t* p, float (&f)[8]) { load8(p, f); }
__device__ __forceinline__ void ld8(const float* p, float (&f)[8]) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w; f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
}
__device__ __forceinline__ void st8(bf16_t* p, const float (&f)[8]) { store8(p, f); }
__device__ __forceinline__ void st8(float* p, const float (&f)[8]) {
  reinterpret_cast<float4*>(p)[0] = make_float4(f[0], f[1], f[2], f[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(f[4], f[5], f[6], f[7]);
}

template <typename XT, bool H = false>
__global__ __launch_bounds__(256) void emb_fwd_kernel(const int64_t* __restrict__ idx, const bf16_t* __restrict__ wte,
                                                     const bf16_t* __restrict__ wpe, XT* __restrict__ out, int N,
                                                     int T, int C, uint32_t thresh, float scale, uint64_t salt) {
  const uint64_t seed = nsa_seed(salt);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int t = row % T;
  const int64_t tok = idx[row];
  const bf16_t* a = wte + tok * C;
  const bf16_t* p = wpe + (int64_t)t * C;
  XT* o = out + (int64_t)row * C;
  for (int c = lane * 8; c < C; c += 512) {
    float fa[8], fp[8];
    load8e<H>(a + c, fa);
    load8e<H>(p + c, fp);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = fa[j] + fp[j];
      if (thresh) v = nsa_keep(seed, (uint64_t)row * C + c + j, thresh) ? v * scale : 0.0f;
      fa[j] = v;
    }
    st8(o + c, fa);
  }
}

template <typename XT>
__global__ __launch_bounds__(256) void emb_bwd_wte_kernel(const int64_t* __restrict__ idx,
                                                         const XT* __restrict__ dx, float* __restrict__ dwte, int N,
                                                         int C, uint32_t thresh, float scale, uint64_t salt) {
  const uint64_t seed = nsa_seed(salt);
  extern __shared__ __attribute__((aligned(16))) float stage[];  // [4][C]
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  float* srow = stage + wv * C;
  for (int row = blockIdx.x * 4 + wv; row < N; row += gridDim.x * 4) {
    const XT* d = dx + (int64_t)row * C;
    for (int c = lane * 8; c < C; c += 512) {
      float f[8];
      ld8(d + c, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float v = f[j];
        if (thresh) v = nsa_keep(seed, (uint64_t)row * C + c + j, thresh) ? v * scale : 0.0f;
        srow[c + j] = v;
      }
    }
    // wave-private LDS row: order the row's writes before the cross-lane reads
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    float* g = dwte + idx[row] * C;
    for (int c = lane; c < C; c += 64) atomicAdd(g + c, srow[c]);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

template <typename XT>
__global__ __launch_bounds__(256) void emb_bwd_wpe_kernel(const XT* __restrict__ dx, float* __restrict__ dwpe,
                                                         int B, int T, int C, uint32_t thresh, float scale,
                                                         uint64_t salt) {
  const uint64_t seed = nsa_seed(salt);
  const int octs = C / 8;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= T * octs) return;
  const int t = i / octs;
  const int c = (i % octs) * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  // four batch rows per step: four independent 32-byte loads in flight, summed in b order
  for (int b0 = 0; b0 < B; b0 += 4) {
    float f[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b0 + u < B) ld8(dx + ((int64_t)(b0 + u) * T + t) * C + c, f[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (b0 + u < B) {
        const int64_t row = (int64_t)(b0 + u) * T + t;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float v = f[u][j];
          if (thresh) v = nsa_keep(seed, (uint64_t)row * C + c + j, thresh) ? v * scale : 0.0f;
          acc[j] += v;
        }
      }
    }
  }
  float4* g = reinterpret_cast<float4*>(dwpe + (int64_t)t * C + c);
  float4 g0 = g[0], g1 = g[1];
  g0.x += acc[0];
  g0.y += acc[1];
  g0.z += acc[2];
  g0.w += acc[3];
  g1.x += acc[4];
  g1.y += acc[5];
  g1.z += acc[6];
  g1.w += acc[7];
  g[0] = g0;
  g[1] = g1;
}

// Deterministic dwte without atomics (the sorted path: every micro-step of >= 4096 tokens,
// and the deterministic mode).  The caller stably sorts the token positions by vocab id
// (ids = sorted ids, order = their positions, seg = segment starts by id).  Two regimes,
// one writer per row either way (cdna_hip_programming.md App. B, "scatter-add without
// atomics": split long lists into chunks, add the partial sums in chunk order in a
// further pass):
//   short segments (<= kDetLong tokens; GPT-2's 50304 ids average 2.4 tokens a
//     micro-step): one wave per id sums its tokens' rows in token order (row kernel).
//   long segments (a character corpus: 56 ids, the space ~15% of all tokens): the sorted
//     list is cut into chunks of kDetChunk positions, one wave each; a long segment
//     always crosses a chunk boundary, so each chunk leaves the partial sum of its long
//     runs in part[chunk][slot] (slot 0: the chunk's first run, 1: its last), and the
//     chunk in which the segment ends adds its partials in chunk order (fix kernel).
// Fixed summation order for any schedule: bitwise reproducible.  Rows are gathered four
// (row kernel) or eight (chunk kernel) at a time so that many 16-byte loads per lane are in
// flight (round 4's one-wave-per-id serial walk took 2.3 ms per micro-step on the character
// config, its 5000-token space row).
constexpr int kDetChunk = 16;
constexpr int kDetLong = 64;

template <typename XT>
__global__ __launch_bounds__(256) void emb_bwd_wte_row_kernel(const int64_t* __restrict__ order,
                                                             const int64_t* __restrict__ seg,
                                                             const XT* __restrict__ dx, float* __restrict__ dwte,
                                                             int V, int C, uint32_t thresh, float scale,
                                                             uint64_t salt) {
  const uint64_t seed = nsa_seed(salt);
  const int lane = threadIdx.x & 63;
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (v >= V) return;
  const int64_t beg = seg[v], end = seg[v + 1];
  if (beg == end || end - beg > kDetLong) return;  // empty, or the chunk kernels' segment
  for (int c = lane * 8; c < C; c += 512) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int64_t k = beg; k < end; k += 4) {
      const int n = (int)min((int64_t)4, end - k);
      int64_t rw[4];
      float f[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) rw[u] = u < n ? order[k + u] : 0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < n) ld8(dx + rw[u] * C + c, f[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < n) {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            float x = f[u][jj];
            if (thresh) x = nsa_keep(seed, (uint64_t)rw[u] * C + c + jj, thresh) ? x * scale : 0.0f;
            acc[jj] += x;
          }
        }
    }
    float4* g = reinterpret_cast<float4*>(dwte + (int64_t)v * C + c);
    float4 g0 = g[0], g1 = g[1];
    g0.x += acc[0]; g0.y += acc[1]; g0.z += acc[2]; g0.w += acc[3];
    g1.x += acc[4]; g1.y += acc[5]; g1.z += acc[6]; g1.w += acc[7];
    g[0] = g0;
    g[1] = g1;
  }
}

template <typename XT>
__global__ __launch_bounds__(256) void emb_bwd_wte_chunk_kernel(const int64_t* __restrict__ ids,
                                                               const int64_t* __restrict__ order,
                                                               const int64_t* __restrict__ seg,
                                                               const XT* __restrict__ dx, float* __restrict__ part,
                                                               int N, int C, uint32_t thresh, float scale,
                                                               uint64_t salt) {
  const uint64_t seed = nsa_seed(salt);
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j * kDetChunk >= N) return;
  const int p0 = j * kDetChunk, n = min(N - p0, kDetChunk);
  int64_t id[kDetChunk], rw[kDetChunk];
  uint32_t lmask = 0;  // positions of the chunk that belong to long segments
#pragma unroll
  for (int q = 0; q < kDetChunk; ++q) id[q] = q < n ? ids[p0 + q] : -1;
#pragma unroll
  for (int q = 0; q < kDetChunk; ++q)
    if (q < n && seg[id[q] + 1] - seg[id[q]] > kDetLong) lmask |= 1u << q;
  if (!lmask) return;
#pragma unroll
  for (int q = 0; q < kDetChunk; ++q) rw[q] = (lmask >> q) & 1 ? order[p0 + q] : 0;
  for (int c = lane * 8; c < C; c += 512) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int rs = 0;  // start of the current run
    // a long run crosses a chunk boundary by length: its partial sum always goes to part
    auto flush = [&]() {
      if (!((lmask >> rs) & 1)) return;
      float4* g = reinterpret_cast<float4*>(part + ((int64_t)j * 2 + (rs == 0 ? 0 : 1)) * C + c);
      g[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      g[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    };
#pragma unroll
    for (int b = 0; b < kDetChunk; b += 8) {
      float f[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if ((lmask >> (b + u)) & 1) ld8(dx + rw[b + u] * C + c, f[u]);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int q = b + u;
        if (q < n) {
          if (id[q] != id[rs]) {
            flush();
            rs = q;
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) acc[jj] = 0.0f;
          }
          if ((lmask >> q) & 1) {
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
              float x = f[u][jj];
              if (thresh) x = nsa_keep(seed, (uint64_t)rw[q] * C + c + jj, thresh) ? x * scale : 0.0f;
              acc[jj] += x;
            }
          }
        }
      }
    }
    flush();
  }
}

__global__ __launch_bounds__(256) void emb_bwd_wte_fix_kernel(const int64_t* __restrict__ ids,
                                                             const int64_t* __restrict__ seg,
                                                             const float* __restrict__ part,
                                                             float* __restrict__ dwte, int N, int C) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j == 0 || j * kDetChunk >= N) return;
  const int p0 = j * kDetChunk, pend = min(N, p0 + kDetChunk);
  const int64_t u = ids[p0];
  if (ids[p0 - 1] != u) return;            // the chunk's first run starts here: not a crossing segment
  if (pend < N && ids[pend] == u) return;  // the segment goes on past this chunk
  const int64_t s = seg[u];
  if (seg[u + 1] - s <= kDetLong) return;  // a short segment: the row kernel's
  const int js = (int)(s / kDetChunk);
  const int s1 = s > (int64_t)js * kDetChunk ? 1 : 0;  // slot of the first piece
  for (int c = lane * 8; c < C; c += 512) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i0 = js; i0 <= j; i0 += 8) {
      float f[8][8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (i0 + q <= j) ld8(part + ((int64_t)(i0 + q) * 2 + (i0 + q == js ? s1 : 0)) * C + c, f[q]);
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (i0 + q <= j) {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) acc[jj] += f[q][jj];
        }
    }
    float4* g = reinterpret_cast<float4*>(dwte + u * C + c);
    float4 g0 = g[0], g1 = g[1];
    g0.x += acc[0]; g0.y += acc[1]; g0.z += acc[2]; g0.w += acc[3];
    g1.x += acc[4]; g1.y += acc[5]; g1.z += acc[6]; g1.w += acc[7];
    g[0] = g0;
    g[1] = g1;
  }
}

template <typename XT, bool H = false>
hipError_t launch_fwd(const void* idx, const void* wte, const void* wpe, void* out, int N, int T, int C, float p,
                      uint64_t seed, hipStream_t s) {
  if (C % 8 != 0) return hipErrorInvalidValue;
  const uint32_t th = p > 0.0f ? nsa_drop_thresh(p) : 0u;
  const float scale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  emb_fwd_kernel<XT, H><<<(N + 3) / 4, 256, 0, s>>>((const int64_t*)idx, (const bf16_t*)wte, (const bf16_t*)wpe,
                                                 (XT*)out, N, T, C, th, scale, seed);
  return hipGetLastError();
}

template <typename XT>
hipError_t launch_bwd(const void* idx, const void* dx, void* dwte, void* dwpe, int B, int T, int C, float p,
                      uint64_t seed, hipStream_t s) {
  if (C % 8 != 0) return hipErrorInvalidValue;
  const uint32_t th = p > 0.0f ? nsa_drop_thresh(p) : 0u;
  const float scale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const int N = B * T;
  int grid = (N + 3) / 4;
  if (grid > 2048) grid = 2048;
  emb_bwd_wte_kernel<XT><<<grid, 256, 4 * C * sizeof(float), s>>>((const int64_t*)idx, (const XT*)dx,
                                                                   (float*)dwte, N, C, th, scale, seed);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int work = T * (C / 8);
  emb_bwd_wpe_kernel<XT><<<(work + 255) / 256, 256, 0, s>>>((const XT*)dx, (float*)dwpe, B, T, C, th, scale, seed);
  return hipGetLastError();
}

template <typename XT>
hipError_t launch_bwd_det(const void* ids, const void* order, const void* seg, void* part, const void* dx, void* dwte,
                          void* dwpe, int B, int T, int C, int V, float p, uint64_t seed, hipStream_t s) {
  if (C % 8 != 0) return hipErrorInvalidValue;
  const uint32_t th = p > 0.0f ? nsa_drop_thresh(p) : 0u;
  const float scale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const int N = B * T;
  const int chunks = (N + kDetChunk - 1) / kDetChunk;
  emb_bwd_wte_row_kernel<XT><<<(V + 3) / 4, 256, 0, s>>>((const int64_t*)order, (const int64_t*)seg,
                                                          (const XT*)dx, (float*)dwte, V, C, th, scale, seed);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  emb_bwd_wte_chunk_kernel<XT><<<(chunks + 3) / 4, 256, 0, s>>>((const int64_t*)ids, (const int64_t*)order,
                                                                (const int64_t*)seg, (const XT*)dx, (float*)part,
                                                                N, C, th, scale, seed);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  emb_bwd_wte_fix_kernel<<<(chunks + 3) / 4, 256, 0, s>>>((const int64_t*)ids, (const int64_t*)seg,
                                                          (const float*)part, (float*)dwte, N, C);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int work = T * (C / 8);
  emb_bwd_wpe_kernel<XT><<<(work + 255) / 256, 256, 0, s>>>((const XT*)dx, (float*)dwpe, B, T, C, th, scale, seed);
  return hipGetLastError();
}

}  // namespace

// idx: dense int64 [B*T] (callers pass a contiguous tensor); out / dx: bf16
NSA_DEFINE_RNG_ADVANCE(nsa_rng_advance_emb)

NSA_API hipError_t nsa_embedding_fwd(const void* idx, const void* wte, const void* wpe, void* out, int N, int T,
                                     int C, float p, uint64_t seed, hipStream_t s) {
  return launch_fwd<bf16_t>(idx, wte, wpe, out, N, T, C, p, seed, s);
}

NSA_API hipError_t nsa_embedding_bwd(const void* idx, const void* dx, void* dwte, void* dwpe, int B, int T, int C,
                                     float p, uint64_t seed, hipStream_t s) {
  return launch_bwd<bf16_t>(idx, dx, dwte, dwpe, B, T, C, p, seed, s);
}

// the same with an fp32 residual stream (out / dx fp32)
NSA_API hipError_t nsa_embedding_fwd_x32(const void* idx, const void* wte, const void* wpe, void* out, int N, int T,
                                         int C, float p, uint64_t seed, hipStream_t s) {
  return launch_fwd<float>(idx, wte, wpe, out, N, T, C, p, seed, s);
}

NSA_API hipError_t nsa_embedding_bwd_x32(const void* idx, const void* dx, void* dwte, void* dwpe, int B, int T,
                                         int C, float p, uint64_t seed, hipStream_t s) {
  return launch_bwd<float>(idx, dx, dwte, dwpe, B, T, C, p, seed, s);
}

// fp16 weight shadows (dtype float16), fp32 stream; the backward reads only the fp32 stream
NSA_API hipError_t nsa_embedding_fwd_x32_h(const void* idx, const void* wte, const void* wpe, void* out, int N, int T,
                                           int C, float p, uint64_t seed, hipStream_t s) {
  return launch_fwd<float, true>(idx, wte, wpe, out, N, T, C, p, seed, s);
}

// deterministic backward (order: token positions stably sorted by id, seg: [V + 1] offsets)
NSA_API hipError_t nsa_embedding_bwd_det(const void* ids, const void* order, const void* seg, void* part,
                                         const void* dx, void* dwte, void* dwpe, int B, int T, int C, int V,
                                         int dx_fp32, float p, uint64_t seed, hipStream_t s) {
  if (dx_fp32) return launch_bwd_det<float>(ids, order, seg, part, dx, dwte, dwpe, B, T, C, V, p, seed, s);
  return launch_bwd_det<bf16_t>(ids, order, seg, part, dx, dwte, dwpe, B, T, C, V, p, seed, s);
}
