// Sorted, atomic-free scatter-add of rows: out[ids[p]] += f(order[p]) over the positions p of
// a stably sorted index list (cdna_hip_programming.md App. B, "scatter-add without atomics":
// one writer per destination row, long lists split into chunks whose partial sums a further
// pass adds in chunk order).  Shared by the embedding backward (embedding.hip: f = the
// token's dropout-masked dx row) and the cross-entropy's onehot dW term (xent_fused.hip).
//
// Inputs: ids[N] sorted destination ids (negative = skip: they sort first), order[N] the
// source rows in that order, seg[V + 1] the segment starts (searchsorted over ids), part a
// [2 * ceil(N / kSegChunk), C] fp32 workspace.  F::load(row, id, c, f[8]) yields columns
// c .. c + 7 of source row `row` (whose destination is `id`).  Two regimes:
//   short segments (<= kSegLong positions; GPT-2's 50304 ids average 2.4 tokens a micro-step):
//     one wave per id sums its rows in sorted order, four gathered per step (row kernel);
//   long segments (a character corpus: the space is ~15% of all tokens): the sorted list is
//     cut into chunks of kSegChunk positions, one wave each; a long segment always crosses
//     a chunk boundary, so each chunk leaves the partial sum of its long runs in
//     part[chunk][slot] (slot 0: the chunk's first run, 1: its last), and the chunk in which
//     the segment ends adds its partials in chunk order (fix kernel).
// Fixed summation order for any schedule: bitwise reproducible.  C % 8 == 0.
#pragma once

#include "common.h"

namespace {

constexpr int kSegChunk = 16;
constexpr int kSegLong = 64;

__device__ __forceinline__ void seg_rmw8(float* p, const float (&acc)[8]) {
  float4* g = reinterpret_cast<float4*>(p);
  float4 g0 = g[0], g1 = g[1];
  g0.x += acc[0]; g0.y += acc[1]; g0.z += acc[2]; g0.w += acc[3];
  g1.x += acc[4]; g1.y += acc[5]; g1.z += acc[6]; g1.w += acc[7];
  g[0] = g0;
  g[1] = g1;
}

template <typename IT, class F>
__global__ __launch_bounds__(256) void seg_row_kernel(const int64_t* __restrict__ order, const int64_t* __restrict__ seg,
                                                      F f, float* __restrict__ out, int ldo, int V, int C) {
  const int lane = threadIdx.x & 63;
  const int v = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (v >= V) return;
  const int64_t beg = seg[v], end = seg[v + 1];
  if (beg == end || end - beg > kSegLong) return;  // empty, or the chunk kernels' segment
  // one walk of the segment covers two 512-column halves (C = 768: one walk instead of two,
  // so the dependent seg -> order -> row loads run once per id); per column the rows are
  // still added in sorted order, so the sums are bitwise those of one walk per half
  for (int c = lane * 8; c < C; c += 1024) {
    const bool two = c + 512 < C;
    float acc[2][8] = {{0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0, 0, 0}};
    for (int64_t k = beg; k < end; k += 4) {
      const int n = (int)min((int64_t)4, end - k);
      int64_t rw[4];
      float x[4][2][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) rw[u] = u < n ? order[k + u] : 0;
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < n) {
          f.load(rw[u], (int64_t)v, c, x[u][0]);
          if (two) f.load(rw[u], (int64_t)v, c + 512, x[u][1]);
        }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < n) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[0][j] += x[u][0][j];
          if (two) {
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[1][j] += x[u][1][j];
          }
        }
    }
    seg_rmw8(out + (int64_t)v * ldo + c, acc[0]);
    if (two) seg_rmw8(out + (int64_t)v * ldo + c + 512, acc[1]);
  }
}

template <typename IT, class F>
__global__ __launch_bounds__(256) void seg_chunk_kernel(const IT* __restrict__ ids, const int64_t* __restrict__ order,
                                                        const int64_t* __restrict__ seg, F f,
                                                        float* __restrict__ part, int N, int C) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j * kSegChunk >= N) return;
  const int p0 = j * kSegChunk, n = min(N - p0, kSegChunk);
  int64_t id[kSegChunk], rw[kSegChunk];
  uint32_t lmask = 0;  // positions of the chunk that belong to long segments
#pragma unroll
  for (int q = 0; q < kSegChunk; ++q) id[q] = q < n ? (int64_t)ids[p0 + q] : -1;
#pragma unroll
  for (int q = 0; q < kSegChunk; ++q)
    if (id[q] >= 0 && seg[id[q] + 1] - seg[id[q]] > kSegLong) lmask |= 1u << q;
  if (!lmask) return;
#pragma unroll
  for (int q = 0; q < kSegChunk; ++q) rw[q] = (lmask >> q) & 1 ? order[p0 + q] : 0;
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
    for (int b = 0; b < kSegChunk; b += 8) {
      float x[8][8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if ((lmask >> (b + u)) & 1) f.load(rw[b + u], id[b + u], c, x[u]);
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
            for (int jj = 0; jj < 8; ++jj) acc[jj] += x[u][jj];
          }
        }
      }
    }
    flush();
  }
}

template <typename IT>
__global__ __launch_bounds__(256) void seg_fix_kernel(const IT* __restrict__ ids, const int64_t* __restrict__ seg,
                                                      const float* __restrict__ part, float* __restrict__ out,
                                                      int ldo, int N, int C) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j == 0 || j * kSegChunk >= N) return;
  const int p0 = j * kSegChunk, pend = min(N, p0 + kSegChunk);
  const int64_t u = ids[p0];
  if (u < 0) return;
  if ((int64_t)ids[p0 - 1] != u) return;            // the chunk's first run starts here: not a crossing segment
  if (pend < N && (int64_t)ids[pend] == u) return;  // the segment goes on past this chunk
  const int64_t s = seg[u];
  if (seg[u + 1] - s <= kSegLong) return;  // a short segment: the row kernel's
  const int js = (int)(s / kSegChunk);
  const int s1 = s > (int64_t)js * kSegChunk ? 1 : 0;  // slot of the first piece
  for (int c = lane * 8; c < C; c += 512) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i0 = js; i0 <= j; i0 += 8) {
      float x[8][8];
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (i0 + q <= j) {
          const float* pp = part + ((int64_t)(i0 + q) * 2 + (i0 + q == js ? s1 : 0)) * C + c;
          const float4 a = reinterpret_cast<const float4*>(pp)[0], b = reinterpret_cast<const float4*>(pp)[1];
          x[q][0] = a.x; x[q][1] = a.y; x[q][2] = a.z; x[q][3] = a.w;
          x[q][4] = b.x; x[q][5] = b.y; x[q][6] = b.z; x[q][7] = b.w;
        }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (i0 + q <= j) {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) acc[jj] += x[q][jj];
        }
    }
    seg_rmw8(out + u * ldo + c, acc);
  }
}

// Small destination tables (V x C fp32 fits the LDS, e.g. a character vocabulary): each
// workgroup adds its rows into an LDS copy of the table (ds_add_f32) and stores the copy as
// its partial table (part[blockIdx]); seg_lds_reduce_kernel adds the partials into `out` in
// workgroup order.  Unsorted ids (negative or >= V = skip); the LDS adds land in arrival
// order, so not bitwise reproducible (the sorted passes above are).  Against per-row global
// atomics on a 65-row table (every token hitting the same few rows: the chip serialises on
// them) this moves the contention into the LDS.  The table is padded by one dword per 8
// columns: a lane adds 8 consecutive columns, so unpadded lanes l and l + 4 of a 32-lane
// group hit one bank (8-way conflicts); at stride 9 the 32 lanes take 32 banks.  The table
// takes most of a CU's LDS (one workgroup per CU), so the rows are spread over every CU.
// Measured at the char shape (16384 rows, 65 x 384): one global atomic per table element to
// flush, 128 workgroups x 4 waves, unpadded: 80 us; partial tables, 64 x 16 waves: 130 us.
constexpr int kSegLdsThreads = 256;
constexpr int kSegLdsRows = 64;  // rows per workgroup (16 per wave)

__device__ __forceinline__ int seg_lds_pad(int c) { return c + (c >> 3); }

template <typename IT, class F>
__global__ __launch_bounds__(kSegLdsThreads) void seg_lds_kernel(const IT* __restrict__ ids, F f,
                                                                 float* __restrict__ part, int N, int V, int C) {
  extern __shared__ __attribute__((aligned(16))) float tab[];  // [V][C + C / 8]
  const int Cp = C + (C >> 3);
  for (int i = threadIdx.x; i < V * Cp; i += kSegLdsThreads) tab[i] = 0.0f;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  constexpr int kW = kSegLdsThreads / 64;
  const int stride = gridDim.x * kW;
  for (int r0 = blockIdx.x * kW + (threadIdx.x >> 6); r0 < N; r0 += 4 * stride) {
    int64_t rw[4], id[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      rw[u] = r0 + (int64_t)u * stride;
      id[u] = rw[u] < N ? (int64_t)ids[rw[u]] : -1;
    }
    for (int c = lane * 8; c < C; c += 512) {
      float x[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (id[u] >= 0 && id[u] < V) f.load(rw[u], id[u], c, x[u]);
      const int pc = seg_lds_pad(c);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (id[u] >= 0 && id[u] < V) {
#pragma unroll
          for (int j = 0; j < 8; ++j) atomicAdd(&tab[id[u] * Cp + pc + j], x[u][j]);
        }
    }
  }
  __syncthreads();
  float* pp = part + (int64_t)blockIdx.x * V * C;
  for (int i = threadIdx.x; i < V * C; i += kSegLdsThreads) {
    const int v = i / C, c = i - v * C;
    pp[i] = tab[v * Cp + seg_lds_pad(c)];
  }
}

// out[i / C][i % C] += sum over g < G of part[g][i], g in order; 4 waves per workgroup split
// the G partials of 256 consecutive elements (a float4 per lane) and combine through LDS
__global__ __launch_bounds__(256) void seg_lds_reduce_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                             int ldo, int G, int VC, int C) {
  __shared__ float4 red[3][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = (blockIdx.x * 64 + lane) * 4;
  float4 a{0.f, 0.f, 0.f, 0.f};
  if (i < VC) {
    int g = w;
    for (; g + 12 < G; g += 16) {  // 4 loads in flight per lane
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(part + (int64_t)(g + 4 * u) * VC + i);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
    for (; g < G; g += 4) {
      const float4 v = *reinterpret_cast<const float4*>(part + (int64_t)g * VC + i);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  }
  if (w > 0) red[w - 1][lane] = a;
  __syncthreads();
  if (w == 0 && i < VC) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      a.x += red[u][lane].x; a.y += red[u][lane].y; a.z += red[u][lane].z; a.w += red[u][lane].w;
    }
    float* o = out + (int64_t)(i / C) * ldo + i % C;  // C % 4 == 0: the 4 stay in one row
    o[0] += a.x; o[1] += a.y; o[2] += a.z; o[3] += a.w;
  }
}

constexpr int kSegLdsBytes = 128 * 1024;  // LDS table budget of seg_lds_kernel (padded V x C fp32)

// part: G x V x C floats (16-byte aligned), G = seg_lds_parts(N)
inline int seg_lds_parts(int N) {
  const int g = (N + kSegLdsRows - 1) / kSegLdsRows;
  return g < 1 ? 1 : (g > 256 ? 256 : g);
}

template <typename IT, class F>
hipError_t seg_scatter_add_lds(const IT* ids, F f, float* part, float* out, int ldo, int N, int V, int C,
                               hipStream_t s) {
  if (C % 8 != 0 || (size_t)V * (C + C / 8) * 4 > (size_t)kSegLdsBytes || (uintptr_t)part % 16)
    return hipErrorInvalidValue;
  const int G = seg_lds_parts(N);
  static bool attr = [] {  // dynamic LDS above 64 KB (one workgroup per CU)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&seg_lds_kernel<IT, F>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kSegLdsBytes) == hipSuccess;
  }();
  if (!attr) return hipErrorInvalidValue;
  seg_lds_kernel<IT, F><<<G, kSegLdsThreads, (size_t)V * (C + C / 8) * 4, s>>>(ids, f, part, N, V, C);
  const int VC = V * C;
  seg_lds_reduce_kernel<<<(VC / 4 + 63) / 64, 256, 0, s>>>(part, out, ldo, G, VC, C);
  return hipGetLastError();
}

// the three passes; part: 2 * ceil(N / kSegChunk) rows of C floats
template <typename IT, class F>
hipError_t seg_scatter_add(const IT* ids, const int64_t* order, const int64_t* seg, float* part, F f, float* out,
                           int ldo, int N, int V, int C, hipStream_t s) {
  if (C % 8 != 0 || ldo % 4 != 0) return hipErrorInvalidValue;
  const int chunks = (N + kSegChunk - 1) / kSegChunk;
  seg_row_kernel<IT, F><<<(V + 3) / 4, 256, 0, s>>>(order, seg, f, out, ldo, V, C);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  seg_chunk_kernel<IT, F><<<(chunks + 3) / 4, 256, 0, s>>>(ids, order, seg, f, part, N, C);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  seg_fix_kernel<IT><<<(chunks + 3) / 4, 256, 0, s>>>(ids, seg, part, out, ldo, N, C);
  return hipGetLastError();
}

}  // namespace
