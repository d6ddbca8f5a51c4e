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
#include "segsum.h"

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

// Atomic-free dwte (the sorted path: micro-steps of >= 64K tokens, and the deterministic
// mode): the caller stably sorts the token positions by vocab id and segsum.h's passes add
// each id's dropout-masked dx rows into its row of dwte, one writer per row (the chunked form
// for frequent ids: round 4's one-wave-per-id serial walk took 2.3 ms per micro-step on the
// character config, its 5000-token space row; profiles/r5_emb_bwd.md).
template <typename XT>
struct EmbRow {
  const XT* dx;
  int C;
  uint32_t thresh;
  float scale;
  uint64_t salt;
  __device__ __forceinline__ void load(int64_t row, int64_t, int c, float (&f)[8]) const {
    ld8(dx + row * C + c, f);
    if (thresh) {
      const uint64_t seed = nsa_seed(salt);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = nsa_keep(seed, (uint64_t)row * C + c + j, thresh) ? f[j] * scale : 0.0f;
    }
  }
};

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
  const EmbRow<XT> f{(const XT*)dx, C, th, scale, seed};
  hipError_t e = seg_scatter_add<int64_t, EmbRow<XT>>((const int64_t*)ids, (const int64_t*)order, (const int64_t*)seg,
                                                      (float*)part, f, (float*)dwte, C, B * T, V, C, s);
  if (e != hipSuccess) return e;
  const int work = T * (C / 8);
  emb_bwd_wpe_kernel<XT><<<(work + 255) / 256, 256, 0, s>>>((const XT*)dx, (float*)dwpe, B, T, C, th, scale, seed);
  return hipGetLastError();
}

}  // namespace

template <typename XT>
hipError_t launch_bwd_lds(const void* idx, const void* dx, void* dwte, void* dwpe, void* part, int B, int T, int C,
                          int V, float p, uint64_t seed, hipStream_t s) {
  if (C % 8 != 0) return hipErrorInvalidValue;
  const uint32_t th = p > 0.0f ? nsa_drop_thresh(p) : 0u;
  const float scale = p > 0.0f ? 1.0f / (1.0f - p) : 1.0f;
  const EmbRow<XT> f{(const XT*)dx, C, th, scale, seed};
  hipError_t e = seg_scatter_add_lds<int64_t, EmbRow<XT>>((const int64_t*)idx, f, (float*)part, (float*)dwte, C, B * T,
                                                           V, C, s);
  if (e != hipSuccess) return e;
  const int work = T * (C / 8);
  emb_bwd_wpe_kernel<XT><<<(work + 255) / 256, 256, 0, s>>>((const XT*)dx, (float*)dwpe, B, T, C, th, scale, seed);
  return hipGetLastError();
}

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

// small vocabularies (V x C fp32 <= 128 KB): the LDS-privatised scatter-add (segsum.h), not
// per-row global atomics on a few hot rows; arrival order (not the deterministic mode's path)
// part: nsa_seg_lds_parts(B * T) x V x C floats of scratch
NSA_API hipError_t nsa_embedding_bwd_lds(const void* idx, const void* dx, void* dwte, void* dwpe, void* part, int B,
                                         int T, int C, int V, int dx_fp32, float p, uint64_t seed, hipStream_t s) {
  if (dx_fp32) return launch_bwd_lds<float>(idx, dx, dwte, dwpe, part, B, T, C, V, p, seed, s);
  return launch_bwd_lds<bf16_t>(idx, dx, dwte, dwpe, part, B, T, C, V, p, seed, s);
}

// partial tables the LDS scatter-add over N rows writes (segsum.h seg_lds_parts)
NSA_API int nsa_seg_lds_parts(int N) { return seg_lds_parts(N); }
