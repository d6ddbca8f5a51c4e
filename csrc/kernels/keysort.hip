// Stable sort of small integer keys (token ids, cross-entropy targets with -1 = ignored) for
// the sorted, atomic-free scatter-adds of segsum.h (the torch / rocprim
// radix sort, merge, searchsorted, arange and fill kernels off the training step).
//
// Output, exactly what torch.sort(keys, stable=True) + torch.searchsorted(ids, arange(V + 1))
// give: ids[N] the keys in ascending order (same dtype as the input), order[N] (int64) the
// positions they came from, equal keys in position order, and seg[V + 1] (int64) with
// seg[v] = #{keys < v} (negative keys sort first and lie below seg[0]).
//
// Keys -1 .. V - 1 are shifted by one into 16-bit digits 0 .. V (V + 1 <= 65536) and sorted
// LSD by 8-bit digit, one pass per digit that is not constant (V + 1 <= 256: one pass).  A
// pass is three kernels over chunks of 4096 keys (one 256-thread workgroup each):
//   hist     per-chunk digit histogram in LDS -> hist[digit][chunk]
//   scan     one workgroup: exclusive prefix sum over hist in digit-major, chunk-minor order
//            (the start of every (digit, chunk) run in the output)
//   scatter  the chunk again in 16 rounds of 256 keys in position order; a key's rank among
//            equal digits of its round comes from 8 ballots (the lanes whose digit matches on
//            every bit) plus the counts of the lower waves, so equal digits keep position order
//            (stable) and the result does not depend on scheduling
// and seg is one binary search per vocabulary id over the sorted keys.
#include "common.h"

namespace {

constexpr int KS_THR = 256;
constexpr int KS_PER = 16;                 // keys per thread per chunk
constexpr int KS_CHUNK = KS_THR * KS_PER;  // 4096
constexpr int KS_BINS = 256;

template <typename IT>
__device__ __forceinline__ uint32_t ks_digit0(const IT* keys, int i) {
  return (uint32_t)((int64_t)keys[i] + 1);  // -1 .. V-1 -> 0 .. V
}

// first pass reads the caller's keys (IT), later passes the 16-bit ping-pong copy
template <typename IT, bool FIRST>
__device__ __forceinline__ uint32_t ks_load(const IT* keys, const uint16_t* k16, int i) {
  if constexpr (FIRST) return ks_digit0(keys, i);
  else return k16[i];
}

template <typename IT, bool FIRST>
__global__ __launch_bounds__(KS_THR) void ks_hist_kernel(const IT* __restrict__ keys, const uint16_t* __restrict__ k16,
                                                         int N, int shift, int nchunks, int* __restrict__ hist) {
  __shared__ int h[KS_BINS];
  h[threadIdx.x] = 0;
  __syncthreads();
  const int base = blockIdx.x * KS_CHUNK;
#pragma unroll 4
  for (int r = 0; r < KS_PER; ++r) {
    const int i = base + r * KS_THR + threadIdx.x;
    if (i < N) atomicAdd(&h[(ks_load<IT, FIRST>(keys, k16, i) >> shift) & 0xff], 1);
  }
  __syncthreads();
  hist[threadIdx.x * nchunks + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan of n ints in place, one 1024-thread workgroup
__global__ __launch_bounds__(1024) void ks_scan_kernel(int* __restrict__ a, int n) {
  __shared__ int wsum[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (n + 1023) / 1024;
  const int b = tid * per, e = min(n, b + per);
  int s = 0;
  for (int i = b; i < e; ++i) s += a[i];
  // inclusive scan of the per-thread sums over the workgroup
  int v = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  if (lane == 63) wsum[w] = v;
  __syncthreads();
  if (w == 0) {
    int x = lane < 16 ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int u = __shfl_up(x, o, 64);
      if (lane >= o) x += u;
    }
    if (lane < 16) wsum[lane] = x;
  }
  __syncthreads();
  int run = v - s + (w > 0 ? wsum[w - 1] : 0);  // exclusive prefix of this thread's range
  for (int i = b; i < e; ++i) {
    const int t = a[i];
    a[i] = run;
    run += t;
  }
}

// LAST: write the caller's outputs (ids in IT, order as int64) instead of the ping-pong copy
template <typename IT, bool FIRST, bool LAST>
__global__ __launch_bounds__(KS_THR) void ks_scatter_kernel(const IT* __restrict__ keys, const uint16_t* __restrict__ k16,
                                                            const int* __restrict__ p32, int N, int shift, int nchunks,
                                                            const int* __restrict__ scan, uint16_t* __restrict__ k16_out,
                                                            int* __restrict__ p32_out, IT* __restrict__ ids_out,
                                                            int64_t* __restrict__ order_out) {
  __shared__ int off[KS_BINS];
  __shared__ int wcnt[4][KS_BINS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  off[tid] = scan[tid * nchunks + blockIdx.x];
  const unsigned long long lt = (1ull << lane) - 1ull;
  const int base = blockIdx.x * KS_CHUNK;
  for (int r = 0; r < KS_PER; ++r) {
#pragma unroll
    for (int q = 0; q < 4; ++q) wcnt[q][tid] = 0;
    __syncthreads();  // off (first round) and the cleared counts are visible
    const int i = base + r * KS_THR + tid;
    const bool valid = i < N;
    uint32_t key = 0;
    int pos = 0;
    if (valid) {
      key = ks_load<IT, FIRST>(keys, k16, i);
      pos = FIRST ? i : p32[i];
    }
    const uint32_t d = (key >> shift) & 0xff;
    // lanes whose digit equals this lane's on all 8 bits (only valid lanes)
    unsigned long long peers = __ballot(valid);
#pragma unroll
    for (int bit = 0; bit < 8; ++bit) {
      const unsigned long long ones = __ballot(valid && ((d >> bit) & 1));
      peers &= ((d >> bit) & 1) ? ones : ~ones;
    }
    const int rank_w = __popcll(peers & lt);
    if (valid && rank_w == 0) wcnt[w][d] = __popcll(peers);  // the lowest lane of each digit group
    __syncthreads();
    if (valid) {
      int dst = off[d] + rank_w;
      for (int q = 0; q < w; ++q) dst += wcnt[q][d];
      if constexpr (LAST) {
        ids_out[dst] = (IT)((int64_t)key - 1);
        order_out[dst] = pos;
      } else {
        k16_out[dst] = (uint16_t)key;
        p32_out[dst] = pos;
      }
    }
    __syncthreads();  // every lane has read off / wcnt of this round
    off[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
  }
}

// seg[v] = #{ids < v}, v = 0 .. V (lower bound in the sorted ids)
template <typename IT>
__global__ __launch_bounds__(KS_THR) void ks_seg_kernel(const IT* __restrict__ ids, int N, int V,
                                                        int64_t* __restrict__ seg) {
  const int v = blockIdx.x * KS_THR + threadIdx.x;
  if (v > V) return;
  int lo = 0, hi = N;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int64_t)ids[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  seg[v] = lo;
}

template <typename IT>
hipError_t keysort(const IT* keys, int N, int V, IT* ids, int64_t* order, int64_t* seg, void* ws, hipStream_t s) {
  if (N < 1 || V < 1 || V + 1 > 65536) return hipErrorInvalidValue;
  const int nchunks = (N + KS_CHUNK - 1) / KS_CHUNK;
  char* p = static_cast<char*>(ws);
  int* hist = reinterpret_cast<int*>(p);
  p += (size_t)KS_BINS * nchunks * 4;
  uint16_t* k16[2] = {reinterpret_cast<uint16_t*>(p), reinterpret_cast<uint16_t*>(p) + N};
  p += ((size_t)2 * N * 2 + 15) / 16 * 16;
  int* p32[2] = {reinterpret_cast<int*>(p), reinterpret_cast<int*>(p) + N};
  const bool two = V + 1 > 256;  // keys 0 .. V: the high digit is constant below 256
  for (int pass = 0; pass < (two ? 2 : 1); ++pass) {
    const int shift = 8 * pass;
    const bool first = pass == 0, last = pass == (two ? 1 : 0);
    const uint16_t* kin = first ? nullptr : k16[0];
    const int* pin = first ? nullptr : p32[0];
    if (first) ks_hist_kernel<IT, true><<<nchunks, KS_THR, 0, s>>>(keys, kin, N, shift, nchunks, hist);
    else ks_hist_kernel<IT, false><<<nchunks, KS_THR, 0, s>>>(keys, kin, N, shift, nchunks, hist);
    ks_scan_kernel<<<1, 1024, 0, s>>>(hist, KS_BINS * nchunks);
    if (first && last)
      ks_scatter_kernel<IT, true, true><<<nchunks, KS_THR, 0, s>>>(keys, kin, pin, N, shift, nchunks, hist, nullptr,
                                                                  nullptr, ids, order);
    else if (first)
      ks_scatter_kernel<IT, true, false><<<nchunks, KS_THR, 0, s>>>(keys, kin, pin, N, shift, nchunks, hist, k16[0],
                                                                   p32[0], nullptr, nullptr);
    else
      ks_scatter_kernel<IT, false, true><<<nchunks, KS_THR, 0, s>>>(keys, kin, pin, N, shift, nchunks, hist, nullptr,
                                                                   nullptr, ids, order);
  }
  ks_seg_kernel<IT><<<(V + 1 + KS_THR - 1) / KS_THR, KS_THR, 0, s>>>(ids, N, V, seg);
  return hipGetLastError();
}

}  // namespace

// workspace bytes of nsa_keysort for N keys
NSA_API int64_t nsa_keysort_ws_bytes(int N) {
  const int64_t nchunks = (N + KS_CHUNK - 1) / KS_CHUNK;
  return (int64_t)KS_BINS * nchunks * 4 + ((int64_t)2 * N * 2 + 15) / 16 * 16 + (int64_t)2 * N * 4;
}

// key64 = 1: keys / ids are int64 (token ids), 0: int32 (cross-entropy targets)
NSA_API hipError_t nsa_keysort(const void* keys, int key64, int N, int V, void* ids, void* order, void* seg, void* ws,
                               hipStream_t s) {
  if (key64)
    return keysort<int64_t>(static_cast<const int64_t*>(keys), N, V, static_cast<int64_t*>(ids),
                            static_cast<int64_t*>(order), static_cast<int64_t*>(seg), ws, s);
  return keysort<int32_t>(static_cast<const int32_t*>(keys), N, V, static_cast<int32_t*>(ids),
                          static_cast<int64_t*>(order), static_cast<int64_t*>(seg), ws, s);
}
