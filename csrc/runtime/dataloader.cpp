// Native prefetching batch sampler for nanoGPT-format token files.
//
// Semantics follow nanoGPT's get_batch: a batch is
// `batch` windows at offsets i ~ U[0, n_tokens - block), x = data[i:i+T],
// y = data[i+1:i+1+T] widened from uint16 to int64.  The difference is the
// runtime: the file is mmapped once, and a background thread keeps a ring of
// `prefetch` ready batches so the training thread's get_batch is one memcpy
// into a pinned staging buffer (the H2D copy then runs async on the GPU).
//
// C ABI (bound with ctypes from nanosandbox_amd/data/loader.py):
//   void*   nsa_loader_create(const char* path, int block, int batch, uint64 seed, int prefetch)
//   int     nsa_loader_next(void* h, int64_t* x, int64_t* y)      // 0 on success
//   int64_t nsa_loader_num_tokens(void* h)
//   void    nsa_loader_destroy(void* h)

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

// splitmix64-seeded xoshiro256** : fast, good-quality, per-loader stream.
struct Rng {
  uint64_t s[4];
  static uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  explicit Rng(uint64_t seed) {
    for (auto& v : s) v = splitmix(seed);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  // unbiased integer in [0, n) (Lemire's method)
  uint64_t below(uint64_t n) {
    __uint128_t m = (__uint128_t)next() * n;
    uint64_t l = (uint64_t)m;
    if (l < n) {
      uint64_t t = -n % n;
      while (l < t) {
        m = (__uint128_t)next() * n;
        l = (uint64_t)m;
      }
    }
    return (uint64_t)(m >> 64);
  }
};

struct Batch {
  std::vector<int64_t> x, y;
};

struct Loader {
  const uint16_t* data = nullptr;
  size_t n_tokens = 0;
  size_t map_bytes = 0;
  int fd = -1;
  int block = 0, batch = 0, prefetch = 0;
  Rng rng{0};
  std::mutex mu;
  std::condition_variable cv_ready, cv_space;
  std::deque<Batch> ready;
  std::atomic<bool> stop{false};
  std::thread worker;

  void fill(Batch& b) {
    const size_t T = (size_t)block;
    b.x.resize((size_t)batch * T);
    b.y.resize((size_t)batch * T);
    for (int r = 0; r < batch; ++r) {
      const size_t i = (size_t)rng.below(n_tokens - T);
      const uint16_t* src = data + i;
      int64_t* xr = b.x.data() + (size_t)r * T;
      int64_t* yr = b.y.data() + (size_t)r * T;
      for (size_t t = 0; t < T; ++t) {
        xr[t] = src[t];
        yr[t] = src[t + 1];
      }
    }
  }

  void run() {
    while (!stop.load()) {
      Batch b;
      fill(b);
      std::unique_lock<std::mutex> lk(mu);
      cv_space.wait(lk, [&] { return stop.load() || (int)ready.size() < prefetch; });
      if (stop.load()) return;
      ready.push_back(std::move(b));
      cv_ready.notify_one();
    }
  }
};

}  // namespace

extern "C" {

void* nsa_loader_create(const char* path, int block, int batch, uint64_t seed, int prefetch) {
  int fd = ::open(path, O_RDONLY);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < (off_t)(2 * (block + 2))) {
    ::close(fd);
    return nullptr;
  }
  void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    ::close(fd);
    return nullptr;
  }
  madvise(m, (size_t)st.st_size, MADV_RANDOM);
  auto* L = new Loader();
  L->data = static_cast<const uint16_t*>(m);
  L->map_bytes = (size_t)st.st_size;
  L->n_tokens = (size_t)st.st_size / sizeof(uint16_t);
  L->fd = fd;
  L->block = block;
  L->batch = batch;
  L->prefetch = prefetch > 0 ? prefetch : 2;
  L->rng = Rng(seed);
  L->worker = std::thread([L] { L->run(); });
  return L;
}

int nsa_loader_next(void* h, int64_t* x, int64_t* y) {
  auto* L = static_cast<Loader*>(h);
  if (!L) return 1;
  Batch b;
  {
    std::unique_lock<std::mutex> lk(L->mu);
    L->cv_ready.wait(lk, [&] { return !L->ready.empty(); });
    b = std::move(L->ready.front());
    L->ready.pop_front();
    L->cv_space.notify_one();
  }
  std::memcpy(x, b.x.data(), b.x.size() * sizeof(int64_t));
  std::memcpy(y, b.y.data(), b.y.size() * sizeof(int64_t));
  return 0;
}

int64_t nsa_loader_num_tokens(void* h) {
  auto* L = static_cast<Loader*>(h);
  return L ? (int64_t)L->n_tokens : -1;
}

void nsa_loader_destroy(void* h) {
  auto* L = static_cast<Loader*>(h);
  if (!L) return;
  {
    std::lock_guard<std::mutex> lk(L->mu);
    L->stop.store(true);
  }
  L->cv_space.notify_all();
  L->cv_ready.notify_all();
  if (L->worker.joinable()) L->worker.join();
  munmap(const_cast<uint16_t*>(L->data), L->map_bytes);
  ::close(L->fd);
  delete L;
}

}  // extern "C"
