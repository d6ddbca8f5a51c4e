// Host-side stress driver for the native prefetching loader (csrc/runtime/dataloader.cpp),
// built and run under AddressSanitizer + UBSan and under ThreadSanitizer by
// tests/test_sanitizers.py (race detection / sanitizers on host code).
//
// It writes a token file whose token at position p is (p * 7 + 3) % 65521, then for
// several (block, batch, prefetch) shapes: pulls batches and checks every window
// against the formula (x[t] = data[i + t], y[t] = data[i + t + 1], i in range), and
// destroys loaders at random points while the producer thread is mid-fill or blocked on
// a full ring (the shutdown path TSan watches).  Exit code 0 = all checks passed.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

extern "C" {
void* nsa_loader_create(const char* path, int block, int batch, uint64_t seed, int prefetch);
int nsa_loader_next(void* h, int64_t* x, int64_t* y);
int64_t nsa_loader_num_tokens(void* h);
void nsa_loader_destroy(void* h);
}

static uint16_t tok(int64_t p) { return (uint16_t)((p * 7 + 3) % 65521); }

static int check_batch(const std::vector<int64_t>& x, const std::vector<int64_t>& y, int block, int batch,
                       int64_t n) {
  for (int r = 0; r < batch; ++r) {
    const int64_t* xr = x.data() + (int64_t)r * block;
    const int64_t* yr = y.data() + (int64_t)r * block;
    // recover the window start from x[0]: tokens are a bijection on positions < 65521
    int64_t i = -1;
    for (int64_t p = 0; p < n && p < 65521; ++p)
      if (tok(p) == xr[0]) {
        i = p;
        break;
      }
    if (i < 0 || i + block >= n) return 1;
    for (int t = 0; t < block; ++t)
      if (xr[t] != tok(i + t) || yr[t] != tok(i + t + 1)) return 2;
  }
  return 0;
}

int main(int argc, char** argv) {
  const std::string path = argc > 1 ? argv[1] : "/tmp/nsa_loader_stress.bin";
  const int64_t n = 60000;  // < 65521: x[0] identifies the window start
  {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return 10;
    for (int64_t p = 0; p < n; ++p) {
      const uint16_t v = tok(p);
      std::fwrite(&v, sizeof v, 1, f);
    }
    std::fclose(f);
  }
  struct Shape {
    int block, batch, prefetch;
  };
  const Shape shapes[] = {{8, 1, 1}, {64, 4, 2}, {256, 16, 4}, {1024, 3, 8}};
  int failures = 0;
  for (const Shape& s : shapes) {
    void* h = nsa_loader_create(path.c_str(), s.block, s.batch, 1234 + s.block, s.prefetch);
    if (!h || nsa_loader_num_tokens(h) != n) return 11;
    std::vector<int64_t> x((size_t)s.block * s.batch), y(x.size());
    for (int it = 0; it < 40; ++it) {
      if (nsa_loader_next(h, x.data(), y.data()) != 0) return 12;
      failures += check_batch(x, y, s.block, s.batch, n) != 0;
    }
    nsa_loader_destroy(h);
  }
  // shutdown races: destroy right after create, after a few batches, and while the
  // producer is blocked on a full ring (sleep lets it fill every slot)
  for (int k = 0; k < 30; ++k) {
    void* h = nsa_loader_create(path.c_str(), 32, 2, (uint64_t)k, 1 + k % 3);
    if (!h) return 13;
    std::vector<int64_t> x(64), y(64);
    for (int it = 0; it < k % 4; ++it) nsa_loader_next(h, x.data(), y.data());
    if (k % 5 == 0) std::this_thread::sleep_for(std::chrono::milliseconds(2));
    nsa_loader_destroy(h);
  }
  // a loader per thread, used concurrently (separate handles share nothing)
  std::vector<std::thread> ts;
  std::vector<int> bad(4, 0);
  for (int t = 0; t < 4; ++t)
    ts.emplace_back([&, t] {
      void* h = nsa_loader_create(path.c_str(), 128, 2, 99 + t, 2);
      std::vector<int64_t> x(256), y(256);
      for (int it = 0; it < 25; ++it) {
        nsa_loader_next(h, x.data(), y.data());
        bad[t] += check_batch(x, y, 128, 2, n) != 0;
      }
      nsa_loader_destroy(h);
    });
  for (auto& th : ts) th.join();
  for (int b : bad) failures += b;
  std::remove(path.c_str());
  if (failures) {
    std::fprintf(stderr, "loader_stress: %d bad batches\n", failures);
    return 1;
  }
  std::printf("loader_stress: ok\n");
  return 0;
}
