// RCCL collective micro-benchmark for sizing DDP gradient buckets over xGMI
// (traceability row "C1-C6 -> csrc/comm/rccl_bench.cpp").
//
// Why it exists: the flat-buffer reducer (nanosandbox_amd/parallel/reducer.py) launches
// one all-reduce per bucket as soon as backward has produced the bucket's gradients.
// On MI355X every GPU has 7 point-to-point xGMI links (~153 GB/s each), so a ring
// all-reduce is per-link bound and RCCL needs messages of tens of MiB before its
// channels spread over the links; too-small buckets pay launch + latency per bucket,
// too-large ones delay the first launch and shrink the overlap with backward.  This
// tool measures bus bandwidth vs message size and prints the smallest size that
// reaches a given fraction of the best bus bandwidth — the recommended
// `ddp_bucket_mb`.
//
// Two launch modes (both one RCCL rank per GPU):
//   * single process, all visible GPUs:   rccl_bench --ranks 8
//     (ncclCommInitAll + one HIP stream per device, collectives grouped)
//   * one process per GPU (torchrun / any launcher setting RANK, WORLD_SIZE,
//     LOCAL_RANK):   rccl_bench --id-file /dev/shm/rccl.id
//     rank 0 writes the ncclUniqueId to the file (atomic rename), the others poll it.
//
// Output: one JSON line per (op, size) and a final {"recommend_bucket_mb": ...} line.
// Build: python -m nanosandbox_amd.build (hipcc --offload-arch=gfx950 ... -lrccl).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#define HIP_OK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                      \
    }                                                                                    \
  } while (0)
#define NCCL_OK(x)                                                                       \
  do {                                                                                   \
    ncclResult_t r_ = (x);                                                               \
    if (r_ != ncclSuccess) {                                                             \
      std::fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      std::exit(3);                                                                      \
    }                                                                                    \
  } while (0)

namespace {

enum class Op { AllReduce, ReduceScatter, AllGather, Broadcast };

struct Options {
  int ranks = 0;  // single-process mode: number of GPUs (0 = all visible)
  std::string id_file;
  double min_mb = 1.0, max_mb = 512.0;
  int iters = 20, warmup = 5;
  ncclDataType_t dtype = ncclFloat32;
  std::vector<Op> ops{Op::AllReduce};
  double target = 0.9;  // fraction of the best bus bandwidth for the recommendation
};

const char* op_name(Op o) {
  switch (o) {
    case Op::AllReduce: return "all_reduce";
    case Op::ReduceScatter: return "reduce_scatter";
    case Op::AllGather: return "all_gather";
    default: return "broadcast";
  }
}

// bus-bandwidth factor of the ring algorithms (bytes on the busiest link / message size)
double bus_factor(Op o, int n) {
  if (n <= 1) return 1.0;
  switch (o) {
    case Op::AllReduce: return 2.0 * (n - 1) / n;
    case Op::ReduceScatter:
    case Op::AllGather: return double(n - 1) / n;
    default: return 1.0;
  }
}

size_t elem_size(ncclDataType_t t) { return t == ncclFloat32 ? 4 : 2; }

ncclResult_t run_op(Op o, void* buf, void* out, size_t count, ncclDataType_t t, int nranks, ncclComm_t comm,
                    hipStream_t s) {
  switch (o) {
    case Op::AllReduce: return ncclAllReduce(buf, buf, count, t, ncclSum, comm, s);
    case Op::ReduceScatter: return ncclReduceScatter(buf, out, count / nranks, t, ncclSum, comm, s);
    case Op::AllGather: return ncclAllGather(out, buf, count / nranks, t, comm, s);
    default: return ncclBroadcast(buf, buf, count, t, 0, comm, s);
  }
}

int env_int(const char* k, int dflt) {
  const char* v = std::getenv(k);
  return v ? std::atoi(v) : dflt;
}

Options parse(int argc, char** argv) {
  Options o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", a.c_str());
        std::exit(1);
      }
      return argv[++i];
    };
    if (a == "--ranks") o.ranks = std::stoi(next());
    else if (a == "--id-file") o.id_file = next();
    else if (a == "--min-mb") o.min_mb = std::stod(next());
    else if (a == "--max-mb") o.max_mb = std::stod(next());
    else if (a == "--iters") o.iters = std::stoi(next());
    else if (a == "--warmup") o.warmup = std::stoi(next());
    else if (a == "--target") o.target = std::stod(next());
    else if (a == "--dtype") {
      std::string d = next();
      o.dtype = d == "bf16" ? ncclBfloat16 : ncclFloat32;
    } else if (a == "--ops") {
      o.ops.clear();
      std::string s = next();
      size_t p = 0;
      while (p <= s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        std::string t = s.substr(p, q - p);
        if (t == "all_reduce") o.ops.push_back(Op::AllReduce);
        else if (t == "reduce_scatter") o.ops.push_back(Op::ReduceScatter);
        else if (t == "all_gather") o.ops.push_back(Op::AllGather);
        else if (t == "broadcast") o.ops.push_back(Op::Broadcast);
        p = q + 1;
      }
    } else if (a == "-h" || a == "--help") {
      std::printf(
          "rccl_bench [--ranks N | --id-file PATH] [--min-mb 1] [--max-mb 512] [--iters 20] [--warmup 5]\n"
          "           [--dtype f32|bf16] [--ops all_reduce,reduce_scatter,all_gather,broadcast] [--target 0.9]\n");
      std::exit(0);
    } else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      std::exit(1);
    }
  }
  return o;
}

// rank 0 publishes the id by atomic rename; the others poll for up to 120 s
ncclUniqueId exchange_id(const std::string& path, int rank) {
  ncclUniqueId id;
  if (rank == 0) {
    NCCL_OK(ncclGetUniqueId(&id));
    const std::string tmp = path + ".tmp";
    std::ofstream f(tmp, std::ios::binary);
    f.write(id.internal, NCCL_UNIQUE_ID_BYTES);
    f.close();
    std::rename(tmp.c_str(), path.c_str());
    return id;
  }
  for (int t = 0; t < 12000; ++t) {
    std::ifstream f(path, std::ios::binary);
    if (f.good()) {
      f.read(id.internal, NCCL_UNIQUE_ID_BYTES);
      if (f.gcount() == NCCL_UNIQUE_ID_BYTES) return id;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  std::fprintf(stderr, "rank %d: timed out waiting for %s\n", rank, path.c_str());
  std::exit(4);
}

}  // namespace

int main(int argc, char** argv) {
  Options opt = parse(argc, argv);
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  if (ndev < 1) {
    std::fprintf(stderr, "no GPU visible\n");
    return 5;
  }

  const bool multi_proc = !opt.id_file.empty();
  const int world = multi_proc ? env_int("WORLD_SIZE", 1) : (opt.ranks > 0 ? std::min(opt.ranks, ndev) : ndev);
  const int rank = multi_proc ? env_int("RANK", 0) : 0;
  const int local_rank = multi_proc ? env_int("LOCAL_RANK", rank) : 0;
  const int nlocal = multi_proc ? 1 : world;  // devices driven by this process

  std::vector<int> devs(nlocal);
  for (int i = 0; i < nlocal; ++i) devs[i] = multi_proc ? local_rank % ndev : i;
  std::vector<ncclComm_t> comms(nlocal);
  if (multi_proc) {
    ncclUniqueId id = exchange_id(opt.id_file, rank);
    HIP_OK(hipSetDevice(devs[0]));
    NCCL_OK(ncclCommInitRank(&comms[0], world, id, rank));
  } else {
    NCCL_OK(ncclCommInitAll(comms.data(), nlocal, devs.data()));
  }

  const size_t esz = elem_size(opt.dtype);
  const size_t max_bytes = (size_t)(opt.max_mb * 1024 * 1024);
  std::vector<void*> buf(nlocal), out(nlocal);
  std::vector<hipStream_t> streams(nlocal);
  for (int i = 0; i < nlocal; ++i) {
    HIP_OK(hipSetDevice(devs[i]));
    HIP_OK(hipMalloc(&buf[i], max_bytes));
    HIP_OK(hipMalloc(&out[i], max_bytes));
    HIP_OK(hipMemset(buf[i], 0, max_bytes));
    HIP_OK(hipStreamCreateWithFlags(&streams[i], hipStreamNonBlocking));
  }

  auto launch_all = [&](Op o, size_t count) {
    NCCL_OK(ncclGroupStart());
    for (int i = 0; i < nlocal; ++i) NCCL_OK(run_op(o, buf[i], out[i], count, opt.dtype, world, comms[i], streams[i]));
    NCCL_OK(ncclGroupEnd());
  };
  auto sync_all = [&]() {
    for (int i = 0; i < nlocal; ++i) {
      HIP_OK(hipSetDevice(devs[i]));
      HIP_OK(hipStreamSynchronize(streams[i]));
    }
  };

  double best_bus = 0.0;
  std::vector<std::pair<double, double>> ar_curve;  // (MiB, bus GB/s) of all_reduce
  for (Op o : opt.ops) {
    for (double mb = opt.min_mb; mb <= opt.max_mb + 1e-9; mb *= 2.0) {
      size_t bytes = (size_t)(mb * 1024 * 1024);
      size_t count = bytes / esz;
      count -= count % (size_t)(world * 64);  // divisible for reduce_scatter / all_gather
      if (count == 0) continue;
      for (int w = 0; w < opt.warmup; ++w) launch_all(o, count);
      sync_all();
      const auto t0 = std::chrono::steady_clock::now();
      for (int it = 0; it < opt.iters; ++it) launch_all(o, count);
      sync_all();
      const double us =
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / opt.iters;
      const double algbw = (double)(count * esz) / (us * 1e-6) / 1e9;
      const double busbw = algbw * bus_factor(o, world);
      if (rank == 0)
        std::printf(
            "{\"op\": \"%s\", \"ranks\": %d, \"dtype\": \"%s\", \"mib\": %.3f, \"time_us\": %.1f, "
            "\"algbw_GBps\": %.2f, \"busbw_GBps\": %.2f}\n",
            op_name(o), world, opt.dtype == ncclFloat32 ? "f32" : "bf16", count * esz / 1048576.0, us, algbw, busbw);
      if (o == Op::AllReduce) {
        ar_curve.emplace_back(count * esz / 1048576.0, busbw);
        best_bus = std::max(best_bus, busbw);
      }
    }
  }
  if (rank == 0 && !ar_curve.empty()) {
    double rec = ar_curve.back().first;
    for (auto& p : ar_curve)
      if (p.second >= opt.target * best_bus) {
        rec = p.first;
        break;
      }
    std::printf("{\"recommend_bucket_mb\": %.1f, \"best_busbw_GBps\": %.2f, \"target_fraction\": %.2f, \"ranks\": %d}\n",
                rec, best_bus, opt.target, world);
  }
  std::fflush(stdout);
  for (int i = 0; i < nlocal; ++i) {
    HIP_OK(hipSetDevice(devs[i]));
    HIP_OK(hipFree(buf[i]));
    HIP_OK(hipFree(out[i]));
    HIP_OK(hipStreamDestroy(streams[i]));
    ncclCommDestroy(comms[i]);
  }
  if (multi_proc && rank == 0) std::remove(opt.id_file.c_str());
  return 0;
}
