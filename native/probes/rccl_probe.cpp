// RCCL all-reduce probe, bf16 sum, message sizes 1 MiB .. 1 GiB (256 MiB with --quick): algbw and
// busbw per size, across the GPUs of one node or, with a TCP-bootstrapped unique id, of all nodes.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <thread>
#include <vector>

#include "bootstrap.h"

#define HCK(x)                                                                               \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(2);                                                                               \
    }                                                                                        \
  } while (0)
#define NCK(x)                                                                                  \
  do {                                                                                          \
    ncclResult_t r_ = (x);                                                                      \
    if (r_ != ncclSuccess) {                                                                    \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      exit(2);                                                                                  \
    }                                                                                           \
  } while (0)

// One communicator over every GPU of every node: `nodes` processes (one per node, as the runner
// starts them), each owning all its local GPUs as ranks node_rank*ndev + d, initialised with
// ncclCommInitRank from an ncclUniqueId that node 0 creates and serves over TCP (bootstrap.h) --
// the same unique-id rendezvous a torchrun/RCCL job performs, not ncclCommInitAll's in-process
// shortcut.  nodes == 1 runs the same path with no network exchange.  busbw = algbw*2(W-1)/W
// (ring-bound; compare with one xGMI link, ~153 GB/s, intra-node).
std::string rccl_allreduce_probe_mp(int nodes, int node_rank, const std::string& master, int port, bool quick,
                                    double* best_busbw, std::string* err) {
  int ndev = 0;
  HCK(hipGetDeviceCount(&ndev));
  const int world = nodes * ndev;
  ncclUniqueId id;
  std::thread server;
  std::string serve_err;
  if (node_rank == 0) {
    NCK(ncclGetUniqueId(&id));
    if (nodes > 1)
      server = std::thread([&] { serve_err = dsa::bootstrap_serve(port, &id, sizeof id, nodes - 1, 300000); });
  } else {
    std::string e = dsa::bootstrap_fetch(master, port, node_rank, &id, sizeof id, 300000);
    if (!e.empty()) {
      if (err) *err = e;
      return "null";
    }
  }
  std::vector<ncclComm_t> comms((size_t)ndev);
  NCK(ncclGroupStart());
  for (int d = 0; d < ndev; ++d) {
    HCK(hipSetDevice(d));
    NCK(ncclCommInitRank(&comms[(size_t)d], world, id, node_rank * ndev + d));
  }
  NCK(ncclGroupEnd());
  if (server.joinable()) server.join();
  if (!serve_err.empty() && err) *err = serve_err;
  size_t max_bytes = (quick ? 256ull : 1024ull) << 20;
  std::vector<void*> buf((size_t)ndev);
  std::vector<hipStream_t> st((size_t)ndev);
  for (int d = 0; d < ndev; ++d) {
    HCK(hipSetDevice(d));
    HCK(hipMalloc(&buf[(size_t)d], max_bytes));
    HCK(hipMemset(buf[(size_t)d], 0, max_bytes));
    HCK(hipStreamCreate(&st[(size_t)d]));
  }
  std::string out = "[";
  *best_busbw = 0;
  bool first = true;
  for (size_t bytes = 1 << 20; bytes <= max_bytes; bytes *= 4) {
    size_t count = bytes / 2;  // bf16
    auto run = [&](int reps) {
      for (int r = 0; r < reps; ++r) {
        NCK(ncclGroupStart());
        for (int d = 0; d < ndev; ++d)
          NCK(ncclAllReduce(buf[(size_t)d], buf[(size_t)d], count, ncclBfloat16, ncclSum, comms[(size_t)d],
                            st[(size_t)d]));
        NCK(ncclGroupEnd());
      }
      for (int d = 0; d < ndev; ++d) {
        HCK(hipSetDevice(d));
        HCK(hipStreamSynchronize(st[(size_t)d]));
      }
    };
    run(2);
    const int reps = quick ? 5 : 20;
    hipEvent_t e0, e1;
    HCK(hipSetDevice(0));
    HCK(hipEventCreate(&e0));
    HCK(hipEventCreate(&e1));
    HCK(hipEventRecord(e0, st[0]));
    run(reps);
    HCK(hipSetDevice(0));
    HCK(hipEventRecord(e1, st[0]));
    HCK(hipEventSynchronize(e1));
    float ms = 0;
    HCK(hipEventElapsedTime(&ms, e0, e1));
    double sec = ms * 1e-3 / reps;
    double algbw = bytes / sec / 1e9;
    double busbw = world > 1 ? algbw * 2.0 * (world - 1) / world : 0.0;
    if (busbw > *best_busbw) *best_busbw = busbw;
    char b[200];
    snprintf(b, sizeof b, "%s{\"bytes\": %zu, \"time_us\": %.1f, \"algbw_gb_s\": %.1f, \"busbw_gb_s\": %.1f}",
             first ? "" : ", ", bytes, sec * 1e6, algbw, busbw);
    out += b;
    first = false;
    HCK(hipEventDestroy(e0));
    HCK(hipEventDestroy(e1));
  }
  out += "]";
  for (int d = 0; d < ndev; ++d) {
    HCK(hipSetDevice(d));
    HCK(hipFree(buf[(size_t)d]));
    HCK(hipStreamDestroy(st[(size_t)d]));
    ncclCommDestroy(comms[(size_t)d]);
  }
  return out;
}
