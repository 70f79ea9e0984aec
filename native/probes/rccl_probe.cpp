// RCCL all-reduce probe, bf16 sum, message sizes 1 MiB .. 1 GiB (256 MiB with --quick): algbw and
// busbw per size, one process per GPU across the GPUs of one node or, with a TCP-bootstrapped
// unique id, of all nodes.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include <string>
#include <thread>
#include <vector>

#include "ranks.h"

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

// One communicator over every GPU of every node, in the job's process layout: one process per GPU
// (ranks.h forks them before this process touches HIP), global rank node_rank*G + local, every rank
// calling ncclCommInitRank with the ncclUniqueId that global rank 0 creates and serves over TCP at
// master:port (bootstrap.h) -- exactly what a `torchrun --nproc-per-node=G` job does through its
// TCP store, not ncclCommInitAll's or a group-initialised single-process shortcut.
//
// Each rank first checks the sum of an fp32 all-reduce (every rank contributes rank+1), then times
// an in-place bf16 sum sweep (1 MiB .. 1 GiB, 256 MiB with --quick, at most --max-mib: the
// runner's concurrent pre-flight caps it so the probe takes little HBM and link time beside a
// starting job) on its own stream.  The parent
// takes, per size, the slowest local rank: algbw = bytes / time, busbw = algbw * 2(W-1)/W
// (ring-bound; compare with one xGMI link, ~153 GB/s, intra-node).  At W == 1 RCCL moves no data
// between GPUs, so the sweep is reported with busbw null: it proves the bootstrap and the
// communicator, it is not a bandwidth measurement.
static std::string rank_body(const dsa::RankCtx& c, const std::string& id_bytes, bool quick, size_t cap_bytes) {
  ncclUniqueId id;
  memcpy(&id, id_bytes.data(), sizeof id);
  HCK(hipSetDevice(c.local));
  ncclComm_t comm;
  NCK(ncclCommInitRank(&comm, c.world, id, c.rank));
  hipStream_t st;
  HCK(hipStreamCreate(&st));
  // correctness: sum of (rank + 1) over all ranks, exact in fp32
  const int nchk = 1024;
  std::vector<float> h((size_t)nchk, (float)(c.rank + 1));
  float* dchk = nullptr;
  HCK(hipMalloc(&dchk, nchk * sizeof(float)));
  HCK(hipMemcpy(dchk, h.data(), nchk * sizeof(float), hipMemcpyHostToDevice));
  NCK(ncclAllReduce(dchk, dchk, nchk, ncclFloat32, ncclSum, comm, st));
  HCK(hipStreamSynchronize(st));
  HCK(hipMemcpy(h.data(), dchk, nchk * sizeof(float), hipMemcpyDeviceToHost));
  const float want = (float)c.world * (c.world + 1) / 2.0f;
  bool ok = true;
  for (float v : h) ok = ok && v == want;
  HCK(hipFree(dchk));
  size_t max_bytes = (quick ? 256ull : 1024ull) << 20;
  if (cap_bytes >= (1u << 20) && cap_bytes < max_bytes) max_bytes = cap_bytes;
  void* buf = nullptr;
  HCK(hipMalloc(&buf, max_bytes));
  HCK(hipMemset(buf, 0, max_bytes));
  std::string times = "[";
  for (size_t bytes = 1 << 20; bytes <= max_bytes; bytes *= 4) {
    const size_t count = bytes / 2;  // bf16
    for (int r = 0; r < 2; ++r) NCK(ncclAllReduce(buf, buf, count, ncclBfloat16, ncclSum, comm, st));
    const int reps = quick ? 5 : 20;
    hipEvent_t e0, e1;
    HCK(hipEventCreate(&e0));
    HCK(hipEventCreate(&e1));
    HCK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) NCK(ncclAllReduce(buf, buf, count, ncclBfloat16, ncclSum, comm, st));
    HCK(hipEventRecord(e1, st));
    HCK(hipEventSynchronize(e1));
    float ms = 0;
    HCK(hipEventElapsedTime(&ms, e0, e1));
    char b[64];
    snprintf(b, sizeof b, "%s%.2f", times.size() > 1 ? ", " : "", ms * 1e3 / reps);
    times += b;
    HCK(hipEventDestroy(e0));
    HCK(hipEventDestroy(e1));
  }
  times += "]";
  HCK(hipFree(buf));
  HCK(hipStreamDestroy(st));
  ncclCommDestroy(comm);
  char head[96];
  snprintf(head, sizeof head, "{\"rank\": %d, \"sum_ok\": %s, \"times_us\": ", c.rank, ok ? "true" : "false");
  return head + times + "}";
}

// Numbers of a rank's result line ("times_us": [...]) -- the line is our own fixed format.
static std::vector<double> parse_times(const std::string& line) {
  std::vector<double> v;
  size_t p = line.find("\"times_us\": [");
  if (p == std::string::npos) return v;
  p += 13;
  while (p < line.size() && line[p] != ']') {
    char* end = nullptr;
    double x = strtod(line.c_str() + p, &end);
    if (end == line.c_str() + p) break;
    v.push_back(x);
    p = (size_t)(end - line.c_str());
    while (p < line.size() && (line[p] == ',' || line[p] == ' ')) ++p;
  }
  return v;
}

std::string rccl_allreduce_probe_mp(int gpus_per_node, int nodes, int node_rank, const std::string& master, int port,
                                    bool quick, int timeout_ms, double* best_busbw, int* world_out, std::string* err,
                                    int max_mib) {
  const size_t cap_bytes = max_mib > 0 ? (size_t)max_mib << 20 : 0;
  const int world = nodes * gpus_per_node;
  *world_out = world;
  *best_busbw = 0;
  std::string e;
  auto results = dsa::run_ranks(
      gpus_per_node, nodes, node_rank, master, port, sizeof(ncclUniqueId),
      [](std::string& id) {
        ncclUniqueId u;
        if (ncclGetUniqueId(&u) != ncclSuccess) return std::string("ncclGetUniqueId failed");
        memcpy(&id[0], &u, sizeof u);
        return std::string();
      },
      [quick, cap_bytes](const dsa::RankCtx& c, const std::string& id) { return rank_body(c, id, quick, cap_bytes); },
      timeout_ms, &e);
  std::vector<double> worst;  // per size: slowest local rank (us)
  for (auto& r : results) {
    if (r.line.find("\"sum_ok\": false") != std::string::npos && e.empty())
      e = "rank " + std::to_string(node_rank * gpus_per_node + r.local) + ": all-reduce sum mismatch";
    if (r.line.find("\"error\"") != std::string::npos && e.empty()) e = r.line;
    auto t = parse_times(r.line);
    if (t.size() > worst.size()) worst.resize(t.size(), 0.0);
    for (size_t k = 0; k < t.size(); ++k) worst[k] = std::max(worst[k], t[k]);
  }
  if (!e.empty() && err) *err = e;
  std::string out = "[";
  size_t bytes = 1 << 20;
  for (size_t k = 0; k < worst.size(); ++k, bytes *= 4) {
    const double sec = worst[k] * 1e-6;
    const double algbw = sec > 0 ? bytes / sec / 1e9 : 0.0;
    const double busbw = world > 1 ? algbw * 2.0 * (world - 1) / world : 0.0;
    if (busbw > *best_busbw) *best_busbw = busbw;
    char b[200];
    snprintf(b, sizeof b, "%s{\"bytes\": %zu, \"time_us\": %.1f, \"algbw_gb_s\": %.1f, \"busbw_gb_s\": %.1f}",
             k ? ", " : "", bytes, worst[k], algbw, busbw);
    out += b;
  }
  return out + "]";
}
