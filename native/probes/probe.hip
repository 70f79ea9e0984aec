// dstack-probe: per-GPU health probes for MI355X hosts (hand-written HIP, gfx950).
//
//   dstack-probe [--quick] [--json] [--hbm] [--mfma] [--xgmi] [--rccl] [--device N]
//
// * HBM:  streaming copy over 2 x 1 GiB buffers, 16-byte (dwordx4) loads/stores, one element per
//         thread over a full grid -> achieved TB/s (MI355X measured ceiling ~6.3 TB/s, spec 8).
// * MFMA: register-resident bf16 (v_mfma_f32_32x32x16_bf16) and fp8 (block-scaled 32x32x64 f8f6f4) loops,
//         4 independent accumulators per wave, 4 waves per CU on every CU -> dense TFLOPS and the
//         implied clock; a throttled or faulty GPU shows up as a low number.
// * xGMI: hipMemcpyPeerAsync of 256 MiB for every ordered GPU pair -> GB/s matrix (a healthy
//         MI355X link moves ~100+ GB/s one-way; PCIe-routed pairs are far slower).
// * RCCL: all-reduce bf16 sweep across all visible GPUs (see rccl_probe.cpp).
// Results are one JSON document; exit status 1 if any GPU falls below the health thresholds.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "ranks.h"

#define CK(x)                                                                                    \
  do {                                                                                           \
    hipError_t e_ = (x);                                                                         \
    if (e_ != hipSuccess) {                                                                      \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);     \
      exit(2);                                                                                   \
    }                                                                                            \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ------------------------------------------------------------------------------------------------
// One 16-byte element per thread over a full grid (n/256 blocks): blocks are dispatched in address
// order, so the chip streams memory front to back.  Measured on MI355X (tools/diag/hbm_variants.hip,
// 1 GiB copy): 6.18 TB/s, vs 4.2-4.8 TB/s for grid-stride loops (8-32 blocks/CU, 1 or 4 loads in
// flight, nt loads) whose every iteration jumps across the whole buffer.
__global__ __launch_bounds__(256) void copy_kernel(const f4* __restrict__ src, f4* __restrict__ dst, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void fill_kernel(f4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = f4{1.f, 2.f, 3.f, (float)(i & 1023)};
}

// bf16 MFMA loop: 4 independent 32x32 accumulators per wave; operands derived from the lane id so
// the compiler cannot constant-fold; the checksum store keeps everything live.
__global__ __launch_bounds__(256) void mfma_bf16_kernel(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)(0.001f * (float)((lane + j) & 7));
    b[j] = (__bf16)(0.002f * (float)((lane * 3 + j) & 7));
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;  // never true; keeps MFMAs live
}

// fp8 at the CDNA4 rate: the block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3 operands, unit
// E8M0 scales) runs a 32x32x64 product in twice the cycles of the bf16 32x32x16, i.e. 2x the bf16
// rate; the non-scaled 32x32x16_fp8_fp8 only matches bf16 (measured 2427 TF, profiles/probe_r1.json)
typedef int i32x8 __attribute__((ext_vector_type(8)));
__global__ __launch_bounds__(256) void mfma_fp8_kernel(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  i32x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = 0x38302820 + ((lane + j) & 7);
    b[j] = 0x39312921 + ((lane * 7 + j) & 7);
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 0, 0, 0, 127, 0, 127);
    c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c1, 0, 0, 0, 127, 0, 127);
    c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c2, 0, 0, 0, 127, 0, 127);
    c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c3, 0, 0, 0, 127, 0, 127);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 1234.5f) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// ------------------------------------------------------------------------------------------------
static float time_ms(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

static double hbm_probe(int dev, bool quick) {
  CK(hipSetDevice(dev));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, dev));
  size_t bytes = (quick ? 256ull : 1024ull) << 20;
  size_t n = bytes / sizeof(f4);
  f4 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  int grid = p.multiProcessorCount * 8;
  fill_kernel<<<grid, 256>>>(a, n);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int cgrid = (int)((n + 255) / 256);
  copy_kernel<<<cgrid, 256>>>(a, b, n);  // warm
  const int reps = quick ? 5 : 20;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) copy_kernel<<<cgrid, 256>>>(r & 1 ? b : a, r & 1 ? a : b, n);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  double tb_s = 2.0 * bytes * reps / (time_ms(e0, e1) * 1e-3) / 1e12;
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return tb_s;
}

static double mfma_probe(int dev, bool quick, bool fp8) {
  CK(hipSetDevice(dev));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, dev));
  float* out;
  CK(hipMalloc(&out, (size_t)p.multiProcessorCount * 256 * 4 * sizeof(float)));
  const int iters = quick ? 20000 : 100000;
  const int blocks = p.multiProcessorCount * 2;  // 2 blocks x 4 waves per CU = 2 waves per SIMD
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto launch = [&](int it) {
    if (fp8)
      mfma_fp8_kernel<<<blocks, 256>>>(out, it);
    else
      mfma_bf16_kernel<<<blocks, 256>>>(out, it);
  };
  launch(1000);
  CK(hipEventRecord(e0));
  launch(iters);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  // bf16 32x32x16 MFMA = 2*32*32*16 FLOP, fp8 32x32x64 = 2*32*32*64; 4 per iteration per wave;
  // 4 waves per block
  double flops = 2.0 * 32 * 32 * (fp8 ? 64 : 16) * 4.0 * iters * 4.0 * blocks;
  double tflops = flops / (time_ms(e0, e1) * 1e-3) / 1e12;
  CK(hipFree(out));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return tflops;
}

static std::vector<std::vector<double>> xgmi_probe(int ndev, bool quick) {
  std::vector<std::vector<double>> m((size_t)ndev, std::vector<double>((size_t)ndev, 0.0));
  size_t bytes = (quick ? 64ull : 256ull) << 20;
  std::vector<void*> buf((size_t)ndev);
  for (int d = 0; d < ndev; ++d) {
    CK(hipSetDevice(d));
    CK(hipMalloc(&buf[(size_t)d], bytes));
    for (int e = 0; e < ndev; ++e) {
      if (e == d) continue;
      int can = 0;
      CK(hipDeviceCanAccessPeer(&can, d, e));
      if (can) (void)hipDeviceEnablePeerAccess(e, 0);
    }
  }
  (void)hipGetLastError();
  for (int s = 0; s < ndev; ++s)
    for (int d = 0; d < ndev; ++d) {
      if (s == d) continue;
      CK(hipSetDevice(s));
      hipStream_t st;
      CK(hipStreamCreate(&st));
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      CK(hipMemcpyPeerAsync(buf[(size_t)d], d, buf[(size_t)s], s, bytes, st));
      const int reps = quick ? 3 : 10;
      CK(hipEventRecord(e0, st));
      for (int r = 0; r < reps; ++r) CK(hipMemcpyPeerAsync(buf[(size_t)d], d, buf[(size_t)s], s, bytes, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      m[(size_t)s][(size_t)d] = (double)bytes * reps / (time_ms(e0, e1) * 1e-3) / 1e9;
      CK(hipEventDestroy(e0));
      CK(hipEventDestroy(e1));
      CK(hipStreamDestroy(st));
    }
  for (int d = 0; d < ndev; ++d) {
    CK(hipSetDevice(d));
    CK(hipFree(buf[(size_t)d]));
  }
  return m;
}

// rccl_probe.cpp
std::string rccl_allreduce_probe_mp(int gpus_per_node, int nodes, int node_rank, const std::string& master, int port,
                                    bool quick, int timeout_ms, double* best_busbw, int* world_out, std::string* err,
                                    int max_mib);


// Per-SKU baselines: what THIS probe measures on a healthy part (not the datasheet peaks), so a
// threshold of min_fraction x baseline flags a GPU running well below its siblings (throttling,
// a bad HBM stack, a degraded link).  MI355X: profiles/probe_r1q.json (6.05 TB/s copy, 2.10 PF
// bf16, 4.98 PF fp8).  MI300X-class numbers are scaled from its datasheet ratios.  Unknown parts
// fall back to absolute floors far below any current Instinct part.
struct Baseline {
  const char* sku;
  double hbm_tb_s, bf16_tflops, fp8_tflops;
};
static Baseline baseline_for(int dev) {
  hipDeviceProp_t p{};
  if (hipGetDeviceProperties(&p, dev) != hipSuccess) return {"unknown", 2.5, 600.0, 0.0};
  const std::string arch = p.gcnArchName;
  if (arch.rfind("gfx950", 0) == 0) return {"MI355X", 6.0, 2100.0, 4900.0};
  if (arch.rfind("gfx942", 0) == 0) return {"MI300X", 4.2, 900.0, 1800.0};
  return {"unknown", 2.5, 600.0, 0.0};
}

int main(int argc, char** argv) {
  bool quick = false, json = false, want_hbm = false, want_mfma = false, want_xgmi = false, want_rccl = false;
  int only_dev = -1;
  double min_hbm = -1, min_mfma = -1;  // absolute overrides; default: min_fraction x per-SKU baseline
  double min_fraction = 0.8;
  int rccl_nodes = 1, node_rank = 0, master_port = 29600, gpus_per_node = 0;
  int rccl_max_mib = 0;  // 0: the full sweep
  int rccl_timeout_ms = 300000;  // per-rank bootstrap + sweep budget (the runner derives it from its own limit)
  std::string master = "127.0.0.1";
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a == "--quick") quick = true;
    else if (a == "--json") json = true;
    else if (a == "--hbm") want_hbm = true;
    else if (a == "--mfma") want_mfma = true;
    else if (a == "--xgmi") want_xgmi = true;
    else if (a == "--rccl") want_rccl = true;
    else if (a == "--device" && i + 1 < argc) only_dev = atoi(argv[++i]);
    else if (a == "--min-hbm-tbs" && i + 1 < argc) min_hbm = atof(argv[++i]);
    else if (a == "--min-mfma-tflops" && i + 1 < argc) min_mfma = atof(argv[++i]);
    else if (a == "--min-fraction" && i + 1 < argc) min_fraction = atof(argv[++i]);
    else if (a == "--nodes" && i + 1 < argc) rccl_nodes = atoi(argv[++i]);
    else if (a == "--node-rank" && i + 1 < argc) node_rank = atoi(argv[++i]);
    else if (a == "--master" && i + 1 < argc) master = argv[++i];
    else if (a == "--master-port" && i + 1 < argc) master_port = atoi(argv[++i]);
    else if (a == "--gpus-per-node" && i + 1 < argc) gpus_per_node = atoi(argv[++i]);
    else if (a == "--max-mib" && i + 1 < argc) rccl_max_mib = atoi(argv[++i]);
    else if (a == "--timeout-ms" && i + 1 < argc) {
      const int t = atoi(argv[++i]);
      if (t > 0) rccl_timeout_ms = t;
    }
    else {
      fprintf(stderr,
              "usage: dstack-probe [--quick] [--json] [--hbm] [--mfma] [--xgmi] [--rccl] [--device N]\n"
              "                    [--min-fraction F | --min-hbm-tbs X --min-mfma-tflops Y]\n"
              "                    [--rccl [--gpus-per-node G] --nodes N --node-rank R --master HOST --master-port P\n"
              "                     [--timeout-ms T] [--max-mib M]]\n");
      return 2;
    }
  }
  if (!want_hbm && !want_mfma && !want_xgmi && !want_rccl) want_hbm = want_mfma = want_xgmi = true;
  // RCCL first: its one-process-per-GPU ranks are forked before THIS process makes any HIP call
  std::string rccl_json, rccl_err;
  if (want_rccl && only_dev < 0) {
    const int g = gpus_per_node > 0 ? gpus_per_node : dsa::count_gpus_no_hip();
    if (g <= 0) {
      rccl_err = "no GPUs visible";
    } else {
      double best = 0;
      int world = 0;
      std::string sweep = rccl_allreduce_probe_mp(g, rccl_nodes, node_rank, master, master_port, quick,
                                                  rccl_timeout_ms, &best, &world, &rccl_err, rccl_max_mib);
      char b[256];
      snprintf(b, sizeof b, "\"rccl_world\": %d, \"rccl_gpus_per_node\": %d, \"rccl\": ", world, g);
      rccl_json = b + sweep + ", ";
      if (world > 1) {
        snprintf(b, sizeof b, "\"rccl_busbw_gb_s\": %.1f, ", best);
        rccl_json += b;
      } else {
        rccl_json += "\"rccl_busbw_gb_s\": null, \"rccl_note\": \"world 1: no inter-GPU traffic; bootstrap and "
                     "communicator check only, not a bandwidth measurement\", ";
      }
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    printf("{\"healthy\": false, \"message\": \"no HIP devices\"}\n");
    return 1;
  }
  std::string out = "{";
  bool healthy = true;
  std::string failing;
  std::vector<int> devs;
  for (int d = 0; d < ndev; ++d)
    if (only_dev < 0 || d == only_dev) devs.push_back(d);
  char buf[512];
  const Baseline base = baseline_for(devs[0]);
  const double thr_hbm = min_hbm >= 0 ? min_hbm : min_fraction * base.hbm_tb_s;
  const double thr_mfma = min_mfma >= 0 ? min_mfma : min_fraction * base.bf16_tflops;
  snprintf(buf, sizeof buf,
           "\"sku\": \"%s\", \"baseline\": {\"hbm_tb_s\": %.2f, \"mfma_bf16_tflops\": %.0f, \"mfma_fp8_tflops\": %.0f}, "
           "\"thresholds\": {\"hbm_tb_s\": %.2f, \"mfma_bf16_tflops\": %.0f}, ",
           base.sku, base.hbm_tb_s, base.bf16_tflops, base.fp8_tflops, thr_hbm, thr_mfma);
  out += buf;
  auto fail = [&](int dev, const char* what, double v, double thr) {
    healthy = false;
    snprintf(buf, sizeof buf, "%sGPU %d %s %.2f < %.2f", failing.empty() ? "" : "; ", dev, what, v, thr);
    failing += buf;
  };
  if (want_hbm) {
    out += "\"hbm_tb_s\": [";
    for (size_t k = 0; k < devs.size(); ++k) {
      double v = hbm_probe(devs[k], quick);
      if (v < thr_hbm) fail(devs[k], "HBM TB/s", v, thr_hbm);
      snprintf(buf, sizeof buf, "%s%.3f", k ? ", " : "", v);
      out += buf;
    }
    out += "], ";
  }
  if (want_mfma) {
    out += "\"mfma_bf16_tflops\": [";
    for (size_t k = 0; k < devs.size(); ++k) {
      double v = mfma_probe(devs[k], quick, false);
      if (v < thr_mfma) fail(devs[k], "bf16 TFLOPS", v, thr_mfma);
      snprintf(buf, sizeof buf, "%s%.1f", k ? ", " : "", v);
      out += buf;
    }
    out += "], \"mfma_fp8_tflops\": [";
    for (size_t k = 0; k < devs.size(); ++k) {
      snprintf(buf, sizeof buf, "%s%.1f", k ? ", " : "", mfma_probe(devs[k], quick, true));
      out += buf;
    }
    out += "], ";
  }
  if (want_xgmi && ndev > 1 && only_dev < 0) {
    auto m = xgmi_probe(ndev, quick);
    out += "\"xgmi_gb_s\": [";
    for (int s = 0; s < ndev; ++s) {
      out += s ? ", [" : "[";
      for (int d = 0; d < ndev; ++d) {
        snprintf(buf, sizeof buf, "%s%.1f", d ? ", " : "", m[(size_t)s][(size_t)d]);
        out += buf;
      }
      out += "]";
    }
    out += "], ";
  }
  if (want_rccl && only_dev < 0) {
    out += rccl_json;
    if (!rccl_err.empty()) {
      healthy = false;
      for (auto& ch : rccl_err)
        if (ch == '"' || ch == '\\' || ch == '\n') ch = '\'';  // the message is a JSON string
      failing += (failing.empty() ? "" : "; ") + ("RCCL: " + rccl_err);
    }
  }
  snprintf(buf, sizeof buf, "\"devices\": %d, \"healthy\": %s, ", (int)devs.size(), healthy ? "true" : "false");
  out += buf;
  out += "\"message\": \"" + failing + "\"}";
  if (json)
    printf("%s\n", out.c_str());
  else
    printf("dstack-probe: %s\n", out.c_str());
  return healthy ? 0 : 1;
}
