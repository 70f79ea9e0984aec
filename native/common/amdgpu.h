// AMD GPU discovery, xGMI topology and live metrics for the native agents.
//
// Primary source: the amdsmi C library (libamd_smi.so, dlopen'ed so the agents still start on
// CPU-only hosts).  Fallback: sysfs (/sys/class/drm/renderD*/device, KFD topology) for discovery.
// Replaces the reference's `docker run amd-smi static --json` + CSV parsing
// (runner/internal/shim/host/gpu.go:149-196, runner/internal/metrics/metrics.go:172-203).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "json.h"

namespace dsa {

struct AmdGpu {
  int index = 0;             // PCI BDF order on the host (amdsmi and sysfs discovery agree on it)
  std::string name;          // catalog name, e.g. MI355X
  std::string market_name;   // raw amdsmi market name
  std::string arch;          // gfx950
  uint64_t vram_mib = 0;
  std::string bdf;           // 0000:23:00.0
  std::string render_node;   // /dev/dri/renderD128
  int drm_render = -1;
  int numa_node = -1;
  std::string serial;
};

struct AmdGpuMetrics {
  int index = 0;
  double util_percent = 0;
  uint64_t vram_used_bytes = 0;
  uint64_t vram_total_bytes = 0;
  double power_w = 0;
  double temp_c = 0;
};

class AmdSmi {
 public:
  static AmdSmi& instance();
  bool available() const { return ok_; }
  std::vector<AmdGpu> discover();
  // xgmi[i][j] = 1 if a direct xGMI link joins GPU i and j (hops == 1), 0 otherwise
  std::vector<std::vector<int>> xgmi_matrix();
  std::vector<AmdGpuMetrics> metrics();

 private:
  AmdSmi();
  bool ok_ = false;
  void* lib_ = nullptr;
  std::vector<void*> handles_;
};

// catalog name from an amdsmi market name ("AMD Instinct MI355 OAM" -> "MI355X")
std::string amd_catalog_name(const std::string& market_name);
// sysfs-only discovery (no amdsmi): render nodes with vendor 0x1002
std::vector<AmdGpu> discover_amd_gpus_sysfs();
// all AMD GPUs on this host (amdsmi, else sysfs)
std::vector<AmdGpu> discover_amd_gpus();

Json gpu_to_json(const AmdGpu& g);

// choose `count` GPUs out of `free_idx` maximising xGMI connectivity (fully connected first),
// preferring one NUMA node; returns empty if impossible
std::vector<int> pick_gpus_xgmi(const std::vector<int>& free_idx, int count,
                                const std::vector<std::vector<int>>& xgmi, const std::vector<int>& numa);

}  // namespace dsa
