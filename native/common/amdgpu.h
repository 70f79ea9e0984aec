// AMD GPU discovery, xGMI topology and live metrics for the native agents.
//
// Primary source: the amdsmi C library (libamd_smi.so, dlopen'ed so the agents still start on
// CPU-only hosts).  Fallback: sysfs (/sys/class/drm/renderD*/device, KFD topology) for discovery.
// Replaces the reference's `docker run amd-smi static --json` + CSV parsing
// (runner/internal/shim/host/gpu.go:149-196, runner/internal/metrics/metrics.go:172-203).
#pragma once
#include <amd_smi/amdsmi.h>

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
  double mem_activity_percent = -1;  // UMC (HBM controller) activity, -1 when not reported
  uint64_t vram_used_bytes = 0;
  uint64_t vram_total_bytes = 0;
  double power_w = 0;
  double temp_c = 0;
  // xGMI (amdsmi gpu_metrics): per-link accumulated traffic (KiB since driver load) and link
  // state; the server turns two samples into per-GPU xGMI read / write throughput
  int xgmi_links_total = 0;  // links reported by the device (0: no xGMI data)
  int xgmi_links_up = 0;
  int xgmi_link_speed_gbps = 0;  // per-link bitrate (GB/s) as reported by the SMU
  int xgmi_link_width = 0;
  uint64_t xgmi_read_kb = 0;  // sum over links
  uint64_t xgmi_write_kb = 0;
  std::vector<uint64_t> xgmi_read_kb_link, xgmi_write_kb_link;
};

class AmdSmi {
 public:
  static AmdSmi& instance();
  bool available() const { return ok_; }
  size_t count() const { return handles_.size(); }
  std::vector<AmdGpu> discover();
  // xgmi[i][j] = 1 if a direct xGMI link joins GPU i and j (hops == 1), 0 otherwise
  std::vector<std::vector<int>> xgmi_matrix();
  std::vector<AmdGpuMetrics> metrics();

 private:
  AmdSmi();
  void fill_xgmi(void* handle, AmdGpuMetrics& m);
  bool ok_ = false;
  void* lib_ = nullptr;
  std::vector<void*> handles_;
};

// catalog name from an amdsmi market name ("AMD Instinct MI355 OAM" -> "MI355X")
std::string amd_catalog_name(const std::string& market_name);
// sysfs-only discovery (no amdsmi): render nodes with vendor 0x1002
std::vector<AmdGpu> discover_amd_gpus_sysfs();
// all AMD GPUs on this host (amdsmi, else sysfs; DSTACK_SYSFS_ROOT forces the sysfs path)
std::vector<AmdGpu> discover_amd_gpus();
// direct-xGMI adjacency of `gpus` (their order) from the KFD topology's io_links (type 11)
std::vector<std::vector<int>> xgmi_matrix_sysfs(const std::vector<AmdGpu>& gpus);
// amdsmi's matrix when it enumerates the same GPUs, else the KFD-topology one
std::vector<std::vector<int>> xgmi_matrix(const std::vector<AmdGpu>& gpus);

Json gpu_to_json(const AmdGpu& g);
// one GPU's sample in the runner's metrics wire format (gpu_* keys, optional "xgmi" object)
Json gpu_metrics_to_json(const AmdGpuMetrics& m);

// xGMI fields of AmdGpuMetrics from amdsmi gpu_metrics / link status (either may be null;
// all-ones fields are "not reported")
void fill_xgmi_from(const amdsmi_gpu_metrics_t* gm, const amdsmi_xgmi_link_status_t* ls, AmdGpuMetrics& m);

// choose `count` GPUs out of `free_idx` maximising xGMI connectivity (fully connected first),
// preferring one NUMA node; returns empty if impossible
std::vector<int> pick_gpus_xgmi(const std::vector<int>& free_idx, int count,
                                const std::vector<std::vector<int>>& xgmi, const std::vector<int>& numa);

}  // namespace dsa
