// Runner hardware metrics: cgroup v2/v1 CPU and memory + amdsmi GPU util/VRAM/power/temp, HBM
// controller activity and xGMI link state / accumulated traffic.
// Reference: runner/internal/metrics/metrics.go:21-256 (nvidia-smi / amd-smi CSV / hl-smi).
#include <stdlib.h>

#include <algorithm>
#include <sstream>

#include "../common/amdgpu.h"
#include "../common/net.h"

namespace dsa {

static bool read_u64(const std::string& path, uint64_t& v) {
  std::string s;
  if (!read_file(path, s)) return false;
  s = trim(s);
  if (s.empty() || s == "max") return false;
  v = strtoull(s.c_str(), nullptr, 10);
  return true;
}

static uint64_t stat_field(const std::string& path, const std::string& key) {
  std::string s;
  if (!read_file(path, s)) return 0;
  std::istringstream ss(s);
  std::string k;
  uint64_t v;
  while (ss >> k >> v)
    if (k == key) return v;
  return 0;
}

Json collect_metrics(const std::vector<int>& gpu_filter) {
  Json m = Json::object();
  m.set("timestamp_micro", (long long)now_micros());
  uint64_t cpu_usec = 0, mem = 0, inactive = 0;
  if (path_exists("/sys/fs/cgroup/cgroup.controllers")) {  // cgroup v2
    cpu_usec = stat_field("/sys/fs/cgroup/cpu.stat", "usage_usec");
    read_u64("/sys/fs/cgroup/memory.current", mem);
    inactive = stat_field("/sys/fs/cgroup/memory.stat", "inactive_file");
  } else {  // cgroup v1
    uint64_t ns = 0;
    if (read_u64("/sys/fs/cgroup/cpuacct/cpuacct.usage", ns)) cpu_usec = ns / 1000;
    read_u64("/sys/fs/cgroup/memory/memory.usage_in_bytes", mem);
    inactive = stat_field("/sys/fs/cgroup/memory/memory.stat", "total_inactive_file");
  }
  m.set("cpu_usage_micro", (long long)cpu_usec);
  m.set("memory_usage_bytes", (long long)mem);
  m.set("memory_working_set_bytes", (long long)(mem > inactive ? mem - inactive : 0));
  Json gpus = Json::array();
  auto& smi = AmdSmi::instance();
  if (smi.available()) {
    for (auto& g : smi.metrics()) {
      if (!gpu_filter.empty() &&
          std::find(gpu_filter.begin(), gpu_filter.end(), g.index) == gpu_filter.end())
        continue;
      Json j = gpu_metrics_to_json(g);
      gpus.push_back(j);
    }
  }
  m.set("gpus", gpus);
  return m;
}

}  // namespace dsa
