// Implementation of amdgpu.h.
#include "amdgpu.h"

#include <amd_smi/amdsmi.h>
#include <dirent.h>
#include <dlfcn.h>
#include <limits.h>
#include <stdlib.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstring>
#include <limits>
#include <map>
#include <regex>

#include "net.h"

namespace dsa {

namespace {
typedef amdsmi_status_t (*fn_init)(uint64_t);
typedef amdsmi_status_t (*fn_sockets)(uint32_t*, amdsmi_socket_handle*);
typedef amdsmi_status_t (*fn_procs)(amdsmi_socket_handle, uint32_t*, amdsmi_processor_handle*);
typedef amdsmi_status_t (*fn_asic)(amdsmi_processor_handle, amdsmi_asic_info_t*);
typedef amdsmi_status_t (*fn_vraminfo)(amdsmi_processor_handle, amdsmi_vram_info_t*);
typedef amdsmi_status_t (*fn_bdf)(amdsmi_processor_handle, amdsmi_bdf_t*);
typedef amdsmi_status_t (*fn_enum)(amdsmi_processor_handle, amdsmi_enumeration_info_t*);
typedef amdsmi_status_t (*fn_activity)(amdsmi_processor_handle, amdsmi_engine_usage_t*);
typedef amdsmi_status_t (*fn_vramusage)(amdsmi_processor_handle, amdsmi_vram_usage_t*);
typedef amdsmi_status_t (*fn_power)(amdsmi_processor_handle, amdsmi_power_info_t*);
typedef amdsmi_status_t (*fn_temp)(amdsmi_processor_handle, amdsmi_temperature_type_t, amdsmi_temperature_metric_t,
                                   int64_t*);
typedef amdsmi_status_t (*fn_link)(amdsmi_processor_handle, amdsmi_processor_handle, uint64_t*, amdsmi_link_type_t*);
typedef amdsmi_status_t (*fn_gpu_metrics)(amdsmi_processor_handle, amdsmi_gpu_metrics_t*);
typedef amdsmi_status_t (*fn_xgmi_status)(amdsmi_processor_handle, amdsmi_xgmi_link_status_t*);

struct Fns {
  fn_init init = nullptr;
  fn_sockets sockets = nullptr;
  fn_procs procs = nullptr;
  fn_asic asic = nullptr;
  fn_vraminfo vraminfo = nullptr;
  fn_bdf bdf = nullptr;
  fn_enum enumeration = nullptr;
  fn_activity activity = nullptr;
  fn_vramusage vramusage = nullptr;
  fn_power power = nullptr;
  fn_temp temp = nullptr;
  fn_link link = nullptr;
  fn_gpu_metrics gpu_metrics = nullptr;
  fn_xgmi_status xgmi_status = nullptr;
} F;

std::string bdf_str(const amdsmi_bdf_t& b) {
  char buf[32];
  snprintf(buf, sizeof buf, "%04lx:%02lx:%02lx.%lx", (unsigned long)b.domain_number, (unsigned long)b.bus_number,
           (unsigned long)b.device_number, (unsigned long)b.function_number);
  return buf;
}

int numa_of_bdf(const std::string& bdf) {
  std::string s;
  if (read_file("/sys/bus/pci/devices/" + bdf + "/numa_node", s)) return atoi(s.c_str());
  return -1;
}
}  // namespace

std::string amd_catalog_name(const std::string& market_name) {
  static const std::regex re("^(?:AMD )?(?:Instinct )?(MI\\d{1,3}[A-Za-z]?(?:-\\w+)?)(?:\\s|$)",
                             std::regex::icase);
  std::smatch m;
  std::string name = market_name;
  if (std::regex_search(market_name, m, re)) name = m[1].str();
  for (auto& c : name) c = (char)toupper((unsigned char)c);
  if (name == "MI300X-O") return "MI300X";
  if (name == "MI355") return "MI355X";
  if (name == "MI350") return "MI350X";
  if (name == "MI325") return "MI325X";
  return name;
}

AmdSmi& AmdSmi::instance() {
  static AmdSmi inst;
  return inst;
}

AmdSmi::AmdSmi() {
  const char* names[] = {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"};
  for (auto* n : names) {
    lib_ = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (lib_) break;
  }
  if (!lib_) return;
#define SYM(field, name) F.field = reinterpret_cast<decltype(F.field)>(dlsym(lib_, name))
  SYM(init, "amdsmi_init");
  SYM(sockets, "amdsmi_get_socket_handles");
  SYM(procs, "amdsmi_get_processor_handles");
  SYM(asic, "amdsmi_get_gpu_asic_info");
  SYM(vraminfo, "amdsmi_get_gpu_vram_info");
  SYM(bdf, "amdsmi_get_gpu_device_bdf");
  SYM(enumeration, "amdsmi_get_gpu_enumeration_info");
  SYM(activity, "amdsmi_get_gpu_activity");
  SYM(vramusage, "amdsmi_get_gpu_vram_usage");
  SYM(power, "amdsmi_get_power_info");
  SYM(temp, "amdsmi_get_temp_metric");
  SYM(link, "amdsmi_topo_get_link_type");
  SYM(gpu_metrics, "amdsmi_get_gpu_metrics_info");
  SYM(xgmi_status, "amdsmi_get_gpu_xgmi_link_status");
#undef SYM
  if (!F.init || !F.sockets || !F.procs) return;
  if (F.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return;
  uint32_t ns = 0;
  if (F.sockets(&ns, nullptr) != AMDSMI_STATUS_SUCCESS || ns == 0) return;
  std::vector<amdsmi_socket_handle> socks(ns);
  F.sockets(&ns, socks.data());
  for (uint32_t s = 0; s < ns; ++s) {
    uint32_t np = 0;
    if (F.procs(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
    std::vector<amdsmi_processor_handle> ph(np);
    F.procs(socks[s], &np, ph.data());
    for (auto h : ph) handles_.push_back(h);
  }
  // canonical GPU order = PCI BDF order, whatever order amdsmi reports its handles in: discover(),
  // xgmi_matrix() and metrics() index the same sorted list, and the sysfs fallback sorts the same
  // way, so an index means the same physical GPU on every path
  if (F.bdf) {
    std::vector<std::pair<std::string, amdsmi_processor_handle>> keyed;
    for (auto h : handles_) {
      amdsmi_bdf_t b{};
      keyed.emplace_back(F.bdf(h, &b) == AMDSMI_STATUS_SUCCESS ? bdf_str(b) : std::string("~"), h);
    }
    std::stable_sort(keyed.begin(), keyed.end(), [](auto& a, auto& b) { return a.first < b.first; });
    for (size_t i = 0; i < keyed.size(); ++i) handles_[i] = keyed[i].second;
  }
  ok_ = !handles_.empty();
}

std::vector<AmdGpu> AmdSmi::discover() {
  std::vector<AmdGpu> out;
  for (size_t i = 0; i < handles_.size(); ++i) {
    AmdGpu g;
    g.index = (int)i;
    auto h = handles_[i];
    amdsmi_asic_info_t asic{};
    if (F.asic && F.asic(h, &asic) == AMDSMI_STATUS_SUCCESS) {
      g.market_name = asic.market_name;
      g.name = amd_catalog_name(g.market_name);
      g.serial = asic.asic_serial;
      if (asic.target_graphics_version != UINT64_MAX) {
        char buf[32];
        snprintf(buf, sizeof buf, "gfx%lx", (unsigned long)asic.target_graphics_version);
        g.arch = buf;
      }
    }
    amdsmi_vram_info_t vi{};
    if (F.vraminfo && F.vraminfo(h, &vi) == AMDSMI_STATUS_SUCCESS) g.vram_mib = vi.vram_size;
    amdsmi_bdf_t b{};
    if (F.bdf && F.bdf(h, &b) == AMDSMI_STATUS_SUCCESS) g.bdf = bdf_str(b);
    amdsmi_enumeration_info_t en{};
    if (F.enumeration && F.enumeration(h, &en) == AMDSMI_STATUS_SUCCESS) {
      g.drm_render = (int)en.drm_render;
      g.render_node = "/dev/dri/renderD" + std::to_string(en.drm_render);
    }
    if (g.render_node.empty() && !g.bdf.empty()) {
      char target[PATH_MAX];
      std::string link = "/dev/dri/by-path/pci-" + g.bdf + "-render";
      ssize_t n = readlink(link.c_str(), target, sizeof target - 1);
      if (n > 0) {
        target[n] = 0;
        std::string t = target;
        g.render_node = "/dev/dri/" + t.substr(t.rfind('/') + 1);
      }
    }
    g.numa_node = g.bdf.empty() ? -1 : numa_of_bdf(g.bdf);
    out.push_back(g);
  }
  return out;
}

std::vector<std::vector<int>> AmdSmi::xgmi_matrix() {
  size_t n = handles_.size();
  std::vector<std::vector<int>> m(n, std::vector<int>(n, 0));
  if (!F.link) return m;
  for (size_t i = 0; i < n; ++i)
    for (size_t j = 0; j < n; ++j) {
      if (i == j) continue;
      uint64_t hops = 0;
      amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
      if (F.link(handles_[i], handles_[j], &hops, &t) == AMDSMI_STATUS_SUCCESS && t == AMDSMI_LINK_TYPE_XGMI &&
          hops <= 1)
        m[i][j] = 1;
    }
  return m;
}

namespace {
// amdsmi marks fields a device does not report with all-ones
template <class T>
bool valid(T v) {
  return v != std::numeric_limits<T>::max();
}
}  // namespace

void fill_xgmi_from(const amdsmi_gpu_metrics_t* gm, const amdsmi_xgmi_link_status_t* ls, AmdGpuMetrics& m) {
  int links = 0;
  if (gm) {
    if (valid(gm->xgmi_link_speed)) m.xgmi_link_speed_gbps = gm->xgmi_link_speed;
    if (valid(gm->xgmi_link_width)) m.xgmi_link_width = gm->xgmi_link_width;
    for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
      uint64_t r = gm->xgmi_read_data_acc[l], w = gm->xgmi_write_data_acc[l];
      if (!valid(r) && !valid(w)) continue;
      r = valid(r) ? r : 0;
      w = valid(w) ? w : 0;
      m.xgmi_read_kb_link.push_back(r);
      m.xgmi_write_kb_link.push_back(w);
      m.xgmi_read_kb += r;
      m.xgmi_write_kb += w;
      links = l + 1;
    }
  }
  if (ls && ls->total_links > 0) {
    m.xgmi_links_total = (int)std::min<uint32_t>(ls->total_links, AMDSMI_MAX_NUM_XGMI_LINKS);
    m.xgmi_links_up = 0;
    for (int l = 0; l < m.xgmi_links_total; ++l) m.xgmi_links_up += ls->status[l] == AMDSMI_XGMI_LINK_UP;
  } else if (gm) {
    // older SMU firmware: link state only in gpu_metrics v1.7 (xgmi_link_status)
    int total = 0, up = 0;
    for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
      if (!valid(gm->xgmi_link_status[l])) continue;
      ++total;
      up += gm->xgmi_link_status[l] == AMDSMI_XGMI_LINK_UP;
    }
    m.xgmi_links_total = total ? total : links;
    m.xgmi_links_up = total ? up : 0;
  }
}

void AmdSmi::fill_xgmi(void* h, AmdGpuMetrics& m) {
  amdsmi_gpu_metrics_t gm;
  memset(&gm, 0xff, sizeof gm);
  bool have_gm = F.gpu_metrics && F.gpu_metrics(h, &gm) == AMDSMI_STATUS_SUCCESS;
  amdsmi_xgmi_link_status_t ls{};
  bool have_ls = F.xgmi_status && F.xgmi_status(h, &ls) == AMDSMI_STATUS_SUCCESS;
  fill_xgmi_from(have_gm ? &gm : nullptr, have_ls ? &ls : nullptr, m);
}

std::vector<AmdGpuMetrics> AmdSmi::metrics() {
  std::vector<AmdGpuMetrics> out;
  for (size_t i = 0; i < handles_.size(); ++i) {
    AmdGpuMetrics m;
    m.index = (int)i;
    auto h = handles_[i];
    amdsmi_engine_usage_t u{};
    if (F.activity && F.activity(h, &u) == AMDSMI_STATUS_SUCCESS) {
      m.util_percent = u.gfx_activity;
      if (u.umc_activity != UINT32_MAX) m.mem_activity_percent = u.umc_activity;
    }
    amdsmi_vram_usage_t vu{};
    if (F.vramusage && F.vramusage(h, &vu) == AMDSMI_STATUS_SUCCESS) {
      m.vram_used_bytes = (uint64_t)vu.vram_used << 20;
      m.vram_total_bytes = (uint64_t)vu.vram_total << 20;
    }
    amdsmi_power_info_t p{};
    if (F.power && F.power(h, &p) == AMDSMI_STATUS_SUCCESS) {
      uint32_t w = p.current_socket_power != UINT32_MAX ? p.current_socket_power : p.average_socket_power;
      if (w != UINT32_MAX) m.power_w = w;
    }
    int64_t t = 0;
    if (F.temp && F.temp(h, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS)
      m.temp_c = (double)t;
    fill_xgmi(h, m);
    out.push_back(m);
  }
  return out;
}

Json gpu_metrics_to_json(const AmdGpuMetrics& g) {
  Json j = Json::object();
  j.set("gpu_memory_usage_bytes", (long long)g.vram_used_bytes);
  j.set("gpu_memory_total_bytes", (long long)g.vram_total_bytes);
  j.set("gpu_util_percent", g.util_percent);
  j.set("gpu_power_watts", g.power_w);
  j.set("gpu_temperature_c", g.temp_c);
  if (g.mem_activity_percent >= 0) j.set("gpu_mem_activity_percent", g.mem_activity_percent);
  if (g.xgmi_links_total > 0 || g.xgmi_read_kb || g.xgmi_write_kb) {
    Json x = Json::object();
    x.set("links_total", g.xgmi_links_total);
    x.set("links_up", g.xgmi_links_up);
    x.set("link_speed_gbps", g.xgmi_link_speed_gbps);
    x.set("link_width", g.xgmi_link_width);
    x.set("read_kb", (long long)g.xgmi_read_kb);
    x.set("write_kb", (long long)g.xgmi_write_kb);
    j.set("xgmi", x);
  }
  return j;
}

std::vector<AmdGpu> discover_amd_gpus_sysfs() {
  std::vector<AmdGpu> out;
  // DSTACK_SYSFS_ROOT: a fake /sys tree (tests)
  const char* root_env = getenv("DSTACK_SYSFS_ROOT");
  const std::string root = root_env ? root_env : "";
  DIR* d = opendir((root + "/sys/class/drm").c_str());
  if (!d) return out;
  std::vector<int> renders;
  while (auto* e = readdir(d)) {
    std::string n = e->d_name;
    if (n.rfind("renderD", 0) == 0) renders.push_back(atoi(n.c_str() + 7));
  }
  closedir(d);
  std::sort(renders.begin(), renders.end());
  for (int r : renders) {
    std::string base = root + "/sys/class/drm/renderD" + std::to_string(r) + "/device/";
    std::string vendor;
    if (!read_file(base + "vendor", vendor) || trim(vendor) != "0x1002") continue;
    // only GPUs this process can open: sysfs is host-wide, but a container (or a cgroup device
    // filter) exposes only some render nodes -- amdsmi lists exactly those, and so must we
    if (access((root + "/dev/dri/renderD" + std::to_string(r)).c_str(), R_OK | W_OK) != 0) continue;
    AmdGpu g;
    g.index = (int)out.size();
    g.drm_render = r;
    g.render_node = "/dev/dri/renderD" + std::to_string(r);
    char target[PATH_MAX];
    ssize_t n = readlink((root + "/sys/class/drm/renderD" + std::to_string(r) + "/device").c_str(), target,
                         sizeof target - 1);
    if (n > 0) {
      target[n] = 0;
      std::string t = target;
      g.bdf = t.substr(t.rfind('/') + 1);
    }
    std::string vram;
    if (read_file(base + "mem_info_vram_total", vram)) g.vram_mib = std::stoull(trim(vram)) >> 20;
    std::string pn;
    if (read_file(base + "product_name", pn)) g.market_name = trim(pn);
    g.name = g.market_name.empty() ? "AMD GPU" : amd_catalog_name(g.market_name);
    std::string numa;
    g.numa_node = read_file(base + "numa_node", numa) ? atoi(numa.c_str()) : -1;
    out.push_back(g);
  }
  // BDF order (the amdsmi path sorts identically); render-node numbers need not follow the bus
  std::stable_sort(out.begin(), out.end(), [](const AmdGpu& a, const AmdGpu& b) { return a.bdf < b.bdf; });
  for (size_t i = 0; i < out.size(); ++i) out[i].index = (int)i;
  return out;
}

// KFD topology: /sys/class/kfd/kfd/topology/nodes/<n>/{gpu_id, properties, io_links/<k>/properties}.
// A GPU node's properties carry "domain" and "location_id" (bus << 8 | device << 3 | function);
// an io_link of "type 11" (CRAT XGMI) with "node_to" m joins node n to node m directly.
std::vector<std::vector<int>> xgmi_matrix_sysfs(const std::vector<AmdGpu>& gpus) {
  const char* root_env = getenv("DSTACK_SYSFS_ROOT");
  const std::string root = root_env ? root_env : "";
  const std::string nodes_dir = root + "/sys/class/kfd/kfd/topology/nodes";
  std::vector<std::vector<int>> m(gpus.size(), std::vector<int>(gpus.size(), 0));
  auto props = [](const std::string& path) {
    std::map<std::string, long long> p;
    std::string s;
    if (!read_file(path, s)) return p;
    for (auto& line : split(s, '\n')) {
      auto sp = line.find(' ');
      if (sp == std::string::npos) continue;
      p[line.substr(0, sp)] = atoll(line.c_str() + sp + 1);
    }
    return p;
  };
  std::map<long long, int> node_to_gpu;  // KFD node id -> index in `gpus`
  std::vector<long long> gpu_nodes;
  DIR* d = opendir(nodes_dir.c_str());
  if (!d) return m;
  while (auto* e = readdir(d))
    if (e->d_name[0] >= '0' && e->d_name[0] <= '9') gpu_nodes.push_back(atoll(e->d_name));
  closedir(d);
  for (long long n : gpu_nodes) {
    std::string base = nodes_dir + "/" + std::to_string(n);
    std::string gid;
    if (!read_file(base + "/gpu_id", gid) || atoll(gid.c_str()) == 0) continue;  // CPU node
    auto p = props(base + "/properties");
    long long loc = p.count("location_id") ? p["location_id"] : -1, dom = p.count("domain") ? p["domain"] : 0;
    if (loc < 0) continue;
    char bdf[32];
    snprintf(bdf, sizeof bdf, "%04llx:%02llx:%02llx.%llx", dom, (loc >> 8) & 0xff, (loc >> 3) & 0x1f, loc & 7);
    for (size_t i = 0; i < gpus.size(); ++i)
      if (gpus[i].bdf == bdf) node_to_gpu[n] = (int)i;
  }
  for (auto& kv : node_to_gpu) {
    std::string links = nodes_dir + "/" + std::to_string(kv.first) + "/io_links";
    DIR* ld = opendir(links.c_str());
    if (!ld) continue;
    while (auto* e = readdir(ld)) {
      if (e->d_name[0] == '.') continue;
      auto p = props(links + "/" + e->d_name + "/properties");
      if (!p.count("type") || p["type"] != 11 || !p.count("node_to")) continue;
      auto it = node_to_gpu.find(p["node_to"]);
      if (it != node_to_gpu.end() && it->second != kv.second) m[kv.second][it->second] = 1;
    }
    closedir(ld);
  }
  return m;
}

static bool sysfs_override() {
  const char* r = getenv("DSTACK_SYSFS_ROOT");
  return r && *r;
}

std::vector<std::vector<int>> xgmi_matrix(const std::vector<AmdGpu>& gpus) {
  auto& smi = AmdSmi::instance();
  if (!sysfs_override() && smi.available() && smi.count() == gpus.size()) return smi.xgmi_matrix();
  return xgmi_matrix_sysfs(gpus);
}

std::vector<AmdGpu> discover_amd_gpus() {
  if (sysfs_override()) return discover_amd_gpus_sysfs();  // a fake /sys tree wins over the real devices
  auto& smi = AmdSmi::instance();
  if (smi.available()) {
    auto g = smi.discover();
    if (!g.empty()) return g;
  }
  return discover_amd_gpus_sysfs();
}

Json gpu_to_json(const AmdGpu& g) {
  Json j = Json::object();
  j.set("index", g.index);
  j.set("name", g.name);
  j.set("market_name", g.market_name);
  j.set("vendor", "amd");
  j.set("arch", g.arch);
  j.set("memory_mib", (long long)g.vram_mib);
  j.set("bdf", g.bdf);
  j.set("render_node", g.render_node);
  j.set("numa_node", g.numa_node);
  j.set("serial", g.serial);
  return j;
}

std::vector<int> pick_gpus_xgmi(const std::vector<int>& free_idx, int count, const std::vector<std::vector<int>>& xgmi,
                                const std::vector<int>& numa) {
  std::vector<int> empty;
  if (count <= 0 || (int)free_idx.size() < count) return empty;
  if ((int)free_idx.size() == count) return free_idx;
  auto linked = [&](int a, int b) {
    return a < (int)xgmi.size() && b < (int)xgmi[a].size() && xgmi[a][b] > 0;
  };
  auto numa_of = [&](int a) { return a < (int)numa.size() ? numa[a] : -1; };
  // greedy: try each seed, grow by the candidate with most links into the chosen set
  // (ties: same NUMA node, then lower index); score = internal links + NUMA affinity
  std::vector<int> best;
  long best_score = -1;
  for (int seed : free_idx) {
    std::vector<int> sel{seed};
    while ((int)sel.size() < count) {
      int pick = -1;
      long pscore = -1;
      for (int c : free_idx) {
        if (std::find(sel.begin(), sel.end(), c) != sel.end()) continue;
        long s = 0;
        for (int x : sel) s += linked(c, x) ? 4 : 0;
        if (numa_of(c) == numa_of(seed)) s += 1;
        if (s > pscore) {
          pscore = s;
          pick = c;
        }
      }
      sel.push_back(pick);
    }
    long score = 0;
    for (int a : sel)
      for (int b : sel)
        if (a != b) score += linked(a, b) ? 4 : 0;
    for (int a : sel) score += numa_of(a) == numa_of(seed) ? 1 : 0;
    if (score > best_score) {
      best_score = score;
      best = sel;
    }
  }
  std::sort(best.begin(), best.end());
  return best;
}

}  // namespace dsa
