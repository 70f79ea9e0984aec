// Host facts for host_info.json and offers (reference: runner/internal/shim/host/host.go:14-60,
// host_info.go:13-75), authorized_keys editing (authorized_keys.go:16-163) and volume
// preparation (docker.go prepareVolumes + backends/{aws,gcp}.go device resolution).
#include <arpa/inet.h>
#include <dirent.h>
#include <ifaddrs.h>
#include <pwd.h>
#include <sys/statvfs.h>
#include <sys/sysinfo.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <sstream>

#include "../common/amdgpu.h"
#include "../common/net.h"
#include "shim.h"

namespace dsa {

Json collect_host_info(const std::string& disk_path) {
  Json h = Json::object();
  h.set("cpus", (long long)sysconf(_SC_NPROCESSORS_ONLN));
  struct sysinfo si{};
  if (sysinfo(&si) == 0) h.set("memory", (long long)((uint64_t)si.totalram * si.mem_unit));
  struct statvfs vfs{};
  if (statvfs(disk_path.c_str(), &vfs) == 0) h.set("disk_size", (long long)((uint64_t)vfs.f_bavail * vfs.f_frsize));
  Json addrs = Json::array();
  struct ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) == 0) {
    for (auto* p = ifa; p; p = p->ifa_next) {
      if (!p->ifa_addr || p->ifa_addr->sa_family != AF_INET) continue;
      char buf[64];
      inet_ntop(AF_INET, &((struct sockaddr_in*)p->ifa_addr)->sin_addr, buf, sizeof buf);
      std::string ip = buf;
      if (ip.rfind("127.", 0) == 0) continue;
      addrs.push_back(ip + "/" + p->ifa_name);
    }
    freeifaddrs(ifa);
  }
  h.set("addresses", addrs);
  auto gpus = discover_amd_gpus();
  Json gj = Json::array();
  Json numa = Json::object();
  for (auto& g : gpus) {
    gj.push_back(gpu_to_json(g));
    numa.set(std::to_string(g.index), g.numa_node);
  }
  h.set("gpu_vendor", gpus.empty() ? "" : "amd");
  h.set("gpu_count", (long long)gpus.size());
  if (!gpus.empty()) {
    h.set("gpu_name", gpus[0].name);
    h.set("gpu_memory", (long long)gpus[0].vram_mib);
  }
  Json topo = Json::object();
  topo.set("gpus", gj);
  Json xg = Json::array();
  if (!gpus.empty()) {
    for (auto& row : xgmi_matrix(gpus)) {
      Json r = Json::array();
      for (int v : row) r.push_back(v);
      xg.push_back(r);
    }
  }
  topo.set("xgmi", xg);
  topo.set("numa", numa);
  Json nics = Json::array();
  if (DIR* d = opendir("/sys/class/infiniband")) {
    while (auto* e = readdir(d))
      if (e->d_name[0] != '.') nics.push_back(std::string(e->d_name));
    closedir(d);
  }
  topo.set("nics", nics);
  h.set("topology", topo);
  return h;
}

static std::string home_of(const std::string& user) {
  struct passwd* pw = getpwnam(user.c_str());
  if (pw) return pw->pw_dir;
  const char* home = getenv("HOME");
  return home ? home : "/root";
}

static std::string key_body(const std::string& k) {
  auto parts = split(trim(k), ' ');
  return parts.size() >= 2 ? parts[0] + " " + parts[1] : trim(k);
}

bool add_authorized_keys(const std::string& user, const std::vector<std::string>& keys) {
  std::string dir = home_of(user) + "/.ssh";
  mkdirs(dir, 0700);
  std::string path = dir + "/authorized_keys", content;
  read_file(path, content);
  if (!content.empty()) write_file(path + ".dstack.bak", content, 0600);
  for (auto& k : keys) {
    if (trim(k).empty()) continue;
    if (content.find(key_body(k)) != std::string::npos) continue;
    if (!content.empty() && content.back() != '\n') content += "\n";
    content += trim(k) + "\n";
  }
  return write_file(path, content, 0600);
}

bool remove_authorized_keys(const std::string& user, const std::vector<std::string>& keys) {
  std::string path = home_of(user) + "/.ssh/authorized_keys", content;
  if (!read_file(path, content)) return true;
  std::string out;
  for (auto& line : split(content, '\n')) {
    if (line.empty()) continue;
    bool drop = false;
    for (auto& k : keys)
      if (key_body(line) == key_body(k)) drop = true;
    if (!drop) out += line + "\n";
  }
  return write_file(path, out, 0600);
}

}  // namespace dsa
