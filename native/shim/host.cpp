// Host facts for host_info.json and offers (reference: runner/internal/shim/host/host.go:14-60,
// host_info.go:13-75), authorized_keys editing (authorized_keys.go:16-163) and volume
// preparation (docker.go prepareVolumes + backends/{aws,gcp}.go device resolution).
#include <arpa/inet.h>
#include <stdlib.h>
#include <dirent.h>
#include <ifaddrs.h>
#include <pwd.h>
#include <sys/statvfs.h>
#include <sys/sysinfo.h>
#include <openssl/sha.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <iterator>
#include <set>
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
  // the cloud bootstrap could not bring up the amdgpu driver (core/backends/base.py
  // get_amd_driver_commands writes the marker): report why, so the server fails the host instead
  // of registering it with zero GPUs
  {
    const char* m = getenv("DSTACK_AMDGPU_MARKER");
    std::ifstream f(m && *m ? m : "/var/lib/dstack/amdgpu-install.failed");
    if (f) {
      std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
      if (text.size() > 2048) text.resize(2048);
      while (!text.empty() && (text.back() == '\n' || text.back() == ' ')) text.pop_back();
      if (!text.empty()) h.set("gpu_driver_error", text);
    }
  }
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

// Tokens of an authorized_keys line: whitespace-separated, double-quoted option values may hold
// spaces (command="echo hi",no-pty ssh-ed25519 AAAA... comment)
static std::vector<std::string> key_tokens(const std::string& line) {
  std::vector<std::string> out;
  std::string cur;
  bool quoted = false;
  for (char c : line) {
    if (c == '"') quoted = !quoted;
    if (!quoted && (c == ' ' || c == '\t')) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

static bool is_key_type(const std::string& t) {
  return t.rfind("ssh-", 0) == 0 || t.rfind("ecdsa-sha2-", 0) == 0 || t.rfind("sk-ssh-", 0) == 0 ||
         t.rfind("sk-ecdsa-sha2-", 0) == 0;
}

// The key blob of a public key or an authorized_keys line ("[options] type base64 [comment]"):
// the bytes its SHA256 fingerprint is taken over, so two lines name the same key exactly when
// their blobs are equal, whatever their options or comments.  False for a line that holds no
// well-formed key (the blob must decode and start with its own type string).
bool public_key_blob(const std::string& line, std::string& blob) {
  auto t = key_tokens(trim(line));
  for (size_t i = 0; i + 1 < t.size(); ++i) {
    if (!is_key_type(t[i])) continue;
    const std::string& b64 = t[i + 1];
    if (b64.find_first_not_of("ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/=") != std::string::npos)
      return false;
    std::string raw = base64_decode(b64);
    if (raw.size() < 4 + t[i].size()) return false;
    uint32_t n = ((uint32_t)(uint8_t)raw[0] << 24) | ((uint32_t)(uint8_t)raw[1] << 16) |
                 ((uint32_t)(uint8_t)raw[2] << 8) | (uint32_t)(uint8_t)raw[3];
    if (n != t[i].size() || raw.compare(4, n, t[i]) != 0) return false;
    blob = raw;
    return true;
  }
  return false;
}

// OpenSSH-style "SHA256:<unpadded base64>" fingerprint, "" for a malformed key
std::string public_key_fingerprint(const std::string& key) {
  std::string blob;
  if (!public_key_blob(key, blob)) return "";
  unsigned char md[32];
  SHA256(reinterpret_cast<const unsigned char*>(blob.data()), blob.size(), md);
  std::string b64 = base64_encode(std::string(reinterpret_cast<char*>(md), sizeof md));
  while (!b64.empty() && b64.back() == '=') b64.pop_back();
  return "SHA256:" + b64;
}

// Add the well-formed keys of `keys` that the file does not hold yet (by key identity: a key
// already present with other options or another comment is not added twice); other lines are kept
// byte for byte, a backup of the previous file is left next to it.  Malformed keys are skipped.
bool add_authorized_keys(const std::string& user, const std::vector<std::string>& keys) {
  std::string dir = home_of(user) + "/.ssh";
  mkdirs(dir, 0700);
  std::string path = dir + "/authorized_keys", content;
  read_file(path, content);
  if (!content.empty()) write_file(path + ".dstack.bak", content, 0600);
  std::set<std::string> have;
  for (auto& line : split(content, '\n')) {
    std::string b;
    if (public_key_blob(line, b)) have.insert(b);
  }
  for (auto& k : keys) {
    std::string b;
    if (!public_key_blob(k, b) || have.count(b)) continue;
    have.insert(b);
    if (!content.empty() && content.back() != '\n') content += "\n";
    content += trim(k) + "\n";
  }
  return write_file(path, content, 0600);
}

// Remove every line that holds one of `keys` (with any options / comment); other lines, comments
// and malformed lines stay.  A missing file is fine.
bool remove_authorized_keys(const std::string& user, const std::vector<std::string>& keys) {
  std::string path = home_of(user) + "/.ssh/authorized_keys", content;
  if (!read_file(path, content)) return true;
  std::set<std::string> drop;
  for (auto& k : keys) {
    std::string b;
    if (public_key_blob(k, b)) drop.insert(b);
  }
  std::string out;
  for (auto& line : split(content, '\n')) {
    if (line.empty()) continue;
    std::string b;
    if (public_key_blob(line, b) && drop.count(b)) continue;
    out += line + "\n";
  }
  return write_file(path, out, 0600);
}

}  // namespace dsa
