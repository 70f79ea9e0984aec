// Network volumes on the host (reference: DockerRunner volume preparation
// runner/internal/shim/docker.go `prepareVolumes`/`formatAndMountVolume`, device resolvers
// runner/internal/shim/backends/{aws,gcp}.go).
//
// For every volume of a task: resolve the block device the cloud attached, make an ext4 filesystem
// if the volume is new and has none, and mount it at <root>/<name> (default /dstack-volumes).
// Local-backend volumes are plain host directories and are used in place.  Tools are run with
// posix_spawnp (the shim is multi-threaded; no fork+malloc) and never through a shell.
#include <fcntl.h>
#include <spawn.h>
#include <sys/mount.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../common/net.h"
#include "shim.h"

extern char** environ;

namespace dsa {

// run argv[0] (PATH lookup), capture stdout; returns the exit status (-1 if it could not start)
int run_capture(const std::vector<std::string>& argv, std::string& out) {
  out.clear();
  int fds[2];
  if (pipe(fds) != 0) return -1;
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, fds[1], 1);
  posix_spawn_file_actions_addclose(&fa, fds[0]);
  posix_spawn_file_actions_addopen(&fa, 2, "/dev/null", O_WRONLY, 0);
  std::vector<char*> av;
  for (auto& a : argv) av.push_back(const_cast<char*>(a.c_str()));
  av.push_back(nullptr);
  pid_t pid = 0;
  int rc = posix_spawnp(&pid, av[0], &fa, nullptr, av.data(), environ);
  posix_spawn_file_actions_destroy(&fa);
  close(fds[1]);
  if (rc != 0) {
    close(fds[0]);
    return -1;
  }
  char buf[4096];
  ssize_t n;
  while ((n = read(fds[0], buf, sizeof buf)) > 0) out.append(buf, (size_t)n);
  close(fds[0]);
  int st = 0;
  while (waitpid(pid, &st, 0) < 0 && errno == EINTR) {
  }
  return WIFEXITED(st) ? WEXITSTATUS(st) : -1;
}

// AWS NVMe EBS: the controller serial is the volume id without the dash ("vol-0abc" -> "vol0abc").
// `lsblk_json` is the output of `lsblk -J -o NAME,SERIAL,TYPE` (children = partitions).  The first
// partition is used when the disk is partitioned (backends/aws.go).
std::string aws_device_from_lsblk(const std::string& lsblk_json, const std::string& volume_id) {
  std::string serial;
  for (char c : volume_id)
    if (c != '-') serial += c;
  Json j;
  try {
    j = Json::parse(lsblk_json);
  } catch (...) {
    return "";
  }
  for (auto& d : j["blockdevices"].items()) {
    if (trim(d["serial"].str()) != serial) continue;
    const Json& ch = d["children"];
    if (ch.is_array() && ch.size() > 0) return "/dev/" + ch[(size_t)0]["name"].str();
    return "/dev/" + d["name"].str();
  }
  return "";
}

// Xen-era name mapping: the API's /dev/sdX shows up as /dev/xvdX
std::string aws_xvd_name(const std::string& device_name) {
  if (device_name.rfind("/dev/sd", 0) == 0) return "/dev/xvd" + device_name.substr(7);
  return device_name;
}

std::string resolve_volume_device(const Json& v) {
  const std::string backend = v["backend"].str(), id = v["volume_id"].str(), dev = v["device_name"].str();
  if (backend == "aws") {
    std::string out;
    if (run_capture({"lsblk", "-J", "-o", "NAME,SERIAL,TYPE"}, out) == 0) {
      std::string d = aws_device_from_lsblk(out, id);
      if (!d.empty()) return d;
    }
    if (!dev.empty() && path_exists(dev)) return dev;
    std::string x = aws_xvd_name(dev);
    return path_exists(x) ? x : "";
  }
  if (backend == "gcp") {  // persistent disks appear under their device name (backends/gcp.go)
    std::string p = "/dev/disk/by-id/google-" + (dev.empty() ? v["name"].str() : dev);
    return path_exists(p) ? p : "";
  }
  return (!dev.empty() && path_exists(dev)) ? dev : "";
}

static bool mounted_at(const std::string& target) {
  std::string m;
  if (!read_file("/proc/mounts", m)) return false;
  for (auto& line : split(m, '\n')) {
    auto f = split(line, ' ');
    if (f.size() > 1 && f[1] == target) return true;
  }
  return false;
}

bool prepare_volume(const Json& v, const std::string& root, std::string& host_path, std::string& err) {
  const std::string name = v["name"].str();
  if (name.empty() || name.find('/') != std::string::npos || name == "." || name == "..") {
    err = "invalid volume name '" + name + "'";
    return false;
  }
  if (v["backend"].str() == "local") {  // a host directory (LocalCompute.create_volume)
    host_path = v["volume_id"].str().empty() ? root + "/" + name : v["volume_id"].str();
    if (!mkdirs(host_path)) {
      err = "cannot create " + host_path;
      return false;
    }
    return true;
  }
  host_path = root + "/" + name;
  if (mounted_at(host_path)) return true;  // shim restart or a second job on the instance
  std::string dev = resolve_volume_device(v);
  if (dev.empty()) {
    err = "block device of volume " + name + " (" + v["volume_id"].str() + ") not found";
    return false;
  }
  std::string fstype;
  int rc = run_capture({"blkid", "-o", "value", "-s", "TYPE", dev}, fstype);
  fstype = trim(fstype);
  if (rc != 0 && rc != 2) {  // 2 = no filesystem signature
    err = "blkid " + dev + " failed";
    return false;
  }
  if (fstype.empty()) {
    if (!v["init_fs"].as_bool(false)) {
      err = "volume " + name + " has no filesystem and is external (not formatting it)";
      return false;
    }
    std::string out;
    LOGI("volume %s: mkfs.ext4 %s", name.c_str(), dev.c_str());
    if (run_capture({"mkfs.ext4", "-F", dev}, out) != 0) {
      err = "mkfs.ext4 " + dev + " failed";
      return false;
    }
    fstype = "ext4";
  }
  if (!mkdirs(host_path)) {
    err = "cannot create " + host_path;
    return false;
  }
  if (mount(dev.c_str(), host_path.c_str(), fstype.c_str(), 0, nullptr) != 0) {
    err = "mount " + dev + " on " + host_path + ": " + strerror(errno);
    return false;
  }
  LOGI("volume %s: %s (%s) mounted on %s", name.c_str(), dev.c_str(), fstype.c_str(), host_path.c_str());
  return true;
}

// tasks using each mounted volume: a volume shared by two jobs of one instance stays mounted until
// the last of them is removed (the server detaches it only then, too)
static std::mutex g_vol_mu;
static std::map<std::string, int> g_vol_users;

bool prepare_volumes(Task& t, const std::string& root, std::map<std::string, std::string>& paths,
                     std::string& err) {
  std::lock_guard<std::mutex> g(g_vol_mu);
  for (auto& v : t.config.volumes.items()) {
    std::string p;
    if (!prepare_volume(v, root, p, err)) return false;
    paths[v["name"].str()] = p;
    ++g_vol_users[v["name"].str()];
  }
  return true;
}

bool unmount_volumes(const Task& t, const std::string& root) {
  std::lock_guard<std::mutex> g(g_vol_mu);
  bool ok = true;
  for (auto& v : t.config.volumes.items()) {
    auto it = g_vol_users.find(v["name"].str());
    if (it == g_vol_users.end()) continue;  // never prepared by this shim process
    if (--it->second > 0) continue;
    g_vol_users.erase(it);
    if (v["backend"].str() == "local") continue;
    std::string p = root + "/" + v["name"].str();
    if (mounted_at(p) && umount2(p.c_str(), 0) != 0) {
      LOGW("umount %s: %s", p.c_str(), strerror(errno));
      ok = false;
    }
  }
  return ok;
}

}  // namespace dsa
