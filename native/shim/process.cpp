// Process task driver: runs the dstack-runner as a child process of the shim, without Docker.
// Used by the local backend, by bare-metal SSH hosts without a container runtime and by the
// CPU-only tests.  GPU isolation: the granted GPUs are exported as HIP_VISIBLE_DEVICES (host
// numbering), so ROCm in the job sees exactly those devices.
#include <fcntl.h>
#include <signal.h>

#include <atomic>
#include <sys/wait.h>
#include <unistd.h>

#include <cstring>
#include <thread>

#include "../common/net.h"
#include "shim.h"

extern char** environ;

namespace dsa {

// Process-group ids of runner children, readable from a signal handler: when the shim is stopped,
// process-driver tasks (plain child processes, unlike containers) must not outlive it.
static std::atomic<int> g_child_pgids[512];

void register_child_pgid(int pgid) {
  for (auto& slot : g_child_pgids) {
    int expected = 0;
    if (slot.compare_exchange_strong(expected, pgid)) return;
  }
}

void unregister_child_pgid(int pgid) {
  for (auto& slot : g_child_pgids) {
    int expected = pgid;
    if (slot.compare_exchange_strong(expected, 0)) return;
  }
}

void kill_registered_children(int sig) {  // async-signal-safe
  for (auto& slot : g_child_pgids) {
    int pg = slot.load();
    if (pg > 0) kill(-pg, sig);
  }
}

class ProcessDriver : public TaskDriver {
 public:
  explicit ProcessDriver(ShimOptions o) : o_(std::move(o)) {}
  const char* name() const override { return "process"; }

  bool run(Task& t, std::string& reason, std::string& msg) override {
    if (o_.runner_binary.empty() || !path_exists(o_.runner_binary)) {
      reason = "creating_container_error";
      msg = "dstack-runner binary not found: " + o_.runner_binary;
      return false;
    }
    std::string dir = o_.home + "/tasks/" + t.config.id;
    mkdirs(dir + "/tmp");
    mkdirs(dir + "/home");
    mkdirs(dir + "/workflow");
    // network volumes: mounted on the host, then linked into the task dir like instance mounts
    std::map<std::string, std::string> vol_paths;
    if (!prepare_volumes(t, o_.volumes_root, vol_paths, msg)) {
      reason = "volume_error";
      return false;
    }
    for (auto& m : t.config.volume_mounts.items()) {
      auto it = vol_paths.find(m["name"].str());
      std::string p = m["path"].str();
      if (it == vol_paths.end() || p.empty()) continue;
      std::string link = dir + "/mounts" + p;
      mkdirs(link.substr(0, link.rfind('/')));
      if (symlink(it->second.c_str(), link.c_str()) != 0) LOGW("volume link %s failed", link.c_str());
    }
    // instance mounts: expose host paths inside the task dir (symlinks) for parity with docker
    for (auto& m : t.config.instance_mounts.items()) {
      std::string ip = m["instance_path"].str(), p = m["path"].str();
      if (m["optional"].as_bool() && access(ip.c_str(), F_OK) != 0) continue;
      if (!ip.empty() && !p.empty()) {
        std::string link = dir + "/mounts" + p;
        mkdirs(link.substr(0, link.rfind('/')));
        if (symlink(ip.c_str(), link.c_str()) != 0) LOGW("mount link %s failed", link.c_str());
      }
    }
    // the runner binds an ephemeral port itself and reports it through a file: probing for a free
    // port here and passing it down would race with every other bind on the host
    std::string port_file = dir + "/runner.port";
    unlink(port_file.c_str());
    std::vector<std::string> envs;
    for (char** e = environ; e && *e; ++e) {
      std::string s = *e;
      if (s.rfind("HIP_VISIBLE_DEVICES=", 0) == 0 || s.rfind("ROCR_VISIBLE_DEVICES=", 0) == 0 ||
          s.rfind("CUDA_VISIBLE_DEVICES=", 0) == 0)
        continue;
      envs.push_back(s);
    }
    for (auto& kv : t.config.env) envs.push_back(kv.first + "=" + kv.second);
    if (!t.gpus.empty()) {
      std::string v;
      for (size_t k = 0; k < t.gpus.size(); ++k) v += (k ? "," : "") + std::to_string(t.gpus[k]);
      envs.push_back("HIP_VISIBLE_DEVICES=" + v);
      envs.push_back("DSTACK_GPU_INDICES=" + v);
    } else if (t.config.gpu == 0) {
      envs.push_back("HIP_VISIBLE_DEVICES=-1");  // no GPU granted: hide all devices
    }
    std::vector<std::string> argv = {o_.runner_binary, "--log-level",
                                     std::to_string(o_.runner_log_level >= 0 ? o_.runner_log_level : log_level()), "start",
                                     "--http-port", "0", "--port-file", port_file, "--temp-dir", dir + "/tmp",
                                     "--home-dir", dir + "/home", "--working-dir", dir + "/workflow"};
    if (!o_.probe_binary.empty()) {
      argv.push_back("--probe");
      argv.push_back(o_.probe_binary);
    }
    std::string log_path = dir + "/runner.log";
    // everything the child needs is materialised before fork(): the shim is multi-threaded, so
    // the child may only make async-signal-safe calls (no malloc) until execve
    std::vector<char*> a, e;
    for (auto& s : argv) a.push_back(const_cast<char*>(s.c_str()));
    a.push_back(nullptr);
    for (auto& s : envs) e.push_back(const_cast<char*>(s.c_str()));
    e.push_back(nullptr);
    pid_t pid = fork();
    if (pid < 0) {
      reason = "creating_container_error";
      msg = strerror(errno);
      return false;
    }
    if (pid == 0) {
      setsid();
      int fd = open(log_path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
      if (fd >= 0) {
        dup2(fd, 1);
        dup2(fd, 2);
        close(fd);
      }
      execve(a[0], a.data(), e.data());
      _exit(127);
    }
    register_child_pgid(pid);
    t.pid = pid;
    t.container_name = "process-" + std::to_string(pid);
    auto exited = [&]() {
      int st;
      if (waitpid(pid, &st, WNOHANG) != pid) return false;
      unregister_child_pgid(pid);
      reason = "creating_container_error";
      msg = "runner exited during startup (see " + log_path + ")";
      t.pid = 0;
      return true;
    };
    int port = 0;
    for (int k = 0; k < 1000 && port == 0; ++k) {  // <= 10 s for the runner to bind
      std::string s;
      if (read_file(port_file, s)) port = atoi(s.c_str());
      if (port == 0) {
        if (exited()) return false;
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
      }
    }
    if (port == 0) {
      terminate(t, 1);
      wait(t);
      reason = "creating_container_error";
      msg = "runner did not report its port (see " + log_path + ")";
      t.pid = 0;
      return false;
    }
    t.runner_port = port;
    t.ports = {PortMapping{o_.runner_http_port, port}};
    // wait until the runner accepts connections so the server's first call succeeds
    for (int k = 0; k < 500; ++k) {
      HttpClientRequest r;
      r.port = port;
      r.path = "/api/healthcheck";
      r.timeout_ms = 200;
      if (http_request(r).ok()) break;
      if (exited()) return false;
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    return true;
  }

  void wait(Task& t) override {
    if (t.pid <= 0) return;
    int st = 0;
    waitpid(t.pid, &st, 0);
    unregister_child_pgid(t.pid);
  }

  void terminate(Task& t, int timeout_s) override {
    if (t.pid <= 0) return;
    kill(-t.pid, SIGTERM);
    for (int k = 0; k < timeout_s * 10; ++k) {
      if (kill(t.pid, 0) != 0) return;
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    kill(-t.pid, SIGKILL);
  }

  void remove(Task& t) override {
    std::string dir = o_.home + "/tasks/" + t.config.id;
    std::string out;
    if (run_capture({"rm", "-rf", "--", dir}, out) != 0) LOGW("cannot remove %s", dir.c_str());
    unmount_volumes(t, o_.volumes_root);
  }

 private:
  ShimOptions o_;
};

std::unique_ptr<TaskDriver> make_process_driver(const ShimOptions& o) {
  return std::unique_ptr<TaskDriver>(new ProcessDriver(o));
}

}  // namespace dsa
