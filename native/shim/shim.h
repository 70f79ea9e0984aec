// dstack-shim: host agent (reference: runner/cmd/shim, runner/internal/shim/*).
//
// Runs tasks (one container or process per job) with whole GPUs granted by an xGMI-topology-aware
// GPU lock, reports host_info (amdsmi topology) and serves a small REST API on :10998.
#pragma once
#include <atomic>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../common/json.h"

namespace dsa {

// ---- task model (task.go:12-234) -----------------------------------------------------------
enum class TaskStatus { Pending, Preparing, Pulling, Creating, Running, Terminated };
const char* task_status_name(TaskStatus s);
bool task_transition_allowed(TaskStatus from, TaskStatus to);
std::string unique_container_name(const std::string& base);

struct PortMapping {
  int container = 0;
  int host = 0;
};

struct TaskConfig {
  std::string id, name;
  std::string registry_username, registry_password;
  std::string image_name;
  std::string container_user;
  bool privileged = false;
  int gpu = 0;  // -1 = all, 0 = none, n = count
  std::vector<int> gpu_indices;  // explicit grant (overrides gpu count)
  double cpu = 0;
  int64_t memory = 0;    // bytes, 0 = unlimited
  int64_t shm_size = 0;  // bytes
  std::string network_mode = "host";
  Json volumes = Json::array();
  Json volume_mounts = Json::array();
  Json instance_mounts = Json::array();
  std::string host_ssh_user;
  std::vector<std::string> host_ssh_keys;
  std::vector<std::string> container_ssh_keys;
  std::map<std::string, std::string> env;
  std::vector<int> ports;  // extra container ports to publish (bridge mode)
  static TaskConfig from_json(const Json& j);
};

struct Task {
  TaskConfig config;
  TaskStatus status = TaskStatus::Pending;
  std::string termination_reason, termination_message;
  std::string container_name, container_id;
  std::vector<PortMapping> ports;
  std::vector<int> gpus;  // granted GPU indices (host numbering: BDF order, see amdgpu.h)
  // render nodes of the granted GPUs, resolved from the shim's one discovery snapshot at grant time
  // (the same snapshot the GPU lock and its xGMI matrix were built from) and kept in the container
  // labels, so devices never come from a second, possibly differently ordered, discovery
  std::vector<std::string> render_nodes;
  int runner_port = 0;
  int pid = 0;  // process driver
  int64_t created_ms = 0;
  std::map<std::string, int64_t> timings;  // stage -> ms timestamp (cold-start instrumentation)
  Json to_json() const;
};

// copy-on-get storage (task.go TaskStorage)
class TaskStorage {
 public:
  bool add(const Task& t);
  bool get(const std::string& id, Task& out) const;
  bool update(const Task& t);
  bool set_status(const std::string& id, TaskStatus st, const std::string& reason = "", const std::string& msg = "");
  bool remove(const std::string& id);
  std::vector<std::string> ids() const;

 private:
  mutable std::mutex mu_;
  std::map<std::string, Task> tasks_;
};

// ---- GPU lock (resources.go:31-131), xGMI-topology aware ------------------------------------
class GpuLock {
 public:
  void init(int n_gpus, std::vector<std::vector<int>> xgmi, std::vector<int> numa);
  // count: -1 = all free GPUs; returns granted indices (empty if not enough)
  std::vector<int> acquire(int count);
  bool lock(const std::vector<int>& idx);  // restore state (all-or-nothing)
  void release(const std::vector<int>& idx);
  int free_count() const;
  int total() const { return n_; }

 private:
  mutable std::mutex mu_;
  int n_ = 0;
  std::vector<bool> busy_;
  std::vector<std::vector<int>> xgmi_;
  std::vector<int> numa_;
};

// ---- host info (host.go, host_info.go) ------------------------------------------------------
Json collect_host_info(const std::string& disk_path);
bool public_key_blob(const std::string& line, std::string& blob);
std::string public_key_fingerprint(const std::string& key);
bool add_authorized_keys(const std::string& user, const std::vector<std::string>& keys);
bool remove_authorized_keys(const std::string& user, const std::vector<std::string>& keys);

// ---- drivers ---------------------------------------------------------------------------------
struct ShimOptions {
  std::string home = "/root/.dstack-shim";
  std::string runner_binary;
  std::string runner_download_url;
  std::string probe_binary;
  int runner_http_port = 10999;
  int runner_ssh_port = 10022;
  int runner_log_level = -1;  // -1: the shim's own level
  bool privileged = false;
  std::string docker_socket = "/var/run/docker.sock";
  std::string driver = "auto";  // docker | process | auto
  int pull_timeout_s = 20 * 60;
  std::string volumes_root = "/dstack-volumes";
  std::string infiniband_path = "/dev/infiniband";  // RDMA devices passed through when present
};

class TaskDriver {
 public:
  virtual ~TaskDriver() = default;
  virtual const char* name() const = 0;
  // prepare (volumes, keys), pull, create, start; updates the task via storage
  virtual bool run(Task& t, std::string& reason, std::string& msg) = 0;
  // block until the task's workload exits (called on a dedicated thread)
  virtual void wait(Task& t) = 0;
  virtual void terminate(Task& t, int timeout_s) = 0;
  virtual void remove(Task& t) = 0;
  // re-adopt tasks that survived a shim restart; returns restored tasks
  virtual std::vector<Task> restore() { return {}; }
};

std::unique_ptr<TaskDriver> make_docker_driver(const ShimOptions& o);
std::unique_ptr<TaskDriver> make_process_driver(const ShimOptions& o);
// process-driver children (killed on shim shutdown; see process.cpp)
void register_child_pgid(int pgid);
void unregister_child_pgid(int pgid);
void kill_registered_children(int sig);
bool docker_available(const std::string& socket_path);

// ---- network volumes (volumes.cpp) --------------------------------------------------------------
int run_capture(const std::vector<std::string>& argv, std::string& out);
std::string aws_device_from_lsblk(const std::string& lsblk_json, const std::string& volume_id);
std::string aws_xvd_name(const std::string& device_name);
std::string resolve_volume_device(const Json& v);
// mount (formatting new volumes) and return the host path to bind for the volume
bool prepare_volume(const Json& v, const std::string& root, std::string& host_path, std::string& err);
bool prepare_volumes(Task& t, const std::string& root, std::map<std::string, std::string>& paths,
                     std::string& err);
bool unmount_volumes(const Task& t, const std::string& root);

// shell bootstrap that starts sshd + the runner inside a container (docker.go:873-911)
std::string container_bootstrap_script(const ShimOptions& o, const std::vector<std::string>& keys);

// ---- the shim service --------------------------------------------------------------------------
class Shim {
 public:
  Shim(ShimOptions o, std::unique_ptr<TaskDriver> driver);
  Json submit(const Json& cfg, int& http_status);
  bool get(const std::string& id, Json& out) const;
  Json list() const;
  bool terminate(const std::string& id, const std::string& reason, const std::string& msg, int timeout_s);
  bool remove(const std::string& id, std::string& err);
  Json host_info();
  const char* driver_name() const { return driver_->name(); }
  GpuLock& gpu_lock() { return gpus_; }
  void restore();
  // render nodes of host GPU indices, from the discovery snapshot taken at construction
  std::vector<std::string> render_nodes_of(const std::vector<int>& idx) const;
  // GPU health probe (dstack-probe --quick --json), run asynchronously off the job path: at shim
  // start and on demand.  start_gpu_probe: "started" | "running" | "busy" (GPU tasks hold GPUs)
  // | "unavailable" (no probe binary or no GPUs); a GPU task arriving while it runs pre-empts it
  // (the probe is killed, state "interrupted") and it runs again once the GPUs are all free
  std::string start_gpu_probe();
  Json gpu_health();

 private:
  void run_task(std::string id);
  void probe_main();
  // GPUs released by a task: re-run a probe that a task interrupted once the host is idle again
  void release_gpus(const std::vector<int>& idx);
  ShimOptions opts_;
  std::unique_ptr<TaskDriver> driver_;
  TaskStorage storage_;
  GpuLock gpus_;
  std::vector<std::string> inventory_render_;  // index -> /dev/dri/renderD*
  std::mutex probe_mu_;
  std::condition_variable probe_cv_;
  bool probing_ = false;             // the probe holds every GPU in gpus_ while this is set
  pid_t probe_pid_ = -1;             // its process group, so a GPU task can pre-empt it
  bool probe_interrupted_ = false;   // the last probe was killed for a task: re-probe when idle
  std::string probe_state_ = "idle";  // idle | running | done | failed | interrupted | unavailable
  Json probe_doc_;
  int64_t probe_started_ms_ = 0, probe_ran_ms_ = 0;
  Json host_info_;
  std::mutex hi_mu_;
};

}  // namespace dsa
