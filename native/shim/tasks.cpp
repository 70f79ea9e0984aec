// Task model, storage and the xGMI-aware GPU lock (see shim.h).
#include <algorithm>
#include <random>

#include "../common/amdgpu.h"
#include "../common/net.h"
#include "shim.h"

namespace dsa {

const char* task_status_name(TaskStatus s) {
  switch (s) {
    case TaskStatus::Pending: return "pending";
    case TaskStatus::Preparing: return "preparing";
    case TaskStatus::Pulling: return "pulling";
    case TaskStatus::Creating: return "creating";
    case TaskStatus::Running: return "running";
    case TaskStatus::Terminated: return "terminated";
  }
  return "unknown";
}

// Docker container name for a task: the task's name made safe for Docker ([A-Za-z0-9][A-Za-z0-9_.-]*)
// plus a random suffix, so that a container left behind by an earlier shim (same run name) never
// makes the create fail with a name conflict (task.go generateUniqueName).  Tasks are found again
// by their labels, not by name.
std::string unique_container_name(const std::string& base) {
  std::string n;
  for (char c : base) n += (isalnum((unsigned char)c) || c == '_' || c == '.' || c == '-') ? c : '-';
  if (n.empty() || !isalnum((unsigned char)n[0])) n = "task" + n;
  static thread_local std::mt19937_64 rng{std::random_device{}()};
  char suf[9];
  snprintf(suf, sizeof suf, "%08x", (unsigned)(rng() & 0xffffffffu));
  return n.substr(0, 200) + "-" + suf;
}

bool task_transition_allowed(TaskStatus from, TaskStatus to) {
  if (to == TaskStatus::Terminated) return from != TaskStatus::Terminated;
  switch (from) {
    case TaskStatus::Pending: return to == TaskStatus::Preparing;
    case TaskStatus::Preparing: return to == TaskStatus::Pulling;
    case TaskStatus::Pulling: return to == TaskStatus::Creating;
    case TaskStatus::Creating: return to == TaskStatus::Running;
    default: return false;
  }
}

static std::vector<std::string> str_list(const Json& a) {
  std::vector<std::string> out;
  for (auto& x : a.items()) out.push_back(x.str());
  return out;
}

TaskConfig TaskConfig::from_json(const Json& j) {
  TaskConfig c;
  c.id = j["id"].str();
  c.name = j["name"].str(c.id);
  c.registry_username = j["registry_username"].str();
  c.registry_password = j["registry_password"].str();
  c.image_name = j["image_name"].str();
  c.container_user = j["container_user"].str();
  c.privileged = j["privileged"].as_bool(false);
  c.gpu = (int)j["gpu"].as_int(0);
  for (auto& g : j["gpu_indices"].items()) c.gpu_indices.push_back((int)g.as_int());
  c.cpu = j["cpu"].as_double(0);
  c.memory = j["memory"].as_int(0);
  c.shm_size = j["shm_size"].as_int(0);
  c.network_mode = j["network_mode"].str("host");
  if (j["volumes"].is_array()) c.volumes = j["volumes"];
  if (j["volume_mounts"].is_array()) c.volume_mounts = j["volume_mounts"];
  if (j["instance_mounts"].is_array()) c.instance_mounts = j["instance_mounts"];
  c.host_ssh_user = j["host_ssh_user"].str();
  c.host_ssh_keys = str_list(j["host_ssh_keys"]);
  c.container_ssh_keys = str_list(j["container_ssh_keys"]);
  for (auto& kv : j["env"].members()) c.env[kv.first] = kv.second.str();
  for (auto& p : j["ports"].items()) c.ports.push_back((int)p.as_int());
  return c;
}

Json Task::to_json() const {
  Json j = Json::object();
  j.set("id", config.id);
  j.set("status", task_status_name(status));
  j.set("termination_reason", termination_reason);
  j.set("termination_message", termination_message);
  j.set("container_name", container_name);
  j.set("container_id", container_id);
  Json ports_j = Json::array();
  for (auto& p : ports) {
    Json pj = Json::object();
    pj.set("container", p.container);
    pj.set("host", p.host);
    ports_j.push_back(pj);
  }
  j.set("ports", ports_j);
  Json g = Json::array();
  for (int x : gpus) g.push_back(x);
  j.set("gpus", g);
  Json rn = Json::array();
  for (auto& r : render_nodes) rn.push_back(r);
  j.set("render_nodes", rn);
  j.set("runner_port", runner_port);
  Json tj = Json::object();
  for (auto& kv : timings) tj.set(kv.first, (long long)kv.second);
  j.set("timings", tj);
  return j;
}

bool TaskStorage::add(const Task& t) {
  std::lock_guard<std::mutex> lk(mu_);
  if (tasks_.count(t.config.id)) return false;
  tasks_[t.config.id] = t;
  return true;
}

bool TaskStorage::get(const std::string& id, Task& out) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = tasks_.find(id);
  if (it == tasks_.end()) return false;
  out = it->second;
  return true;
}

bool TaskStorage::update(const Task& t) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = tasks_.find(t.config.id);
  if (it == tasks_.end()) return false;
  it->second = t;
  return true;
}

bool TaskStorage::set_status(const std::string& id, TaskStatus st, const std::string& reason, const std::string& msg) {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = tasks_.find(id);
  if (it == tasks_.end() || !task_transition_allowed(it->second.status, st)) return false;
  it->second.status = st;
  it->second.timings[task_status_name(st)] = now_millis();
  if (st == TaskStatus::Terminated) {
    it->second.termination_reason = reason;
    it->second.termination_message = msg;
  }
  return true;
}

bool TaskStorage::remove(const std::string& id) {
  std::lock_guard<std::mutex> lk(mu_);
  return tasks_.erase(id) > 0;
}

std::vector<std::string> TaskStorage::ids() const {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::string> out;
  for (auto& kv : tasks_) out.push_back(kv.first);
  return out;
}

void GpuLock::init(int n, std::vector<std::vector<int>> xgmi, std::vector<int> numa) {
  std::lock_guard<std::mutex> lk(mu_);
  n_ = n;
  busy_.assign((size_t)n, false);
  xgmi_ = std::move(xgmi);
  numa_ = std::move(numa);
}

std::vector<int> GpuLock::acquire(int count) {
  std::lock_guard<std::mutex> lk(mu_);
  if (count < -1) return {};  // only -1 means "all"; any other negative count is a bad request
  std::vector<int> free_idx;
  for (int k = 0; k < n_; ++k)
    if (!busy_[(size_t)k]) free_idx.push_back(k);
  if (count < 0) count = (int)free_idx.size();
  if (count == 0) return {};
  auto pick = pick_gpus_xgmi(free_idx, count, xgmi_, numa_);
  for (int k : pick) busy_[(size_t)k] = true;
  return pick;
}

bool GpuLock::lock(const std::vector<int>& idx) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int k : idx)
    if (k < 0 || k >= n_ || busy_[(size_t)k]) return false;
  for (int k : idx) busy_[(size_t)k] = true;
  return true;
}

void GpuLock::release(const std::vector<int>& idx) {
  std::lock_guard<std::mutex> lk(mu_);
  for (int k : idx)
    if (k >= 0 && k < n_) busy_[(size_t)k] = false;
}

int GpuLock::free_count() const {
  std::lock_guard<std::mutex> lk(mu_);
  return (int)std::count(busy_.begin(), busy_.end(), false);
}

}  // namespace dsa
