// dstack-runner executor implementation (see executor.h).
#include "executor.h"
#include "rocprof.h"

#include <arpa/inet.h>
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <grp.h>
#include <ifaddrs.h>
#include <net/if.h>
#include <poll.h>
#include <pty.h>
#include <pwd.h>
#include <signal.h>
#include <stdarg.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <stdexcept>

#include <algorithm>
#include <cstring>
#include <map>
#include <sstream>

#include "../common/net.h"

extern char** environ;

namespace dsa {

const char* exec_state_name(ExecState s) {
  switch (s) {
    case ExecState::WaitSubmit: return "wait_submit";
    case ExecState::WaitCode: return "wait_code";
    case ExecState::WaitRun: return "wait_run";
    case ExecState::ServeLogs: return "serve_logs";
    case ExecState::WaitLogsFinished: return "wait_logs_finished";
  }
  return "unknown";
}

// ------------------------------------------------------------------------------------------------
// LogHistory
// ------------------------------------------------------------------------------------------------
void LogHistory::append(const std::string& msg) {
  {
    std::lock_guard<std::mutex> lk(mu_);
    int64_t ts = now_millis();
    if (ts <= last_) ts = last_ + 1;  // strictly increasing surrogate timestamps (timestamp.go)
    last_ = ts;
    events_.push_back(LogEvent{ts, msg});
  }
  cv_.notify_all();
}

std::vector<LogEvent> LogHistory::after(int64_t ts, size_t limit) const {
  std::lock_guard<std::mutex> lk(mu_);
  auto it = std::upper_bound(events_.begin(), events_.end(), ts,
                             [](int64_t t, const LogEvent& e) { return t < e.timestamp; });
  std::vector<LogEvent> out;
  for (; it != events_.end() && out.size() < limit; ++it) out.push_back(*it);
  return out;
}

int64_t LogHistory::last_timestamp() const {
  std::lock_guard<std::mutex> lk(mu_);
  return last_;
}

size_t LogHistory::size() const {
  std::lock_guard<std::mutex> lk(mu_);
  return events_.size();
}

bool LogHistory::wait_after(int64_t ts, int timeout_ms) const {
  std::unique_lock<std::mutex> lk(mu_);
  // system_clock deadline: libstdc++ maps it to pthread_cond_timedwait (steady-clock waits use
  // pthread_cond_clockwait, which ThreadSanitizer does not intercept -> false "double lock")
  const auto deadline = std::chrono::system_clock::now() + std::chrono::milliseconds(timeout_ms);
  return cv_.wait_until(lk, deadline, [&] { return last_ > ts; });
}

// ------------------------------------------------------------------------------------------------
// PATH lookup done in the parent (execvpe may allocate in the child)
std::string resolve_in_path(const std::string& prog, const std::string& path_var) {
  if (prog.find('/') != std::string::npos) return prog;
  size_t start = 0;
  while (start <= path_var.size()) {
    size_t end = path_var.find(':', start);
    if (end == std::string::npos) end = path_var.size();
    std::string dir = path_var.substr(start, end - start);
    if (dir.empty()) dir = ".";
    std::string cand = dir + "/" + prog;
    if (access(cand.c_str(), X_OK) == 0) return cand;
    start = end + 1;
  }
  return prog;
}

// env interpolation: ${VAR} -> value, $$ -> $
// ------------------------------------------------------------------------------------------------
static bool var_start(char c) { return (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || c == '_'; }
static bool var_char(char c) { return var_start(c) || (c >= '0' && c <= '9'); }

// ${NAME} expansion of job env values against the environment built so far (env.go
// interpolateVariables).  Only a well-formed reference is touched: a run of n dollars in front of
// {NAME} is halved, and an odd run leaves the last dollar to expand the variable ($${A} -> ${A},
// $$${A} -> $ + value).  Everything else -- bare $NAME, $$ not followed by a reference, ${}, ${!x},
// ${0x}, an unterminated ${ -- is kept byte for byte, so secrets and passwords containing dollars
// pass through unchanged.  An unset variable expands to "", as in a shell.  `err` is never set
// (kept for the callers' signature).
std::string interpolate_env(const std::string& s, const std::vector<std::pair<std::string, std::string>>& env,
                            std::string* err) {
  (void)err;
  std::string out;
  size_t i = 0;
  while (i < s.size()) {
    if (s[i] != '$') {
      out.push_back(s[i++]);
      continue;
    }
    size_t j = i;
    while (j < s.size() && s[j] == '$') ++j;
    const size_t n = j - i;
    size_t name_end = j + 1;
    bool ref = j < s.size() && s[j] == '{' && name_end < s.size() && var_start(s[name_end]);
    if (ref) {
      while (name_end < s.size() && var_char(s[name_end])) ++name_end;
      ref = name_end < s.size() && s[name_end] == '}';
    }
    if (!ref) {
      out.append(n, '$');
      i = j;
      continue;
    }
    out.append(n / 2, '$');
    const std::string name = s.substr(j + 1, name_end - j - 1);
    if (n % 2 == 0) {
      out += "{" + name + "}";
    } else {
      for (auto it = env.rbegin(); it != env.rend(); ++it)
        if (it->first == name) {
          out += it->second;
          break;
        }
    }
    i = name_end + 1;
  }
  return out;
}

// base/rel for the job's working directory (exec.go joinRelPath): "." is the base itself, a
// relative path may not climb out of it ("..", "a/../.."); an absolute path is taken as is (an
// image directory such as /workspace -- a superset of the reference, which refuses it).
bool join_rel_path(const std::string& base, const std::string& rel, std::string& out, std::string& err) {
  if (!rel.empty() && rel[0] == '/') {
    out = rel;
    return true;
  }
  std::vector<std::string> parts;
  for (auto& p : split(rel, '/')) {
    if (p.empty() || p == ".") continue;
    if (p == "..") {
      if (parts.empty()) {
        err = "working_dir " + rel + " is outside " + base;
        return false;
      }
      parts.pop_back();
      continue;
    }
    parts.push_back(p);
  }
  out = base;
  for (auto& p : parts) out += "/" + p;
  return true;
}

// ------------------------------------------------------------------------------------------------
// Executor
// ------------------------------------------------------------------------------------------------
Executor::Executor(RunnerOptions opts) : opts_(std::move(opts)) {
  mkdirs(opts_.temp_dir);
  code_path_ = opts_.temp_dir + "/code";
}

Executor::~Executor() {
  stop();
  if (worker_.joinable()) worker_.join();
}

void Executor::rlog(const char* fmt, ...) {
  char buf[4096];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  LOGI("%s", buf);
  runner_logs_.append(std::string(buf) + "\n");
}

void Executor::add_state(const std::string& state, const std::string& reason, const std::string& msg,
                         int exit_status) {
  std::lock_guard<std::mutex> lk(states_mu_);
  int64_t ts = now_millis();
  if (!states_.empty() && ts <= states_.back().timestamp) ts = states_.back().timestamp + 1;
  states_.push_back(JobStateEvent{state, ts, reason, msg, exit_status});
}

std::string Executor::submit(const Json& body) {
  if (state_ != ExecState::WaitSubmit) return std::string("submit not allowed in state ") + exec_state_name(state_);
  if (!body.get("job_spec").is_object()) return "job_spec is required";
  submit_body_ = body;
  state_ = ExecState::WaitCode;
  rlog("job submitted: %s", body["run_spec"]["run_name"].str(body["run_name"].str("?")).c_str());
  return "";
}

std::string Executor::upload_code(const std::string& blob) {
  if (state_ != ExecState::WaitCode) return std::string("upload_code not allowed in state ") + exec_state_name(state_);
  if (!write_file(code_path_, blob)) return "cannot write code blob";
  state_ = ExecState::WaitRun;
  rlog("code uploaded: %zu bytes", blob.size());
  return "";
}

std::string Executor::run() {
  if (state_ != ExecState::WaitRun) return std::string("run not allowed in state ") + exec_state_name(state_);
  state_ = ExecState::ServeLogs;
  worker_ = std::thread(&Executor::run_thread, this);
  return "";
}

void Executor::stop() {
  stop_requested_ = true;
  int pg = child_pgid_;
  if (pg > 0) {
    kill(-pg, SIGINT);  // graceful first; exec_job escalates to SIGKILL after 10 s
  }
}

void Executor::wait_finished() {
  std::unique_lock<std::mutex> lk(fin_mu_);
  fin_cv_.wait(lk, [&] { return finished_.load(); });
}

void Executor::mark_pulled(int64_t ts) const {
  (void)ts;
  if (finished_) pulled_after_finish_ = true;
}

Json Executor::pull(int64_t since) const {
  Json out = Json::object();
  Json states = Json::array();
  {
    std::lock_guard<std::mutex> lk(states_mu_);
    for (auto& s : states_) {
      if (s.timestamp <= since) continue;
      Json j = Json::object();
      j.set("state", s.state);
      j.set("timestamp", (long long)s.timestamp);
      j.set("termination_reason", s.termination_reason);
      j.set("termination_message", s.termination_message);
      if (s.exit_status >= 0) j.set("exit_status", s.exit_status);
      states.push_back(j);
    }
  }
  auto enc = [](const std::vector<LogEvent>& evs) {
    Json a = Json::array();
    for (auto& e : evs) {
      Json j = Json::object();
      j.set("timestamp", (long long)e.timestamp);
      j.set("message", base64_encode(e.message));
      a.push_back(j);
    }
    return a;
  };
  const size_t limit = 5000;
  auto jl = job_logs_.after(since, limit);
  auto rl = runner_logs_.after(since, limit);
  int64_t last = since;
  for (auto& e : jl) last = std::max(last, e.timestamp);
  for (auto& e : rl) last = std::max(last, e.timestamp);
  {
    std::lock_guard<std::mutex> lk(states_mu_);
    for (auto& s : states_) last = std::max(last, s.timestamp);
  }
  out.set("job_states", states);
  {
    std::lock_guard<std::mutex> lk(states_mu_);
    if (!probe_json_.empty()) {
      try {
        out.set("gpu_probe", Json::parse(probe_json_));
      } catch (...) {
      }
    }
    if (!preflight_json_.empty()) {
      try {
        out.set("rccl_preflight", Json::parse(preflight_json_));
      } catch (...) {
      }
    }
  }
  out.set("job_logs", enc(jl));
  out.set("runner_logs", enc(rl));
  out.set("last_updated", (long long)last);
  out.set("has_more", jl.size() >= limit || rl.size() >= limit);
  return out;
}

// RDMA devices with at least one ACTIVE port (/sys/class/infiniband/<dev>/ports/<n>/state =
// "4: ACTIVE"), sorted: the HCAs RCCL should use across nodes (IB, RoCE, AMD AINIC alike)
std::vector<std::string> active_rdma_devices() {
  const char* root_env = getenv("DSTACK_SYSFS_ROOT");
  const std::string base = std::string(root_env ? root_env : "") + "/sys/class/infiniband";
  std::vector<std::string> out;
  DIR* d = opendir(base.c_str());
  if (!d) return out;
  while (auto* e = readdir(d)) {
    std::string dev = e->d_name;
    if (dev == "." || dev == "..") continue;
    DIR* pd = opendir((base + "/" + dev + "/ports").c_str());
    if (!pd) continue;
    bool active = false;
    while (auto* pe = readdir(pd)) {
      std::string st;
      if (pe->d_name[0] != '.' && read_file(base + "/" + dev + "/ports/" + pe->d_name + "/state", st) &&
          st.find("ACTIVE") != std::string::npos)
        active = true;
    }
    closedir(pd);
    if (active) out.push_back(dev);
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

static std::string iface_for_ip(const std::string& ip) {
  struct ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) != 0) return "";
  std::string name;
  for (auto* p = ifa; p; p = p->ifa_next) {
    if (!p->ifa_addr || p->ifa_addr->sa_family != AF_INET) continue;
    char buf[64];
    inet_ntop(AF_INET, &((struct sockaddr_in*)p->ifa_addr)->sin_addr, buf, sizeof buf);
    if (ip == buf) {
      name = p->ifa_name;
      break;
    }
  }
  freeifaddrs(ifa);
  return name;
}

std::vector<std::pair<std::string, std::string>> Executor::build_env() const {
  std::vector<std::pair<std::string, std::string>> env;
  auto set = [&](const std::string& k, const std::string& v) {
    for (auto& kv : env)
      if (kv.first == k) {
        kv.second = v;
        return;
      }
    env.emplace_back(k, v);
  };
  auto has = [&](const std::string& k) {
    for (auto& kv : env)
      if (kv.first == k) return true;
    return false;
  };
  for (char** e = environ; e && *e; ++e) {
    std::string s = *e;
    auto eq = s.find('=');
    if (eq != std::string::npos) env.emplace_back(s.substr(0, eq), s.substr(eq + 1));
  }
  const Json& js = submit_body_["job_spec"];
  const Json& ci = submit_body_["cluster_info"];
  const Json& rs = submit_body_["run_spec"];
  std::string run_name = rs["run_name"].str(submit_body_["run_name"].str());
  std::string repo_id = rs["repo_id"].str(submit_body_["repo_id"].str());
  std::vector<std::string> ips;
  for (auto& ip : ci["job_ips"].items()) ips.push_back(ip.str());
  int node_rank = (int)js["job_num"].as_int(0);
  int nodes = ips.empty() ? (int)js["jobs_per_replica"].as_int(1) : (int)ips.size();
  int gpus_per_node = (int)ci["gpus_per_job"].as_int(0);
  std::string master = ci["master_job_ip"].str(ips.empty() ? "127.0.0.1" : ips[0]);
  std::string ips_joined;
  for (size_t k = 0; k < ips.size(); ++k) ips_joined += (k ? "\n" : "") + ips[k];
  // dstack rendezvous contract (executor.go:213-230)
  set("DSTACK_RUN_NAME", run_name);
  set("DSTACK_REPO_ID", repo_id);
  set("RUN_NAME", run_name);
  set("REPO_ID", repo_id);
  set("DSTACK_NODES_IPS", ips_joined);
  set("DSTACK_MASTER_NODE_IP", master);
  set("DSTACK_NODE_RANK", std::to_string(node_rank));
  set("DSTACK_NODES_NUM", std::to_string(nodes));
  set("DSTACK_GPUS_PER_NODE", std::to_string(gpus_per_node));
  set("DSTACK_GPUS_NUM", std::to_string(nodes * gpus_per_node));
  // MI355X additions: torch rendezvous defaults (torchrun reads PET_* as its CLI defaults) ...
  if (!has("MASTER_ADDR")) set("MASTER_ADDR", master);
  if (!has("MASTER_PORT")) set("MASTER_PORT", "29500");
  set("PET_NNODES", std::to_string(nodes));
  set("PET_NODE_RANK", std::to_string(node_rank));
  set("PET_MASTER_ADDR", master);
  set("PET_MASTER_PORT", "29500");
  if (gpus_per_node > 0) set("PET_NPROC_PER_NODE", std::to_string(gpus_per_node));
  // ... and RCCL over xGMI (intra-node) + RoCE/IB (inter-node)
  if (gpus_per_node > 0 && !has("HIP_VISIBLE_DEVICES")) {
    std::string v;
    for (int g = 0; g < gpus_per_node; ++g) v += (g ? "," : "") + std::to_string(g);
    set("HIP_VISIBLE_DEVICES", v);
  }
  if (!has("HSA_FORCE_FINE_GRAIN_PCIE")) set("HSA_FORCE_FINE_GRAIN_PCIE", "1");
  if (!has("HSA_ENABLE_IPC_MODE_LEGACY")) set("HSA_ENABLE_IPC_MODE_LEGACY", "0");
  if (nodes > 1 && !has("NCCL_SOCKET_IFNAME")) {
    std::string my_ip = node_rank < (int)ips.size() ? ips[node_rank] : "";
    std::string ifname = my_ip.empty() ? "" : iface_for_ip(my_ip);
    if (!ifname.empty()) set("NCCL_SOCKET_IFNAME", ifname);
  }
  if (nodes > 1 && !has("NCCL_IB_HCA")) {
    std::string hcas;
    for (auto& dev : active_rdma_devices()) hcas += (hcas.empty() ? "" : ",") + dev;
    if (!hcas.empty()) set("NCCL_IB_HCA", hcas);
  }
  // secrets (os env < dstack env < secrets < job env)
  for (auto& kv : submit_body_["secrets"].members()) set(kv.first, kv.second.str());
  std::vector<std::pair<std::string, std::string>> jobenv;
  for (auto& kv : js["env"].members()) {
    std::string err;
    set(kv.first, interpolate_env(kv.second.str(), env, &err));
  }
  set("HOME", opts_.home_dir);
  return env;
}

// Every fork of the runner (run_cmd's helpers and the RCCL pre-flight thread, the job's forkpty)
// happens under this lock, and every descriptor it creates is close-on-exec: the concurrent
// pre-flight forks from another thread while the job is being started, and a pipe or pty end
// inherited by the other child would hold that child's EOF open (the probe's output would never
// end while the job runs, or the job's pty would outlive the job in the probe).
static std::mutex g_fork_mu;

// Child side, before exec: nothing but 0/1/2 crosses into the new program (async-signal-safe).
static void close_inherited_fds() {
  if (close_range(3, ~0U, 0) != 0)
    for (int fd = 3; fd < 1024; ++fd) close(fd);
}

// Run argv to completion, collecting stdout+stderr.  `pgid_slot` (optional): the child becomes a
// process-group leader and its pid is published there while it runs, so another thread can stop
// the whole group (the concurrent pre-flight when its job ends first).
static int run_cmd(const std::vector<std::string>& argv, const std::string& cwd, std::string* output,
                   const std::vector<std::pair<std::string, std::string>>* env = nullptr,
                   std::atomic<int>* pgid_slot = nullptr) {
  std::vector<std::string> env_strs;
  if (env)
    for (auto& kv : *env) env_strs.push_back(kv.first + "=" + kv.second);
  std::vector<char*> a, e;
  for (auto& s : argv) a.push_back(const_cast<char*>(s.c_str()));
  a.push_back(nullptr);
  for (auto& s : env_strs) e.push_back(const_cast<char*>(s.c_str()));
  e.push_back(nullptr);
  int pipefd[2];
  pid_t pid;
  {
    std::lock_guard<std::mutex> lk(g_fork_mu);
    if (pipe2(pipefd, O_CLOEXEC) != 0) return -1;
    pid = fork();
    if (pid == 0) {
      if (pgid_slot) setpgid(0, 0);
      dup2(pipefd[1], 1);  // (dup2 clears close-on-exec on 1 and 2)
      dup2(pipefd[1], 2);
      close_inherited_fds();
      if (!cwd.empty() && chdir(cwd.c_str()) != 0) _exit(127);
      if (env) execvpe(a[0], a.data(), e.data());
      execvp(a[0], a.data());
      _exit(127);
    }
  }
  close(pipefd[1]);
  if (pid < 0) {
    close(pipefd[0]);
    return -1;
  }
  if (pgid_slot) {
    setpgid(pid, pid);  // (also in the child: whichever runs first, the group exists before a kill)
    *pgid_slot = pid;
  }
  char buf[4096];
  ssize_t n;
  while ((n = read(pipefd[0], buf, sizeof buf)) > 0)
    if (output) output->append(buf, (size_t)n);
  close(pipefd[0]);
  int st = 0;
  waitpid(pid, &st, 0);
  if (pgid_slot) *pgid_slot = 0;
  return WIFEXITED(st) ? WEXITSTATUS(st) : -1;
}

bool Executor::setup_repo(std::string& err) {
  const Json& rs = submit_body_["run_spec"];
  const Json& repo = rs["repo_data"].is_object() ? rs["repo_data"] : submit_body_["repo_data"];
  std::string type = repo["repo_type"].str("virtual");
  mkdirs(opts_.working_dir);
  std::string blob;
  read_file(code_path_, blob);
  if (type == "remote") {
    const Json& creds = submit_body_["repo_credentials"];
    std::string url = creds["clone_url"].str();
    if (url.empty()) {
      std::string host = repo["repo_host_name"].str(), name = repo["repo_name"].str();
      url = "https://" + host + "/" + name + ".git";
    }
    std::string token = creds["oauth_token"].str();
    if (!token.empty() && url.rfind("https://", 0) == 0) url = "https://" + token + "@" + url.substr(8);
    std::string key = creds["private_key"].str();
    if (!key.empty()) {
      std::string kp = opts_.temp_dir + "/repo_key";
      write_file(kp, key, 0600);
      setenv("GIT_SSH_COMMAND", ("ssh -i " + kp + " -o StrictHostKeyChecking=no").c_str(), 1);
    }
    std::vector<std::string> clone = {"git", "clone"};
    bool single = submit_body_["job_spec"]["single_branch"].as_bool(false);
    std::string branch = repo["repo_branch"].str();
    if (single && !branch.empty()) clone.insert(clone.end(), {"--single-branch", "--branch", branch});
    clone.push_back(url);
    clone.push_back(opts_.working_dir);
    std::string out;
    if (!path_exists(opts_.working_dir + "/.git")) {
      rlog("cloning repo %s", repo["repo_name"].str().c_str());
      if (run_cmd(clone, "", &out) != 0) {
        err = "git clone failed: " + out;
        return false;
      }
    }
    std::string hash = repo["repo_hash"].str();
    if (!hash.empty() && run_cmd({"git", "checkout", hash}, opts_.working_dir, &out) != 0) {
      err = "git checkout failed: " + out;
      return false;
    }
    // the committer identity of the user's local clone (repo_config_name/email), so that commits
    // made inside the job are attributed as on the laptop (repo.go prepareGit -> SetConfig)
    for (const char* k : {"name", "email"}) {
      std::string v = repo[std::string("repo_config_") + k].str();
      if (!v.empty() && run_cmd({"git", "config", std::string("user.") + k, v}, opts_.working_dir, &out) != 0) {
        err = std::string("git config user.") + k + " failed: " + out;
        return false;
      }
    }
    if (!blob.empty()) {
      if (run_cmd({"git", "apply", "--whitespace=nowarn", code_path_}, opts_.working_dir, &out) != 0) {
        err = "git apply failed: " + out;
        return false;
      }
    }
    return true;
  }
  // local / virtual: tar.gz blob
  if (!blob.empty()) {
    std::string out;
    if (run_cmd({"tar", "-xzf", code_path_, "-C", opts_.working_dir}, "", &out) != 0) {
      err = "code extraction failed: " + out;
      return false;
    }
  }
  return true;
}

bool Executor::run_probe() {
  if (opts_.probe_binary.empty() || !path_exists(opts_.probe_binary)) return true;
  std::string out;
  int rc = run_cmd({opts_.probe_binary, "--quick", "--json"}, "", &out);
  job_logs_.append("[dstack] GPU health probe: " + out + (out.empty() || out.back() != '\n' ? "\n" : ""));
  // the last JSON line is the probe document; the server copies it into the instance's health
  std::string doc;
  size_t end = out.find_last_not_of(" \r\n");
  if (end != std::string::npos) {
    size_t begin = out.rfind('\n', end);
    doc = out.substr(begin == std::string::npos ? 0 : begin + 1, end - (begin == std::string::npos ? 0 : begin + 1) + 1);
  }
  if (!doc.empty() && doc[0] == '{') {
    std::lock_guard<std::mutex> lk(states_mu_);
    probe_json_ = doc;
  }
  return rc == 0;
}

// Opt-in RCCL pre-flight for distributed tasks (job env DSTACK_RCCL_PREFLIGHT=1, >1 GPU in the
// job): every node runs the all-reduce probe with ONE communicator over all GPUs of all nodes,
// in the job's own process layout -- one process per GPU (DSTACK_GPUS_PER_NODE ranks per node,
// global rank node_rank*G + local, probes/ranks.h) bootstrapped like the job's RCCL (unique id from
// global rank 0 over TCP at the master node, port MASTER_PORT+1, the job's HIP_VISIBLE_DEVICES /
// NCCL_SOCKET_IFNAME env) -- so a broken fabric or a bad GPU fails the job in seconds with the
// probe's message instead of hanging inside torchrun.  By default it runs CONCURRENTLY with the
// job (DSTACK_RCCL_PREFLIGHT_MODE=concurrent; `blocking` runs it first): on one MI355X the probe
// takes ~6.7 s (profiles/e2e_rccl_preflight_r8d.txt), all of which would otherwise sit on the
// job's cold start, while the job spends its first seconds in imports, model init and the first
// step's compute before its first collective.
bool Executor::wants_rccl_preflight() const {
  const Json& js = submit_body_["job_spec"];
  std::string v = js["env"]["DSTACK_RCCL_PREFLIGHT"].str("");
  if (v.empty() || v == "0" || v == "false") return false;
  const Json& ci = submit_body_["cluster_info"];
  int nodes = ci["job_ips"].size() > 0 ? (int)ci["job_ips"].size() : (int)js["jobs_per_replica"].as_int(1);
  int gpus = (int)ci["gpus_per_job"].as_int(0);
  return v == "force" || nodes * gpus > 1;
}

bool Executor::preflight_concurrent() const {
  const std::string m = submit_body_["job_spec"]["env"]["DSTACK_RCCL_PREFLIGHT_MODE"].str("concurrent");
  return m != "blocking";
}

// The job ended (done, failed, stopped, or killed by max_duration) while the concurrent probe still
// runs: its process group (timeout + probe + one process per GPU) is stopped -- SIGTERM, SIGKILL
// after 5 s -- so the job's result is reported now, not after the probe's own limit.
void Executor::stop_preflight() {
  const int64_t deadline = now_millis() + 5000;
  bool termed = false;
  while (preflight_state_ == 1) {
    const int pg = preflight_pgid_;
    if (pg > 0) {
      if (!termed) {
        job_logs_.append("[dstack] RCCL pre-flight stopped: the job ended first\n");
        kill(-pg, SIGTERM);
        termed = true;
      } else if (now_millis() > deadline) {
        kill(-pg, SIGKILL);
      }
    }
    usleep(20000);
  }
}

bool Executor::run_rccl_preflight(std::string& msg) {
  if (opts_.probe_binary.empty() || !path_exists(opts_.probe_binary)) {
    job_logs_.append("[dstack] RCCL pre-flight skipped: no dstack-probe in this container\n");
    return true;
  }
  auto env = build_env();
  auto get = [&](const std::string& k, const std::string& d) {
    for (auto& kv : env)
      if (kv.first == k) return kv.second;
    return d;
  };
  const int port = atoi(get("MASTER_PORT", "29500").c_str()) + 1;
  // the probe's own per-rank deadline ends before the outer `timeout`, so a hung rank is reported
  // by name ("rank N timed out") instead of as a bare timeout
  int limit_s = atoi(get("DSTACK_RCCL_PREFLIGHT_TIMEOUT", "300").c_str());
  if (limit_s < 20) limit_s = 20;
  const int probe_ms = (limit_s - 15) * 1000 - 5000;  // run_ranks collects up to 5 s past its deadline
  // concurrent mode: a capped sweep (default 1..64 MiB) so the probe holds little HBM and link
  // time beside the starting job; blocking mode: the --quick sweep up to 256 MiB
  const bool concurrent = preflight_concurrent();
  const std::string max_mib = get("DSTACK_RCCL_PREFLIGHT_MAX_MIB", concurrent ? "64" : "0");
  std::vector<std::string> argv = {"timeout", "-k", "10", std::to_string(limit_s),
                                   opts_.probe_binary, "--rccl", "--quick", "--json", "--max-mib", max_mib,
                                   "--timeout-ms", std::to_string(probe_ms),
                                   "--gpus-per-node", get("DSTACK_GPUS_PER_NODE", "0"),
                                   "--nodes", get("DSTACK_NODES_NUM", "1"), "--node-rank", get("DSTACK_NODE_RANK", "0"),
                                   "--master", get("DSTACK_MASTER_NODE_IP", "127.0.0.1"),
                                   "--master-port", std::to_string(port)};
  std::string out;
  const int64_t t0 = now_millis();
  int rc = run_cmd(argv, opts_.working_dir, &out, &env, &preflight_pgid_);
  job_logs_.append(std::string("[dstack] RCCL pre-flight") + (concurrent ? ", concurrent (" : " (") +
                   std::to_string(now_millis() - t0) + " ms, exit " +
                   std::to_string(rc) + "): " + out + (out.empty() || out.back() != '\n' ? "\n" : ""));
  // the probe's document (last JSON line): the server records its busbw / verdict as the
  // instance's health, which the scheduler reads (an unhealthy host gets no new jobs)
  std::string doc, probe_msg;
  size_t end = out.find_last_not_of(" \r\n");
  if (end != std::string::npos) {
    size_t begin = out.rfind('\n', end);
    begin = begin == std::string::npos ? 0 : begin + 1;
    doc = out.substr(begin, end - begin + 1);
  }
  if (!doc.empty() && doc[0] == '{') {
    try {
      Json d = Json::parse(doc);
      probe_msg = d["message"].str("");
      // the server applies its bandwidth floor only to uncontended (blocking) measurements
      d.set("mode", std::string(concurrent ? "concurrent" : "blocking"));
      std::lock_guard<std::mutex> lk(states_mu_);
      preflight_json_ = d.dump();
    } catch (...) {
    }
  }
  if (rc != 0) {
    msg = rc == 124 || rc == 137 ? "RCCL pre-flight timed out" : "RCCL pre-flight failed (exit " + std::to_string(rc) + ")";
    if (!probe_msg.empty()) msg += ": " + probe_msg;
    return false;
  }
  return true;
}

// The repo's credentials made available to the job itself (executor.go setupCredentials): an SSH
// clone key as ~/.ssh/id_rsa, an HTTPS token as the GitHub CLI's ~/.config/gh/hosts.yml, so that
// `git push` / `gh` inside the job work as on the user's machine.  An existing file is never
// overwritten (the job fails instead); the written file is removed when the job ends.  Returns the
// path to remove ("" when nothing was written), or sets `err`.
std::string Executor::setup_credentials(int uid, int gid, std::string& err) {
  const Json& rs = submit_body_["run_spec"];
  const Json& repo = rs["repo_data"].is_object() ? rs["repo_data"] : submit_body_["repo_data"];
  const Json& creds = submit_body_["repo_credentials"];
  if (repo["repo_type"].str() != "remote" || !creds.is_object()) return "";
  std::string url = creds["clone_url"].str();
  bool ssh = url.rfind("ssh://", 0) == 0 || (url.find("://") == std::string::npos && url.find('@') != std::string::npos);
  std::string path, content;
  if (ssh) {
    content = creds["private_key"].str();
    if (content.empty()) {
      err = "private key is missing";
      return "";
    }
    path = opts_.home_dir + "/.ssh/id_rsa";
  } else {
    std::string token = creds["oauth_token"].str();
    if (token.empty()) return "";
    std::string host = url.substr(url.find("://") == std::string::npos ? 0 : url.find("://") + 3);
    host = host.substr(0, host.find_first_of("/:"));
    if (host.find('@') != std::string::npos) host = host.substr(host.find('@') + 1);
    path = opts_.home_dir + "/.config/gh/hosts.yml";
    content = host + ":\n  oauth_token: \"" + token + "\"\n";
  }
  if (path_exists(path)) {
    err = path + " already exists";
    return "";
  }
  std::string dir = path.substr(0, path.rfind('/'));
  mkdirs(dir, 0700);
  if (!write_file(path, content, 0600)) {
    err = "cannot write " + path;
    return "";
  }
  if (getuid() == 0 && uid >= 0) {  // readable by the job's user, not only by the runner
    if (chown(dir.c_str(), (uid_t)uid, (gid_t)(gid >= 0 ? gid : -1)) != 0 ||
        chown(path.c_str(), (uid_t)uid, (gid_t)(gid >= 0 ? gid : -1)) != 0)
      rlog("cannot chown %s to uid %d", path.c_str(), uid);
  }
  rlog("wrote repo credentials to %s", path.c_str());
  return path;
}

int Executor::exec_job(std::string& reason, std::string& msg) {
  const Json& js = submit_body_["job_spec"];
  std::vector<std::string> argv;
  for (auto& c : js["commands"].items()) argv.push_back(c.str());
  if (argv.empty()) {
    reason = "executor_error";
    msg = "empty command";
    return -1;
  }
  auto env = build_env();
  std::string wd = opts_.working_dir, wd_err;
  if (!join_rel_path(opts_.working_dir, js["working_dir"].str(), wd, wd_err)) {
    reason = "executor_error";
    msg = wd_err;
    return -1;
  }
  // DSTACK_ROCPROF=1: wrap the job in rocprofv3 kernel-trace statistics, plus the hardware
  // counters of DSTACK_ROCPROF_COUNTERS (validated against the one-pass budget, runner/rocprof.h);
  // the summaries are appended to the job log when the job ends (rocprof counters in run logs)
  std::string rocprof_dir, counters_spec;
  bool want_rocprof = false;
  for (auto& kv : env) {
    if (kv.first == "DSTACK_ROCPROF" && (kv.second == "1" || kv.second == "true")) want_rocprof = true;
    if (kv.first == "DSTACK_ROCPROF_COUNTERS") counters_spec = kv.second;
  }
  std::vector<std::string> counters = split_counters(counters_spec);
  if (!counters.empty()) want_rocprof = true;
  if (want_rocprof) {
    rocprof_dir = opts_.temp_dir + "/rocprof";
    mkdirs(rocprof_dir);
    std::string perr;
    if (!counters.empty() && !validate_pmc(counters, perr)) {
      job_logs_.append("[dstack] DSTACK_ROCPROF_COUNTERS ignored: " + perr + "\n");
      counters.clear();
    }
    // rocprofv3 goes directly in front of the GPU program (never in front of the job's shell or a
    // launcher: its preloaded library initialises the GPU in the process it wraps)
    std::vector<std::string> wrapped;
    std::string werr;
    std::string path_env = getenv("PATH") ? getenv("PATH") : "/usr/local/bin:/usr/bin:/bin";
    for (auto& kv : env)
      if (kv.first == "PATH") path_env = kv.second;
    if (rocprof_wrap(argv, rocprof_argv(rocprof_dir, counters), wrapped, werr, fs_program_lookup(path_env), wd)) {
      argv = wrapped;
    } else {
      job_logs_.append("[dstack] DSTACK_ROCPROF ignored: " + werr + "; the job runs unprofiled\n");
      rocprof_dir.clear();
    }
  }
  mkdirs(wd);
  std::vector<std::string> envs;
  for (auto& kv : env) envs.push_back(kv.first + "=" + kv.second);
  if (opts_.write_ssh_env) {
    std::string ssh_dir = opts_.home_dir + "/.ssh";
    mkdirs(ssh_dir, 0700);
    std::string content;
    for (auto& e : envs)
      if (e.find('\n') == std::string::npos) content += e + "\n";
    write_file(ssh_dir + "/environment", content, 0600);
  }
  int uid = -1, gid = -1;
  const Json& user = js["user"];
  if (user.is_object()) {
    if (user["uid"].is_number()) uid = (int)user["uid"].as_int();
    if (user["gid"].is_number()) gid = (int)user["gid"].as_int();
    if (uid < 0 && user["username"].is_string()) {
      struct passwd* pw = getpwnam(user["username"].str().c_str());
      if (pw) {
        uid = (int)pw->pw_uid;
        if (gid < 0) gid = (int)pw->pw_gid;
      }
    }
  }
  std::string cred_err;
  const std::string cred_path = setup_credentials(uid, gid, cred_err);
  if (!cred_err.empty()) {
    reason = "executor_error";
    msg = cred_err;
    return -1;
  }
  struct CredCleanup {  // the written key/token goes when the job does, whatever path it takes
    std::string p;
    ~CredCleanup() {
      if (!p.empty()) unlink(p.c_str());
    }
  } cred_cleanup{cred_path};
  // materialise argv/envp (and the resolved executable) before fork(): the runner is
  // multi-threaded (HTTP server), so the child may only make async-signal-safe calls until exec
  std::vector<char*> a, e;
  for (auto& s : argv) a.push_back(const_cast<char*>(s.c_str()));
  a.push_back(nullptr);
  for (auto& s : envs) e.push_back(const_cast<char*>(s.c_str()));
  e.push_back(nullptr);
  std::string path_var = getenv("PATH") ? getenv("PATH") : "/usr/local/bin:/usr/bin:/bin";
  for (auto& kv : env)
    if (kv.first == "PATH") path_var = kv.second;
  std::string exe = resolve_in_path(argv[0], path_var);
  int master = -1;
  struct winsize ws{};
  ws.ws_row = 50;
  ws.ws_col = 200;
  // a pty gives the job line-buffered output and a controlling terminal; sandboxes without
  // /dev/ptmx (e.g. unprivileged CI boxes) fall back to a pipe for stdout+stderr
  bool use_pty = true;
  int pipefd[2] = {-1, -1};
  const char* no_pty = getenv("DSTACK_RUNNER_NO_PTY");
  pid_t pid = -1;
  std::unique_lock<std::mutex> fork_lk(g_fork_mu);
  if (no_pty && *no_pty && *no_pty != '0')
    errno = ENOTSUP;
  else
    pid = forkpty(&master, nullptr, nullptr, &ws);
  if (pid < 0) {
    int pty_errno = errno;
    use_pty = false;
    if (pipe2(pipefd, O_CLOEXEC) != 0) {
      reason = "executor_error";
      msg = std::string("forkpty failed: ") + strerror(pty_errno) + "; pipe failed: " + strerror(errno);
      fork_lk.unlock();
      return -1;
    }
    rlog("forkpty unavailable (%s): using a pipe", strerror(pty_errno));
    pid = fork();
    if (pid < 0) {
      reason = "executor_error";
      msg = std::string("fork failed: ") + strerror(errno);
      fork_lk.unlock();
      close(pipefd[0]);
      close(pipefd[1]);
      return -1;
    }
    if (pid == 0) {
      setsid();
      int devnull = open("/dev/null", O_RDONLY);
      if (devnull >= 0) dup2(devnull, 0);
      dup2(pipefd[1], 1);
      dup2(pipefd[1], 2);
      close(pipefd[0]);
      close(pipefd[1]);
    } else {
      close(pipefd[1]);
      master = pipefd[0];
    }
  }
  if (pid == 0) {
    close_inherited_fds();
    if (chdir(wd.c_str()) != 0) _exit(126);
    if (getuid() == 0 && uid >= 0) {
      if (gid >= 0 && setgid((gid_t)gid) != 0) _exit(126);
      setgroups(0, nullptr);
      if (setuid((uid_t)uid) != 0) _exit(126);
    }
    execve(exe.c_str(), a.data(), e.data());
    static const char kMsg[] = "dstack-runner: exec failed\n";
    if (write(2, kMsg, sizeof kMsg - 1) < 0) _exit(127);
    _exit(127);
  }
  if (use_pty) fcntl(master, F_SETFD, FD_CLOEXEC);  // before any other fork can copy it
  fork_lk.unlock();
  child_pgid_ = pid;  // forkpty()/setsid() make the child a session (and process group) leader
  (void)use_pty;
  add_state("running");
  rlog("job started: pid=%d cwd=%s", pid, wd.c_str());
  int64_t max_duration = js["max_duration"].as_int(0);
  int64_t t0 = now_millis(), stop_at = 0;
  bool timed_out = false;
  bool stopped_by_preflight = false;  // latched while the job runs: a probe failing after the job
                                      // has exited does not rewrite the job's own result
  char buf[65536];
  int status = 0;
  bool exited = false;
  while (true) {
    struct pollfd p{master, POLLIN, 0};
    int r = poll(&p, 1, 200);
    if (r > 0 && (p.revents & POLLIN)) {
      ssize_t n = read(master, buf, sizeof buf);
      if (n > 0) job_logs_.append(std::string(buf, (size_t)n));
    }
    if (!exited) {
      pid_t w = waitpid(pid, &status, WNOHANG);
      if (w == pid) exited = true;
    }
    if (exited) {
      // Drain the pty until read() reports the slave side closed (EIO).  The kernel moves what the
      // child wrote into the master's buffer from a worker, which under load can run well after
      // the exit, so "no POLLIN within a few ms" is not the end of the output; read() after
      // POLLHUP flushes that pending input first.  Bounded: a descendant that keeps the pty open
      // ends the drain after 1 s of silence (5 s at most).
      const int64_t drain_end = now_millis() + 5000;
      while (now_millis() < drain_end) {
        struct pollfd q{master, POLLIN, 0};
        if (poll(&q, 1, 1000) <= 0) break;
        ssize_t n = read(master, buf, sizeof buf);
        if (n <= 0) break;
        job_logs_.append(std::string(buf, (size_t)n));
      }
      break;
    }
    int64_t now = now_millis();
    if (max_duration > 0 && !timed_out && now - t0 > max_duration * 1000) {
      timed_out = true;
      rlog("max_duration exceeded: stopping job");
      kill(-pid, SIGINT);
      stop_at = now;
    }
    if (stop_requested_ && stop_at == 0) stop_at = now;
    if (preflight_state_ == 3 && stop_at == 0) {  // the concurrent RCCL pre-flight failed
      rlog("RCCL pre-flight failed: stopping job");
      kill(-pid, SIGTERM);
      stop_at = now;
      stopped_by_preflight = true;
    }
    if (stop_at > 0 && now - stop_at > 10000) kill(-pid, SIGKILL);  // killDelay (executor.go:74)
  }
  close(master);
  child_pgid_ = 0;
  int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + (WIFSIGNALED(status) ? WTERMSIG(status) : 0);
  if (!rocprof_dir.empty()) {  // one pair of CSVs per profiled process (torchrun: one per rank)
    std::vector<std::string> stats, ctrs;
    DIR* d = opendir(rocprof_dir.c_str());
    if (d) {
      while (auto* e = readdir(d)) {
        std::string n = e->d_name, csv;
        if (n.find("kernel_stats.csv") != std::string::npos && read_file(rocprof_dir + "/" + n, csv))
          stats.push_back(csv);
        if (n.find("counter_collection.csv") != std::string::npos && read_file(rocprof_dir + "/" + n, csv))
          ctrs.push_back(csv);
      }
      closedir(d);
    }
    if (!stats.empty()) job_logs_.append(summarize_kernel_stats(stats, 15));
    if (!ctrs.empty()) job_logs_.append(summarize_counters(ctrs, counters, 15));
  }
  if (timed_out) {
    reason = "max_duration_exceeded";
    return code;
  }
  if (stopped_by_preflight) {
    reason = "executor_error";
    std::lock_guard<std::mutex> lk(states_mu_);
    msg = preflight_err_;
    return code;
  }
  if (stop_requested_) {
    reason = "terminated_by_user";
    return code;
  }
  if (code != 0) {
    reason = "container_exited_with_error";
    msg = "exit status " + std::to_string(code);
  }
  return code;
}

void Executor::run_job_steps() {
  std::string err;
  rlog("setting up repo");
  if (!setup_repo(err)) {
    rlog("repo setup failed: %s", err.c_str());
    add_state("failed", "executor_error", err);
  } else if (submit_body_["job_spec"]["gpu_probe"].as_bool(false) && !run_probe()) {
    add_state("failed", "gpu_health_check_failed", "GPU health probe failed");
  } else if (wants_rccl_preflight() && !preflight_concurrent() && !run_rccl_preflight(err)) {
    add_state("failed", "executor_error", err);
  } else if (stop_requested_) {
    add_state("terminated", "terminated_by_user");
  } else {
    // concurrent pre-flight: the job starts at once (its imports, model init and first step take
    // seconds before its first collective) while the probe checks the fabric beside it; a failed
    // probe stops the job with the probe's message, so a bad fabric still fails the job in
    // seconds, and a good one costs the job's start-up nothing
    std::thread preflight;
    if (wants_rccl_preflight() && preflight_concurrent()) {
      preflight_state_ = 1;
      preflight = std::thread([this] {
        std::string m;
        const bool ok = run_rccl_preflight(m);
        if (!ok) {
          std::lock_guard<std::mutex> lk(states_mu_);
          preflight_err_ = m;
        }
        preflight_state_ = ok ? 2 : 3;
      });
    }
    std::string reason, msg;
    int code = exec_job(reason, msg);
    if (preflight.joinable()) {
      stop_preflight();
      preflight.join();
    }
    if (reason == "max_duration_exceeded" || reason == "terminated_by_user")
      add_state("terminated", reason, msg, code);
    else if (!reason.empty())
      add_state("failed", reason, msg, code);
    else
      add_state("done", "done_by_runner", "", code);
    rlog("job finished: exit_status=%d %s", code, reason.c_str());
  }
}

void Executor::run_thread() {
  // Anything thrown while preparing or running the job fails the job with the error instead of
  // taking the runner down (the job's logs must still be served): executor.go's recover().
  try {
    if (const char* f = getenv("DSTACK_RUNNER_FAULT_INJECT"); f && *f && *f != '0')
      throw std::runtime_error(std::string("injected fault: ") + f);
    run_job_steps();
  } catch (const std::exception& e) {
    rlog("recovered: %s", e.what());
    add_state("failed", "executor_error", std::string("recovered: ") + e.what());
  } catch (...) {
    rlog("recovered: unknown exception");
    add_state("failed", "executor_error", "recovered: unknown exception");
  }
  state_ = ExecState::WaitLogsFinished;
  {
    std::lock_guard<std::mutex> lk(fin_mu_);
    finished_ = true;
  }
  fin_cv_.notify_all();
}

}  // namespace dsa
