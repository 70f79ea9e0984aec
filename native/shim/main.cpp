// dstack-shim entry point + REST API (reference: runner/cmd/shim/main.go:25-205,
// runner/internal/shim/api/{server.go:33-55,handlers.go:13-123}).
//
//   dstack-shim [--log-level N] [--shim-home DIR] [--shim-http-port 10998] [--host 0.0.0.0]
//               [--runner-binary-path PATH] [--runner-download-url URL] [--probe-binary PATH]
//               [--runner-http-port 10999] [--runner-ssh-port 10022] [--driver docker|process|auto]
//               [--runner-log-level N] [--privileged] [--service] [--no-startup-probe]
//
// Environment defaults (flags override): DSTACK_SHIM_HOME, DSTACK_SHIM_HTTP_PORT,
// DSTACK_SHIM_LOG_LEVEL, DSTACK_RUNNER_BINARY_PATH, DSTACK_RUNNER_DOWNLOAD_URL,
// DSTACK_RUNNER_HTTP_PORT, DSTACK_RUNNER_SSH_PORT, DSTACK_RUNNER_LOG_LEVEL,
// DSTACK_DOCKER_PRIVILEGED, DSTACK_SERVICE_MODE.
#include <signal.h>
#include <stdlib.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <thread>

#include "../common/amdgpu.h"
#include "../common/net.h"
#include "shim.h"

namespace dsa {

static const char* SHIM_VERSION = "0.1.0+mi355x";

Shim::Shim(ShimOptions o, std::unique_ptr<TaskDriver> driver) : opts_(std::move(o)), driver_(std::move(driver)) {
  // ONE discovery: the lock's indices, the xGMI matrix rows and the render nodes handed to
  // containers all refer to this snapshot (BDF order, amdgpu.h)
  auto gpus = discover_amd_gpus();
  std::vector<int> numa;
  for (auto& g : gpus) {
    numa.push_back(g.numa_node);
    inventory_render_.push_back(g.render_node);
  }
  auto xgmi = xgmi_matrix(gpus);  // amdsmi, else the KFD topology's xGMI io_links
  if (xgmi.size() != gpus.size()) xgmi.clear();  // never a mismatched topology
  gpus_.init((int)gpus.size(), xgmi, numa);
  LOGI("shim: driver=%s gpus=%zu", driver_->name(), gpus.size());
}

std::vector<std::string> Shim::render_nodes_of(const std::vector<int>& idx) const {
  std::vector<std::string> out;
  for (int i : idx)
    if (i >= 0 && i < (int)inventory_render_.size() && !inventory_render_[(size_t)i].empty())
      out.push_back(inventory_render_[(size_t)i]);
  return out;
}

void Shim::restore() {
  for (auto& t : driver_->restore()) {
    gpus_.lock(t.gpus);
    storage_.add(t);
    LOGI("restored task %s (%s)", t.config.id.c_str(), task_status_name(t.status));
    if (t.status == TaskStatus::Running) {
      std::string id = t.config.id;
      std::thread([this, id] {
        Task cur;
        if (!storage_.get(id, cur)) return;
        driver_->wait(cur);
        storage_.set_status(id, TaskStatus::Terminated, "container_exited", "");
        release_gpus(cur.gpus);
      }).detach();
    }
  }
}

Json Shim::host_info() {
  std::lock_guard<std::mutex> lk(hi_mu_);
  if (host_info_.is_null()) host_info_ = collect_host_info(opts_.home);
  return host_info_;
}

Json Shim::submit(const Json& cfg, int& http_status) {
  TaskConfig c = TaskConfig::from_json(cfg);
  if (c.id.empty()) {
    http_status = 400;
    return Json("task id is required");
  }
  Task t;
  t.config = c;
  t.created_ms = now_millis();
  t.timings["submitted"] = t.created_ms;
  if (!storage_.add(t)) {
    http_status = 409;
    return Json("task already exists");
  }
  http_status = 200;
  std::thread(&Shim::run_task, this, c.id).detach();
  return t.to_json();
}

std::string Shim::start_gpu_probe() {
  if (opts_.probe_binary.empty() || !path_exists(opts_.probe_binary) || inventory_render_.empty()) {
    std::lock_guard<std::mutex> lk(probe_mu_);
    probe_state_ = "unavailable";
    return "unavailable";
  }
  std::lock_guard<std::mutex> lk(probe_mu_);
  if (probing_) return "running";
  // the probe saturates every GPU: never beside a job.  All GPUs are taken here, under probe_mu_
  // (tasks grant under the same mutex), so a task either got its GPUs first (-> "busy") or finds
  // probing_ set and pre-empts the probe -- never a probe running next to a job.
  std::vector<int> all;
  for (int i = 0; i < gpus_.total(); ++i) all.push_back(i);
  if (!gpus_.lock(all)) return "busy";
  probing_ = true;
  probe_interrupted_ = false;
  probe_pid_ = -1;
  probe_state_ = "running";
  probe_started_ms_ = now_millis();
  std::thread(&Shim::probe_main, this).detach();
  return "started";
}

void Shim::probe_main() {
  // the probe runs as its own process group, so a GPU task can kill it (and its children) at once
  std::string out;
  int rc = -1;
  int pfd[2];
  if (pipe(pfd) == 0) {
    std::vector<std::string> argv = {opts_.probe_binary, "--quick", "--json"};
    std::vector<char*> a;
    for (auto& x : argv) a.push_back(const_cast<char*>(x.c_str()));
    a.push_back(nullptr);
    pid_t pid = fork();
    if (pid == 0) {
      setpgid(0, 0);
      dup2(pfd[1], 1);
      close(pfd[0]);
      close(pfd[1]);
      execv(a[0], a.data());
      _exit(127);
    }
    close(pfd[1]);
    if (pid > 0) {
      bool killed_early = false;
      {
        std::lock_guard<std::mutex> lk(probe_mu_);
        probe_pid_ = pid;
        killed_early = probe_interrupted_;  // pre-empted before the pid was known
      }
      if (killed_early) kill(-pid, SIGKILL), kill(pid, SIGKILL);
      char buf[4096];
      ssize_t n;
      while ((n = read(pfd[0], buf, sizeof buf)) > 0) out.append(buf, (size_t)n);
      int st = 0;
      waitpid(pid, &st, 0);
      rc = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
    }
    close(pfd[0]);
  }
  Json doc;
  for (auto& line : split(out, '\n')) {
    std::string l = trim(line);
    if (l.empty() || l[0] != '{') continue;
    try {
      doc = Json::parse(l);
    } catch (...) {
    }
  }
  {
    std::lock_guard<std::mutex> lk(probe_mu_);
    probe_pid_ = -1;
    std::vector<int> all;
    for (int i = 0; i < gpus_.total(); ++i) all.push_back(i);
    gpus_.release(all);  // under probe_mu_: a waiting task grants right after this block
    if (probe_interrupted_) {
      probe_state_ = "interrupted";  // the previous result (if any) stays the instance's health
    } else {
      probe_ran_ms_ = now_millis();
      if (doc.is_object()) {
        probe_doc_ = doc;
        probe_state_ = "done";
      } else {
        probe_state_ = "failed";
        Json e = Json::object();
        e.set("healthy", false);
        e.set("message", "probe exited " + std::to_string(rc) + " without a result: " + out.substr(0, 300));
        probe_doc_ = e;
      }
    }
    probing_ = false;
  }
  probe_cv_.notify_all();
  LOGI("gpu health probe %s in %lld ms", probe_state_.c_str(), (long long)(now_millis() - probe_started_ms_));
}

void Shim::release_gpus(const std::vector<int>& idx) {
  bool reprobe = false;
  {
    std::lock_guard<std::mutex> lk(probe_mu_);
    gpus_.release(idx);
    reprobe = probe_interrupted_ && !probing_ && gpus_.free_count() == gpus_.total();
  }
  if (reprobe) {
    LOGI("host idle again: re-running the interrupted GPU health probe");
    start_gpu_probe();
  }
}

Json Shim::gpu_health() {
  std::lock_guard<std::mutex> lk(probe_mu_);
  Json j = Json::object();
  j.set("state", probe_state_);
  j.set("started_at_ms", (long long)probe_started_ms_);
  j.set("ran_at_ms", (long long)probe_ran_ms_);
  j.set("result", probe_doc_.is_object() ? probe_doc_ : Json());
  return j;
}

void Shim::run_task(std::string id) {
  Task t;
  if (!storage_.get(id, t)) return;
  storage_.set_status(id, TaskStatus::Preparing);
  // GPU grant: explicit indices (server-side xGMI placement) or a count resolved here.  Granted
  // under probe_mu_, like the probe's own all-GPU lock: a health probe holding the GPUs is
  // pre-empted (killed; it re-runs when the host is idle) instead of delaying the job behind it.
  std::vector<int> granted;
  if (t.config.gpu != 0 || !t.config.gpu_indices.empty()) {
    std::unique_lock<std::mutex> lk(probe_mu_);
    if (probing_) {
      probe_interrupted_ = true;
      if (probe_pid_ > 0) {
        kill(-probe_pid_, SIGKILL);
        kill(probe_pid_, SIGKILL);
      }
      LOGI("task %s pre-empts the running GPU health probe", id.c_str());
      probe_cv_.wait_for(lk, std::chrono::seconds(30), [this] { return !probing_; });
    }
    std::string why;
    if (!t.config.gpu_indices.empty()) {
      if (gpus_.lock(t.config.gpu_indices)) granted = t.config.gpu_indices;
      else why = "requested GPUs are busy";
    } else {
      granted = gpus_.acquire(t.config.gpu);
      if (granted.empty() || (t.config.gpu > 0 && (int)granted.size() != t.config.gpu)) {
        gpus_.release(granted);
        granted.clear();
        why = "not enough free GPUs";
      }
    }
    if (!why.empty()) {
      lk.unlock();
      storage_.set_status(id, TaskStatus::Terminated, "creating_container_error", why);
      return;
    }
  }
  if (!storage_.get(id, t)) return;
  t.gpus = granted;
  t.render_nodes = render_nodes_of(granted);
  storage_.update(t);
  if (!t.config.host_ssh_keys.empty() && !t.config.host_ssh_user.empty())
    add_authorized_keys(t.config.host_ssh_user, t.config.host_ssh_keys);
  storage_.set_status(id, TaskStatus::Pulling);
  storage_.set_status(id, TaskStatus::Creating);
  if (!storage_.get(id, t)) return;
  std::string reason, msg;
  bool ok = driver_->run(t, reason, msg);
  Task cur;
  if (storage_.get(id, cur)) {
    t.status = cur.status;
    t.timings.insert(cur.timings.begin(), cur.timings.end());
    storage_.update(t);
  }
  if (!ok) {
    LOGW("task %s failed to start: %s", id.c_str(), msg.c_str());
    release_gpus(granted);
    storage_.set_status(id, TaskStatus::Terminated, reason, msg);
    return;
  }
  storage_.set_status(id, TaskStatus::Running);
  LOGI("task %s running (runner port %d, gpus %zu)", id.c_str(), t.runner_port, granted.size());
  driver_->wait(t);
  release_gpus(granted);
  storage_.set_status(id, TaskStatus::Terminated, "done_by_runner", "");
  if (!t.config.host_ssh_keys.empty() && !t.config.host_ssh_user.empty())
    remove_authorized_keys(t.config.host_ssh_user, t.config.host_ssh_keys);
}

bool Shim::get(const std::string& id, Json& out) const {
  Task t;
  if (!storage_.get(id, t)) return false;
  out = t.to_json();
  return true;
}

Json Shim::list() const {
  Json j = Json::object();
  Json ids = Json::array();
  for (auto& id : storage_.ids()) ids.push_back(id);
  j.set("ids", ids);
  return j;
}

bool Shim::terminate(const std::string& id, const std::string& reason, const std::string& msg, int timeout_s) {
  Task t;
  if (!storage_.get(id, t)) return false;
  if (t.status == TaskStatus::Terminated) return true;
  driver_->terminate(t, timeout_s);
  storage_.set_status(id, TaskStatus::Terminated, reason.empty() ? "terminated_by_server" : reason, msg);
  return true;
}

bool Shim::remove(const std::string& id, std::string& err) {
  Task t;
  if (!storage_.get(id, t)) {
    err = "not found";
    return false;
  }
  if (t.status != TaskStatus::Terminated) {
    err = "task is not terminated";
    return false;
  }
  driver_->remove(t);
  storage_.remove(id);
  return true;
}

}  // namespace dsa

using namespace dsa;

int main(int argc, char** argv) {
  ShimOptions o;
  const char* home = getenv("HOME");
  o.home = std::string(home ? home : "/root") + "/.dstack-shim";
  int port = 10998;
  std::string host = "0.0.0.0";
  bool service = false;
  bool startup_probe = true;
  if (const char* v = getenv("DSTACK_SHIM_STARTUP_PROBE")) startup_probe = std::string(v) != "0";
  // environment defaults (the reference's EnvVars, main.go:40-124); command-line flags override them
  auto env = [](const char* name) -> const char* {
    const char* v = getenv(name);
    return v && *v ? v : nullptr;
  };
  auto env_true = [&](const char* name) {
    const char* v = env(name);
    if (!v) return false;
    std::string s = v;
    return s == "1" || s == "true" || s == "TRUE" || s == "True" || s == "yes";
  };
  if (const char* v = env("DSTACK_SHIM_HOME")) o.home = v;
  if (const char* v = env("DSTACK_SHIM_HTTP_PORT")) port = atoi(v);
  if (const char* v = env("DSTACK_SHIM_LOG_LEVEL")) set_log_level(atoi(v));
  if (const char* v = env("DSTACK_RUNNER_BINARY_PATH")) o.runner_binary = v;
  if (const char* v = env("DSTACK_RUNNER_DOWNLOAD_URL")) o.runner_download_url = v;
  if (const char* v = env("DSTACK_RUNNER_HTTP_PORT")) o.runner_http_port = atoi(v);
  if (const char* v = env("DSTACK_RUNNER_SSH_PORT")) o.runner_ssh_port = atoi(v);
  if (const char* v = env("DSTACK_RUNNER_LOG_LEVEL")) o.runner_log_level = atoi(v);
  if (env_true("DSTACK_DOCKER_PRIVILEGED")) o.privileged = true;
  if (env_true("DSTACK_SERVICE_MODE")) service = true;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--log-level") set_log_level(atoi(next().c_str()));
    else if (a == "--shim-home") o.home = next();
    else if (a == "--shim-http-port") port = atoi(next().c_str());
    else if (a == "--host") host = next();
    else if (a == "--runner-binary-path") o.runner_binary = next();
    else if (a == "--runner-download-url") o.runner_download_url = next();
    else if (a == "--probe-binary") o.probe_binary = next();
    else if (a == "--runner-http-port") o.runner_http_port = atoi(next().c_str());
    else if (a == "--runner-ssh-port") o.runner_ssh_port = atoi(next().c_str());
    else if (a == "--runner-log-level") o.runner_log_level = atoi(next().c_str());
    else if (a == "--driver") o.driver = next();
    else if (a == "--volumes-root") o.volumes_root = next();
    else if (a == "--privileged") o.privileged = true;
    else if (a == "--service") service = true;
    else if (a == "--no-startup-probe") startup_probe = false;
    else if (a == "--version") {
      printf("%s\n", SHIM_VERSION);
      return 0;
    } else if (a == "--list-gpus") {  // both discovery paths, for checking they agree (BDF order)
      Json j = Json::object();
      Json smi = Json::array(), sys = Json::array();
      if (AmdSmi::instance().available())
        for (auto& g : AmdSmi::instance().discover()) smi.push_back(gpu_to_json(g));
      for (auto& g : discover_amd_gpus_sysfs()) sys.push_back(gpu_to_json(g));
      j.set("amdsmi", smi);
      j.set("sysfs", sys);
      printf("%s\n", j.dump().c_str());
      return 0;
    } else if (a == "--gpu-metrics") {  // one amdsmi sample per GPU (runner wire format), then exit
      Json arr = Json::array();
      if (AmdSmi::instance().available())
        for (auto& m : AmdSmi::instance().metrics()) {
          Json j = gpu_metrics_to_json(m);
          j.set("index", m.index);
          arr.push_back(j);
        }
      printf("%s\n", arr.dump().c_str());
      return 0;
    } else if (a == "--host-info") {  // print host_info.json and exit (used by SSH-fleet deploy)
      printf("%s\n", collect_host_info("/").dump().c_str());
      return 0;
    } else {
      fprintf(stderr, "unknown flag %s\n", a.c_str());
      return 2;
    }
  }
  signal(SIGPIPE, SIG_IGN);
  struct sigaction sa{};
  sa.sa_handler = [](int sig) {
    kill_registered_children(SIGTERM);
    _exit(sig == SIGTERM ? 0 : 128 + sig);
  };
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  mkdirs(o.home);
  if (o.runner_binary.empty()) o.runner_binary = o.home + "/dstack-runner";
  if (!path_exists(o.runner_binary) && !o.runner_download_url.empty()) {  // runner.go:18-109
    LOGI("downloading runner from %s", o.runner_download_url.c_str());
    // http:// or https:// (verified TLS, redirects followed); written to a temp name and renamed,
    // so a crash mid-download never leaves a truncated runner behind (runner.go:18-109)
    auto r = http_get_url(o.runner_download_url, 10 * 60 * 1000);
    const std::string tmp = o.runner_binary + ".download";
    if (!r.ok() || !write_file(tmp, r.body, 0755) || ::rename(tmp.c_str(), o.runner_binary.c_str()) != 0) {
      LOGE("runner download failed: %d %s", r.status, r.error.c_str());
      ::unlink(tmp.c_str());
      return 1;
    }
  }
  bool use_docker = o.driver == "docker" || (o.driver == "auto" && docker_available(o.docker_socket));
  Shim shim(o, use_docker ? make_docker_driver(o) : make_process_driver(o));
  shim.restore();
  if (service) write_file(o.home + "/host_info.json", shim.host_info().dump());

  HttpServer srv(host, port);
  srv.route("GET", "/api/healthcheck", [&](HttpRequest&) {
    Json j = Json::object();
    j.set("service", "dstack-shim");
    j.set("version", SHIM_VERSION);
    j.set("api_version", 2);  // 2: tasks + /api/gpu_health (server ShimClient negotiates on this)
    j.set("driver", shim.driver_name());
    j.set("gpus_free", shim.gpu_lock().free_count());
    j.set("gpus_total", shim.gpu_lock().total());
    j.set("gpu_health", shim.gpu_health()["state"].str());
    return HttpResponse::json(j);
  });
  // GPU health (HIP HBM/MFMA probes, relative per-SKU thresholds): read the latest result, or
  // start a probe (202; 409 while GPU tasks run)
  srv.route("GET", "/api/gpu_health", [&](HttpRequest&) { return HttpResponse::json(shim.gpu_health()); });
  srv.route("POST", "/api/gpu_health/probe", [&](HttpRequest&) {
    std::string st = shim.start_gpu_probe();
    Json j = Json::object();
    j.set("state", st);
    return HttpResponse::json(j, st == "started" || st == "running" ? 202 : (st == "busy" ? 409 : 200));
  });
  srv.route("GET", "/api/host_info", [&](HttpRequest&) { return HttpResponse::json(shim.host_info()); });
  srv.route("GET", "/api/tasks", [&](HttpRequest&) { return HttpResponse::json(shim.list()); });
  srv.route("GET", "/api/tasks/{id}", [&](HttpRequest& r) {
    Json j;
    if (!shim.get(r.params["id"], j)) return HttpResponse::error(404, "task not found");
    return HttpResponse::json(j);
  });
  srv.route("POST", "/api/tasks", [&](HttpRequest& r) {
    Json body;
    try {
      body = r.json();
    } catch (const std::exception& e) {
      return HttpResponse::error(400, e.what());
    }
    int st = 200;
    Json out = shim.submit(body, st);
    return st == 200 ? HttpResponse::json(out) : HttpResponse::error(st, out.str());
  });
  srv.route("POST", "/api/tasks/{id}/terminate", [&](HttpRequest& r) {
    Json body = r.body.empty() ? Json::object() : Json::parse(r.body);
    if (!shim.terminate(r.params["id"], body["termination_reason"].str(), body["termination_message"].str(),
                        (int)body["timeout"].as_int(10)))
      return HttpResponse::error(404, "task not found");
    Json j;
    shim.get(r.params["id"], j);
    return HttpResponse::json(j);
  });
  srv.route("POST", "/api/tasks/{id}/remove", [&](HttpRequest& r) {
    std::string err;
    if (!shim.remove(r.params["id"], err)) return HttpResponse::error(err == "not found" ? 404 : 409, err);
    return HttpResponse::json(Json::object());
  });
  if (srv.start() < 0) return 1;
  LOGI("dstack-shim %s listening on %s:%d (driver %s)", SHIM_VERSION, host.c_str(), srv.port(), shim.driver_name());
  // print the bound port for supervisors that start us with --shim-http-port 0
  printf("DSTACK_SHIM_PORT=%d\n", srv.port());
  fflush(stdout);
  // first health probe right after start, asynchronously: the server reads it at registration
  // (GET /api/gpu_health) with no job waiting on it
  if (startup_probe) shim.start_gpu_probe();
  srv.serve_forever();
  return 0;
}
