// Docker task driver: talks to the Docker Engine API over /var/run/docker.sock (no SDK).
// Reference: runner/internal/shim/docker.go:52-1158.  MI355X-specific container config:
// /dev/kfd + the granted /dev/dri/renderD* nodes, --ipc=host, group video/render,
// seccomp=unconfined + SYS_PTRACE (rocgdb/rocprof inside the job), /dev/infiniband + unlimited
// memlock for RCCL over RoCE/IB, shm sized from the request.
#include <unistd.h>

#include <cstring>
#include <sstream>
#include <thread>

#include "../common/amdgpu.h"
#include "../common/net.h"
#include "shim.h"

namespace dsa {

bool docker_available(const std::string& socket_path) {
  if (!path_exists(socket_path)) return false;
  HttpClientRequest r;
  r.unix_socket = socket_path;
  r.path = "/_ping";
  r.timeout_ms = 2000;
  return http_request(r).ok();
}

std::string container_bootstrap_script(const ShimOptions& o, const std::vector<std::string>& keys) {
  std::string authorized;
  for (auto& k : keys) authorized += k + "\n";
  // single-quoted for the shell: a key comment may contain a quote ("alice's laptop")
  std::string quoted;
  for (char c : authorized) quoted += c == '\'' ? std::string("'\\''") : std::string(1, c);
  authorized = quoted;
  // The runner (the job's critical path) is exec'd at once; sshd -- installed first when the image
  // lacks it, which can take a minute of package downloads -- comes up in a background subshell.
  // `dstack attach` retries until it listens (core/services/ssh/attach.py).  The reference installs
  // and starts sshd synchronously before the runner (runner/internal/shim/docker.go:873-911).
  std::ostringstream s;
  s << "set -e\n"
    << "mkdir -p ~/.ssh && chmod 700 ~/.ssh\n"
    << "printf '%s' '" << authorized << "' >> ~/.ssh/authorized_keys && chmod 600 ~/.ssh/authorized_keys\n"
    << "(\n"
    << "  export DEBIAN_FRONTEND=noninteractive\n"
    << "  if ! command -v sshd >/dev/null 2>&1; then\n"
    << "    (apt-get update -qq && apt-get install -y -qq openssh-server) || (yum install -y -q openssh-server) || "
       "(apk add -q openssh-server) || true\n"
    << "  fi\n"
    << "  mkdir -p /run/sshd\n"
    << "  if command -v sshd >/dev/null 2>&1; then ssh-keygen -A || true; "
    << "$(command -v sshd) -p " << o.runner_ssh_port
    << " -o PermitUserEnvironment=yes -o PasswordAuthentication=no -o PidFile=none || true; fi\n"
    << ") </dev/null >/dev/null 2>&1 &\n"
    << "exec /usr/local/bin/dstack-runner --log-level " << (o.runner_log_level >= 0 ? o.runner_log_level : log_level()) << " start --http-port " << o.runner_http_port
    << " --temp-dir /tmp/runner --home-dir \"$HOME\" --working-dir /workflow --ssh-env"
    << (o.probe_binary.empty() ? "" : " --probe /usr/local/bin/dstack-probe") << "\n";
  return s.str();
}

namespace {

std::string url_escape(const std::string& s) {
  std::string out;
  for (unsigned char c : s) {
    if (isalnum(c) || c == '-' || c == '_' || c == '.' || c == '~' || c == '/' || c == ':')
      out.push_back((char)c);
    else {
      char b[4];
      snprintf(b, sizeof b, "%%%02X", c);
      out += b;
    }
  }
  return out;
}

class DockerDriver : public TaskDriver {
 public:
  explicit DockerDriver(ShimOptions o) : o_(std::move(o)) {}
  const char* name() const override { return "docker"; }

  HttpClientResponse call(const std::string& method, const std::string& path, const std::string& body = "",
                          int timeout_ms = 60000, std::function<bool(const std::string&)> on_chunk = nullptr,
                          std::map<std::string, std::string> headers = {}) {
    HttpClientRequest r;
    r.unix_socket = o_.docker_socket;
    r.method = method;
    r.path = path;
    r.body = body;
    r.timeout_ms = timeout_ms;
    r.on_chunk = on_chunk;
    r.headers = headers;
    return http_request(r);
  }

  bool pull(const Task& t, std::string& msg) {
    std::string image = t.config.image_name, tag = "latest";
    auto slash = image.rfind('/'), colon = image.rfind(':');
    if (colon != std::string::npos && (slash == std::string::npos || colon > slash)) {
      tag = image.substr(colon + 1);
      image = image.substr(0, colon);
    }
    // already present?
    if (call("GET", "/images/" + url_escape(t.config.image_name) + "/json").ok()) return true;
    std::map<std::string, std::string> headers;
    if (!t.config.registry_username.empty()) {
      Json auth = Json::object();
      auth.set("username", t.config.registry_username);
      auth.set("password", t.config.registry_password);
      headers["X-Registry-Auth"] = base64_encode(auth.dump());
    }
    std::string last_error;
    auto r = call("POST", "/images/create?fromImage=" + url_escape(image) + "&tag=" + url_escape(tag), "",
                  o_.pull_timeout_s * 1000,
                  [&](const std::string& chunk) {
                    for (auto& line : split(chunk, '\n')) {
                      if (trim(line).empty()) continue;
                      try {
                        Json j = Json::parse(line);
                        if (j.has("error")) last_error = j["error"].str();
                      } catch (...) {
                      }
                    }
                    return true;
                  },
                  headers);
    if (!r.ok() || !last_error.empty()) {
      msg = "pull failed: " + (last_error.empty() ? r.error + r.body : last_error);
      return false;
    }
    return true;
  }

  bool run(Task& t, std::string& reason, std::string& msg) override {
    std::map<std::string, std::string> vol_paths;
    if (!prepare_volumes(t, o_.volumes_root, vol_paths, msg)) {
      reason = "volume_error";
      return false;
    }
    if (!pull(t, msg)) {
      reason = "creating_container_error";
      return false;
    }
    t.timings["pulled"] = now_millis();
    std::vector<std::string> keys = t.config.container_ssh_keys;
    Json cfg = Json::object();
    cfg.set("Image", t.config.image_name);
    Json ep = Json::array();
    ep.push_back("/bin/sh");
    ep.push_back("-c");
    cfg.set("Entrypoint", ep);
    Json cmd = Json::array();
    cmd.push_back(container_bootstrap_script(o_, keys));
    cfg.set("Cmd", cmd);
    if (!t.config.container_user.empty()) cfg.set("User", t.config.container_user);
    Json env = Json::array();
    for (auto& kv : t.config.env) env.push_back(kv.first + "=" + kv.second);
    cfg.set("Env", env);
    Json labels = Json::object();
    labels.set("dstack.task_id", t.config.id);
    std::string gl;
    for (size_t k = 0; k < t.gpus.size(); ++k) gl += (k ? "," : "") + std::to_string(t.gpus[k]);
    labels.set("dstack.gpus", gl);
    std::string rl;
    for (size_t k = 0; k < t.render_nodes.size(); ++k) rl += (k ? "," : "") + t.render_nodes[k];
    labels.set("dstack.render_nodes", rl);
    cfg.set("Labels", labels);
    Json hc = Json::object();
    Json binds = Json::array();
    binds.push_back(o_.runner_binary + ":/usr/local/bin/dstack-runner:ro");
    if (!o_.probe_binary.empty()) binds.push_back(o_.probe_binary + ":/usr/local/bin/dstack-probe:ro");
    for (auto& m : t.config.instance_mounts.items()) {
      // optional mounts are skipped when the host path does not exist (e.g. a cache dir)
      if (m["optional"].as_bool() && access(m["instance_path"].str().c_str(), F_OK) != 0) continue;
      binds.push_back(m["instance_path"].str() + ":" + m["path"].str());
    }
    for (auto& m : t.config.volume_mounts.items()) {
      auto it = vol_paths.find(m["name"].str());
      std::string host = it != vol_paths.end() ? it->second : o_.volumes_root + "/" + m["name"].str();
      binds.push_back(host + ":" + m["path"].str());
    }
    hc.set("Binds", binds);
    hc.set("NetworkMode", t.config.network_mode);
    hc.set("Privileged", t.config.privileged || o_.privileged);
    hc.set("IpcMode", "host");
    Json cap = Json::array();
    cap.push_back("SYS_PTRACE");
    hc.set("CapAdd", cap);
    Json sec = Json::array();
    sec.push_back("seccomp=unconfined");
    hc.set("SecurityOpt", sec);
    if (t.config.shm_size > 0) hc.set("ShmSize", (long long)t.config.shm_size);
    if (t.config.memory > 0) hc.set("Memory", (long long)t.config.memory);
    if (t.config.cpu > 0) hc.set("NanoCpus", (long long)(t.config.cpu * 1e9));
    Json devices = Json::array();
    auto add_dev = [&](const std::string& p) {
      Json d = Json::object();
      d.set("PathOnHost", p);
      d.set("PathInContainer", p);
      d.set("CgroupPermissions", "rwm");
      devices.push_back(d);
    };
    if (!t.gpus.empty()) {
      // /dev/kfd (the compute queue device) + exactly the granted render nodes: the container's
      // ROCm runtime then enumerates only the job's GPUs, in host BDF order
      add_dev("/dev/kfd");
      for (auto& rn : t.render_nodes) add_dev(rn);
      Json groups = Json::array();
      groups.push_back("video");
      groups.push_back("render");
      hc.set("GroupAdd", groups);
    }
    if (!o_.infiniband_path.empty() && path_exists(o_.infiniband_path)) {  // RCCL over RoCE/IB (docker.go:1039-1062)
      add_dev(o_.infiniband_path);
      Json ul = Json::array();
      Json m = Json::object();
      m.set("Name", "memlock");
      m.set("Soft", -1);
      m.set("Hard", -1);
      ul.push_back(m);
      hc.set("Ulimits", ul);
    }
    hc.set("Devices", devices);
    if (t.config.network_mode == "bridge") {
      Json pb = Json::object();
      Json exposed = Json::object();
      std::vector<int> ports = {o_.runner_http_port, o_.runner_ssh_port};
      for (int p : t.config.ports) ports.push_back(p);
      for (int p : ports) {
        Json binding = Json::array();
        Json b = Json::object();
        b.set("HostPort", "");
        binding.push_back(b);
        pb.set(std::to_string(p) + "/tcp", binding);
        exposed.set(std::to_string(p) + "/tcp", Json::object());
      }
      hc.set("PortBindings", pb);
      cfg.set("ExposedPorts", exposed);
    }
    cfg.set("HostConfig", hc);
    std::string cname = unique_container_name(t.config.name.empty() ? t.config.id : t.config.name);
    auto cr = call("POST", "/containers/create?name=" + url_escape(cname), cfg.dump());
    if (!cr.ok()) {
      reason = "creating_container_error";
      msg = "create failed: " + cr.body + cr.error;
      return false;
    }
    t.container_id = Json::parse(cr.body)["Id"].str();
    t.container_name = cname;
    auto sr = call("POST", "/containers/" + t.container_id + "/start");
    if (!sr.ok()) {
      reason = "creating_container_error";
      msg = "start failed: " + sr.body + sr.error;
      return false;
    }
    inspect_ports(t);
    return true;
  }

  void inspect_ports(Task& t) {
    auto r = call("GET", "/containers/" + t.container_id + "/json");
    if (!r.ok()) return;
    Json j = Json::parse(r.body);
    t.ports.clear();
    for (auto& kv : j["NetworkSettings"]["Ports"].members()) {
      int cport = atoi(kv.first.c_str());
      if (kv.second.is_array() && kv.second.size() > 0) {
        int hport = atoi(kv.second[(size_t)0]["HostPort"].str().c_str());
        t.ports.push_back(PortMapping{cport, hport});
        if (cport == o_.runner_http_port) t.runner_port = hport;
      }
    }
    if (t.config.network_mode == "host") {
      t.runner_port = o_.runner_http_port;
      t.ports.push_back(PortMapping{o_.runner_http_port, o_.runner_http_port});
    }
  }

  void wait(Task& t) override {
    if (t.container_id.empty()) return;
    call("POST", "/containers/" + t.container_id + "/wait", "", 2000000000);
  }

  void terminate(Task& t, int timeout_s) override {
    if (t.container_id.empty()) return;
    call("POST", "/containers/" + t.container_id + "/stop?t=" + std::to_string(timeout_s), "",
         (timeout_s + 30) * 1000);
  }

  void remove(Task& t) override {
    if (!t.container_id.empty()) call("DELETE", "/containers/" + t.container_id + "?force=1&v=1");
    unmount_volumes(t, o_.volumes_root);
  }

  std::vector<Task> restore() override {
    std::vector<Task> out;
    auto r = call("GET", "/containers/json?all=1&filters=" + url_escape("{\"label\":[\"dstack.task_id\"]}"));
    if (!r.ok()) return out;
    Json arr = Json::parse(r.body);
    for (auto& c : arr.items()) {
      Task t;
      t.config.id = c["Labels"]["dstack.task_id"].str();
      t.container_id = c["Id"].str();
      t.container_name = c["Names"][(size_t)0].str();
      for (auto& g : split(c["Labels"]["dstack.gpus"].str(), ','))
        if (!g.empty()) t.gpus.push_back(atoi(g.c_str()));
      for (auto& rn : split(c["Labels"]["dstack.render_nodes"].str(), ','))
        if (!rn.empty()) t.render_nodes.push_back(rn);
      std::string state = c["State"].str();
      t.status = state == "running" ? TaskStatus::Running : TaskStatus::Terminated;
      // the runner port depends on the network mode (host: fixed; bridge: the published port)
      if (c["HostConfig"].has("NetworkMode")) t.config.network_mode = c["HostConfig"]["NetworkMode"].str();
      inspect_ports(t);
      out.push_back(t);
    }
    return out;
  }

 private:
  ShimOptions o_;
};

}  // namespace

std::unique_ptr<TaskDriver> make_docker_driver(const ShimOptions& o) {
  return std::unique_ptr<TaskDriver>(new DockerDriver(o));
}

}  // namespace dsa
