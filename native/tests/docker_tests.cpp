// DockerDriver against a fake Docker Engine API served on a unix socket (reference analogue:
// runner/internal/shim/docker_test.go, which needs a real daemon; this one pins the exact
// requests instead).  Also: GPU discovery order (sysfs fallback sorted by PCI BDF, independent of
// render-node numbering) on a fake /sys tree.
//
// Build + run: make -C native test   (or build/docker_tests directly)
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../common/amdgpu.h"
#include "../common/json.h"
#include "../common/net.h"
#include "../shim/shim.h"

using namespace dsa;

static int g_failed = 0, g_run = 0;
#define CHECK(cond)                                                      \
  do {                                                                   \
    if (!(cond)) {                                                       \
      fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failed;                                                        \
    }                                                                    \
  } while (0)

static void run(const char* name, const std::function<void()>& fn) {
  int before = g_failed;
  ++g_run;
  fn();
  fprintf(stderr, "%s %s\n", g_failed == before ? "ok  " : "FAIL", name);
}

// ---- fake Docker Engine -------------------------------------------------------------------------
struct Req {
  std::string method, target, body;
  std::map<std::string, std::string> headers;  // lower-case keys
};
struct Resp {
  int status = 200;
  std::string body;
  std::vector<std::string> chunks;  // non-empty: Transfer-Encoding: chunked, one chunk each
};

class FakeDocker {
 public:
  using Handler = std::function<Resp(const Req&)>;
  explicit FakeDocker(Handler h) : h_(std::move(h)) {
    char tmpl[] = "/tmp/fake-docker-XXXXXX";
    dir_ = mkdtemp(tmpl);
    path_ = dir_ + "/docker.sock";
    fd_ = ::socket(AF_UNIX, SOCK_STREAM, 0);
    struct sockaddr_un a{};
    a.sun_family = AF_UNIX;
    snprintf(a.sun_path, sizeof a.sun_path, "%s", path_.c_str());
    if (::bind(fd_, (struct sockaddr*)&a, sizeof a) != 0 || ::listen(fd_, 16) != 0) {
      fprintf(stderr, "fake docker: bind failed\n");
      exit(2);
    }
    th_ = std::thread([this] { loop(); });
  }
  ~FakeDocker() {
    stop_ = true;
    ::shutdown(fd_, SHUT_RDWR);
    ::close(fd_);
    th_.join();
    ::unlink(path_.c_str());
    ::rmdir(dir_.c_str());
  }
  const std::string& path() const { return path_; }
  std::vector<Req> requests() {
    std::lock_guard<std::mutex> lk(mu_);
    return reqs_;
  }
  Req last(const std::string& method, const std::string& prefix) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = reqs_.rbegin(); it != reqs_.rend(); ++it)
      if (it->method == method && it->target.rfind(prefix, 0) == 0) return *it;
    return Req{};
  }

 private:
  static bool read_line(int fd, std::string& buf, std::string& line) {
    while (true) {
      auto p = buf.find("\r\n");
      if (p != std::string::npos) {
        line = buf.substr(0, p);
        buf.erase(0, p + 2);
        return true;
      }
      char c[4096];
      ssize_t n = ::recv(fd, c, sizeof c, 0);
      if (n <= 0) return false;
      buf.append(c, (size_t)n);
    }
  }
  void serve(int c) {
    std::string buf, line;
    Req r;
    if (!read_line(c, buf, line)) return;
    auto s1 = line.find(' '), s2 = line.rfind(' ');
    r.method = line.substr(0, s1);
    r.target = line.substr(s1 + 1, s2 - s1 - 1);
    while (read_line(c, buf, line) && !line.empty()) {
      auto k = line.find(':');
      std::string key = line.substr(0, k);
      for (auto& ch : key) ch = (char)tolower((unsigned char)ch);
      r.headers[key] = trim(line.substr(k + 1));
    }
    size_t len = r.headers.count("content-length") ? (size_t)atol(r.headers["content-length"].c_str()) : 0;
    while (buf.size() < len) {
      char cb[4096];
      ssize_t n = ::recv(c, cb, sizeof cb, 0);
      if (n <= 0) break;
      buf.append(cb, (size_t)n);
    }
    r.body = buf.substr(0, len);
    {
      std::lock_guard<std::mutex> lk(mu_);
      reqs_.push_back(r);
    }
    Resp resp = h_(r);
    std::string out = "HTTP/1.1 " + std::to_string(resp.status) + " X\r\nContent-Type: application/json\r\n";
    if (!resp.chunks.empty()) {
      out += "Transfer-Encoding: chunked\r\n\r\n";
      char hex[32];
      for (auto& ch : resp.chunks) {
        snprintf(hex, sizeof hex, "%zx\r\n", ch.size());
        out += hex + ch + "\r\n";
      }
      out += "0\r\n\r\n";
    } else {
      out += "Content-Length: " + std::to_string(resp.body.size()) + "\r\n\r\n" + resp.body;
    }
    size_t off = 0;
    while (off < out.size()) {
      ssize_t w = ::send(c, out.data() + off, out.size() - off, MSG_NOSIGNAL);
      if (w <= 0) break;
      off += (size_t)w;
    }
  }
  void loop() {
    while (!stop_) {
      int c = ::accept(fd_, nullptr, nullptr);
      if (c < 0) continue;
      serve(c);
      ::close(c);
    }
  }
  Handler h_;
  std::string dir_, path_;
  int fd_ = -1;
  std::atomic<bool> stop_{false};
  std::thread th_;
  std::mutex mu_;
  std::vector<Req> reqs_;
};

static bool has_str(const Json& arr, const std::string& v) {
  for (auto& x : arr.items())
    if (x.is_string() && x.str() == v) return true;
  return false;
}

static std::string tmpdir() {
  char tmpl[] = "/tmp/docker-tests-XXXXXX";
  return mkdtemp(tmpl);
}

// a default engine: image absent (404 -> pull), pull ok, create -> Id, start ok, inspect -> ports
static Resp default_engine(const Req& r) {
  if (r.method == "GET" && r.target.rfind("/images/", 0) == 0) return Resp{404, R"({"message":"No such image"})", {}};
  if (r.method == "POST" && r.target.rfind("/images/create", 0) == 0)
    return Resp{200, "", {R"({"status":"Pulling from rocm/pytorch"})" "\n", R"({"status":"Download complete"})" "\n"}};
  if (r.method == "POST" && r.target.rfind("/containers/create", 0) == 0) return Resp{201, R"({"Id":"c0ffee"})", {}};
  if (r.method == "POST" && r.target == "/containers/c0ffee/start") return Resp{204, "", {}};
  if (r.method == "GET" && r.target == "/containers/c0ffee/json")
    return Resp{200, R"({"NetworkSettings":{"Ports":{"10999/tcp":[{"HostIp":"0.0.0.0","HostPort":"32768"}],)"
                     R"("10022/tcp":[{"HostPort":"32769"}],"8000/tcp":[{"HostPort":"32770"}]}}})", {}};
  return Resp{404, R"({"message":"unexpected"})", {}};
}

static Task gpu_task() {
  Task t;
  t.config.id = "task-1";
  t.config.name = "run-1-0-0";
  t.config.image_name = "rocm/pytorch:latest";
  t.config.network_mode = "bridge";
  t.config.shm_size = 8LL << 30;
  t.config.memory = 64LL << 30;
  t.config.cpu = 16;
  t.config.ports = {8000};
  t.config.registry_username = "u";
  t.config.registry_password = "p";
  t.config.container_ssh_keys = {"ssh-ed25519 AAAA key@test"};
  t.config.env["DSTACK_RUN_NAME"] = "run-1";
  t.gpus = {1, 3};
  t.render_nodes = {"/dev/dri/renderD136", "/dev/dri/renderD152"};
  return t;
}

int main() {
  set_log_level(0);

  run("docker create body: AMD devices, groups, binds, limits, bridge ports, labels", [] {
    FakeDocker fd(default_engine);
    std::string tmp = tmpdir();
    mkdirs(tmp + "/ib");
    mkdirs(tmp + "/models");
    ShimOptions o;
    o.docker_socket = fd.path();
    o.runner_binary = "/opt/dstack/dstack-runner";
    o.volumes_root = tmp + "/vols";
    o.infiniband_path = tmp + "/ib";
    auto drv = make_docker_driver(o);
    Task t = gpu_task();
    Json im = Json::object();
    im.set("instance_path", tmp + "/models");
    im.set("path", "/models");
    im.set("optional", false);
    t.config.instance_mounts.push_back(im);
    Json opt = Json::object();  // optional + missing on the host: skipped
    opt.set("instance_path", tmp + "/no-such-cache");
    opt.set("path", "/cache");
    opt.set("optional", true);
    t.config.instance_mounts.push_back(opt);
    Json vm = Json::object();
    vm.set("name", "ckpt");
    vm.set("path", "/checkpoints");
    t.config.volume_mounts.push_back(vm);
    std::string reason, msg;
    CHECK(drv->run(t, reason, msg));
    CHECK(t.container_id == "c0ffee");
    CHECK(t.runner_port == 32768);
    CHECK(t.ports.size() == 3);

    // the image was looked up, then pulled with the registry auth header
    Req pull = fd.last("POST", "/images/create");
    CHECK(pull.target == "/images/create?fromImage=rocm/pytorch&tag=latest");
    Json auth = Json::parse(base64_decode(pull.headers["x-registry-auth"]));
    CHECK(auth["username"].str() == "u" && auth["password"].str() == "p");

    Req cr = fd.last("POST", "/containers/create");
    CHECK(cr.target.rfind("/containers/create?name=run-1-0-0-", 0) == 0 &&
          cr.target.size() == std::string("/containers/create?name=run-1-0-0-").size() + 8);
    Json b = Json::parse(cr.body);
    CHECK(b["Image"].str() == "rocm/pytorch:latest");
    CHECK(b["Entrypoint"][(size_t)0].str() == "/bin/sh" && b["Entrypoint"][(size_t)1].str() == "-c");
    const std::string script = b["Cmd"][(size_t)0].str();
    CHECK(script.find("sshd") != std::string::npos && script.find("-p 10022") != std::string::npos);
    CHECK(script.find("exec /usr/local/bin/dstack-runner") != std::string::npos);
    CHECK(script.find("--http-port 10999") != std::string::npos);
    CHECK(script.find("ssh-ed25519 AAAA key@test") != std::string::npos);
    CHECK(has_str(b["Env"], "DSTACK_RUN_NAME=run-1"));
    CHECK(b["Labels"]["dstack.task_id"].str() == "task-1");
    CHECK(b["Labels"]["dstack.gpus"].str() == "1,3");
    CHECK(b["Labels"]["dstack.render_nodes"].str() == "/dev/dri/renderD136,/dev/dri/renderD152");
    const Json& hc = b["HostConfig"];
    // devices: /dev/kfd + ONLY the granted render nodes (+ RDMA), all rwm
    std::vector<std::string> devs;
    for (auto& d : hc["Devices"].items()) {
      devs.push_back(d["PathOnHost"].str());
      CHECK(d["PathInContainer"].str() == d["PathOnHost"].str() && d["CgroupPermissions"].str() == "rwm");
    }
    CHECK((devs == std::vector<std::string>{"/dev/kfd", "/dev/dri/renderD136", "/dev/dri/renderD152", tmp + "/ib"}));
    CHECK(has_str(hc["GroupAdd"], "video") && has_str(hc["GroupAdd"], "render"));
    CHECK(hc["IpcMode"].str() == "host");
    CHECK(has_str(hc["CapAdd"], "SYS_PTRACE") && has_str(hc["SecurityOpt"], "seccomp=unconfined"));
    CHECK(hc["ShmSize"].as_int() == (8LL << 30) && hc["Memory"].as_int() == (64LL << 30));
    CHECK(hc["NanoCpus"].as_int() == 16000000000LL);
    CHECK(hc["NetworkMode"].str() == "bridge" && !hc["Privileged"].as_bool());
    // memlock unlimited for RDMA
    CHECK(hc["Ulimits"][(size_t)0]["Name"].str() == "memlock" && hc["Ulimits"][(size_t)0]["Soft"].as_int() == -1);
    // binds: runner binary (ro), the instance mount, the network volume; the missing optional one skipped
    CHECK(has_str(hc["Binds"], "/opt/dstack/dstack-runner:/usr/local/bin/dstack-runner:ro"));
    CHECK(has_str(hc["Binds"], tmp + "/models:/models"));
    CHECK(has_str(hc["Binds"], tmp + "/vols/ckpt:/checkpoints"));
    CHECK(hc["Binds"].size() == 3);
    // bridge mode publishes runner HTTP + SSH and the app port on ephemeral host ports
    for (const char* p : {"10999/tcp", "10022/tcp", "8000/tcp"}) {
      CHECK(hc["PortBindings"].has(p) && hc["PortBindings"][p][(size_t)0]["HostPort"].str().empty());
      CHECK(b["ExposedPorts"].has(p));
    }
    run_capture({"rm", "-rf", "--", tmp}, msg);
  });

  run("docker host network, no GPU, no RDMA: no devices, runner on its fixed port", [] {
    FakeDocker fd([](const Req& r) {
      if (r.method == "GET" && r.target.rfind("/images/", 0) == 0) return Resp{200, R"({"Id":"sha256:1"})", {}};
      return default_engine(r);
    });
    ShimOptions o;
    o.docker_socket = fd.path();
    o.runner_binary = "/r";
    o.infiniband_path = "/nonexistent/infiniband";
    auto drv = make_docker_driver(o);
    Task t;
    t.config.id = "cpu";
    t.config.image_name = "ubuntu:22.04";
    std::string reason, msg;
    CHECK(drv->run(t, reason, msg));
    for (auto& r : fd.requests()) CHECK(r.target.rfind("/images/create", 0) != 0);  // present: no pull
    Json hc = Json::parse(fd.last("POST", "/containers/create").body)["HostConfig"];
    CHECK(hc["Devices"].size() == 0 && !hc.has("GroupAdd") && !hc.has("Ulimits") && !hc.has("PortBindings"));
    CHECK(hc["NetworkMode"].str() == "host");
    CHECK(t.runner_port == 10999);
  });

  run("docker pull stream error mid-stream fails the task", [] {
    FakeDocker fd([](const Req& r) {
      if (r.method == "POST" && r.target.rfind("/images/create", 0) == 0)
        return Resp{200, "", {R"({"status":"Pulling fs layer"})" "\n",
                              R"({"errorDetail":{"message":"unauthorized"},"error":"pull access denied for x"})" "\n"}};
      return default_engine(r);
    });
    ShimOptions o;
    o.docker_socket = fd.path();
    auto drv = make_docker_driver(o);
    Task t = gpu_task();
    std::string reason, msg;
    CHECK(!drv->run(t, reason, msg));
    CHECK(reason == "creating_container_error");
    CHECK(msg.find("pull access denied for x") != std::string::npos);
    for (auto& r : fd.requests()) CHECK(r.target.rfind("/containers/create", 0) != 0);
  });

  run("docker start failure fails the task", [] {
    FakeDocker fd([](const Req& r) {
      if (r.method == "POST" && r.target == "/containers/c0ffee/start")
        return Resp{500, R"({"message":"error gathering device information while adding custom device \"/dev/kfd\""})", {}};
      return default_engine(r);
    });
    ShimOptions o;
    o.docker_socket = fd.path();
    auto drv = make_docker_driver(o);
    Task t = gpu_task();
    std::string reason, msg;
    CHECK(!drv->run(t, reason, msg));
    CHECK(reason == "creating_container_error" && msg.find("start failed") != std::string::npos);
    CHECK(msg.find("/dev/kfd") != std::string::npos);
  });

  run("container bootstrap script runs: keys (quotes included), sshd flags, runner exec", [] {
    ShimOptions o;
    o.runner_ssh_port = 10022;
    o.runner_http_port = 10999;
    std::string script = container_bootstrap_script(o, {"ssh-ed25519 AAAAkey1 alice's laptop", "ssh-rsa AAAAkey2"});
    char tmpl[] = "/tmp/dsa_boot_XXXXXX";
    std::string dir = mkdtemp(tmpl);
    std::string bin = dir + "/bin", home = dir + "/home", log = dir + "/calls.log";
    mkdirs(bin);
    mkdirs(home);
    // stand-ins: sshd / ssh-keygen record their argv; the runner path and /run/sshd are redirected
    auto stub = [&](const std::string& name) {
      write_file(bin + "/" + name, "#!/bin/sh\necho \"" + name + " $*\" >> " + log + "\n", 0755);
    };
    stub("sshd");
    stub("ssh-keygen");
    stub("dstack-runner");
    auto replace_all = [](std::string s, const std::string& a, const std::string& b) {
      for (size_t p = s.find(a); p != std::string::npos; p = s.find(a, p + b.size())) s.replace(p, a.size(), b);
      return s;
    };
    script = replace_all(script, "/usr/local/bin/dstack-runner", bin + "/dstack-runner");
    script = replace_all(script, "/run/sshd", dir + "/run-sshd");
    write_file(dir + "/boot.sh", script, 0755);
    std::string cmd = "env -i HOME=" + home + " PATH=" + bin + ":/usr/bin:/bin sh " + dir + "/boot.sh 2>&1";
    FILE* f = popen(cmd.c_str(), "r");
    char buf[512];
    std::string out;
    while (f && fgets(buf, sizeof buf, f)) out += buf;
    int rc = f ? pclose(f) : -1;
    CHECK(rc == 0);
    std::string keys, calls;
    read_file(home + "/.ssh/authorized_keys", keys);
    for (int i = 0; i < 100; ++i) {  // sshd starts in the background, after the runner's exec
      read_file(log, calls);
      if (calls.find("sshd -p") != std::string::npos) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    CHECK(keys == "ssh-ed25519 AAAAkey1 alice's laptop\nssh-rsa AAAAkey2\n");
    CHECK(calls.find("ssh-keygen -A") != std::string::npos);
    CHECK(calls.find("sshd -p 10022 -o PermitUserEnvironment=yes -o PasswordAuthentication=no") != std::string::npos);
    CHECK(calls.find("dstack-runner --log-level") != std::string::npos);
    CHECK(calls.find("start --http-port 10999 --temp-dir /tmp/runner --home-dir " + home) != std::string::npos);
    if (rc != 0) fprintf(stderr, "%s\n%s\n", script.c_str(), out.c_str());
  });

  run("container bootstrap: the runner starts before a missing sshd is installed", [] {
    // an image without sshd: the stand-in package manager takes 1.5 s and then provides sshd; the
    // runner must have been exec'd long before that, and sshd must still come up afterwards
    ShimOptions o;
    o.runner_ssh_port = 10022;
    o.runner_http_port = 10999;
    std::string script = container_bootstrap_script(o, {"ssh-ed25519 AAAAkey1"});
    char tmpl[] = "/tmp/dsa_boot2_XXXXXX";
    std::string dir = mkdtemp(tmpl);
    std::string bin = dir + "/bin", home = dir + "/home", log = dir + "/calls.log";
    mkdirs(bin);
    mkdirs(home);
    auto stamp = [&](const std::string& name) {
      return "echo \"" + name + " $(date +%s%N)\" >> " + log + "\n";
    };
    write_file(bin + "/apt-get",
               "#!/bin/sh\n" + stamp("apt-get-start") + "[ \"$1\" = update ] && exit 0\nsleep 1.5\n" +
                   "cat > " + bin + "/sshd <<'EOS'\n#!/bin/sh\n" + stamp("sshd") + "EOS\nchmod +x " + bin + "/sshd\n" +
                   stamp("apt-get-done"),
               0755);
    write_file(bin + "/ssh-keygen", "#!/bin/sh\nexit 0\n", 0755);
    write_file(bin + "/dstack-runner", "#!/bin/sh\n" + stamp("runner"), 0755);
    auto replace_all = [](std::string s, const std::string& a, const std::string& b) {
      for (size_t p = s.find(a); p != std::string::npos; p = s.find(a, p + b.size())) s.replace(p, a.size(), b);
      return s;
    };
    script = replace_all(script, "/usr/local/bin/dstack-runner", bin + "/dstack-runner");
    script = replace_all(script, "/run/sshd", dir + "/run-sshd");
    write_file(dir + "/boot.sh", script, 0755);
    std::string out;
    int rc = run_capture({"env", "-i", "HOME=" + home, "PATH=" + bin + ":/usr/bin:/bin", "sh", dir + "/boot.sh"}, out);
    CHECK(rc == 0);
    std::string calls;
    for (int i = 0; i < 100; ++i) {  // the background install finishes after the runner
      read_file(log, calls);
      if (calls.find("sshd ") != std::string::npos) break;
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    auto at = [&](const std::string& name) {
      size_t p = calls.find(name + " ");
      return p == std::string::npos ? -1LL : std::stoll(calls.substr(p + name.size() + 1, 19));
    };
    CHECK(at("runner") > 0 && at("apt-get-done") > 0 && at("sshd") > 0);
    CHECK(at("runner") < at("apt-get-done"));  // the job did not wait for the package install
    CHECK(at("apt-get-done") - at("runner") > 1000000000LL);
    CHECK(at("sshd") >= at("apt-get-done"));
    run_capture({"rm", "-rf", "--", dir}, out);
  });

  run("docker restore rebuilds tasks and the GPU lock from labels", [] {
    FakeDocker fd([](const Req& r) {
      if (r.method == "GET" && r.target.rfind("/containers/json", 0) == 0) {
        CHECK(r.target.find("all=1") != std::string::npos && r.target.find("dstack.task_id") != std::string::npos);
        return Resp{200, R"([{"Id":"c0ffee","Names":["/run-a"],"State":"running","HostConfig":{"NetworkMode":"bridge"},)"
                         R"("Labels":{"dstack.task_id":"ta","dstack.gpus":"0,1","dstack.render_nodes":"/dev/dri/renderD128,/dev/dri/renderD136"}},)"
                         R"({"Id":"dead","Names":["/run-b"],"State":"exited","Labels":{"dstack.task_id":"tb","dstack.gpus":""}}])",
                    {}};
      }
      if (r.method == "GET" && r.target == "/containers/dead/json") return Resp{200, R"({"NetworkSettings":{"Ports":{}}})", {}};
      return default_engine(r);
    });
    ShimOptions o;
    o.docker_socket = fd.path();
    auto drv = make_docker_driver(o);
    auto tasks = drv->restore();
    CHECK(tasks.size() == 2);
    if (tasks.size() == 2) {
      CHECK(tasks[0].config.id == "ta" && tasks[0].status == TaskStatus::Running);
      CHECK((tasks[0].gpus == std::vector<int>{0, 1}));
      CHECK((tasks[0].render_nodes == std::vector<std::string>{"/dev/dri/renderD128", "/dev/dri/renderD136"}));
      CHECK(tasks[0].runner_port == 32768 && tasks[0].container_name == "/run-a");
      CHECK(tasks[1].config.id == "tb" && tasks[1].status == TaskStatus::Terminated && tasks[1].gpus.empty());
      GpuLock lock;
      lock.init(4, {}, {});
      CHECK(lock.lock(tasks[0].gpus) && lock.free_count() == 2);
      CHECK(!lock.lock({1}));  // a restored grant is really held
    }
  });

  run("docker terminate / remove call stop and force-delete", [] {
    FakeDocker fd([](const Req& r) {
      if (r.method == "POST" && r.target.rfind("/containers/c0ffee/stop", 0) == 0) return Resp{204, "", {}};
      if (r.method == "DELETE") return Resp{204, "", {}};
      return default_engine(r);
    });
    ShimOptions o;
    o.docker_socket = fd.path();
    o.volumes_root = "/nonexistent-volumes-root";
    auto drv = make_docker_driver(o);
    Task t;
    t.container_id = "c0ffee";
    drv->terminate(t, 7);
    drv->remove(t);
    CHECK(fd.last("POST", "/containers/c0ffee/stop").target == "/containers/c0ffee/stop?t=7");
    CHECK(fd.last("DELETE", "/containers/c0ffee").target == "/containers/c0ffee?force=1&v=1");
  });

  run("GPU order: sysfs discovery sorted by PCI BDF, not by render-node number", [] {
    // renderD128 sits on the highest bus and renderD129 on the lowest: the index (== GPU-lock index,
    // == xGMI matrix row on the amdsmi path, which sorts by BDF too) must follow the bus
    std::string root = tmpdir();
    struct G {
      int render;
      const char* bdf;
      const char* numa;
    };
    const G gs[] = {{128, "0000:f5:00.0", "1"}, {129, "0000:05:00.0", "0"}, {130, "0000:75:00.0", "0"}};
    mkdirs(root + "/sys/class/drm");
    mkdirs(root + "/devices");
    mkdirs(root + "/dev/dri");
    for (auto& g : gs) {
      std::string dev = root + "/devices/" + g.bdf;
      mkdirs(dev);
      write_file(dev + "/vendor", "0x1002\n");
      write_file(dev + "/product_name", "AMD Instinct MI355X\n");
      write_file(dev + "/mem_info_vram_total", std::to_string(288ULL << 30) + "\n");
      write_file(dev + "/numa_node", std::string(g.numa) + "\n");
      mkdirs(root + "/sys/class/drm/renderD" + std::to_string(g.render));
      write_file(root + "/dev/dri/renderD" + std::to_string(g.render), "");
      CHECK(symlink(dev.c_str(), (root + "/sys/class/drm/renderD" + std::to_string(g.render) + "/device").c_str()) == 0);
    }
    // a fourth GPU on the host that this process cannot open (not in its container): not listed
    {
      std::string dev = root + "/devices/0000:02:00.0";
      mkdirs(dev);
      write_file(dev + "/vendor", "0x1002\n");
      mkdirs(root + "/sys/class/drm/renderD200");
      CHECK(symlink(dev.c_str(), (root + "/sys/class/drm/renderD200/device").c_str()) == 0);
    }
    setenv("DSTACK_SYSFS_ROOT", root.c_str(), 1);
    auto gpus = discover_amd_gpus_sysfs();
    unsetenv("DSTACK_SYSFS_ROOT");
    CHECK(gpus.size() == 3);
    if (gpus.size() == 3) {
      CHECK(gpus[0].bdf == "0000:05:00.0" && gpus[0].render_node == "/dev/dri/renderD129" && gpus[0].index == 0);
      CHECK(gpus[1].bdf == "0000:75:00.0" && gpus[1].render_node == "/dev/dri/renderD130");
      CHECK(gpus[2].bdf == "0000:f5:00.0" && gpus[2].render_node == "/dev/dri/renderD128" && gpus[2].numa_node == 1);
      CHECK(gpus[0].name == "MI355X" && gpus[0].vram_mib == (288ULL << 10));
    }
    std::string out;
    run_capture({"rm", "-rf", "--", root}, out);
  });

  fprintf(stderr, "%d/%d test groups passed\n", g_run - (g_failed ? 1 : 0), g_run);
  return g_failed ? 1 : 0;
}
