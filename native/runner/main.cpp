// dstack-runner: in-container agent.  HTTP API on :10999 (reference: runner/internal/runner/api/
// server.go:37-134, http.go:19-124, ws.go:18-62; CLI: runner/cmd/runner/cmd.go:13-75).
//
//   dstack-runner [--log-level N] start --http-port 10999 --temp-dir /tmp/runner
//                 --home-dir /root --working-dir /workflow [--ssh-env] [--probe PATH]
//                 [--port-file PATH]
//
// --http-port 0 binds an ephemeral port; --port-file then receives the bound port (written to a
// temp file and renamed, so a reader never sees a partial number).  The process shim driver uses
// this instead of probing for a free port first, which races with every other bind on the host.
//
// Lifecycle: wait <= 5 min for /api/submit, run the job, then keep serving until the job's logs
// were pulled after completion (or 30 s), then exit.
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <thread>

#include "../common/net.h"
#include "executor.h"

namespace dsa {
Json collect_metrics(const std::vector<int>& gpu_filter);
}

using namespace dsa;

static const char* VERSION = "0.1.0+mi355x";

static void usage() {
  fprintf(stderr,
          "usage: dstack-runner [--log-level N] start [--http-port P] [--temp-dir D] [--home-dir D]\n"
          "                     [--working-dir D] [--ssh-env] [--probe PATH] [--submit-timeout S]\n"
          "                     [--port-file PATH]\n");
}

int main(int argc, char** argv) {
  int http_port = 10999;
  int submit_timeout_s = 300;
  RunnerOptions opts;
  bool start = false;
  std::string port_file;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&](const char* name) -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "missing value for %s\n", name);
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--log-level") set_log_level(atoi(next("--log-level").c_str()));
    else if (a == "start") start = true;
    else if (a == "--http-port") http_port = atoi(next("--http-port").c_str());
    else if (a == "--temp-dir") opts.temp_dir = next("--temp-dir");
    else if (a == "--home-dir") opts.home_dir = next("--home-dir");
    else if (a == "--working-dir") opts.working_dir = next("--working-dir");
    else if (a == "--ssh-env") opts.write_ssh_env = true;
    else if (a == "--probe") opts.probe_binary = next("--probe");
    else if (a == "--port-file") port_file = next("--port-file");
    else if (a == "--submit-timeout") submit_timeout_s = atoi(next("--submit-timeout").c_str());
    else if (a == "--version") {
      printf("%s\n", VERSION);
      return 0;
    } else {
      usage();
      return 2;
    }
  }
  if (!start) {
    usage();
    return 2;
  }
  signal(SIGPIPE, SIG_IGN);
  Executor ex(opts);
  // the job runs in its own session: forward termination to its process group
  static std::atomic<int>* g_job_pgid = nullptr;
  g_job_pgid = ex.child_pgid_ptr();
  struct sigaction sa{};
  sa.sa_handler = [](int sig) {
    int pg = g_job_pgid ? g_job_pgid->load() : 0;
    if (pg > 0) kill(-pg, SIGKILL);
    _exit(128 + sig);
  };
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  HttpServer srv("0.0.0.0", http_port);
  std::atomic<bool> stop_server{false};

  srv.route("GET", "/api/healthcheck", [&](HttpRequest&) {
    Json j = Json::object();
    j.set("service", "dstack-runner");
    j.set("version", VERSION);
    j.set("state", exec_state_name(ex.state()));
    return HttpResponse::json(j);
  });
  srv.route("GET", "/api/metrics", [&](HttpRequest&) { return HttpResponse::json(collect_metrics({})); });
  srv.route("POST", "/api/submit", [&](HttpRequest& r) {
    Json body;
    try {
      body = r.json();
    } catch (const std::exception& e) {
      return HttpResponse::error(400, e.what());
    }
    std::string err = ex.submit(body);
    return err.empty() ? HttpResponse::json(Json::object()) : HttpResponse::error(409, err);
  });
  srv.route("POST", "/api/upload_code", [&](HttpRequest& r) {
    std::string err = ex.upload_code(r.body);
    return err.empty() ? HttpResponse::json(Json::object()) : HttpResponse::error(409, err);
  });
  srv.route("POST", "/api/run", [&](HttpRequest&) {
    std::string err = ex.run();
    return err.empty() ? HttpResponse::json(Json::object()) : HttpResponse::error(409, err);
  });
  srv.route("GET", "/api/pull", [&](HttpRequest& r) {
    int64_t ts = atoll(r.q("timestamp", "0").c_str());
    // optional long-poll: ?wait_ms=N returns as soon as anything newer than ts exists
    int wait_ms = std::min(atoi(r.q("wait_ms", "0").c_str()), 30000);
    if (wait_ms > 0 && !ex.finished()) ex.job_logs().wait_after(ts, wait_ms);
    Json out = ex.pull(ts);
    ex.mark_pulled(ts);
    return HttpResponse::json(out);
  });
  srv.route("POST", "/api/stop", [&](HttpRequest&) {
    ex.stop();
    return HttpResponse::json(Json::object());
  });
  srv.websocket("/logs_ws", [&](HttpRequest&, WsConn& ws) {
    int64_t ts = 0;
    while (!ws.closed()) {
      auto evs = ex.job_logs().after(ts, 1000);
      for (auto& e : evs) {
        if (!ws.send_binary(e.message)) return;
        ts = e.timestamp;
      }
      if (evs.empty()) {
        if (ex.finished() && ex.job_logs().last_timestamp() <= ts) break;
        ex.job_logs().wait_after(ts, 100);
        if (!ws.poll_peer(0)) return;
      }
    }
    ws.close(1000);
  });

  if (srv.start() < 0) {
    LOGE("cannot listen on port %d", http_port);
    return 1;
  }
  LOGI("dstack-runner %s listening on :%d", VERSION, srv.port());
  if (!port_file.empty()) {
    std::string tmp = port_file + ".tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    if (!f || fprintf(f, "%d\n", srv.port()) < 0 || fclose(f) != 0 || rename(tmp.c_str(), port_file.c_str()) != 0) {
      LOGE("cannot write the port file %s", port_file.c_str());
      return 1;
    }
  }
  std::thread server_thread([&] { srv.serve_forever(); });

  // lifecycle supervisor
  int64_t t0 = now_millis();
  while (ex.state() == ExecState::WaitSubmit || ex.state() == ExecState::WaitCode || ex.state() == ExecState::WaitRun) {
    if (ex.state() == ExecState::WaitSubmit && now_millis() - t0 > submit_timeout_s * 1000LL) {
      LOGW("no job submitted within %d s, exiting", submit_timeout_s);
      srv.stop();
      server_thread.join();
      return 0;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
  ex.wait_finished();
  int64_t tf = now_millis();
  while (!ex.logs_consumed_after_finish() && now_millis() - tf < 30000)
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  std::this_thread::sleep_for(std::chrono::milliseconds(200));  // let the final pull response flush
  LOGI("job finished and logs served; exiting");
  srv.stop();
  server_thread.join();
  return 0;
}
