// dstack-runner executor: the in-container job state machine.
// Reference behaviour: runner/internal/executor/{executor.go,states.go,logs.go,timestamp.go,
// query.go,repo.go,env.go} — re-designed in C++ for the MI355X build.
#pragma once
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../common/json.h"

namespace dsa {

// RDMA devices with an ACTIVE port (NCCL_IB_HCA for multi-node jobs); DSTACK_SYSFS_ROOT for tests
std::vector<std::string> active_rdma_devices();

// executor states (states.go:3-9)
enum class ExecState { WaitSubmit, WaitCode, WaitRun, ServeLogs, WaitLogsFinished };
const char* exec_state_name(ExecState s);

struct LogEvent {
  int64_t timestamp;  // unique, strictly increasing ms (surrogate counter inside one ms)
  std::string message;
};

// append-only history with binary-searchable timestamps (logs.go + query.go)
class LogHistory {
 public:
  void append(const std::string& msg);
  std::vector<LogEvent> after(int64_t ts, size_t limit = 10000) const;
  int64_t last_timestamp() const;
  size_t size() const;
  // block until an event newer than `ts` exists or `timeout_ms` passes
  bool wait_after(int64_t ts, int timeout_ms) const;

 private:
  mutable std::mutex mu_;
  mutable std::condition_variable cv_;
  std::vector<LogEvent> events_;
  int64_t last_ = 0;
};

struct JobStateEvent {
  std::string state;  // running | done | failed | terminated
  int64_t timestamp;
  std::string termination_reason;
  std::string termination_message;
  int exit_status = -1;
};

struct RunnerOptions {
  std::string temp_dir = "/tmp/runner";
  std::string home_dir = "/root";
  std::string working_dir = "/workflow";
  bool write_ssh_env = false;
  std::string probe_binary;  // dstack-probe (HIP health probes), optional
};

class Executor {
 public:
  std::atomic<int>* child_pgid_ptr() { return &child_pgid_; }
  explicit Executor(RunnerOptions opts);
  ~Executor();

  ExecState state() const { return state_; }
  // handlers (return "" on success or an error message)
  std::string submit(const Json& body);
  std::string upload_code(const std::string& blob);
  std::string run();
  void stop();

  Json pull(int64_t since) const;
  const LogHistory& job_logs() const { return job_logs_; }
  const LogHistory& runner_logs() const { return runner_logs_; }
  bool finished() const { return finished_; }
  bool logs_consumed_after_finish() const { return pulled_after_finish_; }
  void mark_pulled(int64_t ts) const;
  void wait_finished();

  // exported for tests: the environment built for a job
  std::vector<std::pair<std::string, std::string>> build_env() const;

 private:
  void run_thread();
  void run_job_steps();
  std::string setup_credentials(int uid, int gid, std::string& err);
  void add_state(const std::string& state, const std::string& reason = "", const std::string& msg = "",
                 int exit_status = -1);
  void rlog(const char* fmt, ...) __attribute__((format(printf, 2, 3)));
  bool setup_repo(std::string& err);
  bool run_probe();
  bool wants_rccl_preflight() const;
  bool preflight_concurrent() const;
  bool run_rccl_preflight(std::string& msg);
  void stop_preflight();
  int exec_job(std::string& reason, std::string& msg);

  RunnerOptions opts_;
  std::atomic<ExecState> state_{ExecState::WaitSubmit};
  Json submit_body_;
  std::string code_path_;
  LogHistory job_logs_, runner_logs_;
  mutable std::mutex states_mu_;
  std::vector<JobStateEvent> states_;
  std::thread worker_;
  std::atomic<bool> finished_{false};
  std::atomic<bool> stop_requested_{false};
  std::atomic<int> child_pgid_{0};
  std::string probe_json_;  // last dstack-probe result (JSON), guarded by states_mu_
  std::string preflight_json_;  // last RCCL pre-flight document
  // concurrent pre-flight (DSTACK_RCCL_PREFLIGHT_MODE=concurrent, the default): 0 none, 1 running,
  // 2 passed, 3 failed (the job is stopped with preflight_err_, guarded by states_mu_)
  std::atomic<int> preflight_state_{0};
  std::atomic<int> preflight_pgid_{0};  // the running probe's process group (0: none)
  std::string preflight_err_;
  mutable std::atomic<bool> pulled_after_finish_{false};
  std::mutex fin_mu_;
  std::condition_variable fin_cv_;
};

bool join_rel_path(const std::string& base, const std::string& rel, std::string& out, std::string& err);

// ${VAR} interpolation with $$ escape (env.go:60-134)
std::string interpolate_env(const std::string& s, const std::vector<std::pair<std::string, std::string>>& env,
                            std::string* err);

}  // namespace dsa
