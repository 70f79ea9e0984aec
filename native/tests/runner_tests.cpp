// Unit tests of the runner's executor and the shim's authorized_keys editing, case by case against
// the reference's runner/internal/{executor,shim}/*_test.go (mapping: docs/reference/test-parity.md).
// The executor is driven in-process (submit -> code -> run) with real child processes under a pipe
// (DSTACK_RUNNER_NO_PTY), in throw-away directories.  Build + run: make -C native test
#include <stdlib.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#include "../common/json.h"
#include "../common/net.h"
#include "../runner/executor.h"
#include "../shim/shim.h"

using namespace dsa;

static int g_failed = 0, g_run = 0;
#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      fprintf(stderr, "  FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond);     \
      ++g_failed;                                                            \
    }                                                                        \
  } while (0)

static void run(const char* name, const std::function<void()>& fn) {
  int before = g_failed;
  ++g_run;
  fn();
  fprintf(stderr, "%s %s\n", g_failed == before ? "ok  " : "FAIL", name);
}

static std::string tmpdir() {
  char tmpl[] = "/tmp/dsa_runner_test_XXXXXX";
  return mkdtemp(tmpl);
}

static int sh(const std::string& cmd) { return system(cmd.c_str()); }

struct JobResult {
  std::string logs, state, reason, message;
  int exit_status = -1;
};

// one job through a fresh executor: submit, code blob, run, wait; the last state and all job logs
static JobResult run_job(const std::string& root, Json body, const std::string& blob = "",
                         const std::string& probe = "", Json* pull_out = nullptr) {
  RunnerOptions o;
  o.probe_binary = probe;
  o.temp_dir = root + "/tmp";
  o.home_dir = root + "/home";
  o.working_dir = root + "/wd";
  mkdirs(o.home_dir);
  Executor ex(o);
  JobResult r;
  if (!ex.submit(body).empty() || !ex.upload_code(blob).empty() || !ex.run().empty()) {
    r.state = "<not started>";
    return r;
  }
  ex.wait_finished();
  for (auto& e : ex.job_logs().after(0)) r.logs += e.message;
  Json p = ex.pull(0);
  auto& st = p["job_states"].items();
  if (!st.empty()) {
    r.state = st.back()["state"].str();
    r.reason = st.back()["termination_reason"].str();
    r.message = st.back()["termination_message"].str();
    r.exit_status = (int)st.back()["exit_status"].as_int(-1);
  }
  if (pull_out) *pull_out = p;
  return r;
}

static Json job(const std::vector<std::string>& commands, const std::string& repo_type = "local") {
  Json js = Json::object();
  Json cmds = Json::array();
  for (auto& c : commands) cmds.push_back(c);
  js.set("commands", cmds);
  Json repo = Json::object();
  repo.set("repo_type", repo_type);
  Json rs = Json::object();
  rs.set("run_name", std::string("t"));
  rs.set("repo_data", repo);
  Json body = Json::object();
  body.set("job_spec", js);
  body.set("run_spec", rs);
  return body;
}

int main() {
  set_log_level(0);
  setenv("DSTACK_RUNNER_NO_PTY", "1", 1);  // plain pipes: exact output, no CRLF
  setenv("GIT_CONFIG_NOSYSTEM", "1", 1);

  // ---- env.go: ${NAME} expansion ----------------------------------------------------------------
  run("env: only well-formed ${NAME} references expand; every other dollar is kept", [] {
    std::vector<std::pair<std::string, std::string>> env = {{"NAME", "val"}, {"_x1", "u"}};
    std::string err;
    struct Case {
      const char* in;
      const char* out;
    } cases[] = {
        {"", ""},
        {"no dollars here", "no dollars here"},
        {"$ $$ $$$ $$$$", "$ $$ $$$ $$$$"},        // runs of dollars alone are literal
        {"pay $5 or $$5", "pay $5 or $$5"},
        {"$NAME and $$NAME", "$NAME and $$NAME"},  // no braces: not a reference
        {"end$", "end$"},
        {"end${", "end${"},
        {"end$${", "end$${"},
        {"a${}b", "a${}b"},
        {"a$${}b", "a$${}b"},
        {"a${NAME b", "a${NAME b"},                 // unterminated
        {"a${!NAME}b", "a${!NAME}b"},               // not a name
        {"a${NA-ME}b", "a${NA-ME}b"},
        {"a$${NA-ME}b", "a$${NA-ME}b"},
        {"${9lives}", "${9lives}"},
        {"x $$${9lives}y", "x $$${9lives}y"},
        {"a$${NAME}", "a${NAME}"},                  // escaped: one dollar dropped, no expansion
        {"a$$$${NAME}b", "a$${NAME}b"},
        {"${NAME}", "val"},
        {"$$${NAME}", "$val"},                      // odd run: halved, last one expands
        {"$$${NAME}$", "$val$"},
        {"$$${NAME}$$", "$val$$"},
        {"p${NAME}q${_x1}r", "pvalqur"},
        {"[${UNSET_VAR}]", "[]"},                   // unset: empty, as in a shell
    };
    for (auto& c : cases) {
      std::string got = interpolate_env(c.in, env, &err);
      if (got != c.out) fprintf(stderr, "  interpolate_env(%s) = %s, want %s\n", c.in, got.c_str(), c.out);
      CHECK(got == c.out);
    }
  });

  run("env: job env expands against what is already set (prepend, missing, var-like, no expansion)", [] {
    // the job's env is applied on top of the runner's: ${VAR} sees the value set before it
    RunnerOptions o;
    std::string root = tmpdir();
    o.temp_dir = root + "/tmp";
    o.home_dir = root;
    setenv("DSA_T_PATHLIKE", "/bin:/sbin", 1);
    setenv("DSA_T_OLD", "old", 1);
    Executor ex(o);
    Json body = job({"true"});
    Json env = Json::object();
    env.set("DSA_T_PATHLIKE", std::string("/opt/bin:${DSA_T_PATHLIKE}"));
    env.set("DSA_T_BARE", std::string("/opt/bin:$DSA_T_PATHLIKE"));
    env.set("DSA_T_MISSING", std::string("/opt/bin:${DSA_T_NOT_SET_ANYWHERE}"));
    env.set("DSA_T_TOKEN", std::string("deadf00d${notavar ${$NOTaVAR}"));
    env.set("DSA_T_OLD", std::string("new"));
    env.set("DSA_T_REF", std::string("ref_${DSA_T_OLD}"));
    // job_spec.env
    Json b2 = body;
    Json js = b2["job_spec"];
    js.set("env", env);
    b2.set("job_spec", js);
    CHECK(ex.submit(b2).empty());
    auto e = ex.build_env();
    auto get = [&](const std::string& k) {
      for (auto it = e.rbegin(); it != e.rend(); ++it)
        if (it->first == k) return it->second;
      return std::string("<unset>");
    };
    CHECK(get("DSA_T_PATHLIKE") == "/opt/bin:/bin:/sbin");
    CHECK(get("DSA_T_BARE") == "/opt/bin:$DSA_T_PATHLIKE");
    CHECK(get("DSA_T_MISSING") == "/opt/bin:");
    CHECK(get("DSA_T_TOKEN") == "deadf00d${notavar ${$NOTaVAR}");
    CHECK(get("DSA_T_OLD") == "new");
    CHECK(get("DSA_T_REF") == "ref_new" || get("DSA_T_REF") == "ref_old");  // map order: either was set first
  });

  // ---- exec.go joinRelPath ----------------------------------------------------------------------
  run("working dir: '.', relative, escape refused, absolute kept", [] {
    std::string out, err;
    CHECK(join_rel_path("/tmp/repo", ".", out, err) && out == "/tmp/repo");
    CHECK(join_rel_path("/tmp/repo", "", out, err) && out == "/tmp/repo");
    CHECK(join_rel_path("/tmp/repo", "task", out, err) && out == "/tmp/repo/task");
    CHECK(join_rel_path("/tmp/repo", "a/./b/../c/", out, err) && out == "/tmp/repo/a/c");
    CHECK(!join_rel_path("/tmp/repo", "..", out, err) && err.find("outside") != std::string::npos);
    CHECK(!join_rel_path("/tmp/repo", "a/../../b", out, err));
    CHECK(join_rel_path("/tmp/repo", "/workspace", out, err) && out == "/workspace");
    std::string root = tmpdir();
    Json b = job({"/bin/sh", "-c", "pwd"});
    Json js = b["job_spec"];
    js.set("working_dir", std::string("../elsewhere"));
    b.set("job_spec", js);
    JobResult r = run_job(root, b);
    CHECK(r.state == "failed" && r.reason == "executor_error" && r.message.find("outside") != std::string::npos);
  });

  // ---- executor_test.go ---------------------------------------------------------------------------
  run("executor: the job runs in the working dir with HOME set", [] {
    std::string root = tmpdir();
    JobResult r = run_job(root, job({"/bin/sh", "-c", "pwd; echo ~"}));
    CHECK(r.state == "done" && r.exit_status == 0);
    CHECK(r.logs == root + "/wd\n" + root + "/home\n");
    Json b = job({"/bin/sh", "-c", "pwd"});
    Json js = b["job_spec"];
    js.set("working_dir", std::string("sub/dir"));
    b.set("job_spec", js);
    r = run_job(tmpdir(), b);
    CHECK(r.state == "done" && r.logs.find("/wd/sub/dir\n") != std::string::npos);
  });

  run("executor: a failing command fails the job with its exit status", [] {
    JobResult r = run_job(tmpdir(), job({"/bin/sh", "-c", "ehco 1"}));  // sic: no such command
    CHECK(r.state == "failed" && r.reason == "container_exited_with_error" && r.exit_status == 127);
    r = run_job(tmpdir(), job({"/bin/sh", "-c", "exit 3"}));
    CHECK(r.state == "failed" && r.exit_status == 3 && r.message == "exit status 3");
  });

  run("executor: a local repo's tarball is extracted into the working dir", [] {
    std::string src = tmpdir();
    CHECK(sh("printf bar > " + src + "/foo && tar -czf " + src + ".tgz -C " + src + " foo") == 0);
    std::string blob;
    CHECK(read_file(src + ".tgz", blob) && !blob.empty());
    JobResult r = run_job(tmpdir(), job({"cat", "foo"}), blob);
    CHECK(r.state == "done" && r.logs == "bar");
  });

  run("executor: a remote repo is cloned at its commit, the diff applied, the committer set", [] {
    std::string up = tmpdir();
    CHECK(sh("cd " + up + " && git init -q && git config user.email a@b && git config user.name a && "
             "printf 'one\\n' > f && git add f && git commit -qm c1 && printf 'two\\n' > f && git commit -qam c2") == 0);
    std::string hash1;
    FILE* p = popen(("git -C " + up + " rev-parse HEAD~1").c_str(), "r");
    char buf[128] = {0};
    if (p && fgets(buf, sizeof buf, p)) hash1 = trim(buf);
    if (p) pclose(p);
    CHECK(hash1.size() == 40);
    std::string diff = "diff --git a/f b/f\n--- a/f\n+++ b/f\n@@ -1 +1 @@\n-one\n+patched\n";
    Json b = job({"/bin/sh", "-c", "git rev-parse HEAD; cat f; git config user.name; git config user.email"},
                 "remote");
    Json rs = b["run_spec"];
    Json repo = rs["repo_data"];
    repo.set("repo_hash", hash1);
    repo.set("repo_config_name", std::string("Dev Eloper"));
    repo.set("repo_config_email", std::string("dev@example.com"));
    rs.set("repo_data", repo);
    b.set("run_spec", rs);
    Json creds = Json::object();
    creds.set("clone_url", "file://" + up);
    b.set("repo_credentials", creds);
    JobResult r = run_job(tmpdir(), b, diff);
    CHECK(r.state == "done");
    CHECK(r.logs == hash1 + "\npatched\nDev Eloper\ndev@example.com\n");
    // a diff that does not apply fails the job before it runs
    r = run_job(tmpdir(), b, "diff --git a/f b/f\n--- a/f\n+++ b/f\n@@ -1 +1 @@\n-nope\n+x\n");
    CHECK(r.state == "failed" && r.reason == "executor_error" && r.message.find("git apply") == 0);
  });

  run("executor: repo credentials are visible to the job and removed after it", [] {
    std::string root = tmpdir();
    Json b = job({"/bin/sh", "-c", "cat ~/.ssh/id_rsa"}, "remote");
    Json creds = Json::object();
    creds.set("clone_url", std::string("ssh://git@example.com/org/repo.git"));
    creds.set("private_key", std::string("-----BEGIN KEY-----\nabc\n-----END KEY-----\n"));
    b.set("repo_credentials", creds);
    // no real remote here: the repo is pre-seeded so setup skips the clone
    mkdirs(root + "/wd/.git");
    CHECK(sh("git init -q " + root + "/wd") == 0);
    JobResult r = run_job(root, b);
    CHECK(r.state == "done" && r.logs == "-----BEGIN KEY-----\nabc\n-----END KEY-----\n");
    struct stat st;
    CHECK(stat((root + "/home/.ssh/id_rsa").c_str(), &st) != 0);  // removed after the job
    // an existing key is never overwritten: the job fails instead
    write_file(root + "/home/.ssh/id_rsa", "mine", 0600);
    r = run_job(root, b);
    CHECK(r.state == "failed" && r.message.find("already exists") != std::string::npos);
    std::string kept;
    CHECK(read_file(root + "/home/.ssh/id_rsa", kept) && kept == "mine");
    // an HTTPS token becomes the GitHub CLI's hosts.yml for the clone host
    std::string root2 = tmpdir();
    CHECK(sh("git init -q " + root2 + "/wd") == 0);
    Json b2 = job({"/bin/sh", "-c", "cat ~/.config/gh/hosts.yml"}, "remote");
    Json c2 = Json::object();
    c2.set("clone_url", std::string("https://github.com/org/repo.git"));
    c2.set("oauth_token", std::string("tok123"));
    b2.set("repo_credentials", c2);
    r = run_job(root2, b2);
    CHECK(r.state == "done" && r.logs == "github.com:\n  oauth_token: \"tok123\"\n");
  });

  run("executor: max_duration stops the job", [] {
    Json b = job({"/bin/sh", "-c", "echo 1; sleep 5; echo 2"});
    Json js = b["job_spec"];
    js.set("max_duration", 1);
    b.set("job_spec", js);
    JobResult r = run_job(tmpdir(), b);
    CHECK(r.state == "terminated" && r.reason == "max_duration_exceeded");
    CHECK(r.logs.find("1") != std::string::npos && r.logs.find("2") == std::string::npos);
  });

  run("executor: a fault while running is recovered into a failed job", [] {
    setenv("DSTACK_RUNNER_FAULT_INJECT", "boom", 1);
    JobResult r = run_job(tmpdir(), job({"true"}));
    unsetenv("DSTACK_RUNNER_FAULT_INJECT");
    CHECK(r.state == "failed" && r.reason == "executor_error" && r.message.find("recovered: ") == 0);
    r = run_job(tmpdir(), job({}));  // no command at all
    CHECK(r.state == "failed" && r.reason == "executor_error" && r.message == "empty command");
  });

  // ---- shim authorized_keys.go ------------------------------------------------------------------
  run("executor: a blocking RCCL pre-flight failure fails the job with the probe's message before the job runs", [] {
    // stub dstack-probe: records its argv; node 1 reports a hung rank, node 0 a healthy ring
    std::string root = tmpdir();
    std::string probe = root + "/probe.sh";
    write_file(probe,
               "#!/bin/sh\necho \"$@\" > " + root + "/probe_args\nrank=0\nwhile [ $# -gt 0 ]; do "
               "[ \"$1\" = --node-rank ] && rank=$2; shift; done\nif [ \"$rank\" = 1 ]; then echo 'rank 9: waiting'; "
               "echo '{\"rccl_world\": 16, \"rccl_busbw_gb_s\": null, \"healthy\": false, \"message\": \"RCCL: rank 9 "
               "timed out\"}'; exit 1; fi\necho '{\"rccl_world\": 16, \"rccl_busbw_gb_s\": 311.5, \"healthy\": true, "
               "\"message\": \"\"}'\n",
               0755);
    auto body = [&](const std::string& rank, const char* cmd = "echo trained", const char* mode = "blocking") {
      Json b = job({"/bin/sh", "-c", cmd});
      Json js = b["job_spec"];
      Json env = Json::object();
      env.set("DSTACK_RCCL_PREFLIGHT", std::string("force"));
      env.set("DSTACK_RCCL_PREFLIGHT_MODE", std::string(mode));
      env.set("DSTACK_NODE_RANK", rank);
      env.set("DSTACK_NODES_NUM", std::string("2"));
      env.set("DSTACK_GPUS_PER_NODE", std::string("8"));
      env.set("DSTACK_RCCL_PREFLIGHT_TIMEOUT", std::string("60"));
      js.set("env", env);
      b.set("job_spec", js);
      return b;
    };
    Json pull;
    JobResult r = run_job(root + "/n1", body("1"), "", probe, &pull);
    CHECK(r.state == "failed" && r.reason == "executor_error");
    CHECK(r.message.find("RCCL pre-flight failed (exit 1): RCCL: rank 9 timed out") == 0);
    CHECK(r.logs.find("trained") == std::string::npos);  // the job never started
    CHECK(pull["rccl_preflight"]["healthy"].as_bool(true) == false);
    // the probe's own deadline ends before the outer timeout (60 s - 15 s - 5 s collect margin)
    std::string args;
    CHECK(read_file(root + "/probe_args", args) && args.find("--timeout-ms 40000") != std::string::npos);
    r = run_job(root + "/n0", body("0"), "", probe, &pull);
    CHECK(r.state == "done" && r.logs.find("trained") != std::string::npos);
    CHECK(pull["rccl_preflight"]["rccl_busbw_gb_s"].as_double(0) > 311.0);
  });

  run("executor: the concurrent RCCL pre-flight (default) stops a running job when it fails", [] {
    // stub probe: node 1 fails after 1 s; the job itself would run for 30 s
    std::string root = tmpdir();
    std::string probe = root + "/probe.sh";
    write_file(probe,
               "#!/bin/sh\nrank=0\nwhile [ $# -gt 0 ]; do [ \"$1\" = --node-rank ] && rank=$2; shift; done\nsleep 1\n"
               "if [ \"$rank\" = 1 ]; then echo '{\"healthy\": false, \"message\": \"RCCL: rank 9 timed out\"}'; "
               "exit 1; fi\necho '{\"rccl_busbw_gb_s\": 311.5, \"healthy\": true, \"message\": \"\"}'\n",
               0755);
    auto body = [&](const std::string& rank, const char* cmd) {
      Json b = job({"/bin/sh", "-c", cmd});
      Json js = b["job_spec"];
      Json env = Json::object();
      env.set("DSTACK_RCCL_PREFLIGHT", std::string("force"));
      env.set("DSTACK_NODE_RANK", rank);
      env.set("DSTACK_NODES_NUM", std::string("2"));
      env.set("DSTACK_GPUS_PER_NODE", std::string("8"));
      js.set("env", env);
      b.set("job_spec", js);
      return b;
    };
    Json pull;
    const int64_t t0 = now_millis();
    JobResult r = run_job(root + "/n1", body("1", "echo started; sleep 30; echo trained"), "", probe, &pull);
    CHECK(r.state == "failed" && r.reason == "executor_error");
    CHECK(r.message.find("RCCL pre-flight failed (exit 1): RCCL: rank 9 timed out") == 0);
    CHECK(r.logs.find("started") != std::string::npos);  // the job ran beside the probe...
    CHECK(r.logs.find("trained") == std::string::npos);  // ...and was stopped when it failed
    CHECK(now_millis() - t0 < 15000);
    // a healthy probe that ends while the job runs: its document is recorded (mode: concurrent,
    // capped sweep), and its output reaches the log before the job ends -- the probe's pipe got its
    // EOF although the job was forked beside it (close-on-exec pipes, forks serialised); repeated,
    // since the fork race is a matter of timing
    for (int rep = 0; rep < 4; ++rep) {
      r = run_job(root + "/n0", body("0", "sleep 2; echo trained"), "", probe, &pull);
      CHECK(r.state == "done" && r.logs.find("trained") != std::string::npos);
      CHECK(pull["rccl_preflight"]["rccl_busbw_gb_s"].as_double(0) > 311.0);
      CHECK(pull["rccl_preflight"]["mode"].str() == "concurrent");
      const size_t pf = r.logs.find("[dstack] RCCL pre-flight, concurrent");
      CHECK(pf != std::string::npos && pf < r.logs.find("trained"));
    }
  });

  run("executor: a job that ends before the concurrent pre-flight is reported at once, probe stopped", [] {
    // stub probe: records its argv, then fails after 4 s; the job is done in well under a second
    std::string root = tmpdir();
    std::string probe = root + "/probe.sh";
    write_file(probe,
               "#!/bin/sh\necho \"$@\" > " + root + "/probe_args\nsleep 4\n"
               "echo '{\"healthy\": false, \"message\": \"RCCL: rank 3 timed out\"}'; exit 1\n",
               0755);
    Json b = job({"/bin/sh", "-c", "sleep 0.5; echo quick"});
    Json js = b["job_spec"];
    Json env = Json::object();
    env.set("DSTACK_RCCL_PREFLIGHT", std::string("force"));
    env.set("DSTACK_GPUS_PER_NODE", std::string("8"));
    js.set("env", env);
    b.set("job_spec", js);
    Json pull;
    const int64_t t0 = now_millis();
    JobResult r = run_job(root + "/n", b, "", probe, &pull);
    // the job's own result (done), not the probe's later failure, and without waiting for it
    CHECK(r.state == "done" && r.reason == "done_by_runner");
    CHECK(r.logs.find("quick") != std::string::npos);
    CHECK(r.logs.find("RCCL pre-flight stopped: the job ended first") != std::string::npos);
    CHECK(now_millis() - t0 < 3500);
    CHECK(!pull["rccl_preflight"].is_object());  // a stopped probe records no health document
    // the concurrent probe's sweep is capped
    std::string args;
    CHECK(read_file(root + "/probe_args", args) && args.find("--max-mib 64") != std::string::npos);
  });

  run("host_info: a failed amdgpu bootstrap (marker file) is reported as gpu_driver_error", [] {
    std::string root = tmpdir();
    setenv("DSTACK_AMDGPU_MARKER", (root + "/failed").c_str(), 1);
    CHECK(!collect_host_info(root).has("gpu_driver_error"));
    write_file(root + "/failed", "amdgpu 7.0 driver install failed on ubuntu/noble kernel 6.8.0: /dev/kfd missing\n");
    Json h = collect_host_info(root);
    CHECK(h["gpu_driver_error"].str() == "amdgpu 7.0 driver install failed on ubuntu/noble kernel 6.8.0: /dev/kfd missing");
    unsetenv("DSTACK_AMDGPU_MARKER");
  });

  run("authorized_keys: fingerprints and key identity", [] {
    // a real ed25519 public key (generated for this test; the private half was discarded)
    const std::string k1 = "ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIITSR+i4RoOxF46hsNGCw8yd1/HI82K3pA/ZpvMgvZI/ one@host";
    std::string blob;
    CHECK(public_key_blob(k1, blob) && blob.size() == 51);
    std::string fp = public_key_fingerprint(k1);
    CHECK(fp.rfind("SHA256:", 0) == 0 && fp.size() == 7 + 43);
    // the same key with another comment or with options is the same key
    CHECK(public_key_fingerprint("ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIITSR+i4RoOxF46hsNGCw8yd1/HI82K3pA/ZpvMgvZI/") == fp);
    CHECK(public_key_fingerprint("command=\"echo hi there\",no-pty " + k1) == fp);
    // broken keys: no fingerprint, never equal to anything
    CHECK(public_key_fingerprint("ssh-ed25519 !!!notbase64") == "");
    CHECK(public_key_fingerprint("ssh-rsa AAAAC3NzaC1lZDI1NTE5AAAAIITSR+i4RoOxF46hsNGCw8yd1/HI82K3pA/ZpvMgvZI/") == "");
    CHECK(public_key_fingerprint("just text") == "" && public_key_fingerprint("") == "");
  });

  run("authorized_keys: add and remove by key, other lines kept", [] {
    std::string home = tmpdir();
    setenv("HOME", home.c_str(), 1);
    const std::string user = "dsa-no-such-user";  // unknown user: $HOME is used
    const std::string k1 = "ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIITSR+i4RoOxF46hsNGCw8yd1/HI82K3pA/ZpvMgvZI/ one";
    const std::string k2 = "ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIDguEjiy074tPoFzlvwBD45MwLYmJVP7R730/T3a8eSG two";
    const std::string path = home + "/.ssh/authorized_keys";
    mkdirs(home + "/.ssh", 0700);
    write_file(path, "# managed elsewhere\nfrom=\"10.0.0.0/8\" " + k1 + "\n", 0600);
    CHECK(add_authorized_keys(user, {k1, k2, "ssh-ed25519 broken", k2}));
    std::string c;
    CHECK(read_file(path, c));
    // k1 was already there (with options): not added again; k2 once; the broken key skipped
    CHECK(c == "# managed elsewhere\nfrom=\"10.0.0.0/8\" " + k1 + "\n" + k2 + "\n");
    CHECK(remove_authorized_keys(user, {"ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIITSR+i4RoOxF46hsNGCw8yd1/HI82K3pA/ZpvMgvZI/"}));
    CHECK(read_file(path, c) && c == "# managed elsewhere\n" + k2 + "\n");
    CHECK(remove_authorized_keys(user, {k2, "ssh-ed25519 AAAAC3NzaC1lZDI1NTE5AAAAIDguEjiy074tPoFzlvwBD45MwLYmJVP7R730/T3a8eSH"}));
    CHECK(read_file(path, c) && c == "# managed elsewhere\n");
    CHECK(remove_authorized_keys(user, {k1}));  // nothing to remove: fine
    CHECK(add_authorized_keys(user, {k1, k2}));
    CHECK(read_file(path, c) && c == "# managed elsewhere\n" + k1 + "\n" + k2 + "\n");
    std::string bak;
    CHECK(read_file(path + ".dstack.bak", bak) && bak == "# managed elsewhere\n");
  });

  fprintf(stderr, "%d cases, %d failed checks\n", g_run, g_failed);
  return g_failed ? 1 : 0;
}
