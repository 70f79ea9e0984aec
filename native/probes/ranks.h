// One process per GPU, bootstrapped like the job: the RCCL pre-flight runs the same process layout
// a `torchrun --nproc-per-node=G` job does -- G ranks per node, global rank = node_rank*G + local,
// one ncclUniqueId created by global rank 0 and handed to every other rank (local and remote) over
// TCP at master:port (bootstrap.h).  The parent forks the ranks BEFORE it makes any HIP call (a
// process that has initialised the GPU must never fork or exec a GPU user), collects one result
// line per rank over pipes, and only aggregates.
//
// Header-only and HIP/RCCL-free: the rank body and the id factory are callbacks, so the fork /
// bootstrap / collect machinery is unit-tested on the CPU with a stub 128-byte id
// (native/tests/native_tests.cpp); probes/rccl_probe.cpp plugs in ncclGetUniqueId and a
// hipSetDevice + ncclCommInitRank + all-reduce sweep body.
#pragma once
#include <dirent.h>
#include <poll.h>
#include <signal.h>
#include <stdlib.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "bootstrap.h"

namespace dsa {

struct RankCtx {
  int local = 0, local_size = 1, node_rank = 0, nodes = 1, rank = 0, world = 1;
};

struct RankResult {
  int local = 0;
  int exit_status = -1;  // child exit code (128+signal if killed)
  std::string line;      // what the body returned (one line), "" if the rank died first
};

// GPUs this node's job sees, without touching HIP: HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES when
// set (the shim exports the granted set), else the KFD topology's GPU nodes (gpu_id != 0) under
// DSTACK_SYSFS_ROOT (tests) or /.
inline int count_gpus_no_hip() {
  for (const char* var : {"HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"}) {
    const char* v = getenv(var);
    if (!v) continue;
    std::string s = v;
    if (s.empty() || s == "-1") return 0;
    int n = 1;
    for (char c : s) n += c == ',';
    return n;
  }
  const char* root_env = getenv("DSTACK_SYSFS_ROOT");
  const std::string dir = std::string(root_env ? root_env : "") + "/sys/class/kfd/kfd/topology/nodes";
  int n = 0;
  if (DIR* d = opendir(dir.c_str())) {
    while (auto* e = readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      std::string p = dir + "/" + e->d_name + "/gpu_id";
      if (FILE* f = fopen(p.c_str(), "r")) {
        long long id = 0;
        if (fscanf(f, "%lld", &id) == 1 && id != 0) ++n;
        fclose(f);
      }
    }
    closedir(d);
  }
  return n;
}

// Fork `local_size` rank processes of node `node_rank` (of `nodes`).  In global rank 0 `make_id`
// fills the id (returns "" or an error) and a thread serves it on `port` to the other world-1 ranks;
// every other rank fetches it from master:port.  `body(ctx, id)` runs in the child and returns its
// result line.  Children that do not report within `timeout_ms` are killed.  Returns one result per
// local rank (ordered by local index); *err gets the first bootstrap/timeout error, if any.
inline std::vector<RankResult> run_ranks(int local_size, int nodes, int node_rank, const std::string& master, int port,
                                         size_t id_len, const std::function<std::string(std::string&)>& make_id,
                                         const std::function<std::string(const RankCtx&, const std::string&)>& body,
                                         int timeout_ms, std::string* err) {
  std::vector<RankResult> out((size_t)local_size);
  std::vector<pid_t> pids((size_t)local_size, -1);
  std::vector<int> fds((size_t)local_size, -1);
  const int world = nodes * local_size;
  for (int l = 0; l < local_size; ++l) {
    out[(size_t)l].local = l;
    int p[2];
    if (pipe(p) != 0) {
      if (err && err->empty()) *err = "pipe failed";
      continue;
    }
    pid_t pid = fork();
    if (pid == 0) {  // ---- rank process ----
      ::close(p[0]);
      RankCtx c;
      c.local = l;
      c.local_size = local_size;
      c.node_rank = node_rank;
      c.nodes = nodes;
      c.rank = node_rank * local_size + l;
      c.world = world;
      std::string id(id_len, '\0'), e, line;
      std::thread server;
      std::string serve_err;
      if (c.rank == 0) {
        e = make_id(id);
        if (e.empty() && world > 1)
          server = std::thread([&] { serve_err = bootstrap_serve(port, id.data(), id.size(), world - 1, timeout_ms); });
      } else {
        e = bootstrap_fetch(master, port, c.rank, &id[0], id.size(), timeout_ms);
      }
      line = e.empty() ? body(c, id) : "{\"error\": \"bootstrap: " + e + "\"}";
      if (server.joinable()) server.join();
      if (!serve_err.empty()) line = "{\"error\": \"bootstrap: " + serve_err + "\"}";
      line += "\n";
      for (size_t off = 0; off < line.size();) {  // a pipe, not a socket: write(), not send()
        ssize_t w = ::write(p[1], line.data() + off, line.size() - off);
        if (w <= 0) break;
        off += (size_t)w;
      }
      ::close(p[1]);
      _exit(e.empty() && serve_err.empty() ? 0 : 3);
    }
    ::close(p[1]);
    if (pid < 0) {
      ::close(p[0]);
      if (err && err->empty()) *err = "fork failed";
      continue;
    }
    pids[(size_t)l] = pid;
    fds[(size_t)l] = p[0];
  }
  // collect every rank's line (children write once, then exit)
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms + 5000);
  for (int l = 0; l < local_size; ++l) {
    int fd = fds[(size_t)l];
    if (fd < 0) continue;
    std::string acc;
    char buf[4096];
    for (;;) {
      const int left = (int)std::chrono::duration_cast<std::chrono::milliseconds>(
                           deadline - std::chrono::steady_clock::now()).count();
      struct pollfd pf{fd, POLLIN, 0};
      if (left <= 0 || ::poll(&pf, 1, left) <= 0) {
        if (err && err->empty()) *err = "rank " + std::to_string(node_rank * local_size + l) + " timed out";
        break;
      }
      ssize_t n = ::read(fd, buf, sizeof buf);
      if (n <= 0) break;
      acc.append(buf, (size_t)n);
    }
    ::close(fd);
    while (!acc.empty() && (acc.back() == '\n' || acc.back() == '\r')) acc.pop_back();
    out[(size_t)l].line = acc;
  }
  for (int l = 0; l < local_size; ++l) {
    pid_t pid = pids[(size_t)l];
    if (pid <= 0) continue;
    int st = 0;
    // a rank that reported exits right after closing its pipe; one that is still running at the
    // deadline (hung in a collective, or silent) is killed, so the grid of ranks always drains
    pid_t w = 0;
    while ((w = waitpid(pid, &st, WNOHANG)) == 0 && std::chrono::steady_clock::now() < deadline)
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    if (w == 0) {
      kill(pid, SIGKILL);
      waitpid(pid, &st, 0);
    }
    out[(size_t)l].exit_status = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
    if (out[(size_t)l].exit_status != 0 && err && err->empty())
      *err = "rank " + std::to_string(node_rank * local_size + l) + " exited " +
             std::to_string(out[(size_t)l].exit_status);
  }
  return out;
}

}  // namespace dsa
