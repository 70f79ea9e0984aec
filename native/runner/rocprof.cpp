// Implementation of rocprof.h.
#include "rocprof.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cctype>
#include <map>
#include <set>
#include <sstream>

namespace dsa {

std::vector<std::string> split_counters(const std::string& spec) {
  std::vector<std::string> out;
  std::string cur;
  for (char c : spec) {
    if (c == ',' || c == ' ' || c == '\t' || c == '\n') {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur += c;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

namespace {
std::string base_counter(const std::string& c) {
  for (const char* suf : {"_sum", "_avr", "_min", "_max"}) {
    size_t n = strlen(suf);
    if (c.size() > n && c.compare(c.size() - n, n, suf) == 0) return c.substr(0, c.size() - n);
  }
  return c;
}

bool valid_name(const std::string& c) {
  if (c.empty() || c.size() > 64) return false;
  for (char ch : c)
    if (!(isalnum((unsigned char)ch) || ch == '_')) return false;
  return true;
}
}  // namespace

bool validate_pmc(const std::vector<std::string>& counters, std::string& err) {
  static const std::map<std::string, int> limits = {{"SQ", 8}, {"TCC", 4}, {"TCP", 4},
                                                    {"TA", 2}, {"TD", 2},  {"GRBM", 2}};
  // derived metrics whose hardware cost is known
  static const std::map<std::string, std::pair<std::string, int>> derived = {{"FETCH_SIZE", {"TCC", 3}},
                                                                             {"WRITE_SIZE", {"TCC", 2}}};
  if (counters.empty()) {
    err = "no counters";
    return false;
  }
  std::map<std::string, int> used;
  std::set<std::string> seen;
  for (auto& c : counters) {
    if (!valid_name(c)) {
      err = "bad counter name '" + c + "'";
      return false;
    }
    std::string b = base_counter(c);
    if (!seen.insert(b).second) continue;
    auto d = derived.find(b);
    if (d != derived.end()) {
      used[d->second.first] += d->second.second;
      continue;
    }
    size_t us = b.find('_');
    std::string block = us == std::string::npos ? "" : b.substr(0, us);
    if (!limits.count(block)) {
      err = "counter '" + c + "' is not an SQ/TCC/TCP/TA/TD/GRBM counter or a known derived metric";
      return false;
    }
    used[block] += 1;
  }
  for (auto& kv : used) {
    int lim = limits.at(kv.first);
    if (kv.second > lim) {
      err = kv.first + " block needs " + std::to_string(kv.second) + " counters, one pass holds " +
            std::to_string(lim) + " (split the set over several runs)";
      return false;
    }
  }
  return true;
}

std::vector<std::string> rocprof_argv(const std::string& out_dir, const std::vector<std::string>& counters) {
  std::vector<std::string> a = {"rocprofv3", "--kernel-trace", "--stats"};
  if (!counters.empty()) {
    a.push_back("--pmc");
    a.insert(a.end(), counters.begin(), counters.end());
  }
  for (const char* s : {"--output-format", "csv", "-d"}) a.push_back(s);
  a.push_back(out_dir);
  for (const char* s : {"-o", "job_%pid%", "--"}) a.push_back(s);
  return a;
}

namespace {
std::string base_name(const std::string& p) {
  size_t k = p.rfind('/');
  return k == std::string::npos ? p : p.substr(k + 1);
}

bool is_assignment(const std::string& w) {
  if (w.empty() || !(isalpha((unsigned char)w[0]) || w[0] == '_')) return false;
  for (size_t i = 1; i < w.size(); ++i) {
    if (w[i] == '=') return true;
    if (!(isalnum((unsigned char)w[i]) || w[i] == '_')) return false;
  }
  return false;
}

std::string shell_quote(const std::string& w) {
  bool plain = !w.empty();
  for (char c : w)
    if (!(isalnum((unsigned char)c) || strchr("_-./=,:%+@", c))) plain = false;
  if (plain) return w;
  std::string q = "'";
  for (char c : w) q += c == '\'' ? std::string("'\\''") : std::string(1, c);
  return q + "'";
}

struct Word {
  std::string text;  // unquoted
  size_t begin = 0;  // offset in the segment
};

// Top-level command separators of a shell script: "&&", "||", ";", "\n", "|", "&" outside quotes,
// $( ), ( ) and backticks.  Returns false on unbalanced quoting.
bool split_script(const std::string& s, std::vector<std::pair<size_t, size_t>>& segs, std::vector<std::string>& seps) {
  size_t start = 0;
  int depth = 0;
  bool sq = false, dq = false, bt = false;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (sq) {
      if (c == '\'') sq = false;
      continue;
    }
    if (c == '\\') {
      ++i;
      continue;
    }
    if (dq) {
      if (c == '"') dq = false;
      continue;
    }
    if (c == '\'') sq = true;
    else if (c == '"') dq = true;
    else if (c == '`') bt = !bt;
    else if (c == '(') ++depth;
    else if (c == ')') --depth;
    else if (c == '#' && depth == 0 && !bt && (i == 0 || isspace((unsigned char)s[i - 1]))) {
      while (i < s.size() && s[i] != '\n') ++i;
      --i;
    } else if (depth == 0 && !bt) {
      std::string sep;
      if ((c == '&' || c == '|') && i + 1 < s.size() && s[i + 1] == c) sep = std::string(2, c);
      else if (c == '|') sep = "|";
      else if (c == '&' && !(i > 0 && (s[i - 1] == '>' || s[i - 1] == '<')) && !(i + 1 < s.size() && s[i + 1] == '>'))
        sep = "&";
      else if (c == ';' || c == '\n') sep = std::string(1, c);
      if (!sep.empty()) {
        segs.emplace_back(start, i);
        seps.push_back(sep == "\n" ? ";" : sep);
        i += sep.size() - 1;
        start = i + 1;
      }
    }
  }
  segs.emplace_back(start, s.size());
  return !sq && !dq && !bt && depth == 0;
}

std::vector<Word> split_words(const std::string& s) {
  std::vector<Word> out;
  Word cur;
  bool in = false, sq = false, dq = false;
  for (size_t i = 0; i < s.size(); ++i) {
    const char c = s[i];
    if (!in && !isspace((unsigned char)c)) {
      in = true;
      cur = Word{};
      cur.begin = i;
    }
    if (!in) continue;
    if (sq) {
      if (c == '\'') sq = false;
      else cur.text += c;
    } else if (dq) {
      if (c == '"') dq = false;
      else if (c == '\\' && i + 1 < s.size()) cur.text += s[++i];
      else cur.text += c;
    } else if (c == '\'') {
      sq = true;
    } else if (c == '"') {
      dq = true;
    } else if (c == '\\' && i + 1 < s.size()) {
      cur.text += s[++i];
    } else if (isspace((unsigned char)c)) {
      out.push_back(cur);
      in = false;
    } else {
      cur.text += c;
    }
  }
  if (in) out.push_back(cur);
  return out;
}

// programs that must never sit between rocprofv3 and the GPU program (they fork/exec it)
const std::set<std::string>& wrappers() {
  static const std::set<std::string> w = {
      "bash", "sh", "dash", "zsh", "ksh", "env", "timeout", "nohup", "numactl", "taskset", "sudo", "su", "time",
      "nice", "ionice", "stdbuf", "xargs", "chrt", "setsid", "strace", "ltrace", "gdb", "valgrind", "rocprofv3",
      "rocprof", "rocprofv2", "rocprof-compute", "omniperf", "mpirun", "mpiexec", "srun", "accelerate",
      "deepspeed", "ray", "make", "parallel", "watch", "flock", "script", "tini", "dumb-init"};
  return w;
}

// torchrun options that take a value (both spellings); everything else starting with '-' is a flag
bool torchrun_opt_takes_value(const std::string& o) {
  static const std::set<std::string> v = {
      "--nnodes", "--nproc-per-node", "--nproc_per_node", "--rdzv-backend", "--rdzv_backend", "--rdzv-endpoint",
      "--rdzv_endpoint", "--rdzv-id", "--rdzv_id", "--rdzv-conf", "--rdzv_conf", "--max-restarts", "--max_restarts",
      "--monitor-interval", "--monitor_interval", "--start-method", "--start_method", "--role", "--master-addr",
      "--master_addr", "--master-port", "--master_port", "--local-addr", "--local_addr", "--node-rank",
      "--node_rank", "--log-dir", "--log_dir", "--redirects", "-r", "--tee", "-t", "--local-ranks-filter",
      "--local_ranks_filter", "--logs-specs", "--logs_specs", "--rdzv-timeout"};
  return v.count(o) > 0;
}
}  // namespace

bool rocprof_wrap(const std::vector<std::string>& job, const std::vector<std::string>& rp, std::vector<std::string>& out,
                  std::string& err) {
  if (job.empty()) {
    err = "empty command";
    return false;
  }
  const std::string prog0 = base_name(job[0]);
  const bool shell = prog0 == "bash" || prog0 == "sh" || prog0 == "dash" || prog0 == "zsh";
  if (!shell) {  // an entrypoint argv: the program is argv[0]
    if (wrappers().count(prog0) || prog0 == "torchrun") {
      err = "the job's program '" + prog0 + "' is a launcher/wrapper, not the GPU program";
      return false;
    }
    out = rp;
    out.insert(out.end(), job.begin(), job.end());
    return true;
  }
  // {shell, [-l...]-c, script}: rewrite the script's last simple command
  if (job.size() != 3 || job[1].empty() || job[1][0] != '-' || job[1].find('c') == std::string::npos) {
    err = "the job runs '" + job[0] + "' without a single -c script";
    return false;
  }
  const std::string& script = job[2];
  std::vector<std::pair<size_t, size_t>> segs;
  std::vector<std::string> seps;
  if (!split_script(script, segs, seps)) {
    err = "unbalanced quotes or parentheses in the job script";
    return false;
  }
  auto blank = [&](size_t k) {
    for (size_t i = segs[k].first; i < segs[k].second; ++i)
      if (!isspace((unsigned char)script[i])) return false;
    return true;
  };
  int last = (int)segs.size() - 1;
  while (last >= 0 && blank((size_t)last)) --last;
  if (last < 0) {
    err = "empty job script";
    return false;
  }
  for (int k = last; k < (int)seps.size(); ++k)
    if (seps[(size_t)k] != ";") {
      err = "the job script ends in '" + seps[(size_t)k] + "' (a background job or pipeline)";
      return false;
    }
  if (last > 0 && seps[(size_t)last - 1] != "&&" && seps[(size_t)last - 1] != ";") {
    err = "the job's last command follows '" + seps[(size_t)last - 1] + "' (a pipeline or an || branch)";
    return false;
  }
  const size_t s0 = segs[(size_t)last].first, s1 = segs[(size_t)last].second;
  const std::string seg = script.substr(s0, s1 - s0);
  auto words = split_words(seg);
  size_t w = 0;
  while (w < words.size() && is_assignment(words[w].text)) ++w;
  if (w < words.size() && words[w].text == "exec") ++w;
  if (w >= words.size()) {
    err = "the job's last command has no program";
    return false;
  }
  static const std::set<std::string> keywords = {"if", "for", "while", "until", "case", "select", "function", "{",
                                                 "(", "!", "[[", "then", "do", "done", "fi", "}"};
  const std::string& first = words[w].text;
  if (keywords.count(first) || first[0] == '(' || first[0] == '{') {
    err = "the job's last command is a compound command ('" + first + "')";
    return false;
  }
  const std::string prog = base_name(first);
  std::string rp_text;
  for (size_t i = 0; i < rp.size(); ++i) rp_text += (i ? " " : "") + shell_quote(rp[i]);
  // where the profiler goes in the segment, and what it wraps
  size_t insert_at = words[w].begin;
  std::string inserted = "exec " + rp_text + " ";
  const bool py = prog.rfind("python", 0) == 0;
  const bool via_module = py && w + 2 < words.size() && words[w + 1].text == "-m" &&
                          (words[w + 2].text == "torch.distributed.run" || words[w + 2].text == "torch.distributed.launch");
  if (prog == "torchrun" || via_module) {
    size_t i = w + (via_module ? 3 : 1);
    bool no_python = false;
    for (; i < words.size(); ++i) {
      const std::string& o = words[i].text;
      if (o.empty() || o[0] != '-') break;
      if (o == "--no-python" || o == "--no_python") no_python = true;
      else if (o == "-m" || o == "--module" || o == "--run-path" || o == "--run_path") {
        err = "torchrun " + o + " cannot be combined with per-rank profiling";
        return false;
      }
      if (o.find('=') == std::string::npos && torchrun_opt_takes_value(o)) ++i;
    }
    if (i >= words.size()) {
      err = "torchrun without a training script";
      return false;
    }
    if (no_python && (wrappers().count(base_name(words[i].text)) || base_name(words[i].text) == "torchrun")) {
      err = "torchrun --no-python runs '" + words[i].text + "', a launcher/wrapper, not the GPU program";
      return false;
    }
    insert_at = words[i].begin;
    inserted = (no_python ? "" : "--no-python ") + rp_text + (no_python ? " " : " python3 -u ");
  } else if (wrappers().count(prog)) {
    err = "the job's last command runs '" + prog + "', a launcher/wrapper, not the GPU program";
    return false;
  }
  std::string new_seg = seg.substr(0, insert_at) + inserted + seg.substr(insert_at);
  if (prog == "torchrun" || via_module) {  // the launcher itself replaces the shell too
    size_t pw = words[w].begin;
    if (w == 0 || words[w - 1].text != "exec") new_seg = new_seg.substr(0, pw) + "exec " + new_seg.substr(pw);
  } else if (w > 0 && words[w - 1].text == "exec") {  // "exec prog" -> "exec rocprofv3 ... -- prog"
    size_t eb = words[w - 1].begin;
    new_seg = seg.substr(0, eb) + inserted + seg.substr(insert_at);
  }
  out = {job[0], job[1], script.substr(0, s0) + new_seg + script.substr(s1)};
  return true;
}

std::vector<std::string> parse_csv_record(const std::string& line) {
  std::vector<std::string> out;
  std::string cur;
  bool q = false;
  for (size_t i = 0; i < line.size(); ++i) {
    char c = line[i];
    if (q) {
      if (c == '"') {
        if (i + 1 < line.size() && line[i + 1] == '"') {
          cur += '"';
          ++i;
        } else {
          q = false;
        }
      } else {
        cur += c;
      }
    } else if (c == '"') {
      q = true;
    } else if (c == ',') {
      out.push_back(cur);
      cur.clear();
    } else if (c != '\r') {
      cur += c;
    }
  }
  out.push_back(cur);
  return out;
}

static std::string short_kernel(const std::string& k) {
  std::string s = k.substr(0, k.find('('));  // drop the argument list
  return s.size() > 60 ? s.substr(0, 57) + "..." : s;
}

std::string summarize_kernel_stats(const std::vector<std::string>& csvs, int top) {
  struct Acc {
    double calls = 0, total_ns = 0;
  };
  std::map<std::string, Acc> acc;
  double all_ns = 0;
  for (auto& csv : csvs) {
    std::istringstream ss(csv);
    std::string line;
    if (!std::getline(ss, line)) continue;
    auto hdr = parse_csv_record(line);
    int nm = -1, ca = -1, to = -1;
    for (size_t i = 0; i < hdr.size(); ++i) {
      if (hdr[i] == "Name" || hdr[i] == "Kernel_Name") nm = (int)i;
      if (hdr[i] == "Calls") ca = (int)i;
      if (hdr[i] == "TotalDurationNs") to = (int)i;
    }
    if (nm < 0 || ca < 0 || to < 0) continue;
    while (std::getline(ss, line)) {
      auto r = parse_csv_record(line);
      if ((int)r.size() <= std::max({nm, ca, to})) continue;
      auto& a = acc[r[nm]];
      a.calls += strtod(r[ca].c_str(), nullptr);
      const double t = strtod(r[to].c_str(), nullptr);
      a.total_ns += t;
      all_ns += t;
    }
  }
  if (acc.empty()) return "";
  std::vector<std::pair<double, std::string>> order;
  for (auto& kv : acc) order.emplace_back(kv.second.total_ns, kv.first);
  std::sort(order.rbegin(), order.rend());
  std::string out = "\n[dstack] rocprofv3 kernel statistics (" + std::to_string(csvs.size()) + " process" +
                    (csvs.size() == 1 ? "" : "es") + ", top " + std::to_string(top) +
                    " by total time):\n  kernel | calls | total ms | avg us | %\n";
  for (int i = 0; i < (int)order.size() && i < top; ++i) {
    const auto& a = acc[order[i].second];
    char buf[128];
    snprintf(buf, sizeof buf, " | %.0f | %.3f | %.2f | %.2f", a.calls, a.total_ns * 1e-6,
             a.calls > 0 ? a.total_ns / a.calls * 1e-3 : 0.0, all_ns > 0 ? 100.0 * a.total_ns / all_ns : 0.0);
    out += "  " + order[i].second.substr(0, 200) + buf + "\n";
  }
  return out;
}

std::string summarize_counters(const std::vector<std::string>& csvs, const std::vector<std::string>& counters,
                               int top) {
  std::map<std::string, std::map<std::string, double>> sums;
  std::map<std::string, std::set<std::string>> dispatches;
  for (size_t f = 0; f < csvs.size(); ++f) {
    std::istringstream ss(csvs[f]);
    std::string line;
    if (!std::getline(ss, line)) continue;
    auto hdr = parse_csv_record(line);
    auto col = [&](const char* n) -> int {
      for (size_t i = 0; i < hdr.size(); ++i)
        if (hdr[i] == n) return (int)i;
      return -1;
    };
    int kn = col("Kernel_Name"), cn = col("Counter_Name"), cv = col("Counter_Value"), di = col("Dispatch_Id");
    if (kn < 0 || cn < 0 || cv < 0) continue;
    int need = std::max({kn, cn, cv, di}) + 1;
    while (std::getline(ss, line)) {
      auto r = parse_csv_record(line);
      if ((int)r.size() < need) continue;
      sums[r[kn]][r[cn]] += strtod(r[cv].c_str(), nullptr);
      if (di >= 0) dispatches[r[kn]].insert(std::to_string(f) + ":" + r[di]);  // ids restart per process
    }
  }
  if (sums.empty()) return "";
  std::vector<std::string> cols = counters;
  if (cols.empty())
    for (auto& kv : sums.begin()->second) cols.push_back(kv.first);
  std::vector<std::pair<double, std::string>> order;
  for (auto& kv : sums) order.emplace_back(kv.second.count(cols[0]) ? kv.second.at(cols[0]) : 0.0, kv.first);
  std::sort(order.rbegin(), order.rend());
  std::string out = "\n[dstack] rocprofv3 counters per kernel (summed over dispatches, top " + std::to_string(top) +
                    " by " + cols[0] + "):\n  kernel | dispatches";
  for (auto& c : cols) out += " | " + c;
  out += "\n";
  for (int i = 0; i < (int)order.size() && i < top; ++i) {
    auto& name = order[i].second;
    out += "  " + short_kernel(name) + " | " + std::to_string(dispatches[name].size());
    for (auto& c : cols) {
      char buf[48];
      auto it = sums[name].find(c);
      snprintf(buf, sizeof buf, "%.6g", it == sums[name].end() ? 0.0 : it->second);
      out += std::string(" | ") + buf;
    }
    out += "\n";
  }
  return out;
}

}  // namespace dsa
