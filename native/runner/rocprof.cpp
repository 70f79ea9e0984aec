// Implementation of rocprof.h.
#include "rocprof.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

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
  size_t end = 0;    // one past its last character
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
      cur.end = i;
      out.push_back(cur);
      in = false;
    } else {
      cur.text += c;
    }
  }
  if (in) {
    cur.end = s.size();
    out.push_back(cur);
  }
  return out;
}

// "<<" outside quotes (a heredoc; "<<<" here-strings are single-line and fine)
bool has_heredoc(const std::string& s) {
  bool sq = false, dq = false;
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
    else if (c == '<' && i + 1 < s.size() && s[i + 1] == '<') {
      if (i + 2 < s.size() && s[i + 2] == '<') {
        i += 2;
        continue;
      }
      return true;
    }
  }
  return false;
}

bool is_elf(const std::string& h) { return h.size() >= 4 && h.compare(0, 4, "\x7f" "ELF") == 0; }

bool is_python_name(const std::string& p) { return base_name(p).rfind("python", 0) == 0; }

// "#!/usr/bin/env -S python3 -u" -> interpreter "python3", extra {"-u"}.  False without "#!".
bool parse_shebang(const std::string& head, std::string& interp, std::vector<std::string>& extra) {
  if (head.size() < 2 || head[0] != '#' || head[1] != '!') return false;
  const size_t nl = head.find('\n');
  const std::string line = head.substr(2, nl == std::string::npos ? std::string::npos : nl - 2);
  std::vector<std::string> toks;
  for (auto& w : split_words(line)) toks.push_back(w.text);
  size_t i = 0;
  if (!toks.empty() && base_name(toks[0]) == "env") {
    ++i;
    while (i < toks.size() && (toks[i][0] == '-' || is_assignment(toks[i]))) {
      if (toks[i] == "-u" || toks[i] == "--unset" || toks[i] == "-C" || toks[i] == "--chdir") ++i;
      ++i;
    }
  }
  interp = i < toks.size() ? toks[i] : "";
  extra.assign(toks.begin() + (long)std::min(i + 1, toks.size()), toks.end());
  return true;
}

// The program rocprofv3 will start, checked on disk.  OK as is when it is an ELF binary; a "#!"
// Python script is replaced by its interpreter + the script (`replace`); anything else is refused.
bool check_program(const std::string& prog, const ProgramLookup& look, const std::string& cwd,
                   std::vector<std::string>& replace, std::string& err) {
  replace.clear();
  if (!look) return true;  // no filesystem view (text-rewrite unit tests)
  const ProgramInfo pi = look(prog, cwd);
  if (!pi.found) {
    err = "cannot find the job's program '" + prog + "' to check that it is not a script";
    return false;
  }
  if (is_elf(pi.head)) return true;
  std::string interp;
  std::vector<std::string> extra;
  if (!parse_shebang(pi.head, interp, extra)) {
    err = "'" + prog + "' is neither an ELF binary nor a #! script (a shell would run it)";
    return false;
  }
  if (!is_python_name(interp)) {
    err = "'" + prog + "' is a #! script run by '" + (interp.empty() ? std::string("?") : interp) +
          "', not by Python";
    return false;
  }
  const ProgramInfo ip = look(interp, cwd);
  if (!ip.found || !is_elf(ip.head)) {
    err = "the interpreter '" + interp + "' of '" + prog + "' is not an ELF binary (a shim or wrapper script)";
    return false;
  }
  replace.push_back(interp);
  replace.insert(replace.end(), extra.begin(), extra.end());
  replace.push_back(prog);
  return true;
}

// the Python a launcher (torchrun, accelerate, deepspeed: console scripts) runs under, from its
// shebang; "python3" when it cannot be read
std::string launcher_python(const std::string& launcher, const ProgramLookup& look, const std::string& cwd) {
  if (!look) return "python3";
  const ProgramInfo pi = look(launcher, cwd);
  std::string interp;
  std::vector<std::string> extra;
  if (pi.found && parse_shebang(pi.head, interp, extra) && is_python_name(interp)) {
    const ProgramInfo ip = look(interp, cwd);
    if (ip.found && is_elf(ip.head)) return interp;
  }
  return "python3";
}

// programs that must never sit between rocprofv3 and the GPU program (they fork/exec it)
const std::set<std::string>& wrappers() {
  static const std::set<std::string> w = {
      "bash", "sh", "dash", "zsh", "ksh", "env", "timeout", "nohup", "numactl", "taskset", "sudo", "su", "time",
      "nice", "ionice", "stdbuf", "xargs", "chrt", "setsid", "strace", "ltrace", "gdb", "valgrind", "rocprofv3",
      "rocprof", "rocprofv2", "rocprof-compute", "omniperf", "mpirun", "mpiexec", "srun", "accelerate",
      "deepspeed", "ray", "make", "parallel", "watch", "flock", "script", "tini", "dumb-init", "uv", "uvx",
      "poetry", "conda", "mamba", "micromamba", "pixi", "pipenv", "hatch", "pdm", "rye", "npx", "nix-shell",
      "apptainer", "singularity", "docker", "podman", "firejail", "xvfb-run", "catchsegv", "sg", "runuser"};
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

ProgramLookup fs_program_lookup(const std::string& path_env) {
  return [path_env](const std::string& prog, const std::string& cwd) {
    ProgramInfo pi;
    auto probe = [&](const std::string& f, bool need_exec) {
      struct stat st;
      if (stat(f.c_str(), &st) != 0 || !S_ISREG(st.st_mode)) return false;
      if (need_exec && access(f.c_str(), X_OK) != 0) return false;
      pi.found = true;
      pi.path = f;
      if (FILE* fp = fopen(f.c_str(), "rb")) {
        char buf[256];
        size_t n = fread(buf, 1, sizeof buf, fp);
        pi.head.assign(buf, n);
        fclose(fp);
      }
      return true;
    };
    if (prog.find('/') != std::string::npos) {
      probe(prog[0] == '/' ? prog : (cwd.empty() ? std::string(".") : cwd) + "/" + prog, false);
      return pi;
    }
    size_t a = 0;
    while (a <= path_env.size()) {
      size_t b = path_env.find(':', a);
      if (b == std::string::npos) b = path_env.size();
      std::string dir = path_env.substr(a, b - a);
      if (dir.empty()) dir = ".";
      if (dir[0] != '/') dir = (cwd.empty() ? std::string(".") : cwd) + "/" + dir;
      if (probe(dir + "/" + prog, true)) break;
      a = b + 1;
    }
    return pi;
  };
}

bool rocprof_wrap(const std::vector<std::string>& job, const std::vector<std::string>& rp, std::vector<std::string>& out,
                  std::string& err, const ProgramLookup& look, const std::string& cwd) {
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
    std::vector<std::string> rep;
    if (!check_program(job[0], look, cwd, rep, err)) return false;
    out = rp;
    if (rep.empty()) out.push_back(job[0]);
    else out.insert(out.end(), rep.begin(), rep.end());
    out.insert(out.end(), job.begin() + 1, job.end());
    return true;
  }
  // {shell, [-l...]-c, script}: rewrite the script's last simple command
  if (job.size() != 3 || job[1].empty() || job[1][0] != '-' || job[1].find('c') == std::string::npos) {
    err = "the job runs '" + job[0] + "' without a single -c script";
    return false;
  }
  const std::string& script = job[2];
  if (has_heredoc(script)) {
    err = "the job script has a heredoc (<<): its body lines are not commands";
    return false;
  }
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
  // the directory the last command runs in: `cd DIR` segments before it (a DIR with expansions
  // makes relative program paths unresolvable)
  std::string run_cwd = cwd;
  bool cwd_known = true;
  for (int k = 0; k < last; ++k) {
    auto ws = split_words(script.substr(segs[(size_t)k].first, segs[(size_t)k].second - segs[(size_t)k].first));
    if (ws.empty() || (ws[0].text != "cd" && ws[0].text != "pushd")) continue;
    const std::string d = ws.size() > 1 ? ws[1].text : std::string("~");
    if (d.find_first_of("$~`*?") != std::string::npos || d == "-") cwd_known = false;
    else if (d[0] == '/') run_cwd = d, cwd_known = true;
    else run_cwd = (run_cwd.empty() ? std::string(".") : run_cwd) + "/" + d;
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
  auto check = [&](const std::string& p, std::vector<std::string>& rep) {
    if (!cwd_known && p.find('/') != std::string::npos && p[0] != '/') {
      err = "cannot resolve '" + p + "': the script changes to a directory with an expansion first";
      return false;
    }
    return check_program(p, look, run_cwd, rep, err);
  };
  auto join = [](const std::vector<std::string>& v) {
    std::string r;
    for (size_t i = 0; i < v.size(); ++i) r += (i ? " " : "") + shell_quote(v[i]);
    return r;
  };
  const std::string prog = base_name(first);
  const std::string rp_text = join(rp);
  const bool py = is_python_name(prog);
  static const std::set<std::string> py_launchers = {"accelerate", "accelerate.commands.launch",
                                                      "accelerate.commands.accelerate_cli", "deepspeed",
                                                      "deepspeed.launcher.runner", "deepspeed.launcher.launch",
                                                      "torch.distributed.launch"};
  // torch.distributed.run, or dstack_amd's torch-free launcher with the same options
  const bool via_module = py && w + 2 < words.size() && words[w + 1].text == "-m" &&
                          (words[w + 2].text == "torch.distributed.run" ||
                           words[w + 2].text == "dstack_amd.workloads.launch");
  if (py && w + 2 < words.size() && words[w + 1].text == "-m" && py_launchers.count(words[w + 2].text) &&
      words[w + 2].text != "torch.distributed.run") {
    err = "'python -m " + words[w + 2].text + "' is a launcher: run it as torchrun / accelerate launch / deepspeed";
    return false;
  }
  std::string new_seg;
  bool launcher = false;
  if (prog == "torchrun" || via_module) {
    launcher = true;
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
    std::string inserted;
    size_t cut = words[i].begin;
    if (no_python) {
      if (wrappers().count(base_name(words[i].text)) || base_name(words[i].text) == "torchrun") {
        err = "torchrun --no-python runs '" + words[i].text + "', a launcher/wrapper, not the GPU program";
        return false;
      }
      std::vector<std::string> rep;
      if (!check(words[i].text, rep)) return false;
      inserted = rp_text + " " + (rep.empty() ? seg.substr(words[i].begin, words[i].end - words[i].begin) : join(rep));
      cut = words[i].end;
    } else {
      // every rank runs under the launcher's own interpreter (its shebang; the python word itself
      // for `python -m torch.distributed.run`), not whatever "python3" is first on PATH
      const std::string rank_py = via_module ? words[w].text : launcher_python(first, look, run_cwd);
      inserted = "--no-python " + rp_text + " " + shell_quote(rank_py) + " -u ";
    }
    new_seg = seg.substr(0, words[i].begin) + inserted + seg.substr(no_python ? cut : words[i].begin);
  } else if (prog == "accelerate" || prog == "deepspeed") {
    launcher = true;
    size_t i = w + 1;
    if (prog == "accelerate") {
      if (i >= words.size() || words[i].text != "launch") {
        err = "'accelerate' without 'launch' is not a training launch";
        return false;
      }
      ++i;
    }
    size_t script_at = words.size();
    for (; i < words.size(); ++i) {
      const std::string& o = words[i].text;
      if (o == "-m" || o == "--module" || o == "--no_python" || o == "--no-python") {
        err = prog + " " + o + " cannot be combined with per-rank profiling";
        return false;
      }
      if (!o.empty() && o[0] != '-' && o.size() > 3 && o.compare(o.size() - 3, 3, ".py") == 0) {
        script_at = i;
        break;
      }
    }
    if (script_at >= words.size()) {
      err = prog + " without a training script (*.py)";
      return false;
    }
    const std::string rank_py = launcher_python(first, look, run_cwd);
    new_seg = seg.substr(0, words[script_at].begin) + "--no_python " + rp_text + " " + shell_quote(rank_py) + " -u " +
              seg.substr(words[script_at].begin);
  } else if (wrappers().count(prog)) {
    err = "the job's last command runs '" + prog + "', a launcher/wrapper, not the GPU program";
    return false;
  } else {
    std::vector<std::string> rep;
    if (!check(first, rep)) return false;
    const std::string prog_text = rep.empty() ? seg.substr(words[w].begin, words[w].end - words[w].begin) : join(rep);
    size_t from = words[w].begin;
    if (w > 0 && words[w - 1].text == "exec") from = words[w - 1].begin;  // "exec prog" -> "exec rocprofv3 ... -- prog"
    new_seg = seg.substr(0, from) + "exec " + rp_text + " " + prog_text + seg.substr(words[w].end);
  }
  if (launcher) {  // the launcher itself replaces the shell too
    size_t pw = words[w].begin;
    if (w == 0 || words[w - 1].text != "exec") new_seg = new_seg.substr(0, pw) + "exec " + new_seg.substr(pw);
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
