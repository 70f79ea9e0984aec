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
  for (const char* s : {"-o", "job", "--"}) a.push_back(s);
  return a;
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

std::string summarize_kernel_stats(const std::string& csv, int top) {
  std::istringstream ss(csv);
  std::string line, out = "\n[dstack] rocprofv3 kernel statistics (top " + std::to_string(top) + "):\n";
  int k = 0;
  while (std::getline(ss, line) && k <= top) {
    out += "  " + line.substr(0, 240) + "\n";
    ++k;
  }
  return k ? out : "";
}

std::string summarize_counters(const std::string& csv, const std::vector<std::string>& counters, int top) {
  std::istringstream ss(csv);
  std::string line;
  if (!std::getline(ss, line)) return "";
  auto hdr = parse_csv_record(line);
  auto col = [&](const char* n) -> int {
    for (size_t i = 0; i < hdr.size(); ++i)
      if (hdr[i] == n) return (int)i;
    return -1;
  };
  int kn = col("Kernel_Name"), cn = col("Counter_Name"), cv = col("Counter_Value"), di = col("Dispatch_Id");
  if (kn < 0 || cn < 0 || cv < 0) return "";
  std::map<std::string, std::map<std::string, double>> sums;
  std::map<std::string, std::set<std::string>> dispatches;
  int need = std::max({kn, cn, cv, di}) + 1;
  while (std::getline(ss, line)) {
    auto r = parse_csv_record(line);
    if ((int)r.size() < need) continue;
    sums[r[kn]][r[cn]] += strtod(r[cv].c_str(), nullptr);
    if (di >= 0) dispatches[r[kn]].insert(r[di]);
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
