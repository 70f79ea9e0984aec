// Native scheduler and KV-page allocator of the dstack_amd serving engine (continuous batching).
//
// The reference orchestrator has no serving engine: its services run vLLM/TGI containers
// (reference examples/deployment/{vllm,tgi}, docs/blog/posts/amd-mi300x-inference-benchmark.md).
// This is the MI355X-native engine's host-side runtime, in C++ so the per-step planning
// (page allocation, admission, preemption, block-table packing) never shows up next to a
// 10-30 ms decode step, even at hundreds of sequences.
//
// Model: every sequence owns a list of fixed-size KV pages (PAGE tokens each, see
// ops/csrc/paged_attn.hip).  A step is either a PREFILL step (the prompts of newly admitted
// sequences, plus recomputation of preempted ones) or a DECODE step (one new token for every
// running sequence).  Preemption = recompute: when a running sequence needs a new page and none
// is free, the most recently admitted sequence releases its pages and goes back to the head of
// the waiting queue with all its tokens as its new prompt (tokens stay with the caller).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <deque>
#include <stdexcept>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace {

struct Seq {
  int64_t id = 0;
  int num_tokens = 0;    // prompt + generated so far
  int num_cached = 0;    // tokens whose K/V are in the cache
  int max_tokens = 0;    // cap on num_tokens (prompt + max new tokens)
  int64_t admitted = -1;  // admission order (for preemption: newest first)
  bool running = false;
  std::vector<int32_t> pages;
};

int round_up(int x, int m) { return (x + m - 1) / m * m; }

class Scheduler {
 public:
  Scheduler(int num_pages, int page_size, int max_batch, int max_prefill_tokens, int max_model_len, int pad_to)
      : page_size_(page_size),
        max_batch_(max_batch),
        max_prefill_tokens_(max_prefill_tokens),
        max_model_len_(max_model_len),
        pad_to_(pad_to) {
    if (num_pages <= 0 || page_size <= 0 || max_batch <= 0 || max_prefill_tokens <= 0 || pad_to <= 0)
      throw std::invalid_argument("scheduler: sizes must be positive");
    free_.reserve(num_pages);
    for (int p = num_pages - 1; p >= 0; --p) free_.push_back(p);
    num_pages_ = num_pages;
    table_width_ = (max_model_len + page_size - 1) / page_size;
  }

  void add(int64_t id, int prompt_len, int max_tokens) {
    if (seqs_.count(id)) throw std::invalid_argument("scheduler: duplicate sequence id");
    if (prompt_len <= 0) throw std::invalid_argument("scheduler: empty prompt");
    if (prompt_len >= max_model_len_) throw std::invalid_argument("scheduler: prompt longer than max_model_len");
    if (pages_for(prompt_len + 1) > num_pages_)
      throw std::invalid_argument("scheduler: prompt does not fit in the KV cache");
    Seq s;
    s.id = id;
    s.num_tokens = prompt_len;
    s.max_tokens = std::min(max_tokens, max_model_len_);
    seqs_[id] = std::move(s);
    waiting_.push_back(id);
  }

  // one more token was sampled for `id` (its K/V get written by the next decode step)
  void append(int64_t id) {
    Seq& s = get(id);
    s.num_tokens += 1;
  }

  // after a step: the K/V of every token but the newest are cached
  void mark_computed(int64_t id) {
    Seq& s = get(id);
    s.num_cached = s.num_tokens;
  }

  void finish(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) return;
    release(it->second);
    waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), id), waiting_.end());
    running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    seqs_.erase(it);
  }

  bool is_done(int64_t id) const {
    auto it = seqs_.find(id);
    return it == seqs_.end() || it->second.num_tokens >= it->second.max_tokens;
  }

  // Plan the next step.  Returns a dict with
  //   kind: "prefill" | "decode" | "idle"
  //   seq_ids [n], preempted [k]
  //   prefill: starts [n] (first token to compute = 0), lens [n] (tokens to compute), offsets [n]
  //            (row of each sequence in the padded token buffer), rows (total padded rows),
  //            positions [rows], slots [rows] (-1 on padding rows)
  //   decode:  positions [n], slots [n], ctx_lens [n], block_tables [n, width]
  py::dict schedule(bool prefer_decode) {
    py::dict out;
    std::vector<int64_t> preempted;
    // admission of waiting sequences (prefill-first unless the caller asks to run decodes)
    const bool can_admit = !waiting_.empty() && (int)running_.size() < max_batch_;
    if (can_admit && !(prefer_decode && !running_.empty())) {
      std::vector<int64_t> ids;
      int rows = 0;
      while (!waiting_.empty() && (int)(running_.size() + ids.size()) < max_batch_) {
        Seq& s = get(waiting_.front());
        const int need = pages_for(s.num_tokens + 1) - (int)s.pages.size();
        const int padded = round_up(s.num_tokens, pad_to_);
        if (!ids.empty() && rows + padded > max_prefill_tokens_) break;
        if (need > (int)free_.size()) break;
        grow(s, s.num_tokens + 1);
        s.num_cached = 0;
        s.running = true;
        s.admitted = admit_counter_++;
        ids.push_back(s.id);
        rows += padded;
        waiting_.pop_front();
      }
      if (!ids.empty()) {
        for (auto id : ids) running_.push_back(id);
        const int n = (int)ids.size();
        py::array_t<int32_t> starts(n), lens(n), offsets(n), positions(rows), slots(rows);
        auto st = starts.mutable_unchecked<1>();
        auto ln = lens.mutable_unchecked<1>();
        auto of = offsets.mutable_unchecked<1>();
        auto ps = positions.mutable_unchecked<1>();
        auto sl = slots.mutable_unchecked<1>();
        int row = 0;
        for (int i = 0; i < n; ++i) {
          const Seq& s = get(ids[i]);
          st(i) = 0;
          ln(i) = s.num_tokens;
          of(i) = row;
          const int padded = round_up(s.num_tokens, pad_to_);
          for (int t = 0; t < padded; ++t) {
            ps(row + t) = t < s.num_tokens ? t : 0;
            sl(row + t) = t < s.num_tokens ? slot_of(s, t) : -1;
          }
          row += padded;
        }
        out["kind"] = "prefill";
        out["seq_ids"] = ids;
        out["starts"] = starts;
        out["lens"] = lens;
        out["offsets"] = offsets;
        out["rows"] = rows;
        out["positions"] = positions;
        out["slots"] = slots;
        out["preempted"] = preempted;
        return out;
      }
    }
    if (running_.empty()) {
      out["kind"] = "idle";
      out["seq_ids"] = std::vector<int64_t>{};
      out["preempted"] = preempted;
      return out;
    }
    // decode: every running sequence computes its newest token (position num_tokens - 1)
    // running_ is in admission order, so the newest sequence (the preemption victim) is always
    // at or after the one being grown: removing it never shifts the entries already handled
    size_t i = 0;
    while (i < running_.size()) {
      Seq& s = get(running_[i]);
      bool self_preempted = false;
      while (pages_for(s.num_tokens) > (int)s.pages.size() && free_.empty()) {
        const int64_t victim = running_.back();
        preempt(victim, preempted);
        if (victim == s.id) {
          self_preempted = true;
          break;
        }
      }
      if (self_preempted) continue;
      grow(s, s.num_tokens);
      ++i;
    }
    const int n = (int)running_.size();
    if (n == 0) {
      out["kind"] = "idle";
      out["seq_ids"] = std::vector<int64_t>{};
      out["preempted"] = preempted;
      return out;
    }
    py::array_t<int32_t> positions(n), slots(n), ctx(n);
    py::array_t<int32_t> tables({n, table_width_});
    auto ps = positions.mutable_unchecked<1>();
    auto sl = slots.mutable_unchecked<1>();
    auto cx = ctx.mutable_unchecked<1>();
    auto tb = tables.mutable_unchecked<2>();
    for (int i = 0; i < n; ++i) {
      const Seq& s = get(running_[i]);
      ps(i) = s.num_tokens - 1;
      sl(i) = slot_of(s, s.num_tokens - 1);
      cx(i) = s.num_tokens;
      const int np = (int)s.pages.size();
      for (int j = 0; j < table_width_; ++j) tb(i, j) = j < np ? s.pages[j] : 0;
    }
    out["kind"] = "decode";
    out["seq_ids"] = running_;
    out["positions"] = positions;
    out["slots"] = slots;
    out["ctx_lens"] = ctx;
    out["block_tables"] = tables;
    out["preempted"] = preempted;
    return out;
  }

  int free_pages() const { return (int)free_.size(); }
  int num_pages() const { return num_pages_; }
  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  int table_width() const { return table_width_; }
  int page_size() const { return page_size_; }
  std::vector<int32_t> pages(int64_t id) { return get(id).pages; }
  int num_tokens(int64_t id) { return get(id).num_tokens; }

 private:
  Seq& get(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::out_of_range("scheduler: unknown sequence id");
    return it->second;
  }
  const Seq& get(int64_t id) const {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::out_of_range("scheduler: unknown sequence id");
    return it->second;
  }
  int pages_for(int tokens) const { return (tokens + page_size_ - 1) / page_size_; }
  int32_t slot_of(const Seq& s, int t) const { return s.pages[t / page_size_] * page_size_ + t % page_size_; }

  void grow(Seq& s, int tokens) {
    const int need = pages_for(tokens);
    while ((int)s.pages.size() < need) {
      if (free_.empty()) throw std::runtime_error("scheduler: out of KV pages");
      s.pages.push_back(free_.back());
      free_.pop_back();
    }
  }
  void release(Seq& s) {
    for (auto p : s.pages) free_.push_back(p);
    s.pages.clear();
  }
  void preempt(int64_t id, std::vector<int64_t>& preempted) {
    Seq& s = get(id);
    release(s);
    s.running = false;
    s.num_cached = 0;
    running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    waiting_.push_front(id);
    preempted.push_back(id);
  }

  int page_size_, max_batch_, max_prefill_tokens_, max_model_len_, pad_to_;
  int num_pages_ = 0, table_width_ = 0;
  int64_t admit_counter_ = 0;
  std::vector<int32_t> free_;
  std::unordered_map<int64_t, Seq> seqs_;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;
};

}  // namespace

PYBIND11_MODULE(_sched, m) {
  m.doc() = "dstack_amd serving: native continuous-batching scheduler and KV-page allocator";
  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<int, int, int, int, int, int>(), py::arg("num_pages"), py::arg("page_size"),
           py::arg("max_batch"), py::arg("max_prefill_tokens"), py::arg("max_model_len"), py::arg("pad_to") = 128)
      .def("add", &Scheduler::add, py::arg("seq_id"), py::arg("prompt_len"), py::arg("max_tokens"))
      .def("append", &Scheduler::append)
      .def("mark_computed", &Scheduler::mark_computed)
      .def("finish", &Scheduler::finish)
      .def("is_done", &Scheduler::is_done)
      .def("schedule", &Scheduler::schedule, py::arg("prefer_decode") = false)
      .def("pages", &Scheduler::pages)
      .def("num_tokens", &Scheduler::num_tokens)
      .def_property_readonly("free_pages", &Scheduler::free_pages)
      .def_property_readonly("num_pages", &Scheduler::num_pages)
      .def_property_readonly("num_waiting", &Scheduler::num_waiting)
      .def_property_readonly("num_running", &Scheduler::num_running)
      .def_property_readonly("table_width", &Scheduler::table_width)
      .def_property_readonly("page_size", &Scheduler::page_size);
}
