// Implementation of tokloader.h.
#include "tokloader.h"

#include <fcntl.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <numeric>
#include <random>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int32_t kMagic = 20240520;
constexpr size_t kHeaderBytes = 256 * 4;

struct Shard {
  const uint8_t* base = nullptr;  // start of the token data
  void* map = nullptr;
  size_t map_len = 0;
  uint64_t tokens = 0;
  int bytes = 2;
};

struct Batch {
  uint64_t index;
  std::vector<int32_t> tokens;
};

}  // namespace

struct TokLoader {
  std::vector<Shard> shards;
  std::vector<uint64_t> shard_window_start;  // prefix sums of windows per shard
  uint64_t windows = 0, tokens = 0;
  int seq_len = 0, batch = 0, rank = 0, world = 1, prefetch = 2;
  uint64_t seed = 0;

  // epoch order cache (the producer thread only)
  uint64_t order_epoch = UINT64_MAX;
  std::vector<uint32_t> order;

  std::mutex mu;
  std::condition_variable cv;
  std::deque<Batch> ready;
  uint64_t next_produce = 0;   // batch index the producer builds next
  uint64_t generation = 0;     // bumped by seek: in-flight batches of an older generation are dropped
  bool stop = false;
  std::thread producer;

  uint64_t batches_per_epoch() const { return windows / ((uint64_t)batch * world); }

  const std::vector<uint32_t>& epoch_order(uint64_t epoch) {
    if (order_epoch != epoch) {
      order.resize(windows);
      std::iota(order.begin(), order.end(), 0u);
      std::mt19937_64 rng(seed * 0x9E3779B97F4A7C15ULL + epoch);
      std::shuffle(order.begin(), order.end(), rng);
      order_epoch = epoch;
    }
    return order;
  }

  void fill_window(uint64_t w, int32_t* dst) const {
    size_t s = std::upper_bound(shard_window_start.begin(), shard_window_start.end(), w) - shard_window_start.begin() - 1;
    const Shard& sh = shards[s];
    uint64_t off = (w - shard_window_start[s]) * (uint64_t)seq_len;  // windows share their boundary token
    const int n = seq_len + 1;
    if (sh.bytes == 2) {
      const uint16_t* p = reinterpret_cast<const uint16_t*>(sh.base) + off;
      for (int i = 0; i < n; ++i) dst[i] = p[i];
    } else {
      const uint32_t* p = reinterpret_cast<const uint32_t*>(sh.base) + off;
      for (int i = 0; i < n; ++i) dst[i] = (int32_t)p[i];
    }
  }

  void build(uint64_t index, std::vector<int32_t>& out) {
    const uint64_t bpe = batches_per_epoch();
    const uint64_t epoch = index / bpe, within = index % bpe;
    const auto& ord = epoch_order(epoch);
    out.resize((size_t)batch * (seq_len + 1));
    for (int j = 0; j < batch; ++j) {
      uint64_t slot = (within * world + rank) * (uint64_t)batch + j;
      fill_window(ord[slot], out.data() + (size_t)j * (seq_len + 1));
    }
  }

  void run() {
    std::vector<int32_t> buf;
    for (;;) {
      uint64_t idx, gen;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || (int)ready.size() < prefetch; });
        if (stop) return;
        idx = next_produce++;
        gen = generation;
      }
      build(idx, buf);  // outside the lock: the consumer keeps reading ready batches
      std::lock_guard<std::mutex> lk(mu);
      if (gen != generation) continue;  // a seek happened meanwhile
      ready.push_back(Batch{idx, buf});
      cv.notify_all();
    }
  }
};

namespace {

void set_err(char* err, int len, const std::string& msg) {
  if (err && len > 0) snprintf(err, (size_t)len, "%s", msg.c_str());
}

bool map_shard(const char* path, int token_bytes, Shard& sh, std::string& msg) {
  int fd = open(path, O_RDONLY);
  if (fd < 0) {
    msg = std::string("cannot open ") + path + ": " + strerror(errno);
    return false;
  }
  struct stat st{};
  fstat(fd, &st);
  size_t len = (size_t)st.st_size;
  if (len == 0) {
    close(fd);
    msg = std::string("empty shard ") + path;
    return false;
  }
  void* m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    msg = std::string("mmap failed for ") + path;
    return false;
  }
  madvise(m, len, MADV_RANDOM);
  sh.map = m;
  sh.map_len = len;
  const int32_t* hdr = static_cast<const int32_t*>(m);
  if (len >= kHeaderBytes && hdr[0] == kMagic) {  // llm.c shard
    sh.bytes = hdr[1] == 2 ? 4 : 2;
    sh.tokens = (uint64_t)(uint32_t)hdr[2];
    sh.base = static_cast<const uint8_t*>(m) + kHeaderBytes;
    if (kHeaderBytes + sh.tokens * sh.bytes > len) {
      msg = std::string("truncated shard ") + path;
      return false;
    }
  } else {
    if (token_bytes != 2 && token_bytes != 4) {
      msg = std::string(path) + ": no llm.c header, token_bytes must be 2 or 4";
      return false;
    }
    sh.bytes = token_bytes;
    sh.tokens = len / token_bytes;
    sh.base = static_cast<const uint8_t*>(m);
  }
  return true;
}

}  // namespace

extern "C" {

TokLoader* tl_open(const char* const* paths, int n_paths, int token_bytes, int seq_len, int batch, uint64_t seed,
                   int rank, int world, int prefetch, char* err, int err_len) {
  if (n_paths <= 0 || seq_len <= 0 || batch <= 0 || world <= 0 || rank < 0 || rank >= world) {
    set_err(err, err_len, "invalid arguments");
    return nullptr;
  }
  auto l = std::make_unique<TokLoader>();
  l->seq_len = seq_len;
  l->batch = batch;
  l->seed = seed;
  l->rank = rank;
  l->world = world;
  l->prefetch = std::max(1, prefetch);
  for (int i = 0; i < n_paths; ++i) {
    Shard sh;
    std::string msg;
    if (!map_shard(paths[i], token_bytes, sh, msg)) {
      for (auto& s : l->shards) munmap(s.map, s.map_len);
      if (sh.map) munmap(sh.map, sh.map_len);
      set_err(err, err_len, msg);
      return nullptr;
    }
    uint64_t w = sh.tokens > (uint64_t)seq_len ? (sh.tokens - 1) / seq_len : 0;
    l->shard_window_start.push_back(l->windows);
    l->windows += w;
    l->tokens += sh.tokens;
    l->shards.push_back(sh);
  }
  if (l->windows > UINT32_MAX) {
    set_err(err, err_len, "corpus has more than 2^32 windows; use a longer seq_len or fewer shards per loader");
    tl_close(l.release());
    return nullptr;
  }
  if (l->batches_per_epoch() == 0) {
    set_err(err, err_len, "corpus smaller than one global batch (batch x world windows of seq_len + 1 tokens)");
    tl_close(l.release());
    return nullptr;
  }
  TokLoader* p = l.release();
  p->producer = std::thread([p] { p->run(); });
  return p;
}

int tl_next(TokLoader* l, int32_t* out, uint64_t* batch_index) {
  std::unique_lock<std::mutex> lk(l->mu);
  l->cv.wait(lk, [&] { return l->stop || !l->ready.empty(); });
  if (l->ready.empty()) return -1;
  Batch b = std::move(l->ready.front());
  l->ready.pop_front();
  l->cv.notify_all();
  lk.unlock();
  memcpy(out, b.tokens.data(), b.tokens.size() * sizeof(int32_t));
  if (batch_index) *batch_index = b.index;
  return 0;
}

void tl_seek(TokLoader* l, uint64_t batch_index) {
  std::lock_guard<std::mutex> lk(l->mu);
  l->ready.clear();
  l->next_produce = batch_index;
  ++l->generation;
  l->cv.notify_all();
}

uint64_t tl_num_windows(const TokLoader* l) { return l->windows; }
uint64_t tl_num_tokens(const TokLoader* l) { return l->tokens; }
uint64_t tl_batches_per_epoch(const TokLoader* l) { return l->batches_per_epoch(); }

void tl_close(TokLoader* l) {
  if (!l) return;
  {
    std::lock_guard<std::mutex> lk(l->mu);
    l->stop = true;
    l->cv.notify_all();
  }
  if (l->producer.joinable()) l->producer.join();
  for (auto& s : l->shards) munmap(s.map, s.map_len);
  delete l;
}

}  // extern "C"
