// Native token-window batch loader (host runtime, no device code).
//
// Replaces the reference's Python-side batching — per-sample slicing + torch.stack in
// get_batch (gpt/gpt-jax.ipynb:491-497, gemma/gemma.ipynb:116-129) and the sliding-window
// CausalDataset behind a DataLoader (deepseekv3/deepseekv3.ipynb:715-726) — with a
// C++ producer pool:
//   * tokens come from a read-only mmap of a flat binary file (uint16 or int32 ids) or
//     from an in-memory int32/uint16/int64 tensor (kept alive by the loader);
//   * batch i is a pure function of (seed, rank, i): window starts are a counter hash,
//     so resume = seek(i) and different ranks draw disjoint-in-expectation streams;
//   * `threads` workers fill a ring of `depth` slots ahead of the consumer; each slot
//     is one [2, B, T] int64 tensor (x = [0], y = [1], optionally in pinned memory so
//     the host->device copy is a DMA that overlaps compute);
//   * next() blocks only if the ring is empty; no Python code runs per sample.
#include <torch/custom_class.h>
#include <torch/library.h>
#include <ATen/ATen.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <fcntl.h>
#include <mutex>
#include <stdexcept>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
#include <vector>

namespace spa {

static inline uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

struct TokenLoader : torch::CustomClassHolder {
  // source
  at::Tensor keep_;            // tensor source (kept alive)
  void* map_ = nullptr;
  size_t map_bytes_ = 0;
  const uint8_t* base_ = nullptr;
  int64_t n_tokens_ = 0;
  int elem_ = 4;               // bytes per token id: 2 (uint16), 4 (int32), 8 (int64)
  // shape / stream
  int64_t B_, T_, seed_, rank_, world_;
  bool pin_, sequential_;
  int depth_;
  // ring state
  std::mutex mu_;
  std::condition_variable cv_ready_, cv_space_;
  std::deque<std::pair<int64_t, at::Tensor>> ready_;
  int64_t next_produce_ = 0;   // next batch index a worker will claim
  int64_t next_consume_ = 0;   // batch index next() returns
  int64_t epoch_ = 0;          // bumped by seek(): stale batches are dropped
  bool stop_ = false;
  std::vector<std::thread> workers_;

  TokenLoader(const std::string& path, int64_t elem_bytes, at::Tensor tokens, int64_t B, int64_t T, int64_t seed,
              int64_t rank, int64_t world, int64_t threads, int64_t depth, bool pin, bool sequential)
      : B_(B), T_(T), seed_(seed), rank_(rank), world_(world), pin_(pin), sequential_(sequential),
        depth_((int)std::max<int64_t>(1, depth)) {
    TORCH_CHECK(B > 0 && T > 0 && world > 0 && rank >= 0 && rank < world, "TokenLoader: bad shape/rank");
    if (!path.empty()) {
      TORCH_CHECK(elem_bytes == 2 || elem_bytes == 4, "TokenLoader: file ids must be uint16 or int32");
      int fd = ::open(path.c_str(), O_RDONLY);
      TORCH_CHECK(fd >= 0, "TokenLoader: cannot open ", path);
      struct stat st;
      ::fstat(fd, &st);
      map_bytes_ = (size_t)st.st_size;
      map_ = ::mmap(nullptr, map_bytes_, PROT_READ, MAP_PRIVATE, fd, 0);
      ::close(fd);
      TORCH_CHECK(map_ != MAP_FAILED, "TokenLoader: mmap failed for ", path);
      ::madvise(map_, map_bytes_, MADV_RANDOM);
      base_ = (const uint8_t*)map_;
      elem_ = (int)elem_bytes;
      n_tokens_ = (int64_t)(map_bytes_ / elem_);
    } else {
      TORCH_CHECK(tokens.defined() && tokens.device().is_cpu() && tokens.dim() == 1, "TokenLoader: 1-D CPU tokens");
      keep_ = tokens.contiguous();
      auto dt = keep_.scalar_type();
      TORCH_CHECK(dt == at::kInt || dt == at::kLong || dt == at::kShort || dt == at::kUInt16,
                  "TokenLoader: int16/uint16/int32/int64 ids");
      elem_ = (int)keep_.element_size();
      base_ = (const uint8_t*)keep_.data_ptr();
      n_tokens_ = keep_.numel();
    }
    TORCH_CHECK(n_tokens_ > T + 1, "TokenLoader: stream shorter than one window");
    const int nt = (int)std::max<int64_t>(1, threads);
    for (int i = 0; i < nt; ++i) workers_.emplace_back([this] { work(); });
  }

  ~TokenLoader() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_space_.notify_all();
    cv_ready_.notify_all();
    for (auto& t : workers_) t.join();
    if (map_) ::munmap(map_, map_bytes_);
  }

  inline int64_t tok(int64_t i) const {
    switch (elem_) {
      case 2: { uint16_t v; std::memcpy(&v, base_ + i * 2, 2); return v; }
      case 4: { int32_t v; std::memcpy(&v, base_ + i * 4, 4); return v; }
      default: { int64_t v; std::memcpy(&v, base_ + i * 8, 8); return v; }
    }
  }

  // window start of sample b of batch i
  int64_t start(int64_t i, int64_t b) const {
    const int64_t span = n_tokens_ - T_ - 1;
    if (sequential_) {   // strided walk: rank r, batch i, row b -> window (i*B*world + r*B + b)*T
      const int64_t w = (i * world_ + rank_) * B_ + b;
      return (w * T_) % (span + 1);
    }
    const uint64_t h = mix64(mix64(mix64((uint64_t)seed_) ^ (uint64_t)rank_) ^ ((uint64_t)i * 0x1000003ULL + b));
    return (int64_t)(h % (uint64_t)(span + 1));
  }

  at::Tensor make(int64_t i) const {
    auto opts = at::TensorOptions().dtype(at::kLong).pinned_memory(pin_);
    at::Tensor out = at::empty({2, B_, T_}, opts);
    int64_t* x = out.data_ptr<int64_t>();
    int64_t* y = x + B_ * T_;
    for (int64_t b = 0; b < B_; ++b) {
      const int64_t s = start(i, b);
      int64_t* xr = x + b * T_;
      int64_t* yr = y + b * T_;
      int64_t prev = tok(s);
      for (int64_t t = 0; t < T_; ++t) {
        const int64_t nx = tok(s + t + 1);
        xr[t] = prev;
        yr[t] = nx;
        prev = nx;
      }
    }
    return out;
  }

  void work() {
    for (;;) {
      int64_t i, ep;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_space_.wait(lk, [&] { return stop_ || next_produce_ - next_consume_ < depth_; });
        if (stop_) return;
        i = next_produce_++;
        ep = epoch_;
      }
      at::Tensor t = make(i);
      {
        std::lock_guard<std::mutex> g(mu_);
        if (ep != epoch_) continue;          // seek() happened meanwhile: drop
        ready_.emplace_back(i, std::move(t));
      }
      cv_ready_.notify_all();
    }
  }

  // returns [2, B, T] int64 (x = [0], y = [1]) for the current position, then advances
  at::Tensor next() {
    std::unique_lock<std::mutex> lk(mu_);
    at::Tensor out;
    cv_ready_.wait(lk, [&] {
      if (stop_) return true;
      for (auto& p : ready_)
        if (p.first == next_consume_) return true;
      return false;
    });
    TORCH_CHECK(!stop_, "TokenLoader stopped");
    for (auto it = ready_.begin(); it != ready_.end(); ++it) {
      if (it->first == next_consume_) {
        out = std::move(it->second);
        ready_.erase(it);
        break;
      }
    }
    ++next_consume_;
    lk.unlock();
    cv_space_.notify_all();
    return out;
  }

  void seek(int64_t i) {
    {
      std::lock_guard<std::mutex> g(mu_);
      ++epoch_;
      ready_.clear();
      next_consume_ = next_produce_ = i;
    }
    cv_space_.notify_all();
  }

  int64_t position() {
    std::lock_guard<std::mutex> g(mu_);
    return next_consume_;
  }
  int64_t num_tokens() const { return n_tokens_; }
  // synchronous, stateless access (tests / eval)
  at::Tensor batch_at(int64_t i) const { return make(i); }
};

}  // namespace spa

TORCH_LIBRARY_FRAGMENT(spa, m) {
  m.class_<spa::TokenLoader>("TokenLoader")
      .def(torch::init<std::string, int64_t, at::Tensor, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                       int64_t, bool, bool>())
      .def("next", &spa::TokenLoader::next)
      .def("seek", &spa::TokenLoader::seek)
      .def("position", &spa::TokenLoader::position)
      .def("num_tokens", &spa::TokenLoader::num_tokens)
      .def("batch_at", &spa::TokenLoader::batch_at);
}
