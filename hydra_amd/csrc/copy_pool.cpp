// copy_pool.cpp -- see copy_pool.h.
#include "copy_pool.h"
#include "options.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

namespace hydra {
namespace {

struct Piece {
  char* dst;
  const char* src;
  size_t bytes;
};

struct Batch {
  std::vector<Piece> pieces;
  std::atomic<size_t> next{0};   // next unclaimed piece
  std::atomic<size_t> done{0};   // pieces copied
  std::atomic<int> helpers{0};   // helpers holding a pointer to this batch
  // claim and copy pieces until none is left
  void work() {
    for (;;) {
      const size_t i = next.fetch_add(1, std::memory_order_relaxed);
      if (i >= pieces.size()) return;
      std::memcpy(pieces[i].dst, pieces[i].src, pieces[i].bytes);
      done.fetch_add(1, std::memory_order_release);
    }
  }
};

class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; i++) std::thread([this] { loop(); }).detach();  // live for the process
  }
  void post(Batch* b) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(b);
    }
    cv_.notify_all();
  }
  // the caller is done with b: no helper may pick it up any more
  void retire(Batch* b) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = std::find(q_.begin(), q_.end(), b);
    if (it != q_.end()) q_.erase(it);
  }

 private:
  void loop() {
    for (;;) {
      Batch* b;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return !q_.empty(); });
        b = q_.front();
        if (b->next.load(std::memory_order_relaxed) >= b->pieces.size()) {
          q_.pop_front();  // every piece claimed: nothing here for anyone
          continue;
        }
        b->helpers.fetch_add(1, std::memory_order_relaxed);  // under the lock: b is alive
      }
      b->work();
      b->helpers.fetch_sub(1, std::memory_order_release);
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Batch*> q_;
};

int helper_count() {  // HYDRA_OPT_COPY_THREADS when the pool starts (the first large copy)
  static const int n = (int)opt(HYDRA_OPT_COPY_THREADS);
  return n;
}

Pool* pool() {
  static Pool* p = helper_count() > 0 ? new Pool(helper_count()) : nullptr;
  return p;
}

}  // namespace

void copy_all(const CopyJob* jobs, size_t count) {
  size_t total = 0;
  for (size_t i = 0; i < count; i++) total += jobs[i].bytes;
  Pool* p = total >= kFanoutMin ? pool() : nullptr;
  if (!p) {
    for (size_t i = 0; i < count; i++) std::memcpy(jobs[i].dst, jobs[i].src, jobs[i].bytes);
    return;
  }
  Batch b;
  b.pieces.reserve(total / kCopyPiece + count);
  for (size_t i = 0; i < count; i++)
    for (size_t o = 0; o < jobs[i].bytes; o += kCopyPiece)
      b.pieces.push_back({static_cast<char*>(jobs[i].dst) + o,
                          static_cast<const char*>(jobs[i].src) + o,
                          std::min(kCopyPiece, jobs[i].bytes - o)});
  p->post(&b);
  b.work();  // the caller copies too
  p->retire(&b);
  // every piece copied, and no helper still holds b
  while (b.done.load(std::memory_order_acquire) < b.pieces.size() ||
         b.helpers.load(std::memory_order_acquire) != 0)
    __builtin_ia32_pause();
}

}  // namespace hydra
