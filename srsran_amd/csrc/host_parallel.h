// srsran_amd/csrc/host_parallel.h -- a small persistent host thread pool for the per-subframe host work of a batch
// call (blind-search replay, DCI unpacking, grants): independent per subframe, so a batch of 2,048 splits into
// contiguous chunks.  MI355_HOST_THREADS sets the pool size (default min(8, hardware threads / 2); 1 = serial).
// A caller that finds the pool busy (another object's call in another thread) runs its loop serially.  An exception
// thrown by fn in any part is caught there, every part still completes (so fn stays alive until no worker can call
// it), and the first one is rethrown to the caller.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <exception>
#include <functional>
#include <mutex>
#include <stdint.h>
#include <stdlib.h>
#include <thread>
#include <vector>

namespace mi355 {

class HostPool {
public:
  static HostPool& get()
  {
    static HostPool p;
    return p;
  }

  // fn(begin, end) over [0, n) in chunks of at least min_chunk; returns after every chunk ran
  void parallel_for(uint32_t n, uint32_t min_chunk, const std::function<void(uint32_t, uint32_t)>& fn)
  {
    const uint32_t T = std::min<uint32_t>((uint32_t)workers_.size() + 1, (n + min_chunk - 1) / std::max(1u, min_chunk));
    std::unique_lock<std::mutex> busy(use_, std::try_to_lock);
    if (T <= 1 || !busy.owns_lock()) {
      if (n) fn(0, n);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(m_);
      // a worker of the previous call may still be about to claim (and miss) a part: let it leave first, or it
      // would claim a part of this call twice.  Workers enter under m_, so none can start while it is held.
      while (inside_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
      fn_    = &fn;
      n_     = n;
      parts_ = T;
      left_.store(T, std::memory_order_relaxed);
      next_.store(1, std::memory_order_relaxed); // part 0 is the caller's
      gen_++;
    }
    cv_.notify_all();
    run_part(0);
    while (true) { // help with the remaining parts, then wait for the workers' in-flight ones
      const uint32_t k = next_.fetch_add(1, std::memory_order_acq_rel);
      if (k >= parts_) break;
      run_part(k);
    }
    while (left_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    std::exception_ptr err;
    {
      std::lock_guard<std::mutex> lk(err_m_);
      err.swap(err_);
    }
    if (err) std::rethrow_exception(err);
  }

  ~HostPool()
  {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

private:
  HostPool()
  {
    uint32_t T = 0;
    const uint32_t hw = std::max(1u, std::thread::hardware_concurrency());
    if (const char* e = getenv("MI355_HOST_THREADS")) {
      const long v = strtol(e, nullptr, 10); // clamped to [1, hardware threads]
      T            = (uint32_t)std::min<long>(std::max<long>(v, 1), (long)hw);
    } else {
      T = std::min(8u, std::max(1u, hw / 2));
    }
    for (uint32_t i = 1; i < T; i++) workers_.emplace_back([this] { loop(); });
  }

  void run_part(uint32_t k)
  {
    const uint32_t b = (uint32_t)((uint64_t)n_ * k / parts_), e = (uint32_t)((uint64_t)n_ * (k + 1) / parts_);
    if (b < e) {
      try {
        (*fn_)(b, e);
      } catch (...) {
        std::lock_guard<std::mutex> lk(err_m_);
        if (!err_) err_ = std::current_exception();
      }
    }
    left_.fetch_sub(1, std::memory_order_acq_rel);
  }

  void loop()
  {
    uint64_t seen = 0;
    while (true) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        inside_.fetch_add(1, std::memory_order_relaxed);
      }
      while (true) {
        const uint32_t k = next_.fetch_add(1, std::memory_order_acq_rel);
        if (k >= parts_) break;
        run_part(k);
      }
      inside_.fetch_sub(1, std::memory_order_release);
    }
  }

  std::vector<std::thread>                         workers_;
  std::mutex                                       m_, use_, err_m_;
  std::exception_ptr                               err_;
  std::condition_variable                          cv_;
  const std::function<void(uint32_t, uint32_t)>*  fn_ = nullptr;
  uint32_t                                         n_ = 0, parts_ = 0;
  uint64_t                                         gen_ = 0;
  bool                                             stop_ = false;
  std::atomic<uint32_t>                            next_{0}, left_{0}, inside_{0};
};

inline void host_parallel_for(uint32_t n, uint32_t min_chunk, const std::function<void(uint32_t, uint32_t)>& fn)
{
  HostPool::get().parallel_for(n, min_chunk, fn);
}

} // namespace mi355
