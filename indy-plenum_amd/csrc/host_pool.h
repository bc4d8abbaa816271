// host_pool.h -- persistent host helper threads for the native host path
// (csrc/hostpack.cpp's batch scan, edverify.hip's staging copy).
//
// Threads created per call start next to the thread that spawns them, and the
// scheduler spreads short-lived threads only after milliseconds; pooled
// helpers sleep on a condition variable between calls and wake wherever the
// scheduler has already placed them (profiles/r02y: the drop-in's end to end
// 18.2-18.9 -> 21.8-22.4 M requests/s on 1M requests, 3.5-4.5 -> 5.4-5.5 M on
// 10k).  One pool per library; a child process after fork() (which has none
// of the parent's threads) builds a pool of its own.
#pragma once
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <unistd.h>

#include <condition_variable>
#include <exception>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace {

// CPUs for t workers: the calling thread's CPU, then the next t - 1 CPUs of
// the process's affinity mask (wrapping).
inline std::vector<int> worker_cpus(int t) {
  std::vector<int> all, out;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof set, &set) == 0)
    for (int c = 0; c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &set)) all.push_back(c);
  if (all.empty()) return out;
  const int cur = sched_getcpu();
  size_t at = 0;
  while (at < all.size() && all[at] != cur) ++at;
  if (at == all.size()) at = 0;
  for (int w = 0; w < t; ++w) out.push_back(all[(at + (size_t)w) % all.size()]);
  return out;
}

// Helper threads kept from call to call (workers 1..t-1; the caller is worker
// 0).  EDV_SCAN_PIN=1 pins each helper to its own CPU (worker_cpus) when it is
// created.
class HostPool {
 public:
  // f(w) for w in [1, t) on the helpers while the caller runs f(0); returns
  // when every f has returned.  An exception thrown by any f (e.g. bad_alloc
  // from a worker's buffer growth) is caught where it is thrown, every helper
  // is still waited for, and the first one is rethrown on the caller -- so no
  // helper calls std::terminate and the caller never unwinds while helpers
  // still run the job.
  // A call while another is running (engines of several devices staging at
  // once) runs on threads of its own.
  void run(int t, const std::function<void(int)>& f) {
    std::exception_ptr err;
    std::mutex err_mu;
    const std::function<void(int)> g = [&](int w) {
      try {
        f(w);
      } catch (...) {
        std::lock_guard<std::mutex> l(err_mu);
        if (!err) err = std::current_exception();
      }
    };
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock()) {
      std::vector<std::thread> th;
      for (int w = 1; w < t; ++w) {
        try {
          th.emplace_back(g, w);
        } catch (...) {  // no thread: run its share here
          g(w);
        }
      }
      g(0);
      for (auto& x : th) x.join();
      if (err) std::rethrow_exception(err);
      return;
    }
    std::unique_lock<std::mutex> lk(mu_);
    while ((int)th_.size() < t - 1) {
      const int w = (int)th_.size() + 1;
      try {
        th_.emplace_back([this, w, seen = gen_] { helper(w, seen); });
      } catch (...) {
        t = w;  // fewer helpers: workers 0..w-1 (run_chunks' shared counter covers every item)
        break;
      }
      if (have_aff_) (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof aff_, &aff_);
      const char* pin_env = getenv("EDV_SCAN_PIN");
      if (pin_env && pin_env[0] == '1') {
        const std::vector<int> cpus = worker_cpus(w + 1);
        if ((size_t)w < cpus.size()) {
          cpu_set_t one;
          CPU_ZERO(&one);
          CPU_SET(cpus[(size_t)w], &one);
          (void)pthread_setaffinity_np(th_.back().native_handle(), sizeof one, &one);  // best effort
        }
      }
    }
    job_ = &g;
    active_ = t;
    pending_ = t - 1;
    ++gen_;
    lk.unlock();
    cv_work_.notify_all();
    g(0);
    lk.lock();
    cv_done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
    lk.unlock();
    if (err) std::rethrow_exception(err);
  }
  // Every helper's CPU set (best effort; EDV_SCAN_NUMA: the NUMA node the batch's objects live on)
  void set_affinity(const cpu_set_t& set) {
    std::unique_lock<std::mutex> busy(run_mu_);
    std::lock_guard<std::mutex> lk(mu_);
    for (std::thread& x : th_) (void)pthread_setaffinity_np(x.native_handle(), sizeof set, &set);
    aff_ = set;
    have_aff_ = true;
  }
  bool same_affinity(const cpu_set_t& set) {
    std::lock_guard<std::mutex> lk(mu_);
    return have_aff_ && CPU_EQUAL(&aff_, &set);
  }
  static HostPool& get() {
    static std::mutex m;
    static HostPool* pool = nullptr;
    static pid_t owner = 0;
    std::lock_guard<std::mutex> g(m);
    if (!pool || owner != getpid()) {  // (after fork the old pool's threads do not exist: leak it)
      pool = new HostPool;
      owner = getpid();
    }
    return *pool;
  }

 private:
  void helper(int w, uint64_t seen) {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_work_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (w >= active_) continue;
      const std::function<void(int)>* f = job_;
      lk.unlock();
      (*f)(w);
      lk.lock();
      if (--pending_ == 0) cv_done_.notify_one();
    }
  }
  std::mutex run_mu_;  // one run() at a time on the helpers
  std::mutex mu_;
  std::condition_variable cv_work_, cv_done_;
  std::vector<std::thread> th_;  // never joined: the helpers live as long as the process
  const std::function<void(int)>* job_ = nullptr;
  uint64_t gen_ = 0;
  int active_ = 0, pending_ = 0;
  cpu_set_t aff_;
  bool have_aff_ = false;
};

}  // namespace
