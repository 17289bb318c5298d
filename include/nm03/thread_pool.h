// nm03/thread_pool.h — fixed-size host worker pool + task groups. Replaces the reference's
// `#pragma omp parallel for schedule(auto)` fork/join (main_parallel.cpp:336-343) with a
// persistent pool that loader, encoder and file-writer tasks of several in-flight batches share,
// so patient and batch boundaries never idle the workers.
#pragma once

#include <linux/futex.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <unistd.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace nm03 {

// Tasks carry a priority (lower runs first; FIFO among equals). The engine uses the batch index,
// so the loads and exports of earlier batches overtake later ones: the first batch reaches the GPU
// after ~batch/threads loads instead of after every in-flight slot's loads (pipeline fill), and the
// last batches' exports are not queued behind anything (drain).
//
// Idle workers spin on the queue size, then sleep on a futex word that every push bumps (an
// eventcount): a wake-up costs a futex wake only when a worker sleeps, and woken workers do not
// queue up again on a condition variable's mutex when they return from the wait. (A spin-then-block
// lock for the heap was tried in round 6 and made it worse: 13% of the pool's CPU in try_lock,
// profiles/r6/cpu_profile/.)
class ThreadPool {
 public:
  // `on_start(i)` runs first on worker thread i (e.g. CPU pinning).
  explicit ThreadPool(int n, std::function<void(int)> on_start = {}) {
    if (n < 1) n = 1;
    for (int i = 0; i < n; ++i)
      workers_.emplace_back([this, on_start, i] {
        pthread_setname_np(pthread_self(), "nm03-pool");  // per-thread CPU accounting (bench.py)
        worker_index_ref() = i;
        if (on_start) on_start(i);
        loop();
      });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    stop_flag_.store(true, std::memory_order_seq_cst);
    wake(1 << 30);
    for (auto& t : workers_) t.join();
  }
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;

  void submit(std::function<void()> f, uint64_t prio = 0) {
    {
      std::lock_guard<std::mutex> g(m_);
      push(std::move(f), prio);
    }
    wake(1);
  }
  // `n` copies of `f` under one lock (bulk fan-out of a parallel-for).
  void submit_n(int n, const std::function<void()>& f, uint64_t prio = 0) {
    {
      std::lock_guard<std::mutex> g(m_);
      for (int i = 0; i < n; ++i) push(f, prio);
    }
    wake(n);
  }
  int size() const { return (int)workers_.size(); }
  // Index of the calling pool worker thread (-1 outside any pool).
  static int current_worker() { return worker_index_ref(); }

 private:
  struct Task {
    uint64_t prio, seq;
    std::function<void()> f;
  };
  static int& worker_index_ref() {
    static thread_local int idx = -1;
    return idx;
  }
  static bool later(const Task& a, const Task& b) { return a.prio != b.prio ? a.prio > b.prio : a.seq > b.seq; }
  void push(std::function<void()> f, uint64_t prio) {
    q_.push_back(Task{prio, seq_++, std::move(f)});
    std::push_heap(q_.begin(), q_.end(), later);
    queued_.store(q_.size(), std::memory_order_relaxed);
  }
  // After a push (outside the lock): bump the eventcount, wake up to n sleepers.
  void wake(int n) {
    wake_seq_.fetch_add(1, std::memory_order_seq_cst);
    if (sleepers_.load(std::memory_order_seq_cst) > 0)
      syscall(SYS_futex, reinterpret_cast<uint32_t*>(&wake_seq_), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
  }
  // Spin (polling the queue size without the lock) for up to spin_us before sleeping: a task
  // submitted shortly after the queue ran dry starts without a futex wake-up and the scheduler's
  // wake-up latency.
  // Measured on the shared boxes (profiles/r3/pool_spin/): 0 / 50 / 200 µs gave 329–398k /
  // 345–398k / 357–398k slices/s over 4 interleaved rounds at equal host CPU per step — equal on
  // quiet boxes, up to +20% when other tenants load the host (delayed wake-ups).
  static constexpr int kSpinUs = 200;
  // NM03_POOL_SPIN_US overrides kSpinUs (A/B experiments).
  static int spin_us() {
    static const int v = [] {
      const char* e = std::getenv("NM03_POOL_SPIN_US");
      return e && *e ? std::max(0, std::atoi(e)) : kSpinUs;
    }();
    return v;
  }
  void loop() {
    const int spin = spin_us();
    for (;;) {
      if (queued_.load(std::memory_order_relaxed) == 0 && spin > 0) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin);
        // the clock is read every 64 polls, not every poll (a vDSO call each)
        for (int k = 0; queued_.load(std::memory_order_relaxed) == 0 && !stop_flag_.load(std::memory_order_relaxed);
             ++k) {
          __builtin_ia32_pause();
          if ((k & 63) == 63 && std::chrono::steady_clock::now() >= until) break;
        }
      }
      std::function<void()> f;
      uint32_t seq = 0;
      {
        std::lock_guard<std::mutex> g(m_);
        if (!q_.empty()) {
          std::pop_heap(q_.begin(), q_.end(), later);
          f = std::move(q_.back().f);
          q_.pop_back();
          queued_.store(q_.size(), std::memory_order_relaxed);
        } else {
          if (stop_) return;
          seq = wake_seq_.load(std::memory_order_seq_cst);  // a push after this unlock bumps it
        }
      }
      if (f) {
        f();
        continue;
      }
      sleepers_.fetch_add(1, std::memory_order_seq_cst);
      while (wake_seq_.load(std::memory_order_seq_cst) == seq && !stop_flag_.load(std::memory_order_seq_cst)) {
        timespec ts{0, 50 * 1000 * 1000};  // bounded: a missed wake-up costs at most this
        syscall(SYS_futex, reinterpret_cast<uint32_t*>(&wake_seq_), FUTEX_WAIT_PRIVATE, seq, &ts, nullptr, 0);
      }
      sleepers_.fetch_sub(1, std::memory_order_seq_cst);
    }
  }
  std::vector<std::thread> workers_;
  std::vector<Task> q_;  // binary heap on (prio, seq)
  std::atomic<size_t> queued_{0};     // q_.size(), readable without the lock (spin phase)
  std::atomic<bool> stop_flag_{false};
  std::atomic<uint32_t> wake_seq_{0};  // eventcount: bumped by every push (futex word)
  std::atomic<int> sleepers_{0};
  uint64_t seq_ = 0;
  std::mutex m_;
  bool stop_ = false;
};

inline int64_t thread_cpu_now_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

// Counts outstanding tasks; wait() blocks until all submitted through it finished. The count is an
// atomic: only the task that brings it to zero takes the mutex (to wake a sleeping waiter), so the
// 16 runners of a for_each finishing together do not queue on a lock.
class TaskGroup {
 public:
  explicit TaskGroup(ThreadPool& p) : pool_(p) {}
  void run(std::function<void()> f, uint64_t prio = 0) {
    pending_.fetch_add(1, std::memory_order_acq_rel);
    pool_.submit(
        [this, f = std::move(f)] {
          f();
          done(1);
        },
        prio);
  }
  // fn(i) for i in [0, n): min(n, pool size, max_runners) runners pull indices from a shared
  // counter. `max_runners` > 0 bounds how many items run concurrently (file creation on tmpfs: the
  // inode allocation and release serialise on per-filesystem locks, so 16 concurrent creators
  // cost 3.7x the CPU per file of one, tools/create_probe.cpp); the other workers take other
  // tasks meanwhile. With `cpu_ns`, each runner adds the thread CPU time of its whole share (two
  // clock reads per runner instead of two per item: a thread-CPU clock read is a system call).
  void for_each(size_t n, std::function<void(size_t)> fn, uint64_t prio = 0, std::atomic<int64_t>* cpu_ns = nullptr,
                int max_runners = 0) {
    if (n == 0) return;
    size_t cap = (size_t)pool_.size();
    if (max_runners > 0) cap = std::min(cap, (size_t)max_runners);
    const int runners = (int)std::min<size_t>(n, cap);
    auto st = std::make_shared<ForEach>();
    st->n = n;
    st->fn = std::move(fn);
    pending_.fetch_add((size_t)runners, std::memory_order_acq_rel);
    pool_.submit_n(
        runners,
        [this, st, cpu_ns] {
          const int64_t c0 = cpu_ns ? thread_cpu_now_ns() : 0;
          for (size_t i; (i = st->next.fetch_add(1)) < st->n;) st->fn(i);
          if (cpu_ns) cpu_ns->fetch_add(thread_cpu_now_ns() - c0, std::memory_order_relaxed);
          done(1);
        },
        prio);
  }
  // With spin_us > 0, spins that long on the pending count before sleeping: the waiter then
  // continues without a wake-up.
  void wait(int spin_us = 0) {
    const int spin = spin_us;
    if (spin > 0 && pending_.load(std::memory_order_acquire) != 0) {
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin);
      while (pending_.load(std::memory_order_acquire) != 0 && std::chrono::steady_clock::now() < until)
        __builtin_ia32_pause();
    }
    // Under m_ even when the count is already zero: the finishing task may still hold it (done()).
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return pending_.load(std::memory_order_acquire) == 0; });
  }
  ~TaskGroup() { wait(); }

 private:
  struct ForEach {
    std::atomic<size_t> next{0};
    size_t n = 0;
    std::function<void(size_t)> fn;
  };
  void done(size_t k) {
    // Lock-free unless this task may finish the group. The final decrement happens under m_: a
    // waiter that sees the count reach zero without the lock then takes m_ before it returns (and
    // the group may be destroyed), so it cannot return while the finishing task still uses m_ or cv_.
    size_t cur = pending_.load(std::memory_order_acquire);
    while (cur > k)
      if (pending_.compare_exchange_weak(cur, cur - k, std::memory_order_acq_rel, std::memory_order_acquire)) return;
    std::lock_guard<std::mutex> g(m_);
    if (pending_.fetch_sub(k, std::memory_order_acq_rel) == k) cv_.notify_all();
  }
  ThreadPool& pool_;
  std::mutex m_;
  std::condition_variable cv_;
  std::atomic<size_t> pending_{0};
};

}  // namespace nm03
