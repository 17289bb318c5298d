// nm03/thread_pool.h — fixed-size host worker pool + task groups. Replaces the reference's
// `#pragma omp parallel for schedule(auto)` fork/join (main_parallel.cpp:336-343) with a
// persistent pool that loader, encoder and file-writer tasks of several in-flight batches share,
// so patient and batch boundaries never idle the workers.
#pragma once

#include <pthread.h>
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
    stop_flag_.store(true, std::memory_order_relaxed);
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;

  void submit(std::function<void()> f, uint64_t prio = 0) {
    {
      std::lock_guard<std::mutex> g(m_);
      push(std::move(f), prio);
    }
    cv_.notify_one();
  }
  // `n` copies of `f` under one lock (bulk fan-out of a parallel-for).
  void submit_n(int n, const std::function<void()>& f, uint64_t prio = 0) {
    {
      std::lock_guard<std::mutex> g(m_);
      for (int i = 0; i < n; ++i) push(f, prio);
    }
    if (n == 1)
      cv_.notify_one();
    else
      cv_.notify_all();
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
  // Spin (polling the queue size without the lock) for up to spin_us before sleeping on the
  // condition variable: a task submitted shortly after the queue ran dry starts without a futex
  // wake-up and the scheduler's wake-up latency.
  // Measured on the shared boxes (profiles/r3/pool_spin/): 0 / 50 / 200 µs gave 329–398k /
  // 345–398k / 357–398k slices/s over 4 interleaved rounds at equal host CPU per step — equal on
  // quiet boxes, up to +20% when other tenants load the host (delayed wake-ups).
  static constexpr int kSpinUs = 200;
  void loop() {
    for (;;) {
      std::function<void()> f;
      if (queued_.load(std::memory_order_relaxed) == 0) {
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(kSpinUs);
        while (queued_.load(std::memory_order_relaxed) == 0 && !stop_flag_.load(std::memory_order_relaxed) &&
               std::chrono::steady_clock::now() < until)
          __builtin_ia32_pause();
      }
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        std::pop_heap(q_.begin(), q_.end(), later);
        f = std::move(q_.back().f);
        q_.pop_back();
        queued_.store(q_.size(), std::memory_order_relaxed);
      }
      f();
    }
  }
  std::vector<std::thread> workers_;
  std::vector<Task> q_;  // binary heap on (prio, seq)
  std::atomic<size_t> queued_{0};     // q_.size(), readable without the lock (spin phase)
  std::atomic<bool> stop_flag_{false};
  uint64_t seq_ = 0;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
};

inline int64_t thread_cpu_now_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return (int64_t)ts.tv_sec * 1000000000 + ts.tv_nsec;
}

// Counts outstanding tasks; wait() blocks until all submitted through it finished.
class TaskGroup {
 public:
  explicit TaskGroup(ThreadPool& p) : pool_(p) {}
  void run(std::function<void()> f, uint64_t prio = 0) {
    {
      std::lock_guard<std::mutex> g(m_);
      ++pending_;
      pending_a_.store(pending_, std::memory_order_release);
    }
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
    {
      std::lock_guard<std::mutex> g(m_);
      pending_ += (size_t)runners;
      pending_a_.store(pending_, std::memory_order_release);
    }
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
    if (spin > 0 && pending_a_.load(std::memory_order_acquire) != 0) {
      const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(spin);
      while (pending_a_.load(std::memory_order_acquire) != 0 && std::chrono::steady_clock::now() < until)
        __builtin_ia32_pause();
    }
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return pending_ == 0; });
  }
  ~TaskGroup() { wait(); }

 private:
  struct ForEach {
    std::atomic<size_t> next{0};
    size_t n = 0;
    std::function<void(size_t)> fn;
  };
  void done(size_t k) {
    std::lock_guard<std::mutex> g(m_);
    pending_ -= k;
    pending_a_.store(pending_, std::memory_order_release);
    if (pending_ == 0) cv_.notify_all();
  }
  ThreadPool& pool_;
  std::mutex m_;
  std::condition_variable cv_;
  size_t pending_ = 0;
  std::atomic<size_t> pending_a_{0};  // pending_, readable without the lock (wait's spin phase)
};

}  // namespace nm03
