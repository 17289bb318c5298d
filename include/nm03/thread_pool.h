// nm03/thread_pool.h — fixed-size host worker pool + task groups. Replaces the reference's
// `#pragma omp parallel for schedule(auto)` fork/join (main_parallel.cpp:336-343) with a
// persistent pool that loader, encoder and file-writer tasks of several in-flight batches share,
// so patient and batch boundaries never idle the workers.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace nm03 {

class ThreadPool {
 public:
  explicit ThreadPool(int n) {
    if (n < 1) n = 1;
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  ThreadPool(const ThreadPool&) = delete;
  ThreadPool& operator=(const ThreadPool&) = delete;

  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  int size() const { return (int)workers_.size(); }

 private:
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::vector<std::thread> workers_;
  std::deque<std::function<void()>> q_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false;
};

// Counts outstanding tasks; wait() blocks until all submitted through it finished.
class TaskGroup {
 public:
  explicit TaskGroup(ThreadPool& p) : pool_(p) {}
  void run(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(m_);
      ++pending_;
    }
    pool_.submit([this, f = std::move(f)] {
      f();
      std::lock_guard<std::mutex> g(m_);
      if (--pending_ == 0) cv_.notify_all();
    });
  }
  void wait() {
    std::unique_lock<std::mutex> g(m_);
    cv_.wait(g, [this] { return pending_ == 0; });
  }
  ~TaskGroup() { wait(); }

 private:
  ThreadPool& pool_;
  std::mutex m_;
  std::condition_variable cv_;
  size_t pending_ = 0;
};

}  // namespace nm03
