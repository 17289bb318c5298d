// Deferred data plane (nm03/comm.h make_deferred_comm): the shared-memory control plane carries
// the start-up collectives while the device transport (RCCL, or a test fake) comes up on the rank's
// start-up thread; promote() moves every later collective onto it, or — when some rank could not
// bring it up — keeps every rank on the control plane together.
//
// State machine (the start-up thread drives the first three transitions, promote() the rest):
//   kIdle --start_data_plane--> kStarting --(transport made)--> kStarted --settle--> kReady
//                                         \--(uid / make failed)--> kFailed  <--settle (peer failed,
//                                                                              timeout, abort, cancel)
//   fail_data_plane(): kIdle --> kFailed (this rank never starts: its HIP start-up failed)
// Every failure is published through the segment (mark_data_plane_failed, and rank 0's
// publish_uid_failed), so peers settling their own transport abandon it at once instead of waiting
// for a rank that never joins (one failing rank turned into a 30-minute stall).
// promote() is the only collective: the ranks agree on "all ready" over the control plane.
#include <chrono>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <thread>

#include "nm03/comm.h"

namespace nm03 {

namespace {

double mono_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class DeferredComm final : public Comm {
 public:
  DeferredComm(int rank, int size, int device, std::shared_ptr<ShmSegment> seg, double timeout_s, DataPlaneFactory f)
      : rank_(rank), size_(size), dev_(device), seg_(std::move(seg)), timeout_(timeout_s > 0 ? timeout_s : comm_timeout_s()),
        factory_(std::move(f)), host_(make_host_comm(seg_, rank, timeout_s)), t_created_(mono_s()) {}
  ~DeferredComm() override {
    // A transport never promoted (fallback, or the job ended first) is abandoned, not destroyed:
    // destroying an RCCL communicator is a collective with peers that may be gone.
    std::lock_guard<std::mutex> g(m_);
    if (dp_ && !promoted_) dp_->abort_transport();
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* backend() const override { return fallback_ ? "host" : promoted_ ? dp_->backend() : "rccl"; }

  void broadcast(void* buf, size_t bytes, int root) override { plane().broadcast(buf, bytes, root); }
  void allgather(const void* send, size_t bytes, void* recv) override { plane().allgather(send, bytes, recv); }
  void allreduce_sum_i64(int64_t* v, size_t n) override { plane().allreduce_sum_i64(v, n); }
  void allreduce_max_f64(double* v, size_t n) override { plane().allreduce_max_f64(v, n); }
  void barrier() override { plane().barrier(); }
  void sendrecv(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src) override {
    plane().sendrecv(send, sbytes, dst, recv, rbytes, src);
  }
  // Device data always goes over the data plane (promoting implicitly: every rank reaches these together).
  void sendrecv_device(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src,
                       void* stream) override {
    promote();
    if (fallback_) return Comm::sendrecv_device(send, sbytes, dst, recv, rbytes, src, stream);  // staged, host plane
    dp_->sendrecv_device(send, sbytes, dst, recv, rbytes, src, stream);
  }
  int64_t allreduce_sum_i64_device(int64_t* v, void* stream) override {
    promote();
    if (fallback_) return Comm::allreduce_sum_i64_device(v, stream);
    return dp_->allreduce_sum_i64_device(v, stream);
  }
  bool device_native() const override { return promoted_ && dp_->device_native(); }
  int transport_size() const override { return promoted_ ? dp_->transport_size() : -1; }
  int transport_rank() const override { return promoted_ ? dp_->transport_rank() : -1; }
  int transport_device() const override { return promoted_ ? dp_->transport_device() : -1; }
  void ready() override { promote(); }

  void start_data_plane() override {
    {
      std::lock_guard<std::mutex> g(m_);
      if (state_ != kIdle) return;
      state_ = kStarting;
      t_start_ = mono_s();
    }
    std::unique_ptr<Comm> c;
    std::exception_ptr err;
    try {
      std::vector<uint8_t> uid;
      if (rank_ == 0) {
        try {
          uid = factory_.unique_id();
        } catch (...) {
          seg_->publish_uid_failed();  // the other ranks fail fast and agree on the fallback
          throw;
        }
        seg_->publish_uid(uid);
      } else {
        uid = seg_->wait_uid(rank_, timeout_);
      }
      c = factory_.make(rank_, size_, uid, dev_, seg_, timeout_);
      if (!c) throw CommError("data plane factory returned no transport");
    } catch (...) {
      err = std::current_exception();
      seg_->mark_data_plane_failed(rank_);
    }
    {
      std::lock_guard<std::mutex> g(m_);
      dp_ = std::move(c);
      err_ = err;
      state_ = err ? kFailed : kStarted;
    }
    cv_.notify_all();
  }

  void fail_data_plane(const std::string& why) override {
    {
      std::lock_guard<std::mutex> g(m_);
      if (state_ != kIdle) return;
      state_ = kFailed;
      err_ = std::make_exception_ptr(CommError(why));
      t_start_ = mono_s();
    }
    seg_->mark_data_plane_failed(rank_);
    if (rank_ == 0) seg_->publish_uid_failed();
    cv_.notify_all();
  }

  void settle_data_plane(const std::atomic<bool>* cancel) override {
    {
      std::lock_guard<std::mutex> g(m_);
      if (state_ != kStarted) return;  // idle, failed or already settled
      state_ = kSettling;
    }
    const double t0 = mono_s();
    const State end = settle_loop(cancel);
    {
      std::lock_guard<std::mutex> g(m_);
      state_ = end;
      times_.settle_s = mono_s() - t0;
      if (end == kReady) times_.init_upper_s = mono_s() - t_start_;
    }
    cv_.notify_all();
  }

  // Every rank brings its data plane up (settled on the start-up thread, or here), then the ranks
  // agree on the control plane: all ready → every later collective on the data plane; any rank
  // failed (a transport error, a timeout: not a dead peer — the job abort flag still ends the job)
  // → all stay on the control plane and say so (backend() "host", fallback_error()).
  void promote() override {
    if (promoted_ || fallback_) return;
    const double t0 = mono_s();
    bool start_here = false;
    {
      std::lock_guard<std::mutex> g(m_);
      start_here = state_ == kIdle;
    }
    if (start_here) start_data_plane();  // nobody started it: start it on this thread
    settle_data_plane(nullptr);            // a no-op when the start-up thread settled it
    std::string err;
    try {
      std::unique_lock<std::mutex> g(m_);
      // Bounded, abort-aware wait for a start-up thread still inside start/settle. That thread began
      // before t0 (else state_ was kIdle and this thread started it) and is itself bounded: the uid
      // wait by timeout_, the settle loop by its own timeout_ — so this net must outlast both, or a
      // slow start (a loaded host) ends here as a job abort instead of the settle's agreed fallback.
      const double deadline = t0 + 2 * timeout_ + 1.0;
      while (state_ == kStarting || state_ == kSettling) {
        cv_.wait_for(g, std::chrono::milliseconds(2));
        if (state_ != kStarting && state_ != kSettling) break;
        seg_->check_abort(rank_);
        if (mono_s() > deadline) {
          seg_->raise_abort(rank_);
          throw CommError("data plane start-up timed out on rank " + std::to_string(rank_));
        }
      }
      if (state_ == kFailed) std::rethrow_exception(err_);
    } catch (const std::exception& e) {
      if (seg_->aborted()) throw;  // a peer died: the job ends, no fallback
      err = e.what();
    }
    int64_t failed = err.empty() ? 0 : 1;
    host_->allreduce_sum_i64(&failed, 1);  // agreement on the control plane
    times_.wait_s = mono_s() - t0;
    times_.start_s = t_start_ > 0 ? t_start_ - t_created_ : -1;
    if (times_.init_upper_s == 0 && t_start_ > 0) times_.init_upper_s = mono_s() - t_start_;
    if (failed == 0) {
      promoted_ = true;
      dp_->set_abort_segment(seg_);
      return;
    }
    fallback_ = true;
    {
      std::lock_guard<std::mutex> g(m_);
      if (dp_) dp_->abort_transport();  // ready here, but a peer's is not: nobody uses it
    }
    fallback_error_ = err.empty() ? std::to_string(failed) + " rank(s) could not bring the data plane up" : err;
  }
  std::string fallback_error() const override { return fallback_error_; }
  DataPlaneTimes data_plane_times() const override { return times_; }
  void set_abort_segment(std::shared_ptr<ShmSegment> seg) override {
    std::lock_guard<std::mutex> g(m_);  // dp_ is written by the start-up thread
    if (dp_) dp_->set_abort_segment(std::move(seg));
  }

 private:
  enum State { kIdle, kStarting, kStarted, kSettling, kReady, kFailed };

  // Polls this rank's transport until it is ready, or abandons it: a peer's start failed, the job
  // was aborted (a rank died), the caller cancelled, or the deadline passed. Runs without m_ held
  // (dp_ is not replaced while the state is kSettling).
  State settle_loop(const std::atomic<bool>* cancel) {
    const double deadline = mono_s() + timeout_;
    auto give_up = [&](const std::string& why, bool publish) {
      if (publish) seg_->mark_data_plane_failed(rank_);
      dp_->abort_transport();
      err_ = std::make_exception_ptr(CommError(why));
      return kFailed;
    };
    try {
      for (;;) {
        if (dp_->poll_ready()) return kReady;
        if (const int f = seg_->data_plane_failed_rank(); f >= 0 && f != rank_)
          return give_up("rank " + std::to_string(f) + " could not start the data plane", false);
        if (seg_->aborted()) {
          const int r = seg_->abort_rank();
          return give_up("rank " + std::to_string(r) + " failed; job aborted", false);
        }
        if (cancel && cancel->load(std::memory_order_acquire)) return give_up("start-up cancelled", true);
        if (mono_s() > deadline)
          return give_up("data plane initialisation timed out after " + std::to_string((int)timeout_) + " s on rank " +
                             std::to_string(rank_),
                         true);
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
    } catch (const std::exception& e) {  // the transport reported an error
      seg_->mark_data_plane_failed(rank_);
      dp_->abort_transport();
      err_ = std::current_exception();
      return kFailed;
    }
  }

  Comm& plane() { return promoted_ ? *dp_ : *host_; }
  int rank_, size_, dev_;
  std::shared_ptr<ShmSegment> seg_;
  double timeout_;
  DataPlaneFactory factory_;
  std::unique_ptr<Comm> host_, dp_;
  double t_created_, t_start_ = 0;
  std::mutex m_;
  std::condition_variable cv_;
  State state_ = kIdle;
  std::exception_ptr err_;
  bool promoted_ = false;  // only the rank's main thread reads/writes it
  bool fallback_ = false;  // the data plane failed on some rank: the control plane carries everything
  std::string fallback_error_;
  DataPlaneTimes times_;
};

}  // namespace

std::unique_ptr<Comm> make_deferred_comm(int rank, int size, int device, std::shared_ptr<ShmSegment> seg,
                                         double timeout_s, DataPlaneFactory factory) {
  if (!seg) throw CommError("deferred comm needs a shared segment");
  if (!factory.unique_id || !factory.make) throw CommError("deferred comm needs a data plane factory");
  return std::make_unique<DeferredComm>(rank, size, device, std::move(seg), timeout_s, std::move(factory));
}

std::unique_ptr<Comm> make_deferred_rccl_comm(int rank, int size, int device, std::shared_ptr<ShmSegment> seg,
                                              double timeout_s) {
  return make_deferred_comm(rank, size, device, std::move(seg), timeout_s, rccl_data_plane());
}

}  // namespace nm03
