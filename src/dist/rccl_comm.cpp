// RCCL communicator (nm03/comm.h): collectives on a device staging buffer on a private stream,
// i.e. over xGMI between the MI355X of one node. The communicator is created non-blocking
// (ncclConfig_t.blocking = 0) so that initialisation, like every later wait, is a bounded poll:
// a peer that died or never arrived ends in ncclCommAbort + CommError after NM03_COMM_TIMEOUT_S
// (or at once when the launcher raised the job abort flag), never in a hang.
#include <dlfcn.h>
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <exception>
#include <mutex>
#include <thread>
#include <type_traits>

#include "nm03/comm.h"

namespace nm03 {

namespace {

double mono_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void hip_ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw CommError(std::string(what) + ": " + hipGetErrorString(e));
}

// RCCL's entry points, resolved from librccl when the first communicator needs them. Linking
// librccl (573 MB, with its device code registered with the HIP runtime by its static
// constructors) put ≈ 3 ms into every process's start-up before main, single-rank runs included;
// loaded here it costs a multi-rank job nothing on the critical path (the deferred communicator
// starts RCCL on the start-up thread while the ranks process).
struct RcclApi {
#define NM03_RCCL_FN(name) decltype(&::name) name = nullptr;
  NM03_RCCL_FN(ncclGetUniqueId)
  NM03_RCCL_FN(ncclCommInitRankConfig)
  NM03_RCCL_FN(ncclGetErrorString)
  NM03_RCCL_FN(ncclBroadcast)
  NM03_RCCL_FN(ncclAllGather)
  NM03_RCCL_FN(ncclAllReduce)
  NM03_RCCL_FN(ncclSend)
  NM03_RCCL_FN(ncclRecv)
  NM03_RCCL_FN(ncclGroupStart)
  NM03_RCCL_FN(ncclGroupEnd)
  NM03_RCCL_FN(ncclCommCount)
  NM03_RCCL_FN(ncclCommUserRank)
  NM03_RCCL_FN(ncclCommCuDevice)
  NM03_RCCL_FN(ncclCommGetAsyncError)
  NM03_RCCL_FN(ncclCommAbort)
  NM03_RCCL_FN(ncclCommDestroy)
#undef NM03_RCCL_FN
  std::string error;  // why the library or a symbol could not be loaded (empty: usable)
};

const RcclApi& rccl_api() {
  static const RcclApi api = [] {
    RcclApi a;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen(ROCM_LIB_DIR "/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      a.error = std::string("cannot load librccl.so.1: ") + (e ? e : "unknown error");
      return a;
    }
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      if (!fn && a.error.empty()) a.error = std::string("librccl.so.1 lacks ") + name;
    };
#define NM03_RCCL_SYM(name) sym(a.name, #name);
    NM03_RCCL_SYM(ncclGetUniqueId)
    NM03_RCCL_SYM(ncclCommInitRankConfig)
    NM03_RCCL_SYM(ncclGetErrorString)
    NM03_RCCL_SYM(ncclBroadcast)
    NM03_RCCL_SYM(ncclAllGather)
    NM03_RCCL_SYM(ncclAllReduce)
    NM03_RCCL_SYM(ncclSend)
    NM03_RCCL_SYM(ncclRecv)
    NM03_RCCL_SYM(ncclGroupStart)
    NM03_RCCL_SYM(ncclGroupEnd)
    NM03_RCCL_SYM(ncclCommCount)
    NM03_RCCL_SYM(ncclCommUserRank)
    NM03_RCCL_SYM(ncclCommCuDevice)
    NM03_RCCL_SYM(ncclCommGetAsyncError)
    NM03_RCCL_SYM(ncclCommAbort)
    NM03_RCCL_SYM(ncclCommDestroy)
#undef NM03_RCCL_SYM
    return a;
  }();
  if (!api.error.empty()) throw CommError(api.error);
  return api;
}

class RcclComm final : public Comm {
 public:
  RcclComm(int rank, int size, const std::vector<uint8_t>& uid, int device, std::shared_ptr<ShmSegment> seg,
           double timeout_s, bool settle_now = true)
      : rank_(rank), size_(size), dev_(device), seg_(std::move(seg)),
        timeout_(timeout_s > 0 ? timeout_s : comm_timeout_s()) {
    if (uid.size() != sizeof(ncclUniqueId)) throw CommError("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    hip_ck(hipSetDevice(dev_), "hipSetDevice");
    hip_ck(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = rccl_api().ncclCommInitRankConfig(&comm_, size_, id, rank_, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      release();
      throw CommError(std::string("ncclCommInitRank: ") + rccl_api().ncclGetErrorString(r));
    }
    if (!settle_now) return;
    try {
      ready();
    } catch (...) {
      release();
      throw;
    }
  }
  void ready() override {
    if (settled_) return;
    if (!comm_) throw CommError("RCCL communicator was aborted");
    settle("ncclCommInitRank");
    settled_ = true;
  }
  bool poll_ready() override {
    if (settled_) return true;
    if (!comm_) throw CommError("RCCL communicator was aborted");
    ncclResult_t ar = ncclSuccess;
    const ncclResult_t q = rccl_api().ncclCommGetAsyncError(comm_, &ar);
    if (q != ncclSuccess) fail(std::string("ncclCommInitRank: ncclCommGetAsyncError: ") + rccl_api().ncclGetErrorString(q));
    if (ar == ncclInProgress) return false;
    if (ar != ncclSuccess) fail(std::string("ncclCommInitRank: ") + rccl_api().ncclGetErrorString(ar));
    settled_ = true;
    return true;
  }
  void abort_transport() override {
    if (comm_) {
      (void)rccl_api().ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }
  ~RcclComm() override { release(); }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* backend() const override { return "rccl"; }

  void broadcast(void* buf, size_t bytes, int root) override {
    if (!bytes) return;
    uint8_t* d = stage(bytes);
    if (rank_ == root) hip_ck(hipMemcpyAsync(d, buf, bytes, hipMemcpyHostToDevice, stream_), "H2D");
    issue(rccl_api().ncclBroadcast(d, d, bytes, ncclUint8, root, comm_, stream_), "ncclBroadcast");
    hip_ck(hipMemcpyAsync(buf, d, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
    wait("ncclBroadcast");
  }
  void allgather(const void* send, size_t bytes, void* recv) override {
    if (!bytes) return;
    uint8_t* d = stage(bytes * (size_t)(size_ + 1));
    uint8_t* dsend = d + bytes * (size_t)size_;
    hip_ck(hipMemcpyAsync(dsend, send, bytes, hipMemcpyHostToDevice, stream_), "H2D");
    issue(rccl_api().ncclAllGather(dsend, d, bytes, ncclUint8, comm_, stream_), "ncclAllGather");
    hip_ck(hipMemcpyAsync(recv, d, bytes * size_, hipMemcpyDeviceToHost, stream_), "D2H");
    wait("ncclAllGather");
  }
  void allreduce_sum_i64(int64_t* v, size_t n) override { reduce(v, n, ncclInt64, ncclSum); }
  void allreduce_max_f64(double* v, size_t n) override { reduce(v, n, ncclFloat64, ncclMax); }
  void barrier() override {
    int64_t one = 1;
    allreduce_sum_i64(&one, 1);
  }
  void sendrecv(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src) override {
    if (dst < 0) sbytes = 0;
    if (src < 0) rbytes = 0;
    if (!sbytes && !rbytes) return;
    uint8_t* d = stage(sbytes + rbytes);
    uint8_t* drecv = d + sbytes;
    if (sbytes) hip_ck(hipMemcpyAsync(d, send, sbytes, hipMemcpyHostToDevice, stream_), "H2D");
    // One group: the send to the successor and the receive from the predecessor progress
    // together (a halo exchange where every rank sends first would otherwise deadlock).
    issue(rccl_api().ncclGroupStart(), "ncclGroupStart");
    if (sbytes) issue(rccl_api().ncclSend(d, sbytes, ncclUint8, dst, comm_, stream_), "ncclSend");
    if (rbytes) issue(rccl_api().ncclRecv(drecv, rbytes, ncclUint8, src, comm_, stream_), "ncclRecv");
    issue(rccl_api().ncclGroupEnd(), "ncclGroupEnd");
    if (rbytes) hip_ck(hipMemcpyAsync(recv, drecv, rbytes, hipMemcpyDeviceToHost, stream_), "D2H");
    wait("ncclSend/ncclRecv");
  }
  // z-slab planes straight between device buffers on the caller's stream: nothing staged, nothing
  // waited for here (the stream orders the exchange behind the producer and before the consumers).
  void sendrecv_device(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src,
                       void* stream) override {
    if (dst < 0) sbytes = 0;
    if (src < 0) rbytes = 0;
    if (!sbytes && !rbytes) return;
    bind_device();
    ready();
    if (!comm_) throw CommError("RCCL communicator was aborted");
    if (seg_) seg_->check_abort(rank_);
    auto st = static_cast<hipStream_t>(stream);
    issue(rccl_api().ncclGroupStart(), "ncclGroupStart");
    if (sbytes) issue(rccl_api().ncclSend(send, sbytes, ncclUint8, dst, comm_, st), "ncclSend");
    if (rbytes) issue(rccl_api().ncclRecv(recv, rbytes, ncclUint8, src, comm_, st), "ncclRecv");
    issue(rccl_api().ncclGroupEnd(), "ncclGroupEnd");
  }
  int64_t allreduce_sum_i64_device(int64_t* v, void* stream) override {
    bind_device();
    ready();
    if (!comm_) throw CommError("RCCL communicator was aborted");
    if (seg_) seg_->check_abort(rank_);
    auto st = static_cast<hipStream_t>(stream);
    if (!h_word_) hip_ck(hipHostMalloc((void**)&h_word_, 8, hipHostMallocDefault), "hipHostMalloc");
    issue(rccl_api().ncclAllReduce(v, v, 1, ncclInt64, ncclSum, comm_, st), "ncclAllReduce");
    hip_ck(hipMemcpyAsync(h_word_, v, 8, hipMemcpyDeviceToHost, st), "D2H");
    wait("ncclAllReduce (device)", st);
    return *h_word_;
  }
  bool device_native() const override { return true; }
  int transport_size() const override {
    if (!settled_) return -1;
    int n = -1;
    if (!comm_ || rccl_api().ncclCommCount(comm_, &n) != ncclSuccess) return -1;
    return n;
  }
  int transport_rank() const override {
    if (!settled_) return -1;
    int r = -1;
    if (!comm_ || rccl_api().ncclCommUserRank(comm_, &r) != ncclSuccess) return -1;
    return r;
  }
  int transport_device() const override {
    if (!settled_) return -1;
    int d = -1;
    if (!comm_ || rccl_api().ncclCommCuDevice(comm_, &d) != ncclSuccess) return -1;
    return d;
  }
  void set_abort_segment(std::shared_ptr<ShmSegment> seg) override { seg_ = std::move(seg); }

 private:
  void reduce(void* v, size_t n, ncclDataType_t t, ncclRedOp_t op) {
    if (!n) return;
    const size_t bytes = n * 8;
    uint8_t* d = stage(bytes);
    hip_ck(hipMemcpyAsync(d, v, bytes, hipMemcpyHostToDevice, stream_), "H2D");
    issue(rccl_api().ncclAllReduce(d, d, n, t, op, comm_, stream_), "ncclAllReduce");
    hip_ck(hipMemcpyAsync(v, d, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
    wait("ncclAllReduce");
  }
  // Collectives may run on any thread of the rank (the CLI's main thread never called hipSetDevice:
  // the start-up thread owns the device until the engine exists): every entry point that makes HIP
  // calls selects the communicator's device first, so staging buffers and copies land on it, not on
  // the calling thread's default device 0.
  void bind_device() { hip_ck(hipSetDevice(dev_), "hipSetDevice"); }
  uint8_t* stage(size_t bytes) {
    bind_device();
    ready();
    if (!comm_) throw CommError("RCCL communicator was aborted");
    if (seg_) seg_->check_abort(rank_);
    if (bytes > cap_) {
      if (buf_) hip_ck(hipFree(buf_), "hipFree");
      buf_ = nullptr;
      cap_ = std::max<size_t>(bytes, 1 << 20);
      hip_ck(hipMalloc(&buf_, cap_), "hipMalloc comm");
    }
    return (uint8_t*)buf_;
  }
  // A non-blocking communicator may return ncclInProgress from an enqueue: poll until settled.
  void issue(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return;
    if (r != ncclInProgress) fail(std::string(what) + ": " + rccl_api().ncclGetErrorString(r));
    settle(what);
  }
  void settle(const char* what) {
    const double deadline = mono_s() + timeout_;
    for (;;) {
      ncclResult_t ar = ncclSuccess;
      const ncclResult_t q = rccl_api().ncclCommGetAsyncError(comm_, &ar);
      if (q != ncclSuccess) fail(std::string(what) + ": ncclCommGetAsyncError: " + rccl_api().ncclGetErrorString(q));
      if (ar == ncclSuccess) return;
      if (ar != ncclInProgress) fail(std::string(what) + ": " + rccl_api().ncclGetErrorString(ar));
      poll_guards(what, deadline);
    }
  }
  void wait(const char* what, hipStream_t s = nullptr) {
    const double deadline = mono_s() + timeout_;
    for (;;) {
      const hipError_t q = hipStreamQuery(s ? s : stream_);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) fail(std::string(what) + ": " + hipGetErrorString(q));
      ncclResult_t ar = ncclSuccess;
      if (rccl_api().ncclCommGetAsyncError(comm_, &ar) != ncclSuccess || (ar != ncclSuccess && ar != ncclInProgress))
        fail(std::string(what) + ": RCCL async error: " + rccl_api().ncclGetErrorString(ar));
      poll_guards(what, deadline);
    }
  }
  void poll_guards(const char* what, double deadline) {
    if (seg_ && seg_->aborted()) {
      const int r = seg_->abort_rank();
      fail(r == rank_ ? std::string(what) + ": aborted" : "rank " + std::to_string(r) + " failed; job aborted");
    }
    if (mono_s() > deadline) {
      if (seg_) seg_->raise_abort(rank_);
      fail(std::string(what) + " timed out after " + std::to_string((int)timeout_) + " s on rank " +
           std::to_string(rank_) + "; set NM03_COMM_TIMEOUT_S to wait longer");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  [[noreturn]] void fail(const std::string& msg) {
    if (comm_) {
      (void)rccl_api().ncclCommAbort(comm_);
      comm_ = nullptr;
    }
    throw CommError(msg);
  }
  void release() {
    if (comm_) {
      // A healthy communicator is destroyed; an aborted one was already released by fail().
      (void)rccl_api().ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
    if (buf_) (void)hipFree(buf_);
    buf_ = nullptr;
    if (h_word_) (void)hipHostFree(h_word_);
    h_word_ = nullptr;
    if (stream_) (void)hipStreamDestroy(stream_);
    stream_ = nullptr;
  }
  int rank_, size_, dev_;
  std::shared_ptr<ShmSegment> seg_;
  double timeout_;
  hipStream_t stream_ = nullptr;
  ncclComm_t comm_ = nullptr;
  void* buf_ = nullptr;
  size_t cap_ = 0;
  int64_t* h_word_ = nullptr;  // pinned landing word of allreduce_sum_i64_device
  bool settled_ = false;       // ncclCommInitRankConfig completed (ready())
};

}  // namespace

std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::vector<uint8_t>& uid, int device,
                                     std::shared_ptr<ShmSegment> seg, double timeout_s, bool settle_now) {
  return std::make_unique<RcclComm>(rank, size, uid, device, std::move(seg), timeout_s, settle_now);
}

DataPlaneFactory rccl_data_plane() {
  DataPlaneFactory f;
  f.unique_id = [] { return rccl_unique_id(); };
  f.make = [](int rank, int size, const std::vector<uint8_t>& uid, int device, std::shared_ptr<ShmSegment> seg,
              double timeout_s) { return make_rccl_comm(rank, size, uid, device, std::move(seg), timeout_s, /*settle_now=*/false); };
  return f;
}

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  const ncclResult_t r = rccl_api().ncclGetUniqueId(&id);
  if (r != ncclSuccess) throw CommError(std::string("ncclGetUniqueId: ") + rccl_api().ncclGetErrorString(r));
  std::vector<uint8_t> v(sizeof(id));
  std::memcpy(v.data(), &id, sizeof(id));
  return v;
}

}  // namespace nm03
