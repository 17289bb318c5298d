// Comm implementations: loopback (threads), self, RCCL over xGMI, and the fork-based launcher.
#include "nm03/comm.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>

#include "nm03/common.h"

namespace nm03 {

// ---------------------------------------------------------------------------------------------
// Serialisation helpers
// ---------------------------------------------------------------------------------------------
void ByteWriter::u32(uint32_t v) {
  for (int i = 0; i < 4; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
void ByteWriter::u64(uint64_t v) {
  for (int i = 0; i < 8; ++i) b.push_back((uint8_t)(v >> (8 * i)));
}
void ByteWriter::f64(double v) {
  uint64_t u;
  std::memcpy(&u, &v, 8);
  u64(u);
}
void ByteWriter::str(const std::string& s) {
  u32((uint32_t)s.size());
  b.insert(b.end(), s.begin(), s.end());
}
uint32_t ByteReader::u32() {
  if (pos + 4 > n) throw std::runtime_error("message underflow");
  uint32_t v = 0;
  for (int i = 0; i < 4; ++i) v |= (uint32_t)p[pos + i] << (8 * i);
  pos += 4;
  return v;
}
uint64_t ByteReader::u64() {
  if (pos + 8 > n) throw std::runtime_error("message underflow");
  uint64_t v = 0;
  for (int i = 0; i < 8; ++i) v |= (uint64_t)p[pos + i] << (8 * i);
  pos += 8;
  return v;
}
double ByteReader::f64() {
  uint64_t u = u64();
  double d;
  std::memcpy(&d, &u, 8);
  return d;
}
std::string ByteReader::str() {
  uint32_t len = u32();
  if (pos + len > n) throw std::runtime_error("message underflow");
  std::string s((const char*)p + pos, len);
  pos += len;
  return s;
}

void Comm::broadcast_bytes(std::vector<uint8_t>& buf, int root) {
  int64_t len = (int64_t)buf.size();
  broadcast(&len, sizeof(len), root);
  buf.resize((size_t)len);
  if (len) broadcast(buf.data(), (size_t)len, root);
}

std::vector<std::vector<uint8_t>> Comm::allgather_bytes(const std::vector<uint8_t>& mine) {
  const int n = size();
  int64_t len = (int64_t)mine.size();
  std::vector<int64_t> lens((size_t)n);
  allgather(&len, sizeof(len), lens.data());
  const int64_t mx = *std::max_element(lens.begin(), lens.end());
  std::vector<uint8_t> send((size_t)std::max<int64_t>(mx, 1), 0), recv((size_t)std::max<int64_t>(mx, 1) * n);
  std::copy(mine.begin(), mine.end(), send.begin());
  allgather(send.data(), send.size(), recv.data());
  std::vector<std::vector<uint8_t>> out((size_t)n);
  for (int r = 0; r < n; ++r)
    out[r].assign(recv.begin() + (size_t)r * send.size(), recv.begin() + (size_t)r * send.size() + lens[r]);
  return out;
}

// ---------------------------------------------------------------------------------------------
// Loopback: shared hub, every collective = deposit + barrier + read + barrier.
// ---------------------------------------------------------------------------------------------
namespace {

struct Hub {
  int n;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<std::vector<uint8_t>> slots;
  explicit Hub(int n_) : n(n_), slots((size_t)n_) {}
  void sync() {
    std::unique_lock<std::mutex> g(m);
    const uint64_t gen = generation;
    if (++arrived == n) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(g, [&] { return generation != gen; });
    }
  }
};

class LoopbackComm final : public Comm {
 public:
  LoopbackComm(std::shared_ptr<Hub> h, int r) : hub_(std::move(h)), rank_(r) {}
  int rank() const override { return rank_; }
  int size() const override { return hub_->n; }
  const char* backend() const override { return "loopback"; }
  void broadcast(void* buf, size_t bytes, int root) override {
    if (rank_ == root) hub_->slots[root].assign((uint8_t*)buf, (uint8_t*)buf + bytes);
    hub_->sync();
    if (rank_ != root) std::memcpy(buf, hub_->slots[root].data(), bytes);
    hub_->sync();
  }
  void allgather(const void* send, size_t bytes, void* recv) override {
    hub_->slots[rank_].assign((const uint8_t*)send, (const uint8_t*)send + bytes);
    hub_->sync();
    for (int r = 0; r < hub_->n; ++r) std::memcpy((uint8_t*)recv + (size_t)r * bytes, hub_->slots[r].data(), bytes);
    hub_->sync();
  }
  void allreduce_sum_i64(int64_t* v, size_t n) override {
    std::vector<int64_t> all(n * hub_->n);
    allgather(v, n * sizeof(int64_t), all.data());
    for (size_t i = 0; i < n; ++i) {
      int64_t s = 0;
      for (int r = 0; r < hub_->n; ++r) s += all[(size_t)r * n + i];
      v[i] = s;
    }
  }
  void allreduce_max_f64(double* v, size_t n) override {
    std::vector<double> all(n * hub_->n);
    allgather(v, n * sizeof(double), all.data());
    for (size_t i = 0; i < n; ++i) {
      double s = all[i];
      for (int r = 1; r < hub_->n; ++r) s = std::max(s, all[(size_t)r * n + i]);
      v[i] = s;
    }
  }
  void barrier() override { hub_->sync(); }

 private:
  std::shared_ptr<Hub> hub_;
  int rank_;
};

class SelfComm final : public Comm {
 public:
  int rank() const override { return 0; }
  int size() const override { return 1; }
  const char* backend() const override { return "self"; }
  void broadcast(void*, size_t, int) override {}
  void allgather(const void* send, size_t bytes, void* recv) override { std::memcpy(recv, send, bytes); }
  void allreduce_sum_i64(int64_t*, size_t) override {}
  void allreduce_max_f64(double*, size_t) override {}
  void barrier() override {}
};

// ---------------------------------------------------------------------------------------------
// RCCL: collectives on a device staging buffer on a private stream.
// ---------------------------------------------------------------------------------------------
void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw DeviceError(std::string(what) + ": " + ncclGetErrorString(r));
}
void hip_ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw DeviceError(std::string(what) + ": " + hipGetErrorString(e));
}

class RcclComm final : public Comm {
 public:
  RcclComm(int rank, int size, const std::vector<uint8_t>& uid, int device) : rank_(rank), size_(size), dev_(device) {
    if (uid.size() != sizeof(ncclUniqueId)) throw DeviceError("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    hip_ck(hipSetDevice(dev_), "hipSetDevice");
    hip_ck(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    nccl_check(ncclCommInitRank(&comm_, size_, id, rank_), "ncclCommInitRank");
  }
  ~RcclComm() override {
    if (comm_) ncclCommDestroy(comm_);
    if (buf_) (void)hipFree(buf_);
    if (stream_) (void)hipStreamDestroy(stream_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* backend() const override { return "rccl"; }

  void broadcast(void* buf, size_t bytes, int root) override {
    if (!bytes) return;
    uint8_t* d = stage(bytes);
    if (rank_ == root) hip_ck(hipMemcpyAsync(d, buf, bytes, hipMemcpyHostToDevice, stream_), "H2D");
    nccl_check(ncclBroadcast(d, d, bytes, ncclUint8, root, comm_, stream_), "ncclBroadcast");
    hip_ck(hipMemcpyAsync(buf, d, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
    wait();
  }
  void allgather(const void* send, size_t bytes, void* recv) override {
    if (!bytes) return;
    uint8_t* d = stage(bytes * (size_t)(size_ + 1));
    uint8_t* dsend = d + bytes * (size_t)size_;
    hip_ck(hipMemcpyAsync(dsend, send, bytes, hipMemcpyHostToDevice, stream_), "H2D");
    nccl_check(ncclAllGather(dsend, d, bytes, ncclUint8, comm_, stream_), "ncclAllGather");
    hip_ck(hipMemcpyAsync(recv, d, bytes * size_, hipMemcpyDeviceToHost, stream_), "D2H");
    wait();
  }
  void allreduce_sum_i64(int64_t* v, size_t n) override { reduce(v, n, ncclInt64, ncclSum); }
  void allreduce_max_f64(double* v, size_t n) override { reduce(v, n, ncclFloat64, ncclMax); }
  void barrier() override {
    int64_t one = 1;
    allreduce_sum_i64(&one, 1);
  }

 private:
  void reduce(void* v, size_t n, ncclDataType_t t, ncclRedOp_t op) {
    if (!n) return;
    const size_t bytes = n * 8;
    uint8_t* d = stage(bytes);
    hip_ck(hipMemcpyAsync(d, v, bytes, hipMemcpyHostToDevice, stream_), "H2D");
    nccl_check(ncclAllReduce(d, d, n, t, op, comm_, stream_), "ncclAllReduce");
    hip_ck(hipMemcpyAsync(v, d, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
    wait();
  }
  uint8_t* stage(size_t bytes) {
    if (bytes > cap_) {
      if (buf_) hip_ck(hipFree(buf_), "hipFree");
      cap_ = std::max<size_t>(bytes, 1 << 20);
      hip_ck(hipMalloc(&buf_, cap_), "hipMalloc comm");
    }
    return (uint8_t*)buf_;
  }
  void wait() {
    // Poll with an async-error check so a dead peer surfaces as an error instead of a hang.
    for (;;) {
      hipError_t q = hipStreamQuery(stream_);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) hip_ck(q, "comm stream");
      ncclResult_t ar = ncclSuccess;
      nccl_check(ncclCommGetAsyncError(comm_, &ar), "ncclCommGetAsyncError");
      nccl_check(ar, "RCCL async error");
      usleep(50);
    }
  }
  int rank_, size_, dev_;
  hipStream_t stream_ = nullptr;
  ncclComm_t comm_ = nullptr;
  void* buf_ = nullptr;
  size_t cap_ = 0;
};

bool read_full(int fd, void* p, size_t n) {
  uint8_t* q = (uint8_t*)p;
  while (n) {
    ssize_t r = ::read(fd, q, n);
    if (r <= 0) return false;
    q += r;
    n -= (size_t)r;
  }
  return true;
}
bool write_full(int fd, const void* p, size_t n) {
  const uint8_t* q = (const uint8_t*)p;
  while (n) {
    ssize_t r = ::write(fd, q, n);
    if (r <= 0) return false;
    q += r;
    n -= (size_t)r;
  }
  return true;
}

}  // namespace

std::vector<std::unique_ptr<Comm>> make_loopback_group(int n) {
  auto hub = std::make_shared<Hub>(n);
  std::vector<std::unique_ptr<Comm>> v;
  for (int i = 0; i < n; ++i) v.push_back(std::make_unique<LoopbackComm>(hub, i));
  return v;
}

std::unique_ptr<Comm> make_self_comm() { return std::make_unique<SelfComm>(); }

std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::vector<uint8_t>& uid, int device) {
  return std::make_unique<RcclComm>(rank, size, uid, device);
}

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::vector<uint8_t> v(sizeof(id));
  std::memcpy(v.data(), &id, sizeof(id));
  return v;
}

int launch_ranks(int n, const std::function<int(int, int, Comm&)>& body, bool use_rccl) {
  if (n <= 1) {
    auto c = make_self_comm();
    return body(0, 1, *c);
  }
  std::vector<int> wfd;
  std::vector<pid_t> kids;
  int my_rank = 0, rfd = -1;
  for (int r = 1; r < n; ++r) {
    int p[2];
    if (pipe(p) != 0) throw std::runtime_error("pipe() failed");
    pid_t pid = fork();
    if (pid < 0) throw std::runtime_error("fork() failed");
    if (pid == 0) {
      ::close(p[1]);
      for (int fd : wfd) ::close(fd);
      my_rank = r;
      rfd = p[0];
      kids.clear();
      break;
    }
    ::close(p[0]);
    wfd.push_back(p[1]);
    kids.push_back(pid);
  }
  int rc = 0;
  try {
    std::unique_ptr<Comm> comm;
    if (my_rank == 0) {
      std::vector<uint8_t> id = use_rccl ? rccl_unique_id() : std::vector<uint8_t>(128, 0);
      for (int fd : wfd) {
        if (!write_full(fd, id.data(), id.size())) throw std::runtime_error("cannot send unique id to a rank");
        ::close(fd);
      }
      if (use_rccl) comm = make_rccl_comm(0, n, id, 0);
    } else {
      std::vector<uint8_t> id(128);
      if (!read_full(rfd, id.data(), id.size())) throw std::runtime_error("cannot receive unique id");
      ::close(rfd);
      if (use_rccl) comm = make_rccl_comm(my_rank, n, id, my_rank);
    }
    if (!comm) comm = make_self_comm();
    rc = body(my_rank, n, *comm);
  } catch (const std::exception& e) {
    fprintf(stderr, "Fatal error on rank %d: %s\n", my_rank, e.what());
    rc = 1;
  }
  if (my_rank != 0) {
    fflush(stdout);
    fflush(stderr);
    _exit(rc);
  }
  for (size_t i = 0; i < kids.size(); ++i) {
    int st = 0;
    if (waitpid(kids[i], &st, 0) < 0) {
      rc = rc ? rc : 1;
      continue;
    }
    const int code = WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0);
    if (code != 0) {
      fprintf(stderr, "Rank %zu exited with status %d\n", i + 1, code);
      if (!rc) rc = code;
    }
  }
  return rc;
}

}  // namespace nm03
