// Comm implementations: loopback (threads), self, host (shared segment across processes), and the
// fork-based launcher with its supervisor. RCCL lives in rccl_comm.cpp, the segment in shm.cpp.
#include "nm03/comm.h"

#include <signal.h>
#include <sys/prctl.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <thread>

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

std::vector<RankDevice> gather_rank_devices(Comm& comm, const RankDevice& m) {
  ByteWriter w;
  w.i32(m.device);
  w.str(m.bus_id);
  w.i32(m.node);
  w.str(m.cpus);
  w.i32(m.threads);
  w.i32(m.transport_size);
  w.i32(m.transport_device);
  w.str(m.error);
  std::vector<RankDevice> out;
  for (const auto& b : comm.allgather_bytes(w.b)) {
    ByteReader r(b.data(), b.size());
    RankDevice d;
    d.device = r.i32();
    d.bus_id = r.str();
    d.node = r.i32();
    d.cpus = r.str();
    d.threads = r.i32();
    d.transport_size = r.i32();
    d.transport_device = r.i32();
    d.error = r.str();
    out.push_back(std::move(d));
  }
  return out;
}

std::string duplicate_device(const std::vector<RankDevice>& all) {
  for (size_t a = 0; a < all.size(); ++a)
    for (size_t b = a + 1; b < all.size(); ++b)
      if (!all[a].bus_id.empty() && all[a].bus_id == all[b].bus_id)
        return "ranks " + std::to_string(a) + " and " + std::to_string(b) + " resolved to the same GPU " + all[a].bus_id;
  return "";
}

namespace {
std::string json_str(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\';
    if ((unsigned char)c >= 0x20) o += c;
  }
  return o + "\"";
}
}  // namespace

std::string rank_devices_json(const std::vector<RankDevice>& all) {
  auto arr = [&](const char* key, auto get) {
    std::string o = std::string("\"") + key + "\": [";
    for (size_t r = 0; r < all.size(); ++r) o += (r ? ", " : "") + get(all[r]);
    return o + "]";
  };
  return "{" + arr("device", [](const RankDevice& d) { return std::to_string(d.device); }) + ", " +
         arr("bus_id", [](const RankDevice& d) { return json_str(d.bus_id); }) + ", " +
         arr("numa_node", [](const RankDevice& d) { return std::to_string(d.node); }) + ", " +
         arr("cpus", [](const RankDevice& d) { return json_str(d.cpus); }) + ", " +
         arr("threads", [](const RankDevice& d) { return std::to_string(d.threads); }) + ", " +
         arr("transport_size", [](const RankDevice& d) { return std::to_string(d.transport_size); }) + ", " +
         arr("transport_device", [](const RankDevice& d) { return std::to_string(d.transport_device); }) + "}";
}

namespace {

// Reductions shared by the host-memory comms: all-gather, then fold in rank order.
template <class T, class Op>
void fold_allgather(Comm& c, T* v, size_t n, Op op) {
  std::vector<T> all(n * (size_t)c.size());
  c.allgather(v, n * sizeof(T), all.data());
  for (size_t i = 0; i < n; ++i) {
    T s = all[i];
    for (int r = 1; r < c.size(); ++r) s = op(s, all[(size_t)r * n + i]);
    v[i] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// Loopback: shared hub, every collective = deposit + barrier + read + barrier.
// ---------------------------------------------------------------------------------------------
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
    } else if (!cv.wait_for(g, std::chrono::duration<double>(comm_timeout_s()), [&] { return generation != gen; })) {
      throw CommError("loopback collective timed out");
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
    fold_allgather(*this, v, n, [](int64_t a, int64_t b) { return a + b; });
  }
  void allreduce_max_f64(double* v, size_t n) override {
    fold_allgather(*this, v, n, [](double a, double b) { return std::max(a, b); });
  }
  void barrier() override { hub_->sync(); }
  void sendrecv(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src) override {
    hub_->slots[rank_].assign((const uint8_t*)send, (const uint8_t*)send + (dst >= 0 ? sbytes : 0));
    hub_->sync();
    if (src >= 0) {
      if (hub_->slots[src].size() != rbytes) throw CommError("sendrecv: size mismatch with the sender");
      std::memcpy(recv, hub_->slots[src].data(), rbytes);
    }
    hub_->sync();
  }

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
  void sendrecv(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src) override {
    if (dst == 0 && src == 0) {
      if (sbytes != rbytes) throw CommError("sendrecv: size mismatch with the sender");
      std::memmove(recv, send, rbytes);
    }
  }
};

// ---------------------------------------------------------------------------------------------
// Host comm: ranks in separate processes over a ShmSegment. Payloads larger than a slot move in
// slot-sized chunks; every chunk is deposit + barrier + read + barrier.
// ---------------------------------------------------------------------------------------------
class HostComm final : public Comm {
 public:
  HostComm(std::shared_ptr<ShmSegment> seg, int rank, double timeout_s)
      : seg_(std::move(seg)), rank_(rank), timeout_(timeout_s > 0 ? timeout_s : comm_timeout_s()) {
    if (rank_ < 0 || rank_ >= seg_->size()) throw CommError("host comm rank out of range");
  }
  int rank() const override { return rank_; }
  int size() const override { return seg_->size(); }
  const char* backend() const override { return "host"; }
  void broadcast(void* buf, size_t bytes, int root) override {
    const size_t cap = seg_->slot_bytes();
    for (size_t off = 0; off < bytes; off += cap) {
      const size_t len = std::min(cap, bytes - off);
      if (rank_ == root) std::memcpy(seg_->slot(root), (uint8_t*)buf + off, len);
      seg_->barrier(rank_, timeout_);
      if (rank_ != root) std::memcpy((uint8_t*)buf + off, seg_->slot(root), len);
      seg_->barrier(rank_, timeout_);
    }
  }
  void allgather(const void* send, size_t bytes, void* recv) override {
    const size_t cap = seg_->slot_bytes();
    const int n = size();
    for (size_t off = 0; off < bytes; off += cap) {
      const size_t len = std::min(cap, bytes - off);
      std::memcpy(seg_->slot(rank_), (const uint8_t*)send + off, len);
      seg_->barrier(rank_, timeout_);
      for (int r = 0; r < n; ++r) std::memcpy((uint8_t*)recv + (size_t)r * bytes + off, seg_->slot(r), len);
      seg_->barrier(rank_, timeout_);
    }
  }
  void allreduce_sum_i64(int64_t* v, size_t n) override {
    fold_allgather(*this, v, n, [](int64_t a, int64_t b) { return a + b; });
  }
  void allreduce_max_f64(double* v, size_t n) override {
    fold_allgather(*this, v, n, [](double a, double b) { return std::max(a, b); });
  }
  void barrier() override { seg_->barrier(rank_, timeout_); }
  void sendrecv(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src) override {
    // Every rank must run the same number of slot rounds: agree on the largest message first.
    int64_t len = dst >= 0 ? (int64_t)sbytes : 0;
    std::vector<int64_t> lens((size_t)size());
    allgather(&len, sizeof(len), lens.data());
    if (src >= 0 && lens[(size_t)src] != (int64_t)rbytes) throw CommError("sendrecv: size mismatch with the sender");
    const size_t mx = (size_t)*std::max_element(lens.begin(), lens.end());
    const size_t cap = seg_->slot_bytes();
    for (size_t off = 0; off < mx; off += cap) {
      if (off < (size_t)len) std::memcpy(seg_->slot(rank_), (const uint8_t*)send + off, std::min(cap, (size_t)len - off));
      seg_->barrier(rank_, timeout_);
      if (src >= 0 && off < rbytes) std::memcpy((uint8_t*)recv + off, seg_->slot(src), std::min(cap, rbytes - off));
      seg_->barrier(rank_, timeout_);
    }
  }

 private:
  std::shared_ptr<ShmSegment> seg_;
  int rank_;
  double timeout_;
};

double mono_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int exit_code(int st) { return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + (WIFSIGNALED(st) ? WTERMSIG(st) : 0); }

// Supervisor: reap every rank; the first non-zero exit raises the abort flag, stragglers get
// `grace` seconds to notice, then SIGTERM, then SIGKILL.
int supervise(std::vector<pid_t>& kids, ShmSegment& seg, double grace) {
  const int n = (int)kids.size();
  int alive = n, rc = 0;
  std::vector<int> codes((size_t)n, 0);
  double fail_t = -1;
  int signals_sent = 0;
  while (alive > 0) {
    // Only our own rank processes are reaped (the caller may have other children, e.g. Python).
    bool reaped = false;
    for (int r = 0; r < n; ++r) {
      if (kids[r] <= 0) continue;
      int st = 0;
      const pid_t p = waitpid(kids[r], &st, WNOHANG);
      if (p == 0 || (p < 0 && errno == EINTR)) continue;
      kids[r] = -1;
      --alive;
      reaped = true;
      const int code = p < 0 ? 1 : exit_code(st);
      codes[r] = code;
      if (code != 0) {
        fprintf(stderr, "Rank %d exited with status %d\n", r, code);
        fflush(stderr);
        if (!rc) {
          rc = code;
          fail_t = mono_s();
          seg.raise_abort(r);
        }
      }
    }
    if (reaped || alive == 0) continue;
    if (!rc) {
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
      continue;
    }
    // A rank failed and nobody else exited yet: escalate on stragglers once the grace periods pass.
    const double waited = mono_s() - fail_t;
    if (signals_sent < 2 && waited > grace * (signals_sent + 1)) {
      const int sig = signals_sent == 0 ? SIGTERM : SIGKILL;
      for (int r = 0; r < n; ++r)
        if (kids[r] > 0) {
          fprintf(stderr, "Rank %d still running %.1f s after the failure: sending %s\n", r, waited,
                  sig == SIGTERM ? "SIGTERM" : "SIGKILL");
          kill(kids[r], sig);
        }
      fflush(stderr);
      ++signals_sent;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  // The job's status is the root cause's: the rank that raised the abort first (peers that only
  // failed because of it exit 1, possibly before the supervisor reaped the culprit).
  const int root = seg.abort_rank();
  if (rc && root >= 0 && root < n && codes[root] != 0) rc = codes[root];
  return rc;
}

}  // namespace

std::vector<std::unique_ptr<Comm>> make_loopback_group(int n) {
  auto hub = std::make_shared<Hub>(n);
  std::vector<std::unique_ptr<Comm>> v;
  for (int i = 0; i < n; ++i) v.push_back(std::make_unique<LoopbackComm>(hub, i));
  return v;
}

std::unique_ptr<Comm> make_self_comm() { return std::make_unique<SelfComm>(); }

std::unique_ptr<Comm> make_host_comm(std::shared_ptr<ShmSegment> seg, int rank, double timeout_s) {
  return std::make_unique<HostComm>(std::move(seg), rank, timeout_s);
}

std::string LaunchOptions::resolve(int n) const {
  if (comm == "rccl" || comm == "host") return comm;
  if (comm != "auto") throw CommError("unknown comm backend '" + comm + "' (rccl | host | auto)");
  // RCCL refuses two ranks on one device ("Duplicate GPU detected"): shared-device runs use host.
  return (n > 1 && device_override >= 0) ? "host" : "rccl";
}

LaunchOptions LaunchOptions::from_env() {
  LaunchOptions o;
  if (const char* e = std::getenv("NM03_COMM"); e && *e) o.comm = e;
  if (const char* e = std::getenv("NM03_DEVICE_OVERRIDE"); e && *e) o.device_override = std::atoi(e);
  // Ranks under this launcher's supervisor: a dead rank raises the abort flag at once, so the
  // deadline is not what detects a dead peer. Rank 0 may plan (wipe, list, scan headers) while
  // the others wait, and ranks wait for the slowest shard at the end — healthy phases of any
  // length, so the default is generous: 30 minutes. It still turns a rank that is alive but stuck
  // (a GPU hang) into an error on its peers instead of a job that never ends.
  // NM03_COMM_TIMEOUT_S overrides.
  const char* t = std::getenv("NM03_COMM_TIMEOUT_S");
  o.timeout_s = (t && *t) ? comm_timeout_s() : kSupervisedDeadlineS;
  return o;
}

int launch_ranks(int n, const std::function<int(int, int, Comm&)>& body, const LaunchOptions& opts) {
  if (n <= 1) {
    if (opts.comm == "rccl") {
      // An explicit RCCL request keeps the multi-rank communicator's life cycle (deferred start on
      // the start-up thread, settle, promotion) at one rank, in this process.
      auto seg = ShmSegment::create_anonymous(1);
      auto c = make_deferred_rccl_comm(0, 1, opts.device_of(0), seg, opts.timeout_s);
      return body(0, 1, *c);
    }
    auto c = make_self_comm();
    return body(0, 1, *c);
  }
  const std::string backend = opts.resolve(n);
  auto seg = ShmSegment::create_anonymous(n);
  fflush(stdout);  // buffered output must not be duplicated into the children
  fflush(stderr);
  const pid_t supervisor = getpid();
  std::vector<pid_t> kids;
  for (int r = 0; r < n; ++r) {
    const pid_t pid = fork();
    if (pid < 0) {
      seg->raise_abort(-2);
      for (pid_t k : kids) kill(k, SIGTERM);
      for (pid_t k : kids) waitpid(k, nullptr, 0);
      throw std::runtime_error("fork() failed");
    }
    if (pid == 0) {
      // Rank process: dies with the supervisor; runs the body on its own device.
      prctl(PR_SET_PDEATHSIG, SIGTERM);
      if (getppid() != supervisor) _exit(1);
      int rc = 0;
      try {
        std::unique_ptr<Comm> comm;
        if (backend == "rccl") {
          // The body starts RCCL (start_data_plane) once HIP is up and promotes it after its
          // start-up; until then the shared-memory control plane carries the collectives.
          comm = make_deferred_rccl_comm(r, n, opts.device_of(r), seg, opts.timeout_s);
        } else {
          comm = make_host_comm(seg, r, opts.timeout_s);
        }
        rc = body(r, n, *comm);
      } catch (const CommError& e) {
        fprintf(stderr, "Rank %d: communication failed: %s\n", r, e.what());
        rc = 1;
      } catch (const std::exception& e) {
        fprintf(stderr, "Fatal error on rank %d: %s\n", r, e.what());
        rc = 1;
      }
      if (rc != 0) seg->raise_abort(r);  // peers blocked in a collective fail now, not at the deadline
      fflush(stdout);
      fflush(stderr);
      _exit(rc);
    }
    kids.push_back(pid);
  }
  return supervise(kids, *seg, opts.grace_s);
}

}  // namespace nm03
