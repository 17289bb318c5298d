// Process-shared control segment (nm03/comm.h ShmSegment): a header of atomics (barrier
// generation, abort flag, attach count, RCCL unique id) followed by one data slot per rank.
// Waits spin briefly, then sleep on the generation word with FUTEX_WAIT (shared, not private:
// the word lives in a MAP_SHARED mapping used by several processes) in ≤1 ms steps so deadline
// and abort flag are re-checked.
#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <random>
#include <thread>

#include "nm03/comm.h"

namespace nm03 {

namespace {

constexpr uint64_t kMagic = 0x4e4d30335348u;  // "NM03SH"
constexpr size_t kHeaderBytes = 4096;

double mono_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void futex_wait(std::atomic<uint32_t>* w, uint32_t expected, long ns) {
  timespec ts{0, ns};
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expected, &ts, nullptr, 0);
}
void futex_wake_all(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, 0x7fffffff, nullptr, nullptr, 0);
}

}  // namespace

struct ShmSegment::Header {
  uint64_t magic;
  int32_t n;
  uint32_t pad0;
  uint64_t slot_bytes;
  alignas(64) std::atomic<uint32_t> arrived;
  alignas(64) std::atomic<uint32_t> gen;  // futex word: barrier generation, bumped on abort too
  alignas(64) std::atomic<int32_t> abort_rank;
  std::atomic<uint32_t> abort;
  std::atomic<uint32_t> attached;
  std::atomic<uint32_t> uid_ready;
  std::atomic<int32_t> dp_failed_rank;  // first rank whose data plane could not start (-1: none)
  uint8_t uid[128];
};
static_assert(sizeof(ShmSegment::Header) <= kHeaderBytes, "header too large");
static_assert(std::atomic<uint32_t>::is_always_lock_free, "process-shared atomics must be lock-free");

double comm_timeout_s() {
  static const double t = [] {
    const char* e = std::getenv("NM03_COMM_TIMEOUT_S");
    const double v = e && *e ? std::atof(e) : 120.0;
    return v > 0 ? v : 120.0;
  }();
  return t;
}

ShmSegment::~ShmSegment() {
  if (!unlink_name_.empty()) shm_unlink(unlink_name_.c_str());
  if (h_) munmap(h_, map_bytes_);
}

int ShmSegment::size() const { return h_->n; }
size_t ShmSegment::slot_bytes() const { return h_->slot_bytes; }
uint8_t* ShmSegment::slot(int r) const {
  return reinterpret_cast<uint8_t*>(h_) + kHeaderBytes + (size_t)r * h_->slot_bytes;
}

static void init_header(ShmSegment::Header* h, int n, size_t slot_bytes) {
  new (h) ShmSegment::Header();
  h->n = n;
  h->slot_bytes = slot_bytes;
  h->arrived.store(0);
  h->gen.store(0);
  h->abort_rank.store(-1);
  h->abort.store(0);
  h->attached.store(1);  // the creator
  h->uid_ready.store(0);
  h->dp_failed_rank.store(-1);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  reinterpret_cast<std::atomic<uint64_t>*>(&h->magic)->store(kMagic, std::memory_order_release);
}

std::shared_ptr<ShmSegment> ShmSegment::create_anonymous(int n, size_t slot_bytes) {
  if (n < 1) throw CommError("segment needs at least one rank");
  slot_bytes = (slot_bytes + 4095) / 4096 * 4096;
  const size_t bytes = kHeaderBytes + (size_t)n * slot_bytes;
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) throw CommError("mmap of the shared comm segment failed");
  std::shared_ptr<ShmSegment> s(new ShmSegment());
  s->h_ = static_cast<Header*>(p);
  s->map_bytes_ = bytes;
  init_header(s->h_, n, slot_bytes);
  s->h_->attached.store((uint32_t)n);  // children inherit the mapping
  return s;
}

std::shared_ptr<ShmSegment> ShmSegment::create_named(int n, std::string* name, size_t slot_bytes) {
  if (n < 1) throw CommError("segment needs at least one rank");
  slot_bytes = (slot_bytes + 4095) / 4096 * 4096;
  const size_t bytes = kHeaderBytes + (size_t)n * slot_bytes;
  std::random_device rd;
  const bool given = !name->empty();
  for (int attempt = 0; attempt < (given ? 1 : 8); ++attempt) {
    char buf[96];
    if (given)
      snprintf(buf, sizeof(buf), "%s", name->c_str());
    else
      snprintf(buf, sizeof(buf), "/nm03-comm-%d-%08x%08x", (int)getpid(), rd(), rd());
    const int fd = shm_open(buf, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) continue;
    if (ftruncate(fd, (off_t)bytes) != 0) {
      close(fd);
      shm_unlink(buf);
      throw CommError("ftruncate of the shared comm segment failed");
    }
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      shm_unlink(buf);
      throw CommError("mmap of the shared comm segment failed");
    }
    std::shared_ptr<ShmSegment> s(new ShmSegment());
    s->h_ = static_cast<Header*>(p);
    s->map_bytes_ = bytes;
    s->unlink_name_ = buf;  // unlinked at the latest when the creator goes away
    init_header(s->h_, n, slot_bytes);
    *name = buf;
    return s;
  }
  throw CommError("cannot create a shared comm segment in /dev/shm");
}

std::shared_ptr<ShmSegment> ShmSegment::attach_named(const std::string& name, int n, double timeout_s) {
  const double deadline = mono_s() + timeout_s;
  for (;;) {
    const int fd = shm_open(name.c_str(), O_RDWR, 0);
    if (fd >= 0) {
      struct stat st {};
      if (fstat(fd, &st) == 0 && st.st_size >= (off_t)kHeaderBytes) {
        void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (p == MAP_FAILED) throw CommError("mmap of " + name + " failed");
        auto* h = static_cast<Header*>(p);
        if (reinterpret_cast<std::atomic<uint64_t>*>(&h->magic)->load(std::memory_order_acquire) == kMagic) {
          if (h->n != n) {
            munmap(p, (size_t)st.st_size);
            throw CommError("comm segment " + name + " was created for " + std::to_string(h->n) + " ranks, not " +
                            std::to_string(n));
          }
          std::shared_ptr<ShmSegment> s(new ShmSegment());
          s->h_ = h;
          s->map_bytes_ = (size_t)st.st_size;
          h->attached.fetch_add(1, std::memory_order_acq_rel);
          futex_wake_all(&h->gen);
          return s;
        }
        munmap(p, (size_t)st.st_size);
      } else {
        close(fd);
      }
    }
    if (mono_s() > deadline) throw CommError("timed out attaching to comm segment " + name);
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
}

void ShmSegment::wait_attached_and_unlink(double timeout_s) {
  const double deadline = mono_s() + timeout_s;
  while (h_->attached.load(std::memory_order_acquire) < (uint32_t)h_->n) {
    check_abort(0);
    if (mono_s() > deadline) {
      raise_abort(0);
      throw CommError("timed out waiting for " + std::to_string(h_->n) + " ranks to attach (" +
                      std::to_string(h_->attached.load()) + " did)");
    }
    const uint32_t g = h_->gen.load();
    futex_wait(&h_->gen, g, 1000000);
  }
  if (!unlink_name_.empty()) {
    shm_unlink(unlink_name_.c_str());
    unlink_name_.clear();
  }
}

void ShmSegment::raise_abort(int rank) {
  int32_t none = -1;
  h_->abort_rank.compare_exchange_strong(none, rank);
  h_->abort.store(1, std::memory_order_release);
  h_->gen.fetch_add(1, std::memory_order_acq_rel);  // wakes futex sleepers; they see the flag
  futex_wake_all(&h_->gen);
}
bool ShmSegment::aborted() const { return h_->abort.load(std::memory_order_acquire) != 0; }
int ShmSegment::abort_rank() const { return aborted() ? h_->abort_rank.load() : -1; }
void ShmSegment::check_abort(int self) const {
  if (!aborted()) return;
  const int r = h_->abort_rank.load();
  throw CommError(r == self ? "collective aborted" : "rank " + std::to_string(r) + " failed; job aborted");
}

void ShmSegment::publish_uid(const std::vector<uint8_t>& uid) {
  if (uid.size() > sizeof(h_->uid)) throw CommError("unique id too large");
  std::memcpy(h_->uid, uid.data(), uid.size());
  h_->uid_ready.store((uint32_t)uid.size(), std::memory_order_release);
}

constexpr uint32_t kUidFailed = 0xFFFFFFFFu;

void ShmSegment::publish_uid_failed() { h_->uid_ready.store(kUidFailed, std::memory_order_release); }

std::vector<uint8_t> ShmSegment::wait_uid(int self, double timeout_s) const {
  const double deadline = mono_s() + timeout_s;
  uint32_t len;
  while ((len = h_->uid_ready.load(std::memory_order_acquire)) == 0) {
    check_abort(self);
    if (const int f = data_plane_failed_rank(); f >= 0)
      throw CommError("rank " + std::to_string(f) + " could not start the data plane");
    if (mono_s() > deadline) throw CommError("timed out waiting for the RCCL unique id from rank 0");
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  if (len == kUidFailed) throw CommError("rank 0 could not create the RCCL unique id");
  return std::vector<uint8_t>(h_->uid, h_->uid + len);
}

void ShmSegment::mark_data_plane_failed(int rank) {
  int32_t none = -1;
  h_->dp_failed_rank.compare_exchange_strong(none, rank, std::memory_order_acq_rel);
}
int ShmSegment::data_plane_failed_rank() const { return h_->dp_failed_rank.load(std::memory_order_acquire); }

void ShmSegment::barrier(int self, double timeout_s) {
  check_abort(self);
  const uint32_t g = h_->gen.load(std::memory_order_acquire);
  if (h_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)h_->n) {
    h_->arrived.store(0, std::memory_order_relaxed);
    h_->gen.fetch_add(1, std::memory_order_release);  // publishes arrived = 0 and the slot data
    futex_wake_all(&h_->gen);
    return;
  }
  const double deadline = mono_s() + timeout_s;
  for (int spin = 0; h_->gen.load(std::memory_order_acquire) == g; ++spin) {
    if (aborted()) check_abort(self);
    if (spin < 2000) {
      __builtin_ia32_pause();
      continue;
    }
    if (mono_s() > deadline) {
      const uint32_t arrived = h_->arrived.load();
      raise_abort(self);
      throw CommError("collective timed out after " + std::to_string((int)timeout_s) + " s on rank " +
                      std::to_string(self) + " (" + std::to_string(arrived) + " of " + std::to_string(h_->n) +
                      " ranks arrived); set NM03_COMM_TIMEOUT_S to wait longer");
    }
    futex_wait(&h_->gen, g, 1000000);
  }
  // A generation bump by raise_abort also ends the wait: report it.
  check_abort(self);
}

}  // namespace nm03
