// nm03/comm.h — rank communication for multi-GPU data parallelism.
//
// The reference has no inter-process communication at all (one process, OpenMP fork/join,
// main_parallel.cpp:336-343). Here one process drives one MI355X; ranks exchange only small
// control messages — the serialized work list (broadcast from rank 0), per-rank slice statuses
// and stage timings (all-gather), success counts (all-reduce) and the barrier that brackets the
// timed region. No pixel data crosses GPUs: each rank reads its own DICOMs and writes its own JPEGs.
//
//   RcclComm      — RCCL (ncclBroadcast / ncclAllGather / ncclAllReduce) on device staging
//                   buffers, i.e. over xGMI inside an 8×MI355X node. Non-blocking init and
//                   deadline-bounded waits: a dead or stuck peer ends in ncclCommAbort + CommError.
//   HostComm      — ranks of one node over a process-shared memory segment (futex barrier, one
//                   slot per rank). Used when ranks share a GPU (RCCL refuses two ranks per
//                   device: rehearsals on a one-GPU box) or when NM03_COMM=host.
//   LoopbackComm  — N in-process ranks (threads) sharing memory; the test double used by the CPU
//                   test-suite (no GPU needed).
//
// Failure model (the reference turns every failure into a message + continue or
// exit 1, main_parallel.cpp:352-356, 377-380, 406-409): the shared segment carries a job-wide
// abort flag; the launcher raises it the moment a rank exits non-zero, so peers blocked in a
// collective fail within milliseconds instead of hanging, and the job exits with "Rank k exited
// with status s". Blocking waits also have a deadline as a hang detector (a rank alive but stuck):
// NM03_COMM_TIMEOUT_S, default 120 s for independently launched ranks (bench.py, torchrun), off
// for the CLI launcher's supervised ranks unless the variable is set.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace nm03 {

// A collective could not complete: timeout, a peer failed (abort flag), or an RCCL error.
class CommError : public std::runtime_error {
 public:
  explicit CommError(const std::string& m) : std::runtime_error(m) {}
};

class ShmSegment;

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual const char* backend() const = 0;
  // Host-buffer collectives (implementations stage through device memory when needed).
  virtual void broadcast(void* buf, size_t bytes, int root) = 0;
  virtual void allgather(const void* send, size_t bytes, void* recv) = 0;  // recv: size()*bytes
  virtual void allreduce_sum_i64(int64_t* v, size_t n) = 0;
  virtual void allreduce_max_f64(double* v, size_t n) = 0;
  virtual void barrier() = 0;
  // Neighbour exchange (collective: every rank calls it): send `sbytes` to rank `dst` and receive
  // `rbytes` from rank `src`; -1 = no such peer. Used for z-slab halo planes. RCCL:
  // grouped ncclSend/ncclRecv over xGMI; host comms: through the segment slots.
  virtual void sendrecv(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src) = 0;
  // Device-memory forms for the z-slab exchange: `send` / `recv` / `v` are device
  // pointers and `stream` the caller's hipStream_t. RCCL enqueues grouped ncclSend/ncclRecv (and
  // ncclAllReduce) on `stream`, straight from and into those buffers over xGMI: no host staging and
  // no host synchronisation for the exchange. The other comms stage through pinned host memory with
  // asynchronous copies on `stream` and one synchronisation per call.
  virtual void sendrecv_device(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src,
                               void* stream);
  // Sums the int64 at device address `v` over all ranks — in place: device *v holds the total for
  // work enqueued on `stream` afterwards (every backend) — and returns the total on the host once
  // everything enqueued on `stream` before it has completed (a bounded wait).
  virtual int64_t allreduce_sum_i64_device(int64_t* v, void* stream);
  // True when the device forms above move data device to device (RCCL).
  virtual bool device_native() const { return false; }

  // What the transport itself reports — RCCL: ncclCommCount / ncclCommUserRank / ncclCommCuDevice —
  // so a run record can show that N ranks really formed one communicator over N devices. Host
  // comms report size() / rank() / -1.
  virtual int transport_size() const { return size(); }
  virtual int transport_rank() const { return rank(); }
  virtual int transport_device() const { return -1; }
  // Watch this segment's job abort flag in every bounded wait from now on (RCCL; the host comms
  // always do). Lets a driver bring a communicator up without the flag — a failed init must not
  // abort the job when a fallback exists — and attach it once every rank agreed.
  virtual void set_abort_segment(std::shared_ptr<ShmSegment>) {}
  // Blocks (bounded) until the transport is usable: RCCL settles a non-blocking
  // ncclCommInitRankConfig. Every collective does it first anyway; no-op for the host comms.
  virtual void ready() {}

  // Non-blocking readiness of a transport whose initialisation was started without settling it
  // (make_rccl_comm settle_now=false): true once usable; throws CommError when it failed.
  virtual bool poll_ready() { return true; }
  // Abandons the transport without a collective (ncclCommAbort): a peer could not bring it up.
  virtual void abort_transport() {}

  // ---- deferred data plane (launch_ranks' RCCL ranks, make_deferred_comm; no-ops elsewhere) -----
  // Starts the device transport's initialisation (the ncclUniqueId hand-off through the segment and
  // a non-blocking ncclCommInitRankConfig) on the calling thread, which must already have brought up
  // HIP on the rank's device. Errors are published to the peers through the segment at once and
  // surface at promote().
  virtual void start_data_plane() {}
  // After start_data_plane(), on the same thread: waits (bounded, abort- and `cancel`-aware) until
  // this rank's transport is usable or some rank's start failed (then it is abandoned, and every
  // rank learns it through the segment instead of waiting for a peer that never joins). The CLI's
  // start-up thread settles RCCL here, BEFORE it builds the engine: RCCL's initialisation never
  // overlaps the engine's construction or its launches.
  virtual void settle_data_plane(const std::atomic<bool>* cancel = nullptr) { (void)cancel; }
  // This rank cannot start its data plane (e.g. its HIP start-up failed): tells the peers through the
  // segment (rank 0 also unblocks their wait for the unique id) so that they fall back at once.
  virtual void fail_data_plane(const std::string& why) { (void)why; }
  // Collective (every rank at the same point): waits (bounded, abort-aware) until the device
  // transport is up and carries every later collective on it. Before it, host-buffer collectives
  // use the shared-memory control plane; device-memory ones promote implicitly.
  virtual void promote() {}
  struct DataPlaneTimes {
    double start_s = -1;      // start_data_plane's begin, seconds after the comm was created (-1: never)
    double settle_s = 0;      // time settle_data_plane() waited for the transport (start-up thread)
    double wait_s = 0;        // time promote() blocked waiting for the transport
    double init_upper_s = 0;  // start → transport usable, upper bound (observed at settle or promote)
  };
  virtual DataPlaneTimes data_plane_times() const { return {}; }
  // Non-empty when promote() found the device transport unusable on some rank and every rank stayed
  // on the control plane (the reason); "" otherwise.
  virtual std::string fallback_error() const { return ""; }

  // Helpers built on the primitives.
  void broadcast_bytes(std::vector<uint8_t>& buf, int root);                        // resizes on non-roots
  std::vector<std::vector<uint8_t>> allgather_bytes(const std::vector<uint8_t>& mine);  // variable sizes
};

// Deadline of one blocking collective wait: NM03_COMM_TIMEOUT_S (default 120 s). A hang detector,
// not a phase budget: ranks started by launch_ranks wait up to 30 minutes unless the variable is
// set (its supervisor turns a dead rank into the abort flag within milliseconds).
double comm_timeout_s();
constexpr double kNoDeadline = 1e9;  // ≈ 30 years
// Default collective deadline of ranks under launch_ranks' supervisor (LaunchOptions::from_env).
constexpr double kSupervisedDeadlineS = 1800.0;

// ---- process-shared control segment -------------------------------------------------------------
// Host collectives, the RCCL unique-id hand-off and the job abort flag live here.
class ShmSegment {
 public:
  ~ShmSegment();
  int size() const;
  size_t slot_bytes() const;
  // Anonymous MAP_SHARED mapping: create BEFORE fork, every child inherits it.
  static std::shared_ptr<ShmSegment> create_anonymous(int n, size_t slot_bytes = 1 << 20);
  // Named segment for independently launched ranks (torchrun): rank 0 creates it under a fresh
  // random name (or under *name when non-empty, e.g. a job id handed out by a launcher) and
  // publishes the name out of band (e.g. the torch TCPStore); the others attach.
  // Rank 0's object unlinks the name once every rank has attached (the mapping stays valid).
  static std::shared_ptr<ShmSegment> create_named(int n, std::string* name, size_t slot_bytes = 1 << 20);
  static std::shared_ptr<ShmSegment> attach_named(const std::string& name, int n, double timeout_s);
  // Rank 0 (named creator): wait until all n ranks attached, then unlink the name.
  void wait_attached_and_unlink(double timeout_s);

  // Abort flag: the first caller records `rank` as the failed one; waiters wake and throw.
  void raise_abort(int rank);
  bool aborted() const;
  int abort_rank() const;  // -1 when not aborted
  // Throws CommError if the job was aborted.
  void check_abort(int self) const;

  // RCCL unique id (128 bytes) published by rank 0, awaited by the others (deadline + abort).
  // publish_uid_failed: rank 0 could not create one; waiters throw at once instead of timing out
  // (so do they when some rank marked its data plane failed).
  void publish_uid(const std::vector<uint8_t>& uid);
  void publish_uid_failed();
  std::vector<uint8_t> wait_uid(int self, double timeout_s) const;
  // Data-plane start-up failure of some rank (the first one is recorded): peers settling their own
  // transport abandon it instead of waiting for a rank that never joins. Not a job abort.
  void mark_data_plane_failed(int rank);
  int data_plane_failed_rank() const;  // -1 when no rank failed

  // Generation barrier across all ranks of the segment; deadline + abort aware.
  void barrier(int self, double timeout_s);
  uint8_t* slot(int r) const;

  struct Header;

 private:
  ShmSegment() = default;
  Header* h_ = nullptr;
  size_t map_bytes_ = 0;
  std::string unlink_name_;
};

// In-process loopback group of n ranks; comms[i]->rank() == i. Each must be used by its own thread.
std::vector<std::unique_ptr<Comm>> make_loopback_group(int n);

// Host collectives over a shared segment (one comm per rank process).
// timeout_s ≤ 0: comm_timeout_s().
std::unique_ptr<Comm> make_host_comm(std::shared_ptr<ShmSegment> seg, int rank, double timeout_s = -1);

// RCCL communicator for `rank` of `size`, bound to HIP device `device`. `unique_id` is the
// 128-byte ncclUniqueId produced by rank 0 (rccl_unique_id()). `seg` (optional) supplies the job
// abort flag that bounded waits also watch.
// `settle_now` false: ncclCommInitRankConfig is only started; ready() / the first collective settle it.
std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::vector<uint8_t>& unique_id, int device,
                                     std::shared_ptr<ShmSegment> seg = nullptr, double timeout_s = -1,
                                     bool settle_now = true);
// How a deferred communicator makes its data plane: rank 0's unique id, and every rank's transport
// from it (initialisation started, not settled). rccl_data_plane(): RCCL. Tests inject fakes that
// succeed, fail, stall or never become ready on chosen ranks (tests/native/unit_tests.cpp).
struct DataPlaneFactory {
  std::function<std::vector<uint8_t>()> unique_id;
  std::function<std::unique_ptr<Comm>(int rank, int size, const std::vector<uint8_t>& uid, int device,
                                      std::shared_ptr<ShmSegment> seg, double timeout_s)>
      make;
};
DataPlaneFactory rccl_data_plane();
// The communicator launch_ranks gives an RCCL rank: the shared-memory control plane (host comm over
// `seg`) for the start-up collectives, the data plane created by start_data_plane() and settled by
// settle_data_plane() — both on the rank's start-up thread, after hipInit and before the engine is
// built — and used from promote() on and for every device collective.
std::unique_ptr<Comm> make_deferred_comm(int rank, int size, int device, std::shared_ptr<ShmSegment> seg,
                                         double timeout_s, DataPlaneFactory factory);
std::unique_ptr<Comm> make_deferred_rccl_comm(int rank, int size, int device, std::shared_ptr<ShmSegment> seg,
                                              double timeout_s = -1);
std::vector<uint8_t> rccl_unique_id();

// Single-rank communicator (no-ops).
std::unique_ptr<Comm> make_self_comm();

// ---- launcher ----------------------------------------------------------------------------------
struct LaunchOptions {
  // "rccl" | "host" | "auto" (default; NM03_COMM overrides): RCCL when every rank has its own
  // GPU, the host comm when ranks share one (device_override ≥ 0). An explicit "rccl" also gives a
  // single-rank job the deferred RCCL communicator (one rank, no fork): the multi-rank start-up,
  // settle and promotion path, exercisable on a one-GPU box.
  std::string comm = "auto";
  // ≥ 0: every rank uses this HIP device (NM03_DEVICE_OVERRIDE), e.g. N ranks on a one-GPU box.
  int device_override = -1;
  // After the first failed rank, peers get this long to fail on the abort flag by themselves
  // before they are sent SIGTERM (and SIGKILL after the same again).
  double grace_s = 5.0;
  // Collective deadline for the ranks' comms; ≤ 0: comm_timeout_s().
  double timeout_s = -1;
  int device_of(int rank) const { return device_override >= 0 ? device_override : rank; }
  // The backend actually used for n ranks.
  std::string resolve(int n) const;
  // Defaults from the environment (NM03_COMM, NM03_DEVICE_OVERRIDE).
  static LaunchOptions from_env();
};

// n == 1: body runs in this process with a self comm. n > 1: fork n rank processes BEFORE any HIP
// call (fork after HIP init is unsafe); this process becomes a supervisor that never touches the
// GPU: it reaps ranks as they exit, raises the abort flag on the first non-zero exit, prints
// "Rank k exited with status s", terminates stragglers after the grace period, and returns the
// first non-zero status (0 when every rank succeeded). Children die with the supervisor
// (PR_SET_PDEATHSIG). Rank r runs body(r, n, comm) on device opts.device_of(r).
int launch_ranks(int n, const std::function<int(int rank, int size, Comm& comm)>& body,
                 const LaunchOptions& opts = LaunchOptions::from_env());

// ---- rank ↔ device identity ----------------------------------------------------------------------
// What every rank records about where it runs, all-gathered before the engines start, so a run
// record (CLI --json, bench JSON) answers "did N ranks really drive N distinct GPUs?" by itself.
struct RankDevice {
  int device = -1;          // HIP device index
  std::string bus_id;       // PCI bus id of that device (numa::device_bus_id)
  int node = -1;            // its NUMA node
  std::string cpus;         // the rank's CPU partition (cpulist form)
  int threads = 0;          // host pool threads
  int transport_size = 0;   // Comm::transport_size() (RCCL: ncclCommCount)
  int transport_device = -1;  // Comm::transport_device() (RCCL: ncclCommCuDevice)
  std::string error;        // set-up failure on this rank ("" = fine)
};
std::vector<RankDevice> gather_rank_devices(Comm& comm, const RankDevice& mine);
// "ranks a and b resolved to the same GPU <bus>" for the first duplicate bus id, "" if none.
std::string duplicate_device(const std::vector<RankDevice>& all);
// JSON object of per-rank arrays {"device": [...], "bus_id": [...], ...}.
std::string rank_devices_json(const std::vector<RankDevice>& all);

// Simple binary (de)serialisation helpers for messages.
struct ByteWriter {
  std::vector<uint8_t> b;
  void u32(uint32_t v);
  void i32(int32_t v) { u32((uint32_t)v); }
  void u64(uint64_t v);
  void f64(double v);
  void str(const std::string& s);
};
struct ByteReader {
  const uint8_t* p;
  size_t n, pos = 0;
  ByteReader(const uint8_t* d, size_t len) : p(d), n(len) {}
  uint32_t u32();
  int32_t i32() { return (int32_t)u32(); }
  uint64_t u64();
  double f64();
  std::string str();
};

}  // namespace nm03
