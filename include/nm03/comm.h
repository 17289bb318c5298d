// nm03/comm.h — rank communication for multi-GPU data parallelism.
//
// The reference has no inter-process communication at all (one process, OpenMP fork/join,
// main_parallel.cpp:336-343). Here one process drives one MI355X; ranks exchange only small
// control messages — the serialized work list (broadcast from rank 0), per-rank slice statuses
// and stage timings (all-gather), success counts (all-reduce) and the barrier that brackets the
// timed region. No pixel data crosses GPUs: each rank reads its own DICOMs and writes its own JPEGs.
//
//   RcclComm      — RCCL (ncclBroadcast / ncclAllGather / ncclAllReduce) on device staging
//                   buffers, i.e. over xGMI inside an 8×MI355X node.
//   LoopbackComm  — N in-process ranks (threads) sharing memory; the test double used by the CPU
//                   test-suite (no GPU needed).
#pragma once

#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace nm03 {

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

  // Helpers built on the primitives.
  void broadcast_bytes(std::vector<uint8_t>& buf, int root);                        // resizes on non-roots
  std::vector<std::vector<uint8_t>> allgather_bytes(const std::vector<uint8_t>& mine);  // variable sizes
};

// In-process loopback group of n ranks; comms[i]->rank() == i. Each must be used by its own thread.
std::vector<std::unique_ptr<Comm>> make_loopback_group(int n);

// RCCL communicator for `rank` of `size`, bound to HIP device `device`. `unique_id` is the
// 128-byte ncclUniqueId produced by rank 0 (rccl_unique_id()).
std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::vector<uint8_t>& unique_id, int device);
std::vector<uint8_t> rccl_unique_id();

// Single-rank communicator (no-ops).
std::unique_ptr<Comm> make_self_comm();

// Fork `n-1` child processes BEFORE any HIP call (fork after HIP init is unsafe), hand every rank
// the RCCL unique id through pipes, and run body(rank, n, comm) in each. Returns rank 0's exit
// code or the first non-zero child status (a dead rank makes the job fail).
// `use_rccl=false` gives every rank a self/loopback-free comm (testing the launcher only).
int launch_ranks(int n, const std::function<int(int rank, int size, Comm& comm)>& body, bool use_rccl = true);

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
