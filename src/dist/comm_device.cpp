// Device-memory collectives of the host-side comms (nm03/comm.h Comm::sendrecv_device /
// allreduce_sum_i64_device): staged through pinned host memory. RcclComm overrides both with
// device-to-device RCCL calls on the caller's stream.
//
// Staging (per calling thread, grown on demand): [send | recv] pinned. Order on `stream`:
// D2H(send) → synchronise → host sendrecv → H2D(recv), asynchronous. The staging is reused safely:
// the next call's D2H is enqueued behind this call's H2D on the same stream, and the host only
// writes the staging after that D2H has completed.
#include <hip/hip_runtime_api.h>

#include <algorithm>

#include "nm03/comm.h"

namespace nm03 {

namespace {

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw CommError(std::string(what) + ": " + hipGetErrorString(e));
}

struct PinnedStage {
  uint8_t* p = nullptr;
  size_t cap = 0;
  ~PinnedStage() {
    if (p) (void)hipHostFree(p);
  }
  uint8_t* get(size_t bytes) {
    if (bytes > cap) {
      if (p) ck(hipHostFree(p), "hipHostFree");
      p = nullptr;
      cap = std::max<size_t>(bytes, 64 << 10);
      ck(hipHostMalloc((void**)&p, cap, hipHostMallocDefault), "hipHostMalloc comm stage");
    }
    return p;
  }
};

thread_local PinnedStage t_stage;

}  // namespace

void Comm::sendrecv_device(const void* send, size_t sbytes, int dst, void* recv, size_t rbytes, int src, void* stream) {
  if (dst < 0) sbytes = 0;
  if (src < 0) rbytes = 0;
  auto st = static_cast<hipStream_t>(stream);
  uint8_t* h = t_stage.get(sbytes + rbytes);
  if (sbytes) ck(hipMemcpyAsync(h, send, sbytes, hipMemcpyDeviceToHost, st), "D2H comm stage");
  ck(hipStreamSynchronize(st), "comm stage sync");
  sendrecv(h, sbytes, dst, h + sbytes, rbytes, src);  // collective: called even with nothing to move
  if (rbytes) ck(hipMemcpyAsync(recv, h + sbytes, rbytes, hipMemcpyHostToDevice, st), "H2D comm stage");
}

int64_t Comm::allreduce_sum_i64_device(int64_t* v, void* stream) {
  auto st = static_cast<hipStream_t>(stream);
  auto* h = reinterpret_cast<int64_t*>(t_stage.get(8));
  ck(hipMemcpyAsync(h, v, 8, hipMemcpyDeviceToHost, st), "D2H comm stage");
  ck(hipStreamSynchronize(st), "comm stage sync");
  int64_t x = *h;
  allreduce_sum_i64(&x, 1);
  return x;
}

}  // namespace nm03
