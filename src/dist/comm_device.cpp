// Device-memory collectives of the host-side comms (nm03/comm.h Comm::sendrecv_device /
// allreduce_sum_i64_device): staged through pinned host memory. RcclComm overrides both with
// device-to-device RCCL calls on the caller's stream.
//
// Staging (per calling thread, grown on demand): [send | recv] pinned. Order on `stream`:
// D2H(send) → synchronise → host sendrecv → H2D(recv), asynchronous. An event recorded after every
// H2D out of the staging is waited for before the host writes it again (or frees it to grow it), so
// a call on another stream than the previous one cannot overwrite bytes still being copied.
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
  hipEvent_t copied = nullptr;  // recorded after the last H2D out of the staging
  bool pending = false;
  ~PinnedStage() {
    if (pending) (void)hipEventSynchronize(copied);
    if (copied) (void)hipEventDestroy(copied);
    if (p) (void)hipHostFree(p);
  }
  // An H2D out of the staging was enqueued on `st`.
  void copy_out_enqueued(hipStream_t st) {
    if (!copied) ck(hipEventCreateWithFlags(&copied, hipEventDisableTiming), "hipEventCreate comm stage");
    ck(hipEventRecord(copied, st), "hipEventRecord comm stage");
    pending = true;
  }
  uint8_t* get(size_t bytes) {
    if (pending) {
      ck(hipEventSynchronize(copied), "comm stage reuse");
      pending = false;
    }
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
  if (rbytes) {
    ck(hipMemcpyAsync(recv, h + sbytes, rbytes, hipMemcpyHostToDevice, st), "H2D comm stage");
    t_stage.copy_out_enqueued(st);
  }
}

int64_t Comm::allreduce_sum_i64_device(int64_t* v, void* stream) {
  auto st = static_cast<hipStream_t>(stream);
  auto* h = reinterpret_cast<int64_t*>(t_stage.get(8));
  ck(hipMemcpyAsync(h, v, 8, hipMemcpyDeviceToHost, st), "D2H comm stage");
  ck(hipStreamSynchronize(st), "comm stage sync");
  int64_t x = *h;
  allreduce_sum_i64(&x, 1);
  *h = x;  // the sum back into device *v, in place like the RCCL form (comm.h)
  ck(hipMemcpyAsync(v, h, 8, hipMemcpyHostToDevice, st), "H2D comm stage");
  t_stage.copy_out_enqueued(st);
  return x;
}

}  // namespace nm03
