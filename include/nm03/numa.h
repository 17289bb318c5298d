// nm03/numa.h — host NUMA placement for one rank. An MI355X node has two sockets with four GPUs
// each; a rank's loader/writer threads and its pinned upload/download buffers belong on the socket
// its GPU hangs off, so page-cache reads, blob writes and the SDMA/PCIe traffic stay local.
#pragma once

#include <sched.h>

#include <string>
#include <vector>

namespace nm03::numa {

// NUMA node of HIP device `device` (sysfs numa_node of its PCI function), or -1 if unknown.
int device_node(int device);
// CPUs of NUMA node `node` intersected with this process's allowed CPUs (empty if unknown).
std::vector<int> node_cpus(int node);
// Parses a sysfs cpulist such as "0-63,128-191".
std::vector<int> parse_cpulist(const std::string& s);

// Placement for the threads and pinned memory of one engine. Disabled by NM03_NUMA=0 or when the
// topology is unknown / single-node.
class Placement {
 public:
  explicit Placement(int device);
  bool active() const { return !cpus_.empty(); }
  int node() const { return node_; }
  // Pins the calling thread to the node's CPUs (no-op when inactive).
  void bind_this_thread() const;
  // Runs `f` with the calling thread temporarily pinned to the node (first-touch / pinned
  // allocations land on it), restoring the previous affinity afterwards.
  template <class F>
  void run_bound(F&& f) const {
    cpu_set_t old;
    const bool saved = active() && sched_getaffinity(0, sizeof(old), &old) == 0;
    if (saved) bind_this_thread();
    f();
    if (saved) sched_setaffinity(0, sizeof(old), &old);
  }
  std::string describe() const;

 private:
  int node_ = -1;
  std::vector<int> cpus_;
};

}  // namespace nm03::numa
