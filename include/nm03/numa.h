// nm03/numa.h — host CPU placement for the ranks of one node. An MI355X node has two sockets with
// four GPUs each; a rank's loader/writer threads and its pinned upload/download buffers belong on
// the socket its GPU hangs off, so page-cache reads, blob writes and the SDMA/PCIe traffic stay
// local — and the ranks that share a socket must not share CPUs.
//
// The reference runs one process with omp_set_num_threads(16) for the whole machine
// (main_parallel.cpp:401). Here every rank gets a disjoint partition of its GPU's NUMA node —
// whole physical cores, contiguous (so a partition spans as few L3 domains as possible) — and a
// pool sized to that partition and to its share of the process CPU budget (affinity mask ∩
// cgroup quota), at most 16 threads: N ranks never oversubscribe the node's CPUs.
#pragma once

#include <sched.h>

#include <string>
#include <vector>

namespace nm03::numa {

// NUMA node of HIP device `device` (sysfs numa_node of its PCI function), or -1 if unknown.
int device_node(int device);
// PCI bus id of HIP device `device` ("0000:05:00.0", lower case), or "" if HIP cannot tell.
std::string device_bus_id(int device);
// CPUs of NUMA node `node` intersected with this process's allowed CPUs (empty if unknown).
std::vector<int> node_cpus(int node);
// Parses a sysfs cpulist such as "0-63,128-191".
std::vector<int> parse_cpulist(const std::string& s);
// CPUs this process may run on (sched_getaffinity), ascending.
std::vector<int> allowed_cpus();
// CPU budget of this process: the allowed CPUs capped by the cgroup v2 quota
// (`<cgroup_root>/cpu.max`, "max" = no cap).
int cpu_budget(const std::string& cgroup_root = "/sys/fs/cgroup");

// Host CPU topology (from `<sysfs>/devices/system/...`, so tests can use a fake tree).
struct Topology {
  std::vector<int> nodes;                    // NUMA node ids with allowed CPUs, ascending
  std::vector<std::vector<int>> node_cpus;   // per entry of `nodes`: allowed CPUs, ascending
  std::vector<long> core_of;                 // cpu -> physical core key (package << 20 | core id); -1 unknown
  std::vector<long> l3_of;                   // cpu -> L3 domain key (package << 20 | cache id); -1 unknown
  int node_index(int node) const;            // index into `nodes`, -1 if absent
};
// `allowed` empty: the calling process's affinity mask.
Topology read_topology(const std::string& sysfs = "/sys", const std::vector<int>& allowed = {});

// The CPU partition of one rank.
struct RankCpus {
  int node = -1;           // NUMA node of the rank's GPU (-1: unknown, partition of all CPUs)
  int index = 0, count = 1;  // this rank is partition `index` of `count` on its node
  std::vector<int> cpus;   // disjoint from every other local rank's
  int threads = 1;         // pool threads: min(cap, |cpus|, share − min(2, share/4)), share = budget / local ranks, ≥ 1
};
// `rank_nodes[r]` = NUMA node of local rank r's GPU (-1 unknown). The ranks on one node split its
// allowed CPUs into `count` groups of whole physical cores (SMT siblings stay together), in rank
// order; ranks with an unknown node split the CPUs no known-node rank uses (or all, if none).
// With more ranks than cores on a node, partitions fall back to single logical CPUs (and, past
// that, are shared round-robin: a partition is never empty).
RankCpus rank_partition(const Topology& topo, const std::vector<int>& rank_nodes, int local_rank, int budget,
                        int cap = 16);
// "0-7,64-71" form of a CPU list.
std::string format_cpulist(const std::vector<int>& cpus);

// Placement for the threads and pinned memory of one engine. Disabled by NM03_NUMA=0. With an
// explicit CPU list (a rank partition) the engine binds to exactly those CPUs; without, to the
// whole NUMA node of its GPU on multi-node hosts (single-node hosts: unbound).
class Placement {
 public:
  explicit Placement(int device, const std::vector<int>& cpus = {});
  bool active() const { return !cpus_.empty(); }
  int node() const { return node_; }
  const std::vector<int>& cpus() const { return cpus_; }
  // Pins the calling thread to the placement's CPUs (no-op when inactive).
  void bind_this_thread() const;
  // Pool workers float over the whole set (bind_this_thread). Measured and removed in round 4:
  // one physical core per worker (round-3 NM03_PIN=core: host-only 283–304k vs 365–392k slices/s) and
  // workers + work keyed to L3 domains (NM03_PIN=l3: writes get slower when the threads spread
  // over more L3 domains, 17 → 29 µs per JPEG pair; profiles/r3/host_pin/, profiles/r3/pin_l3/).
  // Runs `f` with the calling thread temporarily pinned (first-touch / pinned allocations land on
  // the node), restoring the previous affinity afterwards.
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
