// Host NUMA placement and per-rank CPU partitions (include/nm03/numa.h).
#include "nm03/numa.h"

#include <dirent.h>
#include <hip/hip_runtime_api.h>
#include <pthread.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <map>
#include <set>
#include <sstream>

namespace nm03::numa {

static std::string read_line(const std::string& path) {
  std::ifstream f(path);
  std::string s;
  if (f) std::getline(f, s);
  return s;
}

std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string part;
  while (std::getline(ss, part, ',')) {
    if (part.empty() || !std::isdigit((unsigned char)part[0])) continue;
    const size_t dash = part.find('-');
    const int a = std::atoi(part.c_str());
    const int b = dash == std::string::npos ? a : std::atoi(part.c_str() + dash + 1);
    for (int c = a; c <= b && c < CPU_SETSIZE; ++c) out.push_back(c);
  }
  return out;
}

std::string format_cpulist(const std::vector<int>& cpus) {
  std::vector<int> v(cpus);
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  std::string out;
  for (size_t i = 0; i < v.size();) {
    size_t j = i;
    while (j + 1 < v.size() && v[j + 1] == v[j] + 1) ++j;
    if (!out.empty()) out += ",";
    out += std::to_string(v[i]);
    if (j > i) out += "-" + std::to_string(v[j]);
    i = j + 1;
  }
  return out;
}

std::string device_bus_id(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return "";
  std::string id(bus);
  for (auto& ch : id) ch = (char)std::tolower((unsigned char)ch);
  return id;
}

int device_node(int device) {
  const std::string id = device_bus_id(device);
  if (id.empty()) return -1;
  const std::string v = read_line("/sys/bus/pci/devices/" + id + "/numa_node");
  if (v.empty()) return -1;
  return std::atoi(v.c_str());
}

std::vector<int> allowed_cpus() {
  std::vector<int> out;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return out;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) out.push_back(c);
  return out;
}

int cpu_budget(const std::string& cgroup_root) {
  int n = (int)allowed_cpus().size();
  if (n < 1) n = 1;
  std::istringstream in(read_line(cgroup_root + "/cpu.max"));
  std::string quota;
  long period = 0;
  if (in >> quota >> period && quota != "max" && period > 0) {
    const long q = std::atol(quota.c_str()) / period;
    n = std::min<long>(n, std::max<long>(1, q));
  }
  return n;
}

std::vector<int> node_cpus(int node) {
  if (node < 0) return {};
  std::vector<int> cpus = parse_cpulist(read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return {};
  cpus.erase(std::remove_if(cpus.begin(), cpus.end(), [&](int c) { return !CPU_ISSET(c, &allowed); }), cpus.end());
  return cpus;
}

int Topology::node_index(int node) const {
  for (size_t i = 0; i < nodes.size(); ++i)
    if (nodes[i] == node) return (int)i;
  return -1;
}

Topology read_topology(const std::string& sysfs, const std::vector<int>& allowed_in) {
  const std::vector<int> allowed = allowed_in.empty() ? allowed_cpus() : allowed_in;
  const std::set<int> ok(allowed.begin(), allowed.end());
  Topology t;
  std::vector<int> ids;
  if (DIR* d = opendir((sysfs + "/devices/system/node").c_str())) {
    while (dirent* e = readdir(d)) {
      const std::string nm = e->d_name;
      if (nm.size() > 4 && nm.compare(0, 4, "node") == 0 && std::isdigit((unsigned char)nm[4]))
        ids.push_back(std::atoi(nm.c_str() + 4));
    }
    closedir(d);
  }
  std::sort(ids.begin(), ids.end());
  for (int id : ids) {
    std::vector<int> cpus = parse_cpulist(read_line(sysfs + "/devices/system/node/node" + std::to_string(id) + "/cpulist"));
    cpus.erase(std::remove_if(cpus.begin(), cpus.end(), [&](int c) { return !ok.count(c); }), cpus.end());
    std::sort(cpus.begin(), cpus.end());
    if (cpus.empty()) continue;
    t.nodes.push_back(id);
    t.node_cpus.push_back(std::move(cpus));
  }
  if (t.nodes.empty()) {  // no NUMA information: one node with every allowed CPU
    t.nodes.push_back(0);
    t.node_cpus.push_back(std::vector<int>(ok.begin(), ok.end()));
  }
  const int maxc = ok.empty() ? 0 : *ok.rbegin() + 1;
  t.core_of.assign((size_t)maxc, -1);
  t.l3_of.assign((size_t)maxc, -1);
  for (int c : allowed) {
    const std::string cpu = sysfs + "/devices/system/cpu/cpu" + std::to_string(c);
    const std::string core = read_line(cpu + "/topology/core_id"), pkg = read_line(cpu + "/topology/physical_package_id");
    const long pk = (long)std::max(0, std::atoi(pkg.c_str())) << 20;
    if (!core.empty()) t.core_of[(size_t)c] = pk | std::atol(core.c_str());
    if (read_line(cpu + "/cache/index3/level") == "3") {
      const std::string id = read_line(cpu + "/cache/index3/id");
      if (!id.empty()) t.l3_of[(size_t)c] = pk | std::atol(id.c_str());
    }
  }
  return t;
}

namespace {

// Group `cpus` (ascending) by physical core, cores in order of their first CPU.
std::vector<std::vector<int>> cores_of(const Topology& t, const std::vector<int>& cpus) {
  std::vector<std::vector<int>> cores;
  std::map<long, size_t> at;
  for (int c : cpus) {
    long key = (size_t)c < t.core_of.size() ? t.core_of[(size_t)c] : -1;
    if (key < 0) key = (1L << 40) + c;  // unknown: every CPU is its own core
    auto it = at.find(key);
    if (it == at.end()) {
      at.emplace(key, cores.size());
      cores.push_back({c});
    } else {
      cores[it->second].push_back(c);
    }
  }
  return cores;
}

}  // namespace

RankCpus rank_partition(const Topology& t, const std::vector<int>& rank_nodes, int local_rank, int budget, int cap) {
  RankCpus r;
  const int n = (int)rank_nodes.size();
  if (local_rank < 0 || local_rank >= n) return r;
  // A rank's node counts only if the topology knows it; others share the leftover CPUs.
  auto known = [&](int q) { return t.node_index(rank_nodes[(size_t)q]) >= 0; };
  const bool mine_known = known(local_rank);
  r.node = mine_known ? rank_nodes[(size_t)local_rank] : -1;
  std::vector<int> pool;
  if (mine_known) {
    pool = t.node_cpus[(size_t)t.node_index(r.node)];
  } else {
    std::set<int> used;
    for (int q = 0; q < n; ++q)
      if (known(q))
        for (int c : t.node_cpus[(size_t)t.node_index(rank_nodes[(size_t)q])]) used.insert(c);
    for (const auto& cs : t.node_cpus)
      for (int c : cs)
        if (!used.count(c)) pool.push_back(c);
    if (pool.empty())
      for (const auto& cs : t.node_cpus) pool.insert(pool.end(), cs.begin(), cs.end());
    std::sort(pool.begin(), pool.end());
  }
  // Ranks sharing this pool, in rank order.
  r.count = 0;
  r.index = 0;
  for (int q = 0; q < n; ++q) {
    const bool same = mine_known ? (known(q) && rank_nodes[(size_t)q] == r.node) : !known(q);
    if (!same) continue;
    if (q == local_rank) r.index = r.count;
    ++r.count;
  }
  const int m = std::max(1, r.count), j = r.index;
  if (!pool.empty()) {
    const auto cores = cores_of(t, pool);
    const size_t C = cores.size(), P = pool.size();
    if (C >= (size_t)m) {
      for (size_t k = C * j / m; k < C * (j + 1) / m; ++k) r.cpus.insert(r.cpus.end(), cores[k].begin(), cores[k].end());
    } else if (P >= (size_t)m) {
      // Fewer cores than ranks: split the logical CPUs, siblings adjacent.
      std::vector<int> flat;
      for (const auto& c : cores) flat.insert(flat.end(), c.begin(), c.end());
      for (size_t k = P * j / m; k < P * (j + 1) / m; ++k) r.cpus.push_back(flat[k]);
    } else {
      r.cpus.push_back(pool[(size_t)j % P]);
    }
    std::sort(r.cpus.begin(), r.cpus.end());
  }
  // The rank's CPU share keeps up to 2 CPUs for its other threads (slot threads, the HIP runtime's
  // event thread, the launcher): with all 16 of a 16-CPU quota given to the pool, the cgroup was
  // throttled 0.5–1 ms per 465-slice step and the headline was lower than with 14 pool threads
  // (394k at 18.9 ms of CPU vs 403k at 17.3 ms, interleaved, profiles/r6/ab_pool/). A share above
  // the cap + 2 is unaffected (the 8-GPU node's 32-CPU partitions keep 16 pool threads).
  const int share = std::max(1, budget / std::max(1, n));
  const int pool_share = std::max(1, share - std::min(2, share / 4));
  r.threads = std::max(1, std::min({cap, (int)std::max<size_t>(1, r.cpus.size()), pool_share}));
  return r;
}

Placement::Placement(int device, const std::vector<int>& cpus) {
  const char* e = std::getenv("NM03_NUMA");
  if (e && *e == '0') return;
  if (!cpus.empty()) {  // a rank partition: exactly these CPUs (within the affinity mask)
    const std::vector<int> ok = allowed_cpus();
    for (int c : cpus)
      if (std::binary_search(ok.begin(), ok.end(), c)) cpus_.push_back(c);
    node_ = device_node(device);
  } else if (!read_line("/sys/devices/system/node/node1/cpulist").empty()) {  // multi-node host: the GPU's node
    node_ = device_node(device);
    cpus_ = node_cpus(node_);
  }
}

void Placement::bind_this_thread() const {
  if (cpus_.empty()) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : cpus_) CPU_SET(c, &set);
  (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
}

std::string Placement::describe() const {
  if (cpus_.empty()) return "numa: off";
  return "numa: node " + std::to_string(node_) + " (" + std::to_string(cpus_.size()) + " cpus: " +
         format_cpulist(cpus_) + ")";
}

}  // namespace nm03::numa
