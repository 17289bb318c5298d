// Host NUMA placement (include/nm03/numa.h).
#include "nm03/numa.h"

#include <hip/hip_runtime_api.h>
#include <pthread.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
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

int device_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
  std::string id(bus);
  for (auto& ch : id) ch = (char)std::tolower((unsigned char)ch);
  const std::string v = read_line("/sys/bus/pci/devices/" + id + "/numa_node");
  if (v.empty()) return -1;
  return std::atoi(v.c_str());
}

std::vector<int> node_cpus(int node) {
  if (node < 0) return {};
  std::vector<int> cpus = parse_cpulist(read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return {};
  cpus.erase(std::remove_if(cpus.begin(), cpus.end(), [&](int c) { return !CPU_ISSET(c, &allowed); }), cpus.end());
  return cpus;
}

Placement::Placement(int device) {
  const char* e = std::getenv("NM03_NUMA");
  if (e && *e == '0') return;
  // Only worth it on multi-node hosts.
  if (read_line("/sys/devices/system/node/node1/cpulist").empty()) return;
  node_ = device_node(device);
  cpus_ = node_cpus(node_);
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
  return "numa: node " + std::to_string(node_) + " (" + std::to_string(cpus_.size()) + " cpus)";
}

}  // namespace nm03::numa
