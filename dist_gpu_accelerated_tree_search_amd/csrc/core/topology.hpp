// Host topology: which NUMA node / CPUs sit next to a GPU, and thread pinning.
//
// Parity: ref common/get_numa_affinity.py (parses lscpu + rocm-smi --showtoponuma
// into an affinity.txt that no C code reads). Here the GPU's PCI bus id (from
// hipDeviceGetPCIBusId, passed in by the HIP side) is looked up in sysfs and the
// host thread driving that GPU is pinned to the CPUs of the GPU's NUMA node.
#pragma once

#include <sched.h>

#include <cctype>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace tts {

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}
inline std::vector<int> parse_cpulist(const std::string& s) {
  std::vector<int> out;
  std::stringstream ss(s);
  std::string tok;
  while (std::getline(ss, tok, ',')) {
    while (!tok.empty() && std::isspace(static_cast<unsigned char>(tok.back()))) tok.pop_back();
    while (!tok.empty() && std::isspace(static_cast<unsigned char>(tok.front()))) tok.erase(tok.begin());
    if (tok.empty()) continue;
    const auto dash = tok.find('-');
    try {
      if (dash == std::string::npos) {
        out.push_back(std::stoi(tok));
      } else {
        const int a = std::stoi(tok.substr(0, dash)), b = std::stoi(tok.substr(dash + 1));
        for (int c = a; c <= b; ++c) out.push_back(c);
      }
    } catch (...) {
      return {};
    }
  }
  return out;
}

inline std::string read_first_line(const std::string& path) {
  std::ifstream f(path);
  std::string line;
  if (f) std::getline(f, line);
  return line;
}

// NUMA node of a PCI device ("0000:c1:00.0"), -1 if unknown.
inline int pci_numa_node(std::string bus_id) {
  for (auto& c : bus_id) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  const std::string v = read_first_line("/sys/bus/pci/devices/" + bus_id + "/numa_node");
  if (v.empty()) return -1;
  try {
    return std::stoi(v);
  } catch (...) {
    return -1;
  }
}

inline std::vector<int> numa_cpus(int node) {
  if (node < 0) return {};
  return parse_cpulist(read_first_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"));
}

// CPUs this process may run on.
inline std::vector<int> allowed_cpus() {
  std::vector<int> out;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return out;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) out.push_back(c);
  return out;
}

// Pin the calling thread to `cpus` intersected with the allowed set; returns
// false (and leaves the affinity alone) if the intersection is empty.
inline bool pin_current_thread(const std::vector<int>& cpus) {
  const std::vector<int> ok = allowed_cpus();
  cpu_set_t set;
  CPU_ZERO(&set);
  int n = 0;
  for (int c : cpus)
    for (int a : ok)
      if (a == c && c < CPU_SETSIZE) {
        CPU_SET(c, &set);
        ++n;
      }
  if (n == 0) return false;
  return sched_setaffinity(0, sizeof(set), &set) == 0;
}

}  // namespace tts
