// HIP-side host support for the runner: peer staging buffers for GPU -> GPU
// steals over xGMI, GPU -> NUMA CPU sets, and roctx trace hooks.
#pragma once

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <mutex>
#include <string>
#include <vector>

#include "../core/runner.hpp"
#include "../core/topology.hpp"
#include "../core/trace.hpp"
#include "device_common.hpp"

namespace tts {

// Enable peer access between every pair of visible GPUs once per process, so
// hipMemcpy between two devices' buffers goes straight over xGMI.
inline void enable_all_peer_access() {
  static std::once_flag once;
  std::call_once(once, [] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (int a = 0; a < n; ++a)
      for (int b = 0; b < n; ++b) {
        if (a == b) continue;
        int ok = 0;
        if (hipDeviceCanAccessPeer(&ok, a, b) != hipSuccess || !ok) continue;
        (void)hipSetDevice(a);
        const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
      }
    (void)hipSetDevice(cur);
    (void)hipGetLastError();
  });
}

class HipStaging final : public DeviceStaging {
 public:
  HipStaging() { enable_all_peer_access(); }
  void* alloc(int device, size_t bytes) override {
    TTS_HIP_CHECK(hipSetDevice(device));
    void* p = nullptr;
    TTS_HIP_CHECK(hipMalloc(&p, std::max<size_t>(bytes, 1)));
    return p;
  }
  void release(int device, void* p) override {
    (void)hipSetDevice(device);
    (void)hipFree(p);
  }
  uintptr_t make_event(int device) override {
    TTS_HIP_CHECK(hipSetDevice(device));
    hipEvent_t e = nullptr;
    TTS_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return reinterpret_cast<uintptr_t>(e);
  }
  void free_event(int device, uintptr_t ev) override {
    (void)hipSetDevice(device);
    if (ev) (void)hipEventDestroy(reinterpret_cast<hipEvent_t>(ev));
  }
};

inline std::string device_pci_bus_id(int device) {
  char buf[64] = {0};
  if (hipDeviceGetPCIBusId(buf, sizeof(buf), device) != hipSuccess) return {};
  return std::string(buf);
}

// CPUs of the NUMA node closest to `device` (empty when unknown).
inline std::vector<int> device_cpus(int device) { return numa_cpus(pci_numa_node(device_pci_bus_id(device))); }

inline void install_roctx_hooks() {
  trace_hooks().push = &roctxRangePushA;
  trace_hooks().pop = &roctxRangePop;
}

}  // namespace tts
