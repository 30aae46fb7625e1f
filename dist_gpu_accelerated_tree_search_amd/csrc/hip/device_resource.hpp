// Objects that hold HIP (and RCCL) resources register here, so that everything is
// released while the runtime is still alive: the Python module's atexit hook
// (bindings/py_hip.cpp) calls release_all() before interpreter teardown. An engine
// otherwise freed from Py_Finalize — after the HIP runtime or a profiler's tool library
// (rocprofv3 --memory-copy-trace) had begun its own teardown — died with SIGSEGV in
// __cxa_finalize on runs that had used pinned spill blocks (profiles/r3/spill/README.md).
#pragma once

#include <mutex>
#include <set>

namespace tts {

class DeviceResource {
 public:
  DeviceResource() {
    std::lock_guard<std::mutex> lk(reg().mu);
    reg().live.insert(this);
  }
  virtual ~DeviceResource() {
    std::lock_guard<std::mutex> lk(reg().mu);
    reg().live.erase(this);
  }
  DeviceResource(const DeviceResource&) = delete;
  DeviceResource& operator=(const DeviceResource&) = delete;
  // Idempotent; the object is unusable afterwards (its destructor frees nothing more).
  virtual void release() = 0;

  // Releases every live object (engines first, in reverse creation order is not
  // needed: they share no resource). Returns how many were live.
  static int release_all() {
    std::set<DeviceResource*> live;
    {
      std::lock_guard<std::mutex> lk(reg().mu);
      live = reg().live;
    }
    for (DeviceResource* r : live) r->release();
    return static_cast<int>(live.size());
  }
  static int live_count() {
    std::lock_guard<std::mutex> lk(reg().mu);
    return static_cast<int>(reg().live.size());
  }

 private:
  struct Registry {
    std::mutex mu;
    std::set<DeviceResource*> live;
  };
  // never destroyed: no static-destructor ordering against the runtime's own teardown
  static Registry& reg() {
    static Registry* r = new Registry;
    return *r;
  }
};

}  // namespace tts
