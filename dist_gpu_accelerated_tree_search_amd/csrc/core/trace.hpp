// Named ranges for external profilers (roctx under rocprofv3 --marker-trace).
// The host-only core has no ROCm dependency: the HIP module / GPU CLIs install
// roctxRangePushA / roctxRangePop here at load time; otherwise ranges are no-ops.
#pragma once

namespace tts {

struct TraceHooks {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
};

inline TraceHooks& trace_hooks() {
  static TraceHooks h;
  return h;
}

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(trace_hooks().push != nullptr) {
    if (on_) trace_hooks().push(name);
  }
  ~TraceRange() {
    if (on_ && trace_hooks().pop) trace_hooks().pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace tts

#define TTS_TRACE_CAT2(a, b) a##b
#define TTS_TRACE_CAT(a, b) TTS_TRACE_CAT2(a, b)
#define TTS_RANGE(name) ::tts::TraceRange TTS_TRACE_CAT(tts_range_, __LINE__)(name)
