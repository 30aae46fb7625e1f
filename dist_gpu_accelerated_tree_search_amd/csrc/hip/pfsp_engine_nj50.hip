// Kernel instantiations for the 50-job node bucket (one TU per bucket so the
// instantiations compile in parallel).
#include "pfsp_engine.hpp"

namespace tts {
TTS_PFSP_DEFINE_BUCKET(50)

// 21-50 jobs on front nodes with 64-bit job sets (pfsp_front_probe / pfsp_front_time
// dispatch here from the 20-job TU)
FrontProbeResult pfsp_front_probe_nj50(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                       const EngineConfig& cfg, unsigned cap, int split_rank, int split_world,
                                       size_t split_min) {
  return with_machine_bucket(in.machines, [&](auto mm) {
    return pfsp_front_probe_t<decltype(mm)::value, 50>(in, lb, nodes, n, best, cfg, cap, split_rank, split_world,
                                                       split_min);
  });
}
std::vector<double> pfsp_front_time_nj50(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                         const EngineConfig& cfg, int reps) {
  return with_machine_bucket(in.machines, [&](auto mm) {
    return pfsp_front_time_t<decltype(mm)::value, 50>(in, lb, nodes, n, best, cfg, reps);
  });
}
}  // namespace tts
