// Kernel instantiations for the 20-job node bucket (one TU per bucket so the
// instantiations compile in parallel).
#include "pfsp_engine.hpp"

namespace tts {
TTS_PFSP_DEFINE_BUCKET(20)

FrontProbeResult pfsp_front_probe(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                  const EngineConfig& cfg, unsigned cap, int split_rank, int split_world,
                                  size_t split_min) {
  if (!pfsp_front_ok(in, lb)) throw std::invalid_argument("front probe: the front layout does not apply");
  if (in.jobs > 20) return pfsp_front_probe_nj50(in, lb, nodes, n, best, cfg, cap, split_rank, split_world, split_min);
  return with_machine_bucket(in.machines, [&](auto mm) {
    return pfsp_front_probe_t<decltype(mm)::value>(in, lb, nodes, n, best, cfg, cap, split_rank, split_world,
                                                   split_min);
  });
}
std::vector<double> pfsp_front_time(const PfspInstance& in, int lb, const void* nodes, size_t n, int best,
                                    const EngineConfig& cfg, int reps) {
  if (!pfsp_front_ok(in, lb)) throw std::invalid_argument("front timing: the front layout does not apply");
  if (in.jobs > 20) return pfsp_front_time_nj50(in, lb, nodes, n, best, cfg, reps);
  return with_machine_bucket(in.machines, [&](auto mm) {
    return pfsp_front_time_t<decltype(mm)::value>(in, lb, nodes, n, best, cfg, reps);
  });
}

}  // namespace tts
