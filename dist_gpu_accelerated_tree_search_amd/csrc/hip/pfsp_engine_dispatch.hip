// Run-time dispatch of PFSP engines / bound evaluation over the job-count buckets.
#include "pfsp_engine.hpp"

namespace tts {

std::unique_ptr<IEngine> make_pfsp_engine(const PfspInstance& in, int lb, const EngineConfig& cfg) {
  switch (pfsp_bucket(in.jobs)) {
    case 20: return make_pfsp_engine_nj20(in, lb, cfg);
    case 50: return make_pfsp_engine_nj50(in, lb, cfg);
    case 100: return make_pfsp_engine_nj100(in, lb, cfg);
    case 200: return make_pfsp_engine_nj200(in, lb, cfg);
    default: return make_pfsp_engine_nj500(in, lb, cfg);
  }
}

std::vector<int> pfsp_gpu_bounds(const PfspInstance& in, int lb, const void* parents, size_t n, int best, int device) {
  switch (pfsp_bucket(in.jobs)) {
    case 20: return pfsp_gpu_bounds_nj20(in, lb, parents, n, best, device);
    case 50: return pfsp_gpu_bounds_nj50(in, lb, parents, n, best, device);
    case 100: return pfsp_gpu_bounds_nj100(in, lb, parents, n, best, device);
    case 200: return pfsp_gpu_bounds_nj200(in, lb, parents, n, best, device);
    default: return pfsp_gpu_bounds_nj500(in, lb, parents, n, best, device);
  }
}

std::vector<int> pfsp_expand_probe(const PfspInstance& in, int lb, const void* parents, size_t n, int best, int device,
                                   int variant, int reps, std::vector<double>* timing, ExpandProbeResult* extra) {
  switch (pfsp_bucket(in.jobs)) {
    case 20: return pfsp_expand_probe_nj20(in, lb, parents, n, best, device, variant, reps, timing, extra);
    case 50: return pfsp_expand_probe_nj50(in, lb, parents, n, best, device, variant, reps, timing, extra);
    case 100: return pfsp_expand_probe_nj100(in, lb, parents, n, best, device, variant, reps, timing, extra);
    case 200: return pfsp_expand_probe_nj200(in, lb, parents, n, best, device, variant, reps, timing, extra);
    default: return pfsp_expand_probe_nj500(in, lb, parents, n, best, device, variant, reps, timing, extra);
  }
}

ExpandProbeResult pfsp_lb1_expand_probe(const PfspInstance& in, const void* parents, size_t n, int best, int device) {
  switch (pfsp_bucket(in.jobs)) {
    case 20: return pfsp_lb1_expand_probe_nj20(in, parents, n, best, device);
    case 50: return pfsp_lb1_expand_probe_nj50(in, parents, n, best, device);
    case 100: return pfsp_lb1_expand_probe_nj100(in, parents, n, best, device);
    case 200: return pfsp_lb1_expand_probe_nj200(in, parents, n, best, device);
    default: return pfsp_lb1_expand_probe_nj500(in, parents, n, best, device);
  }
}

}  // namespace tts
