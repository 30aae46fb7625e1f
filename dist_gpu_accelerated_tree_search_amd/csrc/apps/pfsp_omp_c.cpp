// Multi-core PFSP B&B CLI (ref pfsp/pfsp_omp_c.c:372-434): -C threads, -w work
// stealing, -m / -M thresholds; appends a row to multigpu.csv like the reference.
#include <climits>
#include <thread>

#include "../core/drivers_cpu.hpp"

int main(int argc, char* argv[]) {
  tts::PfspArgs a = tts::parse_pfsp_args(argc, argv);
  a.D = 0;
  const int nproc = static_cast<int>(std::thread::hardware_concurrency());
  if (a.C > nproc) {
    std::printf("Execution Terminated. More processing units requested than the ones available\n");
    return 1;
  }
  if (a.C == 0) {
    std::printf("No processing units requested. Please set C to at least 1\n");
    return 1;
  }
  const tts::PfspInstance in = tts::make_taillard_instance(a.inst);
  tts::print_pfsp_settings(a.inst, in.machines, in.jobs, a.ub, a.lb, a.D, a.C, a.ws, 1, a.L, 2);
  const int best0 = a.ub == 1 ? in.best_known : INT_MAX;
  tts::MulticoreConfig cfg;
  cfg.m = a.m;
  cfg.batch = 20000;
  cfg.steal_cap = static_cast<size_t>(5) * a.M;
  cfg.work_stealing = a.ws == 1;
  const tts::RunResult r = tts::run_pfsp_cpu(in, a.lb, best0, a.C, cfg, true);
  tts::print_pfsp_results(r.best, r.tree, r.sol, r.elapsed);
  tts::write_csv_multi_gpu("multigpu.csv", a.inst, a.lb, a.D, a.C, a.ws, r.best, a.m, a.M, a.T, r.tree, r.sol, r.elapsed,
                           r.workers);
  return 0;
}
