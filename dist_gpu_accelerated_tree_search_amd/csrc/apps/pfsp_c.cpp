// Sequential PFSP B&B CLI (ref pfsp/pfsp_c.c:75-99): same flags, stdout block.
#include <climits>

#include "../core/drivers_cpu.hpp"

int main(int argc, char* argv[]) {
  const tts::PfspArgs a = tts::parse_pfsp_args(argc, argv);
  const tts::PfspInstance in = tts::make_taillard_instance(a.inst);
  tts::print_pfsp_settings(a.inst, in.machines, in.jobs, a.ub, a.lb, 0, 0, 0, 1, 0, 0);
  const int best0 = a.ub == 1 ? in.best_known : INT_MAX;
  const tts::RunResult r = tts::run_pfsp_cpu(in, a.lb, best0, 0, tts::MulticoreConfig{}, false);
  std::printf("\nExploration terminated.\n");
  tts::print_pfsp_results(r.best, r.tree, r.sol, r.elapsed);
  return 0;
}
