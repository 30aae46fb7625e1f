// Sequential N-Queens backtracking CLI (ref nqueens/nqueens_c.c:150-166).
#include "../core/drivers_cpu.hpp"

int main(int argc, char* argv[]) {
  const tts::QueensArgs a = tts::parse_queens_args(argc, argv, false);
  tts::print_queens_settings(a.N, a.g, "Sequential C++");
  const tts::RunResult r = tts::run_queens_cpu(a.N, a.g, 0, tts::MulticoreConfig{}, false);
  std::printf("\nExploration terminated.");
  tts::print_queens_results(r.tree, r.sol, r.elapsed);
  return 0;
}
