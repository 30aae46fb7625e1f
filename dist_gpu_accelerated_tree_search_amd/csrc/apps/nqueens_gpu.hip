// Native N-Queens GPU CLI, one process (ref nqueens/nqueens_gpu_cuda.cu and
// nqueens_multigpu_cuda.cu): -N -g -m -M -D. The reference's multi-GPU version
// splits statically with no work stealing; here the D device engines share work.
#include <algorithm>
#include <cstdlib>
#include <memory>

#include "../core/drivers_cpu.hpp"
#include "../core/multi_engine.hpp"
#include "../core/runner.hpp"
#include "../hip/host_support.hpp"
#include "../hip/queens_engine.hpp"

using namespace tts;

int main(int argc, char* argv[]) {
  install_roctx_hooks();
  const QueensArgs a = parse_queens_args(argc, argv, true);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  if (a.D > ndev) {
    std::printf("Execution Terminated. More GPU devices requested than the ones available\n");
    return 1;
  }
  char banner[96];
  std::snprintf(banner, sizeof banner, "Multi-GPU C++/HIP (%d GPUs)", a.D);
  print_queens_settings(a.N, a.g, banner);
  // K engines per GPU (one stream and host thread each) with the solve split between them
  // in the graph, as one engine per GPU: N=17 33 -> 18 ms with 3 on one MI355X
  // (profiles/r6/queens/lazy_xfer_ab.txt); TTS_STREAMS overrides
  int K = 3;
  if (const char* s = std::getenv("TTS_STREAMS")) K = std::max(1, std::atoi(s));
  const size_t window = size_t(1) << 19;  // the kernel's largest parent window
  std::vector<std::unique_ptr<IEngine>> subs;   // destroyed after the multi-engines below
  std::vector<std::unique_ptr<IEngine>> owned;
  std::vector<IEngine*> engines;
  for (int d = 0; d < a.D; ++d) {
    std::vector<IEngine*> mine;
    for (int k = 0; k < K; ++k) {
      EngineConfig cfg;
      cfg.device = d;
      cfg.max_parents = window;
      cfg.ring_bytes = (size_t(16) << 30) / static_cast<size_t>(K);
      subs.push_back(make_queens_engine(a.N, a.g, cfg));
      mine.push_back(subs.back().get());
    }
    if (K == 1) {
      engines.push_back(mine[0]);
      continue;
    }
    MultiConfig mc;
    mc.needy_below = window / 16;
    mc.donor_min = window / 4;
    mc.split_min = 512;
    owned.push_back(std::make_unique<MultiEngine>(std::move(mine), std::make_unique<HipStaging>(), mc));
    engines.push_back(owned.back().get());
  }
  const double t0 = now_s();
  QueensProblem prob(a.N, a.g);
  Pool<QueensNode> pool;
  pool.push_back_free(prob.root());
  u64 tree = 0, sol = 0;
  int best = 0;
  bfs_warmup(prob, pool, static_cast<size_t>(a.D) * a.m, best, tree, sol);
  const double t1 = now_s();
  print_phase("Initial search on CPU completed", tree, sol, t1 - t0);
  std::vector<std::vector<uint8_t>> init(a.D);
  for (int w = 0; w < a.D; ++w) {
    Pool<QueensNode> mine;
    mine.round_robin_from(pool, w, a.D);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(mine.data());
    init[w].assign(p, p + mine.size() * sizeof(QueensNode));
  }
  RunnerConfig rc;
  rc.m = a.m;
  rc.steal_cap = static_cast<size_t>(5) * a.M;
  rc.merge_env();
  for (auto* e : engines) rc.worker_cpus.push_back(device_cpus(e->device()));
  HipStaging staging;
  const auto rep = run_workers(engines, init, best, rc, &staging);
  for (auto& r : rep) {
    tree += r.st.tree;
    sol += r.st.sol;
  }
  const double t2 = now_s();
  print_phase("Search on GPU completed", tree, sol, t2 - t1);
  std::printf("\nExploration terminated.\n");
  print_queens_results(tree, sol, t2 - t0);
  return 0;
}
