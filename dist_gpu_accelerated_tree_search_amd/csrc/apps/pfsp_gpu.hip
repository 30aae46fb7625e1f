// Native multi-GPU PFSP B&B CLI, one process (ref pfsp/pfsp_multigpu_cuda.c:513-588):
//   -D GPUs (one host thread + device-resident engine each), -C 1 adds a CPU worker
//   with the remaining hardware threads, -w work sharing between workers,
//   -m / -M / -T thresholds, the reference's stdout blocks and multigpu.csv row.
// The multi-process (RCCL) equivalent is `python -m dist_gpu_accelerated_tree_search_amd pfsp -D N`.
#include <climits>
#include <cstdlib>
#include <thread>

#include "../core/cpu_engine.hpp"
#include "../core/drivers_cpu.hpp"
#include "../core/runner.hpp"
#include "../hip/host_support.hpp"
#include "../hip/pfsp_engine.hpp"

using namespace tts;

int main(int argc, char* argv[]) {
  install_roctx_hooks();
  PfspArgs a = parse_pfsp_args(argc, argv);
  if (a.C < 0 || a.C > 1) {
    std::printf("C is set to %d. Invalid option for this version.\nChoose 0 to unable and 1 to enable multi-core. "
                "Mapping automatically done.\n", a.C);
    return 1;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess) ndev = 0;
  if (a.D > ndev) {
    std::printf("Execution Terminated. More GPU devices requested than the ones available\n");
    return 1;
  }
  if (a.D == 0 && a.C == 0) {
    std::printf("No processing units requested. Please set D or C to at least 1\n");
    return 1;
  }
  const PfspInstance in = make_taillard_instance(a.inst);
  const int hw = static_cast<int>(std::thread::hardware_concurrency());
  const int cpu_threads = a.C ? std::max(1, hw - a.D) : 0;
  print_pfsp_settings(a.inst, in.machines, in.jobs, a.ub, a.lb, a.D, a.C, a.ws, 1, a.L, 2);
  for (int d = 0; d < a.D; ++d) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, d) == hipSuccess)
      std::printf("GPU %d: %s (%s), %d CUs, %.0f GB\n", d, p.name, p.gcnArchName, p.multiProcessorCount,
                  p.totalGlobalMem / 1e9);
  }
  int best = a.ub == 1 ? in.best_known : INT_MAX;
  const size_t max_parents = std::getenv("TTS_MAX_PARENTS") ? std::strtoull(std::getenv("TTS_MAX_PARENTS"), nullptr, 10)
                                                           : (size_t(1) << 18);

  std::vector<std::unique_ptr<IEngine>> owned;
  for (int d = 0; d < a.D; ++d) {
    EngineConfig cfg;
    cfg.device = d;
    cfg.max_parents = max_parents;
    owned.push_back(make_pfsp_engine(in, a.lb, cfg));
  }
  const int host_lb = a.lb == 1 ? 0 : a.lb;  // ref: CPU workers use LB1_d for LB1
  // the engines' node layout (front nodes for LB1 / LB1_d on 20-job instances)
  return with_pfsp_problem(in, host_lb, [&](auto prob) {
    using Problem = decltype(prob);
    using Node = typename Problem::Node;
    if (cpu_threads > 0) owned.push_back(std::make_unique<CpuEngine<Problem>>(prob, a.T, cpu_threads));
    std::vector<IEngine*> engines;
    for (auto& e : owned) engines.push_back(e.get());
    const int W = static_cast<int>(engines.size());

    // Step 1: host breadth-first warm-up to W*m nodes
    const double t0 = now_s();
    Pool<Node> pool;
    pool.push_back_free(prob.root());
    u64 tree = 0, sol = 0;
    bfs_warmup(prob, pool, static_cast<size_t>(W) * a.m, best, tree, sol);
    const double t1 = now_s();
    print_phase("Initial search on CPU completed", tree, sol, t1 - t0);

    // Step 2: all workers, round-robin split (ref roundRobin_distribution)
    std::vector<std::vector<uint8_t>> init(W);
    for (int w = 0; w < W; ++w) {
      Pool<Node> mine;
      mine.round_robin_from(pool, w, W);
      const uint8_t* p = reinterpret_cast<const uint8_t*>(mine.data());
      init[w].assign(p, p + mine.size() * sizeof(Node));
    }
    RunnerConfig rc;
    rc.m = a.m;
    rc.steal_cap = static_cast<size_t>(5) * a.M;
    rc.work_sharing = a.ws == 1;
    // GPU workers: needy below a quarter of the parent window, donors from one
    // window; the CPU worker: the reference's m / 2m, at most 4*T per steal
    for (auto* e : engines) {
      const bool gpu = e->device() >= 0;
      const size_t nb = gpu ? std::max<size_t>(a.m, max_parents / 4) : static_cast<size_t>(a.m);
      rc.needy_below.push_back(nb);
      rc.donor_min.push_back(gpu ? std::max(2 * nb, max_parents) : 2 * nb);
      rc.recv_cap.push_back(gpu ? rc.steal_cap : std::min<size_t>(rc.steal_cap, static_cast<size_t>(4) * a.T));
    }
    rc.merge_env();
    for (auto* e : engines) rc.worker_cpus.push_back(e->device() >= 0 ? device_cpus(e->device()) : std::vector<int>{});
    HipStaging staging;
    const auto rep = run_workers(engines, init, best, rc, &staging);
    std::vector<WorkerStats> ws(W);
    for (int w = 0; w < W; ++w) {
      tree += rep[w].st.tree;
      sol += rep[w].st.sol;
      ws[w].tree = rep[w].st.tree;
      ws[w].sol = rep[w].st.sol;
      ws[w].gen_child = rep[w].st.tree;
      ws[w].steals = rep[w].steals;
      ws[w].success_steals = rep[w].success_steals;
      ws[w].terminations = rep[w].idle_rounds;
      ws[w].t_termination = rep[w].t_termination;
      ws[w].t_memcpy = rep[w].st.t_memcpy;
      ws[w].t_malloc = rep[w].st.t_malloc;
      ws[w].t_kernel = rep[w].t_run;
      ws[w].t_pool_ops = rep[w].t_comm;
      ws[w].t_idle = rep[w].t_idle;
    }
    const double t2 = now_s();
    print_phase("Search on Parallel GPU completed", tree, sol, t2 - t1);
    // Step 3: the device engines drain their pools; nothing is left for the host
    print_phase("Final on CPU completed", tree, sol, 0.0);
    std::printf("\nExploration terminated.\n");
    print_pfsp_results(best, tree, sol, t2 - t0);
    write_csv_multi_gpu("multigpu.csv", a.inst, a.lb, a.D, W - a.D, a.ws, best, a.m, a.M, a.T, tree, sol, t2 - t0, ws);
    return 0;
  });
}
