// Host runtime self-test for sanitizer builds (the reference has no
// TSan/ASan targets). Exercises every concurrent host path with golden checks:
//   * multicore_search (work-stealing CPU threads, shared incumbent)
//   * run_workers with CPU engines (round barrier, leader plan, host staging,
//     watchdog thread, fault injection)
//   * multithreaded CpuEngine batches
// Build: g++ -O1 -g -fsanitize=thread (or address,undefined) ... ; exit code 0 = pass.
#include <chrono>
#include <cstdio>
#include <stdexcept>
#include <thread>
#include <memory>
#include <vector>

#include "../core/cpu_engine.hpp"
#include "../core/drivers_cpu.hpp"
#include "../core/hybrid_engine.hpp"
#include "../core/multi_engine.hpp"
#include "../core/runner.hpp"

using namespace tts;

static int failures = 0;
#define CHECK(c)                                                      \
  do {                                                                \
    if (!(c)) {                                                       \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

template <class Problem>
static void runner_case(Problem prob, int W, int threads, u64 gold_tree, u64 gold_sol, int best0, int gold_best,
                        unsigned fail_pct) {
  using Node = typename Problem::Node;
  Pool<Node> pool;
  pool.push_back_free(prob.root());
  u64 tree = 0, sol = 0;
  int best = best0;
  bfs_warmup(prob, pool, static_cast<size_t>(W) * 25, best, tree, sol);
  std::vector<std::unique_ptr<IEngine>> owned;
  std::vector<IEngine*> es;
  for (int w = 0; w < W; ++w) {
    owned.push_back(std::make_unique<CpuEngine<Problem>>(prob, 256, threads));
    es.push_back(owned.back().get());
  }
  std::vector<std::vector<uint8_t>> init(W);
  for (int w = 0; w < W; ++w) {
    Pool<Node> mine;
    mine.round_robin_from(pool, w, W);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(mine.data());
    init[w].assign(p, p + mine.size() * sizeof(Node));
  }
  RunnerConfig rc;
  rc.m = 10;
  rc.slice_min = 0.0002;
  rc.slice_max = 0.002;
  rc.watchdog_s = 5.0;
  rc.fault_delay_us = 50;
  rc.fault_steal_fail_pct = fail_pct;
  const auto rep = run_workers(es, init, best, rc);
  for (auto& r : rep) {
    tree += r.st.tree;
    sol += r.st.sol;
  }
  std::printf("runner W=%d threads=%d: tree %llu sol %llu best %d\n", W, threads, tree, sol, best);
  CHECK(tree == gold_tree);
  CHECK(sol == gold_sol);
  CHECK(best == gold_best);
}

int main() {
  // mid-size trees so a TSan build finishes in seconds; references from the
  // sequential driver (no threads involved)
  const PfspInstance in = make_taillard_instance(7);  // LB1_d, -u 1: 271,602 nodes
  MulticoreConfig mc;
  mc.m = 10;
  mc.batch = 500;
  const RunResult seq = run_pfsp_cpu(in, 0, in.best_known, 0, mc, false);
  std::printf("sequential: tree %llu sol %llu best %d\n", seq.tree, seq.sol, seq.best);
  const RunResult& seq_ub = seq;
  CHECK(seq.tree == 271602ull && seq.sol == 28447ull && seq.best == 1234);
  {  // multicore work stealing (ref pfsp_omp_c), known optimum: deterministic tree
    const RunResult r = run_pfsp_cpu(in, 0, seq.best, 4, mc, false);
    std::printf("multicore: tree %llu sol %llu best %d\n", r.tree, r.sol, r.best);
    CHECK(r.tree == seq_ub.tree && r.sol == seq_ub.sol && r.best == seq.best);
  }
  {  // unknown optimum: incumbent shared between threads (small instance)
    const PfspInstance small = make_instance(13, 6, synthetic_processing_times(13, 6, 5));
    const RunResult a = run_pfsp_cpu(small, 0, INT_MAX, 0, mc, false);
    const RunResult b = run_pfsp_cpu(small, 0, INT_MAX, 4, mc, false);
    CHECK(a.best == b.best);
  }
  runner_case(PfspProblem<20>(in, 0), 3, 1, seq_ub.tree, seq_ub.sol, seq.best, seq.best, 30);
  runner_case(PfspProblem<20>(in, 0), 2, 3, seq_ub.tree, seq_ub.sol, seq.best, seq.best, 0);
  // front-carrying nodes (the layout the engines use for LB1 / LB1_d on 20 jobs)
  runner_case(PfspFrontProblem<5>(in, 0), 3, 2, seq_ub.tree, seq_ub.sol, seq.best, seq.best, 30);
  runner_case(QueensProblem(10, 1), 4, 2, 35538ull, 724ull, 0, 0, 50);
  {  // hybrid rank engine (main engine + CPU worker thread), small batches: many hand-overs
    CpuEngine<PfspFrontProblem<5>> main_eng(PfspFrontProblem<5>(in, 0), 16, 1), cpu_eng(PfspFrontProblem<5>(in, 0), 16, 2);
    HybridConfig hc;
    hc.m = 4;
    hc.cpu_cap = 64;
    HybridEngine h(&main_eng, &cpu_eng, hc);
    const auto root = PfspFrontProblem<5>(in, 0).root();
    for (int rep = 0; rep < 2; ++rep) {
      const EngineStats st = h.solve_from(&root, 1, seq.best);
      std::printf("hybrid: tree %llu sol %llu (cpu worker %llu) best %d\n", st.tree, st.sol, st.cpu_tree, st.best);
      CHECK(st.tree == seq_ub.tree && st.sol == seq_ub.sol && st.best == seq.best);
      CHECK(st.cpu_tree > 0);
    }
    // time-sliced like the round loop
    h.begin(&root, 1, seq.best);
    while (h.size() > 0) h.run(-1, 0.002, 1);
    const EngineStats st = h.stats();
    CHECK(st.tree == seq_ub.tree && st.sol == seq_ub.sol);
  }
  {  // several sub-engines run concurrently as one engine, steal-half between slices
    CpuEngine<PfspFrontProblem<5>> a(PfspFrontProblem<5>(in, 0), 16, 1), b(PfspFrontProblem<5>(in, 0), 16, 1),
        c(PfspFrontProblem<5>(in, 0), 16, 1);
    MultiConfig mc2;
    mc2.needy_below = 8;
    mc2.donor_min = 32;
    MultiEngine me({&a, &b, &c}, nullptr, mc2);
    const auto root = PfspFrontProblem<5>(in, 0).root();
    const EngineStats st = me.solve_from(&root, 1, seq.best);
    std::printf("multi: tree %llu sol %llu best %d hand-overs %llu\n", st.tree, st.sol, st.best, me.handovers());
    CHECK(st.tree == seq_ub.tree && st.sol == seq_ub.sol && st.best == seq.best);
    CHECK(me.handovers() > 0);
    me.begin(&root, 1, seq.best);
    while (me.size() > 0) me.run(-1, 0.001, 1);
    const EngineStats s2 = me.stats();
    CHECK(s2.tree == seq_ub.tree && s2.sol == seq_ub.sol);
  }
  {  // sub-engine 0 throws inside a slice: run() rethrows only after the worker threads
     // have left their slices (no sub-engine still running when the caller unwinds)
    struct Throwing final : IEngine {
      IEngine* inner;
      std::atomic<int> calls{0};
      explicit Throwing(IEngine* e) : inner(e) {}
      size_t node_bytes() const override { return inner->node_bytes(); }
      void push_host(const void* n, size_t k) override { inner->push_host(n, k); }
      size_t pop_host(void* o, size_t k) override { return inner->pop_host(o, k); }
      size_t export_device(void* d, size_t k) override { return inner->export_device(d, k); }
      void import_device(const void* s, size_t k) override { inner->import_device(s, k); }
      size_t size() override { return inner->size(); }
      long run(long a, double b, size_t c) override {
        if (++calls >= 12) throw std::runtime_error("injected sub-engine failure");
        return inner->run(std::min<long>(a < 0 ? 4 : a, 4), b, c);
      }
      void begin(const void* n, size_t k, int b) override { inner->begin(n, k, b); }
      EngineStats solve_from(const void* n, size_t k, int b) override { return inner->solve_from(n, k, b); }
      size_t warm_split(int r, int w, size_t win, int p) override { return inner->warm_split(r, w, win, p); }
      void set_split(int r, int w, size_t mp) override { inner->set_split(r, w, mp); }
      bool split_pending() override { return inner->split_pending(); }
      void set_progress_hook(ProgressHook h) override { inner->set_progress_hook(std::move(h)); }
      void set_best(int b) override { inner->set_best(b); }
      int best() override { return inner->best(); }
      void reset_counters() override { inner->reset_counters(); }
      EngineStats stats() override { return inner->stats(); }
      void synchronize() override {}
      uintptr_t stream() const override { return 0; }
      int device() const override { return -1; }
    };
    CpuEngine<PfspFrontProblem<5>> a(PfspFrontProblem<5>(in, 0), 16, 1), b(PfspFrontProblem<5>(in, 0), 16, 1);
    Throwing ta(&a);
    MultiConfig mc3;
    mc3.needy_below = 8;
    mc3.donor_min = 32;
    MultiEngine me({&ta, &b}, nullptr, mc3);
    const auto root = PfspFrontProblem<5>(in, 0).root();
    bool threw = false;
    try {
      (void)me.solve_from(&root, 1, seq.best);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    CHECK(threw);
    const size_t s1 = b.size();  // the worker has left its slice: its pool no longer changes
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    CHECK(b.size() == s1);
    std::printf("multi with a throwing sub-engine: rethrown %d, worker pool stable at %zu\n", threw ? 1 : 0, s1);
  }
  std::printf(failures ? "SELFTEST FAILED\n" : "SELFTEST OK\n");
  return failures ? 1 : 0;
}
