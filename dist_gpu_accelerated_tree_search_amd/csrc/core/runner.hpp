// Single-process multi-worker runner: several engines (GPUs and/or CPU workers)
// driven by one host thread each, sharing work in lock-step rounds.
//
// Parity: ref pfsp/pfsp_multigpu_cuda.c:55-511 — one OpenMP thread per GPU, optional
// CPU worker threads (-C 1), random steal-half work stealing under spin locks,
// BUSY/IDLE termination, checkBest incumbent sharing. Here the same roles run as:
//   * each worker runs its engine for a time slice (device-resident search);
//   * a round = barrier -> leader reads every pool size + incumbent, takes the
//     MIN incumbent, detects termination (all pools empty: exact, nothing is in
//     flight between rounds), plans steal-half transfers (same plan as
//     parallel/comm.py::plan_sharing) -> barrier -> donors move nodes -> barrier
//     -> receivers load them -> next slice.
//   * GPU -> GPU transfers go device pool -> staging buffer on the receiver's
//     device (peer copy over xGMI, DeviceStaging) -> receiver pool; transfers that
//     involve a CPU worker are staged through host memory.
// Aux subsystems: host threads pinned to the NUMA node of their GPU,
// a watchdog that reports (and optionally aborts) a stuck phase, env-driven fault
// injection (TTS_FAULT_DELAY_US, TTS_FAULT_STEAL_FAIL_PCT, TTS_FAULT_STALL), and
// named trace ranges (roctx when the HIP module installs it).
// The multi-process equivalent over RCCL is parallel/runtime.py.
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "dist_rounds.hpp"
#include "engine_api.hpp"
#include "topology.hpp"
#include "trace.hpp"

namespace tts {

struct RunnerConfig {
  size_t m = 25;               // needy below m nodes, donors need >= 2m (unless set per worker)
  size_t steal_cap = 250000;   // ref 5*M
  // per-worker thresholds (plan_transfers): GPU workers in units of their parent
  // window, CPU workers the reference's m / 2m with a 4*T receive cap
  std::vector<size_t> needy_below, donor_min, recv_cap;
  double slice_min = 0.0005;   // seconds of local search between rounds (adaptive)
  double slice_max = 0.05;
  bool work_sharing = true;    // ref -w
  std::vector<std::vector<int>> worker_cpus;  // optional CPU set per worker (pinning)
  double watchdog_s = 0;       // report a phase longer than this (0: off)
  bool watchdog_abort = false; // abort the process after the report
  // fault injection
  unsigned fault_delay_us = 0;        // random extra delay per worker per round
  unsigned fault_steal_fail_pct = 0;  // planned transfers dropped (seeded)
  int fault_stall_worker = -1;        // this worker stalls once (round 1) ...
  double fault_stall_s = 0;           // ... for this long
  unsigned long long fault_seed = 12345;

  // TTS_WATCHDOG_S, TTS_WATCHDOG_ABORT, TTS_FAULT_DELAY_US, TTS_FAULT_STEAL_FAIL_PCT,
  // TTS_FAULT_STALL="worker:seconds"
  void merge_env() {
    auto env = [](const char* k) -> const char* {
      const char* v = std::getenv(k);
      return (v && *v) ? v : nullptr;
    };
    if (auto v = env("TTS_WATCHDOG_S")) watchdog_s = std::atof(v);
    if (auto v = env("TTS_WATCHDOG_ABORT")) watchdog_abort = std::atoi(v) != 0;
    if (auto v = env("TTS_FAULT_DELAY_US")) fault_delay_us = static_cast<unsigned>(std::atol(v));
    if (auto v = env("TTS_FAULT_STEAL_FAIL_PCT")) fault_steal_fail_pct = static_cast<unsigned>(std::atol(v));
    if (auto v = env("TTS_FAULT_STALL")) {
      const std::string s(v);
      const auto c = s.find(':');
      if (c != std::string::npos) {
        fault_stall_worker = std::atoi(s.substr(0, c).c_str());
        fault_stall_s = std::atof(s.substr(c + 1).c_str());
      }
    }
  }
};

struct WorkerReport {
  EngineStats st;
  unsigned long long rounds = 0, sent = 0, received = 0, transfers_in = 0, transfers_out = 0;
  unsigned long long device_transfers = 0, dropped_transfers = 0, watchdog_events = 0;
  unsigned long long steals = 0, success_steals = 0, idle_rounds = 0;  // ref nbSteals / nbSSteals / nbTermination
  unsigned long long early_rounds = 0;  // rounds this worker called early (ran dry while a peer could donate)
  double t_run = 0, t_comm = 0, t_idle = 0, t_termination = 0;
  bool pinned = false;
};

class RoundBarrier {
 public:
  explicit RoundBarrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const unsigned long long gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen != gen_; });
    }
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  unsigned long long gen_ = 0;
};

// Worker phases seen by the watchdog.
enum class Phase : int { Start = 0, Run = 1, Report = 2, Barrier = 3, Transfer = 4, Done = 5 };
inline const char* phase_name(int p) {
  static const char* n[] = {"start", "run", "report", "barrier", "transfer", "done"};
  return (p >= 0 && p <= 5) ? n[p] : "?";
}

// Runs all workers to exhaustion. initial[w] holds worker w's starting nodes
// (node_bytes each). Returns per-worker reports; `best` is updated to the final
// incumbent. Engines must share one node layout.
inline std::vector<WorkerReport> run_workers(const std::vector<IEngine*>& engines,
                                             const std::vector<std::vector<uint8_t>>& initial, int& best,
                                             const RunnerConfig& cfg, DeviceStaging* staging = nullptr) {
  const int W = static_cast<int>(engines.size());
  if (W == 0) return {};
  if (initial.size() != engines.size()) throw std::invalid_argument("one initial node set per worker");
  const size_t nb = engines[0]->node_bytes();
  for (auto* e : engines)
    if (e->node_bytes() != nb) throw std::invalid_argument("workers disagree on the node layout");
  std::vector<WorkerReport> rep(W);
  std::vector<size_t> sizes(W, 0);
  std::vector<int> bests(W, best);
  std::vector<std::vector<uint8_t>> staging_host(W);  // staging_host[r]: nodes bound for worker r
  // device staging: dbuf[r] on worker r's device, written by its (single) donor
  std::vector<void*> dbuf;
  std::vector<size_t> dcap(W, 0), dcount(W, 0);
  std::vector<int> donor_of(W, -1);
  std::vector<std::atomic<unsigned long long>> ready(W);  // round whose transfer to worker r is enqueued
  for (auto& x : ready) x.store(0);
  std::vector<uintptr_t> ready_ev, done_ev;                // [donor * W + receiver] on the donor's device / [receiver]
  std::vector<std::tuple<int, int, size_t>> plan;
  auto per = [&](const std::vector<size_t>& v, size_t dflt) {
    std::vector<size_t> out(W, dflt);
    for (int x = 0; x < W && x < static_cast<int>(v.size()); ++x) out[x] = v[x];
    return out;
  };
  const std::vector<size_t> needy = per(cfg.needy_below, cfg.m), donor = per(cfg.donor_min, 2 * cfg.m),
                            rcap = per(cfg.recv_cap, cfg.steal_cap);
  // device staging and events, allocated once: a receiving GPU gets a buffer for its
  // largest transfer (recv cap); pairs of GPU workers get an event each way
  bool any_gpu_pair = false;
  for (int x = 0; x < W; ++x)
    for (int y = 0; y < W; ++y) any_gpu_pair |= x != y && engines[x]->device() >= 0 && engines[y]->device() >= 0;
  if (staging && any_gpu_pair && cfg.work_sharing) {
    dbuf.assign(W, nullptr);
    ready_ev.assign(static_cast<size_t>(W) * W, 0);
    done_ev.assign(W, 0);
    for (int x = 0; x < W; ++x) {
      if (engines[x]->device() < 0) continue;
      dcap[x] = std::min<size_t>(rcap[x], (size_t(1) << 30) / std::max<size_t>(1, nb)) * nb;
      dbuf[x] = staging->alloc(engines[x]->device(), dcap[x]);
      done_ev[x] = staging->make_event(engines[x]->device());
      for (int y = 0; y < W; ++y)
        if (y != x && engines[y]->device() >= 0)
          ready_ev[static_cast<size_t>(y) * W + x] = staging->make_event(engines[y]->device());
    }
  }
  bool done = false;
  int gbest = best;
  std::vector<std::atomic<size_t>> live(W);
  for (auto& x : live) x.store(0);
  std::atomic<unsigned long long> request{0};
  std::atomic<int> live_best{best};  // node-wide incumbent, exchanged after every replay
  double slice = cfg.slice_min;
  RoundBarrier bar(W);
  std::mutex stage_mu;
  std::mt19937_64 fault_rng(cfg.fault_seed);

  using clock = std::chrono::steady_clock;
  auto now = [] { return clock::now(); };
  auto secs = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };

  // A worker whose engine throws keeps taking part in the rounds with an empty
  // pool (so no thread waits forever at a barrier); the first error is rethrown.
  std::exception_ptr err;
  std::mutex err_mu;
  auto fail = [&](std::exception_ptr p) {
    std::lock_guard<std::mutex> lk(err_mu);
    if (!err) err = p;
  };

  // ---- watchdog: per-worker heartbeat {phase, round, phase start} ----
  struct Beat {
    std::atomic<int> phase{0};
    std::atomic<unsigned long long> round{0};
    std::atomic<clock::rep> since{0};
    std::atomic<bool> reported{false};
  };
  std::vector<Beat> beats(W);
  auto beat = [&](int w, Phase p) {
    beats[w].since.store(clock::now().time_since_epoch().count(), std::memory_order_relaxed);
    beats[w].reported.store(false, std::memory_order_relaxed);
    beats[w].phase.store(static_cast<int>(p), std::memory_order_release);
  };
  std::atomic<bool> finished{false};
  std::atomic<unsigned long long> watchdog_events{0};
  std::thread watchdog;
  if (cfg.watchdog_s > 0) {
    watchdog = std::thread([&] {
      const auto tick = std::chrono::duration<double>(std::max(0.001, cfg.watchdog_s / 4));
      while (!finished.load()) {
        std::this_thread::sleep_for(tick);
        const clock::rep t = clock::now().time_since_epoch().count();
        for (int w = 0; w < W; ++w) {
          const int ph = beats[w].phase.load(std::memory_order_acquire);
          if (ph == static_cast<int>(Phase::Done) || ph == static_cast<int>(Phase::Barrier)) continue;
          const double age = std::chrono::duration<double>(clock::duration(t - beats[w].since.load())).count();
          if (age < cfg.watchdog_s || beats[w].reported.exchange(true)) continue;
          ++watchdog_events;
          std::fprintf(stderr, "[tts watchdog] worker %d stuck in phase '%s' for %.3f s (round %llu); state:\n", w,
                       phase_name(ph), age, beats[w].round.load());
          for (int x = 0; x < W; ++x)
            std::fprintf(stderr, "  worker %d device %d phase %s round %llu\n", x, engines[x]->device(),
                         phase_name(beats[x].phase.load()), beats[x].round.load());
          std::fflush(stderr);
          if (cfg.watchdog_abort) std::abort();
        }
      }
    });
  }

  auto worker = [&](int w) {
    IEngine* e = engines[w];
    WorkerReport& r = rep[w];
    bool dead = false;
    auto guarded = [&](auto&& f) {
      if (dead) return;
      try {
        f();
      } catch (...) {
        fail(std::current_exception());
        dead = true;
      }
    };
    if (w < static_cast<int>(cfg.worker_cpus.size()) && !cfg.worker_cpus[w].empty())
      r.pinned = pin_current_thread(cfg.worker_cpus[w]);
    std::mt19937 jitter(static_cast<unsigned>(cfg.fault_seed + 7919u * static_cast<unsigned>(w)));
    beat(w, Phase::Start);
    const std::vector<uint8_t>& init = initial[w];
    guarded([&] { e->begin(init.data(), init.size() / nb, best); });
    // early rounds (as in dist_rounds.hpp): publish the live pool size after every
    // replay and exchange the incumbent with every worker (ref checkBest before and
    // after every batch, pfsp_multigpu_cuda.c:30-50,307-312); leave the slice when a
    // dry worker asked for the next round
    e->set_progress_hook([&, w](size_t pool, int& b) {
      live[w].store(pool, std::memory_order_relaxed);
      int cur = live_best.load(std::memory_order_acquire);
      while (b < cur && !live_best.compare_exchange_weak(cur, b, std::memory_order_acq_rel)) {
      }
      if (cur < b) b = cur;
      return cfg.work_sharing && request.load(std::memory_order_acquire) > rep[w].rounds;
    });
    for (;;) {
      const auto t0 = now();
      beat(w, Phase::Run);
      {
        TTS_RANGE("tts.run_slice");
        guarded([&] { e->run(-1, slice, 1); });
      }
      const auto t1 = now();
      r.t_run += secs(t0, t1);
      beat(w, Phase::Report);
      if (cfg.fault_delay_us)
        std::this_thread::sleep_for(std::chrono::microseconds(jitter() % (cfg.fault_delay_us + 1)));
      if (w == cfg.fault_stall_worker && r.rounds == 1 && cfg.fault_stall_s > 0)
        std::this_thread::sleep_for(std::chrono::duration<double>(cfg.fault_stall_s));
      sizes[w] = 0;
      guarded([&] {
        sizes[w] = e->size();
        bests[w] = e->best();
      });
      live[w].store(sizes[w], std::memory_order_relaxed);
      if (cfg.work_sharing && W > 1 && sizes[w] < needy[w]) {  // dry: call the round early if someone can donate
        for (int x = 0; x < W; ++x)
          if (x != w && live[x].load(std::memory_order_relaxed) >= donor[x]) {
            unsigned long long cur = request.load();
            const unsigned long long want = rep[w].rounds + 1;
            while (cur < want && !request.compare_exchange_weak(cur, want)) {
            }
            ++rep[w].early_rounds;
            break;
          }
      }
      beat(w, Phase::Barrier);
      TTS_RANGE("tts.round");
      bar.wait();
      if (w == 0) {  // leader: incumbent, termination, plan
        gbest = *std::min_element(bests.begin(), bests.end());
        size_t total = 0;
        bool starving = false;
        for (int x = 0; x < W; ++x) {
          total += sizes[x];
          starving |= sizes[x] < needy[x];
        }
        done = total == 0;
        plan.clear();
        if (!done && cfg.work_sharing && W > 1 && starving) {
          std::vector<int64_t> sz(sizes.begin(), sizes.end());
          for (const auto& t : plan_transfers(sz, needy, donor, rcap)) plan.emplace_back(t.donor, t.receiver, t.n);
          if (cfg.fault_steal_fail_pct) {
            std::vector<std::tuple<int, int, size_t>> kept;
            for (auto& t : plan) {
              if (fault_rng() % 100 < cfg.fault_steal_fail_pct)
                ++rep[std::get<1>(t)].dropped_transfers;
              else
                kept.push_back(t);
            }
            plan.swap(kept);
          }
        }
        slice = starving ? cfg.slice_min : std::min(cfg.slice_max, slice * 2);
      }
      bar.wait();
      ++r.rounds;
      beats[w].round.store(r.rounds, std::memory_order_relaxed);
      if (done) {
        r.t_comm += secs(t1, now());
        r.t_termination += secs(t1, now());
        break;
      }
      const bool needy_w = cfg.work_sharing && W > 1 && sizes[w] < needy[w];
      if (needy_w) ++r.steals;
      if (gbest < bests[w]) guarded([&] { e->set_best(gbest); });
      if (!plan.empty()) {
        // Only the workers named in the plan take part; the others go straight on to
        // their next slice. A donor enqueues the copy of its pool bottom into the
        // receiver's staging buffer (device staging on the receiver's GPU when both
        // ends are GPUs, peer copy over xGMI; host staging otherwise), records an event
        // and publishes the count; the receiver's stream waits on that event before
        // its import, and the donor of a later round waits on the receiver's "import
        // done" event before it overwrites the buffer. No host sync on either side.
        const unsigned long long round_id = r.rounds;
        beat(w, Phase::Transfer);
        TTS_RANGE("tts.transfer");
        for (const auto& t : plan) {
          const int d = std::get<0>(t), rc = std::get<1>(t);
          const size_t k = std::get<2>(t);
          if (d != w) continue;
          const bool on_device = !dbuf.empty() && dbuf[rc] && e->device() >= 0;
          size_t got = 0;
          if (on_device) {
            guarded([&] {
              e->wait_event(done_ev[rc]);  // the receiver's previous import has read the buffer
              got = e->export_device(dbuf[rc], std::min(k, dcap[rc] / nb));
              e->record_event(ready_ev[static_cast<size_t>(d) * W + rc]);
            });
            ++r.device_transfers;
          } else {
            std::vector<uint8_t> buf(k * nb);
            guarded([&] { got = e->pop_host(buf.data(), k); });
            buf.resize(got * nb);
            std::lock_guard<std::mutex> lk(stage_mu);
            staging_host[rc].insert(staging_host[rc].end(), buf.begin(), buf.end());
          }
          dcount[rc] = on_device ? got : 0;
          donor_of[rc] = d;
          ready[rc].store(round_id, std::memory_order_release);
          r.sent += got;
          ++r.transfers_out;
        }
        bool receiving = false;
        for (const auto& t : plan) receiving |= std::get<1>(t) == w;
        if (receiving) {
          // wait until the donor has enqueued its copy (not until it completed)
          while (ready[w].load(std::memory_order_acquire) != round_id) std::this_thread::yield();
          size_t in = 0;
          if (dcount[w]) {
            const int d = donor_of[w];
            guarded([&] {
              e->wait_event(ready_ev[static_cast<size_t>(d) * W + w]);
              e->import_device(dbuf[w], dcount[w]);
              e->record_event(done_ev[w]);
            });
            in += dcount[w];
            dcount[w] = 0;
          }
          {
            std::vector<uint8_t> host;
            {
              std::lock_guard<std::mutex> lk(stage_mu);
              host.swap(staging_host[w]);
            }
            if (!host.empty()) {
              guarded([&] { e->push_host(host.data(), host.size() / nb); });
              in += host.size() / nb;
            }
          }
          if (in) {
            r.received += in;
            ++r.transfers_in;
          }
          if (needy_w) {
            if (in)
              ++r.success_steals;
            else
              ++r.idle_rounds;
          }
        } else if (needy_w) {
          ++r.idle_rounds;
        }
      }
      if (plan.empty() && needy_w) ++r.idle_rounds;
      if (sizes[w] == 0) {
        r.t_idle += secs(t0, now());
        r.t_termination += secs(t1, now());
      }
      r.t_comm += secs(t1, now());
    }
    beat(w, Phase::Done);
    e->set_progress_hook(nullptr);
    guarded([&] { r.st = e->stats(); });
  };

  std::vector<std::thread> th;
  th.reserve(W);
  for (int w = 0; w < W; ++w) th.emplace_back(worker, w);
  for (auto& t : th) t.join();
  finished = true;
  if (watchdog.joinable()) watchdog.join();
  if (staging) {
    for (int x = 0; x < W; ++x) engines[x]->fence();  // imports may still read the staging buffers
    for (int x = 0; x < static_cast<int>(dbuf.size()); ++x)
      if (dbuf[x]) staging->release(engines[x]->device(), dbuf[x]);
    for (int x = 0; x < static_cast<int>(done_ev.size()); ++x)
      if (done_ev[x]) staging->free_event(engines[x]->device(), done_ev[x]);
    for (size_t i = 0; i < ready_ev.size(); ++i)
      if (ready_ev[i]) staging->free_event(engines[i / W]->device(), ready_ev[i]);
  }
  if (err) std::rethrow_exception(err);
  rep[0].watchdog_events = watchdog_events.load();
  best = gbest;
  for (auto& r : rep) best = std::min(best, r.st.best);
  return rep;
}

}  // namespace tts
