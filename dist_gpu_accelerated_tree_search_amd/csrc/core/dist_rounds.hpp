// Native round loop of the one-process-per-GPU runtime (parallel/runtime.py).
//
// Parity: ref pfsp/pfsp_dist_multigpu_cuda.c:364-469 (the comm thread: Allreduce
// MIN of the incumbent, globalTermination Allgather, needs_work Allgather,
// Allgatherv of donated nodes) and pfsp_multigpu_cuda.c:343-431 (random steal-half
// by idle threads, allIdle termination). Every rank runs:
//
//     search a time slice on the device (graph replays, no host round trips)
//       -> one all-gather of {pool size, incumbent, split pending}
//       -> incumbent = MIN, terminate when every pool is empty (exact: nothing is
//          in flight between rounds), otherwise a deterministic steal-half plan
//          computed identically on every rank, executed as targeted transfers
//          (TransferFn: RCCL send/recv on the engines' transfer streams).
//
// A slice ends early when a peer that ran dry asks for a round while some rank
// holds enough to donate (ShmControl board), so starving GPUs are fed after one
// graph replay, not after a whole slice. Thresholds are in units of the device
// parent window (a GPU with fewer parents than a fraction of its window is
// needy), not the reference's CPU-scale m = 25.
//
// Everything below runs without the GIL; the Python side is called only to move
// nodes (a transfer plan) and to write checkpoints.
#pragma once

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "engine_api.hpp"
#include "shm_control.hpp"
#include "trace.hpp"

namespace tts {

// Collective all-gather plus (optionally) the node-wide board of ShmControl.
class RoundControl {
 public:
  virtual ~RoundControl() = default;
  virtual int rank() const = 0;
  virtual int world() const = 0;
  // out[r*n+i] = value i of rank r; idle() is called now and then while waiting.
  virtual void allgather(const int64_t* v, int n, int64_t* out, const std::function<void()>& idle) = 0;
  virtual bool has_board() const { return false; }
  virtual void publish_size(int64_t) {}
  virtual int64_t peer_size(int) const { return 0; }
  virtual void request_next_round() {}
  virtual void request_current_round() {}
  virtual bool round_requested() const { return false; }
  // live incumbent between rounds (board only): start of a cooperative solve, and
  // offer `b` / get the best offered by any rank in this solve
  virtual void begin_solve() {}
  virtual int exchange_best(int b) { return b; }
};

class ShmRoundControl final : public RoundControl {
 public:
  ShmRoundControl(ShmControl* c, double timeout_s) : c_(c), timeout_(timeout_s) {
    if (!c_ || c_->tag() != ShmControl::layout_tag())
      throw std::invalid_argument("ShmRoundControl: not a ShmControl of this build layout");
  }
  int rank() const override { return c_->rank(); }
  int world() const override { return c_->world(); }
  void allgather(const int64_t* v, int n, int64_t* out, const std::function<void()>& idle) override {
    c_->allgather(v, n, out, timeout_, idle);
  }
  bool has_board() const override { return true; }
  void publish_size(int64_t n) override { c_->publish_size(n); }
  int64_t peer_size(int r) const override { return c_->peer_size(r); }
  void request_next_round() override { c_->request_round(c_->rounds() + 1); }
  void request_current_round() override { c_->request_round(c_->rounds()); }
  bool round_requested() const override { return c_->round_requested(); }
  void begin_solve() override { c_->begin_solve(); }
  int exchange_best(int b) override { return c_->exchange_best(b); }

 private:
  ShmControl* c_;
  double timeout_;
};

// Process-group all-gather supplied by the caller (multi-node jobs, TTS_SHM_CONTROL=0).
class FnRoundControl final : public RoundControl {
 public:
  using Fn = std::function<void(const int64_t*, int, int64_t*)>;
  FnRoundControl(int rank, int world, Fn fn) : rank_(rank), world_(world), fn_(std::move(fn)) {}
  int rank() const override { return rank_; }
  int world() const override { return world_; }
  void allgather(const int64_t* v, int n, int64_t* out, const std::function<void()>&) override { fn_(v, n, out); }

 private:
  int rank_, world_;
  Fn fn_;
};

struct Transfer {
  int donor, receiver;
  size_t n;
};
using Plan = std::vector<Transfer>;

// Deterministic steal-half matching, identical on every rank. Rank r is needy when
// its pool is below needy[r]; donors hold at least donor[r] and are not needy. Each
// needy rank (in rank order) is served by the donor with the most nodes left,
// which hands over half of them, capped at cap[r] of the receiver (ref 5*M for a
// GPU thief, 4*T for a CPU one: pfsp_multigpu_cuda.c:369-372). intra/inter
// restrict pairs to the same node (-w) or to different nodes (-L); node = rank /
// local_world.
// give (optional, per donor): what each rank can export without waiting (a rank with
// work in flight: DeviceEngine::size_exportable); a donor hands over at most that.
inline Plan plan_transfers(const std::vector<int64_t>& sizes, const std::vector<size_t>& needy_below,
                           const std::vector<size_t>& donor_min, const std::vector<size_t>& cap, int local_world = 0,
                           bool intra = true, bool inter = true, const std::vector<int64_t>* give = nullptr) {
  const int n = static_cast<int>(sizes.size());
  const int lw = local_world > 0 ? local_world : std::max(1, n);
  std::vector<int64_t> left = sizes;
  std::vector<int64_t> avail = give ? *give : sizes;
  std::vector<char> needy(n);
  for (int r = 0; r < n; ++r) needy[r] = sizes[r] < static_cast<int64_t>(needy_below[r]);
  Plan plan;
  for (int r = 0; r < n; ++r) {
    if (!needy[r]) continue;
    int d = -1;
    for (int x = 0; x < n; ++x) {
      if (x == r || needy[x] || left[x] < static_cast<int64_t>(donor_min[x]) || avail[x] <= 0) continue;
      const bool same = x / lw == r / lw;
      if (!((intra && same) || (inter && !same))) continue;
      if (d < 0 || left[x] > left[d]) d = x;
    }
    if (d < 0) continue;
    const size_t k = std::min({static_cast<size_t>(left[d] / 2), cap[r], static_cast<size_t>(std::max<int64_t>(0, avail[d]))});
    if (k == 0) continue;
    left[d] -= static_cast<int64_t>(k);
    avail[d] -= static_cast<int64_t>(k);
    left[r] += static_cast<int64_t>(k);
    plan.push_back({d, r, k});
  }
  return plan;
}
// Same thresholds for every rank.
inline Plan plan_transfers(const std::vector<int64_t>& sizes, size_t needy_below, size_t donor_min, size_t cap,
                           int local_world = 0, bool intra = true, bool inter = true) {
  const size_t n = sizes.size();
  return plan_transfers(sizes, std::vector<size_t>(n, needy_below), std::vector<size_t>(n, donor_min),
                        std::vector<size_t>(n, cap), local_world, intra, inter);
}

// One rank's part of a transfer plan as grouped point-to-point calls, in plan order:
// as a donor it sends consecutive slices of its exported block (one export of all its
// outgoing nodes), as a receiver it receives consecutive slices of its staging block.
// Every rank derives its calls from the same plan, so each send has its matching
// receive on the peer inside the same group (RCCL ncclGroupStart / ncclSend /
// ncclRecv / ncclGroupEnd, csrc/hip/rccl_transport.hpp; the reference's Allgatherv of
// every donor's nodes to every rank, pfsp_dist_multigpu_cuda.c:122-137, becomes
// targeted pairs only).
struct P2PCall {
  bool send;
  int peer;
  size_t offset, count;  // in nodes, within this rank's out (send) or in (recv) block
};
inline std::vector<P2PCall> p2p_calls(const Plan& plan, int rank, size_t* total_out = nullptr,
                                      size_t* total_in = nullptr) {
  std::vector<P2PCall> calls;
  size_t out = 0, in = 0;
  for (const auto& t : plan) {
    if (t.n == 0 || t.donor == t.receiver) continue;
    if (t.donor == rank) {
      calls.push_back({true, t.receiver, out, t.n});
      out += t.n;
    }
    if (t.receiver == rank) {
      calls.push_back({false, t.donor, in, t.n});
      in += t.n;
    }
  }
  if (total_out) *total_out = out;
  if (total_in) *total_in = in;
  return calls;
}

struct DistOptions {
  size_t needy_below = 25;   // a rank below this many nodes asks for work
  size_t donor_min = 50;     // a donor holds at least this many
  size_t steal_cap = 250000; // nodes per transfer (ref 5*M)
  double slice_min = 0.0005, slice_max = 0.050;  // adaptive local search between rounds
  bool intra = true, inter = true;                // ref -w / -L
  int local_world = 0;                            // ranks per node (0: all on one node)
  bool early_rounds = true;                       // board-driven early rounds (shm control only)
  long max_rounds = 0;                            // stop after this many rounds in total (0: never)
  double time_limit = 0;                          // stop at the first round after this many seconds
                                                  // on any rank (0: never; throughput time boxes)
  bool live_best = true;                          // exchange the incumbent after every replay (board)
  bool overlap = true;                            // rounds overlap a running replay (IEngine::set_overlap)
  bool trace_incumbent = false;                   // record this rank's incumbent timeline (diagnostics)
  long checkpoint_every = 0;                      // RoundHook every k rounds (0: never)
  double watchdog_s = 0;                          // report a phase longer than this
  bool watchdog_abort = false;
  unsigned fault_delay_us = 0;                    // random delay before each round
  unsigned fault_steal_fail_pct = 0;              // planned transfers dropped (same draw on every rank)
  unsigned long long fault_seed = 12345;
};

// Per-rank outcome; the *_all vectors hold every rank's value after the final
// all-gathers (identical on every rank).
struct DistOutcome {
  int best = 0x7fffffff;
  bool complete = true;
  unsigned long long rounds = 0;
  std::vector<unsigned long long> tree, sol, sent, received, transfers_in, transfers_out, steals, success_steals,
      idle_rounds, early_rounds, dropped, cpu_tree, cpu_sol;
  std::vector<double> t_run, t_comm, t_idle, t_termination, t_load_bal, t_memcpy, t_malloc;
  // rounds this rank spent with a replay in flight (the GPU searching during the round)
  std::vector<unsigned long long> overlapped_rounds;
  // trace_incumbent (this rank only): after every replay where the incumbent changed,
  // {seconds since the rounds began, explored tree so far (engine), own incumbent
  // before the exchange, incumbent after it}; the source of a change is the engine's
  // own leaves when the own value dropped, a peer when only the exchanged one did
  std::vector<std::array<double, 4>> incumbent_events;
  unsigned long long watchdog_events = 0;
};

// Moves the nodes of `plan` that concern this rank; returns (sent, received).
using TransferFn = std::function<std::pair<size_t, size_t>(const Plan&)>;
// Called at a round boundary (no node in flight) every checkpoint_every rounds once
// the split is done, and when max_rounds stops the solve, even while the pool is
// still replicated (then every rank holds the same pool): (round, global
// incumbent, replicated).
using RoundHook = std::function<void(unsigned long long, int, bool)>;

inline DistOutcome run_dist_rounds(IEngine& e, RoundControl& ctl, const DistOptions& o, const TransferFn& xfer,
                                   const RoundHook& hook, unsigned long long rounds0 = 0) {
  using clock = std::chrono::steady_clock;
  auto secs = [](clock::time_point a, clock::time_point b) { return std::chrono::duration<double>(b - a).count(); };
  const int world = ctl.world(), rank = ctl.rank();
  const bool share = (o.intra || o.inter) && world > 1;
  const bool board = share && o.early_rounds && ctl.has_board();
  DistOutcome out;
  unsigned long long rounds = rounds0, sent = 0, received = 0, tin = 0, tout = 0, steals = 0, ssteals = 0,
                     idle_rounds = 0, early = 0, dropped = 0;
  double t_run = 0, t_comm = 0, t_idle = 0, t_term = 0, t_lb = 0;
  double slice = o.slice_min;
  std::mt19937 jitter(static_cast<unsigned>(o.fault_seed * 7919ull + static_cast<unsigned long long>(rank)));

  // ---- watchdog: one heartbeat {phase, since} ----
  std::atomic<int> phase{0};  // 0 run, 1 round, 2 transfer, 3 done
  std::atomic<clock::rep> since{clock::now().time_since_epoch().count()};
  std::atomic<unsigned long long> wd_events{0}, wd_round{rounds0};
  std::atomic<long long> wd_pool{0};
  std::atomic<bool> finished{false};
  auto beat = [&](int p) {
    since.store(clock::now().time_since_epoch().count(), std::memory_order_relaxed);
    phase.store(p, std::memory_order_release);
  };
  std::thread dog;
  if (o.watchdog_s > 0) {
    dog = std::thread([&] {
      static const char* names[] = {"run", "round", "transfer", "done"};
      clock::rep reported = -1;
      while (!finished.load()) {
        std::this_thread::sleep_for(std::chrono::duration<double>(std::max(0.001, o.watchdog_s / 4)));
        const clock::rep s = since.load();
        const int p = phase.load();
        const double age = std::chrono::duration<double>(clock::duration(clock::now().time_since_epoch().count() - s)).count();
        if (p == 3 || age < o.watchdog_s || s == reported) continue;
        reported = s;
        ++wd_events;
        std::fprintf(stderr, "[tts watchdog] rank %d/%d stuck in phase '%s' for %.3f s (round %llu, pool %lld)\n", rank,
                     world, names[p], age, wd_round.load() + 1, wd_pool.load());
        std::fflush(stderr);
        if (o.watchdog_abort) std::abort();
      }
    });
  }
  struct Finish {
    std::atomic<bool>& f;
    std::thread& t;
    ~Finish() {
      f = true;
      if (t.joinable()) t.join();
    }
  } finish{finished, dog};

  // ---- board hook, after every graph replay: publish the live pool size, exchange
  // the incumbent with every rank (a better solution prunes everywhere at once, not
  // at the next round: ref checkBest, pfsp_multigpu_cuda.c:30-50,307-312), and leave
  // the slice on a peer's request ----
  ctl.begin_solve();
  const bool live_best = o.live_best && world > 1;
  const auto t_hook0 = clock::now();
  int last_seen = 0x7fffffff;
  e.set_progress_hook([&](size_t pool, int& best) {
    ctl.publish_size(static_cast<int64_t>(pool));
    const int own = best;
    if (live_best) best = std::min(best, ctl.exchange_best(best));
    if (o.trace_incumbent && best < last_seen) {
      out.incumbent_events.push_back({secs(t_hook0, clock::now()), static_cast<double>(e.tree_known()),
                                      static_cast<double>(own), static_cast<double>(best)});
      last_seen = best;
    }
    return board && ctl.round_requested();
  });
  struct Unhook {
    IEngine& e;
    ~Unhook() { e.set_progress_hook(nullptr); }
  } unhook{e};
  // Overlapped rounds: the slice may end with one replay still running, and the round
  // below (status all-gather, plan, transfers) runs while it does — the reference's
  // comm thread next to its GPU threads (pfsp_dist_multigpu_cuda.c:283,364-469). The
  // status uses the last completed replay's counts (a pool with a replay in flight
  // reports >= 1 node, so termination stays exact: it needs every pool empty with
  // nothing in flight); a lower incumbent is applied at the next replay.
  const bool overlap = o.overlap && share;
  e.set_overlap(overlap);
  struct NoOverlap {
    IEngine& e;
    bool on;
    ~NoOverlap() {
      if (on) e.set_overlap(false);
    }
  } no_overlap{e, overlap};
  unsigned long long overlapped = 0;
  // while some rank starves, slices end without a replay in flight: a donor mid-replay can
  // only export what the replay does not hold, and a skewed start then stayed unbalanced
  // (4 ranks, all work on one: per-rank trees max/mean 1.2-1.6 overlapped, 1.03 not;
  // profiles/r5/skew_overlap.txt); once every rank has work, rounds overlap again
  bool ov_now = overlap;

  // status record: pool size, incumbent, split pending, time up, exportable now
  constexpr int kRec = 5;
  std::vector<int64_t> st(static_cast<size_t>(world) * kRec), sizes(world), gives(world);
  const auto t_begin = clock::now();
  const int lw = o.local_world > 0 ? o.local_world : std::max(1, world);
  // ranks that may donate to this one (the pair filter of plan_transfers)
  auto eligible = [&](int q) {
    const bool same = q / lw == rank / lw;
    return q != rank && ((o.intra && same) || (o.inter && !same));
  };
  for (;;) {
    const auto t0 = clock::now();
    beat(0);
    {
      TTS_RANGE("tts.dist.run_slice");
      e.run(-1, slice, 1);
    }
    const auto t1 = clock::now();
    t_run += secs(t0, t1);
    beat(1);
    const bool flying = overlap && e.in_flight();
    overlapped += flying;
    const int64_t size = static_cast<int64_t>(flying ? e.size_known() : e.size());
    const int64_t give = flying ? static_cast<int64_t>(e.size_exportable()) : size;
    const int mybest = flying ? e.best_known() : e.best();
    const bool pend = flying ? e.split_pending_known() : e.split_pending();
    ctl.publish_size(size);
    wd_pool = size;
    wd_round = rounds;
    if (o.fault_delay_us) std::this_thread::sleep_for(std::chrono::microseconds(jitter() % (o.fault_delay_us + 1)));
    const bool needy = size < static_cast<int64_t>(o.needy_below);
    bool asked = false;
    // a dry rank calls the round early when a peer can donate (else it just waits)
    auto want_work = [&]() {
      if (!board || asked || !needy || pend) return false;
      for (int q = 0; q < world; ++q)
        if (eligible(q) && ctl.peer_size(q) >= static_cast<int64_t>(o.donor_min)) return true;
      return false;
    };
    if (want_work()) {
      ctl.request_next_round();
      asked = true;
      ++early;
    }
    const bool timeup = o.time_limit > 0 && secs(t_begin, clock::now()) >= o.time_limit;
    const int64_t mine[kRec] = {size, mybest, pend ? 1 : 0, timeup ? 1 : 0, give};
    {
      TTS_RANGE("tts.dist.round");
      ctl.allgather(mine, kRec, st.data(), [&] {
        if (want_work()) {
          ctl.request_current_round();
          asked = true;
          ++early;
        }
      });
    }
    ++rounds;
    const auto t2 = clock::now();
    bool replicated = false;
    int gbest = mybest;
    int64_t total = 0;
    bool starving = false, out_of_time = false;
    for (int r = 0; r < world; ++r) {
      sizes[r] = st[r * kRec];
      gbest = std::min<int>(gbest, static_cast<int>(st[r * kRec + 1]));
      replicated |= st[r * kRec + 2] != 0;
      out_of_time |= st[r * kRec + 3] != 0;
      gives[r] = st[r * kRec + 4];
      total += sizes[r];
      starving |= sizes[r] < static_cast<int64_t>(o.needy_below);
    }
    if (gbest < mybest) e.offer_best(gbest);
    if (size == 0) t_idle += secs(t0, t2);
    if (total == 0) {  // every pool is empty and nothing is in flight: exact termination
      t_term += secs(t1, clock::now());
      t_comm += secs(t1, clock::now());
      break;
    }
    if (out_of_time) {  // time box over on some rank: every rank stops at this round
      t_comm += secs(t1, clock::now());
      out.complete = false;
      break;
    }
    if (share && starving && !replicated) {
      const size_t nw = sizes.size();
      Plan plan = plan_transfers(sizes, std::vector<size_t>(nw, o.needy_below), std::vector<size_t>(nw, o.donor_min),
                                 std::vector<size_t>(nw, o.steal_cap), o.local_world, o.intra, o.inter, &gives);
      if (o.fault_steal_fail_pct && !plan.empty()) {
        std::mt19937_64 rng(o.fault_seed * 1000003ull + rounds);  // same draw on every rank
        Plan kept;
        for (const auto& t : plan) {
          if (rng() % 100 < o.fault_steal_fail_pct) {
            if (t.receiver == rank) ++dropped;
          } else {
            kept.push_back(t);
          }
        }
        plan.swap(kept);
      }
      if (needy) ++steals;
      size_t got = 0;
      if (!plan.empty()) {
        beat(2);
        const auto ta = clock::now();
        TTS_RANGE("tts.dist.transfer");
        const auto sr = xfer(plan);
        t_lb += secs(ta, clock::now());
        got = sr.second;
        sent += sr.first;
        received += sr.second;
        for (const auto& t : plan) {
          tout += t.donor == rank;
          tin += t.receiver == rank;
        }
      }
      if (needy) {
        if (got)
          ++ssteals;
        else
          ++idle_rounds;
      }
      slice = o.slice_min;
    } else {
      slice = std::min(o.slice_max, slice * 2);
    }
    if (overlap && (!starving || replicated) != ov_now) {
      ov_now = !ov_now;
      e.set_overlap(ov_now);
    }
    if (size == 0) t_term += secs(t1, clock::now());
    t_comm += secs(t1, clock::now());
    const bool stop = o.max_rounds > 0 && rounds >= static_cast<unsigned long long>(o.max_rounds);
    if (hook && (stop || (!replicated && o.checkpoint_every > 0 &&
                          rounds % static_cast<unsigned long long>(o.checkpoint_every) == 0)))
      hook(rounds, gbest, replicated);
    if (stop) {
      out.complete = false;
      break;
    }
  }
  beat(3);
  if (overlap) e.set_overlap(false);  // waits for a replay still in flight (a time box / max_rounds stop)

  // ---- final reductions: two all-gathers (counters, times) ----
  const EngineStats es = e.stats();
  constexpr int kIv = 15;  // ShmControl::kMaxVals
  const int64_t iv[kIv] = {static_cast<int64_t>(es.tree), static_cast<int64_t>(es.sol), static_cast<int64_t>(sent),
                           static_cast<int64_t>(received), static_cast<int64_t>(tin), static_cast<int64_t>(tout),
                           static_cast<int64_t>(steals), static_cast<int64_t>(ssteals),
                           static_cast<int64_t>(idle_rounds), static_cast<int64_t>(early),
                           static_cast<int64_t>(dropped), es.best, static_cast<int64_t>(wd_events.load()),
                           static_cast<int64_t>(es.cpu_tree), static_cast<int64_t>(es.cpu_sol)};
  std::vector<int64_t> ia(static_cast<size_t>(world) * kIv);
  ctl.allgather(iv, kIv, ia.data(), [] {});
  constexpr int kDv = 8;  // 7 timers + the overlapped-round count (exact as a double)
  double dv[kDv] = {t_run, t_comm, t_idle, t_term, t_lb, es.t_memcpy, es.t_malloc, static_cast<double>(overlapped)};
  int64_t dvi[kDv];
  std::memcpy(dvi, dv, sizeof(dv));
  std::vector<int64_t> da(static_cast<size_t>(world) * kDv);
  ctl.allgather(dvi, kDv, da.data(), [] {});
  out.rounds = rounds;
  out.best = 0x7fffffff;
  auto col = [&](int k) {
    std::vector<unsigned long long> v(world);
    for (int r = 0; r < world; ++r) v[r] = static_cast<unsigned long long>(ia[r * kIv + k]);
    return v;
  };
  out.tree = col(0);
  out.sol = col(1);
  out.sent = col(2);
  out.received = col(3);
  out.transfers_in = col(4);
  out.transfers_out = col(5);
  out.steals = col(6);
  out.success_steals = col(7);
  out.idle_rounds = col(8);
  out.early_rounds = col(9);
  out.dropped = col(10);
  out.cpu_tree = col(13);
  out.cpu_sol = col(14);
  for (int r = 0; r < world; ++r) {
    out.best = std::min<int>(out.best, static_cast<int>(ia[r * kIv + 11]));
    out.watchdog_events += static_cast<unsigned long long>(ia[r * kIv + 12]);
  }
  auto dcol = [&](int k) {
    std::vector<double> v(world);
    for (int r = 0; r < world; ++r) std::memcpy(&v[r], &da[r * kDv + k], sizeof(double));
    return v;
  };
  for (double x : dcol(7)) out.overlapped_rounds.push_back(static_cast<unsigned long long>(x));
  out.t_run = dcol(0);
  out.t_comm = dcol(1);
  out.t_idle = dcol(2);
  out.t_termination = dcol(3);
  out.t_load_bal = dcol(4);
  out.t_memcpy = dcol(5);
  out.t_malloc = dcol(6);
  return out;
}

}  // namespace tts
