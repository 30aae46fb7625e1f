// pybind11 class for the engine contract (csrc/core/engine_api.hpp), shared by the
// CPU module (_tts_cpu) and the HIP module (_tts_hip). Nodes cross the boundary as
// uint8 arrays of shape (n, node_bytes) in the exact device layout.
#pragma once

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <pybind11/functional.h>

#include <functional>
#include <memory>
#include <vector>
#include <stdexcept>

#include "../core/dist_rounds.hpp"
#include "../core/dist_session.hpp"
#include "../core/engine_api.hpp"
#include "../core/hybrid_engine.hpp"
#include "../core/multi_engine.hpp"
#include "../core/runner.hpp"
#include "../core/shm_control.hpp"

namespace py = pybind11;

namespace tts {

inline py::dict engine_stats_dict(const EngineStats& s) {
  py::dict d;
  d["tree"] = s.tree;
  d["sol"] = s.sol;
  d["parents"] = s.parents;
  d["iters"] = s.iters;
  d["best"] = s.best;
  d["launches"] = s.launches;
  d["syncs"] = s.syncs;
  d["spilled"] = s.spilled;
  d["refilled"] = s.refilled;
  d["t_run"] = s.t_run;
  d["t_memcpy"] = s.t_memcpy;
  d["t_malloc"] = s.t_malloc;
  d["device_nodes"] = s.device_nodes;
  d["host_nodes"] = s.host_nodes;
  d["capacity"] = s.capacity;
  d["exports"] = s.exports;
  d["left_inflight"] = s.left_inflight;
  d["overlapped_exports"] = s.overlapped_exports;
  d["imports"] = s.imports;
  d["pinned_bytes"] = s.pinned_bytes;
  d["cpu_tree"] = s.cpu_tree;
  d["cpu_sol"] = s.cpu_sol;
  return d;
}

inline void bind_engine(py::module_& m) {
  using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;
  py::class_<IEngine, std::unique_ptr<IEngine>>(m, "Engine", py::module_local())
      .def_property_readonly("node_bytes", &IEngine::node_bytes)
      .def_property_readonly("device", &IEngine::device)
      .def_property_readonly("stream", &IEngine::stream)
      .def(
          "push",
          [](IEngine& e, U8 a) {
            if (a.ndim() != 2 || static_cast<size_t>(a.shape(1)) != e.node_bytes())
              throw std::invalid_argument("nodes must be a (n, node_bytes) uint8 array");
            e.push_host(a.data(), static_cast<size_t>(a.shape(0)));
          },
          "Push nodes (top of the pool).")
      .def(
          "pop",
          [](IEngine& e, size_t max_n) {
            U8 out({static_cast<py::ssize_t>(max_n), static_cast<py::ssize_t>(e.node_bytes())});
            const size_t n = e.pop_host(out.mutable_data(), max_n);
            return py::array(out[py::slice(0, static_cast<py::ssize_t>(n), 1)]);
          },
          py::arg("max_n"), "Remove up to max_n nodes (oldest first) to a host array.")
      .def(
          "export_to",
          [](IEngine& e, uintptr_t ptr, size_t max_n) { return e.export_device(reinterpret_cast<void*>(ptr), max_n); },
          py::arg("ptr"), py::arg("max_n"), py::call_guard<py::gil_scoped_release>(),
          "Move up to max_n oldest nodes into device memory at ptr (same device); returns the count.")
      .def(
          "import_from",
          [](IEngine& e, uintptr_t ptr, size_t n) { e.import_device(reinterpret_cast<const void*>(ptr), n); },
          py::arg("ptr"), py::arg("n"), py::call_guard<py::gil_scoped_release>(),
          "Append n nodes read from device memory at ptr.")
      .def("size", &IEngine::size, py::call_guard<py::gil_scoped_release>())
      .def("warm_split", &IEngine::warm_split, py::arg("rank"), py::arg("world"), py::arg("window") = 4096,
           py::arg("passes") = 1, py::call_guard<py::gil_scoped_release>(),
           "Redundant deterministic warm-up (passes x 6 steps, parent window) then keep the i % world == rank "
           "share of the pool; warm-up counters stay on rank 0. Returns the kept pool size.")
      .def("run", &IEngine::run, py::arg("max_launches") = -1, py::arg("max_seconds") = 0.0,
           py::arg("stop_below") = 0, py::call_guard<py::gil_scoped_release>())
      .def(
          "solve",
          [](IEngine& e, U8 a, int best) {
            if (a.ndim() != 2 || static_cast<size_t>(a.shape(1)) != e.node_bytes())
              throw std::invalid_argument("nodes must be a (n, node_bytes) uint8 array");
            EngineStats st;
            {
              py::gil_scoped_release nogil;
              st = e.solve_from(a.data(), static_cast<size_t>(a.shape(0)), best);
            }
            return engine_stats_dict(st);
          },
          py::arg("nodes"), py::arg("best"), "Complete solve from these nodes (counters reset); returns stats.")
      .def(
          "begin",
          [](IEngine& e, U8 a, int best) {
            if (a.ndim() != 2 || static_cast<size_t>(a.shape(1)) != e.node_bytes())
              throw std::invalid_argument("nodes must be a (n, node_bytes) uint8 array");
            e.begin(a.data(), static_cast<size_t>(a.shape(0)), best);
          },
          py::arg("nodes"), py::arg("best"), "Fresh start from these nodes (counters reset), without running.")
      .def("set_split", &IEngine::set_split, py::arg("rank"), py::arg("world"), py::arg("min_parents"),
           "Arm the in-search rank split for the next begin() (see engine_api.hpp).")
      .def("split_pending", &IEngine::split_pending, py::call_guard<py::gil_scoped_release>())
      .def_property("best", &IEngine::best, &IEngine::set_best)
      .def("reset_counters", &IEngine::reset_counters)
      .def("stats", [](IEngine& e) { return engine_stats_dict(e.stats()); })
      .def("set_trace", &IEngine::set_trace, py::arg("on"))
      .def(
          "trace",
          [](IEngine& e) {
            std::vector<double> v;
            {
              py::gil_scoped_release nogil;
              v = e.trace();
            }
            py::array_t<double> a({static_cast<py::ssize_t>(v.size() / 3), static_cast<py::ssize_t>(3)});
            std::copy(v.begin(), v.end(), a.mutable_data());
            return a;
          },
          "(n, 3) array of {kind, start ms, end ms}: 0 graph replay, 1 spill D2H, 2 refill H2D")
      .def("synchronize", &IEngine::synchronize, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("transfer_stream", &IEngine::transfer_stream,
                             "Stream on which work-sharing sends/receives are enqueued (0: host engine).")
      .def("fence", &IEngine::fence, py::call_guard<py::gil_scoped_release>(),
           "Wait on the host for every copy enqueued so far.")
      .def("pool_weight", &IEngine::pool_weight, py::arg("w"), py::call_guard<py::gil_scoped_release>(),
           "Sum over the pool of w[depth] (progress measure, see search.progress_weights).");
  m.def(
      "make_hybrid_engine",
      [](py::object gpu, py::object cpu, size_t m_, size_t cpu_cap) -> std::unique_ptr<IEngine> {
        HybridConfig c;
        c.m = std::max<size_t>(1, m_);
        c.cpu_cap = std::max<size_t>(1, cpu_cap);
        return std::make_unique<HybridEngine>(gpu.cast<IEngine*>(), cpu.cast<IEngine*>(), c);
      },
      py::arg("gpu"), py::arg("cpu"), py::arg("m") = 25, py::arg("cpu_cap") = 20000, py::keep_alive<0, 1>(),
      py::keep_alive<0, 2>(),
      "One rank's engine: `gpu` on the calling thread plus the CPU worker `cpu` on its own thread, sharing work "
      "and the incumbent (core/hybrid_engine.hpp; ref -C 1 in the distributed driver).");
}

// Intra-node control plane (csrc/core/shm_control.hpp), bound in both modules so the
// native round loop of either one can use it (dist_rounds takes its address).
inline void bind_shm_control(py::module_& m) {
  using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
  py::class_<ShmControl>(m, "ShmControl", py::module_local())
      .def(py::init<const std::string&, int, int, bool>(), py::arg("name"), py::arg("rank"), py::arg("world"),
           py::arg("create"))
      .def_property_readonly("rank", &ShmControl::rank)
      .def_property_readonly("world", &ShmControl::world)
      .def_property_readonly("rounds", &ShmControl::rounds)
      .def_property_readonly("address", &ShmControl::address)
      .def("unlink", &ShmControl::unlink)
      .def(
          "allgather",
          [](ShmControl& c, I64 vals, double timeout_s) {
            if (vals.ndim() != 1) throw std::invalid_argument("allgather: 1-D int64 values");
            const int n = static_cast<int>(vals.shape(0));
            I64 out({static_cast<py::ssize_t>(c.world()), static_cast<py::ssize_t>(n)});
            const int64_t* src = vals.data();
            int64_t* dst = out.mutable_data();
            {
              py::gil_scoped_release nogil;
              c.allgather(src, n, dst, timeout_s);
            }
            return out;
          },
          py::arg("values"), py::arg("timeout_s") = 600.0,
          "Collective all-gather of up to 15 int64 per rank -> (world, n) array.")
      .def(
          "barrier",
          [](ShmControl& c, double timeout_s) {
            py::gil_scoped_release nogil;
            c.barrier(timeout_s);
          },
          py::arg("timeout_s") = 600.0)
      .def("offer_best", &ShmControl::offer_best, py::arg("best"))
      .def_property_readonly("best", &ShmControl::best)
      .def("publish_size", &ShmControl::publish_size)
      .def("peer_size", &ShmControl::peer_size)
      .def("request_round", &ShmControl::request_round)
      .def_property_readonly("round_requested", &ShmControl::round_requested);
}

// ---- native rounds: options, control plane and callbacks from Python ----
inline DistOptions dist_options_from(const py::dict& o) {
  DistOptions opt;
  auto get = [&](const char* k, auto& v) {
    if (o.contains(k)) v = o[k].cast<std::remove_reference_t<decltype(v)>>();
  };
  get("needy_below", opt.needy_below);
  get("donor_min", opt.donor_min);
  get("steal_cap", opt.steal_cap);
  get("slice_min", opt.slice_min);
  get("slice_max", opt.slice_max);
  get("intra", opt.intra);
  get("inter", opt.inter);
  get("local_world", opt.local_world);
  get("early_rounds", opt.early_rounds);
  get("max_rounds", opt.max_rounds);
  get("time_limit", opt.time_limit);
  get("live_best", opt.live_best);
  get("overlap", opt.overlap);
  get("trace_incumbent", opt.trace_incumbent);
  get("checkpoint_every", opt.checkpoint_every);
  get("watchdog_s", opt.watchdog_s);
  get("watchdog_abort", opt.watchdog_abort);
  get("fault_delay_us", opt.fault_delay_us);
  get("fault_steal_fail_pct", opt.fault_steal_fail_pct);
  get("fault_seed", opt.fault_seed);
  return opt;
}

// A native control plane object (HIP module: RcclTransport) in place of a Python
// all-gather callable: returns null when `obj` is not one.
using NativeControl = std::function<std::unique_ptr<RoundControl>(py::object obj, IEngine* e)>;

inline std::unique_ptr<RoundControl> round_control_from(uintptr_t shm_address, py::object allgather_fn, int rank,
                                                        int world, double timeout_s, const NativeControl& native = {},
                                                        IEngine* e = nullptr) {
  using I64 = py::array_t<int64_t, py::array::c_style | py::array::forcecast>;
  std::unique_ptr<RoundControl> ctl;
  if (!shm_address && native && !allgather_fn.is_none()) ctl = native(allgather_fn, e);
  if (ctl) {
  } else if (shm_address) {
    ctl = std::make_unique<ShmRoundControl>(reinterpret_cast<ShmControl*>(shm_address), timeout_s);
  } else {
    if (allgather_fn.is_none()) throw std::invalid_argument("give a shm address or an allgather_fn");
    ctl = std::make_unique<FnRoundControl>(rank, world, [allgather_fn, world](const int64_t* v, int n, int64_t* out) {
      py::gil_scoped_acquire gil;
      I64 a(static_cast<py::ssize_t>(n));
      std::memcpy(a.mutable_data(), v, sizeof(int64_t) * static_cast<size_t>(n));
      I64 r = allgather_fn(a).cast<I64>();
      if (r.size() != static_cast<py::ssize_t>(world) * n) throw std::runtime_error("allgather_fn: wrong shape");
      std::memcpy(out, r.data(), sizeof(int64_t) * static_cast<size_t>(world) * static_cast<size_t>(n));
    });
  }
  if (ctl->rank() != rank || ctl->world() != world) throw std::invalid_argument("rank/world mismatch");
  return ctl;
}

inline TransferFn transfer_from(py::object transfer_fn) {
  return [transfer_fn](const Plan& p) -> std::pair<size_t, size_t> {
    py::gil_scoped_acquire gil;
    py::list l;
    for (const auto& t : p) l.append(py::make_tuple(t.donor, t.receiver, t.n));
    py::tuple r = transfer_fn(l).cast<py::tuple>();
    return {r[0].cast<size_t>(), r[1].cast<size_t>()};
  };
}

inline RoundHook hook_from(py::object round_hook) {
  RoundHook hook;
  if (!round_hook.is_none())
    hook = [round_hook](unsigned long long r, int b, bool rep) {
      py::gil_scoped_acquire gil;
      round_hook(r, b, rep);
    };
  return hook;
}

// per-rank table as two arrays (one row per rank): cheap to hand to Python
inline py::dict outcome_dict(const DistOutcome& out) {
  const py::ssize_t W = static_cast<py::ssize_t>(out.tree.size());
  py::array_t<int64_t> iv({W, static_cast<py::ssize_t>(13)});
  py::array_t<double> fv({W, static_cast<py::ssize_t>(7)});
  auto I = iv.mutable_unchecked<2>();
  auto F = fv.mutable_unchecked<2>();
  for (py::ssize_t r = 0; r < W; ++r) {
    auto at = [&](const std::vector<unsigned long long>& v) { return r < static_cast<py::ssize_t>(v.size()) ? v[r] : 0ull; };
    const unsigned long long cols[13] = {out.tree[r], out.sol[r], out.sent[r], out.received[r], out.transfers_in[r],
                                         out.transfers_out[r], out.steals[r], out.success_steals[r],
                                         out.idle_rounds[r], out.early_rounds[r], out.dropped[r], at(out.cpu_tree),
                                         at(out.cpu_sol)};
    for (int k = 0; k < 13; ++k) I(r, k) = static_cast<int64_t>(cols[k]);
    const double dc[7] = {out.t_run[r], out.t_comm[r], out.t_idle[r], out.t_termination[r], out.t_load_bal[r],
                          out.t_memcpy[r], out.t_malloc[r]};
    for (int k = 0; k < 7; ++k) F(r, k) = dc[k];
  }
  py::dict d;
  d["best"] = out.best;
  d["complete"] = out.complete;
  d["rounds"] = out.rounds;
  d["watchdog_events"] = out.watchdog_events;
  d["counts"] = iv;  // tree sol sent received transfers_in transfers_out steals success_steals idle_rounds
                     // early_rounds dropped cpu_tree cpu_sol (CPU-worker share of a hybrid rank)
  d["times"] = fv;   // t_run t_comm t_idle t_termination t_load_bal t_memcpy t_malloc
  d["overlapped_rounds"] = out.overlapped_rounds;  // rounds with a replay in flight, per rank
  py::list ev;  // this rank's incumbent timeline (trace_incumbent)
  for (const auto& x : out.incumbent_events) ev.append(py::make_tuple(x[0], x[1], x[2], x[3]));
  d["incumbent_events"] = ev;
  return d;
}

// Builds the Step-1 warm-up of a Python model (PfspModel / QueensModel) in this module.
using WarmupFactory = std::function<WarmupFn(py::object model)>;

struct PyDistSession {
  py::object engine_ref;  // keeps the engine alive
  IEngine* e = nullptr;
  std::unique_ptr<RoundControl> ctl;
  DistOptions opt;
  WarmupFn warm;
  TransferFn xfer;
  RoundHook hook;
  size_t warm_target = 25, split_min = 1;
  bool split = true;
  DistSolveResult last;
};

// dist_rounds(engine, shm_address | allgather_fn, rank, world, options, transfer_fn,
//             round_hook, rounds0, timeout_s) -> dict (core/dist_rounds.hpp)
// DistSession(engine, model, ...).solve(best) -> one native cooperative solve (core/dist_session.hpp)
// A native transport object (HIP module: RcclTransport) in place of a Python
// transfer callable: returns an empty TransferFn when `obj` is not one.
using NativeTransfer = std::function<TransferFn(py::object obj, IEngine* e)>;

inline TransferFn resolve_transfer(const NativeTransfer& native, py::object obj, IEngine* e) {
  if (native) {
    TransferFn f = native(obj, e);
    if (f) return f;
  }
  return transfer_from(obj);
}

inline void bind_dist_rounds(py::module_& m, WarmupFactory warmup_factory, NativeTransfer native = {},
                             NativeControl native_ctl = {}) {
  m.def(
      "p2p_calls",
      [](py::list plan, int rank) {
        Plan pl;
        for (auto t : plan) {
          auto x = t.cast<py::tuple>();
          pl.push_back({x[0].cast<int>(), x[1].cast<int>(), x[2].cast<size_t>()});
        }
        py::list out;
        for (const auto& c : p2p_calls(pl, rank))
          out.append(py::make_tuple(c.send ? "send" : "recv", c.peer, c.offset, c.count));
        return out;
      },
      py::arg("plan"), py::arg("rank"),
      "This rank's grouped point-to-point calls for a transfer plan (csrc/core/dist_rounds.hpp p2p_calls).");
  m.def(
      "plan_transfers",
      [](std::vector<int64_t> sizes, size_t needy_below, size_t donor_min, size_t cap, int local_world, bool intra,
         bool inter, std::vector<int64_t> give) {
        py::list out;
        const size_t n = sizes.size();
        if (!give.empty() && give.size() != n) throw std::invalid_argument("give: one value per rank");
        for (const auto& t : plan_transfers(sizes, std::vector<size_t>(n, needy_below), std::vector<size_t>(n, donor_min),
                                            std::vector<size_t>(n, cap), local_world, intra, inter,
                                            give.empty() ? nullptr : &give))
          out.append(py::make_tuple(t.donor, t.receiver, t.n));
        return out;
      },
      py::arg("sizes"), py::arg("needy_below"), py::arg("donor_min"), py::arg("cap"), py::arg("local_world") = 0,
      py::arg("intra") = true, py::arg("inter") = true, py::arg("give") = std::vector<int64_t>{},
      "give: what each rank can export right now (a rank with a replay in flight); donors hand over at most that.");
  m.def(
      "dist_rounds",
      [native, native_ctl](IEngine& e, uintptr_t shm_address, py::object allgather_fn, int rank, int world, py::dict o,
         py::object transfer_fn, py::object round_hook, unsigned long long rounds0, double timeout_s) {
        const DistOptions opt = dist_options_from(o);
        auto ctl = round_control_from(shm_address, allgather_fn, rank, world, timeout_s, native_ctl, &e);
        const TransferFn xfer = resolve_transfer(native, transfer_fn, &e);
        const RoundHook hook = hook_from(round_hook);
        DistOutcome out;
        {
          py::gil_scoped_release nogil;
          out = run_dist_rounds(e, *ctl, opt, xfer, hook, rounds0);
        }
        return outcome_dict(out);
      },
      py::arg("engine"), py::arg("shm_address"), py::arg("allgather_fn"), py::arg("rank"), py::arg("world"),
      py::arg("options"), py::arg("transfer_fn"), py::arg("round_hook") = py::none(), py::arg("rounds0") = 0,
      py::arg("timeout_s") = 1800.0,
      "Native lock-step rounds of a multi-rank solve until every pool is empty (or max_rounds).");
  py::class_<PyDistSession>(m, "DistSession", py::module_local())
      .def(py::init([warmup_factory, native, native_ctl](py::object engine, py::object model, uintptr_t shm_address, py::object allgather_fn,
                                     int rank, int world, py::dict o, py::object transfer_fn, py::object round_hook,
                                     size_t warm_target, size_t split_min, double timeout_s, bool split) {
             auto s = std::make_unique<PyDistSession>();
             s->split = split;
             s->engine_ref = engine;
             s->e = engine.cast<IEngine*>();
             s->ctl = round_control_from(shm_address, allgather_fn, rank, world, timeout_s, native_ctl, s->e);
             s->opt = dist_options_from(o);
             s->warm = warmup_factory(model);
             s->xfer = resolve_transfer(native, transfer_fn, s->e);
             s->hook = hook_from(round_hook);
             s->warm_target = warm_target;
             s->split_min = split_min;
             return s;
           }),
           py::arg("engine"), py::arg("model"), py::arg("shm_address"), py::arg("allgather_fn"), py::arg("rank"),
           py::arg("world"), py::arg("options"), py::arg("transfer_fn"), py::arg("round_hook") = py::none(),
           py::arg("warm_target") = 25, py::arg("split_min") = 1, py::arg("timeout_s") = 1800.0,
           py::arg("split") = true)
      .def(
          "solve",
          [](PyDistSession& s, int best) {
            {
              py::gil_scoped_release nogil;
              s.last = dist_solve_split(*s.e, *s.ctl, s.opt, s.warm, best, s.warm_target, s.split_min, s.xfer, s.hook,
                                        s.split);
            }
            const auto& r = s.last;
            return py::make_tuple(r.best, r.tree, r.sol, r.rounds, r.complete, r.t_init, r.t_search, r.elapsed);
          },
          py::arg("best"),
          "One cooperative solve: (best, tree, sol, rounds, complete, t_init, t_search, elapsed), global values.")
      .def("outcome", [](const PyDistSession& s) { return outcome_dict(s.last.outcome); },
           "Per-rank counters and timers of the last solve (same layout as dist_rounds).");
}

// run_workers(engines, initial_nodes, best, ...) -> {"best": int, "workers": [dict]}
// `staging` (HIP module only) enables device-to-device steals between GPU engines;
// `cpus_of_device` maps a GPU to its NUMA-local CPUs for thread pinning.
using StagingFactory = std::function<std::unique_ptr<DeviceStaging>()>;
using CpusOfDevice = std::function<std::vector<int>(int)>;

inline void bind_runner(py::module_& m, StagingFactory staging = {}, CpusOfDevice cpus_of_device = {}) {
  using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;
  m.def(
      "run_workers",
      [staging, cpus_of_device](py::list engines, py::list initial, int best, size_t m_, size_t steal_cap,
                                double slice_min, double slice_max, bool ws, bool pin, bool device_steals,
                                double watchdog_s, py::dict faults, std::vector<size_t> needy_below,
                                std::vector<size_t> donor_min, std::vector<size_t> recv_cap) {
        if (engines.size() != initial.size()) throw std::invalid_argument("one initial node array per engine");
        std::vector<IEngine*> es;
        std::vector<std::vector<uint8_t>> init;
        for (size_t i = 0; i < engines.size(); ++i) {
          IEngine* e = engines[i].cast<IEngine*>();
          U8 a = initial[i].cast<U8>();
          if (a.ndim() != 2 || static_cast<size_t>(a.shape(1)) != e->node_bytes())
            throw std::invalid_argument("initial nodes must be (n, node_bytes) uint8 arrays");
          es.push_back(e);
          init.emplace_back(a.data(), a.data() + a.size());
        }
        RunnerConfig cfg;
        cfg.m = m_;
        cfg.steal_cap = steal_cap;
        cfg.slice_min = slice_min;
        cfg.slice_max = slice_max;
        cfg.work_sharing = ws;
        cfg.watchdog_s = watchdog_s;
        cfg.needy_below = std::move(needy_below);
        cfg.donor_min = std::move(donor_min);
        cfg.recv_cap = std::move(recv_cap);
        cfg.merge_env();
        if (faults.contains("delay_us")) cfg.fault_delay_us = faults["delay_us"].cast<unsigned>();
        if (faults.contains("steal_fail_pct")) cfg.fault_steal_fail_pct = faults["steal_fail_pct"].cast<unsigned>();
        if (faults.contains("stall_worker")) cfg.fault_stall_worker = faults["stall_worker"].cast<int>();
        if (faults.contains("stall_s")) cfg.fault_stall_s = faults["stall_s"].cast<double>();
        if (faults.contains("seed")) cfg.fault_seed = faults["seed"].cast<unsigned long long>();
        if (pin && cpus_of_device)
          for (auto* e : es) cfg.worker_cpus.push_back(e->device() >= 0 ? cpus_of_device(e->device()) : std::vector<int>{});
        std::unique_ptr<DeviceStaging> st;
        if (device_steals && staging) st = staging();
        std::vector<WorkerReport> rep;
        {
          py::gil_scoped_release nogil;
          rep = run_workers(es, init, best, cfg, st.get());
        }
        py::list ws_out;
        for (auto& r : rep) {
          py::dict d = engine_stats_dict(r.st);
          d["rounds"] = r.rounds;
          d["sent"] = r.sent;
          d["received"] = r.received;
          d["transfers_in"] = r.transfers_in;
          d["transfers_out"] = r.transfers_out;
          d["device_transfers"] = r.device_transfers;
          d["dropped_transfers"] = r.dropped_transfers;
          d["watchdog_events"] = r.watchdog_events;
          d["pinned"] = r.pinned;
          d["t_run_w"] = r.t_run;
          d["t_comm"] = r.t_comm;
          d["t_idle"] = r.t_idle;
          d["t_termination"] = r.t_termination;
          d["steals"] = r.steals;
          d["success_steals"] = r.success_steals;
          d["idle_rounds"] = r.idle_rounds;
          d["early_rounds"] = r.early_rounds;
          ws_out.append(d);
        }
        py::dict out;
        out["best"] = best;
        out["workers"] = ws_out;
        return out;
      },
      py::arg("engines"), py::arg("initial"), py::arg("best"), py::arg("m") = 25, py::arg("steal_cap") = 250000,
      py::arg("slice_min") = 0.0005, py::arg("slice_max") = 0.05, py::arg("ws") = true, py::arg("pin") = false,
      py::arg("device_steals") = true, py::arg("watchdog_s") = 0.0, py::arg("faults") = py::dict(),
      py::arg("needy_below") = std::vector<size_t>{}, py::arg("donor_min") = std::vector<size_t>{},
      py::arg("recv_cap") = std::vector<size_t>{},
      "Drive several engines (GPUs and/or CPU workers) from one process until all pools are empty.");
  m.def(
      "make_multi_engine",
      [staging](py::list engines, size_t needy_below, size_t donor_min, size_t cap,
                size_t split_min) -> std::unique_ptr<IEngine> {
        std::vector<IEngine*> es;
        for (auto e : engines) es.push_back(e.cast<IEngine*>());
        MultiConfig c;
        c.needy_below = std::max<size_t>(1, needy_below);
        c.donor_min = std::max<size_t>(2, donor_min);
        c.cap = std::max<size_t>(1, cap);
        c.split_min = split_min;
        const bool dev = !es.empty() && es[0]->device() >= 0;
        return std::make_unique<MultiEngine>(std::move(es), dev && staging ? staging() : nullptr, c);
      },
      py::arg("engines"), py::arg("needy_below"), py::arg("donor_min"), py::arg("cap") = size_t(1) << 22,
      py::arg("split_min") = size_t(0), py::keep_alive<0, 1>(),
      "Several engines on one device (one stream and one host thread each) as one engine: concurrent "
      "slices, same-device steal-half between slices (core/multi_engine.hpp).");
  m.def("parse_cpulist", &parse_cpulist);
  m.def("allowed_cpus", &allowed_cpus);
}

}  // namespace tts
