// pybind11 class for the engine contract (csrc/core/engine_api.hpp), shared by the
// CPU module (_tts_cpu) and the HIP module (_tts_hip). Nodes cross the boundary as
// uint8 arrays of shape (n, node_bytes) in the exact device layout.
#pragma once

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <memory>
#include <stdexcept>

#include "../core/engine_api.hpp"
#include "../core/runner.hpp"

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
      .def_property("best", &IEngine::best, &IEngine::set_best)
      .def("reset_counters", &IEngine::reset_counters)
      .def("stats", [](IEngine& e) { return engine_stats_dict(e.stats()); })
      .def("synchronize", &IEngine::synchronize, py::call_guard<py::gil_scoped_release>());
}

// run_workers(engines, initial_nodes, best, ...) -> {"best": int, "workers": [dict]}
inline void bind_runner(py::module_& m) {
  using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;
  m.def(
      "run_workers",
      [](py::list engines, py::list initial, int best, size_t m_, size_t steal_cap, double slice_min, double slice_max,
         bool ws) {
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
        std::vector<WorkerReport> rep;
        {
          py::gil_scoped_release nogil;
          rep = run_workers(es, init, best, cfg);
        }
        py::list ws_out;
        for (auto& r : rep) {
          py::dict d = engine_stats_dict(r.st);
          d["rounds"] = r.rounds;
          d["sent"] = r.sent;
          d["received"] = r.received;
          d["transfers_in"] = r.transfers_in;
          d["transfers_out"] = r.transfers_out;
          d["t_run_w"] = r.t_run;
          d["t_comm"] = r.t_comm;
          d["t_idle"] = r.t_idle;
          ws_out.append(d);
        }
        py::dict out;
        out["best"] = best;
        out["workers"] = ws_out;
        return out;
      },
      py::arg("engines"), py::arg("initial"), py::arg("best"), py::arg("m") = 25, py::arg("steal_cap") = 250000,
      py::arg("slice_min") = 0.0005, py::arg("slice_max") = 0.05, py::arg("ws") = true,
      "Drive several engines (GPUs and/or CPU workers) from one process until all pools are empty.");
}

}  // namespace tts
