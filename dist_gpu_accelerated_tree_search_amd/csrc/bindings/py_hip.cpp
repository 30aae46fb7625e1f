// _tts_hip: gfx950 device engines and kernels. Instances are passed as plain
// (jobs, machines, machine-major p) data so this module shares no C++ types with
// _tts_cpu (the two are built by different compilers).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <climits>
#include <string>

#include "../core/cpu_engine.hpp"
#include "../core/pfsp_front.hpp"
#include "../core/problems.hpp"
#include "../hip/host_support.hpp"
#include "../hip/pfsp_engine.hpp"
#include "../hip/queens_engine.hpp"
#include "engine_binding.hpp"

namespace py = pybind11;
using namespace tts;

namespace {

using U8 = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;

EngineConfig make_cfg(int device, size_t max_parents, size_t ring_bytes, int iters_small, int iters_large,
                      bool use_graphs, uintptr_t stream, int iters_first) {
  EngineConfig c;
  c.device = device;
  c.max_parents = max_parents;
  c.ring_bytes = ring_bytes;
  c.iters_small = iters_small;
  c.iters_large = iters_large;
  c.use_graphs = use_graphs;
  c.external_stream = stream;
  c.iters_first = iters_first;
  return c;
}

}  // namespace

PYBIND11_MODULE(_tts_hip, m) {
  m.doc() = "gfx950 (MI355X) device engines: device-resident pools, fused bound/prune/compact kernels, hipGraphs.";
  bind_engine(m);
  bind_shm_control(m);
  bind_dist_rounds(m, [](py::object model) -> WarmupFn {
    if (py::hasattr(model, "native")) {
      auto inst = std::make_shared<PfspInstance>(make_instance(model.attr("jobs").cast<int>(),
                                                               model.attr("machines").cast<int>(),
                                                               model.attr("native").attr("p").cast<std::vector<int>>()));
      const int lb = model.attr("host_lb").cast<int>();
      return with_pfsp_problem(*inst, lb, [&](auto prob) -> WarmupFn { return make_warmup(inst, prob); });
    }
    return make_warmup(nullptr, QueensProblem(model.attr("N").cast<int>(), model.attr("G").cast<int>()));
  });
  bind_runner(
      m, []() -> std::unique_ptr<DeviceStaging> { return std::make_unique<HipStaging>(); }, &device_cpus);
  if (!std::getenv("TTS_NO_ROCTX")) install_roctx_hooks();
  m.def("device_pci_bus_id", &device_pci_bus_id);
  m.def("device_cpus", &device_cpus, "CPUs of the NUMA node closest to the GPU (empty if unknown).");

  // CPU workers that can be mixed with GPU engines in run_workers (-C 1)
  m.def(
      "make_pfsp_cpu_engine",
      [](int jobs, int machines, std::vector<int> p, int lb, size_t batch, int threads) -> std::unique_ptr<IEngine> {
        auto inst = std::make_shared<PfspInstance>(make_instance(jobs, machines, std::move(p)));
        // LB1 is evaluated with the incremental LB1_d on the CPU (same values); the node
        // layout is the GPU engines' (front nodes where they apply)
        return with_pfsp_problem(*inst, lb == 1 ? 0 : lb, [&](auto prob) -> std::unique_ptr<IEngine> {
          return std::make_unique<OwningCpuEngine<decltype(prob)>>(inst, prob, batch, threads);
        });
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("batch") = 4096,
      py::arg("threads") = 1);
  m.def(
      "make_queens_cpu_engine",
      [](int N, int G, size_t batch, int threads) -> std::unique_ptr<IEngine> {
        return std::make_unique<CpuEngine<QueensProblem>>(QueensProblem(N, G), batch, threads);
      },
      py::arg("N"), py::arg("G") = 1, py::arg("batch") = 4096, py::arg("threads") = 1);

  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
  m.def("device_info", [](int device) {
    hipDeviceProp_t p;
    TTS_HIP_CHECK(hipGetDeviceProperties(&p, device));
    py::dict d;
    d["name"] = std::string(p.name);
    d["arch"] = std::string(p.gcnArchName);
    d["compute_units"] = p.multiProcessorCount;
    d["clock_khz"] = p.clockRate;
    d["total_mem"] = static_cast<size_t>(p.totalGlobalMem);
    d["lds_per_block"] = static_cast<size_t>(p.sharedMemPerBlock);
    d["warp_size"] = p.warpSize;
    return d;
  });

  m.def(
      "make_pfsp_engine",
      [](int jobs, int machines, std::vector<int> p, int lb, int device, size_t max_parents, size_t ring_bytes,
         int iters_small, int iters_large, bool use_graphs, uintptr_t stream, int taillard_id, int iters_first) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p), taillard_id);
        py::gil_scoped_release nogil;
        return make_pfsp_engine(in, lb,
                                make_cfg(device, max_parents, ring_bytes, iters_small, iters_large, use_graphs, stream,
                                         iters_first));
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("device") = 0,
      py::arg("max_parents") = size_t(1) << 18, py::arg("ring_bytes") = size_t(16) << 30, py::arg("iters_small") = 6,
      py::arg("iters_large") = 48, py::arg("use_graphs") = true, py::arg("stream") = 0, py::arg("taillard_id") = 0,
      py::arg("iters_first") = 18);

  m.def(
      "make_queens_engine",
      [](int N, int G, int device, size_t max_parents, size_t ring_bytes, int iters_small, int iters_large,
         bool use_graphs, uintptr_t stream, int iters_first) {
        py::gil_scoped_release nogil;
        return make_queens_engine(
            N, G, make_cfg(device, max_parents, ring_bytes, iters_small, iters_large, use_graphs, stream, iters_first));
      },
      py::arg("N"), py::arg("G") = 1, py::arg("device") = 0, py::arg("max_parents") = size_t(1) << 20,
      py::arg("ring_bytes") = size_t(16) << 30, py::arg("iters_small") = 6, py::arg("iters_large") = 48,
      py::arg("use_graphs") = true, py::arg("stream") = 0, py::arg("iters_first") = 24);

  m.def(
      "pfsp_bounds",
      [](int jobs, int machines, std::vector<int> p, int lb, U8 parents, int best, int device) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        const size_t nb = with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
        if (parents.ndim() != 2 || static_cast<size_t>(parents.shape(1)) != nb)
          throw std::invalid_argument("parents must be a (n, node_bytes) uint8 array");
        std::vector<int> out;
        {
          py::gil_scoped_release nogil;
          out = pfsp_gpu_bounds(in, lb, parents.data(), static_cast<size_t>(parents.shape(0)), best, device);
        }
        py::array_t<int> r(static_cast<py::ssize_t>(out.size()));
        std::memcpy(r.mutable_data(), out.data(), out.size() * sizeof(int));
        return r;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("parents"), py::arg("best") = INT_MAX,
      py::arg("device") = 0);

  m.def(
      "pfsp_expand_probe",
      [](int jobs, int machines, std::vector<int> p, int lb, U8 parents, int best, int device, int variant) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        const size_t nb = with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
        if (parents.ndim() != 2 || static_cast<size_t>(parents.shape(1)) != nb)
          throw std::invalid_argument("parents must be a (n, node_bytes) uint8 array");
        std::vector<int> out;
        {
          py::gil_scoped_release nogil;
          out = pfsp_expand_probe(in, lb, parents.data(), static_cast<size_t>(parents.shape(0)), best, device, variant);
        }
        py::array_t<int> r(static_cast<py::ssize_t>(out.size()));
        std::memcpy(r.mutable_data(), out.data(), out.size() * sizeof(int));
        return r;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("parents"), py::arg("best") = INT_MAX,
      py::arg("device") = 0, py::arg("variant") = 0,
      "One production expand iteration over these parents with the debug output on: every child's bound "
      "(exact LB2 below best, else >= best). variant 0 prefix/suffix, 1 rounds, 2 dense, 3 wave.");
  m.def(
      "pfsp_expand_time",
      [](int jobs, int machines, std::vector<int> p, int lb, U8 parents, int best, int device, int variant, int reps) {
        const PfspInstance in = make_instance(jobs, machines, std::move(p));
        const size_t nb = with_pfsp_bucket(jobs, [](auto nj) { return sizeof(PfspNode<decltype(nj)::value>); });
        if (parents.ndim() != 2 || static_cast<size_t>(parents.shape(1)) != nb)
          throw std::invalid_argument("parents must be a (n, node_bytes) uint8 array");
        std::vector<double> t;
        {
          py::gil_scoped_release nogil;
          (void)pfsp_expand_probe(in, lb, parents.data(), static_cast<size_t>(parents.shape(0)), best, device, variant,
                                  reps, &t);
        }
        py::dict d;
        d["ms_min"] = t[0];
        d["ms_median"] = t[1];
        d["clk_a"] = t[2];
        d["clk_b1"] = t[3];
        d["clk_b2"] = t[4];
        d["clk_c"] = t[5];
        d["chunks"] = t[6];
        d["clk_block_max"] = t[7];
        d["clk_block_mean"] = t[8];
        d["grid"] = t[9];
        const size_t nblk = (t.size() - 10) / 3;
        py::array_t<double> tl({static_cast<py::ssize_t>(nblk), static_cast<py::ssize_t>(3)});
        std::memcpy(tl.mutable_data(), t.data() + 10, nblk * 3 * sizeof(double));
        d["timeline_us"] = tl;
        return d;
      },
      py::arg("jobs"), py::arg("machines"), py::arg("p"), py::arg("lb"), py::arg("parents"), py::arg("best"),
      py::arg("device") = 0, py::arg("variant") = 1, py::arg("reps") = 10,
      "Time one expand iteration over this window (LB2): min/median ms over reps launches on the engine's grid, "
      "and per-chunk shader clocks of phases A, B1, B2, B3+C from one instrumented launch.");

  m.def(
      "queens_labels",
      [](int N, int G, U8 parents, int device) {
        if (parents.ndim() != 2 || parents.shape(1) != static_cast<py::ssize_t>(sizeof(QueensNode)))
          throw std::invalid_argument("parents must be a (n, 16) uint8 array");
        const size_t n = static_cast<size_t>(parents.shape(0));
        std::vector<uint8_t> out;
        {
          py::gil_scoped_release nogil;
          out = queens_gpu_labels(N, G, reinterpret_cast<const QueensNode*>(parents.data()), n, device);
        }
        U8 r({static_cast<py::ssize_t>(n), static_cast<py::ssize_t>(N)});
        std::memcpy(r.mutable_data(), out.data(), out.size());
        return r;
      },
      py::arg("N"), py::arg("G"), py::arg("parents"), py::arg("device") = 0);
}
