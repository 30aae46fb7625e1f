// Native RCCL transport of the one-process-per-GPU runtime.
//
// Ref pfsp_dist_multigpu_cuda.c:122-137,364-469: the comm thread moves donated nodes
// with MPI_Allgather(sizes) + MPI_Allgatherv(nodes), every rank receiving every
// donor's block through host memory. Here one RCCL communicator per process (one GPU
// per rank, over xGMI) carries targeted donor -> receiver pairs only:
//   engine.export_device (pool bottom -> device staging, compute stream; the transfer
//   stream waits for it) -> ncclGroupStart, ncclSend / ncclRecv on the engine's
//   transfer stream, ncclGroupEnd -> engine.import_device (the compute stream waits for
//   the transfer stream, then appends) — stream-ordered, no host wait, no Python.
// The communicator is built from an ncclUniqueId that rank 0 creates and the caller
// distributes (parallel/comm.py: one broadcast over the process group). The library is
// the librccl.so.1 that torch has already loaded (same SONAME): one RCCL per process.
#pragma once

#include <rccl/rccl.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <functional>
#include <thread>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../core/dist_rounds.hpp"
#include "../core/engine_api.hpp"
#include "device_common.hpp"
#include "device_resource.hpp"

#define TTS_NCCL_CHECK(expr)                                                                               \
  do {                                                                                                     \
    ncclResult_t _r = (expr);                                                                              \
    if (_r != ncclSuccess)                                                                                 \
      throw std::runtime_error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + __FILE__ + ":" + \
                               std::to_string(__LINE__) + " in " #expr);                                   \
  } while (0)

namespace tts {

class RcclTransport final : public DeviceResource {
 public:
  static std::vector<uint8_t> new_id() {
    ncclUniqueId id;
    TTS_NCCL_CHECK(ncclGetUniqueId(&id));
    return std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&id), reinterpret_cast<uint8_t*>(&id) + sizeof(id));
  }

  RcclTransport(const std::vector<uint8_t>& id, int rank, int world, int device)
      : rank_(rank), world_(world), device_(device) {
    if (id.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("RcclTransport: bad unique id size");
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("RcclTransport: bad rank/world");
    ncclUniqueId uid;
    std::memcpy(&uid, id.data(), sizeof(uid));
    TTS_HIP_CHECK(hipSetDevice(device_));
    TTS_NCCL_CHECK(ncclCommInitRank(&comm_, world, uid, rank));
  }
  ~RcclTransport() override { release(); }
  void release() override {
    if (released_) return;
    released_ = true;
    (void)hipSetDevice(device_);
    for (int b = 0; b < 2; ++b)
      if (buf_[b]) {
        (void)hipDeviceSynchronize();
        (void)hipFree(buf_[b]);
        buf_[b] = nullptr;
      }
    if (dctl_) {
      (void)hipDeviceSynchronize();
      (void)hipFree(dctl_);
      dctl_ = nullptr;
    }
    if (hctl_) (void)hipHostFree(hctl_);
    hctl_ = nullptr;
    if (own_) (void)hipStreamDestroy(own_);
    own_ = nullptr;
    if (ev_) (void)hipEventDestroy(ev_);
    ev_ = nullptr;
    if (comm_) (void)ncclCommDestroy(comm_);
    comm_ = nullptr;
  }
  RcclTransport(const RcclTransport&) = delete;
  RcclTransport& operator=(const RcclTransport&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return device_; }
  unsigned long long transfers() const { return transfers_; }
  unsigned long long bytes_sent() const { return bytes_sent_; }
  unsigned long long bytes_recv() const { return bytes_recv_; }

  // The plan's transfers that concern this rank (every rank calls this with the same
  // plan, in the same round); returns (nodes sent, nodes received).
  std::pair<size_t, size_t> execute(const Plan& plan, IEngine& e) {
    if (released_) throw std::runtime_error("RCCL transport closed");
    size_t nout = 0, nin = 0;
    const std::vector<P2PCall> calls = p2p_calls(plan, rank_, &nout, &nin);
    if (calls.empty()) return {0, 0};
    if (e.device() != device_) throw std::invalid_argument("RcclTransport: engine on another device");
    TTS_HIP_CHECK(hipSetDevice(device_));
    const size_t nb = e.node_bytes();
    hipStream_t xs = reinterpret_cast<hipStream_t>(e.transfer_stream());
    if (!xs) throw std::invalid_argument("RcclTransport: engine has no transfer stream (GPU engines only)");
    uint8_t* out = static_cast<uint8_t*>(staging(0, nout * nb, xs));
    uint8_t* in = static_cast<uint8_t*>(staging(1, nin * nb, xs));
    if (nout) {
      const size_t got = e.export_device(out, nout);
      if (got != nout)
        throw std::runtime_error("rank " + std::to_string(rank_) + ": planned to send " + std::to_string(nout) +
                                 " nodes, the pool gave " + std::to_string(got));
    }
    TTS_NCCL_CHECK(ncclGroupStart());
    for (const P2PCall& c : calls) {
      if (c.send)
        TTS_NCCL_CHECK(ncclSend(out + c.offset * nb, c.count * nb, ncclUint8, c.peer, comm_, xs));
      else
        TTS_NCCL_CHECK(ncclRecv(in + c.offset * nb, c.count * nb, ncclUint8, c.peer, comm_, xs));
    }
    TTS_NCCL_CHECK(ncclGroupEnd());
    if (nin) e.import_device(in, nin);
    ++transfers_;
    bytes_sent_ += nout * nb;
    bytes_recv_ += nin * nb;
    return {nout, nin};
  }

  // Round status all-gather on the communicator (the control plane off the node-local
  // shm board: several nodes, or TTS_SHM_CONTROL=0; ref MPI_Allreduce / MPI_Allgather of
  // the comm thread, pfsp_dist_multigpu_cuda.c:69-88,372,385): this rank's n values go
  // to a device buffer, one in-place ncclAllGather runs on the engine's transfer stream
  // — after the previous round's send / recv there, so two collectives of this
  // communicator are never in flight at once — and the host waits for the gathered
  // (world, n) block to land in pinned memory. No Python, no second communicator.
  //
  // The wait is bounded by timeout_s (parallel/comm.py sets the job's): a dead or diverged
  // peer aborts the communicator (ncclCommAbort) and the call throws, so the round loop
  // fails instead of hanging every rank. `idle` runs while the collective is pending.
  void allgather_i64(const int64_t* v, int n, int64_t* out, IEngine& e,
                     const std::function<void()>& idle = std::function<void()>()) {
    if (released_) throw std::runtime_error("RCCL transport closed");
    if (n < 0 || n > kCtlVals) throw std::invalid_argument("RcclTransport::allgather_i64: at most 16 values");
    TTS_HIP_CHECK(hipSetDevice(device_));
    hipStream_t xs = reinterpret_cast<hipStream_t>(e.transfer_stream());
    if (!xs) xs = ctl_stream();
    if (!dctl_) {
      TTS_HIP_CHECK(hipMalloc(&dctl_, static_cast<size_t>(world_) * kCtlVals * sizeof(int64_t)));
      TTS_HIP_CHECK(hipHostMalloc(&hctl_, static_cast<size_t>(world_) * kCtlVals * sizeof(int64_t), hipHostMallocDefault));
    }
    if (n == 0) {
      wait_bounded(xs, idle);
      return;
    }
    std::memcpy(hctl_ + static_cast<size_t>(rank_) * n, v, sizeof(int64_t) * n);
    TTS_HIP_CHECK(hipMemcpyAsync(dctl_ + static_cast<size_t>(rank_) * n, hctl_ + static_cast<size_t>(rank_) * n,
                                 sizeof(int64_t) * n, hipMemcpyHostToDevice, xs));
    TTS_NCCL_CHECK(ncclAllGather(dctl_ + static_cast<size_t>(rank_) * n, dctl_, static_cast<size_t>(n), ncclInt64,
                                 comm_, xs));
    TTS_HIP_CHECK(hipMemcpyAsync(hctl_, dctl_, sizeof(int64_t) * n * world_, hipMemcpyDeviceToHost, xs));
    wait_bounded(xs, idle);
    std::memcpy(out, hctl_, sizeof(int64_t) * n * world_);
    ++collectives_;
  }
  unsigned long long collectives() const { return collectives_; }
  double timeout_s() const { return timeout_s_; }
  void set_timeout_s(double t) { timeout_s_ = t; }

  // World-1 check of the whole path on one GPU: n nodes go pool -> staging -> RCCL send
  // to self / receive from self -> staging -> pool. Returns the nodes moved.
  size_t self_loop(IEngine& e, size_t n) {
    TTS_HIP_CHECK(hipSetDevice(device_));
    const size_t nb = e.node_bytes();
    hipStream_t xs = reinterpret_cast<hipStream_t>(e.transfer_stream());
    if (!xs) throw std::invalid_argument("RcclTransport: GPU engines only");
    uint8_t* out = static_cast<uint8_t*>(staging(0, n * nb, xs));
    uint8_t* in = static_cast<uint8_t*>(staging(1, n * nb, xs));
    const size_t got = e.export_device(out, n);
    if (got == 0) return 0;
    TTS_NCCL_CHECK(ncclGroupStart());
    TTS_NCCL_CHECK(ncclSend(out, got * nb, ncclUint8, rank_, comm_, xs));
    TTS_NCCL_CHECK(ncclRecv(in, got * nb, ncclUint8, rank_, comm_, xs));
    TTS_NCCL_CHECK(ncclGroupEnd());
    e.import_device(in, got);
    return got;
  }

  // Every rank sends a rank-stamped pattern of `bytes` to every peer and checks what it
  // receives word by word (the node-transfer path, before any solve relies on it).
  // `corrupt` flips one received word (fault injection). Returns {peers, seconds}.
  std::pair<int, double> preflight(size_t bytes, bool corrupt = false) {
    TTS_HIP_CHECK(hipSetDevice(device_));
    const size_t words = std::max<size_t>(1, bytes / 4);
    std::vector<int> peers;
    for (int p = 0; p < world_; ++p)
      if (p != rank_) peers.push_back(p);
    if (peers.empty()) return {0, 0.0};
    hipStream_t s = nullptr;
    TTS_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t np = peers.size();
    std::vector<uint32_t> src(np * words), got(np * words, 0);
    auto pat = [](size_t i, int from, int to) {
      return static_cast<uint32_t>((i * 2654435761ull + static_cast<unsigned>(from) * 0x9E3779B1u +
                                    static_cast<unsigned>(to) * 0x85EBCA77u + 12345u) & 0x7fffffffu);
    };
    for (size_t k = 0; k < np; ++k)
      for (size_t i = 0; i < words; ++i) src[k * words + i] = pat(i, rank_, peers[k]);
    uint32_t *dsrc = nullptr, *ddst = nullptr;
    TTS_HIP_CHECK(hipMalloc(&dsrc, src.size() * 4));
    TTS_HIP_CHECK(hipMalloc(&ddst, got.size() * 4));
    TTS_HIP_CHECK(hipMemcpy(dsrc, src.data(), src.size() * 4, hipMemcpyHostToDevice));
    TTS_HIP_CHECK(hipMemset(ddst, 0, got.size() * 4));
    hipEvent_t e0, e1;
    TTS_HIP_CHECK(hipEventCreate(&e0));
    TTS_HIP_CHECK(hipEventCreate(&e1));
    TTS_HIP_CHECK(hipEventRecord(e0, s));
    std::string err;
    try {
      TTS_NCCL_CHECK(ncclGroupStart());
      for (size_t k = 0; k < np; ++k) {
        TTS_NCCL_CHECK(ncclSend(dsrc + k * words, words * 4, ncclUint8, peers[k], comm_, s));
        TTS_NCCL_CHECK(ncclRecv(ddst + k * words, words * 4, ncclUint8, peers[k], comm_, s));
      }
      TTS_NCCL_CHECK(ncclGroupEnd());
      TTS_HIP_CHECK(hipEventRecord(e1, s));
      TTS_HIP_CHECK(hipStreamSynchronize(s));
      TTS_HIP_CHECK(hipMemcpy(got.data(), ddst, got.size() * 4, hipMemcpyDeviceToHost));
    } catch (const std::exception& x) {
      err = x.what();
    }
    float ms = 0;
    if (err.empty()) (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(dsrc);
    (void)hipFree(ddst);
    (void)hipStreamDestroy(s);
    if (!err.empty())
      throw std::runtime_error("rank " + std::to_string(rank_) + ": RCCL point-to-point preflight failed (" +
                               std::to_string(np) + " peers): " + err);
    if (corrupt) got[0] ^= 1u;
    std::string bad;
    for (size_t k = 0; k < np; ++k)
      for (size_t i = 0; i < words; ++i)
        if (got[k * words + i] != pat(i, peers[k], rank_)) {
          bad += (bad.empty() ? "" : ",") + std::to_string(peers[k]);
          break;
        }
    if (!bad.empty())
      throw std::runtime_error("rank " + std::to_string(rank_) + ": RCCL preflight: data received from rank(s) " +
                               bad + " does not match what they sent; node transfers would corrupt the pools");
    return {static_cast<int>(np), ms * 1e-3};
  }

 private:
  // Wait for everything queued on xs, at most timeout_s: on expiry the communicator is
  // aborted (its pending operations end) and the call throws.
  void wait_bounded(hipStream_t xs, const std::function<void()>& idle) {
    if (!ev_) TTS_HIP_CHECK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
    TTS_HIP_CHECK(hipEventRecord(ev_, xs));
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 0;; ++spins) {
      const hipError_t q = hipEventQuery(ev_);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) TTS_HIP_CHECK(q);
      if (idle) idle();
      if ((spins & 255) == 255) {
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (timeout_s_ > 0 && dt > timeout_s_) {
          if (comm_) (void)ncclCommAbort(comm_);
          comm_ = nullptr;
          released_ = true;
          throw std::runtime_error("rank " + std::to_string(rank_) + ": RCCL round all-gather did not complete in " +
                                   std::to_string(timeout_s_) + " s (a peer died or left the round loop); "
                                   "communicator aborted");
        }
        std::this_thread::yield();
      }
    }
  }

  // Staging block `which` (0 out, 1 in) of at least `bytes`; a grown block replaces the
  // old one only after the transfer stream has drained (an RCCL op may still read it).
  void* staging(int which, size_t bytes, hipStream_t xs) {
    if (bytes == 0) return buf_[which];
    if (cap_[which] < bytes) {
      if (buf_[which]) {
        TTS_HIP_CHECK(hipStreamSynchronize(xs));
        TTS_HIP_CHECK(hipFree(buf_[which]));
        buf_[which] = nullptr;
      }
      size_t c = std::max<size_t>(size_t(64) << 20, cap_[which]);
      while (c < bytes) c *= 2;
      TTS_HIP_CHECK(hipMalloc(&buf_[which], c));
      cap_[which] = c;
    }
    return buf_[which];
  }

  hipStream_t ctl_stream() {
    if (!own_) TTS_HIP_CHECK(hipStreamCreateWithFlags(&own_, hipStreamNonBlocking));
    return own_;
  }
  static constexpr int kCtlVals = 16;
  int64_t* dctl_ = nullptr;   // (world, n) gathered status, device
  int64_t* hctl_ = nullptr;   // pinned host image
  hipStream_t own_ = nullptr;  // for engines without a transfer stream
  hipEvent_t ev_ = nullptr;    // completion of a bounded wait
  double timeout_s_ = 1800.0;
  unsigned long long collectives_ = 0;
  ncclComm_t comm_ = nullptr;
  bool released_ = false;
  int rank_, world_, device_;
  void* buf_[2] = {nullptr, nullptr};
  size_t cap_[2] = {0, 0};
  unsigned long long transfers_ = 0, bytes_sent_ = 0, bytes_recv_ = 0;
};

// The round loop's control plane over the RCCL communicator (no shm board): the status
// all-gather and the final reductions of run_dist_rounds are ncclAllGather calls.
class RcclRoundControl final : public RoundControl {
 public:
  RcclRoundControl(RcclTransport* t, IEngine* e) : t_(t), e_(e) {}
  int rank() const override { return t_->rank(); }
  int world() const override { return t_->world(); }
  void allgather(const int64_t* v, int n, int64_t* out, const std::function<void()>& idle) override {
    t_->allgather_i64(v, n, out, *e_, idle);
  }

 private:
  RcclTransport* t_;
  IEngine* e_;
};

}  // namespace tts
