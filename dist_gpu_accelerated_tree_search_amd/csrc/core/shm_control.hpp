// Intra-node control plane for the one-process-per-GPU runtime: the small status
// exchanges of every round (pool size, incumbent, termination, final counters)
// go through a POSIX shared-memory segment instead of RCCL collectives.
//
// Why: a round's record is a few int64 per rank. Over RCCL each exchange is a
// host->device copy, a collective kernel and a device->host copy with a stream
// sync (tens of microseconds); ta014 LB1 solves in ~0.4 ms on one MI355X, so
// two such collectives per solve would eat most of the gain of a second GPU.
// Through shared memory an all-gather is one cache-line store per rank and a
// spin on the others' lines (~1 us). Node payloads still move GPU -> GPU over
// xGMI (RCCL send/recv, parallel/comm.py).
//
// Parity: the reference's intra-node coordination is also shared memory — C11
// atomics and spin locks between OpenMP threads (ref pfsp_multigpu_cuda.c:30-50
// checkBest, common/util.c:4-38 allIdle); its inter-node rounds are MPI
// Allreduce/Allgather (ref pfsp_dist_multigpu_cuda.c:364-469). Here processes
// replace threads, the segment replaces the shared address space, and the
// all-gather has collective semantics (every rank calls it in the same order).
//
// Protocol: slot[parity][rank] = {seq, values}. Round r writes parity r&1, then
// publishes seq = r (release) and waits until every rank's seq reaches r
// (acquire). A rank can only write parity r&1 again at round r+2, which needs
// every rank to have posted round r+1, i.e. to have finished reading round r —
// so two buffers are enough and no reset is ever needed. A rank that does not
// arrive within the timeout raises (failure detection).
//
// Board (not collective): every rank publishes its live pool size after each
// graph replay, and a rank that ran dry while a peer holds enough work to donate
// requests the next round early (request_round). Ranks still searching see the
// request between two replays and join the round at once instead of finishing
// their time slice — the counterpart of the reference's immediate steal attempt
// by an idle thread (ref pfsp_multigpu_cuda.c:343-404).
#pragma once

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace tts {

class ShmControl {
 public:
  static constexpr int kMaxVals = 15;
  static constexpr uint64_t kMagic = 0x7474735f63746c32ull;  // "tts_ctl2"

  // create=true: make (or replace) the segment `name` (rank 0); otherwise open it.
  ShmControl(const std::string& name, int rank, int world, bool create) : name_(name), rank_(rank), world_(world) {
    if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("ShmControl: bad rank/world");
    if (name.empty() || name[0] != '/') throw std::invalid_argument("ShmControl: name must start with '/'");
    bytes_ = sizeof(Header) + static_cast<size_t>(world) * sizeof(Board) + 2 * static_cast<size_t>(world) * sizeof(Slot);
    int fd = -1;
    if (create) {
      (void)shm_unlink(name.c_str());  // stale segment of a crashed run
      fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(create " + name + "): " + std::strerror(errno));
      if (ftruncate(fd, static_cast<off_t>(bytes_)) != 0) {
        const int e = errno;
        close(fd);
        (void)shm_unlink(name.c_str());
        throw std::runtime_error(std::string("ftruncate: ") + std::strerror(e));
      }
    } else {
      fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
      struct stat sb;
      if (fstat(fd, &sb) != 0 || static_cast<size_t>(sb.st_size) < bytes_) {
        close(fd);
        throw std::runtime_error("ShmControl: segment " + name + " has the wrong size (world mismatch?)");
      }
    }
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error(std::string("mmap: ") + std::strerror(errno));
    base_ = static_cast<char*>(p);
    hdr_ = reinterpret_cast<Header*>(base_);
    board_ = reinterpret_cast<Board*>(base_ + sizeof(Header));
    slots_ = reinterpret_cast<Slot*>(base_ + sizeof(Header) + static_cast<size_t>(world) * sizeof(Board));
    if (create) {
      std::memset(base_, 0, bytes_);  // ftruncate already zeroes; be explicit
      hdr_->world = world;
      hdr_->best.store(INT64_MAX, std::memory_order_relaxed);
      std::atomic_thread_fence(std::memory_order_release);
      hdr_->magic.store(kMagic, std::memory_order_release);
    } else {
      if (hdr_->magic.load(std::memory_order_acquire) != kMagic || hdr_->world != world) {
        munmap(base_, bytes_);
        throw std::runtime_error("ShmControl: segment " + name + " is not initialised for this world size");
      }
    }
  }

  ~ShmControl() {
    if (base_) munmap(base_, bytes_);
  }
  ShmControl(const ShmControl&) = delete;
  ShmControl& operator=(const ShmControl&) = delete;

  // Remove the name once every rank has mapped the segment (the mapping stays valid).
  void unlink() { (void)shm_unlink(name_.c_str()); }

  int rank() const { return rank_; }
  int world() const { return world_; }
  uint64_t rounds() const { return round_; }

  // out[r * n + i] = value i of rank r. Collective: every rank calls it in the same order.
  void allgather(const int64_t* vals, int n, int64_t* out, double timeout_s) {
    allgather(vals, n, out, timeout_s, [] {});
  }
  // Same, calling idle() now and then while waiting for the other ranks.
  template <class Idle>
  void allgather(const int64_t* vals, int n, int64_t* out, double timeout_s, Idle&& idle) {
    if (n < 0 || n > kMaxVals) throw std::invalid_argument("ShmControl::allgather: at most 15 values");
    const uint64_t r = ++round_;
    const int par = static_cast<int>(r & 1);
    Slot& mine = slot(par, rank_);
    for (int i = 0; i < n; ++i) mine.v[i] = vals[i];
    mine.seq.store(r, std::memory_order_release);
    const auto t0 = std::chrono::steady_clock::now();
    for (int q = 0; q < world_; ++q) {
      Slot& s = slot(par, q);
      unsigned spins = 0;
      while (s.seq.load(std::memory_order_acquire) < r) {
        if ((++spins & 63) == 0) idle();
        if (spins < 2048) {
          __builtin_ia32_pause();
          continue;
        }
        std::this_thread::yield();
        if ((spins & 255) == 0 && timeout_s > 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
          throw std::runtime_error("ShmControl: rank " + std::to_string(q) + " did not reach round " +
                                   std::to_string(r) + " within " + std::to_string(timeout_s) + " s");
      }
      for (int i = 0; i < n; ++i) out[q * n + i] = s.v[i];
    }
  }

  void barrier(double timeout_s) {
    int64_t dummy = 0;
    allgather(&dummy, 0, &dummy, timeout_s);
  }

  // Node-wide incumbent: atomic MIN visible to every rank at once (checkBest).
  int64_t offer_best(int64_t b) {
    int64_t cur = hdr_->best.load(std::memory_order_relaxed);
    while (b < cur && !hdr_->best.compare_exchange_weak(cur, b, std::memory_order_acq_rel)) {
    }
    return b < cur ? b : cur;
  }
  int64_t best() const { return hdr_->best.load(std::memory_order_acquire); }

  // Live incumbent of the current cooperative solve, exchanged after every graph
  // replay (not only at round boundaries). The word is (solve epoch << 32) | best,
  // so a solve never inherits the previous solve's incumbent: every rank calls
  // begin_solve() once per solve, in the same order, like the all-gathers.
  uint32_t begin_solve() { return ++epoch_; }
  int exchange_best(int b) {
    if (epoch_ == 0) return b;  // no solve begun: nothing to exchange with
    const uint64_t mine = (static_cast<uint64_t>(epoch_) << 32) | static_cast<uint32_t>(b);
    uint64_t cur = hdr_->solve_best.load(std::memory_order_acquire);
    for (;;) {
      const uint32_t ce = static_cast<uint32_t>(cur >> 32);
      const int cb = static_cast<int>(static_cast<uint32_t>(cur));
      if (ce > epoch_) return b;               // a peer has already moved on to the next solve
      if (ce == epoch_ && cb <= b) return cb;  // a peer's incumbent is at least as good
      if (hdr_->solve_best.compare_exchange_weak(cur, mine, std::memory_order_acq_rel)) return b;
    }
  }

  // ---- board ----
  void publish_size(int64_t n) { board_[rank_].size.store(n, std::memory_order_relaxed); }
  int64_t peer_size(int r) const { return board_[r].size.load(std::memory_order_relaxed); }
  // Ask every rank to join round `r` (the next all-gather) as soon as it can.
  void request_round(uint64_t r) {
    uint64_t cur = hdr_->request.load(std::memory_order_relaxed);
    while (cur < r && !hdr_->request.compare_exchange_weak(cur, r, std::memory_order_acq_rel)) {
    }
  }
  // Has a peer asked for an all-gather this rank has not joined yet?
  bool round_requested() const { return hdr_->request.load(std::memory_order_acquire) > round_; }

  // Object identity for a native caller built by the other compiler (the g++ and
  // hipcc modules share this header): address + layout tag.
  uintptr_t address() const { return reinterpret_cast<uintptr_t>(this); }
  static uint64_t layout_tag() { return kMagic ^ (static_cast<uint64_t>(sizeof(ShmControl)) << 48); }
  uint64_t tag() const { return tag_; }

 private:
  struct alignas(128) Header {
    std::atomic<uint64_t> magic;
    int world;
    int pad;
    std::atomic<int64_t> best;
    std::atomic<uint64_t> request;  // highest all-gather round requested early
    std::atomic<uint64_t> solve_best;  // (solve epoch << 32) | live incumbent (exchange_best)
  };
  struct alignas(128) Board {
    std::atomic<int64_t> size;  // live pool size of the rank
  };
  struct alignas(128) Slot {
    std::atomic<uint64_t> seq;
    int64_t v[kMaxVals];
  };
  static_assert(sizeof(Slot) == 128, "one cache-line pair per slot");
  static_assert(std::atomic<uint64_t>::is_always_lock_free, "lock-free atomics needed across processes");

  Slot& slot(int par, int r) { return slots_[par * world_ + r]; }

  std::string name_;
  int rank_, world_;
  size_t bytes_ = 0;
  char* base_ = nullptr;
  Header* hdr_ = nullptr;
  Board* board_ = nullptr;
  Slot* slots_ = nullptr;
  uint64_t round_ = 0;
  uint32_t epoch_ = 0;  // cooperative solves begun (begin_solve)
  uint64_t tag_ = layout_tag();
};

}  // namespace tts
