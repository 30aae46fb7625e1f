// Pinned host extension of a device pool: the oldest nodes of the ring live here
// when the ring (HBM) runs out of room.
//
// Parity: the reference's pools are growable host arrays (ref pfsp/lib/Pool_atom.c:
// 75-110 pushBackBulk, 154-194 popBackBulk) that every batch copies to the GPU
// with synchronous pageable cudaMemcpy. Here the device ring is the pool, and this
// store only extends its bottom: [spill (host, oldest) | ring bot .. ring top].
//   * blocks are hipHostMalloc'd (pinned) and recycled, so every copy is an
//     asynchronous DMA on the engine's transfer stream;
//   * a spill moves the ring bottom into a new top block (D2H), a refill moves the
//     newest spilled nodes back under the ring bottom (H2D); both run while graph
//     replays keep expanding the ring top — the engine reserves the ring span a
//     copy touches until its event has completed (DeviceEngine::reserved_);
//   * host pops (pop_host, checkpoints) take the oldest nodes first.
#pragma once

#include <algorithm>
#include <cstring>
#include <deque>
#include <vector>

#include "device_common.hpp"

namespace tts {

template <class Node>
class PinnedSpill {
 public:
  struct Block {
    Node* h = nullptr;
    size_t cap = 0;
    size_t lo = 0, hi = 0;      // live nodes h[lo, hi), oldest first
    hipEvent_t ev = nullptr;    // last copy touching the block
    bool pending = false;       // ev not known to be complete
  };

  explicit PinnedSpill(size_t block_nodes) : block_nodes_(std::max<size_t>(1, block_nodes)) {}
  ~PinnedSpill() { free_all(); }
  // Every pinned block back to the runtime now (the engine's release(), before runtime
  // teardown); the spill is empty and unusable for copies in flight afterwards.
  void free_all() {
    for (auto& b : blocks_) release(b);
    for (auto& b : free_) release(b);
    blocks_.clear();
    free_.clear();
    n_ = 0;
  }
  PinnedSpill(const PinnedSpill&) = delete;
  PinnedSpill& operator=(const PinnedSpill&) = delete;

  size_t size() const { return n_; }
  // Nodes the next pop_to_device can return at most (the newest block's).
  size_t top_count() {
    trim();
    return blocks_.empty() ? 0 : blocks_.back().hi - blocks_.back().lo;
  }
  bool empty() const { return n_ == 0; }
  size_t block_nodes() const { return block_nodes_; }

  // D2H: `n` contiguous device nodes become the newest spilled nodes (one or more
  // new top blocks). Enqueued on `s`; returns after enqueueing. `on_block(ev, k)`
  // is told the event that completes each piece of k nodes.
  template <class F>
  void push_from_device(const Node* src, size_t n, hipStream_t s, F&& on_block) {
    while (n) {
      Block b = take_free();
      const size_t k = std::min(n, b.cap);
      TTS_HIP_CHECK(hipMemcpyAsync(b.h, src, k * sizeof(Node), hipMemcpyDeviceToHost, s));
      TTS_HIP_CHECK(hipEventRecord(b.ev, s));
      b.pending = true;
      b.lo = 0;
      b.hi = k;
      blocks_.push_back(b);
      n_ += k;
      on_block(b.ev, k);
      src += k;
      n -= k;
    }
  }

  // Host nodes become the newest spilled nodes (synchronous memcpy into pinned blocks).
  void push_host(const Node* src, size_t n) {
    while (n) {
      if (blocks_.empty() || blocks_.back().hi == blocks_.back().cap) {
        Block b = take_free();
        b.lo = b.hi = 0;
        blocks_.push_back(b);
      }
      Block& t = blocks_.back();
      wait(t);
      const size_t k = std::min(n, t.cap - t.hi);
      std::memcpy(t.h + t.hi, src, k * sizeof(Node));
      t.hi += k;
      n_ += k;
      src += k;
      n -= k;
    }
  }

  // H2D: the newest `n` spilled nodes (at most one block's worth) go to dst, oldest
  // first, enqueued on `s`. Returns the count and the event that completes it.
  // `s` must be the stream of the D2H copies (push_from_device): a block still
  // being filled is then read after its fill in stream order, without a host wait.
  size_t pop_to_device(Node* dst, size_t n, hipStream_t s, hipEvent_t* done) {
    trim();
    if (blocks_.empty() || n == 0) return 0;
    Block& t = blocks_.back();
    const size_t k = std::min(n, t.hi - t.lo);
    TTS_HIP_CHECK(hipMemcpyAsync(dst, t.h + (t.hi - k), k * sizeof(Node), hipMemcpyHostToDevice, s));
    TTS_HIP_CHECK(hipEventRecord(t.ev, s));
    t.pending = true;
    t.hi -= k;
    n_ -= k;
    *done = t.ev;
    trim();
    return k;
  }

  // Oldest-first host pop (pop_host / checkpoints): completes pending copies.
  size_t pop_oldest(Node* dst, size_t n) {
    size_t got = 0;
    while (got < n && !blocks_.empty()) {
      Block& b = blocks_.front();
      wait(b);
      const size_t k = std::min(n - got, b.hi - b.lo);
      std::memcpy(dst + got, b.h + b.lo, k * sizeof(Node));
      b.lo += k;
      n_ -= k;
      got += k;
      if (b.lo == b.hi) {
        free_.push_back(b);
        blocks_.pop_front();
      }
    }
    return got;
  }

  // Everything, oldest first, left in place (host copy; completes pending copies).
  void snapshot(std::vector<Node>& out) {
    out.clear();
    out.reserve(n_);
    for (auto& b : blocks_) {
      wait(b);
      out.insert(out.end(), b.h + b.lo, b.h + b.hi);
    }
  }

  void clear() {
    for (auto& b : blocks_) {
      wait(b);
      free_.push_back(b);
    }
    blocks_.clear();
    n_ = 0;
  }

  // Keep the i % world == rank nodes (oldest first numbering).
  void keep_strided(int rank, int world) {
    std::vector<Node> all;
    snapshot(all);
    clear();
    std::vector<Node> mine;
    for (size_t i = static_cast<size_t>(rank); i < all.size(); i += static_cast<size_t>(world)) mine.push_back(all[i]);
    push_host(mine.data(), mine.size());
  }

  size_t pinned_bytes() const { return (blocks_.size() + free_.size()) * block_nodes_ * sizeof(Node); }

 private:
  Block take_free() {
    if (!free_.empty()) {
      Block b = free_.back();
      free_.pop_back();
      wait(b);
      return b;
    }
    Block b;
    b.cap = block_nodes_;
    TTS_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&b.h), b.cap * sizeof(Node), hipHostMallocDefault));
    TTS_HIP_CHECK(hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
    return b;
  }
  void wait(Block& b) {
    if (b.pending) {
      TTS_HIP_CHECK(hipEventSynchronize(b.ev));
      b.pending = false;
    }
  }
  void trim() {
    while (!blocks_.empty() && blocks_.back().lo == blocks_.back().hi) {
      free_.push_back(blocks_.back());
      blocks_.pop_back();
    }
  }
  static void release(Block& b) {
    if (b.ev) {
      (void)hipEventSynchronize(b.ev);
      (void)hipEventDestroy(b.ev);
    }
    if (b.h) (void)hipHostFree(b.h);
    b.h = nullptr;
    b.ev = nullptr;
  }

  size_t block_nodes_;
  size_t n_ = 0;
  std::deque<Block> blocks_;  // oldest block first
  std::vector<Block> free_;
};

}  // namespace tts
