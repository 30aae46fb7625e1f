// Host work pool: a growable array deque with an optional spin lock and bulk ops.
//
// Parity: ref pfsp/lib/Pool_atom.{h,c} (SinglePool_atom) and nqueens/lib/Pool.c.
// Same operations and the same bulk semantics:
//   pop_back_bulk(m, M, out, ratio) returns min(size/ratio, M) nodes taken from the
//   back, and only when size >= ratio*m (ref Pool_atom.c:154-194);
//   round_robin(src, id, step) gives element id, id+step, ... and the tail to the
//   last worker (ref Pool_atom.c:14-36).
// Differences by design: std::atomic_flag-style lock with acquire/release order
// (the reference's locked popBack CASes false->false and never locks,
// Pool_atom.c:119); 64-bit sizes; memcpy bulk moves.
#pragma once

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <type_traits>

namespace tts {

class SpinLock {
 public:
  void lock() {
    while (flag_.exchange(true, std::memory_order_acquire)) {
      while (flag_.load(std::memory_order_relaxed)) {
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
      }
    }
  }
  bool try_lock() { return !flag_.load(std::memory_order_relaxed) && !flag_.exchange(true, std::memory_order_acquire); }
  void unlock() { flag_.store(false, std::memory_order_release); }

 private:
  std::atomic<bool> flag_{false};
};

template <typename T>
class Pool {
  static_assert(std::is_trivially_copyable<T>::value, "pool elements must be trivially copyable");

 public:
  static constexpr size_t kInitialCapacity = 1024;

  Pool() { reserve_exact(kInitialCapacity); }
  ~Pool() { std::free(data_); }
  Pool(const Pool&) = delete;
  Pool& operator=(const Pool&) = delete;
  Pool(Pool&& o) noexcept : data_(o.data_), cap_(o.cap_), front_(o.front_), size_(o.size_) {
    o.data_ = nullptr;
    o.cap_ = o.front_ = o.size_ = 0;
  }

  size_t size() const { return size_; }
  size_t size_relaxed() const { return __atomic_load_n(&size_, __ATOMIC_RELAXED); }
  bool empty() const { return size_ == 0; }
  size_t capacity() const { return cap_; }
  SpinLock& lock() { return lock_; }
  T* data() { return data_ + front_; }
  const T* data() const { return data_ + front_; }
  void clear() { front_ = size_ = 0; }

  // ---- unlocked ("Free") operations: caller owns the pool ----
  void push_back_free(const T& v) {
    ensure(1);
    data_[front_ + size_] = v;
    set_size(size_ + 1);
  }
  void push_back_bulk_free(const T* v, size_t n) {
    if (n == 0) return;
    ensure(n);
    std::memcpy(static_cast<void*>(data_ + front_ + size_), v, n * sizeof(T));
    set_size(size_ + n);
  }
  bool pop_back_free(T& out) {
    if (size_ == 0) return false;
    set_size(size_ - 1);
    out = data_[front_ + size_];
    return true;
  }
  bool pop_front_free(T& out) {
    if (size_ == 0) return false;
    out = data_[front_];
    ++front_;
    set_size(size_ - 1);
    return true;
  }
  // Returns min(size/ratio, M) nodes from the back if size >= ratio*m, else 0.
  size_t pop_back_bulk_free(size_t m, size_t M, T* out, size_t ratio = 1) {
    if (size_ < ratio * m || size_ == 0) return 0;
    const size_t n = std::min(size_ / ratio, M);
    set_size(size_ - n);
    std::memcpy(static_cast<void*>(out), data_ + front_ + size_, n * sizeof(T));
    return n;
  }
  // Removes the n back elements, exposing them in place (valid until next push).
  const T* pop_back_span_free(size_t n) {
    n = std::min(n, size_);
    set_size(size_ - n);
    return data_ + front_ + size_;
  }

  // ---- locked operations ----
  void push_back(const T& v) {
    lock_.lock();
    push_back_free(v);
    lock_.unlock();
  }
  void push_back_bulk(const T* v, size_t n) {
    lock_.lock();
    push_back_bulk_free(v, n);
    lock_.unlock();
  }
  bool pop_back(T& out) {
    lock_.lock();
    const bool ok = pop_back_free(out);
    lock_.unlock();
    return ok;
  }
  size_t pop_back_bulk(size_t m, size_t M, T* out, size_t ratio = 1) {
    lock_.lock();
    const size_t n = pop_back_bulk_free(m, M, out, ratio);
    lock_.unlock();
    return n;
  }

  // Static cyclic distribution of src to worker `id` of `step` (caller owns both).
  void round_robin_from(const Pool& src, size_t id, size_t step) {
    const size_t n = src.size_;
    const size_t c = n / step;
    const size_t l = n - (step - 1) * c;
    ensure(l);
    const T* s = src.data_ + src.front_;
    for (size_t i = 0; i < c; ++i) data_[front_ + size_ + i] = s[id + i * step];
    size_t added = c;
    if (id == step - 1) {
      for (size_t i = c; i < l; ++i) data_[front_ + size_ + i] = s[step * c + i - c];
      added = l;
    }
    set_size(size_ + added);
  }

 private:
  void set_size(size_t s) { __atomic_store_n(&size_, s, __ATOMIC_RELAXED); }
  void reserve_exact(size_t c) {
    T* nd = static_cast<T*>(std::realloc(data_, c * sizeof(T)));
    if (!nd) throw std::bad_alloc();
    data_ = nd;
    cap_ = c;
  }
  void ensure(size_t extra) {
    const size_t need = front_ + size_ + extra;
    if (need <= cap_) return;
    if (front_ > 0 && size_ + extra <= cap_ / 2) {  // reclaim the consumed front first
      std::memmove(static_cast<void*>(data_), data_ + front_, size_ * sizeof(T));
      front_ = 0;
      return;
    }
    size_t c = cap_ ? cap_ : kInitialCapacity;
    while (c < need) c *= 2;
    reserve_exact(c);
  }

  T* data_ = nullptr;
  size_t cap_ = 0, front_ = 0, size_ = 0;
  SpinLock lock_;
};

}  // namespace tts
