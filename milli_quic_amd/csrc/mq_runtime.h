// mq_runtime.h — host-side bookkeeping of libmq_aead.so that needs no GPU to reason about:
//   * DeviceRegistry: the device each calling thread has selected (mq_device_init), validated once
//     per device (gfx950), and a scoped guard that runs one call on an object's device and gives
//     the caller's current HIP device back afterwards — the library never leaves another device
//     current on a thread than the one the thread chose;
//   * SideStreams: the side streams of the forked tile kernels (the AES hot-key kernel, the ChaCha
//     list of a mixed batch), one set per (device, caller stream), so batches pipelined on several
//     caller streams never wait on each other through a shared side stream. Entries are bounded
//     (least recently used evicted) and released explicitly with mq_stream_release.
// Everything is templated on a Backend (mq_host.cpp: HIP; tests/csrc/test_runtime.cpp: a fake
// backend that checks the bookkeeping on the CPU under ASan/UBSan).
//
// Backend interface (static members):
//   typedef ... Stream, Event;
//   int count();                     devices visible (0 on error)
//   bool usable(int dev);            a gfx950
//   int cus(int dev);                compute units (0 on error)
//   int get();                       the calling thread's current device (-1 on error)
//   bool set(int dev);               make dev current on the calling thread
//   bool stream_create(Stream*);     non-blocking stream on the current device
//   void stream_destroy(Stream);     waits for its work, then destroys
//   bool event_create(Event*);       no timing
//   void event_destroy(Event);
//   bool record(Event, Stream);      event after the stream's work so far
//   bool wait(Stream, Event);        the stream's later work waits for the event
#pragma once
#include <cstdint>
#include <list>
#include <memory>
#include <mutex>
#include <vector>

namespace mq {

// The calling thread's selection: -1 = none (follow the thread's current HIP device).
inline int& thread_device() {
  static thread_local int dev = -1;
  return dev;
}

template <class B>
class DeviceRegistry {
 public:
  // mq_device_init: validate, make current on this thread, remember. A failed selection keeps
  // the thread's previous choice. Returns false when the device is absent or not a gfx950.
  bool select(int dev) {
    if (!valid(dev) || !B::set(dev)) return false;
    thread_device() = dev;
    return true;
  }

  // The device calls of this thread run on: its selection, else its current HIP device.
  // -1 when neither is a usable gfx950.
  int current() {
    const int sel = thread_device();
    if (sel >= 0) return sel;
    const int cur = B::get();
    return valid(cur) ? cur : -1;
  }

  // gfx950 check, cached per device (process-wide, the answer never changes)
  bool valid(int dev) {
    if (dev < 0) return false;
    std::lock_guard<std::mutex> lk(mu_);
    if (count_ < 0) count_ = B::count();
    if (dev >= count_) return false;
    if ((size_t)dev >= state_.size()) state_.resize((size_t)count_, 0);
    if (state_[(size_t)dev] == 0) state_[(size_t)dev] = B::usable(dev) ? 1 : -1;
    return state_[(size_t)dev] == 1;
  }

  // compute units of a valid device (cached)
  int cus(int dev) {
    if (!valid(dev)) return 0;
    std::lock_guard<std::mutex> lk(mu_);
    if ((size_t)dev >= cus_.size()) cus_.resize((size_t)count_, 0);
    if (cus_[(size_t)dev] <= 0) cus_[(size_t)dev] = B::cus(dev);
    return cus_[(size_t)dev];
  }

  // Runs the enclosing call on `dev` and restores the thread's current device on exit (a no-op
  // when dev is already current).
  class Guard {
   public:
    explicit Guard(int dev) : prev_(B::get()), ok_(dev >= 0) {
      if (ok_ && prev_ != dev) {
        ok_ = B::set(dev);
        switched_ = ok_;
      }
    }
    ~Guard() {
      if (switched_ && prev_ >= 0) (void)B::set(prev_);
    }
    bool ok() const { return ok_; }
    Guard(const Guard&) = delete;
    Guard& operator=(const Guard&) = delete;

   private:
    int prev_;
    bool ok_, switched_ = false;
  };

 private:
  std::mutex mu_;
  int count_ = -1;
  std::vector<int8_t> state_;  // 0 unknown, 1 gfx950, -1 unusable
  std::vector<int> cus_;
};

// Side streams per (device, caller stream). kSides streams each, with a fork event (recorded on
// the caller's stream) and one join event per side stream.
template <class B, int kSides = 2>
class SideStreams {
 public:
  typedef typename B::Stream Stream;
  typedef typename B::Event Event;
  static constexpr int kSteps = 8;  // caller -> side hand-offs of one fork (chunked pipelines)

  typedef void (*Hook)(Stream);  // called with each side stream before it is destroyed

  struct Entry {
    int dev = -1;
    Stream caller{};
    Stream side[kSides]{};
    Event fork{}, join[kSides]{}, step[kSteps]{};
    bool ok = false;
    Hook on_destroy = nullptr;
    std::mutex mu;  // one fork/launch/join sequence at a time
    ~Entry() {
      // stream_destroy waits for the side stream's work; run it on the entry's device
      typename DeviceRegistry<B>::Guard g(dev);
      for (int k = 0; k < kSides; ++k) {
        if (side[k] && on_destroy) on_destroy(side[k]);  // e.g. its schedule slot back (mq_host.cpp)
        if (side[k]) B::stream_destroy(side[k]);
        if (join[k]) B::event_destroy(join[k]);
      }
      for (int k = 0; k < kSteps; ++k)
        if (step[k]) B::event_destroy(step[k]);
      if (fork) B::event_destroy(fork);
    }
  };

  // One forked section on `caller` (device `dev`, current on this thread): the side streams start
  // after the caller's work so far; join() makes the caller wait for everything launched on them.
  // Holds the entry for its lifetime (an evicted entry is destroyed when its last fork ends).
  class Fork {
   public:
    Fork() = default;
    Fork(std::shared_ptr<Entry> e, int used) : e_(std::move(e)), used_(used) {
      if (e_) lk_ = std::unique_lock<std::mutex>(e_->mu);
    }
    explicit operator bool() const { return e_ != nullptr; }
    Stream side(int k) const { return e_->side[k]; }
    // hand-off k (< kSteps) of a pipeline: side stream `sd`'s later work waits for the caller's
    // work so far (e.g. chunk k built on the caller's stream, then sealed on the side stream)
    bool hand_off(int k, int sd) {
      return k >= 0 && k < kSteps && B::record(e_->step[k], e_->caller) && B::wait(e_->side[sd], e_->step[k]);
    }
    // returns false if a join could not be enqueued (the caller's stream then does not wait)
    bool join() {
      if (!e_ || joined_) return true;
      joined_ = true;
      bool ok = true;
      for (int k = 0; k < used_; ++k)
        ok = B::record(e_->join[k], e_->side[k]) && B::wait(e_->caller, e_->join[k]) && ok;
      return ok;
    }
    ~Fork() { (void)join(); }
    Fork(Fork&&) = default;
    void dismiss() { joined_ = true; }  // nothing was forked: no join to enqueue

   private:
    std::shared_ptr<Entry> e_;
    std::unique_lock<std::mutex> lk_;
    int used_ = 0;
    bool joined_ = false;
  };

  explicit SideStreams(size_t cap = 64, Hook on_destroy = nullptr) : cap_(cap), hook_(on_destroy) {}

  // Fork `used` (<= kSides) side streams off `caller` on device `dev`; an empty Fork (launch on the
  // caller's stream instead) if the streams cannot be created.
  Fork fork(int dev, Stream caller, int used) {
    std::shared_ptr<Entry> e = get(dev, caller);
    if (!e) return Fork();
    Fork f(e, used);
    bool ok = B::record(e->fork, caller);
    for (int k = 0; k < used && ok; ++k) ok = B::wait(e->side[k], e->fork);
    if (!ok) {  // nothing launched yet: the caller's stream carries the work alone
      f.dismiss();
      return Fork();
    }
    return f;
  }

  // Drops the entries of `caller` (every device). Their side streams are destroyed once no fork
  // holds them, after their work has finished.
  void release(Stream caller) {
    std::vector<std::shared_ptr<Entry>> dead;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto it = lru_.begin(); it != lru_.end();) {
        if ((*it)->caller == caller) {
          dead.push_back(*it);
          it = lru_.erase(it);
        } else {
          ++it;
        }
      }
    }
    dead.clear();  // outside the registry lock: destruction waits for the GPU
  }

  size_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return lru_.size();
  }

 private:
  std::shared_ptr<Entry> get(int dev, Stream caller) {
    std::shared_ptr<Entry> evicted;
    std::shared_ptr<Entry> e;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto it = lru_.begin(); it != lru_.end(); ++it)
        if ((*it)->dev == dev && (*it)->caller == caller) {
          e = *it;
          lru_.splice(lru_.begin(), lru_, it);  // most recently used first
          return e->ok ? e : nullptr;
        }
      e = std::make_shared<Entry>();
      e->dev = dev;
      e->caller = caller;
      e->on_destroy = hook_;
      bool ok = B::event_create(&e->fork);
      for (int k = 0; k < kSides && ok; ++k) ok = B::stream_create(&e->side[k]) && B::event_create(&e->join[k]);
      for (int k = 0; k < kSteps && ok; ++k) ok = B::event_create(&e->step[k]);
      e->ok = ok;
      lru_.push_front(e);
      if (lru_.size() > cap_) {
        evicted = lru_.back();
        lru_.pop_back();
      }
    }
    evicted.reset();  // outside the registry lock
    return e->ok ? e : nullptr;
  }

  std::mutex mu_;
  std::list<std::shared_ptr<Entry>> lru_;
  size_t cap_;
  Hook hook_;
};

// Device words of the persistent tile kernels' dynamic schedule (mq_tile.h TileSched), one slot per
// (device, stream). Kernels on one stream run one after another and each leaves its slot zeroed
// when its last workgroup ends, so a slot is never used by two kernels at once; kernels that run
// concurrently (a forked side stream) are on other streams and so have other slots. The slots of a
// device are one zeroed allocation made on first use (the caller holds a guard on the device) and
// never freed (a kernel may still be running when the library is unloaded). A stream beyond the
// capacity gets no slot: its kernels take the static schedule. release(stream) waits for the
// stream's work (its kernels may still use the slot), then recycles its slots.
//
// Backend additions: void* alloc_zeroed(size_t bytes)  device memory on the current device (null
// on failure); void stream_sync(Stream)  waits for the stream's work.
template <class B>
class SchedSlots {
 public:
  typedef typename B::Stream Stream;

  SchedSlots(uint32_t slots, size_t slot_bytes) : slots_(slots), bytes_(slot_bytes) {}

  // the slot of (dev, s), assigned on first use; null when none is left or allocation failed
  void* get(int dev, Stream s) {
    if (dev < 0) return nullptr;
    std::lock_guard<std::mutex> lk(mu_);
    if ((size_t)dev >= dev_.size()) dev_.resize((size_t)dev + 1);
    PerDev& d = dev_[(size_t)dev];
    for (const auto& e : d.map)
      if (e.first == s) return d.base + bytes_ * e.second;
    if (!d.base) {
      if (d.failed) return nullptr;
      d.base = (uint8_t*)B::alloc_zeroed(bytes_ * slots_);
      if (!d.base) {
        d.failed = true;
        return nullptr;
      }
    }
    uint32_t idx;
    if (!d.free.empty()) {
      idx = d.free.back();
      d.free.pop_back();
    } else if (d.used < slots_) {
      idx = d.used++;
    } else {
      return nullptr;
    }
    d.map.emplace_back(s, idx);
    return d.base + bytes_ * idx;
  }

  // Recycles the slots of stream s (every device) once its work has finished.
  void release(Stream s) {
    bool had = false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      for (auto& d : dev_)
        for (const auto& e : d.map) had = had || e.first == s;
    }
    if (!had) return;
    B::stream_sync(s);  // outside the lock: its kernels may still count on the slot
    std::lock_guard<std::mutex> lk(mu_);
    for (auto& d : dev_)
      for (auto it = d.map.begin(); it != d.map.end();) {
        if (it->first == s) {
          d.free.push_back(it->second);
          it = d.map.erase(it);
        } else {
          ++it;
        }
      }
  }

  size_t assigned(int dev) {
    std::lock_guard<std::mutex> lk(mu_);
    return (dev >= 0 && (size_t)dev < dev_.size()) ? dev_[(size_t)dev].map.size() : 0;
  }

 private:
  struct PerDev {
    uint8_t* base = nullptr;
    bool failed = false;
    uint32_t used = 0;
    std::vector<std::pair<Stream, uint32_t>> map;
    std::vector<uint32_t> free;
  };
  std::mutex mu_;
  std::vector<PerDev> dev_;
  uint32_t slots_;
  size_t bytes_;
};

}  // namespace mq
