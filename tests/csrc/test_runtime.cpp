// test_runtime.cpp — CPU unit test of the host bookkeeping in milli_quic_amd/csrc/mq_runtime.h
// (per-thread device selection, device guards, side streams per (device, caller stream)) against
// a fake backend that models HIP's per-thread current device and checks every stream / event it
// hands out: created on the right device, never used after destruction, all destroyed at the end.
// Built and run by tests/test_runtime.py with -fsanitize=address,undefined.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "../../milli_quic_amd/csrc/mq_runtime.h"

#define CHECK(c)                                                           \
  do {                                                                     \
    if (!(c)) {                                                            \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      std::abort();                                                        \
    }                                                                      \
  } while (0)

struct FakeObj {
  int dev;
  std::atomic<bool> dead{false};
  std::atomic<int> records{0}, waits{0}, syncs{0};
  explicit FakeObj(int d) : dev(d) {}
};

struct Fake {
  typedef FakeObj* Stream;
  typedef FakeObj* Event;
  static constexpr int kDevices = 4;  // device 2 is not a gfx950
  static std::atomic<int> live_streams, live_events, set_calls, usable_calls;
  static int& cur() {
    static thread_local int d = 0;  // HIP's default: device 0 current on every new thread
    return d;
  }
  static int count() { return kDevices; }
  static bool usable(int d) {
    ++usable_calls;
    return d != 2;
  }
  static int cus(int d) { return d == 3 ? 128 : 256; }
  static int get() { return cur(); }
  static bool set(int d) {
    ++set_calls;
    if (d < 0 || d >= kDevices) return false;
    cur() = d;
    return true;
  }
  static bool stream_create(Stream* s) {
    *s = new FakeObj(cur());
    ++live_streams;
    return true;
  }
  static void stream_destroy(Stream s) {
    CHECK(!s->dead.exchange(true));
    CHECK(cur() == s->dev);  // destroyed on its own device (the entry's guard)
    --live_streams;
    delete s;
  }
  static bool event_create(Event* e) {
    *e = new FakeObj(cur());
    ++live_events;
    return true;
  }
  static void event_destroy(Event e) {
    CHECK(!e->dead.exchange(true));
    --live_events;
    delete e;
  }
  static bool record(Event e, Stream s) {
    CHECK(!e->dead && !s->dead);
    CHECK(e->dev == s->dev);  // HIP: an event is recorded on a stream of its own device
    ++e->records;
    return true;
  }
  static bool wait(Stream s, Event e) {
    CHECK(!e->dead && !s->dead);
    ++s->waits;
    return true;
  }
  static void* alloc_zeroed(size_t bytes) {  // leaked on purpose, as the library's slots are
    ++allocs;
    void* p = std::calloc(1, bytes);
    allocated.push_back(p);
    return p;
  }
  static void stream_sync(Stream s) {
    CHECK(!s->dead);
    ++s->syncs;
  }
  static std::atomic<int> allocs;
  static std::vector<void*> allocated;
};
std::atomic<int> Fake::live_streams{0}, Fake::live_events{0}, Fake::set_calls{0}, Fake::usable_calls{0};
std::atomic<int> Fake::allocs{0};
std::vector<void*> Fake::allocated;

typedef mq::DeviceRegistry<Fake> Devices;

static void test_per_thread_selection() {
  Devices reg;
  CHECK(reg.current() == 0);  // no selection: the thread's current HIP device
  std::atomic<int> ready{0};
  auto body = [&](int dev) {
    CHECK(mq::thread_device() == -1);
    CHECK(reg.select(dev));
    ++ready;
    while (ready.load() < 2) std::this_thread::yield();  // both threads have selected
    for (int k = 0; k < 1000; ++k) {
      CHECK(reg.current() == dev);  // never the other thread's choice
      CHECK(Fake::get() == dev);
    }
    CHECK(!reg.select(2) && !reg.select(7) && !reg.select(-1));  // not a gfx950 / absent
    CHECK(reg.current() == dev && Fake::get() == dev);            // previous selection kept
  };
  std::thread a(body, 1), b(body, 3);
  a.join();
  b.join();
  CHECK(reg.current() == 0 && mq::thread_device() == -1);  // this thread chose nothing
  Fake::set(3);
  CHECK(reg.current() == 3);  // follows the current HIP device while nothing is selected
  Fake::set(2);
  CHECK(reg.current() == -1);  // not a gfx950
  Fake::set(0);
  CHECK(reg.cus(3) == 128 && reg.cus(1) == 256 && reg.cus(2) == 0 && reg.cus(9) == 0);
  const int u = Fake::usable_calls;
  for (int k = 0; k < 100; ++k) CHECK(reg.valid(1) && !reg.valid(2));
  CHECK(Fake::usable_calls == u);  // validated once per device
}

static void test_guard() {
  Fake::set(1);
  const int before = Fake::set_calls;
  {
    Devices::Guard g(1);
    CHECK(g.ok() && Fake::get() == 1);
  }
  CHECK(Fake::set_calls == before);  // already current: no switch
  {
    Devices::Guard g(3);
    CHECK(g.ok() && Fake::get() == 3);
    {
      Devices::Guard h(0);
      CHECK(Fake::get() == 0);
    }
    CHECK(Fake::get() == 3);
  }
  CHECK(Fake::get() == 1);  // the caller's device is back
  {
    Devices::Guard g(-1);
    CHECK(!g.ok() && Fake::get() == 1);
  }
  {
    Devices::Guard g(9);  // set fails: not ok, nothing to restore
    CHECK(!g.ok() && Fake::get() == 1);
  }
  Fake::set(0);
}

static void test_side_streams() {
  {
    mq::SideStreams<Fake, 2> ss(4);
    FakeObj callers[8] = {FakeObj(1), FakeObj(1), FakeObj(1), FakeObj(1),
                          FakeObj(1), FakeObj(1), FakeObj(3), FakeObj(3)};
    std::set<FakeObj*> sides;
    {
      Devices::Guard g(1);
      auto f = ss.fork(1, &callers[0], 2);
      CHECK(f && f.side(0) != f.side(1));
      CHECK(f.side(0)->dev == 1 && f.side(1)->dev == 1);  // created on the caller's device
      CHECK(f.side(0)->waits == 1 && f.side(1)->waits == 1);
      sides.insert(f.side(0));
      CHECK(f.hand_off(0, 1) && f.side(1)->waits == 2);  // a pipeline step: side 1 waits on the caller
      CHECK(!f.hand_off(8, 0) && !f.hand_off(-1, 0));
      CHECK(f.join());
      CHECK(callers[0].waits == 2);  // the caller waits for both side streams
      CHECK(f.join() && callers[0].waits == 2);  // a second join is a no-op
    }
    {
      Devices::Guard g(1);
      auto f = ss.fork(1, &callers[0], 1);  // same (device, caller): same side streams
      CHECK(f && sides.count(f.side(0)) == 1);
      auto h = ss.fork(1, &callers[1], 1);  // another caller stream: its own
      CHECK(h && sides.count(h.side(0)) == 0);
    }  // forks join on scope exit
    CHECK(callers[0].waits == 3 && callers[1].waits == 1);
    CHECK(ss.size() == 2 && Fake::live_streams == 4);
    // LRU bound: 6 callers on device 1 leave the 4 most recent
    for (int k = 2; k < 6; ++k) {
      Devices::Guard g(1);
      auto f = ss.fork(1, &callers[k], 2);
      CHECK(f);
    }
    CHECK(ss.size() == 4 && Fake::live_streams == 8 && Fake::live_events == 4 * (3 + 8));
    ss.release(&callers[5]);
    CHECK(ss.size() == 3 && Fake::live_streams == 6);
    ss.release(&callers[5]);  // nothing left for it
    CHECK(ss.size() == 3);
    // an entry evicted while a fork holds it lives until that fork ends
    mq::SideStreams<Fake, 2> small(1);
    {
      Devices::Guard g(3);
      auto f = small.fork(3, &callers[6], 2);
      CHECK(f);
      std::thread t([&] {
        Devices::Guard g3(3);
        auto h = small.fork(3, &callers[7], 2);  // evicts callers[6]'s entry
        CHECK(h);
      });
      t.join();
      CHECK(small.size() == 1);
      CHECK(!f.side(0)->dead && !f.side(1)->dead);  // still ours
      CHECK(f.join());
    }  // the evicted entry goes with its last fork
    CHECK(Fake::get() == 0);
  }  // registries gone: every stream and event destroyed
  CHECK(Fake::live_streams == 0 && Fake::live_events == 0);
}

static void test_concurrent_forks() {
  mq::SideStreams<Fake, 2> ss(64);
  std::vector<FakeObj*> callers;
  for (int t = 0; t < 8; ++t) callers.push_back(new FakeObj(t % 2 ? 3 : 1));
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t)
    th.emplace_back([&, t] {
      const int dev = t % 2 ? 3 : 1;
      Devices reg;
      CHECK(reg.select(dev));
      for (int k = 0; k < 2000; ++k) {
        // every other fork shares a caller stream with another thread of the same device
        // (serialised per entry)
        FakeObj* c = (k & 1) ? callers[t ^ 2] : callers[t];
        auto f = ss.fork(dev, c, 1 + (k & 1));
        CHECK(f && f.side(0)->dev == dev);
        if (k % 97 == 0) ss.release(callers[(t + 3) % 8]);
      }
    });
  for (auto& x : th) x.join();
  for (auto* c : callers) ss.release(c);
  CHECK(ss.size() == 0 && Fake::live_streams == 0 && Fake::live_events == 0);
  for (auto* c : callers) delete c;
}

// dynamic-schedule slots: one per (device, stream), stable, distinct, bounded; release waits for
// the stream's work before recycling its slot
static void test_sched_slots() {
  mq::SchedSlots<Fake> sl(3, 1024);
  FakeObj s[5] = {FakeObj(1), FakeObj(1), FakeObj(1), FakeObj(1), FakeObj(3)};
  uint8_t* a = (uint8_t*)sl.get(1, &s[0]);
  uint8_t* b = (uint8_t*)sl.get(1, &s[1]);
  uint8_t* c = (uint8_t*)sl.get(1, &s[2]);
  CHECK(a && b && c && a != b && b != c && a != c);
  CHECK(Fake::allocs == 1);  // one allocation per device
  for (uint8_t* p : {a, b, c}) {
    const long d = p - a;
    CHECK(d % 1024 == 0 && d >= -2048 && d <= 2048);
    for (int k = 0; k < 1024; ++k) CHECK(p[k] == 0);  // zeroed
  }
  CHECK(sl.get(1, &s[0]) == a && sl.get(1, &s[2]) == c);  // stable per stream
  CHECK(sl.get(1, &s[3]) == nullptr);                     // capacity: static schedule
  CHECK(sl.get(3, &s[4]) != nullptr && Fake::allocs == 2);  // another device, its own slots
  CHECK(sl.get(-1, &s[0]) == nullptr);
  CHECK(sl.assigned(1) == 3 && sl.assigned(3) == 1);
  sl.release(&s[1]);
  CHECK(s[1].syncs == 1 && s[0].syncs == 0);  // waited for before recycling
  CHECK(sl.assigned(1) == 2);
  CHECK(sl.get(1, &s[3]) == b);  // the recycled slot
  sl.release(&s[1]);
  CHECK(s[1].syncs == 1);  // nothing held: no wait
  // concurrent gets of the same streams agree
  mq::SchedSlots<Fake> many(64, 64);
  std::vector<FakeObj*> st;
  for (int k = 0; k < 16; ++k) st.push_back(new FakeObj(0));
  std::vector<void*> seen[4];
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      for (int k = 0; k < 16; ++k) seen[t].push_back(many.get(0, st[(k + 5 * t) % 16]));
    });
  for (auto& x : th) x.join();
  std::set<void*> uniq;
  for (int k = 0; k < 16; ++k) {
    void* p = many.get(0, st[k]);
    CHECK(p);
    uniq.insert(p);
    for (int t = 0; t < 4; ++t) CHECK(seen[t][(k - 5 * t + 80) % 16] == p);
  }
  CHECK(uniq.size() == 16);
  for (auto* x : st) delete x;
  for (void* p : Fake::allocated) std::free(p);
  Fake::allocated.clear();
}

// side streams give their schedule slots back when their entry is evicted or released (ADVICE
// r04): a server that churns through more caller streams than there are slots keeps a bounded
// number of slots assigned, and a released side stream's slot is recycled, not leaked
static mq::SchedSlots<Fake>* g_churn_slots = nullptr;
static void churn_hook(FakeObj* side) { g_churn_slots->release(side); }

static void test_side_stream_slot_churn() {
  mq::SchedSlots<Fake> slots(1024, 64);
  g_churn_slots = &slots;
  std::vector<FakeObj*> kept;  // callers that never release their stream
  {
    mq::SideStreams<Fake, 2> ss(64, churn_hook);
    Devices::Guard g(1);
    for (int k = 0; k < 600; ++k) {  // 1200 side streams: more than the 1024 slots
      FakeObj* caller = new FakeObj(1);
      CHECK(slots.get(1, caller) != nullptr);  // the caller stream's own slot
      {
        auto f = ss.fork(1, caller, 2);
        CHECK(f);
        CHECK(slots.get(1, f.side(0)) != nullptr);  // e.g. the hot-key AES kernel's slot
        CHECK(slots.get(1, f.side(1)) != nullptr);
      }
      if (k % 3 == 0) {  // some callers release their stream explicitly, the rest are evicted
        slots.release(caller);
        ss.release(caller);
        delete caller;
      } else {
        kept.push_back(caller);
      }
      // at most 64 entries x 2 side streams, plus the callers that never released theirs
      CHECK(slots.assigned(1) <= 2 * 64 + kept.size());
    }
    CHECK(ss.size() == 64 && Fake::live_streams == 128);
  }
  // every side stream's slot came back: only the unreleased callers' own slots remain
  CHECK(slots.assigned(1) == kept.size() && kept.size() == 400);
  CHECK(Fake::live_streams == 0);
  for (FakeObj* c : kept) delete c;
  g_churn_slots = nullptr;
  for (void* p : Fake::allocated) std::free(p);
  Fake::allocated.clear();
}

int main() {
  test_per_thread_selection();
  test_guard();
  test_side_streams();
  test_concurrent_forks();
  test_sched_slots();
  test_side_stream_slot_churn();
  std::printf("runtime ok\n");
  return 0;
}
