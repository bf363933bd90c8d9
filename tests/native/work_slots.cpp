// CPU test of the WorkQueue counter-slot pool of the persistent fused kernels (ozone_amd/csrc/work_slots.cpp) against
// a fake HIP runtime whose events complete only when the test says so (tests/test_work_slots.py builds and runs it):
// a slot is never handed to a second launch while the event behind its last use (or behind its zeroing) is pending,
// it is reused once that event completes, slots never cross devices, capturing streams get none, the pool is bounded,
// a failed event record falls back to draining the stream, and concurrent lease/return cycles from many threads never
// share a slot.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "../../ozone_amd/csrc/kernels.hpp"

namespace {
struct FakeEvent {
  bool pending = false;
  hipStream_t stream = nullptr;
};
std::mutex g_mu;
std::set<FakeEvent *> g_events;
thread_local int g_dev = 0;
std::atomic<int> g_mallocs{0}, g_memsets{0}, g_syncs{0};
std::atomic<bool> g_fail_record{false};
const hipStream_t kCapturing = reinterpret_cast<hipStream_t>(0xCA);

void complete_all() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (FakeEvent *e : g_events) e->pending = false;
}
}  // namespace

extern "C" {
hipError_t hipStreamIsCapturing(hipStream_t st, hipStreamCaptureStatus *cap) {
  *cap = st == kCapturing ? hipStreamCaptureStatusActive : hipStreamCaptureStatusNone;
  return hipSuccess;
}
hipError_t hipGetDevice(int *d) {
  *d = g_dev;
  return hipSuccess;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
hipError_t hipMalloc(void **p, size_t n) {
  *p = std::malloc(n);
  ++g_mallocs;
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void *p) {
  std::free(p);
  return hipSuccess;
}
hipError_t hipMemsetAsync(void *p, int v, size_t n, hipStream_t) {
  std::memset(p, v, n);
  ++g_memsets;
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t *e, unsigned) {
  auto *f = new FakeEvent();
  std::lock_guard<std::mutex> lk(g_mu);
  g_events.insert(f);
  *e = reinterpret_cast<hipEvent_t>(f);
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
  auto *f = reinterpret_cast<FakeEvent *>(e);
  std::lock_guard<std::mutex> lk(g_mu);
  g_events.erase(f);
  delete f;
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t st) {
  if (g_fail_record.load()) return hipErrorInvalidHandle;
  auto *f = reinterpret_cast<FakeEvent *>(e);
  std::lock_guard<std::mutex> lk(g_mu);
  f->pending = true;
  f->stream = st;
  return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e) {
  auto *f = reinterpret_cast<FakeEvent *>(e);
  std::lock_guard<std::mutex> lk(g_mu);
  return f->pending ? hipErrorNotReady : hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t st) {
  ++g_syncs;
  std::lock_guard<std::mutex> lk(g_mu);
  for (FakeEvent *f : g_events)
    if (f->stream == st) f->pending = false;
  return hipSuccess;
}
}

static int failures = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                         \
    }                                                                     \
  } while (0)

static bool zeroed(const ozec::WorkSlot *w) {
  for (int i = 0; i < ozec::kWqInts; ++i)
    if (w->ctr[i] != 0) return false;
  return true;
}

int main() {
  using ozec::WorkSlot;
  const hipStream_t sa = reinterpret_cast<hipStream_t>(0x10), sb = reinterpret_cast<hipStream_t>(0x20);
  // a new slot is zeroed on the launch stream, and its zeroing gates every other lease
  WorkSlot *w1 = ozec::work_lease(sa);
  CHECK(w1 && w1->device == 0 && w1->leased && zeroed(w1) && g_memsets == 1);
  ozec::work_return(w1, sa, false);  // not used (a non-persistent variant): the zeroing event is still pending
  WorkSlot *w2 = ozec::work_lease(sb);
  CHECK(w2 && w2 != w1);
  // a used slot comes back only after the event recorded behind its kernel completes
  ozec::work_return(w2, sb, true);
  WorkSlot *w3 = ozec::work_lease(sa);
  CHECK(w3 && w3 != w1 && w3 != w2);
  ozec::work_return(w3, sa, true);
  complete_all();
  WorkSlot *r1 = ozec::work_lease(sb);
  CHECK(r1 == w1 || r1 == w2 || r1 == w3);  // reused, no new allocation
  CHECK(g_mallocs == 3);
  // a leased slot is never handed out again, whatever its event says
  WorkSlot *r2 = ozec::work_lease(sb);
  CHECK(r2 && r2 != r1);
  ozec::work_return(r1, sb, true);
  ozec::work_return(r2, sb, true);
  // capturing streams get no slot
  CHECK(ozec::work_lease(kCapturing) == nullptr);
  // slots never cross devices
  complete_all();
  std::thread([&] {
    g_dev = 1;
    WorkSlot *d1 = ozec::work_lease(sa);
    CHECK(d1 && d1->device == 1 && d1 != w1 && d1 != w2 && d1 != w3);
    ozec::work_return(d1, sa, true);
  }).join();
  // a failed event record drains the launch stream instead (the slot is then free at once)
  complete_all();
  WorkSlot *f1 = ozec::work_lease(sa);
  g_fail_record = true;
  const int syncs = g_syncs;
  ozec::work_return(f1, sa, true);
  g_fail_record = false;
  CHECK(g_syncs == syncs + 1);
  // concurrent lease / return cycles: no slot is ever leased twice at once
  std::mutex inuse_mu;
  std::set<WorkSlot *> inuse;
  std::atomic<int> shared{0}, got{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&, t] {
      const hipStream_t st = reinterpret_cast<hipStream_t>(static_cast<uintptr_t>(0x100 + t));
      for (int i = 0; i < 2000; ++i) {
        WorkSlot *w = ozec::work_lease(st);
        if (!w) continue;
        ++got;
        {
          std::lock_guard<std::mutex> lk(inuse_mu);
          if (!inuse.insert(w).second) ++shared;
        }
        {
          std::lock_guard<std::mutex> lk(inuse_mu);
          inuse.erase(w);
        }
        ozec::work_return(w, st, true);
        if (i % 7 == 0) complete_all();
      }
    });
  for (auto &th : ts) th.join();
  CHECK(shared == 0 && got > 0);
  // bounded pool: with every event pending, leases stop at 256 slots per process
  std::vector<WorkSlot *> held;
  for (int i = 0; i < 400; ++i) {
    WorkSlot *w = ozec::work_lease(sa);
    if (!w) break;
    held.push_back(w);
  }
  CHECK(held.size() <= 256 && ozec::work_lease(sa) == nullptr);
  if (failures) return 1;
  std::printf("work slots OK (%d mallocs)\n", g_mallocs.load());
  return 0;
}
