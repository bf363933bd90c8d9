// Counter-slot pool of the persistent kernels' WorkQueue (kernels.hpp work_lease / work_return; device.hpp WorkQueue).
// Host code only: tests/native/work_slots.cpp runs it against a fake HIP runtime (tests/test_work_slots.py).
#include <hip/hip_runtime.h>

#include <mutex>
#include <new>
#include <vector>

#include "kernels.hpp"

namespace ozec {

// A launch leases a zeroed slot and hands it back behind an event recorded after the kernel on the launch stream; the
// slot is leased again only once that event has completed, i.e. once the kernel's last wave has put the counters back
// to zero.  Slots are not tied to a stream handle, so concurrent launches never share one, whatever the stream (the null
// stream, hipStreamPerThread, several streams of one caller).  A capturing stream gets no slot: its launches take the
// non-persistent form.
namespace {
std::mutex g_ws_mu;
std::vector<WorkSlot *> g_ws;  // never freed: a handful per device and process
constexpr size_t kMaxWorkSlots = 256;
}  // namespace

WorkSlot *work_lease(hipStream_t st) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) {
    (void)hipGetLastError();
    return nullptr;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_ws_mu);
  for (WorkSlot *w : g_ws) {
    if (w->device != dev || w->leased) continue;
    if (w->recorded) {
      const hipError_t q = hipEventQuery(w->done);
      (void)hipGetLastError();  // hipErrorNotReady must not reach the launch's error check
      if (q != hipSuccess) continue;
    }
    w->leased = true;
    return w;
  }
  if (g_ws.size() >= kMaxWorkSlots) return nullptr;
  auto *w = new (std::nothrow) WorkSlot();
  if (!w) return nullptr;
  w->device = dev;
  void *p = nullptr;
  if (hipMalloc(&p, kWqInts * sizeof(int32_t)) != hipSuccess) {
    (void)hipGetLastError();
    delete w;
    return nullptr;
  }
  // the zeroing is ordered before this launch by the stream, and before a launch on any other stream by the event
  // (a launch that does not count on the slot hands it back without recording one)
  if (hipMemsetAsync(p, 0, kWqInts * sizeof(int32_t), st) != hipSuccess ||
      hipEventCreateWithFlags(&w->done, hipEventDisableTiming) != hipSuccess ||
      hipEventRecord(w->done, st) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipStreamSynchronize(st);
    if (w->done) (void)hipEventDestroy(w->done);
    (void)hipFree(p);
    delete w;
    return nullptr;
  }
  w->ctr = static_cast<int32_t *>(p);
  w->recorded = true;
  w->leased = true;
  g_ws.push_back(w);
  return w;
}

// give the slot back; `used`: a kernel that counts on it was enqueued on `st`
void work_return(WorkSlot *w, hipStream_t st, bool used) {
  if (used) {
    if (hipEventRecord(w->done, st) == hipSuccess) {
      w->recorded = true;
    } else {
      (void)hipGetLastError();
      (void)hipStreamSynchronize(st);  // no event: make sure the kernel is done before anyone else counts on the slot
    }
  }
  std::lock_guard<std::mutex> lk(g_ws_mu);
  w->leased = false;
}

}  // namespace ozec
