// CPU test of libozec's pinned-block cache (ozone_amd/csrc/numa.cpp pinned_alloc / pinned_free) against a fake HIP
// runtime that counts registrations (tests/test_pinned_cache.py builds and runs it under TSan): a freed block stays
// registered and mapped and is handed out again, zeroed, to the next allocation of its placement that it fits without
// wasting more than half of itself; blocks never cross NUMA nodes; past the 4 GiB bound a freed block is really
// unregistered and unmapped; foreign and double frees are refused; concurrent alloc / free cycles never hand one block
// to two owners.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <set>
#include <thread>
#include <vector>

#include "../../ozone_amd/csrc/numa.hpp"

namespace {
std::atomic<int> g_registers{0}, g_unregisters{0};
std::mutex g_mu;
std::set<void *> g_registered;
}  // namespace

extern "C" {
hipError_t hipGetLastError(void) { return hipSuccess; }
// device d is on NUMA node d
hipError_t hipDeviceGetAttribute(int *v, hipDeviceAttribute_t, int device) {
  *v = device;
  return hipSuccess;
}
hipError_t hipDeviceGetPCIBusId(char *, int, int) { return hipErrorInvalidDevice; }
hipError_t hipHostRegister(void *p, size_t, unsigned int) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_registered.insert(p).second) return hipErrorHostMemoryAlreadyRegistered;
  ++g_registers;
  return hipSuccess;
}
hipError_t hipHostUnregister(void *p) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_registered.erase(p)) return hipErrorHostMemoryNotRegistered;
  ++g_unregisters;
  return hipSuccess;
}
hipError_t hipPointerGetAttribute(void *, hipPointer_attribute, hipDeviceptr_t) { return hipErrorInvalidValue; }
}

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

int main() {
  using ozec::pinned_alloc;
  using ozec::pinned_free;
  constexpr size_t MiB = size_t{1} << 20;
  // 1. a freed block is reused, zeroed, without another registration
  void *a = nullptr;
  CHECK(pinned_alloc(5 * MiB, 0, &a) == 0 && a);  // 6 MiB mapped (2 MiB pages)
  CHECK(g_registers == 1);
  std::memset(a, 0x5A, 5 * MiB);
  CHECK(pinned_free(a) == 0);
  CHECK(g_unregisters == 0);
  void *b = nullptr;
  CHECK(pinned_alloc(5 * MiB, 0, &b) == 0 && b == a);
  CHECK(g_registers == 1);
  for (size_t i = 0; i < 5 * MiB; i += 4093) CHECK(static_cast<unsigned char *>(b)[i] == 0);
  // 2. a block more than twice the request is not handed out; another node's block is not either
  CHECK(pinned_free(b) == 0);  // cached: 6 MiB on node 0
  void *c = nullptr;
  CHECK(pinned_alloc(1 * MiB, 0, &c) == 0 && c != a);  // a 2 MiB mapping: the 6 MiB block would waste more than half
  void *d = nullptr;
  CHECK(pinned_alloc(5 * MiB, 1, &d) == 0 && d != a);  // node 1
  void *e = nullptr;
  CHECK(pinned_alloc(6 * MiB, 0, &e) == 0 && e == a);  // fits exactly
  CHECK(g_registers == 3);
  // 3. foreign and double frees are refused
  int x = 0;
  CHECK(pinned_free(&x) == -EINVAL);
  CHECK(pinned_free(e) == 0);
  CHECK(pinned_free(e) == -EINVAL);
  CHECK(pinned_free(c) == 0 && pinned_free(d) == 0);
  CHECK(g_unregisters == 0);
  // 4. past the 4 GiB bound a freed block is unregistered and unmapped (MAP_NORESERVE: untouched pages cost nothing)
  std::vector<void *> big(3);
  for (auto &p : big) CHECK(pinned_alloc(size_t{1800} * MiB, 2, &p) == 0 && p);
  for (auto &p : big) CHECK(pinned_free(p) == 0);
  CHECK(g_unregisters == 1);
  // 5. concurrent cycles from 8 threads: a block is owned by one thread at a time
  std::mutex own_mu;
  std::set<void *> owned;
  std::atomic<bool> clash{false};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&, t] {
      for (int i = 0; i < 200; ++i) {
        void *p = nullptr;
        if (pinned_alloc(static_cast<size_t>(1 + (i + t) % 3) * MiB, t % 2, &p) != 0 || !p) {
          clash = true;
          return;
        }
        {
          std::lock_guard<std::mutex> lk(own_mu);
          if (!owned.insert(p).second) clash = true;
        }
        static_cast<volatile unsigned char *>(p)[0] = static_cast<unsigned char>(t);
        {
          std::lock_guard<std::mutex> lk(own_mu);
          owned.erase(p);
        }
        if (pinned_free(p) != 0) clash = true;
      }
    });
  for (auto &t : ts) t.join();
  CHECK(!clash);
  std::printf("pinned cache OK (%d registrations, %d unregistrations)\n", g_registers.load(), g_unregisters.load());
  return 0;
}
