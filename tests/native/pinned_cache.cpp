// CPU test of libozec's pinned blocks (ozone_amd/csrc/numa.cpp pinned_alloc / pinned_free) against a fake HIP runtime
// that counts registrations (tests/test_pinned_cache.py builds and runs it under TSan): a freed block is unregistered
// at once and its pages returned, and its address range is retired -- mapped PROT_NONE in /proc/self/maps and never
// used for a later block, so nothing libozec registered is registered again at the same address; a refused
// registration unmaps its fresh range; a refused unregistration leaves the block untouched and is counted; the retired
// address space is bounded; foreign and double frees are refused; concurrent alloc / free cycles never hand one block
// to two owners.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../ozone_amd/csrc/numa.hpp"

namespace {
std::atomic<int> g_registers{0}, g_unregisters{0};
std::atomic<bool> g_refuse{false}, g_refuse_unregister{false};
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
  if (g_refuse) return hipErrorHostMemoryAlreadyRegistered;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_registered.insert(p).second) return hipErrorHostMemoryAlreadyRegistered;
  ++g_registers;
  return hipSuccess;
}
hipError_t hipHostUnregister(void *p) {
  if (g_refuse_unregister) return hipErrorUnknown;
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

// the protection of the mapping holding [p, p + len) in /proc/self/maps ("rw-p", "---p"), "" when unmapped
static std::string prot_of(const void *p, size_t len) {
  std::ifstream f("/proc/self/maps");
  std::string line;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = a + len;
  while (std::getline(f, line)) {
    std::istringstream ls(line);
    std::string range, prot;
    ls >> range >> prot;
    const size_t dash = range.find('-');
    const uintptr_t lo = std::stoull(range.substr(0, dash), nullptr, 16), hi = std::stoull(range.substr(dash + 1), nullptr, 16);
    if (lo <= a && b <= hi) return prot;
  }
  return "";
}

int main() {
  using ozec::pinned_alloc;
  using ozec::pinned_free;
  constexpr size_t MiB = size_t{1} << 20;
  // 1. a freed block is unregistered and its range retired (inaccessible, still mapped); the next block of that size
  //    is a fresh range, never the retired one
  void *a = nullptr;
  CHECK(pinned_alloc(5 * MiB, 0, &a) == 0 && a);  // 6 MiB mapped (2 MiB pages)
  CHECK(g_registers == 1 && prot_of(a, 6 * MiB) == "rw-p");
  std::memset(a, 0x5A, 5 * MiB);
  CHECK(pinned_free(a) == 0);
  CHECK(g_unregisters == 1);
  CHECK(prot_of(a, 6 * MiB) == "---p");
  CHECK(ozec::pinned_retired_bytes() == 6 * MiB);
  void *b = nullptr;
  CHECK(pinned_alloc(5 * MiB, 0, &b) == 0 && b && b != a);
  CHECK(g_registers == 2 && prot_of(b, 6 * MiB) == "rw-p" && prot_of(a, 6 * MiB) == "---p");
  for (size_t i = 0; i < 5 * MiB; i += 4093) CHECK(static_cast<unsigned char *>(b)[i] == 0);
  // 2. no later block overlaps any retired range, whatever its size
  std::vector<std::pair<uintptr_t, uintptr_t>> retired = {{reinterpret_cast<uintptr_t>(a), reinterpret_cast<uintptr_t>(a) + 6 * MiB}};
  CHECK(pinned_free(b) == 0);
  retired.push_back({reinterpret_cast<uintptr_t>(b), reinterpret_cast<uintptr_t>(b) + 6 * MiB});
  for (size_t n : {size_t{1}, size_t{2}, size_t{6}, size_t{64}}) {
    void *c = nullptr;
    CHECK(pinned_alloc(n * MiB, 1, &c) == 0 && c);
    const uintptr_t lo = reinterpret_cast<uintptr_t>(c), hi = lo + n * MiB;
    for (const auto &r : retired) CHECK(hi <= r.first || lo >= r.second);
    CHECK(pinned_free(c) == 0);
    retired.push_back({lo, lo + (n * MiB + 2 * MiB - 1) / (2 * MiB) * (2 * MiB)});
  }
  CHECK(ozec::pinned_retired_bytes() == (6 + 6 + 2 + 2 + 6 + 64) * MiB);
  // 3. foreign and double frees are refused
  void *e = nullptr;
  CHECK(pinned_alloc(8 * MiB, 0, &e) == 0 && e);
  int x = 0;
  CHECK(pinned_free(&x) == -EINVAL);
  CHECK(pinned_free(e) == 0);
  CHECK(pinned_free(e) == -EINVAL);
  CHECK(prot_of(e, 8 * MiB) == "---p");
  // 4. a refused registration: the allocation fails and its fresh range is unmapped (it was never registered)
  g_refuse = true;
  void *f = nullptr;
  CHECK(pinned_alloc(2 * MiB, 0, &f) == -ENOMEM && f == nullptr);
  g_refuse = false;
  // 5. an unregistration the runtime refuses: the block stays exactly as it was (mapped, its bytes in place), the
  //    free reports -EBUSY and is counted
  void *g = nullptr;
  CHECK(pinned_alloc(2 * MiB, 0, &g) == 0 && g);
  std::memset(g, 0x77, 2 * MiB);
  g_refuse_unregister = true;
  CHECK(pinned_free(g) == -EBUSY && ozec::pinned_unregister_failures() == 1);
  g_refuse_unregister = false;
  CHECK(prot_of(g, 2 * MiB) == "rw-p" && static_cast<unsigned char *>(g)[2 * MiB - 1] == 0x77);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    CHECK(g_registered.count(g) == 1);
    g_registered.erase(g);  // the fake runtime forgets it: the leak is the test's now
    ++g_unregisters;
  }
  // 6. the retired address space is bounded: past 4096 ranges the oldest go back to the kernel
  const size_t before = ozec::pinned_retired_bytes();
  for (int i = 0; i < 4200; ++i) {
    void *p = nullptr;
    CHECK(pinned_alloc(4096, 0, &p) == 0 && p);
    CHECK(pinned_free(p) == 0);
  }
  CHECK(ozec::pinned_retired_bytes() <= 4096 * 2 * MiB && ozec::pinned_retired_bytes() < before + 4200 * 2 * MiB);
  // 6. concurrent cycles from 8 threads: a block is owned by one thread at a time, every byte of it writable
  std::mutex own_mu;
  std::set<void *> owned;
  std::atomic<bool> clash{false};
  std::vector<std::thread> ts;
  for (int t = 0; t < 8; ++t)
    ts.emplace_back([&, t] {
      for (int i = 0; i < 100; ++i) {
        void *p = nullptr;
        const size_t n = static_cast<size_t>(1 + (i + t) % 3) * MiB;
        if (pinned_alloc(n, t % 2, &p) != 0 || !p) {
          clash = true;
          return;
        }
        {
          std::lock_guard<std::mutex> lk(own_mu);
          if (!owned.insert(p).second) clash = true;
        }
        static_cast<volatile unsigned char *>(p)[0] = static_cast<unsigned char>(t);
        static_cast<volatile unsigned char *>(p)[n - 1] = static_cast<unsigned char>(t);
        {
          std::lock_guard<std::mutex> lk(own_mu);
          owned.erase(p);
        }
        if (pinned_free(p) != 0) clash = true;
      }
    });
  for (auto &t : ts) t.join();
  CHECK(!clash);
  CHECK(g_registers == g_unregisters);  // nothing left registered
  std::printf("pinned blocks OK (%d registrations, %d unregistrations, %zu MiB retired)\n", g_registers.load(),
              g_unregisters.load(), ozec::pinned_retired_bytes() >> 20);
  return 0;
}
