// CPU test of libozec's pinned blocks (ozone_amd/csrc/numa.cpp pinned_alloc / pinned_free) against a fake HIP runtime
// that counts registrations (tests/test_pinned_cache.py builds and runs it under TSan): a freed block is unregistered
// at once and its pages returned, but its address range stays mapped as an inaccessible reservation (PROT_NONE in
// /proc/self/maps), so the kernel never hands a once-registered range out for a pageable buffer; later pinned blocks
// are carved from the reservations (fresh zero pages, registered again), adjacent reservations merge; a registration
// refused over a reused range leaves it reserved; foreign and double frees are refused; concurrent alloc / free
// cycles never hand one block to two owners.
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
std::atomic<bool> g_refuse{false};
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
  // 1. a freed block is unregistered and its range reserved (inaccessible, still mapped); the next block of that size
  //    is carved from it with fresh zero pages and registered again
  void *a = nullptr;
  CHECK(pinned_alloc(5 * MiB, 0, &a) == 0 && a);  // 6 MiB mapped (2 MiB pages)
  CHECK(g_registers == 1 && prot_of(a, 6 * MiB) == "rw-p");
  std::memset(a, 0x5A, 5 * MiB);
  CHECK(pinned_free(a) == 0);
  CHECK(g_unregisters == 1);
  CHECK(prot_of(a, 6 * MiB) == "---p");
  CHECK(ozec::pinned_reserved_bytes() == 6 * MiB);
  void *b = nullptr;
  CHECK(pinned_alloc(5 * MiB, 0, &b) == 0 && b == a);
  CHECK(g_registers == 2 && prot_of(b, 6 * MiB) == "rw-p" && ozec::pinned_reserved_bytes() == 0);
  for (size_t i = 0; i < 5 * MiB; i += 4093) CHECK(static_cast<unsigned char *>(b)[i] == 0);
  // 2. a smaller block is carved from the front of a reservation, the rest stays reserved; freeing it merges them again
  CHECK(pinned_free(b) == 0);
  void *c = nullptr;
  CHECK(pinned_alloc(1 * MiB, 1, &c) == 0 && c == a);  // 2 MiB of the 6 (placement does not matter for a range)
  CHECK(ozec::pinned_reserved_bytes() == 4 * MiB && prot_of(static_cast<uint8_t *>(a) + 2 * MiB, 4 * MiB) == "---p");
  CHECK(pinned_free(c) == 0 && ozec::pinned_reserved_bytes() == 6 * MiB);
  void *d = nullptr;
  CHECK(pinned_alloc(6 * MiB, 0, &d) == 0 && d == a);  // the merged range serves a whole-size block
  // 3. a block larger than every reservation is a fresh mapping
  void *e = nullptr;
  CHECK(pinned_alloc(64 * MiB, 0, &e) == 0 && e && e != a);
  // 4. foreign and double frees are refused
  int x = 0;
  CHECK(pinned_free(&x) == -EINVAL);
  CHECK(pinned_free(e) == 0);
  CHECK(pinned_free(e) == -EINVAL);
  CHECK(pinned_free(d) == 0);
  CHECK(prot_of(e, 64 * MiB) == "---p" && prot_of(d, 6 * MiB) == "---p");
  // 5. a registration refused over a reused range: the allocation fails and the range stays reserved
  const size_t before = ozec::pinned_reserved_bytes();
  g_refuse = true;
  void *f = nullptr;
  CHECK(pinned_alloc(2 * MiB, 0, &f) == -ENOMEM && f == nullptr);
  g_refuse = false;
  CHECK(ozec::pinned_reserved_bytes() == before);
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
  std::printf("pinned blocks OK (%d registrations, %d unregistrations, %zu MiB reserved)\n", g_registers.load(),
              g_unregisters.load(), ozec::pinned_reserved_bytes() >> 20);
  return 0;
}
