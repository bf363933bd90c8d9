#include "numa.hpp"

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
#include <string>
#include <algorithm>
#include <atomic>
#include <deque>
#include <unordered_map>
#include <vector>

namespace ozec {
namespace {

// <linux/mempolicy.h> constants (the image has no libnuma dependency in libozec)
constexpr int kMpolPreferred = 1;
constexpr unsigned kMpolMfMove = 1u << 1;
constexpr int kMpolFNode = 1 << 0;
constexpr int kMpolFAddr = 1 << 1;
constexpr size_t kMaxNodes = 1024;
constexpr size_t kHuge = 2u << 20;

std::mutex g_mu;
std::unordered_map<void *, size_t> g_allocs;  // pinned_alloc'ed regions -> mapped length
// Retired address ranges of freed pinned blocks ("GPU faults").  A freed block is unregistered at once and its
// pages go back to the kernel, but its address range does not come back into use: it is replaced by an inaccessible
// mapping (PROT_NONE, mmap MAP_FIXED over the block, so the range is never unmapped in between) and no later block,
// libozec's or anyone's, is placed there.  Nothing libozec registered with HIP is therefore ever registered again at the
// same address, nor handed out by the kernel as a caller's pageable buffer, while the runtime might still hold state for
// it.  The retired ranges are returned to the kernel oldest first only past kRetiredMax ranges or kRetiredBytes of
// address space (bounded VMAs and VA for a process that allocates and frees pinned memory for months).
struct Range {
  uint8_t *p;
  size_t len;
};
std::deque<Range> g_retired;  // guarded by g_mu, oldest first
size_t g_retired_bytes = 0;   // guarded by g_mu
std::atomic<uint64_t> g_unregister_failures{0};
constexpr size_t kRetiredMax = 4096;
constexpr size_t kRetiredBytes = size_t{4} << 40;  // 4 TiB of address space, no memory behind it
constexpr int kRw = PROT_READ | PROT_WRITE;
constexpr int kAnon = MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE;

// retire a block's range (its pages are released by the PROT_NONE mapping); munmap when the kernel refuses
void retire(void *p, size_t len) {
  if (mmap(p, len, PROT_NONE, kAnon | MAP_FIXED, -1, 0) == MAP_FAILED) {
    munmap(p, len);
    return;
  }
  std::vector<Range> release;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_retired.push_back({static_cast<uint8_t *>(p), len});
    g_retired_bytes += len;
    while (g_retired.size() > kRetiredMax || g_retired_bytes > kRetiredBytes) {
      release.push_back(g_retired.front());
      g_retired_bytes -= g_retired.front().len;
      g_retired.pop_front();
    }
  }
  for (const Range &r : release) munmap(r.p, r.len);
}

size_t page_size() {
  static const size_t ps = static_cast<size_t>(sysconf(_SC_PAGESIZE));
  return ps;
}

bool read_file(const std::string &path, std::string &out) {
  std::ifstream f(path);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

// "0-63,128-191" -> cpu ids
bool parse_cpulist(const std::string &s, cpu_set_t *set) {
  CPU_ZERO(set);
  size_t i = 0;
  bool any = false;
  while (i < s.size()) {
    while (i < s.size() && !std::isdigit(static_cast<unsigned char>(s[i]))) ++i;
    if (i >= s.size()) break;
    size_t j = i;
    while (j < s.size() && std::isdigit(static_cast<unsigned char>(s[j]))) ++j;
    long lo = std::stol(s.substr(i, j - i)), hi = lo;
    if (j < s.size() && s[j] == '-') {
      size_t k = j + 1;
      while (k < s.size() && std::isdigit(static_cast<unsigned char>(s[k]))) ++k;
      hi = std::stol(s.substr(j + 1, k - j - 1));
      j = k;
    }
    for (long c = lo; c <= hi && c < CPU_SETSIZE; ++c) {
      CPU_SET(static_cast<int>(c), set);
      any = true;
    }
    i = j;
  }
  return any;
}

}  // namespace

int device_numa_node(int device) {
  int v = -1;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeHostNumaId, device) == hipSuccess && v >= 0) return v;
  (void)hipGetLastError();
  char bus[64] = {};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  std::string id(bus);
  for (auto &c : id) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  std::string s;
  if (!read_file("/sys/bus/pci/devices/" + id + "/numa_node", s)) return -1;
  try {
    return std::stoi(s);
  } catch (...) {
    return -1;
  }
}

int bind_to_node(void *p, size_t bytes, int node, bool move, bool inner) {
  if (node < 0 || !p || bytes == 0) return 0;
  if (static_cast<size_t>(node) >= kMaxNodes) return -EINVAL;
  // test hook (tests/test_gpu_e2e.py): placement fails as it does under a seccomp profile without CAP_SYS_NICE
  static const bool fail = std::getenv("OZEC_TEST_FAIL_MBIND") != nullptr;
  if (fail) return -EPERM;
  const size_t ps = page_size();
  const uintptr_t a = reinterpret_cast<uintptr_t>(p), b = a + bytes;
  // inner: only the pages wholly inside [p, p + bytes) -- never the neighbours' data on a shared first/last page
  const uintptr_t lo = inner ? (a + ps - 1) / ps * ps : a / ps * ps;
  const uintptr_t hi = inner ? b / ps * ps : (b + ps - 1) / ps * ps;
  if (hi <= lo) return 0;
  unsigned long mask[kMaxNodes / (8 * sizeof(unsigned long))] = {};
  mask[node / (8 * sizeof(unsigned long))] = 1ul << (node % (8 * sizeof(unsigned long)));
  long rc = syscall(SYS_mbind, lo, hi - lo, kMpolPreferred, mask, kMaxNodes, move ? kMpolMfMove : 0u);
  return rc == 0 ? 0 : -errno;
}

int page_node(const void *p) {
  int node = -1;
  long rc = syscall(SYS_get_mempolicy, &node, nullptr, 0ul, p, kMpolFNode | kMpolFAddr);
  return rc == 0 ? node : -1;
}

int pinned_alloc(size_t bytes, int device, void **out) {
  *out = nullptr;
  if (bytes == 0) return 0;
  const size_t len = (bytes + kHuge - 1) / kHuge * kHuge;
  const int node = device >= 0 ? device_numa_node(device) : -1;
  void *p = mmap(nullptr, len, kRw, kAnon, -1, 0);  // always a fresh range (retired ones are never reused)
  if (p == MAP_FAILED) return -ENOMEM;
  (void)madvise(p, len, MADV_HUGEPAGE);  // fewer translations per DMA; best effort
  // placement first (pages are allocated on the first touch, which hipHostRegister does while pinning)
  (void)bind_to_node(p, len, node, false, false);
  if (hipHostRegister(p, len, hipHostRegisterPortable) != hipSuccess) {
    (void)hipGetLastError();
    munmap(p, len);  // never registered: nothing can refer to it
    return -ENOMEM;
  }
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_allocs[p] = len;
  }
  *out = p;
  return 0;
}

int pinned_free(void *p) {
  if (!p) return 0;
  size_t len = 0;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_allocs.find(p);
    if (it == g_allocs.end()) return -EINVAL;
    len = it->second;
    g_allocs.erase(it);
  }
  // the callers have drained every stream that used the block (capi.cpp Slot / E2E, stripe_queue.cpp); hipHostUnregister
  // waits for the device besides.  If the runtime does not release the registration, the block is left exactly as it
  // is -- mapped, registered, its pages in place -- rather than changing pages HIP may still reach (a leak, counted).
  if (hipHostUnregister(p) != hipSuccess) {
    (void)hipGetLastError();
    g_unregister_failures.fetch_add(1, std::memory_order_relaxed);
    return -EBUSY;
  }
  retire(p, len);
  return 0;
}

size_t pinned_retired_bytes() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_retired_bytes;
}

uint64_t pinned_unregister_failures() { return g_unregister_failures.load(std::memory_order_relaxed); }

const void *pinned_alloc_base(const void *p) {
  void *base = nullptr;
  if (hipPointerGetAttribute(&base, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                             reinterpret_cast<hipDeviceptr_t>(const_cast<void *>(p))) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return base;
}

int bind_thread_to_node(int node) {
  if (node < 0) return 0;
  std::string s;
  if (!read_file("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", s)) return -ENOENT;
  cpu_set_t want, have, both;
  if (!parse_cpulist(s, &want)) return -EINVAL;
  if (sched_getaffinity(0, sizeof(have), &have) != 0) return -errno;
  CPU_AND(&both, &want, &have);
  if (CPU_COUNT(&both) == 0) return -EINVAL;  // the process may not run there: leave it alone
  return pthread_setaffinity_np(pthread_self(), sizeof(both), &both) == 0 ? 0 : -EINVAL;
}

}  // namespace ozec
