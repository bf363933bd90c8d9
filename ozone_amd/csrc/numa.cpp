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
// Freed pinned blocks are kept registered and mapped, and handed out again, instead of being unregistered and
// unmapped: a host address range that was registered, unregistered and unmapped can come back from the kernel for an
// unrelated pageable buffer, and HIP's pageable-copy path is suspected of faulting on such ranges ("GPU
// faults").  Per NUMA node of the placement; bounded, past the bound a block is really freed.
struct Cached {
  void *p;
  size_t len;
  int node;
};
std::vector<Cached> g_cache;
std::unordered_map<void *, int> g_nodes;  // pinned_alloc'ed regions -> NUMA node of their placement
size_t g_cached = 0;
constexpr size_t kCacheCap = size_t{4} << 30;

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
  void *hit = nullptr;
  {  // the smallest cached block of this placement that fits, if it wastes at most half of itself
    std::lock_guard<std::mutex> lk(g_mu);
    size_t best = g_cache.size();
    for (size_t i = 0; i < g_cache.size(); ++i)
      if (g_cache[i].node == node && g_cache[i].len >= len && g_cache[i].len <= 2 * len &&
          (best == g_cache.size() || g_cache[i].len < g_cache[best].len))
        best = i;
    if (best < g_cache.size()) {
      const Cached c = g_cache[best];
      g_cache.erase(g_cache.begin() + static_cast<std::ptrdiff_t>(best));
      g_cached -= c.len;
      g_allocs[c.p] = c.len;
      g_nodes[c.p] = node;
      hit = c.p;
    }
  }
  if (hit) {
    std::memset(hit, 0, bytes);  // as a fresh mapping
    *out = hit;
    return 0;
  }
  void *p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (p == MAP_FAILED) return -ENOMEM;
  (void)madvise(p, len, MADV_HUGEPAGE);  // fewer translations per DMA; best effort
  // placement first (pages are allocated on the first touch, which hipHostRegister does while pinning)
  (void)bind_to_node(p, len, node, false, false);
  if (hipHostRegister(p, len, hipHostRegisterPortable) != hipSuccess) {
    (void)hipGetLastError();
    munmap(p, len);
    return -ENOMEM;
  }
  {
    std::lock_guard<std::mutex> lk(g_mu);
    g_allocs[p] = len;
    g_nodes[p] = node;
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
    const int node = g_nodes[p];
    g_nodes.erase(p);
    if (g_cached + len <= kCacheCap) {
      g_cache.push_back({p, len, node});
      g_cached += len;
      return 0;
    }
  }
  (void)hipHostUnregister(p);
  munmap(p, len);
  return 0;
}

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
