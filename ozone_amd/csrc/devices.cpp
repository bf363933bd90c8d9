#include "devices.hpp"

#include <hip/hip_runtime.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/ozec.h"
#include "numa.hpp"

namespace ozec {
namespace {

std::mutex g_mu;
bool g_init = false;
std::vector<int> g_list;             // guarded by g_mu
std::atomic<int> g_policy{-1};       // -1: read OZEC_DEVICE_POLICY on first use
std::atomic<unsigned> g_next{0};     // round-robin cursor of pick_device
std::atomic<unsigned> g_thread_next{0};
std::atomic<unsigned> g_gen{1};          // bumped by set_device_list (threads re-pick their device)
// whether the process chose its devices itself (ozec_set_devices, ozec_set_device_policy, OZEC_DEVICES,
// OZEC_DEVICE_POLICY): only a process that did not gets "current" from note_set_device
std::atomic<bool> g_configured{false};
// the "current" policy in force came from note_set_device, not from the process: a device list or policy chosen
// afterwards replaces it
std::atomic<bool> g_implicit_current{false};

int visible() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

// OZEC_DEVICES: "all" / unset = every visible device, else a comma list of ordinals (invalid entries are skipped)
std::vector<int> default_list(int n) {
  std::vector<int> out;
  const char *e = std::getenv("OZEC_DEVICES");
  if (e && *e && std::strcmp(e, "all") != 0) {
    std::string s(e);
    size_t pos = 0;
    while (pos <= s.size()) {
      size_t c = s.find(',', pos);
      if (c == std::string::npos) c = s.size();
      const std::string tok = s.substr(pos, c - pos);
      char *end = nullptr;
      const long v = std::strtol(tok.c_str(), &end, 10);
      if (!tok.empty() && end && *end == '\0' && v >= 0 && v < n) out.push_back(static_cast<int>(v));
      pos = c + 1;
    }
  }
  if (out.empty())
    for (int d = 0; d < n; ++d) out.push_back(d);
  return out;
}

void ensure_init() {  // caller holds g_mu
  if (g_init) return;
  g_list = default_list(visible());
  g_init = true;
}

bool env_set(const char *name) {
  const char *e = std::getenv(name);
  return e && *e;
}

int caller_node() {
  unsigned cpu = 0, node = 0;
  if (syscall(SYS_getcpu, &cpu, &node, nullptr) != 0) return -1;
  return static_cast<int>(node);
}

// the listed devices a NUMA-policy caller on `node` prefers: those on its node, or all when none is
std::vector<int> near_or_all(const std::vector<int> &list, int node) {
  std::vector<int> near;
  for (int d : list)
    if (node >= 0 && device_numa_node(d) == node) near.push_back(d);
  return near.empty() ? list : near;
}

}  // namespace

std::vector<int> device_list() {
  std::lock_guard<std::mutex> lk(g_mu);
  ensure_init();
  return g_list;
}

int set_device_list(const int *devs, int n) {
  const int vis = visible();
  if (n < 0 || (n > 0 && !devs)) return OZEC_EINVAL;
  for (int i = 0; i < n; ++i)
    if (devs[i] < 0 || devs[i] >= vis) return OZEC_EDEVICE;
  std::lock_guard<std::mutex> lk(g_mu);
  g_list = n > 0 ? std::vector<int>(devs, devs + n) : default_list(vis);
  g_init = true;
  g_configured.store(true, std::memory_order_relaxed);
  if (g_implicit_current.exchange(false)) g_policy.store(-1, std::memory_order_relaxed);  // the default again
  g_gen.fetch_add(1, std::memory_order_release);
  return OZEC_OK;
}

int device_policy() {
  int p = g_policy.load(std::memory_order_relaxed);
  if (p < 0) {
    const char *e = std::getenv("OZEC_DEVICE_POLICY");
    p = e && !std::strcmp(e, "numa") ? 1 : e && !std::strcmp(e, "current") ? 2 : 0;
    g_policy.store(p, std::memory_order_relaxed);
  }
  return p;
}

int set_device_policy(int policy) {
  if (policy < 0 || policy > 2) return OZEC_EINVAL;
  g_policy.store(policy, std::memory_order_relaxed);
  g_configured.store(true, std::memory_order_relaxed);
  g_implicit_current.store(false);
  return OZEC_OK;
}

bool note_set_device() {
  if (g_configured.load(std::memory_order_relaxed) || env_set("OZEC_DEVICES") || env_set("OZEC_DEVICE_POLICY"))
    return false;
  g_policy.store(2, std::memory_order_relaxed);
  g_implicit_current.store(true);
  return true;
}

int pick_device() {
  const int policy = device_policy();
  if (policy == 2) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
      (void)hipGetLastError();
      return -1;
    }
    return dev;
  }
  const std::vector<int> list = device_list();
  if (list.empty()) return -1;
  // NUMA policy: the listed GPUs on the caller's NUMA node, round robin; all of them when none is
  const std::vector<int> cand = policy == 1 ? near_or_all(list, caller_node()) : list;
  return cand[g_next.fetch_add(1, std::memory_order_relaxed) % cand.size()];
}


int thread_device() {
  if (device_policy() == 2) {  // follows the thread's current device, call by call
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) {
      (void)hipGetLastError();
      return -1;
    }
    return d;
  }
  thread_local int dev = -1;
  thread_local unsigned gen = 0;
  const unsigned now = g_gen.load(std::memory_order_acquire);
  if (dev < 0 || gen != now) {  // first call, or the list changed since this thread was given its device
    const std::vector<int> list = device_list();
    if (list.empty()) return -1;
    const std::vector<int> cand = device_policy() == 1 ? near_or_all(list, caller_node()) : list;
    dev = cand[g_thread_next.fetch_add(1, std::memory_order_relaxed) % cand.size()];
    gen = now;
  }
  return dev;
}

size_t split_parts(size_t num_stripes, size_t chunk, size_t ndev) {
  const size_t whole_chunks = num_stripes / (chunk ? chunk : 1);
  size_t parts = ndev < whole_chunks ? ndev : whole_chunks;
  return parts ? parts : 1;
}

void part_range(size_t num_stripes, size_t parts, size_t i, size_t *s0, size_t *s1) {
  const size_t per = (num_stripes + parts - 1) / parts;
  *s0 = i * per < num_stripes ? i * per : num_stripes;
  *s1 = (i + 1) * per < num_stripes ? (i + 1) * per : num_stripes;
}

DeviceScope::DeviceScope(int dev) {
  if (dev < 0) return;
  if (hipGetDevice(&prev_) != hipSuccess) {
    (void)hipGetLastError();
    ok_ = false;
    return;
  }
  if (prev_ == dev) return;
  if (hipSetDevice(dev) != hipSuccess) {
    (void)hipGetLastError();
    ok_ = false;
    return;
  }
  switched_ = true;
}

DeviceScope::~DeviceScope() {
  if (switched_) (void)hipSetDevice(prev_);
}

}  // namespace ozec
