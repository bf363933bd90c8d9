// CPU test of the device list and device policies of libozec (ozone_amd/csrc/devices.cpp) against a fake HIP runtime
// of N devices (tests/test_devices.py builds and runs it): the default list, OZEC_DEVICES, ozec_set_devices with
// duplicates and bad ordinals, round-robin coder binding, the NUMA policy (devices on the caller's node first), the
// "current" policy, per-thread devices of coder-less calls (re-picked after the list changes), and DeviceScope
// restoring the caller's device.
#include <hip/hip_runtime.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <set>
#include <thread>
#include <vector>

#include "../../include/ozec.h"
#include "../../ozone_amd/csrc/devices.hpp"

static int g_count = 4, g_current = 0, g_sets = 0;
static int g_node_of[16];

extern "C" {
hipError_t hipGetDeviceCount(int *n) {
  *n = g_count;
  return hipSuccess;
}
hipError_t hipGetDevice(int *d) {
  *d = g_current;
  return hipSuccess;
}
hipError_t hipSetDevice(int d) {
  if (d < 0 || d >= g_count) return hipErrorInvalidDevice;
  g_current = d;
  ++g_sets;
  return hipSuccess;
}
hipError_t hipGetLastError(void) { return hipSuccess; }
}
namespace ozec {
int device_numa_node(int device) { return g_node_of[device]; }
}  // namespace ozec

static int failures = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                         \
    }                                                                     \
  } while (0)

int main(int argc, char **argv) {
  if (argc == 5 && !std::strcmp(argv[1], "parts")) {  // host-batch partition: "parts S chunk ndev" -> one "s0 s1" a line
    const size_t S = std::strtoull(argv[2], nullptr, 10), chunk = std::strtoull(argv[3], nullptr, 10);
    const size_t parts = ozec::split_parts(S, chunk, std::strtoull(argv[4], nullptr, 10));
    for (size_t i = 0; i < parts; ++i) {
      size_t s0 = 0, s1 = 0;
      ozec::part_range(S, parts, i, &s0, &s1);
      std::printf("%zu %zu\n", s0, s1);
    }
    return 0;
  }
  unsigned cpu = 0, node = 0;
  syscall(SYS_getcpu, &cpu, &node, nullptr);
  // devices 0, 1 on another node than the caller's; 2, 3 on the caller's
  g_node_of[0] = g_node_of[1] = static_cast<int>(node) + 1;
  g_node_of[2] = g_node_of[3] = static_cast<int>(node);

  const char *env = std::getenv("OZEC_DEVICES");
  std::vector<int> want = env ? std::vector<int>{3, 1} : std::vector<int>{0, 1, 2, 3};
  // a process that selects its GPU itself (ozec_set_device) and configured nothing gets the "current" policy; one that
  // chose a list (here OZEC_DEVICES) or a policy keeps it
  CHECK(ozec::note_set_device() == (env == nullptr));
  CHECK(ozec::device_policy() == (env ? 0 : 2));
  if (!env) {  // a device list chosen afterwards replaces that implicit "current" policy for every thread
    const int two[2] = {1, 2};
    CHECK(ozec::set_device_list(two, 2) == OZEC_OK && ozec::device_policy() == 0);
    std::set<int> picked;
    for (int i = 0; i < 4; ++i) picked.insert(ozec::pick_device());
    CHECK((picked == std::set<int>{1, 2}));
    CHECK(!ozec::note_set_device() && ozec::device_policy() == 0);  // configured now: later set_device calls leave it
    CHECK(ozec::set_device_list(nullptr, 0) == OZEC_OK);
  }
  CHECK(ozec::set_device_policy(0) == OZEC_OK);
  CHECK(!ozec::note_set_device() && ozec::device_policy() == 0);
  CHECK(ozec::device_list() == want);  // "3,x,1,9" -> invalid entries skipped
  if (env) {
    CHECK(ozec::set_device_list(nullptr, 0) == OZEC_OK);  // n = 0: the default again (the env list)
    CHECK(ozec::device_list() == want);
  }
  // round robin over the list, duplicates allowed
  const int dup[] = {2, 2, 0};
  CHECK(ozec::set_device_list(dup, 3) == OZEC_OK);
  CHECK(ozec::device_policy() == 0);
  std::vector<int> got;
  for (int i = 0; i < 6; ++i) got.push_back(ozec::pick_device());
  std::multiset<int> ms(got.begin(), got.end());
  CHECK(ms.count(2) == 4 && ms.count(0) == 2);
  for (int i = 0; i + 3 < 6; ++i) CHECK(got[i] == got[i + 3]);  // period = list length
  // bad lists are refused and change nothing
  const int bad[] = {0, 4};
  CHECK(ozec::set_device_list(bad, 2) == OZEC_EDEVICE);
  const int neg[] = {-1};
  CHECK(ozec::set_device_list(neg, 1) == OZEC_EDEVICE);
  CHECK(ozec::set_device_list(nullptr, 2) == OZEC_EINVAL);
  CHECK((ozec::device_list() == std::vector<int>{2, 2, 0}));
  // NUMA policy: only the listed devices on the caller's node, while there are any
  const int all4[] = {0, 1, 2, 3};
  CHECK(ozec::set_device_list(all4, 4) == OZEC_OK);
  CHECK(ozec::set_device_policy(1) == OZEC_OK);
  std::set<int> seen;
  for (int i = 0; i < 8; ++i) seen.insert(ozec::pick_device());
  CHECK((seen == std::set<int>{2, 3}));
  {  // coder-less calls of NUMA-policy threads: a listed device on the thread's node
    std::vector<int> nt(4, -1);
    std::vector<std::thread> th;
    for (int i = 0; i < 4; ++i) th.emplace_back([&, i] { nt[i] = ozec::thread_device(); });
    for (auto &t : th) t.join();
    for (int d : nt) CHECK(d == 2 || d == 3);
  }
  const int far[] = {0, 1};
  CHECK(ozec::set_device_list(far, 2) == OZEC_OK);  // none near: every listed device
  seen.clear();
  for (int i = 0; i < 8; ++i) seen.insert(ozec::pick_device());
  CHECK((seen == std::set<int>{0, 1}));
  // current policy: the caller's device, for coders and coder-less calls
  CHECK(ozec::set_device_policy(2) == OZEC_OK);
  g_current = 3;
  CHECK(ozec::pick_device() == 3 && ozec::thread_device() == 3);
  CHECK(ozec::set_device_policy(7) == OZEC_EINVAL && ozec::device_policy() == 2);
  // per-thread devices of coder-less calls: stable per thread, spread over threads, re-picked after a list change
  CHECK(ozec::set_device_policy(0) == OZEC_OK);
  CHECK(ozec::set_device_list(all4, 4) == OZEC_OK);
  std::vector<int> td(8, -1), td2(8, -1);
  std::vector<std::thread> ts;
  for (int i = 0; i < 8; ++i)
    ts.emplace_back([&, i] {
      td[i] = ozec::thread_device();
      td2[i] = ozec::thread_device();
    });
  for (auto &t : ts) t.join();
  std::multiset<int> tm(td.begin(), td.end());
  for (int d = 0; d < 4; ++d) CHECK(tm.count(d) == 2);
  CHECK(td == td2);
  const int one[] = {1};
  const int before = ozec::thread_device();
  CHECK(before >= 0 && before < 4);
  CHECK(ozec::set_device_list(one, 1) == OZEC_OK);
  CHECK(ozec::thread_device() == 1);
  // DeviceScope switches and restores
  g_current = 0;
  {
    ozec::DeviceScope ds(2);
    CHECK(ds.ok() && g_current == 2);
    {
      ozec::DeviceScope same(2);  // no switch
      CHECK(same.ok() && g_current == 2);
    }
    CHECK(g_current == 2);
  }
  CHECK(g_current == 0);
  {
    ozec::DeviceScope bad_scope(9);
    CHECK(!bad_scope.ok() && g_current == 0);
  }
  CHECK(g_current == 0);
  // no device at all: empty list, nothing to pick
  g_count = 0;
  CHECK(ozec::set_device_list(nullptr, 0) == OZEC_OK);
  CHECK(ozec::device_list().empty() && ozec::pick_device() == -1);
  if (failures) return 1;
  std::printf("devices policy OK\n");
  return 0;
}
