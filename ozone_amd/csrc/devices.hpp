// Which GPUs one drop-in process uses, and which one each coder and host call runs on.
//
// Ozone runs one JVM per datanode or client, not one process per GPU: every ECKeyOutputStream makes its own coder
// (ECKeyOutputStream.java:117), every reconstruction its own decoder (ECBlockReconstructedStripeInputStream.java:232).
// So the library, not the caller, spreads the work over the node's GPUs (SURVEY §7 "lazy singleton per GPU", §8(b)
// process-global per-GPU context, north_star: "a batch is partitioned across the 8 MI355X of one node as per-GPU
// streams"):
//   * the device list: every visible GPU, or OZEC_DEVICES ("0,2,3", "all"), or ozec_set_devices;
//   * a coder is bound to one device of the list when it is made (policy OZEC_DEVICE_POLICY: round_robin, the default;
//     numa -- round robin over the listed GPUs closest to the creating thread's NUMA node; current -- the creating
//     thread's current device, the one-process-per-GPU model); its host-buffer calls and stripe queues run there;
//   * a host batch (ozec_encode_crc_host_batch / ozec_reconstruct_crc_host_batch) is split into contiguous stripe
//     ranges over the whole list, one pipeline per GPU, run at once;
//   * coder-less host calls (CRC of a host buffer) run on a device the calling thread is given on first use;
//   * device-pointer entry points run on the caller's current device (the one its pointers and stream belong to).
#pragma once
#include <cstddef>
#include <vector>

namespace ozec {

// the device list (never empty when a GPU exists; empty when none does)
std::vector<int> device_list();
// replace the list (ordinals must exist; duplicates allowed -- [0, 0] splits a batch in two on one GPU); n = 0
// restores the default.  Returns 0 or a negative OZEC_* status.
int set_device_list(const int *devs, int n);
// the device a new coder is bound to, by the policy
int pick_device();
// the device of this thread's coder-less host calls: given on first use by the policy (round robin over the list, or
// over the listed devices on the thread's NUMA node), re-picked when the list changes; "current": the current device
int thread_device();
// 0 round_robin, 1 numa, 2 current
int device_policy();
int set_device_policy(int policy);
// ozec_set_device was called: a process that picks its GPU itself is a one-process-per-GPU caller, so unless it chose
// a device list or policy (API or environment) the policy becomes "current" -- its coders, host batches and pinned
// buffers then stay on the GPU it selected instead of spreading over GPUs other processes own.  Returns
// whether the policy changed.
bool note_set_device();

// How a host batch of `num_stripes` is split over `ndev` listed devices (capi.cpp host_batch_split): one part per device
// while every part gets at least one pipeline chunk of `chunk` stripes, else fewer parts; part i is the contiguous range
// [s0, s1) = ozone_amd/shard.py stripe_range(num_stripes, i, parts) -- the partition bench.py's ranks use, so a rank's
// registered range is exactly libozec's part for its GPU (bench.py in_process_leg).
size_t split_parts(size_t num_stripes, size_t chunk, size_t ndev);
void part_range(size_t num_stripes, size_t parts, size_t i, size_t *s0, size_t *s1);

// switch the calling thread to `dev` for the scope (restored on exit); ok() false when the switch failed
class DeviceScope {
 public:
  explicit DeviceScope(int dev);
  ~DeviceScope();
  bool ok() const { return ok_; }

 private:
  int prev_ = -1;
  bool switched_ = false, ok_ = true;
};

}  // namespace ozec
