// Per-call counters of the C ABI (ozec_stats): calls, bytes, failures and host time per entry-point family,
// process-wide and lock-free.  SURVEY §5 "Metrics": the reference keeps per-operation counters
// (ECReconstructionMetrics.java:34-41, ContainerClientMetrics.java:41-42); these are what a metrics2 source would
// publish for the GPU coder.  Only the outermost instrumented call of a thread records (an e2e batch that runs the
// fused kernel counts once, as a host batch).
#pragma once
#include <atomic>
#include <chrono>
#include <cstdint>

#include "../../include/ozec.h"

namespace ozec {

struct OpCounters {
  std::atomic<uint64_t> calls{0}, bytes{0}, errors{0}, host_ns{0};
};
extern OpCounters g_stats[OZEC_NUM_OPS];
extern thread_local int g_stat_depth;
extern thread_local bool g_stat_failed;  // set by every error path (set_error / fail)

class StatScope {
 public:
  StatScope(int op, uint64_t bytes) : op_(op), bytes_(bytes), outer_(g_stat_depth++ == 0) {
    if (outer_) {
      g_stat_failed = false;
      t0_ = std::chrono::steady_clock::now();
    }
  }
  ~StatScope() {
    --g_stat_depth;
    if (!outer_) return;
    OpCounters &c = g_stats[op_];
    c.calls.fetch_add(1, std::memory_order_relaxed);
    if (g_stat_failed) {
      c.errors.fetch_add(1, std::memory_order_relaxed);
    } else {
      c.bytes.fetch_add(bytes_, std::memory_order_relaxed);
    }
    const auto ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0_);
    c.host_ns.fetch_add(static_cast<uint64_t>(ns.count()), std::memory_order_relaxed);
  }
  StatScope(const StatScope &) = delete;
  StatScope &operator=(const StatScope &) = delete;

 private:
  int op_;
  uint64_t bytes_;
  bool outer_;
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace ozec
