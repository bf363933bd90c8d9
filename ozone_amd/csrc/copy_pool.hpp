// Parallel host memcpy for the staging paths (pageable caller buffers <-> pinned staging).  One thread copies
// ~10-16 GB/s; the host-buffer ABI (the JNI drop-in path) is bound by that copy, so large copies are split into
// >= 256 KiB pieces over a small process-wide worker pool, the calling thread taking part.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace ozec {

struct CopyTask {
  void *dst;
  const void *src;
  size_t n;
};

// kToStaging: into pinned staging memory that only a DMA engine reads next; kFromStaging: into caller memory
enum class CopyDir { kToStaging, kFromStaging };
// run every task (in any order) and return when all are done, with the workers of the pool of NUMA node `node` (the
// staging buffers' node: the GPU's, numa.hpp; -1 = unbound workers); `shared`: other transfers use host DRAM meanwhile
// (DMA of other chunks or batches, other callers' copies); only copy_stream mode 3 looks at it (copy_pool.cpp)
void parallel_copy(const std::vector<CopyTask> &tasks, CopyDir dir, bool shared = true, int node = -1);
// threads used besides the caller by every node's pool (0 = copy inline); set by ozec_set_tuning("copy_threads", n)
void set_copy_threads(int n);
// how long pool workers and waiting callers poll before sleeping (0: not at all)
void set_copy_spin_us(int64_t us);
int64_t copy_spin_us();
// pieces copied with streaming (non-temporal) stores: 1 both directions, 2 into staging only, 3 only for copies that
// share DRAM with other transfers, 0 plain memcpy, -1 auto (1 where AVX2 exists); set by
// ozec_set_tuning("copy_stream", n); false (nothing changed) outside -1..3
bool set_copy_stream(int mode);

}  // namespace ozec
