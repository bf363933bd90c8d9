// NUMA-local pinned host memory for the per-GPU copy paths (end to end, host DRAM bandwidth and
// the per-GPU PCIe link bound the multi-GPU path; pages on the wrong socket cross the inter-socket fabric on
// every DMA).  A GPU's host NUMA node comes from HIP (hipDeviceAttributeHostNumaId) or sysfs; pages are placed
// with mbind(2) before the first touch and then pinned with hipHostRegister.
#pragma once
#include <cstddef>
#include <cstdint>

namespace ozec {

// host NUMA node closest to `device`, -1 when unknown or the host is not NUMA
int device_numa_node(int device);
// mbind [p, p+bytes) to `node` with MPOL_PREFERRED (MOVE existing pages when move): page-aligned outward, or with
// inner only the pages wholly inside the range (caller memory whose first / last page it may share with others);
// returns 0 or -errno.  node < 0 is a no-op.
int bind_to_node(void *p, size_t bytes, int node, bool move, bool inner);
// node of the page holding p (after it has been touched), -1 if unknown
int page_node(const void *p);
// pinned host allocation whose pages live on the device's node, always in a fresh address range; free with pinned_free.
// A freed block is unregistered and its pages returned, and its address range is retired (PROT_NONE, never reused for
// a later block; returned to the kernel oldest first past a bound): nothing libozec registered is registered again at
// the same address or handed out by the kernel as a pageable buffer soon after ("GPU faults").
// pinned_free returns -EINVAL for a pointer it did not allocate and -EBUSY when the runtime refuses to unregister the
// block (which then stays mapped and registered: a counted leak).
int pinned_alloc(size_t bytes, int device, void **out);
int pinned_free(void *p);
// bytes of address space held by retired blocks (no memory behind them)
size_t pinned_retired_bytes();
// frees whose hipHostUnregister failed (their blocks were left mapped and registered)
uint64_t pinned_unregister_failures();
// start of the pinned / registered host allocation holding p (null when p is not in one): a DMA (a 2D copy's rows
// included) must lie within one allocation
const void *pinned_alloc_base(const void *p);
// pin the calling thread / the copy-pool workers to the CPUs of `node` (intersected with the process mask)
int bind_thread_to_node(int node);

}  // namespace ozec
