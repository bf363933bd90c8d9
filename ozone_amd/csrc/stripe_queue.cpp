// Writer-side stripe batching, built on the public C ABI only.
//
// ECKeyOutputStream encodes one stripe per RawErasureEncoder.encode call (ECKeyOutputStream.java:304; stripe
// queue :114, :501-543).  A stripe queue takes stripes as they fill and runs them in batches: each submitted
// cell is copied into the batch's device buffer on the batch's stream right away (DMA straight from the
// caller's buffer when it is pinned, else through pinned staging), a full batch is one fused encode (+ CRC)
// launch, and parity / CRCs come back by DMA into pinned callers' buffers or through staging.  Several
// batches rotate, so the copies of batch i+1 overlap the kernel and copies of batch i.
//
// All H2D copies go in submission order on ONE stream; a batch's kernel and D2H copies follow on its own
// stream behind an event.  With one H2D stream per batch instead, the H2D copies of all batches in the ring
// shared the link at once, finished together, and their D2H copies then ran with the link's H2D direction
// idle while the submitting thread waited for the oldest batch (rocprofv3 copy trace: H2D busy 119 of
// 147 ms per 1024 stripes; 41 GB/s against a 57 GB/s link).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ozec.h"
#include "copy_pool.hpp"
#include "devices.hpp"
#include "kernels.hpp"
#include "numa.hpp"
#include "stats.hpp"
#include "status.hpp"

namespace {

using ozec::set_error;

std::atomic<uint64_t> g_place_failures{0};  // ozec_host_register calls whose NUMA placement was refused

// batches in the ring: copies of the newest batches keep the link busy while the oldest one drains
constexpr size_t kDefaultBatches = 3;

#define SQ_HIP(call)                                                                                      \
  do {                                                                                                    \
    hipError_t err_ = (call);                                                                             \
    if (err_ != hipSuccess)                                                                               \
      return set_error(OZEC_EDEVICE, std::string("HIP error: ") + hipGetErrorString(err_) + " at " #call); \
  } while (0)

bool is_pinned(const void *p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

struct Pending {
  std::vector<uint8_t *> parity;  // caller's parity buffers (p of them)
  uint32_t *crcs = nullptr;       // caller's CRC buffer or null
  bool parity_staged = false;     // parity comes back through staging (caller buffer not pinned)
};

// A run of equally shaped copies whose sources and destinations both advance by a fixed pitch (one cell group per
// stripe): issued as ONE hipMemcpy2DAsync instead of one copy per stripe.  Cells of consecutive stripes taken from
// one pinned pool (or from the staging area) form such runs; per-copy overhead was what held the queue at 84 % of
// the link while the host batch, which copies rectangles, reached 98 %.
// Start of the pinned allocation holding host pointer p (null when unknown): a 2D copy's rows must lie in one.
const void *alloc_base(const void *p) { return ozec::pinned_alloc_base(p); }

struct CopyRun {
  const uint8_t *src = nullptr;
  uint8_t *dst = nullptr;
  size_t width = 0, spitch = 0, dpitch = 0, height = 0;
  const void *hbase = nullptr;  // pinned allocation of the host side (rows may not leave it)

  bool extends(const uint8_t *s, uint8_t *d, size_t w, const void *hb) const {
    constexpr size_t kMaxPitch = size_t{1} << 30;
    if (!height || w != width || !hb || hb != hbase) return false;
    if (height == 1)  // the second row fixes the pitches: forward, no overlap, within the copy engine's reach
      return s >= src + width && d >= dst + width && static_cast<size_t>(s - src) <= kMaxPitch &&
             static_cast<size_t>(d - dst) <= kMaxPitch;
    return s == src + height * spitch && d == dst + height * dpitch;
  }
  void add(const uint8_t *s, uint8_t *d, size_t w, const void *hb) {
    if (height == 1) {
      spitch = static_cast<size_t>(s - src);
      dpitch = static_cast<size_t>(d - dst);
    } else if (height == 0) {
      src = s, dst = d, width = w, hbase = hb;
    }
    ++height;
  }
  hipError_t issue(hipMemcpyKind kind, hipStream_t st) {
    hipError_t e = hipSuccess;
    if (height == 1) e = hipMemcpyAsync(dst, src, width, kind, st);
    else if (height > 1) e = hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, kind, st);
    height = 0;
    return e;
  }
};

struct Batch {
  hipStream_t stream = nullptr;  // kernel + D2H of this batch
  hipEvent_t copied = nullptr;   // recorded on the queue's H2D stream after this batch's last H2D copy
  hipEvent_t done = nullptr;
  uint8_t *d_units = nullptr;  // [S][k+rows][cell_len]
  uint32_t *d_crcs = nullptr;  // [S][k+rows][nwin]
  uint8_t *h_stage = nullptr;  // pinned [S][k+rows][cell_len], allocated on first pageable use
  uint32_t *h_crcs = nullptr;  // pinned [S][k+rows][nwin]
  size_t n = 0, len = 0;
  uint64_t first_ticket = 0;
  bool in_flight = false;
  std::vector<Pending> pend;
};

}  // namespace

struct ozec_stripe_queue {
  ozec_coder *enc = nullptr;
  int device = 0;  // the queue's GPU (its encoder's); pinned staging lives on its NUMA node
  int node = -1;   // that node (its copy pool, copy_pool.hpp)
  int k = 0, p = 0, rows = 0, ctype = OZEC_CHECKSUM_NONE, big_endian = 0;
  size_t cell_len = 0, S = 0, bpc = 0, nwin_max = 0;
  std::vector<Batch> batches;
  hipStream_t h2d = nullptr;  // every H2D copy, in submission order
  CopyRun h2d_run;            // H2D copies not issued yet (they extend while stripes arrive back to back)
  size_t cur = 0;
  uint64_t next_ticket = 0;
  std::mutex mu;

  // device layout per stripe: k data + p parity cells (all p, so the XOR codec's zero-filled extra outputs --
  // ozec_encode_batch writes them -- stay inside the stripe); CRCs cover the k + rows cells that are coded
  size_t units() const { return static_cast<size_t>(k + rows); }
  size_t stripe_bytes() const { return static_cast<size_t>(k + p) * cell_len; }
  size_t stripe_crcs() const { return units() * nwin_max; }
  size_t nwin(size_t len) const { return bpc ? (len + bpc - 1) / bpc : 0; }

  // queue an H2D copy; consecutive stripes' cells coalesce into one 2D copy, issued once 8 stripes have gathered (the
  // link starts on a batch early) or when the run breaks
  int h2d_copy(uint8_t *dst, const uint8_t *src, size_t bytes) {
    const void *hb = alloc_base(src);
    if (h2d_run.height && (!h2d_run.extends(src, dst, bytes, hb) || h2d_run.height >= 8))
      SQ_HIP(h2d_run.issue(hipMemcpyHostToDevice, h2d));
    h2d_run.add(src, dst, bytes, hb);
    return OZEC_OK;
  }
  int h2d_flush() {
    SQ_HIP(h2d_run.issue(hipMemcpyHostToDevice, h2d));
    return OZEC_OK;
  }

  int launch(Batch &b) {
    if (b.n == 0 || b.in_flight) return OZEC_OK;
    if (int rc = h2d_flush()) return rc;
    const int64_t ss = static_cast<int64_t>(stripe_bytes()), us = static_cast<int64_t>(cell_len);
    uint8_t *d_par = b.d_units + static_cast<size_t>(k) * cell_len;
    const size_t nw = nwin(b.len);
    SQ_HIP(hipEventRecord(b.copied, h2d));
    SQ_HIP(hipStreamWaitEvent(b.stream, b.copied, 0));
    if (ctype == OZEC_CHECKSUM_NONE) {
      if (int rc = ozec_encode_batch(enc, b.d_units, ss, us, d_par, ss, us, b.n, b.len, b.stream)) return rc;
    } else {
      // CRC layout per stripe [unit][window] with a fixed stride of nw windows per unit
      if (int rc = ozec_encode_crc_batch(enc, b.d_units, ss, us, d_par, ss, us, b.n, b.len, ctype, bpc, b.d_crcs,
                                         big_endian, b.stream))
        return rc;
    }
    // parity back: per stripe one copy per run of back-to-back parity cells, coalesced across stripes into 2D copies
    CopyRun d2h;
    for (size_t i = 0; i < b.n; ++i) {
      const Pending &pd = b.pend[i];
      for (int r = 0; r < rows;) {
        const size_t off = i * stripe_bytes() + static_cast<size_t>(k + r) * cell_len;
        uint8_t *dst = pd.parity_staged ? b.h_stage + off : pd.parity[r];
        int run = 1;
        while (!pd.parity_staged && b.len == cell_len && r + run < rows && pd.parity[r + run] == dst + run * b.len)
          ++run;
        if (pd.parity_staged && b.len == cell_len) run = rows - r;  // staging holds the stripe's parity back to back
        const uint8_t *src = b.d_units + off;
        const void *hb = alloc_base(dst);
        if (d2h.height && !d2h.extends(src, dst, run * b.len, hb)) SQ_HIP(d2h.issue(hipMemcpyDeviceToHost, b.stream));
        d2h.add(src, dst, run * b.len, hb);
        r += run;
      }
    }
    SQ_HIP(d2h.issue(hipMemcpyDeviceToHost, b.stream));
    if (ctype != OZEC_CHECKSUM_NONE)
      SQ_HIP(hipMemcpyAsync(b.h_crcs, b.d_crcs, b.n * units() * nw * sizeof(uint32_t), hipMemcpyDeviceToHost,
                            b.stream));
    SQ_HIP(hipEventRecord(b.done, b.stream));
    b.in_flight = true;
    return OZEC_OK;
  }

  int complete(Batch &b) {
    if (!b.in_flight) return OZEC_OK;
    SQ_HIP(hipEventSynchronize(b.done));
    const size_t nw = nwin(b.len);
    std::vector<ozec::CopyTask> tasks;
    for (size_t i = 0; i < b.n; ++i) {
      const Pending &pd = b.pend[i];
      for (int r = 0; r < p; ++r) {
        if (r >= rows) {  // XOR with p > 1: outputs past the first stay zero (XORRawEncoder.java:67-85)
          std::memset(pd.parity[r], 0, b.len);
        } else if (pd.parity_staged) {
          tasks.push_back({pd.parity[r], b.h_stage + i * stripe_bytes() + static_cast<size_t>(k + r) * cell_len, b.len});
        }
      }
      if (pd.crcs && ctype != OZEC_CHECKSUM_NONE)
        tasks.push_back({pd.crcs, b.h_crcs + i * units() * nw, units() * nw * sizeof(uint32_t)});
    }
    ozec::parallel_copy(tasks, ozec::CopyDir::kFromStaging, true, node);
    b.in_flight = false;
    b.n = 0;
    return OZEC_OK;
  }

  int stage_pinned(Batch &b) {
    if (!b.h_stage && ozec::pinned_alloc(S * stripe_bytes(), device, reinterpret_cast<void **>(&b.h_stage)) != 0)
      return set_error(OZEC_ENOMEM, "cannot pin the stripe queue's staging memory");
    return OZEC_OK;
  }
};

extern "C" {

int ozec_host_alloc_on(size_t bytes, int device, void **out) {
  if (!out) return set_error(OZEC_EINVAL, "null output");
  *out = nullptr;
  if (bytes == 0) return OZEC_OK;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    (void)hipGetLastError();
    return set_error(OZEC_EDEVICE, "no such device " + std::to_string(device));
  }
  if (ozec::pinned_alloc(bytes, device, out) != 0)
    return set_error(OZEC_ENOMEM, "cannot allocate " + std::to_string(bytes) + " bytes of pinned host memory");
  return OZEC_OK;
}

int ozec_host_alloc(size_t bytes, void **out) {
  const int dev = ozec::thread_device();  // this thread's GPU (devices.hpp; policy "current": its current device)
  if (dev < 0) return set_error(OZEC_EDEVICE, "no HIP device available");
  return ozec_host_alloc_on(bytes, dev, out);
}

int ozec_host_free(void *p) {
  if (!p) return OZEC_OK;
  const int rc = ozec::pinned_free(p);
  if (rc == -EBUSY)
    return set_error(OZEC_EDEVICE, "the HIP runtime did not unregister the pinned block (left mapped and registered)");
  if (rc != 0) return set_error(OZEC_EINVAL, "pointer was not allocated by ozec_host_alloc");
  return OZEC_OK;
}

uint64_t ozec_host_free_failures(void) { return ozec::pinned_unregister_failures(); }

int ozec_device_numa_node(int device, int *node) {
  if (!node) return set_error(OZEC_EINVAL, "null output");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) {
    (void)hipGetLastError();
    return set_error(OZEC_EDEVICE, "no such device " + std::to_string(device));
  }
  *node = ozec::device_numa_node(device);
  return OZEC_OK;
}

int ozec_host_page_node(const void *p, int *node) {
  if (!p || !node) return set_error(OZEC_EINVAL, "null pointer");
  *node = ozec::page_node(p);
  return OZEC_OK;
}

int ozec_host_copy(void *const *dst, const void *const *src, const size_t *bytes, int count, int to_pinned) {
  if (count < 0 || (count > 0 && (!dst || !src || !bytes))) return set_error(OZEC_EINVAL, "null copy list");
  std::vector<ozec::CopyTask> tasks;
  tasks.reserve(static_cast<size_t>(count));
  for (int i = 0; i < count; ++i) {
    if (bytes[i] == 0) continue;
    if (!dst[i] || !src[i]) return set_error(OZEC_EINVAL, "null pointer in the copy list");
    tasks.push_back({dst[i], src[i], bytes[i]});
  }
  // the pool of the NUMA node of this thread's GPU, whose pinned buffers the copies fill or drain (cached per thread)
  thread_local int dev = -2, node = -1;
  const int d = ozec::thread_device();
  if (d != dev) {
    dev = d;
    node = d >= 0 ? ozec::device_numa_node(d) : -1;
  }
  ozec::parallel_copy(tasks, to_pinned ? ozec::CopyDir::kToStaging : ozec::CopyDir::kFromStaging, true, node);
  return OZEC_OK;
}

int ozec_host_register(void *p, size_t bytes, int device) {
  if (!p) return set_error(OZEC_EINVAL, "null pointer");
  if (bytes == 0) return OZEC_OK;
  const int node = device >= 0 ? ozec::device_numa_node(device) : -1;
  // placement is best effort, as for pinned_alloc: pages not touched yet are placed on the node as hipHostRegister
  // faults them in, touched ones are moved -- only pages wholly inside the range.  Where mbind is refused (EPERM
  // under a seccomp profile without CAP_SYS_NICE, ENOSYS without NUMA) the memory is still pinned where it lies;
  // ozec_host_page_node shows the placement, and the failure is counted in g_place_failures.
  if (ozec::bind_to_node(p, bytes, node, true, true) != 0) g_place_failures.fetch_add(1, std::memory_order_relaxed);
  SQ_HIP(hipHostRegister(p, bytes, hipHostRegisterPortable));
  return OZEC_OK;
}

uint64_t ozec_host_placement_failures(void) { return g_place_failures.load(std::memory_order_relaxed); }

int ozec_host_unregister(void *p) {
  if (!p) return set_error(OZEC_EINVAL, "null pointer");
  SQ_HIP(hipHostUnregister(p));
  return OZEC_OK;
}

int ozec_stripe_queue_create(ozec_coder *enc, size_t cell_len, size_t stripes_per_batch, int checksum_type,
                             size_t bpc, int big_endian, ozec_stripe_queue **out) {
  if (!out) return set_error(OZEC_EINVAL, "null output handle");
  *out = nullptr;
  int codec = 0, k = 0, p = 0, is_dec = 0;
  if (int rc = ozec_coder_info(enc, &codec, &k, &p, &is_dec)) return rc;
  if (is_dec) return set_error(OZEC_EINVAL, "not an encoder");
  if (cell_len == 0 || stripes_per_batch == 0) return set_error(OZEC_EINVAL, "cell_len and stripes_per_batch must be > 0");
  if (checksum_type != OZEC_CHECKSUM_NONE && checksum_type != OZEC_CHECKSUM_CRC32 &&
      checksum_type != OZEC_CHECKSUM_CRC32C)
    return set_error(OZEC_EINVAL, "checksum type must be NONE, CRC32 or CRC32C");
  if (checksum_type != OZEC_CHECKSUM_NONE && bpc == 0) return set_error(OZEC_EINVAL, "bytesPerChecksum must be positive");
  if (ozec_coder_is_closed(enc)) return set_error(OZEC_ECLOSED, "stripe queue: the encoder is closed");
  auto *q = new (std::nothrow) ozec_stripe_queue();
  if (!q) return set_error(OZEC_ENOMEM, "out of memory");
  // the queue co-owns the encoder: it stays allocated until ozec_stripe_queue_free even if its creator releases and
  // frees it first (the queue's launches then fail with OZEC_ECLOSED)
  (void)ozec_coder_retain(enc);
  q->enc = enc;
  q->device = ozec_coder_device(enc);  // the encoder's GPU (devices.hpp)
  q->node = q->device >= 0 ? ozec::device_numa_node(q->device) : -1;
  ozec::DeviceScope ds(q->device);
  if (!ds.ok()) {
    ozec_coder_free(enc);
    delete q;
    return set_error(OZEC_EDEVICE, "cannot select device " + std::to_string(q->device));
  }
  q->k = k;
  q->p = p;
  q->rows = codec == OZEC_CODEC_XOR ? 1 : p;
  q->ctype = checksum_type;
  q->bpc = checksum_type == OZEC_CHECKSUM_NONE ? 0 : bpc;
  q->big_endian = big_endian;
  q->cell_len = cell_len;
  q->S = stripes_per_batch;
  q->nwin_max = q->nwin(cell_len);
  const int64_t qb = ozec::g_tune.queue_batches.load();
  q->batches.resize(qb >= 2 ? static_cast<size_t>(qb) : kDefaultBatches);
  for (Batch &b : q->batches) {
    b.pend.resize(q->S);
    hipError_t e = q->h2d ? hipSuccess : ozec::make_stream(&q->h2d);
    if (e == hipSuccess) e = ozec::make_stream(&b.stream);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&b.copied, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&b.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&b.d_units), q->S * q->stripe_bytes());
    if (e == hipSuccess && q->ctype != OZEC_CHECKSUM_NONE) {
      e = hipMalloc(reinterpret_cast<void **>(&b.d_crcs), q->S * q->stripe_crcs() * sizeof(uint32_t));
      if (e == hipSuccess && ozec::pinned_alloc(q->S * q->stripe_crcs() * sizeof(uint32_t), q->device,
                                                reinterpret_cast<void **>(&b.h_crcs)) != 0)
        e = hipErrorOutOfMemory;
    }
    if (e != hipSuccess) {
      ozec_stripe_queue_free(q);
      return set_error(OZEC_EDEVICE, std::string("HIP error creating the stripe queue: ") + hipGetErrorString(e));
    }
  }
  *out = q;
  return OZEC_OK;
}

int ozec_stripe_queue_submit(ozec_stripe_queue *q, const uint8_t *const *data, uint8_t *const *parity, size_t len,
                             uint32_t *crcs, uint64_t *ticket) {
  ozec::StatScope stat_(OZEC_OP_QUEUE, q ? static_cast<uint64_t>(q->k) * len : 0);
  if (!q) return set_error(OZEC_EINVAL, "null queue");
  if (!data || !parity) return set_error(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  for (int j = 0; j < q->k; ++j)
    if (!data[j]) return set_error(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  for (int r = 0; r < q->p; ++r)
    if (!parity[r]) return set_error(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  if (len == 0 || len > q->cell_len)
    return set_error(OZEC_EINVAL, "stripe length must be in [1, cell_len] (" + std::to_string(q->cell_len) + ")");
  if (ozec_coder_is_closed(q->enc)) return set_error(OZEC_ECLOSED, "stripe queue submit failed: the encoder is closed");
  ozec::DeviceScope ds(q->device);
  if (!ds.ok()) return set_error(OZEC_EDEVICE, "cannot select device " + std::to_string(q->device));
  std::lock_guard<std::mutex> lk(q->mu);
  Batch *b = &q->batches[q->cur];
  // cur only ever points at a filling batch or, once the ring has wrapped, at the oldest in-flight one: that one
  // completes now (its callers' outputs land) and is refilled
  if (b->in_flight)
    if (int rc = q->complete(*b)) return rc;
  if (b->n > 0 && b->len != len) {  // a batch holds one cell length: launch it and move on
    if (int rc = q->launch(*b)) return rc;
    q->cur = (q->cur + 1) % q->batches.size();
    b = &q->batches[q->cur];
    if (b->in_flight)
      if (int rc = q->complete(*b)) return rc;
  }
  if (b->n == 0) {
    b->len = len;
    b->first_ticket = q->next_ticket;
  }
  const size_t i = b->n;
  Pending &pd = b->pend[i];
  pd.parity.assign(parity, parity + q->p);
  pd.crcs = crcs;
  pd.parity_staged = false;
  for (int r = 0; r < q->rows; ++r) pd.parity_staged |= !is_pinned(parity[r]);
  if (pd.parity_staged)
    if (int rc = q->stage_pinned(*b)) return rc;
  // pageable cells are staged first (in parallel), then every cell goes over PCIe; cells laid out back to back
  // in one pinned buffer (or in the staging area) go as one copy
  std::vector<const uint8_t *> src(data, data + q->k);
  std::vector<ozec::CopyTask> tasks;
  for (int j = 0; j < q->k; ++j) {
    if (is_pinned(src[j])) continue;
    if (int rc = q->stage_pinned(*b)) return rc;
    uint8_t *st = b->h_stage + i * q->stripe_bytes() + static_cast<size_t>(j) * q->cell_len;
    tasks.push_back({st, src[j], len});
    src[j] = st;
  }
  ozec::parallel_copy(tasks, ozec::CopyDir::kToStaging, true, q->node);
  for (int j = 0; j < q->k;) {
    const size_t off = i * q->stripe_bytes() + static_cast<size_t>(j) * q->cell_len;
    int run = 1;
    while (len == q->cell_len && j + run < q->k && src[j + run] == src[j] + run * len) ++run;
    if (int rc = q->h2d_copy(b->d_units + off, src[j], run * len)) return rc;
    j += run;
  }
  ++b->n;
  if (ticket) *ticket = q->next_ticket;
  ++q->next_ticket;
  if (b->n == q->S) {
    if (int rc = q->launch(*b)) return rc;
    q->cur = (q->cur + 1) % q->batches.size();
  }
  return OZEC_OK;
}

int ozec_stripe_queue_flush(ozec_stripe_queue *q) {
  ozec::StatScope stat_(OZEC_OP_QUEUE, 0);
  if (!q) return set_error(OZEC_EINVAL, "null queue");
  ozec::DeviceScope ds(q->device);
  if (!ds.ok()) return set_error(OZEC_EDEVICE, "cannot select device " + std::to_string(q->device));
  std::lock_guard<std::mutex> lk(q->mu);
  Batch &b = q->batches[q->cur];
  if (b.n > 0 && !b.in_flight) {
    if (int rc = q->launch(b)) return rc;
    q->cur = (q->cur + 1) % q->batches.size();
  }
  return OZEC_OK;
}

int ozec_stripe_queue_wait(ozec_stripe_queue *q, uint64_t ticket) {
  ozec::StatScope stat_(OZEC_OP_QUEUE, 0);
  if (!q) return set_error(OZEC_EINVAL, "null queue");
  ozec::DeviceScope ds(q->device);
  if (!ds.ok()) return set_error(OZEC_EDEVICE, "cannot select device " + std::to_string(q->device));
  std::lock_guard<std::mutex> lk(q->mu);
  if (ticket >= q->next_ticket) return set_error(OZEC_EINVAL, "unknown ticket " + std::to_string(ticket));
  // complete, oldest first, every batch holding a stripe <= ticket (launching the filling one if needed)
  for (;;) {
    Batch *oldest = nullptr;
    for (Batch &b : q->batches)
      if (b.n > 0 && b.first_ticket <= ticket && (!oldest || b.first_ticket < oldest->first_ticket)) oldest = &b;
    if (!oldest) return OZEC_OK;
    if (!oldest->in_flight) {
      if (int rc = q->launch(*oldest)) return rc;
      if (oldest == &q->batches[q->cur]) q->cur = (q->cur + 1) % q->batches.size();
    }
    if (int rc = q->complete(*oldest)) return rc;
  }
}

int ozec_stripe_queue_info(const ozec_stripe_queue *q, int *num_data, int *num_parity, int *rows, size_t *cell_len,
                           int *checksum_type, size_t *bytes_per_checksum) {
  if (!q) return set_error(OZEC_EINVAL, "null queue");
  if (num_data) *num_data = q->k;
  if (num_parity) *num_parity = q->p;
  if (rows) *rows = q->rows;
  if (cell_len) *cell_len = q->cell_len;
  if (checksum_type) *checksum_type = q->ctype;
  if (bytes_per_checksum) *bytes_per_checksum = q->bpc;
  return OZEC_OK;
}

int ozec_stripe_queue_state(ozec_stripe_queue *q, size_t *in_flight, uint64_t *oldest_in_flight_ticket,
                            size_t *filling) {
  if (!q) return set_error(OZEC_EINVAL, "null queue");
  std::lock_guard<std::mutex> lk(q->mu);
  size_t n = 0, f = 0;
  uint64_t oldest = UINT64_MAX;
  for (const Batch &b : q->batches) {
    if (b.in_flight) {
      ++n;
      oldest = std::min(oldest, b.first_ticket);
    } else {
      f += b.n;
    }
  }
  if (in_flight) *in_flight = n;
  if (oldest_in_flight_ticket) *oldest_in_flight_ticket = oldest;
  if (filling) *filling = f;
  return OZEC_OK;
}

int ozec_stripe_queue_free(ozec_stripe_queue *q) {
  if (!q) return OZEC_OK;
  ozec::DeviceScope ds(q->device);
  int rc = OZEC_OK;
  // Stripes submitted but never waited for are completed here, oldest first: a filling batch is launched and
  // every batch's parity / CRCs land in the callers' buffers before they are released (ozec.h: the buffers
  // stay valid until wait() or free).
  {
    std::lock_guard<std::mutex> lk(q->mu);
    for (;;) {
      Batch *oldest = nullptr;
      for (Batch &b : q->batches)
        if (b.n > 0 && (!oldest || b.first_ticket < oldest->first_ticket)) oldest = &b;
      if (!oldest) break;
      int r = oldest->in_flight ? OZEC_OK : q->launch(*oldest);
      if (r == OZEC_OK) r = q->complete(*oldest);
      if (r != OZEC_OK) {  // drop it: its DMA is waited for below, its callers get nothing
        rc = r;
        oldest->n = 0;
        oldest->in_flight = false;
      }
    }
  }
  // H2D copies of a batch never launched still write its device buffer
  if (q->h2d && q->h2d_flush() != OZEC_OK) rc = OZEC_EDEVICE;
  if (q->h2d && hipStreamSynchronize(q->h2d) != hipSuccess) rc = OZEC_EDEVICE;
  for (Batch &b : q->batches) {
    if (b.stream && hipStreamSynchronize(b.stream) != hipSuccess) rc = OZEC_EDEVICE;
    if (b.d_units) (void)hipFree(b.d_units);
    if (b.d_crcs) (void)hipFree(b.d_crcs);
    if (b.h_stage) (void)ozec::pinned_free(b.h_stage);
    if (b.h_crcs) (void)ozec::pinned_free(b.h_crcs);
    if (b.done) (void)hipEventDestroy(b.done);
    if (b.copied) (void)hipEventDestroy(b.copied);
    if (b.stream) (void)hipStreamDestroy(b.stream);
  }
  if (q->h2d) (void)hipStreamDestroy(q->h2d);
  ozec_coder_free(q->enc);  // the queue's ownership (ozec_stripe_queue_create)
  delete q;
  return rc == OZEC_OK ? OZEC_OK : set_error(rc, "device error while draining the stripe queue");
}

}  // extern "C"
