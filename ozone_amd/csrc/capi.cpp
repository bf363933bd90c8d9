// extern "C" implementation of include/ozec.h.
//
// Runtime model (SURVEY.md §7 "Lifetime"): coders are cheap host handles holding only coding matrices and a
// decode-matrix cache; all device state (stream, pinned staging pool, device scratch, CRC tables) is a
// process-global, lazily created context per GPU, shared by every coder and safe to use from many threads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <functional>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <iterator>
#include <memory>
#include <mutex>
#include <regex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ozec.h"
#include "crc_host.hpp"
#include "devices.hpp"
#include "gf256.hpp"
#include "copy_pool.hpp"
#include "kernels.hpp"
#include "numa.hpp"
#include "stats.hpp"
#include "status.hpp"

namespace {

using ozec::CodeArgs;
using ozec::CrcArgs;
using ozec::CrcMath;
using ozec::CrcType;

thread_local std::string g_error;

int fail(int code, const std::string &msg) {
  g_error = msg;
  ozec::g_stat_failed = true;
  return code;
}

#define OZEC_HIP(call)                                                                              \
  do {                                                                                              \
    hipError_t err_ = (call);                                                                       \
    if (err_ != hipSuccess) return fail(OZEC_EDEVICE, std::string("HIP error: ") + hipGetErrorString(err_) + \
                                                          " at " #call);                            \
  } while (0)

// ------------------------------------------------------------------------------------------------
// per-GPU context

// One staging slot = a private stream + pinned host buffer + device buffer. Host-pointer calls (the JNI
// drop-in path) take a slot from the pool for the duration of the call, so calls from different threads
// overlap on the GPU and on the copy engines instead of serialising on one buffer.
struct Slot {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // D2H of a duplex direct call (staged_pipeline), created on first use
  uint8_t *pinned = nullptr;  // on the device's NUMA node (numa.hpp)
  size_t pinned_cap = 0;
  uint8_t *dbuf = nullptr;
  size_t dbuf_cap = 0;
  std::vector<hipEvent_t> events;
  // host_graph: instantiated graphs of one-chunk staged calls (H2D + kernel + D2H on this slot's buffers), keyed by
  // the bytes their launch depends on; dropped whenever the buffers move
  struct Graph {
    std::vector<uint8_t> key;
    hipGraphExec_t exec;
  };
  std::vector<Graph> graphs;
  size_t graph_next = 0;  // round-robin replacement once kMaxGraphs are held
  static constexpr size_t kMaxGraphs = 8;

  void drop_graphs() {
    for (auto &g : graphs) (void)hipGraphExecDestroy(g.exec);
    graphs.clear();
    graph_next = 0;
  }
  hipGraphExec_t find_graph(const std::vector<uint8_t> &key) const {
    for (const auto &g : graphs)
      if (g.key == key) return g.exec;
    return nullptr;
  }
  void keep_graph(std::vector<uint8_t> key, hipGraphExec_t exec) {
    if (graphs.size() < kMaxGraphs) {
      graphs.push_back({std::move(key), exec});
      return;
    }
    Graph &g = graphs[graph_next++ % kMaxGraphs];
    (void)hipGraphExecDestroy(g.exec);
    g = {std::move(key), exec};
  }

  // device buffer only (calls whose caller buffers are pinned need no staging)
  int reserve_device(size_t bytes) {
    if (bytes > dbuf_cap) {
      drop_graphs();
      if (dbuf) (void)hipFree(dbuf);
      dbuf = nullptr;
      dbuf_cap = 0;
      size_t cap = std::max<size_t>(bytes, 1 << 20);
      OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&dbuf), cap));
      dbuf_cap = cap;
    }
    return OZEC_OK;
  }

  int reserve(size_t bytes, size_t nevents, bool with_device = true) {
    if (bytes > pinned_cap || (with_device && bytes > dbuf_cap)) drop_graphs();
    if (bytes > pinned_cap) {
      if (pinned) (void)ozec::pinned_free(pinned);
      pinned = nullptr;
      pinned_cap = 0;
      size_t cap = std::max<size_t>(bytes, 1 << 20);
      if (ozec::pinned_alloc(cap, device, reinterpret_cast<void **>(&pinned)) != 0)
        return fail(OZEC_ENOMEM, "cannot pin " + std::to_string(cap) + " bytes of staging memory");
      pinned_cap = cap;
    }
    if (with_device && bytes > dbuf_cap) {
      if (dbuf) (void)hipFree(dbuf);
      dbuf = nullptr;
      dbuf_cap = 0;
      size_t cap = std::max<size_t>(bytes, 1 << 20);
      OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&dbuf), cap));
      dbuf_cap = cap;
    }
    while (events.size() < nevents) {
      hipEvent_t e;
      OZEC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      events.push_back(e);
    }
    return OZEC_OK;
  }

  int ensure_events(size_t n) {
    while (events.size() < n) {
      hipEvent_t e;
      OZEC_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      events.push_back(e);
    }
    return OZEC_OK;
  }

  // give the staging buffers back (an idle slot: its stream has drained)
  void shrink() {
    if (stream) (void)hipStreamSynchronize(stream);
    if (stream2) (void)hipStreamSynchronize(stream2);
    drop_graphs();
    if (pinned) (void)ozec::pinned_free(pinned);
    if (dbuf) (void)hipFree(dbuf);
    pinned = dbuf = nullptr;
    pinned_cap = dbuf_cap = 0;
  }
};

// End-to-end pipeline of ozec_encode_crc_host_batch: a ring of NB device chunk buffers; the chunk's H2D copies,
// its kernel and its D2H copies go on three streams ordered by events, so the two copy directions and the
// kernel of consecutive chunks run at once.  One call at a time per device (mu).
struct E2E {
  static constexpr int NB = 4;
  std::mutex mu;
  hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
  hipEvent_t h2d_done[NB] = {}, comp_done[NB] = {}, d2h_done[NB] = {};
  uint8_t *dbuf[NB] = {};
  size_t dcap = 0;
  uint8_t *hstage[NB] = {};  // pinned staging, only for pageable caller buffers
  size_t hcap = 0;

  // give the chunk buffers back; caller holds mu (the last call's streams were drained before it returned)
  void shrink() {
    for (auto &d : dbuf) {
      if (d) (void)hipFree(d);
      d = nullptr;
    }
    for (auto &h : hstage) {
      if (h) (void)ozec::pinned_free(h);
      h = nullptr;
    }
    dcap = hcap = 0;
  }
};

struct DevCtx {
  int device = -1;
  int numa = -1;  // host NUMA node closest to the device
  E2E e2e;
  std::mutex pool_mu;  // guards the slot pool
  std::condition_variable pool_cv;
  std::vector<std::unique_ptr<Slot>> slots;
  std::vector<Slot *> free_slots;
  std::atomic<int> leased{0};       // slots leased to calls in flight
  uint32_t *crc_tables[2][3] = {};  // [type][B = 1, 2, 4]
  uint32_t *g26_tables[2][ozec::kG26Slots] = {};  // [type][kG26Cfg slot]
  uint32_t *nib_tables[2] = {};                   // [type]
  uint32_t *xo_tables[2] = {};                    // [type]
  uint32_t *cv_tables[2] = {};                    // [type]
  uint32_t *bshift_tables[2] = {};                // [type]

  int acquire(Slot **out) {
    std::unique_lock<std::mutex> lk(pool_mu);
    const size_t max_slots = static_cast<size_t>(std::max<int64_t>(1, ozec::g_tune.host_slots.load()));
    pool_cv.wait(lk, [&] { return !free_slots.empty() || slots.size() < max_slots; });
    if (free_slots.empty()) {
      auto s = std::make_unique<Slot>();
      s->device = device;
      OZEC_HIP(ozec::make_stream(&s->stream));
      free_slots.push_back(s.get());
      slots.push_back(std::move(s));
    }
    *out = free_slots.back();
    free_slots.pop_back();
    ++leased;
    return OZEC_OK;
  }

  void release(Slot *s) {
    {
      std::lock_guard<std::mutex> lk(pool_mu);
      free_slots.push_back(s);
      --leased;
    }
    pool_cv.notify_one();
  }
};

struct SlotLease {
  DevCtx *ctx;
  Slot *slot = nullptr;
  explicit SlotLease(DevCtx *c) : ctx(c) {}
  ~SlotLease() {
    if (slot) ctx->release(slot);
  }
};

std::mutex g_ctx_mu;
std::vector<std::unique_ptr<DevCtx>> g_ctx;

// current device of the calling thread, with its context created on first use
int get_ctx(DevCtx **out) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(OZEC_EDEVICE, "no HIP device available");
  int dev = 0;
  OZEC_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_ctx_mu);
  if (g_ctx.size() < static_cast<size_t>(n)) g_ctx.resize(n);
  if (!g_ctx[dev]) {
    auto c = std::make_unique<DevCtx>();
    c->device = dev;
    c->numa = ozec::device_numa_node(dev);
    for (int t = 0; t < 2; ++t)
      for (int b = 0; b < 3; ++b) {
        const auto &blob = CrcMath::get(static_cast<CrcType>(t)).device_tables(1 << b);
        OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&c->crc_tables[t][b]), blob.size() * sizeof(uint32_t)));
        OZEC_HIP(hipMemcpy(c->crc_tables[t][b], blob.data(), blob.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
      }
    for (int t = 0; t < 2; ++t)
      for (int i = 0; i < ozec::kG26Slots; ++i) {
        const auto &blob = CrcMath::get(static_cast<CrcType>(t)).g26_tables(i);
        OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&c->g26_tables[t][i]), blob.size() * sizeof(uint32_t)));
        OZEC_HIP(hipMemcpy(c->g26_tables[t][i], blob.data(), blob.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
      }
    for (int t = 0; t < 2; ++t) {
      const auto &blob = CrcMath::get(static_cast<CrcType>(t)).nib_tables();
      OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&c->nib_tables[t]), blob.size() * sizeof(uint32_t)));
      OZEC_HIP(hipMemcpy(c->nib_tables[t], blob.data(), blob.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
      const auto &xo = CrcMath::get(static_cast<CrcType>(t)).xo_tables();
      OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&c->xo_tables[t]), xo.size() * sizeof(uint32_t)));
      OZEC_HIP(hipMemcpy(c->xo_tables[t], xo.data(), xo.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
      const auto &cv = CrcMath::get(static_cast<CrcType>(t)).cv_tables();
      OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&c->cv_tables[t]), cv.size() * sizeof(uint32_t)));
      OZEC_HIP(hipMemcpy(c->cv_tables[t], cv.data(), cv.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
      const auto &bs = CrcMath::get(static_cast<CrcType>(t)).bshift_tables();
      OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&c->bshift_tables[t]), bs.size() * sizeof(uint32_t)));
      OZEC_HIP(hipMemcpy(c->bshift_tables[t], bs.data(), bs.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    g_ctx[dev] = std::move(c);
  }
  *out = g_ctx[dev].get();
  return OZEC_OK;
}

// NULL selects the device's default (null) stream, as in every HIP/CUDA API: work is then ordered with the
// caller's default-stream operations (torch's default stream handle is 0).
hipStream_t pick_stream(DevCtx *, void *stream) { return static_cast<hipStream_t>(stream); }

constexpr size_t kStageAlign = 256;
inline size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

int crc_type_of(int checksum_type, CrcType *t) {
  if (checksum_type == OZEC_CHECKSUM_CRC32) *t = CrcType::kCrc32;
  else if (checksum_type == OZEC_CHECKSUM_CRC32C) *t = CrcType::kCrc32c;
  else return fail(OZEC_EINVAL, "unsupported checksum type " + std::to_string(checksum_type) +
                                    " (GPU path covers CRC32=2 and CRC32C=3)");
  return OZEC_OK;
}

}  // namespace

int ozec::set_error(int code, const std::string &msg) { return fail(code, msg); }

namespace ozec {
OpCounters g_stats[OZEC_NUM_OPS];
thread_local int g_stat_depth = 0;
thread_local bool g_stat_failed = false;
}  // namespace ozec

// ------------------------------------------------------------------------------------------------
// coder handle

struct ozec_coder {
  int device = -1;  // the GPU its host-buffer calls and stripe queues run on (devices.hpp: chosen at creation)
  int codec = OZEC_CODEC_RS;
  int k = 0, p = 0;
  bool decoder = false;
  std::atomic<bool> closed{false};
  std::atomic<int> refs{1};  // owners: the creator, plus one per ozec_coder_retain (a stripe queue holds one)
  std::vector<uint8_t> parity_rows;  // p x k (RS) -- RSRawEncoder's encodeMatrix rows k..k+p-1
  // decode cache on (erased, valid) like RSRawDecoder.prepareDecoding (RSRawDecoder.java:103-115)
  std::mutex cache_mu;
  bool cache_set = false;
  std::vector<int> cached_erased, cached_valid;
  std::vector<uint8_t> cached_rows;
};

namespace {

int check_open(const ozec_coder *c, const char *what) {
  if (!c) return fail(OZEC_EINVAL, "null coder");
  if (c->closed.load()) return fail(OZEC_ECLOSED, std::string(what) + " failed: the coder is closed");
  return OZEC_OK;
}

// Build the rows x k job for a decode: resolves the units to read and the coefficient rows.
// Mirrors DecodingState.checkParameters (DecodingState.java:35-51), ByteBufferDecodingState input checks
// (ByteBufferDecodingState.java:103-130) and RSRawDecoder.prepareDecoding/processErasures.
int plan_decode(ozec_coder *dec, const bool *present, const int *erased, int n_erased, std::vector<int> &read_units,
                std::vector<uint8_t> &rows) {
  const int n_all = dec->k + dec->p;
  if (n_erased > dec->p) return fail(OZEC_EINVAL, "Too many erased, not recoverable");
  if (n_erased < 0 || (n_erased > 0 && !erased)) return fail(OZEC_EINVAL, "erasedIndexes and outputs mismatch in length");
  for (int i = 0; i < n_erased; ++i)
    if (erased[i] < 0 || erased[i] >= n_all)
      return fail(OZEC_EINVAL, "erased index " + std::to_string(erased[i]) + " out of range");
  std::vector<int> valid;
  for (int u = 0; u < n_all; ++u)
    if (present[u]) valid.push_back(u);
  if (static_cast<int>(valid.size()) < dec->k)
    return fail(OZEC_EINVAL, "No enough valid inputs are provided (" + std::to_string(valid.size()) + " vs. " +
                                 std::to_string(dec->k) + "), not recoverable");
  if (dec->codec == OZEC_CODEC_XOR) {
    // XORRawDecoder.doDecode (XORRawDecoder.java:40-86): XOR every slot except erasedIndexes[0]
    if (n_erased == 0) {
      rows.clear();
      read_units.clear();
      return OZEC_OK;
    }
    read_units.clear();
    for (int u = 0; u < n_all; ++u) {
      if (u == erased[0]) continue;
      if (!present[u]) return fail(OZEC_EINVAL, "input " + std::to_string(u) + " is null (XOR decode reads every unit)");
      read_units.push_back(u);
    }
    rows.assign(read_units.size() * static_cast<size_t>(n_erased), 1);
    return OZEC_OK;
  }
  read_units.assign(valid.begin(), valid.begin() + dec->k);
  std::lock_guard<std::mutex> lk(dec->cache_mu);
  std::vector<int> er(erased, erased + n_erased);
  if (!dec->cache_set || er != dec->cached_erased || valid != dec->cached_valid) {
    std::vector<uint8_t> r;
    if (!ozec::decode_matrix(dec->k, dec->p, read_units.data(), erased, n_erased, r))
      return fail(OZEC_ENOTINVERTIBLE, "Not invertible");
    dec->cached_erased = er;
    dec->cached_valid = valid;
    dec->cached_rows = r;
    dec->cache_set = true;
  }
  rows = dec->cached_rows;
  return OZEC_OK;
}

void fill_coef(CodeArgs &a, int rows, int k, const uint8_t *coef) {
  a.unit_map = ozec::g_tune.unit_map;
  a.k = k;
  a.rows = rows;
  std::memcpy(a.coef, coef, static_cast<size_t>(rows) * k);
  a.all_ones = 1;
  for (int i = 0; i < rows * k; ++i) a.all_ones &= coef[i] == 1;
}

int check_limits(int k, int rows) {
  if (k > OZEC_MAX_K || rows > OZEC_MAX_ROWS)
    return fail(OZEC_EUNSUPPORTED, "schema exceeds GPU kernel limits (k <= " + std::to_string(OZEC_MAX_K) +
                                       ", rows <= " + std::to_string(OZEC_MAX_ROWS) + ")");
  return OZEC_OK;
}

// parity rows of an encoder as coefficient rows (XOR: a single all-ones row)
void encode_rows(const ozec_coder *enc, std::vector<uint8_t> &rows) {
  if (enc->codec == OZEC_CODEC_XOR) rows.assign(static_cast<size_t>(enc->k), 1);
  else rows = enc->parity_rows;
}

int out_rows(const ozec_coder *enc) { return enc->codec == OZEC_CODEC_XOR ? 1 : enc->p; }


bool host_pinned(const void *p) {
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return at.type == hipMemoryTypeHost;
}

// the whole [p, p+n) must lie in ONE registered / pinned allocation: both ends pinned, and in the same allocation (two
// separately pinned buffers that happen to be adjacent, or evenly spaced cells of different allocations, are not one
// DMA source: HIP resolves a copy's host range through the allocation of its start)
bool range_pinned(const void *p, size_t n) {
  if (n == 0) return true;
  const uint8_t *last = static_cast<const uint8_t *>(p) + n - 1;
  if (!host_pinned(p) || !host_pinned(last)) return false;
  const void *b = ozec::pinned_alloc_base(p);
  return b != nullptr && b == ozec::pinned_alloc_base(last);
}

// Host-buffer job through one staging slot, pipelined in chunks: while the GPU copies / codes / copies back
// chunk c, this thread stages chunk c+1 (pageable -> pinned) and unstages chunk c-1 (pinned -> pageable).
// Chunk-major staging layout, chunk c at c * per_chunk: [nin inputs x Cp][nout outputs x Op].
//   launch(d_in, in_stride, d_out, out_stride, off, cl, stream) enqueues the kernel for bytes [off, off+cl)
//   out_bytes(cl) / out_pos(off) give the output bytes a chunk produces and where they go in each output
//   gkey (optional): the bytes the launch depends on besides the slot's buffers and the chunk geometry; with it, a
//   call of one staged chunk up to host_graph bytes per unit replays a cached graph of its three stream operations
//   (one graph launch instead of three operations: 45 -> 34 us for a 64 KiB-cell rs-6-3 stripe)
// the address at which the GPU reaches pinned host memory p (registered or hipHostMalloc'ed; the same address on ROCm),
// null when p is not GPU-mapped
uint8_t *dev_view(const void *p) {
  void *dp = nullptr;
  if (hipHostGetDevicePointer(&dp, const_cast<void *>(p), 0) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return static_cast<uint8_t *>(dp);
}

// caller-moved bytes (ozec_encode_cb / ozec_decode_cb): fill puts input bytes [off, off + cl) of every input into the
// staging pointers, drain takes output bytes [off, off + cl) of every output from them; nonzero ends the call
struct HostCopies {
  std::function<int(size_t off, size_t cl, uint8_t *const *dst)> fill;
  std::function<int(size_t off, size_t cl, const uint8_t *const *src)> drain;
};

//   zc: the launch may read and write pinned host memory in place (zero copy, TuneKnobs::host_zero_copy): the kernel
//   reaches the caller's pinned buffers, or the slot's pinned staging, over PCIe, with no H2D / D2H operation
//   cb: the caller moves the bytes (in / out unused): the staged path with its copies replaced by cb's
template <class Launch, class OutBytes, class OutPos>
int staged_pipeline(DevCtx *ctx, int nin, const uint8_t *const *in, size_t len, size_t gran, int nout,
                    uint8_t *const *out, OutBytes out_bytes, OutPos out_pos, Launch launch,
                    const std::vector<uint8_t> *gkey = nullptr, bool zc = false, const HostCopies *cb = nullptr) {
  constexpr size_t kMaxChunks = 64;
  SlotLease lease(ctx);
  if (int rc = ctx->acquire(&lease.slot)) return rc;
  Slot *s = lease.slot;
  // Chunk size: every chunk costs ~20 us of stream-operation latency, so a lone caller does best with few large
  // chunks (host_chunk, 4 MiB per unit: one chunk for 1 MiB cells); with other calls in flight the link and the
  // staging copies are shared, and overlapping the copies of one call's chunks pays (host_chunk_shared, 512 KiB:
  // measured at T = 4 / 16 callers)
  int64_t want = ozec::g_tune.host_chunk.load();
  const int64_t shared_chunk = ozec::g_tune.host_chunk_shared.load();
  if (ctx->leased.load() > 1 && shared_chunk > 0) want = std::min(want, shared_chunk);
  size_t chunk = static_cast<size_t>(std::max<int64_t>(1, want));
  chunk = std::max(chunk, (len + kMaxChunks - 1) / kMaxChunks);
  chunk = std::max(gran, chunk / gran * gran);
  // zero copy for a call alone on the GPU's slots: concurrent callers keep the SDMA copies, which together fill the link
  // (four JNI threads: 52 GB/s through copies, 43 with every call zero-copy, profiles/r06/zero_copy/) -- except small
  // cells (host_zc_shared_max), whose calls are latency-bound and leave the link half idle
  const int64_t zc_small = ozec::g_tune.host_zc_shared_max.load(std::memory_order_relaxed);
  const bool zc_here = ctx->leased.load() <= 1 || (zc_small > 0 && len <= static_cast<size_t>(zc_small));
  const int64_t zc_grid = zc && zc_here ? ozec::g_tune.host_zero_copy.load(std::memory_order_relaxed) : 0;
  // zero copy, one call in one chunk: host_zc_chunks column chunks (2) of at least 256 KiB per unit, so the staging
  // copies of one overlap the kernel on another (1 MiB-cell rs-6-3 stripe from pageable cells 289 -> 239 us; four
  // chunks 360, profiles/r06/percall/)
  const int64_t zch = ozec::g_tune.host_zc_chunks.load(std::memory_order_relaxed);
  if (zc_grid > 0 && zch > 1 && chunk >= len && len >= static_cast<size_t>(zch) * (size_t{256} << 10))
    chunk = std::max(gran, round_up((len + zch - 1) / zch, gran));
  if (chunk >= len) chunk = len;
  const size_t nch = (len + chunk - 1) / chunk;
  const size_t cp = round_up(chunk, kStageAlign), op = round_up(out_bytes(chunk), kStageAlign);
  const size_t per_chunk = nin * cp + nout * op;
  // On an early error return, chunks already queued may still be copying into / out of the slot's buffers:
  // drain the slot's stream before the lease hands the slot to the next caller (declared after the lease, so
  // it runs first).
  struct DrainOnExit {
    Slot *s;
    ~DrainOnExit() {
      (void)hipStreamSynchronize(s->stream);
      if (s->stream2) (void)hipStreamSynchronize(s->stream2);
    }
  } drain{s};
  // Caller buffers that are all pinned (ozec_host_alloc / ozec_host_register; Java: OzecNative.allocatePinned) are
  // DMA'd in place: no staging copy and no chunking.  Units at one constant stride (a buffer pool's cells) go up and
  // come back as one rectangular copy each way; otherwise one copy per unit, which pays only for large cells (each
  // copy is a stream operation of ~10 us; the staging path moves all units in one)
  auto stride_of = [](const uint8_t *const *b, int n, size_t w, int64_t *st) {
    *st = n > 1 ? b[1] - b[0] : static_cast<int64_t>(w);
    if (*st < static_cast<int64_t>(w)) return false;
    for (int i = 2; i < n; ++i)
      if (b[i] - b[i - 1] != *st) return false;
    return true;
  };
  int64_t sin = 0, sout = 0;
  const size_t obytes = out_bytes(len);
  std::vector<const uint8_t *> obase(nout);
  bool rect = false, direct = false;
  if (!cb) {
    for (int r = 0; r < nout; ++r) obase[r] = out[r] + out_pos(0);
    rect = stride_of(in, nin, len, &sin) && stride_of(obase.data(), nout, obytes, &sout);
    direct = rect || len >= (256u << 10);
    if (rect && direct) {
      direct = range_pinned(in[0], static_cast<size_t>(sin) * (nin - 1) + len) &&
               range_pinned(obase[0], static_cast<size_t>(sout) * (nout - 1) + obytes);
    } else {
      for (int j = 0; j < nin && direct; ++j) direct = range_pinned(in[j], len);
      for (int r = 0; r < nout && direct; ++r) direct = range_pinned(obase[r], obytes);
    }
  }
  if (direct && rect && zc_grid > 0) {
    // zero copy (round 6): the kernel reads the caller's pinned inputs and writes its pinned outputs over PCIe -- one
    // launch, no copy operation (HIP's SDMA engines run a copy at the link rate on some streams and at a third of it
    // on others, profiles/r06/engines/)
    uint8_t *din = dev_view(in[0]), *dout = dev_view(obase[0]);
    if (din && dout) {
      ozec::GridCap cap(zc_grid);
      OZEC_HIP(launch(din, sin, dout, sout, 0, len, s->stream));
      OZEC_HIP(hipStreamSynchronize(s->stream));
      return OZEC_OK;
    }
  }
  if (direct) {
    const size_t dcp = round_up(len, kStageAlign), dop = round_up(obytes, kStageAlign);
    if (int rc = s->reserve_device(nin * dcp + nout * dop)) return rc;
    uint8_t *d = s->dbuf;
    // Duplex (coding calls of large cells): the units go up, through the kernel and back in column chunks, the D2H
    // of chunk c on the slot's second stream while the H2D of chunk c+1 runs on the first, so the two link
    // directions overlap inside one call instead of running one after the other (a lone writer's 1 MiB-cell stripe:
    // 6 MiB up, 3 MiB down).  Coding is byte-position-wise, so a column chunk is a complete call of its own.
    const int64_t duplex = ozec::g_tune.host_duplex.load(std::memory_order_relaxed);
    if (duplex > 0 && len >= static_cast<size_t>(duplex) && obytes == len && out_pos(0) == 0) {
      const size_t cw = std::max<size_t>(256u << 10, round_up((len + 7) / 8, 4096));
      const size_t nc = (len + cw - 1) / cw;
      if (!s->stream2) OZEC_HIP(ozec::make_stream(&s->stream2));
      if (int rc = s->ensure_events(nc)) return rc;
      for (size_t c = 0; c < nc; ++c) {
        const size_t off = c * cw, cl = std::min(cw, len - off);
        if (rect) {
          OZEC_HIP(hipMemcpy2DAsync(d + off, dcp, in[0] + off, static_cast<size_t>(sin), cl, nin, hipMemcpyHostToDevice,
                                    s->stream));
        } else {
          for (int j = 0; j < nin; ++j)
            OZEC_HIP(hipMemcpyAsync(d + j * dcp + off, in[j] + off, cl, hipMemcpyHostToDevice, s->stream));
        }
        OZEC_HIP(launch(d + off, static_cast<int64_t>(dcp), d + nin * dcp + off, static_cast<int64_t>(dop), off, cl,
                        s->stream));
        OZEC_HIP(hipEventRecord(s->events[c], s->stream));
        OZEC_HIP(hipStreamWaitEvent(s->stream2, s->events[c], 0));
        if (rect) {
          OZEC_HIP(hipMemcpy2DAsync(const_cast<uint8_t *>(obase[0]) + off, static_cast<size_t>(sout), d + nin * dcp + off,
                                    dop, cl, nout, hipMemcpyDeviceToHost, s->stream2));
        } else {
          for (int r = 0; r < nout; ++r)
            OZEC_HIP(hipMemcpyAsync(const_cast<uint8_t *>(obase[r]) + off, d + nin * dcp + r * dop + off, cl,
                                    hipMemcpyDeviceToHost, s->stream2));
        }
      }
      OZEC_HIP(hipStreamSynchronize(s->stream2));
      return OZEC_OK;
    }
    if (rect) {
      OZEC_HIP(hipMemcpy2DAsync(d, dcp, in[0], static_cast<size_t>(sin), len, nin, hipMemcpyHostToDevice, s->stream));
    } else {
      for (int j = 0; j < nin; ++j) OZEC_HIP(hipMemcpyAsync(d + j * dcp, in[j], len, hipMemcpyHostToDevice, s->stream));
    }
    OZEC_HIP(launch(d, static_cast<int64_t>(dcp), d + nin * dcp, static_cast<int64_t>(dop), 0, len, s->stream));
    if (rect) {
      OZEC_HIP(hipMemcpy2DAsync(const_cast<uint8_t *>(obase[0]), static_cast<size_t>(sout), d + nin * dcp, dop, obytes,
                                nout, hipMemcpyDeviceToHost, s->stream));
    } else {
      for (int r = 0; r < nout; ++r)
        OZEC_HIP(hipMemcpyAsync(const_cast<uint8_t *>(obase[r]), d + nin * dcp + r * dop, obytes, hipMemcpyDeviceToHost,
                                s->stream));
    }
    OZEC_HIP(hipStreamSynchronize(s->stream));
    return OZEC_OK;
  }
  if (int rc = s->reserve(per_chunk * nch, nch, zc_grid <= 0)) return rc;
  // other calls in flight: their copies and DMA share host DRAM with this call's staging copies (copy_pool.hpp)
  const bool shared = ctx->leased.load() > 1 || nch > 1;
  auto unstage = [&](size_t c) -> int {
    OZEC_HIP(hipEventSynchronize(s->events[c]));
    const size_t off = c * chunk, cl = std::min(chunk, len - off);
    const uint8_t *src = s->pinned + c * per_chunk + nin * cp;
    if (cb) {
      std::vector<const uint8_t *> srcs(nout);
      for (int r = 0; r < nout; ++r) srcs[r] = src + r * op;
      return cb->drain(off, cl, srcs.data());
    }
    std::vector<ozec::CopyTask> tasks;
    for (int r = 0; r < nout; ++r) tasks.push_back({out[r] + out_pos(off), src + r * op, out_bytes(cl)});
    ozec::parallel_copy(tasks, ozec::CopyDir::kFromStaging, shared, ctx->numa);
    return OZEC_OK;
  };
  // chunk c's inputs into the staging at h
  auto stage = [&](size_t c, uint8_t *h) -> int {
    const size_t off = c * chunk, cl = std::min(chunk, len - off);
    if (cb) {
      std::vector<uint8_t *> dsts(nin);
      for (int j = 0; j < nin; ++j) dsts[j] = h + j * cp;
      return cb->fill(off, cl, dsts.data());
    }
    std::vector<ozec::CopyTask> tasks;
    for (int j = 0; j < nin; ++j) tasks.push_back({h + j * cp, in[j] + off, cl});
    ozec::parallel_copy(tasks, ozec::CopyDir::kToStaging, shared, ctx->numa);
    return OZEC_OK;
  };
  if (zc_grid > 0) {
    // zero copy from the slot's pinned staging: stage chunk c, one kernel launch on it in place, unstage chunk c - 1
    // while the kernel runs
    uint8_t *hz = dev_view(s->pinned);
    if (hz) {
      ozec::GridCap cap(zc_grid);
      for (size_t c = 0; c < nch; ++c) {
        const size_t off = c * chunk, cl = std::min(chunk, len - off);
        uint8_t *h = s->pinned + c * per_chunk, *hd = hz + c * per_chunk;
        if (int rc = stage(c, h)) return rc;
        OZEC_HIP(launch(hd, static_cast<int64_t>(cp), hd + nin * cp, static_cast<int64_t>(op), off, cl, s->stream));
        OZEC_HIP(hipEventRecord(s->events[c], s->stream));
        if (c > 0)
          if (int rc = unstage(c - 1)) return rc;
      }
      return unstage(nch - 1);
    }
    if (int rc = s->reserve(per_chunk * nch, nch, true)) return rc;  // not GPU-mapped: the copy path below
  }
  const int64_t graph_max = ozec::g_tune.host_graph.load(std::memory_order_relaxed);
  if (gkey && nch == 1 && graph_max > 0 && len <= static_cast<size_t>(graph_max)) {
    std::vector<uint8_t> key = *gkey;
    const size_t geo[5] = {len, static_cast<size_t>(nin), static_cast<size_t>(nout), cp, op};
    key.insert(key.end(), reinterpret_cast<const uint8_t *>(geo), reinterpret_cast<const uint8_t *>(geo + 5));
    hipGraphExec_t ex = s->find_graph(key);
    uint8_t *h = s->pinned, *d = s->dbuf;
    if (!ex) {  // capture the chunk's three operations once; any failure falls back to the plain operations
      hipGraph_t g = nullptr;
      bool ok = hipStreamBeginCapture(s->stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
      if (ok) {
        ok = hipMemcpyAsync(d, h, nin * cp, hipMemcpyHostToDevice, s->stream) == hipSuccess &&
             launch(d, static_cast<int64_t>(cp), d + nin * cp, static_cast<int64_t>(op), 0, len, s->stream) == hipSuccess &&
             hipMemcpyAsync(h + nin * cp, d + nin * cp, nout * op, hipMemcpyDeviceToHost, s->stream) == hipSuccess;
        ok = hipStreamEndCapture(s->stream, &g) == hipSuccess && ok && g != nullptr;
      }
      if (ok) ok = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) == hipSuccess;
      if (g) (void)hipGraphDestroy(g);
      (void)hipGetLastError();
      if (ok) {
        s->keep_graph(std::move(key), ex);
      } else {
        ex = nullptr;
      }
    }
    if (ex) {
      if (int rc = stage(0, h)) return rc;
      OZEC_HIP(hipGraphLaunch(ex, s->stream));
      OZEC_HIP(hipEventRecord(s->events[0], s->stream));
      return unstage(0);
    }
  }
  for (size_t c = 0; c < nch; ++c) {
    const size_t off = c * chunk, cl = std::min(chunk, len - off);
    uint8_t *h = s->pinned + c * per_chunk, *d = s->dbuf + c * per_chunk;
    if (int rc = stage(c, h)) return rc;
    OZEC_HIP(hipMemcpyAsync(d, h, nin * cp, hipMemcpyHostToDevice, s->stream));
    OZEC_HIP(launch(d, static_cast<int64_t>(cp), d + nin * cp, static_cast<int64_t>(op), off, cl, s->stream));
    OZEC_HIP(hipMemcpyAsync(h + nin * cp, d + nin * cp, nout * op, hipMemcpyDeviceToHost, s->stream));
    OZEC_HIP(hipEventRecord(s->events[c], s->stream));
    if (c > 0)
      if (int rc = unstage(c - 1)) return rc;
  }
  return unstage(nch - 1);
}

// host-buffer coding job (encode / decode): rows outputs from nin inputs
int staged_code(DevCtx *ctx, const CodeArgs &tmpl, const uint8_t *const *in, uint8_t *const *out, size_t len,
                const HostCopies *cb = nullptr) {
  // graph key: the coding parameters the kernel launch reads (the pointers and offsets are the slot's, set below)
  std::vector<uint8_t> key;
  auto put = [&key](const void *p, size_t n) {
    key.insert(key.end(), static_cast<const uint8_t *>(p), static_cast<const uint8_t *>(p) + n);
  };
  const int32_t hdr[5] = {tmpl.k, tmpl.rows, tmpl.all_ones, tmpl.unit_map,
                          ozec::g_tune.gf_variant.load(std::memory_order_relaxed)};
  put(hdr, sizeof(hdr));
  put(tmpl.coef, static_cast<size_t>(tmpl.k) * tmpl.rows * sizeof(tmpl.coef[0]));
  const int64_t tail[2] = {ozec::g_tune.grid.load(std::memory_order_relaxed), tmpl.grp_stripes};
  put(tail, sizeof(tail));
  return staged_pipeline(
      ctx, tmpl.k, in, len, 4096, tmpl.rows, out, [](size_t cl) { return cl; }, [](size_t off) { return off; },
      [&](uint8_t *d_in, int64_t in_stride, uint8_t *d_out, int64_t out_stride, size_t, size_t cl, hipStream_t st) {
        CodeArgs a = tmpl;
        a.in = d_in;
        a.out = d_out;
        a.nstripes = 1;
        a.len = static_cast<int64_t>(cl);
        for (int j = 0; j < a.k; ++j) a.in_off[j] = j * in_stride;
        for (int r = 0; r < a.rows; ++r) a.out_off[r] = r * out_stride;
        return ozec::launch_code(a, st);
      },
      &key, true, cb);
}

}  // namespace

extern "C" {

const char *ozec_last_error(void) { return g_error.c_str(); }

int ozec_version(void) { return 1; }

int ozec_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int ozec_set_device(int device) {
  OZEC_HIP(hipSetDevice(device));
  (void)ozec::note_set_device();
  return OZEC_OK;
}

int ozec_set_devices(const int *devices, int n) {
  if (int rc = ozec::set_device_list(devices, n))
    return fail(rc, rc == OZEC_EDEVICE ? "no such device in the list" : "invalid device list");
  return OZEC_OK;
}

int ozec_get_devices(int *devices, int cap) {
  const std::vector<int> l = ozec::device_list();
  for (size_t i = 0; i < l.size() && static_cast<int>(i) < cap; ++i)
    if (devices) devices[i] = l[i];
  return static_cast<int>(l.size());
}

int ozec_set_device_policy(int policy) {
  if (ozec::set_device_policy(policy)) return fail(OZEC_EINVAL, "unknown device policy " + std::to_string(policy));
  return OZEC_OK;
}

int ozec_device_policy(void) { return ozec::device_policy(); }

int ozec_synchronize(void) {
  OZEC_HIP(hipDeviceSynchronize());
  return OZEC_OK;
}

static int coder_create(int codec, int k, int p, bool decoder, ozec_coder **out) {
  if (!out) return fail(OZEC_EINVAL, "null output handle");
  *out = nullptr;
  if (codec != OZEC_CODEC_RS && codec != OZEC_CODEC_XOR) return fail(OZEC_EINVAL, "unknown codec");
  if (k <= 0 || p <= 0)
    return fail(OZEC_EINVAL, "Data and parity part in EC replication config supposed to be positive numbers");
  // RSRawEncoder.java:42-45 / RSRawDecoder.java:61-64
  if (codec == OZEC_CODEC_RS && k + p >= 256) return fail(OZEC_EINVAL, "Invalid numDataUnits and numParityUnits");
  if (int rc = check_limits(k, codec == OZEC_CODEC_XOR ? 1 : p)) return rc;
  // a GPU coder must not be constructible without a device, so CodecUtil falls back to rs_java
  // (CodecUtil.createRawEncoderWithFallback, CodecUtil.java:62-78)
  const int dev = ozec::pick_device();
  if (dev < 0) return fail(OZEC_EDEVICE, "no HIP device available");
  ozec::DeviceScope ds(dev);
  if (!ds.ok()) return fail(OZEC_EDEVICE, "cannot select device " + std::to_string(dev));
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  auto *c = new (std::nothrow) ozec_coder();
  if (!c) return fail(OZEC_ENOMEM, "out of memory");
  c->device = dev;
  c->codec = codec;
  c->k = k;
  c->p = p;
  c->decoder = decoder;
  if (codec == OZEC_CODEC_RS) {
    std::vector<uint8_t> m = ozec::cauchy_matrix(k, p);
    c->parity_rows.assign(m.begin() + static_cast<size_t>(k) * k, m.end());
  }
  *out = c;
  return OZEC_OK;
}

int ozec_encoder_create(int codec, int k, int p, ozec_coder **out) { return coder_create(codec, k, p, false, out); }
int ozec_decoder_create(int codec, int k, int p, ozec_coder **out) { return coder_create(codec, k, p, true, out); }

int ozec_coder_release(ozec_coder *c) {
  if (!c) return fail(OZEC_EINVAL, "null coder");
  c->closed.store(true);
  return OZEC_OK;
}

void ozec_coder_free(ozec_coder *c) {
  if (c && c->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete c;
}

int ozec_release_staging(void) {
  std::vector<DevCtx *> ctxs;
  {
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    for (auto &c : g_ctx)
      if (c) ctxs.push_back(c.get());
  }
  for (DevCtx *ctx : ctxs) {  // every GPU this process has used
    ozec::DeviceScope ds(ctx->device);
    {
      std::lock_guard<std::mutex> lk(ctx->e2e.mu);
      ctx->e2e.shrink();
    }
    std::lock_guard<std::mutex> lk(ctx->pool_mu);
    for (Slot *s : ctx->free_slots) s->shrink();  // leased slots keep theirs until their call returns
  }
  return OZEC_OK;
}

int ozec_coder_retain(ozec_coder *c) {
  if (!c) return fail(OZEC_EINVAL, "null coder");
  c->refs.fetch_add(1, std::memory_order_relaxed);
  return OZEC_OK;
}

int ozec_coder_is_closed(const ozec_coder *c) { return c && c->closed.load() ? 1 : 0; }

int ozec_coder_device(const ozec_coder *c) {
  if (!c) return fail(OZEC_EINVAL, "null coder");
  return c->device;
}

int ozec_coder_info(const ozec_coder *c, int *codec, int *k, int *p, int *is_decoder) {
  if (!c) return fail(OZEC_EINVAL, "null coder");
  if (codec) *codec = c->codec;
  if (k) *k = c->k;
  if (p) *p = c->p;
  if (is_decoder) *is_decoder = c->decoder;
  return OZEC_OK;
}

// ---- encode ------------------------------------------------------------------------------------

int ozec_encode(ozec_coder *enc, const uint8_t *const *inputs, uint8_t *const *outputs, size_t len) {
  ozec::StatScope stat_(OZEC_OP_ENCODE, enc ? static_cast<uint64_t>(enc->k) * len : 0);
  if (int rc = check_open(enc, "encode")) return rc;
  if (enc->decoder) return fail(OZEC_EINVAL, "not an encoder");
  if (!inputs || !outputs) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  const int k = enc->k, rows = out_rows(enc);
  for (int j = 0; j < k; ++j)
    if (!inputs[j]) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  for (int r = 0; r < rows; ++r)
    if (!outputs[r]) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  if (len == 0) return OZEC_OK;  // RawErasureEncoder.java:73-75
  ozec::DeviceScope ds(enc->device);  // the coder's GPU (devices.hpp)
  if (!ds.ok()) return fail(OZEC_EDEVICE, "cannot select device " + std::to_string(enc->device));
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  CodeArgs a{};
  std::vector<uint8_t> coef;
  encode_rows(enc, coef);
  fill_coef(a, rows, k, coef.data());
  if (int rc = staged_code(ctx, a, inputs, outputs, len)) return rc;
  // XOR with p > 1: the reference zero-fills every output and writes only outputs[0] (XORRawEncoder.java:67-85)
  for (int r = rows; r < enc->p; ++r)
    if (outputs[r]) std::memset(outputs[r], 0, len);
  return OZEC_OK;
}

int ozec_encode_device(ozec_coder *enc, const uint8_t *const *d_inputs, uint8_t *const *d_outputs, size_t len,
                       void *stream) {
  ozec::StatScope stat_(OZEC_OP_ENCODE_DEVICE, enc ? static_cast<uint64_t>(enc->k) * len : 0);
  if (int rc = check_open(enc, "encode")) return rc;
  if (enc->decoder) return fail(OZEC_EINVAL, "not an encoder");
  if (!d_inputs || !d_outputs) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  const int k = enc->k, rows = out_rows(enc);
  for (int j = 0; j < k; ++j)
    if (!d_inputs[j]) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  for (int r = 0; r < rows; ++r)
    if (!d_outputs[r]) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  if (len == 0) return OZEC_OK;
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  CodeArgs a{};
  a.nstripes = 1;
  a.len = static_cast<int64_t>(len);
  std::vector<uint8_t> coef;
  encode_rows(enc, coef);
  fill_coef(a, rows, k, coef.data());
  for (int j = 0; j < k; ++j) a.in_off[j] = reinterpret_cast<intptr_t>(d_inputs[j]);
  for (int r = 0; r < rows; ++r) a.out_off[r] = reinterpret_cast<intptr_t>(d_outputs[r]);
  hipStream_t st = pick_stream(ctx, stream);
  OZEC_HIP(ozec::launch_code(a, st));
  for (int r = rows; r < enc->p; ++r)
    if (d_outputs[r]) OZEC_HIP(hipMemsetAsync(d_outputs[r], 0, len, st));
  return OZEC_OK;
}

int ozec_encode_batch(ozec_coder *enc, const uint8_t *d_in, int64_t in_stripe_stride, int64_t in_unit_stride,
                      uint8_t *d_out, int64_t out_stripe_stride, int64_t out_unit_stride, size_t num_stripes,
                      size_t len, void *stream) {
  ozec::StatScope stat_(OZEC_OP_ENCODE_DEVICE, enc ? static_cast<uint64_t>(enc->k) * len * num_stripes : 0);
  if (int rc = check_open(enc, "encode")) return rc;
  if (enc->decoder) return fail(OZEC_EINVAL, "not an encoder");
  if (len == 0 || num_stripes == 0) return OZEC_OK;
  if (!d_in || !d_out) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  const int k = enc->k, rows = out_rows(enc);
  CodeArgs a{};
  a.in = d_in;
  a.out = d_out;
  a.in_stripe_stride = in_stripe_stride;
  a.out_stripe_stride = out_stripe_stride;
  a.nstripes = static_cast<int64_t>(num_stripes);
  a.len = static_cast<int64_t>(len);
  std::vector<uint8_t> coef;
  encode_rows(enc, coef);
  fill_coef(a, rows, k, coef.data());
  for (int j = 0; j < k; ++j) a.in_off[j] = j * in_unit_stride;
  for (int r = 0; r < rows; ++r) a.out_off[r] = r * out_unit_stride;
  hipStream_t st = pick_stream(ctx, stream);
  OZEC_HIP(ozec::launch_code(a, st));
  for (int r = rows; r < enc->p; ++r)
    OZEC_HIP(hipMemset2DAsync(d_out + r * out_unit_stride, out_stripe_stride, 0, len, num_stripes, st));
  return OZEC_OK;
}

// ---- decode ------------------------------------------------------------------------------------

int ozec_decode(ozec_coder *dec, const uint8_t *const *inputs, const int *erased, int n_erased,
                uint8_t *const *outputs, size_t len) {
  ozec::StatScope stat_(OZEC_OP_DECODE, dec ? static_cast<uint64_t>(dec->k) * len : 0);
  if (int rc = check_open(dec, "decode")) return rc;
  if (!dec->decoder) return fail(OZEC_EINVAL, "not a decoder");
  if (!inputs) return fail(OZEC_EINVAL, "Invalid inputs length");
  const int n_all = dec->k + dec->p;
  bool present[256];
  bool any = false;
  for (int u = 0; u < n_all; ++u) any |= (present[u] = inputs[u] != nullptr);
  if (!any) return fail(OZEC_EINVAL, "Invalid inputs are found, all being null");
  for (int i = 0; i < n_erased; ++i)
    if (!outputs || !outputs[i]) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  std::vector<int> units;
  std::vector<uint8_t> rows;
  if (int rc = plan_decode(dec, present, erased, n_erased, units, rows)) return rc;
  if (len == 0 || n_erased == 0) return OZEC_OK;
  const int nin = static_cast<int>(units.size());
  ozec::DeviceScope ds(dec->device);  // the coder's GPU (devices.hpp)
  if (!ds.ok()) return fail(OZEC_EDEVICE, "cannot select device " + std::to_string(dec->device));
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  CodeArgs a{};
  if (dec->codec == OZEC_CODEC_XOR) fill_coef(a, 1, nin, rows.data());
  else fill_coef(a, n_erased, nin, rows.data());
  if (int rc = check_limits(a.k, a.rows)) return rc;
  std::vector<const uint8_t *> in(nin);
  for (int j = 0; j < nin; ++j) in[j] = inputs[units[j]];
  if (int rc = staged_code(ctx, a, in.data(), outputs, len)) return rc;
  // XOR decode: only erasedIndexes[0] is recovered, further outputs stay zero-filled (XORRawDecoder.java:45-61)
  for (int r = a.rows; r < n_erased; ++r) std::memset(outputs[r], 0, len);
  return OZEC_OK;
}

// ---- host coding with caller-moved bytes (round 6; the JNI glue's heap arrays) --------------------------------

int ozec_encode_cb(ozec_coder *enc, size_t len, ozec_fill_fn fill, ozec_drain_fn drain, void *user) {
  ozec::StatScope stat_(OZEC_OP_ENCODE, enc ? static_cast<uint64_t>(enc->k) * len : 0);
  if (int rc = check_open(enc, "encode")) return rc;
  if (enc->decoder) return fail(OZEC_EINVAL, "not an encoder");
  if (!fill || !drain) return fail(OZEC_EINVAL, "null copy callback");
  if (len == 0) return OZEC_OK;
  const int k = enc->k, rows = out_rows(enc), p = enc->p;
  ozec::DeviceScope ds(enc->device);
  if (!ds.ok()) return fail(OZEC_EDEVICE, "cannot select device " + std::to_string(enc->device));
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  CodeArgs a{};
  std::vector<uint8_t> coef;
  encode_rows(enc, coef);
  fill_coef(a, rows, k, coef.data());
  // XOR with p > 1: the outputs past the first are zero (XORRawEncoder.java:67-85): drained from a zero block
  std::vector<uint8_t> zeros;
  HostCopies cb;
  cb.fill = [&](size_t off, size_t cl, uint8_t *const *dst) { return fill(user, off, cl, dst); };
  cb.drain = [&](size_t off, size_t cl, const uint8_t *const *src) {
    if (rows == p) return drain(user, off, cl, src);
    if (zeros.size() < cl) zeros.assign(cl, 0);
    std::vector<const uint8_t *> all(static_cast<size_t>(p), zeros.data());
    for (int r = 0; r < rows; ++r) all[r] = src[r];
    return drain(user, off, cl, all.data());
  };
  if (int rc = staged_code(ctx, a, nullptr, nullptr, len, &cb)) return rc;
  return OZEC_OK;
}

int ozec_decode_cb(ozec_coder *dec, const uint8_t *present_units, const int *erased, int n_erased, size_t len,
                   ozec_fill_fn fill, ozec_drain_fn drain, void *user) {
  ozec::StatScope stat_(OZEC_OP_DECODE, dec ? static_cast<uint64_t>(dec->k) * len : 0);
  if (int rc = check_open(dec, "decode")) return rc;
  if (!dec->decoder) return fail(OZEC_EINVAL, "not a decoder");
  if (!present_units) return fail(OZEC_EINVAL, "Invalid inputs length");
  if (!fill || !drain) return fail(OZEC_EINVAL, "null copy callback");
  const int n_all = dec->k + dec->p;
  bool present[256];
  bool any = false;
  for (int u = 0; u < n_all; ++u) any |= (present[u] = present_units[u] != 0);
  if (!any) return fail(OZEC_EINVAL, "Invalid inputs are found, all being null");
  std::vector<int> units;
  std::vector<uint8_t> rows;
  if (int rc = plan_decode(dec, present, erased, n_erased, units, rows)) return rc;
  if (len == 0 || n_erased == 0) return OZEC_OK;
  const int nin = static_cast<int>(units.size());
  ozec::DeviceScope ds(dec->device);
  if (!ds.ok()) return fail(OZEC_EDEVICE, "cannot select device " + std::to_string(dec->device));
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  CodeArgs a{};
  if (dec->codec == OZEC_CODEC_XOR) fill_coef(a, 1, nin, rows.data());
  else fill_coef(a, n_erased, nin, rows.data());
  if (int rc = check_limits(a.k, a.rows)) return rc;
  std::vector<uint8_t> zeros;
  HostCopies cb;
  // fill sees every unit's slot (k + p, null for the units not read), as ozec_decode's inputs
  cb.fill = [&](size_t off, size_t cl, uint8_t *const *dst) {
    std::vector<uint8_t *> by_unit(static_cast<size_t>(n_all), nullptr);
    for (int j = 0; j < nin; ++j) by_unit[units[j]] = dst[j];
    return fill(user, off, cl, by_unit.data());
  };
  // XOR decode: only erasedIndexes[0] is recovered, the other outputs are zero (XORRawDecoder.java:45-61)
  cb.drain = [&](size_t off, size_t cl, const uint8_t *const *src) {
    if (a.rows == n_erased) return drain(user, off, cl, src);
    if (zeros.size() < cl) zeros.assign(cl, 0);
    std::vector<const uint8_t *> all(static_cast<size_t>(n_erased), zeros.data());
    for (int r = 0; r < a.rows; ++r) all[r] = src[r];
    return drain(user, off, cl, all.data());
  };
  if (int rc = staged_code(ctx, a, nullptr, nullptr, len, &cb)) return rc;
  return OZEC_OK;
}

int ozec_decode_device(ozec_coder *dec, const uint8_t *const *d_inputs, const int *erased, int n_erased,
                       uint8_t *const *d_outputs, size_t len, void *stream) {
  ozec::StatScope stat_(OZEC_OP_DECODE_DEVICE, dec ? static_cast<uint64_t>(dec->k) * len : 0);
  if (int rc = check_open(dec, "decode")) return rc;
  if (!dec->decoder) return fail(OZEC_EINVAL, "not a decoder");
  if (!d_inputs) return fail(OZEC_EINVAL, "Invalid inputs length");
  const int n_all = dec->k + dec->p;
  bool present[256];
  bool any = false;
  for (int u = 0; u < n_all; ++u) any |= (present[u] = d_inputs[u] != nullptr);
  if (!any) return fail(OZEC_EINVAL, "Invalid inputs are found, all being null");
  for (int i = 0; i < n_erased; ++i)
    if (!d_outputs || !d_outputs[i]) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  std::vector<int> units;
  std::vector<uint8_t> rows;
  if (int rc = plan_decode(dec, present, erased, n_erased, units, rows)) return rc;
  if (len == 0 || n_erased == 0) return OZEC_OK;
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  CodeArgs a{};
  a.nstripes = 1;
  a.len = static_cast<int64_t>(len);
  const int nin = static_cast<int>(units.size());
  if (dec->codec == OZEC_CODEC_XOR) fill_coef(a, 1, nin, rows.data());
  else fill_coef(a, n_erased, nin, rows.data());
  if (int rc = check_limits(a.k, a.rows)) return rc;
  for (int j = 0; j < nin; ++j) a.in_off[j] = reinterpret_cast<intptr_t>(d_inputs[units[j]]);
  for (int r = 0; r < a.rows; ++r) a.out_off[r] = reinterpret_cast<intptr_t>(d_outputs[r]);
  OZEC_HIP(ozec::launch_code(a, st));
  for (int r = a.rows; r < n_erased; ++r) OZEC_HIP(hipMemsetAsync(d_outputs[r], 0, len, st));
  return OZEC_OK;
}

int ozec_decode_batch(ozec_coder *dec, const uint8_t *d_in, int64_t in_stripe_stride, int64_t in_unit_stride,
                      const int *present_units, int num_present, const int *erased, int n_erased, uint8_t *d_out,
                      int64_t out_stripe_stride, int64_t out_unit_stride, size_t num_stripes, size_t len,
                      void *stream) {
  ozec::StatScope stat_(OZEC_OP_DECODE_DEVICE, dec ? static_cast<uint64_t>(dec->k) * len * num_stripes : 0);
  if (int rc = check_open(dec, "decode")) return rc;
  if (!dec->decoder) return fail(OZEC_EINVAL, "not a decoder");
  const int n_all = dec->k + dec->p;
  bool present[256] = {false};
  for (int i = 0; i < num_present; ++i) {
    if (present_units[i] < 0 || present_units[i] >= n_all) return fail(OZEC_EINVAL, "present unit out of range");
    present[present_units[i]] = true;
  }
  std::vector<int> units;
  std::vector<uint8_t> rows;
  if (int rc = plan_decode(dec, present, erased, n_erased, units, rows)) return rc;
  if (len == 0 || num_stripes == 0 || n_erased == 0) return OZEC_OK;
  if (!d_in || !d_out) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  CodeArgs a{};
  a.in = d_in;
  a.out = d_out;
  a.in_stripe_stride = in_stripe_stride;
  a.out_stripe_stride = out_stripe_stride;
  a.nstripes = static_cast<int64_t>(num_stripes);
  a.len = static_cast<int64_t>(len);
  const int nin = static_cast<int>(units.size());
  if (dec->codec == OZEC_CODEC_XOR) fill_coef(a, 1, nin, rows.data());
  else fill_coef(a, n_erased, nin, rows.data());
  if (int rc = check_limits(a.k, a.rows)) return rc;
  for (int j = 0; j < nin; ++j) a.in_off[j] = units[j] * in_unit_stride;
  for (int r = 0; r < a.rows; ++r) a.out_off[r] = r * out_unit_stride;
  OZEC_HIP(ozec::launch_code(a, st));
  for (int r = a.rows; r < n_erased; ++r)
    OZEC_HIP(hipMemset2DAsync(d_out + r * out_unit_stride, out_stripe_stride, 0, len, num_stripes, st));
  return OZEC_OK;
}

// ---- checksums -----------------------------------------------------------------------------------

static int make_crc_args(DevCtx *ctx, int checksum_type, const uint8_t *d_base, int64_t cell_stride, size_t ncells,
                         size_t len, size_t bpc, uint32_t *d_out, int64_t out_cell_stride, int big_endian, int raw,
                         CrcArgs *a) {
  CrcType t;
  if (int rc = crc_type_of(checksum_type, &t)) return rc;
  if (bpc == 0) return fail(OZEC_EINVAL, "bytesPerChecksum must be positive");
  const CrcMath &cm = CrcMath::get(t);
  *a = CrcArgs{};
  a->base = d_base;
  a->cell_stride = cell_stride;
  a->ncells = static_cast<int64_t>(ncells);
  a->len = static_cast<int64_t>(len);
  a->bpc = static_cast<int64_t>(bpc);
  a->nwin = static_cast<int64_t>((len + bpc - 1) / bpc);
  a->out = d_out;
  a->out_cell_stride = out_cell_stride;
  for (int b = 0; b < 3; ++b) a->tables[b] = ctx->crc_tables[static_cast<int>(t)][b];
  for (int i = 0; i < ozec::kG26Slots; ++i) a->g26[i] = ctx->g26_tables[static_cast<int>(t)][i];
  a->nib = ctx->nib_tables[static_cast<int>(t)];
  a->xo = ctx->xo_tables[static_cast<int>(t)];
  a->cv = ctx->cv_tables[static_cast<int>(t)];
  a->bshift = nullptr;  // the run check's shift by bpc: bpc = 4 KiB << i only
  for (int i = 0; i < ozec::kBshiftN; ++i)
    if (bpc == (size_t{4096} << i)) a->bshift = ctx->bshift_tables[static_cast<int>(t)] + i * 224;
  a->init_full = cm.shift(0xffffffffu, bpc);
  a->init_last = cm.shift(0xffffffffu, len - (a->nwin ? (a->nwin - 1) * bpc : 0));
  a->big_endian = big_endian;
  a->raw = raw;
  a->poly = cm.poly();
  a->unit_map = ozec::g_tune.unit_map;
  return OZEC_OK;
}

int ozec_checksum_windows_batch(int checksum_type, const uint8_t *d_base, int64_t cell_stride, size_t num_cells,
                                size_t len, size_t bpc, uint32_t *d_out, int big_endian, void *stream) {
  ozec::StatScope stat_(OZEC_OP_CHECKSUM_DEVICE, static_cast<uint64_t>(len) * num_cells);
  if (len == 0 || num_cells == 0) return OZEC_OK;
  if (!d_base || !d_out) return fail(OZEC_EINVAL, "null buffer");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  CrcArgs a;
  const int64_t nwin = static_cast<int64_t>((len + (bpc ? bpc : 1) - 1) / (bpc ? bpc : 1));
  if (int rc = make_crc_args(ctx, checksum_type, d_base, cell_stride, num_cells, len, bpc, d_out, nwin, big_endian, 0,
                             &a))
    return rc;
  OZEC_HIP(ozec::launch_crc_windows(a, pick_stream(ctx, stream)));
  return OZEC_OK;
}

int ozec_checksum_windows_device(int checksum_type, const uint8_t *d_data, size_t len, size_t bpc, uint32_t *d_out,
                                 int big_endian, void *stream) {
  return ozec_checksum_windows_batch(checksum_type, d_data, 0, 1, len, bpc, d_out, big_endian, stream);
}

// host buffers: stage -> GPU -> copy back; `raw` returns the raw registers (streaming update)
static int checksum_host(int checksum_type, const uint8_t *data, size_t len, size_t bpc, uint32_t *out, int big_endian,
                         int raw) {
  CrcType t;
  if (int rc = crc_type_of(checksum_type, &t)) return rc;
  if (bpc == 0) return fail(OZEC_EINVAL, "bytesPerChecksum must be positive");
  if (len == 0) return OZEC_OK;
  if (!data || !out) return fail(OZEC_EINVAL, "null buffer");
  ozec::DeviceScope ds(ozec::thread_device());  // coder-less host call: this thread's GPU (devices.hpp)
  if (!ds.ok()) return fail(OZEC_EDEVICE, "cannot select this thread's device");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  uint8_t *outs[1] = {reinterpret_cast<uint8_t *>(out)};
  // chunks are whole windows, so every chunk's windows are the call's windows
  const size_t gran = bpc >= 4096 ? bpc : (4096 + bpc - 1) / bpc * bpc;
  return staged_pipeline(
      ctx, 1, &data, len, gran, 1, outs, [bpc](size_t cl) { return (cl + bpc - 1) / bpc * sizeof(uint32_t); },
      [bpc](size_t off) { return off / bpc * sizeof(uint32_t); },
      [&](uint8_t *d_in, int64_t, uint8_t *d_out, int64_t, size_t, size_t cl, hipStream_t st) {
        CrcArgs a;
        const int64_t nw = static_cast<int64_t>((cl + bpc - 1) / bpc);
        if (make_crc_args(ctx, checksum_type, d_in, 0, 1, cl, bpc, reinterpret_cast<uint32_t *>(d_out), nw,
                          big_endian, raw, &a))
          return hipErrorInvalidValue;
        return ozec::launch_crc_windows(a, st);
      });
}

int ozec_checksum_windows(int checksum_type, const uint8_t *data, size_t len, size_t bpc, uint32_t *out,
                          int big_endian) {
  ozec::StatScope stat_(OZEC_OP_CHECKSUM, len);
  return checksum_host(checksum_type, data, len, bpc, out, big_endian, 0);
}

int ozec_checksum_verify(int checksum_type, const uint8_t *data, size_t len, size_t bpc, const uint32_t *expected,
                         size_t num_expected, size_t start_index, int64_t *mismatch_index) {
  ozec::StatScope stat_(OZEC_OP_CHECKSUM, len);
  if (mismatch_index) *mismatch_index = -1;
  if (checksum_type == OZEC_CHECKSUM_NONE) return OZEC_OK;  // Checksum.java:250-253
  if (num_expected == 0) return fail(OZEC_EMISMATCH, "Original checksumData has no checksums");
  if (bpc == 0) return fail(OZEC_EINVAL, "bytesPerChecksum must be positive");
  const size_t nwin = (len + bpc - 1) / bpc;
  if (nwin == 0) return fail(OZEC_EMISMATCH, "Computed checksumData has no checksums");
  std::vector<uint32_t> got(nwin);
  if (int rc = checksum_host(checksum_type, data, len, bpc, got.data(), 0, 0)) return rc;
  for (size_t i = 0; i < nwin; ++i) {
    if (start_index + i >= num_expected)
      return fail(OZEC_EMISMATCH, "Computed checksum has " + std::to_string(nwin) +
                                      " number of checksums. Original checksum has " +
                                      std::to_string(num_expected - std::min(num_expected, start_index)) +
                                      " number of checksums starting from index " + std::to_string(start_index));
    if (got[i] != expected[start_index + i]) {
      if (mismatch_index) *mismatch_index = static_cast<int64_t>(i);
      return fail(OZEC_EMISMATCH, "Checksum mismatch at index " + std::to_string(i));
    }
  }
  return OZEC_OK;
}

uint32_t ozec_crc_reset(int) { return 0xffffffffu; }

int ozec_crc_update(int checksum_type, uint32_t *state, const uint8_t *data, size_t len) {
  ozec::StatScope stat_(OZEC_OP_CHECKSUM, len);
  CrcType t;
  if (int rc = crc_type_of(checksum_type, &t)) return rc;
  if (!state) return fail(OZEC_EINVAL, "null state");
  if (len == 0) return OZEC_OK;
  // raw (zero-init, no final xor) CRCs of 16 KiB windows computed in parallel on the GPU, folded on the host:
  // register after (reg, w) = shift(reg, |w|) ^ f(w)
  constexpr size_t kWin = 16384;
  const size_t nwin = (len + kWin - 1) / kWin;
  std::vector<uint32_t> raw(nwin);
  if (int rc = checksum_host(checksum_type, data, len, kWin, raw.data(), 0, 1)) return rc;
  const CrcMath &cm = CrcMath::get(t);
  uint32_t reg = *state;
  for (size_t i = 0; i < nwin; ++i) reg = cm.shift(reg, std::min(kWin, len - i * kWin)) ^ raw[i];
  *state = reg;
  return OZEC_OK;
}

uint32_t ozec_crc_value(int, uint32_t state) { return ~state; }

// ---- fused encode + CRC --------------------------------------------------------------------------

// fused batch calls by route: one fused kernel, or the unfused kernels (ozec_fused_routes)
static std::atomic<uint64_t> g_route_fused{0}, g_route_unfused{0};

int ozec_fused_routes(uint64_t *fused, uint64_t *unfused) {
  if (fused) *fused = g_route_fused.load(std::memory_order_relaxed);
  if (unfused) *unfused = g_route_unfused.load(std::memory_order_relaxed);
  return OZEC_OK;
}

int ozec_encode_crc_batch(ozec_coder *enc, const uint8_t *d_in, int64_t in_stripe_stride, int64_t in_unit_stride,
                          uint8_t *d_out, int64_t out_stripe_stride, int64_t out_unit_stride, size_t num_stripes,
                          size_t len, int checksum_type, size_t bpc, uint32_t *d_crcs, int big_endian, void *stream) {
  ozec::StatScope stat_(OZEC_OP_FUSED, enc ? static_cast<uint64_t>(enc->k) * len * num_stripes : 0);
  if (int rc = check_open(enc, "encode")) return rc;
  if (enc->decoder) return fail(OZEC_EINVAL, "not an encoder");
  if (len == 0 || num_stripes == 0) return OZEC_OK;
  if (!d_in || !d_out || !d_crcs) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  const int k = enc->k, rows = out_rows(enc), units = k + rows;
  ozec::EncCrcArgs e{};
  CodeArgs &a = e.code;
  a.in = d_in;
  a.out = d_out;
  a.in_stripe_stride = in_stripe_stride;
  a.out_stripe_stride = out_stripe_stride;
  a.nstripes = static_cast<int64_t>(num_stripes);
  a.len = static_cast<int64_t>(len);
  std::vector<uint8_t> coef;
  encode_rows(enc, coef);
  fill_coef(a, rows, k, coef.data());
  for (int j = 0; j < k; ++j) a.in_off[j] = j * in_unit_stride;
  for (int r = 0; r < rows; ++r) a.out_off[r] = r * out_unit_stride;
  const int64_t nwin = static_cast<int64_t>((len + (bpc ? bpc : 1) - 1) / (bpc ? bpc : 1));
  if (int rc = make_crc_args(ctx, checksum_type, nullptr, 0, num_stripes, len, bpc, d_crcs, nwin, big_endian, 0,
                             &e.crc))
    return rc;
  // a small batch of 16-B cells runs faster unfused: the fused kernel gives each (stripe, window) one wave
  if (ozec::encode_crc_supported(a, static_cast<int64_t>(bpc)) &&
      ozec::encode_crc_fused_pays(a, nwin, ozec::g_tune.fused_min_units.load(std::memory_order_relaxed))) {
    OZEC_HIP(ozec::launch_encode_crc(e, st));
    g_route_fused.fetch_add(1, std::memory_order_relaxed);
  } else {
    g_route_unfused.fetch_add(1, std::memory_order_relaxed);
    // unfused: encode, then the CRC pass (crcs[s][u][w] layout kept): one launch over all S x units cells when they
    // sit at one stride (the host batches' device layout [S][k + p][unit pitch]), else one per unit
    OZEC_HIP(ozec::launch_code(a, st));
    const bool uniform = rows == enc->p && in_unit_stride == out_unit_stride && in_stripe_stride == out_stripe_stride &&
                         d_out == d_in + k * in_unit_stride && in_stripe_stride == units * in_unit_stride;
    if (uniform) {
      CrcArgs c = e.crc;
      c.base = d_in;
      c.cell_stride = in_unit_stride;
      c.ncells = static_cast<int64_t>(num_stripes) * units;
      c.out = d_crcs;
      c.out_cell_stride = nwin;
      OZEC_HIP(ozec::launch_crc_windows(c, st));
    }
    for (int u = 0; u < units && !uniform; ++u) {
      CrcArgs c = e.crc;
      c.base = u < k ? d_in + u * in_unit_stride : d_out + (u - k) * out_unit_stride;
      c.cell_stride = u < k ? in_stripe_stride : out_stripe_stride;
      c.out = d_crcs + u * nwin;
      c.out_cell_stride = units * nwin;
      OZEC_HIP(ozec::launch_crc_windows(c, st));
    }
  }
  // XOR with p > 1: every output is reset, only outputs[0] is coded (XORRawEncoder.java:67-85), as in
  // ozec_encode_batch; CRCs cover the coded units only
  for (int r = rows; r < enc->p; ++r)
    OZEC_HIP(hipMemset2DAsync(d_out + r * out_unit_stride, out_stripe_stride, 0, len, num_stripes, st));
  return OZEC_OK;
}

int ozec_encode_crc_block_groups(ozec_coder *enc, uint8_t *d_base, int64_t group_stride, int64_t unit_stride,
                                 size_t num_groups, size_t stripes_per_group, size_t len, int checksum_type, size_t bpc,
                                 uint32_t *d_crcs, int big_endian, void *stream) {
  ozec::StatScope stat_(OZEC_OP_FUSED, enc ? static_cast<uint64_t>(enc->k) * len * num_groups * stripes_per_group : 0);
  if (int rc = check_open(enc, "encode")) return rc;
  if (enc->decoder) return fail(OZEC_EINVAL, "not an encoder");
  if (len == 0 || num_groups == 0 || stripes_per_group == 0) return OZEC_OK;
  if (!d_base || !d_crcs) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  if (stripes_per_group > static_cast<size_t>(INT32_MAX) || num_groups * stripes_per_group > static_cast<size_t>(INT32_MAX))
    return fail(OZEC_EINVAL, "too many stripes for one call");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  const int k = enc->k, rows = out_rows(enc), units = k + rows;
  const int64_t L = static_cast<int64_t>(len);
  uint8_t *d_par = d_base + static_cast<int64_t>(k) * unit_stride;
  const int64_t nwin = static_cast<int64_t>((len + (bpc ? bpc : 1) - 1) / (bpc ? bpc : 1));
  ozec::EncCrcArgs e{};
  CodeArgs &a = e.code;
  a.in = d_base;
  a.out = d_par;
  a.in_stripe_stride = L;  // cells of one block are back to back
  a.out_stripe_stride = L;
  a.grp_stripes = static_cast<int64_t>(stripes_per_group);
  a.in_grp_stride = group_stride;
  a.out_grp_stride = group_stride;
  a.nstripes = static_cast<int64_t>(num_groups * stripes_per_group);
  a.len = L;
  std::vector<uint8_t> coef;
  encode_rows(enc, coef);
  fill_coef(a, rows, k, coef.data());
  for (int j = 0; j < k; ++j) a.in_off[j] = j * unit_stride;
  for (int r = 0; r < rows; ++r) a.out_off[r] = r * unit_stride;
  if (int rc = make_crc_args(ctx, checksum_type, nullptr, 0, a.nstripes, len, bpc, d_crcs, nwin, big_endian, 0, &e.crc))
    return rc;
  if (ozec::encode_crc_supported(a, static_cast<int64_t>(bpc))) {
    OZEC_HIP(ozec::launch_encode_crc(e, st));  // every block group in one launch
  } else {
    for (size_t g = 0; g < num_groups; ++g) {  // layouts the fused kernel does not take: one batch per group
      uint8_t *gb = d_base + static_cast<int64_t>(g) * group_stride;
      if (int rc = ozec_encode_crc_batch(enc, gb, L, unit_stride, gb + static_cast<int64_t>(k) * unit_stride, L,
                                         unit_stride, stripes_per_group, len, checksum_type, bpc,
                                         d_crcs + g * stripes_per_group * units * nwin, big_endian, st))
        return rc;
    }
    return OZEC_OK;
  }
  for (int r = rows; r < enc->p; ++r)  // XOR with p > 1: outputs past the first are reset (XORRawEncoder.java:67-85)
    for (size_t g = 0; g < num_groups; ++g)
      OZEC_HIP(hipMemsetAsync(d_par + static_cast<int64_t>(g) * group_stride + r * unit_stride, 0,
                              stripes_per_group * len, st));
  return OZEC_OK;
}

// ---- end-to-end batch from host memory ----------------------------------------

// one device's share of a host batch, on the calling thread's current device (host_batch_split)
static int encode_crc_host_batch_dev(ozec_coder *enc, const uint8_t *h_in, int64_t in_stripe_stride,
                                     int64_t in_unit_stride, uint8_t *h_out, int64_t out_stripe_stride,
                                     int64_t out_unit_stride, size_t num_stripes, size_t len, int checksum_type,
                                     size_t bpc, uint32_t *h_crcs, int big_endian, size_t stripes_per_chunk) {
  if (int rc = check_open(enc, "encode")) return rc;
  if (enc->decoder) return fail(OZEC_EINVAL, "not an encoder");
  if (len == 0 || num_stripes == 0) return OZEC_OK;
  const bool with_crc = checksum_type != OZEC_CHECKSUM_NONE;
  if (!h_in || !h_out || (with_crc && !h_crcs)) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  if (with_crc) {
    CrcType t;
    if (int rc = crc_type_of(checksum_type, &t)) return rc;
    if (bpc == 0) return fail(OZEC_EINVAL, "bytesPerChecksum must be positive");
  }
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  E2E &P = ctx->e2e;
  std::lock_guard<std::mutex> lk(P.mu);
  const int k = enc->k, p = enc->p, rows = out_rows(enc), units = k + rows;
  const size_t C = std::min(num_stripes, stripes_per_chunk ? stripes_per_chunk
                                                          : static_cast<size_t>(std::max<int64_t>(1, ozec::g_tune.e2e_chunk.load())));
  const size_t nwin = with_crc ? (len + bpc - 1) / bpc : 0;
  // device layout [C][k+p][dunit]: the unit pitch is the cell length (a key's last, partial stripe has any length,
  // ECKeyOutputStream.java:276).  Early in round 5 an odd pitch sent a 700,001-B stripe through the byte-wise kernels
  // (6.0 ms instead of 0.31 ms), so the pitch was rounded up to 16 B at the cost of a 2D copy per stripe; since the
  // kernels take units at any byte offset at full rate (fused_nb.hpp nb_tail, gf_code_vec through buffer
  // descriptors, crc_windows_g26 UA), the plain pitch is faster again: 190 us against 245 us for that stripe
  // (TuneKnobs::host_pitch16 = 1 restores the rounded pitch)
  const size_t dunit = ozec::g_tune.host_pitch16.load(std::memory_order_relaxed) ? round_up(len, 16) : len;
  const size_t dstripe = static_cast<size_t>(k + p) * dunit;
  const size_t dcrc_off = round_up(C * dstripe, kStageAlign);            // then crcs [C][units][nwin]
  const size_t dbytes = dcrc_off + C * units * nwin * sizeof(uint32_t);
  const size_t ncrc = units * nwin;                                      // CRCs per stripe
  // which caller buffers need staging (pageable); the C5 batch is registered, so normally none
  const size_t in_span = (num_stripes - 1) * static_cast<size_t>(in_stripe_stride) +
                         (k - 1) * static_cast<size_t>(in_unit_stride) + len;
  const size_t out_span = (num_stripes - 1) * static_cast<size_t>(out_stripe_stride) +
                          (p - 1) * static_cast<size_t>(out_unit_stride) + len;
  const bool in_pinned = range_pinned(h_in, in_span);
  const bool out_pinned = range_pinned(h_out, out_span);
  const bool crc_pinned = !with_crc || range_pinned(h_crcs, num_stripes * ncrc * sizeof(uint32_t));
  const bool staged = !in_pinned || !out_pinned || !crc_pinned;
  if (!P.h2d) {
    OZEC_HIP(ozec::make_stream(&P.h2d));
    OZEC_HIP(ozec::make_stream(&P.comp));
    OZEC_HIP(ozec::make_stream(&P.d2h));
    for (int b = 0; b < E2E::NB; ++b) {
      OZEC_HIP(hipEventCreateWithFlags(&P.h2d_done[b], hipEventDisableTiming));
      OZEC_HIP(hipEventCreateWithFlags(&P.comp_done[b], hipEventDisableTiming));
      OZEC_HIP(hipEventCreateWithFlags(&P.d2h_done[b], hipEventDisableTiming));
    }
  }
  // drain all three streams on every exit, so no copy of this call outlives it (error paths included)
  struct DrainOnExit {
    E2E &P;
    ~DrainOnExit() {
      (void)hipStreamSynchronize(P.h2d);
      (void)hipStreamSynchronize(P.comp);
      (void)hipStreamSynchronize(P.d2h);
    }
  } drain{P};
  if (dbytes > P.dcap) {
    for (auto &d : P.dbuf) {
      if (d) (void)hipFree(d);
      d = nullptr;
    }
    P.dcap = 0;
    for (auto &d : P.dbuf) OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&d), dbytes));
    P.dcap = dbytes;
  }
  if (staged && dbytes > P.hcap) {
    for (auto &h : P.hstage) {
      if (h) (void)ozec::pinned_free(h);
      h = nullptr;
    }
    P.hcap = 0;
    for (auto &h : P.hstage)
      if (ozec::pinned_alloc(dbytes, ctx->device, reinterpret_cast<void **>(&h)) != 0)
        return fail(OZEC_ENOMEM, "cannot pin " + std::to_string(dbytes) + " bytes of staging memory");
    P.hcap = dbytes;
  }
  const size_t nch = (num_stripes + C - 1) / C;
  // host side of chunk c: copy parity / CRCs of a finished, staged chunk to the caller
  auto unstage = [&](size_t c) -> int {
    const int b = static_cast<int>(c % E2E::NB);
    OZEC_HIP(hipEventSynchronize(P.d2h_done[b]));
    const size_t s0 = c * C, cs = std::min(C, num_stripes - s0);
    std::vector<ozec::CopyTask> tasks;
    if (!out_pinned)
      for (size_t i = 0; i < cs; ++i)
        for (int r = 0; r < p; ++r)
          tasks.push_back({h_out + (s0 + i) * out_stripe_stride + r * out_unit_stride,
                           P.hstage[b] + i * dstripe + static_cast<size_t>(k + r) * dunit, len});
    if (with_crc && !crc_pinned)
      tasks.push_back({h_crcs + s0 * ncrc, P.hstage[b] + dcrc_off, cs * ncrc * sizeof(uint32_t)});
    ozec::parallel_copy(tasks, ozec::CopyDir::kFromStaging, true, ctx->numa);
    return OZEC_OK;
  };
  for (size_t c = 0; c < nch; ++c) {
    const int b = static_cast<int>(c % E2E::NB);
    const size_t s0 = c * C, cs = std::min(C, num_stripes - s0);
    uint8_t *d = P.dbuf[b];
    if (staged) {
      if (c >= static_cast<size_t>(E2E::NB))
        if (int rc = unstage(c - E2E::NB)) return rc;  // frees hstage[b] for this chunk
      if (!in_pinned) {
        std::vector<ozec::CopyTask> tasks;
        for (size_t i = 0; i < cs; ++i)
          for (int j = 0; j < k; ++j)
            tasks.push_back({P.hstage[b] + i * dstripe + static_cast<size_t>(j) * dunit,
                             h_in + (s0 + i) * in_stripe_stride + j * in_unit_stride, len});
        ozec::parallel_copy(tasks, ozec::CopyDir::kToStaging, true, ctx->numa);
      }
    }
    // H2D after the chunk that used this buffer NB chunks ago has left the device.  The host waits for it too
    // (staged calls already did, in unstage): the HIP queues then never hold more than NB chunks of commands.
    // Enqueuing a whole 8192-stripe batch up front (~40 commands per chunk) measured 27 GB/s at 16-stripe chunks
    // against 49 GB/s for the same chunks of a 1024-stripe batch; with the wait, 45-48 GB/s at every size, and
    // 56 GB/s (98 % of the 57.5 GB/s H2D link) with one rectangular copy per chunk and direction
    // (scripts/e2e_probe2.py, profiles/r02/e2e_probe.log).
    if (c >= static_cast<size_t>(E2E::NB)) {
      if (!staged) OZEC_HIP(hipEventSynchronize(P.d2h_done[b]));
      OZEC_HIP(hipStreamWaitEvent(P.h2d, P.d2h_done[b], 0));
    }
    const bool rect = ozec::g_tune.e2e_rect != 0;
    if (!in_pinned) {
      // staged cells are already in the device layout: one copy of the data cells per stripe
      for (size_t i = 0; i < cs; ++i)
        OZEC_HIP(hipMemcpyAsync(d + i * dstripe, P.hstage[b] + i * dstripe, static_cast<size_t>(k) * dunit,
                                hipMemcpyHostToDevice, P.h2d));
    } else if (dunit != len) {
      for (size_t i = 0; i < cs; ++i)  // one rectangular copy per stripe: k rows of len bytes onto the unit pitch
        OZEC_HIP(hipMemcpy2DAsync(d + i * dstripe, dunit, h_in + (s0 + i) * in_stripe_stride,
                                  static_cast<size_t>(in_unit_stride), len, k, hipMemcpyHostToDevice, P.h2d));
    } else if (in_unit_stride == static_cast<int64_t>(len) && rect) {
      // one rectangular copy per chunk: cs rows of k*len bytes, source pitch = the batch's stripe stride
      OZEC_HIP(hipMemcpy2DAsync(d, dstripe, h_in + s0 * in_stripe_stride, static_cast<size_t>(in_stripe_stride),
                                static_cast<size_t>(k) * len, cs, hipMemcpyHostToDevice, P.h2d));
    } else if (in_unit_stride == static_cast<int64_t>(len)) {
      for (size_t i = 0; i < cs; ++i)  // the k data cells of a stripe are one run
        OZEC_HIP(hipMemcpyAsync(d + i * dstripe, h_in + (s0 + i) * in_stripe_stride, static_cast<size_t>(k) * len,
                                hipMemcpyHostToDevice, P.h2d));
    } else {
      for (size_t i = 0; i < cs; ++i)
        for (int j = 0; j < k; ++j)
          OZEC_HIP(hipMemcpyAsync(d + i * dstripe + static_cast<size_t>(j) * len,
                                  h_in + (s0 + i) * in_stripe_stride + j * in_unit_stride, len, hipMemcpyHostToDevice,
                                  P.h2d));
    }
    OZEC_HIP(hipEventRecord(P.h2d_done[b], P.h2d));
    OZEC_HIP(hipStreamWaitEvent(P.comp, P.h2d_done[b], 0));
    const int64_t ds = static_cast<int64_t>(dstripe), us = static_cast<int64_t>(dunit);
    uint32_t *dcrc = reinterpret_cast<uint32_t *>(d + dcrc_off);
    if (with_crc) {
      if (int rc = ozec_encode_crc_batch(enc, d, ds, us, d + static_cast<size_t>(k) * dunit, ds, us, cs, len,
                                         checksum_type, bpc, dcrc, big_endian, P.comp))
        return rc;
    } else {
      if (int rc = ozec_encode_batch(enc, d, ds, us, d + static_cast<size_t>(k) * dunit, ds, us, cs, len, P.comp))
        return rc;
    }
    OZEC_HIP(hipEventRecord(P.comp_done[b], P.comp));
    OZEC_HIP(hipStreamWaitEvent(P.d2h, P.comp_done[b], 0));
    uint8_t *hs = staged ? P.hstage[b] : nullptr;
    if (out_pinned && out_unit_stride == static_cast<int64_t>(len) && dunit == len && rect) {
      OZEC_HIP(hipMemcpy2DAsync(h_out + s0 * out_stripe_stride, static_cast<size_t>(out_stripe_stride),
                                d + static_cast<size_t>(k) * len, dstripe, static_cast<size_t>(p) * len, cs,
                                hipMemcpyDeviceToHost, P.d2h));
    } else for (size_t i = 0; i < cs; ++i) {
      uint8_t *src = d + i * dstripe + static_cast<size_t>(k) * dunit;
      if (!out_pinned) {
        OZEC_HIP(hipMemcpyAsync(hs + i * dstripe + static_cast<size_t>(k) * dunit, src, static_cast<size_t>(p) * dunit,
                                hipMemcpyDeviceToHost, P.d2h));
      } else if (dunit != len) {
        OZEC_HIP(hipMemcpy2DAsync(h_out + (s0 + i) * out_stripe_stride, static_cast<size_t>(out_unit_stride), src,
                                  dunit, len, p, hipMemcpyDeviceToHost, P.d2h));
      } else if (out_unit_stride == static_cast<int64_t>(len)) {
        OZEC_HIP(hipMemcpyAsync(h_out + (s0 + i) * out_stripe_stride, src, static_cast<size_t>(p) * len,
                                hipMemcpyDeviceToHost, P.d2h));
      } else {
        for (int r = 0; r < p; ++r)
          OZEC_HIP(hipMemcpyAsync(h_out + (s0 + i) * out_stripe_stride + r * out_unit_stride, src + r * len, len,
                                  hipMemcpyDeviceToHost, P.d2h));
      }
    }
    if (with_crc)
      OZEC_HIP(hipMemcpyAsync(crc_pinned ? reinterpret_cast<uint8_t *>(h_crcs + s0 * ncrc) : hs + dcrc_off, dcrc,
                              cs * ncrc * sizeof(uint32_t), hipMemcpyDeviceToHost, P.d2h));
    OZEC_HIP(hipEventRecord(P.d2h_done[b], P.d2h));
  }
  if (staged) {
    for (size_t c = nch > static_cast<size_t>(E2E::NB) ? nch - E2E::NB : 0; c < nch; ++c)
      if (int rc = unstage(c)) return rc;
  }
  OZEC_HIP(hipStreamSynchronize(P.d2h));
  return OZEC_OK;
}

// ---- batched verify and fused reconstruction -------------------------------

int ozec_checksum_verify_batch(int checksum_type, const uint8_t *d_base, int64_t cell_stride, size_t num_cells,
                               size_t len, size_t bpc, const uint32_t *d_expected, int expected_big_endian,
                               int32_t *d_mismatch, void *stream) {
  ozec::StatScope stat_(OZEC_OP_CHECKSUM_DEVICE, static_cast<uint64_t>(len) * num_cells);
  if (num_cells == 0) return OZEC_OK;
  if (!d_mismatch) return fail(OZEC_EINVAL, "null mismatch buffer");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  OZEC_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_mismatch), 0x7fffffff, num_cells, st));
  if (len > 0) {
    if (!d_base || !d_expected) return fail(OZEC_EINVAL, "null buffer");
    CrcArgs a;
    const int64_t nwin = static_cast<int64_t>((len + (bpc ? bpc : 1) - 1) / (bpc ? bpc : 1));
    if (int rc = make_crc_args(ctx, checksum_type, d_base, cell_stride, num_cells, len, bpc, nullptr, nwin, 0, 0, &a))
      return rc;
    a.expected = d_expected;
    a.expected_be = expected_big_endian;
    a.mismatch = d_mismatch;
    OZEC_HIP(ozec::launch_crc_windows(a, st));
  }
  OZEC_HIP(ozec::launch_finish_mismatch(d_mismatch, static_cast<int64_t>(num_cells), st));
  return OZEC_OK;
}

int ozec_reconstruct_crc_batch(ozec_coder *dec, const uint8_t *d_in, int64_t in_stripe_stride, int64_t in_unit_stride,
                               const int *present_units, int num_present, const int *erased, int n_erased,
                               uint8_t *d_out, int64_t out_stripe_stride, int64_t out_unit_stride, size_t num_stripes,
                               size_t len, int checksum_type, size_t bpc, const uint32_t *d_expected,
                               int expected_big_endian, uint32_t *d_out_crcs, int out_big_endian, int32_t *d_mismatch,
                               void *stream) {
  ozec::StatScope stat_(OZEC_OP_FUSED, dec ? static_cast<uint64_t>(dec->k) * len * num_stripes : 0);
  if (int rc = check_open(dec, "decode")) return rc;
  if (!dec->decoder) return fail(OZEC_EINVAL, "not a decoder");
  const int n_all = dec->k + dec->p;
  bool present[256] = {false};
  for (int i = 0; i < num_present; ++i) {
    if (present_units[i] < 0 || present_units[i] >= n_all) return fail(OZEC_EINVAL, "present unit out of range");
    present[present_units[i]] = true;
  }
  std::vector<int> units;
  std::vector<uint8_t> rows;
  if (int rc = plan_decode(dec, present, erased, n_erased, units, rows)) return rc;
  if (num_stripes == 0) return OZEC_OK;
  if (!d_in || (n_erased && (!d_out || !d_out_crcs))) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  if (d_expected && !d_mismatch) return fail(OZEC_EINVAL, "verification needs a mismatch buffer");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  hipStream_t st = pick_stream(ctx, stream);
  if (d_mismatch)
    OZEC_HIP(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(d_mismatch), 0x7fffffff, num_stripes, st));
  if (len == 0) {
    if (d_mismatch) OZEC_HIP(ozec::launch_finish_mismatch(d_mismatch, static_cast<int64_t>(num_stripes), st));
    return OZEC_OK;
  }
  const int nin = static_cast<int>(units.size());
  const int nrows = dec->codec == OZEC_CODEC_XOR ? (n_erased ? 1 : 0) : n_erased;
  const int64_t nwin = static_cast<int64_t>((len + (bpc ? bpc : 1) - 1) / (bpc ? bpc : 1));
  ozec::EncCrcArgs e{};
  CodeArgs &a = e.code;
  a.in = d_in;
  a.out = d_out;
  a.in_stripe_stride = in_stripe_stride;
  a.out_stripe_stride = out_stripe_stride;
  a.nstripes = static_cast<int64_t>(num_stripes);
  a.len = static_cast<int64_t>(len);
  if (nrows) {
    fill_coef(a, nrows, nin, rows.data());
    if (int rc = check_limits(a.k, a.rows)) return rc;
  } else {
    a.k = nin;
    a.rows = 0;
  }
  for (int j = 0; j < nin; ++j) a.in_off[j] = units[j] * in_unit_stride;
  for (int r = 0; r < nrows; ++r) a.out_off[r] = r * out_unit_stride;
  if (int rc = make_crc_args(ctx, checksum_type, nullptr, 0, num_stripes, len, bpc, d_out_crcs, nwin, out_big_endian, 0,
                             &e.crc))
    return rc;
  e.crc.expected = d_expected;
  e.crc.expected_be = expected_big_endian;
  e.crc.mismatch = d_mismatch;
  e.verify = 1;
  e.exp_units = n_all;
  for (int j = 0; j < nin; ++j) e.in_unit[j] = units[j];
  if (nrows && n_erased == nrows && ozec::encode_crc_supported(a, static_cast<int64_t>(bpc)) &&
      ozec::encode_crc_fused_pays(a, nwin, ozec::g_tune.rec_min_units.load(std::memory_order_relaxed))) {
    OZEC_HIP(ozec::launch_encode_crc(e, st));
    g_route_fused.fetch_add(1, std::memory_order_relaxed);
  } else {
    g_route_unfused.fetch_add(1, std::memory_order_relaxed);
    // unfused: verify the read units, decode, CRC the rebuilt units
    if (d_expected) {
      for (int j = 0; j < nin; ++j) {
        CrcArgs c = e.crc;
        c.base = d_in + units[j] * in_unit_stride;
        c.cell_stride = in_stripe_stride;
        c.expected = d_expected + units[j] * nwin;
        c.out_cell_stride = n_all * nwin;
        c.mismatch_base = static_cast<int32_t>(units[j] * nwin);
        OZEC_HIP(ozec::launch_crc_windows(c, st));
      }
    }
    if (nrows) OZEC_HIP(ozec::launch_code(a, st));
    // the rebuilt units' CRCs: one launch over all S x n_erased cells when they sit at one stride, else one per unit
    const bool uniform = out_stripe_stride == static_cast<int64_t>(n_erased) * out_unit_stride;
    for (int r = nrows; r < n_erased && uniform; ++r)  // XOR decoders zero-fill outputs beyond erasedIndexes[0]
      OZEC_HIP(hipMemset2DAsync(d_out + r * out_unit_stride, out_stripe_stride, 0, len, num_stripes, st));
    if (uniform && n_erased) {
      CrcArgs c = e.crc;
      c.base = d_out;
      c.cell_stride = out_unit_stride;
      c.ncells = static_cast<int64_t>(num_stripes) * n_erased;
      c.out = d_out_crcs;
      c.out_cell_stride = nwin;
      c.expected = nullptr;
      OZEC_HIP(ozec::launch_crc_windows(c, st));
    }
    for (int r = 0; r < n_erased && !uniform; ++r) {
      if (r >= nrows) {  // XOR decoders zero-fill outputs beyond erasedIndexes[0]
        OZEC_HIP(hipMemset2DAsync(d_out + r * out_unit_stride, out_stripe_stride, 0, len, num_stripes, st));
      }
      CrcArgs c = e.crc;
      c.base = d_out + r * out_unit_stride;
      c.cell_stride = out_stripe_stride;
      c.out = d_out_crcs + r * nwin;
      c.out_cell_stride = n_erased * nwin;
      c.expected = nullptr;
      OZEC_HIP(ozec::launch_crc_windows(c, st));
    }
  }
  if (d_mismatch) OZEC_HIP(ozec::launch_finish_mismatch(d_mismatch, static_cast<int64_t>(num_stripes), st));
  return OZEC_OK;
}

// Fused reconstruction of stripes held in HOST memory: the datanode side of ECReconstructionCoordinator, whose read
// buffers hold the k units it fetched (ECBlockReconstructedStripeInputStream.java:689-694).  The pipeline of
// ozec_encode_crc_host_batch (ring of E2E::NB device chunk buffers, H2D / kernel / D2H on three streams, the host
// waiting for a buffer's previous chunk before refilling it) around ozec_reconstruct_crc_batch.  Only the k units the
// decoder reads cross PCIe, as one rectangular copy per run of consecutive unit indexes per chunk.
static int reconstruct_crc_host_batch_dev(ozec_coder *dec, const uint8_t *h_in, int64_t in_stripe_stride,
                                          int64_t in_unit_stride, const int *present_units, int num_present,
                                          const int *erased, int n_erased, uint8_t *h_out, int64_t out_stripe_stride,
                                          int64_t out_unit_stride, size_t num_stripes, size_t len, int checksum_type,
                                          size_t bpc, const uint32_t *h_expected, int expected_big_endian,
                                          uint32_t *h_out_crcs, int out_big_endian, int32_t *h_mismatch,
                                          size_t stripes_per_chunk) {
  if (int rc = check_open(dec, "decode")) return rc;
  if (!dec->decoder) return fail(OZEC_EINVAL, "not a decoder");
  const int n_all = dec->k + dec->p;
  if (num_present < 0 || (num_present > 0 && !present_units)) return fail(OZEC_EINVAL, "invalid present units");
  bool present[256] = {false};
  for (int i = 0; i < num_present; ++i) {
    if (present_units[i] < 0 || present_units[i] >= n_all) return fail(OZEC_EINVAL, "present unit out of range");
    present[present_units[i]] = true;
  }
  std::vector<int> units;
  std::vector<uint8_t> rows;
  if (int rc = plan_decode(dec, present, erased, n_erased, units, rows)) return rc;
  {
    CrcType t;
    if (int rc = crc_type_of(checksum_type, &t)) return rc;
    if (bpc == 0) return fail(OZEC_EINVAL, "bytesPerChecksum must be positive");
  }
  if (num_stripes == 0 || len == 0) {
    if (h_mismatch)
      for (size_t s = 0; s < num_stripes; ++s) h_mismatch[s] = -1;
    return OZEC_OK;
  }
  if (!h_in || (n_erased && (!h_out || !h_out_crcs))) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  if (h_expected && !h_mismatch) return fail(OZEC_EINVAL, "verification needs a mismatch buffer");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  E2E &P = ctx->e2e;
  std::lock_guard<std::mutex> lk(P.mu);
  const int e = n_erased;
  const size_t C = std::min(num_stripes, stripes_per_chunk ? stripes_per_chunk
                                                          : static_cast<size_t>(std::max<int64_t>(1, ozec::g_tune.e2e_chunk.load())));
  const size_t nwin = (len + bpc - 1) / bpc;
  // device layout of one chunk buffer: input slots [C][k+p][len], rebuilt [C][e][len], expected CRCs [C][k+p][nwin],
  // rebuilt CRCs [C][e][nwin], mismatch [C]
  // 16-B aligned unit pitch, as in encode_crc_host_batch_dev
  const size_t dunit = ozec::g_tune.host_pitch16.load(std::memory_order_relaxed) ? round_up(len, 16) : len;
  const size_t dstripe = static_cast<size_t>(n_all) * dunit, ostripe = static_cast<size_t>(e) * dunit;
  const size_t dout_off = round_up(C * dstripe, kStageAlign);
  const size_t dexp_off = round_up(dout_off + C * ostripe, kStageAlign);
  const size_t dexp_bytes = h_expected ? C * n_all * nwin * sizeof(uint32_t) : 0;
  const size_t docrc_off = round_up(dexp_off + dexp_bytes, kStageAlign);
  const size_t dmis_off = round_up(docrc_off + C * e * nwin * sizeof(uint32_t), kStageAlign);
  const size_t dbytes = dmis_off + C * sizeof(int32_t);
  // runs of consecutive unit indexes among the units read: one rectangular copy per run and chunk
  std::vector<std::pair<int, int>> runs;
  for (int u : units) {
    if (!runs.empty() && runs.back().first + runs.back().second == u) ++runs.back().second;
    else runs.push_back({u, 1});
  }
  const int umax = units.empty() ? 0 : units.back();
  const size_t in_span = (num_stripes - 1) * static_cast<size_t>(in_stripe_stride) +
                         static_cast<size_t>(umax) * static_cast<size_t>(in_unit_stride) + len;
  const size_t out_span = e ? (num_stripes - 1) * static_cast<size_t>(out_stripe_stride) +
                                  static_cast<size_t>(e - 1) * static_cast<size_t>(out_unit_stride) + len
                            : 0;
  const bool in_pinned = range_pinned(h_in, in_span);
  const bool out_pinned = !e || range_pinned(h_out, out_span);
  const bool exp_pinned = !h_expected || range_pinned(h_expected, num_stripes * n_all * nwin * sizeof(uint32_t));
  const bool ocrc_pinned = !e || range_pinned(h_out_crcs, num_stripes * e * nwin * sizeof(uint32_t));
  const bool mis_pinned = !h_expected || range_pinned(h_mismatch, num_stripes * sizeof(int32_t));
  const bool staged = !in_pinned || !out_pinned || !exp_pinned || !ocrc_pinned || !mis_pinned;
  if (!P.h2d) {
    OZEC_HIP(ozec::make_stream(&P.h2d));
    OZEC_HIP(ozec::make_stream(&P.comp));
    OZEC_HIP(ozec::make_stream(&P.d2h));
    for (int b = 0; b < E2E::NB; ++b) {
      OZEC_HIP(hipEventCreateWithFlags(&P.h2d_done[b], hipEventDisableTiming));
      OZEC_HIP(hipEventCreateWithFlags(&P.comp_done[b], hipEventDisableTiming));
      OZEC_HIP(hipEventCreateWithFlags(&P.d2h_done[b], hipEventDisableTiming));
    }
  }
  struct DrainOnExit {
    E2E &P;
    ~DrainOnExit() {
      (void)hipStreamSynchronize(P.h2d);
      (void)hipStreamSynchronize(P.comp);
      (void)hipStreamSynchronize(P.d2h);
    }
  } drain{P};
  if (dbytes > P.dcap) {
    for (auto &d : P.dbuf) {
      if (d) (void)hipFree(d);
      d = nullptr;
    }
    P.dcap = 0;
    for (auto &d : P.dbuf) OZEC_HIP(hipMalloc(reinterpret_cast<void **>(&d), dbytes));
    P.dcap = dbytes;
  }
  if (staged && dbytes > P.hcap) {
    for (auto &h : P.hstage) {
      if (h) (void)ozec::pinned_free(h);
      h = nullptr;
    }
    P.hcap = 0;
    for (auto &h : P.hstage)
      if (ozec::pinned_alloc(dbytes, ctx->device, reinterpret_cast<void **>(&h)) != 0)
        return fail(OZEC_ENOMEM, "cannot pin " + std::to_string(dbytes) + " bytes of staging memory");
    P.hcap = dbytes;
  }
  const size_t nch = (num_stripes + C - 1) / C;
  auto unstage = [&](size_t c) -> int {
    const int b = static_cast<int>(c % E2E::NB);
    OZEC_HIP(hipEventSynchronize(P.d2h_done[b]));
    const size_t s0 = c * C, cs = std::min(C, num_stripes - s0);
    std::vector<ozec::CopyTask> tasks;
    if (!out_pinned)
      for (size_t i = 0; i < cs; ++i)
        for (int r = 0; r < e; ++r)
          tasks.push_back({h_out + (s0 + i) * out_stripe_stride + r * out_unit_stride,
                           P.hstage[b] + dout_off + i * ostripe + static_cast<size_t>(r) * dunit, len});
    if (!ocrc_pinned)
      tasks.push_back({h_out_crcs + s0 * e * nwin, P.hstage[b] + docrc_off, cs * e * nwin * sizeof(uint32_t)});
    if (!mis_pinned) tasks.push_back({h_mismatch + s0, P.hstage[b] + dmis_off, cs * sizeof(int32_t)});
    ozec::parallel_copy(tasks, ozec::CopyDir::kFromStaging, true, ctx->numa);
    return OZEC_OK;
  };
  for (size_t c = 0; c < nch; ++c) {
    const int b = static_cast<int>(c % E2E::NB);
    const size_t s0 = c * C, cs = std::min(C, num_stripes - s0);
    uint8_t *d = P.dbuf[b];
    uint8_t *hs = staged ? P.hstage[b] : nullptr;
    if (staged) {
      if (c >= static_cast<size_t>(E2E::NB))
        if (int rc = unstage(c - E2E::NB)) return rc;
      std::vector<ozec::CopyTask> tasks;
      if (!in_pinned)
        for (size_t i = 0; i < cs; ++i)
          for (int u : units)
            tasks.push_back({hs + i * dstripe + static_cast<size_t>(u) * dunit,
                             h_in + (s0 + i) * in_stripe_stride + u * in_unit_stride, len});
      if (!exp_pinned)
        tasks.push_back({hs + dexp_off, h_expected + s0 * n_all * nwin, cs * n_all * nwin * sizeof(uint32_t)});
      ozec::parallel_copy(tasks, ozec::CopyDir::kToStaging, true, ctx->numa);
    }
    if (c >= static_cast<size_t>(E2E::NB)) {
      if (!staged) OZEC_HIP(hipEventSynchronize(P.d2h_done[b]));
      OZEC_HIP(hipStreamWaitEvent(P.h2d, P.d2h_done[b], 0));
    }
    for (const auto &run : runs) {
      const size_t off = static_cast<size_t>(run.first) * dunit, width = static_cast<size_t>(run.second) * dunit;
      if (!in_pinned) {
        OZEC_HIP(hipMemcpy2DAsync(d + off, dstripe, hs + off, dstripe, width, cs, hipMemcpyHostToDevice, P.h2d));
      } else if (dunit != len) {
        for (size_t i = 0; i < cs; ++i)  // one rectangular copy per stripe and run onto the unit pitch
          OZEC_HIP(hipMemcpy2DAsync(d + i * dstripe + off, dunit,
                                    h_in + (s0 + i) * in_stripe_stride + run.first * in_unit_stride,
                                    static_cast<size_t>(in_unit_stride), len, run.second, hipMemcpyHostToDevice, P.h2d));
      } else if (in_unit_stride == static_cast<int64_t>(len)) {
        OZEC_HIP(hipMemcpy2DAsync(d + off, dstripe, h_in + s0 * in_stripe_stride + off,
                                  static_cast<size_t>(in_stripe_stride), width, cs, hipMemcpyHostToDevice, P.h2d));
      } else {
        for (size_t i = 0; i < cs; ++i)
          for (int u = run.first; u < run.first + run.second; ++u)
            OZEC_HIP(hipMemcpyAsync(d + i * dstripe + static_cast<size_t>(u) * dunit,
                                    h_in + (s0 + i) * in_stripe_stride + u * in_unit_stride, len, hipMemcpyHostToDevice,
                                    P.h2d));
      }
    }
    if (h_expected)
      OZEC_HIP(hipMemcpyAsync(d + dexp_off, exp_pinned ? reinterpret_cast<const uint8_t *>(h_expected + s0 * n_all * nwin)
                                                       : hs + dexp_off,
                              cs * n_all * nwin * sizeof(uint32_t), hipMemcpyHostToDevice, P.h2d));
    OZEC_HIP(hipEventRecord(P.h2d_done[b], P.h2d));
    OZEC_HIP(hipStreamWaitEvent(P.comp, P.h2d_done[b], 0));
    if (int rc = ozec_reconstruct_crc_batch(
            dec, d, static_cast<int64_t>(dstripe), static_cast<int64_t>(dunit), present_units, num_present, erased, e,
            d + dout_off, static_cast<int64_t>(ostripe), static_cast<int64_t>(dunit), cs, len, checksum_type, bpc,
            h_expected ? reinterpret_cast<const uint32_t *>(d + dexp_off) : nullptr, expected_big_endian,
            reinterpret_cast<uint32_t *>(d + docrc_off), out_big_endian,
            h_expected ? reinterpret_cast<int32_t *>(d + dmis_off) : nullptr, P.comp))
      return rc;
    OZEC_HIP(hipEventRecord(P.comp_done[b], P.comp));
    OZEC_HIP(hipStreamWaitEvent(P.d2h, P.comp_done[b], 0));
    if (e) {
      if (!out_pinned) {
        OZEC_HIP(hipMemcpyAsync(hs + dout_off, d + dout_off, cs * ostripe, hipMemcpyDeviceToHost, P.d2h));
      } else if (dunit != len) {
        for (size_t i = 0; i < cs; ++i)
          OZEC_HIP(hipMemcpy2DAsync(h_out + (s0 + i) * out_stripe_stride, static_cast<size_t>(out_unit_stride),
                                    d + dout_off + i * ostripe, dunit, len, e, hipMemcpyDeviceToHost, P.d2h));
      } else if (out_unit_stride == static_cast<int64_t>(len)) {
        OZEC_HIP(hipMemcpy2DAsync(h_out + s0 * out_stripe_stride, static_cast<size_t>(out_stripe_stride), d + dout_off,
                                  ostripe, ostripe, cs, hipMemcpyDeviceToHost, P.d2h));
      } else {
        for (size_t i = 0; i < cs; ++i)
          for (int r = 0; r < e; ++r)
            OZEC_HIP(hipMemcpyAsync(h_out + (s0 + i) * out_stripe_stride + r * out_unit_stride,
                                    d + dout_off + i * ostripe + static_cast<size_t>(r) * len, len, hipMemcpyDeviceToHost,
                                    P.d2h));
      }
      OZEC_HIP(hipMemcpyAsync(ocrc_pinned ? reinterpret_cast<uint8_t *>(h_out_crcs + s0 * e * nwin) : hs + docrc_off,
                              d + docrc_off, cs * e * nwin * sizeof(uint32_t), hipMemcpyDeviceToHost, P.d2h));
    }
    if (h_expected)
      OZEC_HIP(hipMemcpyAsync(mis_pinned ? reinterpret_cast<uint8_t *>(h_mismatch + s0) : hs + dmis_off, d + dmis_off,
                              cs * sizeof(int32_t), hipMemcpyDeviceToHost, P.d2h));
    OZEC_HIP(hipEventRecord(P.d2h_done[b], P.d2h));
  }
  if (staged) {
    for (size_t c = nch > static_cast<size_t>(E2E::NB) ? nch - E2E::NB : 0; c < nch; ++c)
      if (int rc = unstage(c)) return rc;
  }
  OZEC_HIP(hipStreamSynchronize(P.d2h));
  if (!h_expected && h_mismatch)
    for (size_t s = 0; s < num_stripes; ++s) h_mismatch[s] = -1;
  return OZEC_OK;
}

// A host batch split over the device list (devices.hpp): contiguous stripe ranges, part i = stripe_range(S, i, n),
// each run by the single-device pipeline on its own GPU, all at once (part 0 on the calling thread, the others on
// threads of their own).  The coder's GPU takes part 0; a batch too small for one pipeline chunk per GPU stays on it.
// No data crosses between GPUs (north_star: "a batch is partitioned across the 8 MI355X of one node as per-GPU
// streams with no RCCL collectives").  fn(s0, s1) runs with its part's device current.
}  // extern "C"

template <class Fn>
static int host_batch_split(const ozec_coder *c, size_t num_stripes, size_t chunk, Fn fn) {
  std::vector<int> devs = ozec::device_list();
  if (devs.empty()) return fail(OZEC_EDEVICE, "no HIP device available");
  auto it = std::find(devs.begin(), devs.end(), c->device);
  if (it != devs.end()) std::rotate(devs.begin(), it, devs.end());
  else devs.insert(devs.begin(), c->device);  // a coder made before ozec_set_devices dropped its GPU
  const size_t parts = ozec::split_parts(num_stripes, chunk, devs.size());
  auto range = [&](size_t i, size_t *s0, size_t *s1) { ozec::part_range(num_stripes, parts, i, s0, s1); };
  if (parts == 1) {
    ozec::DeviceScope ds(devs[0]);
    if (!ds.ok()) return fail(OZEC_EDEVICE, "cannot select device " + std::to_string(devs[0]));
    return fn(size_t{0}, num_stripes);
  }
  std::vector<int> rcs(parts, OZEC_OK);
  std::vector<std::string> msgs(parts);
  auto run = [&](size_t i) {
    size_t s0, s1;
    range(i, &s0, &s1);
    if (s0 >= s1) return;
    ozec::DeviceScope ds(devs[i]);
    if (!ds.ok()) {
      rcs[i] = OZEC_EDEVICE;
      msgs[i] = "cannot select device " + std::to_string(devs[i]);
      return;
    }
    rcs[i] = fn(s0, s1);
    if (rcs[i]) msgs[i] = g_error;
  };
  // a part no thread can be started for (std::system_error: the process's thread limit, or memory) runs on the calling
  // thread after part 0 -- nothing may escape through the C ABI into the JVM
  std::vector<std::thread> workers;
  size_t threaded = 1;  // parts 1 .. threaded-1 have a thread
  try {
    workers.reserve(parts - 1);
    for (size_t i = 1; i < parts; ++i, ++threaded)
      workers.emplace_back([&, i] {
        ozec::g_stat_depth = 1;  // the caller's call is the one counted (stats.hpp)
        run(i);
      });
  } catch (const std::exception &) {
  }
  run(0);
  for (size_t i = threaded; i < parts; ++i) run(i);
  for (auto &w : workers) w.join();
  for (size_t i = 0; i < parts; ++i)
    if (rcs[i]) return fail(rcs[i], "device " + std::to_string(devs[i]) + ": " + msgs[i]);
  return OZEC_OK;
}

extern "C" {

static size_t e2e_chunk_of(size_t stripes_per_chunk) {
  return stripes_per_chunk ? stripes_per_chunk : static_cast<size_t>(std::max<int64_t>(1, ozec::g_tune.e2e_chunk.load()));
}

int ozec_encode_crc_host_batch(ozec_coder *enc, const uint8_t *h_in, int64_t in_stripe_stride,
                               int64_t in_unit_stride, uint8_t *h_out, int64_t out_stripe_stride,
                               int64_t out_unit_stride, size_t num_stripes, size_t len, int checksum_type,
                               size_t bpc, uint32_t *h_crcs, int big_endian, size_t stripes_per_chunk) {
  ozec::StatScope stat_(OZEC_OP_HOST_BATCH, enc ? static_cast<uint64_t>(enc->k) * len * num_stripes : 0);
  if (int rc = check_open(enc, "encode")) return rc;
  if (enc->decoder) return fail(OZEC_EINVAL, "not an encoder");
  if (len == 0 || num_stripes == 0) return OZEC_OK;
  const bool with_crc = checksum_type != OZEC_CHECKSUM_NONE;
  if (!h_in || !h_out || (with_crc && !h_crcs)) return fail(OZEC_EINVAL, "Invalid buffer found, not allowing null");
  if (with_crc) {  // argument errors as the single-device path reports them, before any split
    CrcType t;
    if (int rc = crc_type_of(checksum_type, &t)) return rc;
    if (bpc == 0) return fail(OZEC_EINVAL, "bytesPerChecksum must be positive");
  }
  const size_t ncrc = with_crc ? static_cast<size_t>(enc->k + out_rows(enc)) * ((len + bpc - 1) / bpc) : 0;
  return host_batch_split(enc, num_stripes, e2e_chunk_of(stripes_per_chunk), [&](size_t s0, size_t s1) {
    return encode_crc_host_batch_dev(enc, h_in + s0 * in_stripe_stride, in_stripe_stride, in_unit_stride,
                                     h_out + s0 * out_stripe_stride, out_stripe_stride, out_unit_stride, s1 - s0, len,
                                     checksum_type, bpc, with_crc ? h_crcs + s0 * ncrc : nullptr, big_endian,
                                     stripes_per_chunk);
  });
}

int ozec_reconstruct_crc_host_batch(ozec_coder *dec, const uint8_t *h_in, int64_t in_stripe_stride,
                                    int64_t in_unit_stride, const int *present_units, int num_present, const int *erased,
                                    int n_erased, uint8_t *h_out, int64_t out_stripe_stride, int64_t out_unit_stride,
                                    size_t num_stripes, size_t len, int checksum_type, size_t bpc,
                                    const uint32_t *h_expected, int expected_big_endian, uint32_t *h_out_crcs,
                                    int out_big_endian, int32_t *h_mismatch, size_t stripes_per_chunk) {
  ozec::StatScope stat_(OZEC_OP_HOST_BATCH, dec ? static_cast<uint64_t>(dec->k) * len * num_stripes : 0);
  if (int rc = check_open(dec, "decode")) return rc;
  if (!dec->decoder) return fail(OZEC_EINVAL, "not a decoder");
  // argument errors (reported in the single-device path's order) and empty batches: no split
  if (num_stripes == 0 || len == 0 || bpc == 0 || n_erased < 0 || !h_in || (n_erased && (!h_out || !h_out_crcs)) ||
      (h_expected && !h_mismatch))
    return reconstruct_crc_host_batch_dev(dec, h_in, in_stripe_stride, in_unit_stride, present_units, num_present,
                                          erased, n_erased, h_out, out_stripe_stride, out_unit_stride, num_stripes, len,
                                          checksum_type, bpc, h_expected, expected_big_endian, h_out_crcs,
                                          out_big_endian, h_mismatch, stripes_per_chunk);
  const size_t nwin = (len + bpc - 1) / bpc, n_all = static_cast<size_t>(dec->k + dec->p);
  return host_batch_split(dec, num_stripes, e2e_chunk_of(stripes_per_chunk), [&](size_t s0, size_t s1) {
    return reconstruct_crc_host_batch_dev(
        dec, h_in + s0 * in_stripe_stride, in_stripe_stride, in_unit_stride, present_units, num_present, erased,
        n_erased, h_out ? h_out + s0 * out_stripe_stride : nullptr, out_stripe_stride, out_unit_stride, s1 - s0, len,
        checksum_type, bpc, h_expected ? h_expected + s0 * n_all * nwin : nullptr, expected_big_endian,
        h_out_crcs ? h_out_crcs + s0 * static_cast<size_t>(n_erased) * nwin : nullptr, out_big_endian,
        h_mismatch ? h_mismatch + s0 : nullptr, stripes_per_chunk);
  });
}

// ---- host-side math ----------------------------------------------------------------------------

int ozec_rs_encode_matrix(int k, int p, uint8_t *matrix) {
  if (!matrix || k <= 0 || p <= 0 || k + p >= 256) return fail(OZEC_EINVAL, "Invalid numDataUnits and numParityUnits");
  std::vector<uint8_t> m = ozec::cauchy_matrix(k, p);
  std::memcpy(matrix, m.data(), m.size());
  return OZEC_OK;
}

int ozec_rs_decode_matrix(int k, int p, const int *valid, const int *erased, int n_erased, uint8_t *out) {
  if (!valid || n_erased < 0 || (n_erased && (!erased || !out)) || k <= 0 || p <= 0 || k + p >= 256)
    return fail(OZEC_EINVAL, "invalid arguments");
  for (int i = 0; i < k; ++i)
    if (valid[i] < 0 || valid[i] >= k + p) return fail(OZEC_EINVAL, "valid index out of range");
  for (int i = 0; i < n_erased; ++i)
    if (erased[i] < 0 || erased[i] >= k + p) return fail(OZEC_EINVAL, "erased index out of range");
  std::vector<uint8_t> rows;
  if (!ozec::decode_matrix(k, p, valid, erased, n_erased, rows)) return fail(OZEC_ENOTINVERTIBLE, "Not invertible");
  if (!rows.empty()) std::memcpy(out, rows.data(), rows.size());
  return OZEC_OK;
}

int ozec_gf_invert_matrix(uint8_t *in, uint8_t *out, int n) {
  if (!in || !out || n <= 0) return fail(OZEC_EINVAL, "invalid arguments");
  if (!ozec::invert_matrix(in, out, n)) return fail(OZEC_ENOTINVERTIBLE, "Not invertible");
  return OZEC_OK;
}

uint8_t ozec_gf_mul(uint8_t a, uint8_t b) { return ozec::GF256::get().mul(a, b); }

int ozec_parse_replication(const char *s, int *codec, int *k, int *p, int *chunk) {
  // ECReplicationConfig(String), ECReplicationConfig.java:96-130
  static const std::regex re("([a-zA-Z]+)-(\\d+)-(\\d+)-(\\d+)([kK])?");
  std::cmatch m;
  if (!s || !std::regex_match(s, m, re))
    return fail(OZEC_EINVAL, std::string("EC replication config should be defined in the form rs-3-2-1024k, "
                                         "rs-6-3-1024k; or rs-10-4-1024k. Provided configuration was: ") +
                                 (s ? s : "null"));
  std::string name = m[1].str();
  for (auto &ch : name) ch = static_cast<char>(std::tolower(ch));
  int c;
  if (name == "rs") c = OZEC_CODEC_RS;
  else if (name == "xor") c = OZEC_CODEC_XOR;
  else return fail(OZEC_EINVAL, "The codec " + m[1].str() + " is invalid. It must be one of rs,xor.");
  long long d = 0, q = 0, cs = 0;
  try {
    d = std::stoll(m[2].str());
    q = std::stoll(m[3].str());
    cs = std::stoll(m[4].str());
  } catch (...) {
    return fail(OZEC_EINVAL, "NumberFormatException");
  }
  if (d > INT32_MAX || q > INT32_MAX || cs > INT32_MAX) return fail(OZEC_EINVAL, "NumberFormatException");
  if (d <= 0 || q <= 0)
    return fail(OZEC_EINVAL, "Data and parity part in EC replication config supposed to be positive numbers");
  if (cs <= 0) return fail(OZEC_EINVAL, "The ecChunkSize (" + std::to_string(cs) + ") be greater than zero");
  if (m[5].matched) cs *= 1024;  // Java int arithmetic wraps here; values that large are rejected upstream
  if (codec) *codec = c;
  if (k) *k = static_cast<int>(d);
  if (p) *p = static_cast<int>(q);
  if (chunk) *chunk = static_cast<int>(static_cast<int32_t>(cs));
  return OZEC_OK;
}

static bool listed(const int *ids, size_t n, int64_t v) {
  for (size_t i = 0; i < n; ++i)
    if (ids[i] == v) return true;
  return false;
}

int ozec_set_tuning(const char *key, int64_t value) {
  if (!key) return fail(OZEC_EINVAL, "null key");
  const std::string k(key);
  auto &t = ozec::g_tune;
  auto bad = [&] { return fail(OZEC_EINVAL, "invalid value " + std::to_string(value) + " for tuning key " + k); };
  if (k == "gf_variant" || k == "crc_variant") {
    const bool gf = k == "gf_variant";
    const int *ids = gf ? ozec::kGfVariants : ozec::kCrcVariants;
    const size_t n = gf ? std::size(ozec::kGfVariants) : std::size(ozec::kCrcVariants);
    if (value != 0 && !listed(ids, n, value)) return bad();
    (gf ? t.gf_variant : t.crc_variant).store(static_cast<int>(value));
  } else if (k == "grid" || k == "crc_grid" || k == "crc_run") {
    if (value < 0) return bad();
    (k == "grid" ? t.grid : k == "crc_grid" ? t.crc_grid : t.crc_run).store(value);
  } else if (k == "unit_map") {
    if (value != 0 && value != 1) return bad();
    t.unit_map.store(static_cast<int>(value));
  } else if (k == "host_chunk") {
    if (value <= 0) return bad();
    t.host_chunk.store(value);
  } else if (k == "host_chunk_shared") {
    if (value < 0) return bad();
    t.host_chunk_shared.store(value);
  } else if (k == "host_slots") {
    if (value <= 0) return bad();
    t.host_slots.store(value);
  } else if (k == "queue_batches") {
    if (value < 0 || value > 64) return bad();
    t.queue_batches.store(value);
  } else if (k == "copy_threads") {
    if (value < 0 || value > 256) return bad();
    ozec::set_copy_threads(static_cast<int>(value));
  } else if (k == "copy_stream") {
    if (!ozec::set_copy_stream(static_cast<int>(value))) return bad();
  } else if (k == "copy_spin_us") {
    if (value < 0 || value > 100000) return bad();
    ozec::set_copy_spin_us(value);
  } else if (k == "e2e_chunk") {
    if (value <= 0) return bad();
    t.e2e_chunk.store(value);
  } else if (k == "e2e_rect") {
    if (value != 0 && value != 1) return bad();
    t.e2e_rect.store(static_cast<int>(value));
  } else if (k == "host_graph") {
    if (value < 0) return bad();
    t.host_graph.store(value);
  } else if (k == "host_duplex") {
    if (value < 0) return bad();
    t.host_duplex.store(value);
  } else if (k == "host_zero_copy") {
    if (value < 0) return bad();
    t.host_zero_copy.store(value);
  } else if (k == "host_zc_shared_max") {
    if (value < 0) return bad();
    t.host_zc_shared_max.store(value);
  } else if (k == "stream_priority") {
    if (value != 0 && value != 1) return bad();
    t.stream_priority.store(static_cast<int>(value));
  } else if (k == "host_zc_chunks") {
    if (value < 1 || value > 16) return bad();
    t.host_zc_chunks.store(value);
  } else if (k == "host_pitch16") {
    if (value != 0 && value != 1) return bad();
    t.host_pitch16.store(static_cast<int>(value));
  } else if (k == "fused_min_units" || k == "rec_min_units" || k == "nb_small_units") {
    if (value < 0) return bad();
    auto &knob = k == "fused_min_units" ? t.fused_min_units : k == "rec_min_units" ? t.rec_min_units : t.nb_small_units;
    knob.store(value);
  } else {
    return fail(OZEC_EINVAL, "unknown tuning key " + k);
  }
  return OZEC_OK;
}

int ozec_get_tuning(const char *key, int64_t *value) {
  if (!key || !value) return fail(OZEC_EINVAL, "null argument");
  const std::string k(key);
  const auto &t = ozec::g_tune;
  if (k == "gf_variant") *value = t.gf_variant.load();
  else if (k == "crc_variant") *value = t.crc_variant.load();
  else if (k == "grid") *value = t.grid.load();
  else if (k == "crc_grid") *value = t.crc_grid.load();
  else if (k == "crc_run") *value = t.crc_run.load();
  else if (k == "unit_map") *value = t.unit_map.load();
  else if (k == "host_chunk") *value = t.host_chunk.load();
  else if (k == "host_chunk_shared") *value = t.host_chunk_shared.load();
  else if (k == "host_slots") *value = t.host_slots.load();
  else if (k == "queue_batches") *value = t.queue_batches.load();
  else if (k == "e2e_chunk") *value = t.e2e_chunk.load();
  else if (k == "e2e_rect") *value = t.e2e_rect.load();
  else if (k == "host_graph") *value = t.host_graph.load();
  else if (k == "host_duplex") *value = t.host_duplex.load();
  else if (k == "host_zero_copy") *value = t.host_zero_copy.load();
  else if (k == "host_zc_chunks") *value = t.host_zc_chunks.load();
  else if (k == "stream_priority") *value = t.stream_priority.load();
  else if (k == "copy_spin_us") *value = ozec::copy_spin_us();
  else if (k == "host_zc_shared_max") *value = t.host_zc_shared_max.load();
  else if (k == "host_pitch16") *value = t.host_pitch16.load();
  else if (k == "fused_min_units") *value = t.fused_min_units.load();
  else if (k == "rec_min_units") *value = t.rec_min_units.load();
  else if (k == "nb_small_units") *value = t.nb_small_units.load();
  else return fail(OZEC_EINVAL, "no readable tuning key " + k);
  return OZEC_OK;
}

int ozec_tuning_variants(const char *key, int *ids, int cap) {
  if (!key) return fail(OZEC_EINVAL, "null key");
  const std::string k(key);
  const int *v;
  size_t n;
  if (k == "gf_variant") {
    v = ozec::kGfVariants;
    n = std::size(ozec::kGfVariants);
  } else if (k == "crc_variant") {
    v = ozec::kCrcVariants;
    n = std::size(ozec::kCrcVariants);
  } else {
    return fail(OZEC_EINVAL, "no variant list for tuning key " + k);
  }
  for (size_t i = 0; i < n && static_cast<int>(i) < cap; ++i)
    if (ids) ids[i] = v[i];
  return static_cast<int>(n);
}

uint32_t ozec_crc_combine(int checksum_type, uint32_t a, uint32_t b, uint64_t len_b) {
  CrcType t;
  if (crc_type_of(checksum_type, &t)) return 0;
  return CrcMath::get(t).combine(a, b, len_b);
}

// ---- COMPOSITE_CRC ------------------------------------------------------------------------------------

int ozec_crc_monomial(int checksum_type, int64_t len, uint32_t *out) {
  CrcType t;
  if (int rc = crc_type_of(checksum_type, &t)) return rc;
  if (!out) return fail(OZEC_EINVAL, "null output");
  if (len < 0) return fail(OZEC_EINVAL, "lengthBytes must be positive, got " + std::to_string(len));
  *out = CrcMath::get(t).monomial(static_cast<uint64_t>(len));
  return OZEC_OK;
}

int ozec_crc_compose(int checksum_type, uint32_t crc_a, uint32_t crc_b, int64_t len_b, uint32_t *out) {
  CrcType t;
  if (int rc = crc_type_of(checksum_type, &t)) return rc;
  if (!out) return fail(OZEC_EINVAL, "null output");
  if (len_b < 0) return fail(OZEC_EINVAL, "lengthBytes must be positive, got " + std::to_string(len_b));
  *out = CrcMath::get(t).combine(crc_a, crc_b, static_cast<uint64_t>(len_b));
  return OZEC_OK;
}

}  // extern "C"

// The shift-by-hint operator is built on the first update that needs it (ECBlockChecksumComputer makes a fresh
// composer per window CRC and only ever takes its `cur == 0` branch, so creation must stay cheap).
struct ozec_crc_composer {
  const CrcMath *cm = nullptr;
  int64_t hint = 0, stripe_len = 0, pos = 0;
  uint32_t cur = 0;
  bool hint_ready = false;
  uint32_t hint_cols[32] = {};
  std::vector<uint8_t> digest;

  void emit() {
    for (int s = 24; s >= 0; s -= 8) digest.push_back(static_cast<uint8_t>(cur >> s));  // CrcUtil.intToBytes
  }
};

extern "C" {

int ozec_crc_composer_create(int checksum_type, int64_t hint, int64_t stripe_length, ozec_crc_composer **out) {
  CrcType t;
  if (int rc = crc_type_of(checksum_type, &t)) return rc;
  if (!out) return fail(OZEC_EINVAL, "null output handle");
  if (hint < 0) return fail(OZEC_EINVAL, "lengthBytes must be positive, got " + std::to_string(hint));
  auto *c = new (std::nothrow) ozec_crc_composer();
  if (!c) return fail(OZEC_ENOMEM, "out of memory");
  c->cm = &CrcMath::get(t);
  c->hint = hint;
  c->stripe_len = stripe_length > 0 ? stripe_length : INT64_MAX;
  *out = c;
  return OZEC_OK;
}

int ozec_crc_composer_update(ozec_crc_composer *c, uint32_t crc, int64_t bpc) {
  if (!c) return fail(OZEC_EINVAL, "null composer");
  if (c->cur == 0) {
    c->cur = crc;
  } else if (bpc == c->hint) {
    if (!c->hint_ready) {
      c->cm->shift_matrix(static_cast<uint64_t>(c->hint), c->hint_cols);
      c->hint_ready = true;
    }
    c->cur = CrcMath::apply(c->hint_cols, c->cur) ^ crc;
  } else {
    if (bpc < 0) return fail(OZEC_EINVAL, "lengthBytes must be positive, got " + std::to_string(bpc));
    c->cur = c->cm->combine(c->cur, crc, static_cast<uint64_t>(bpc));
  }
  c->pos += bpc;
  if (c->pos > c->stripe_len)
    return fail(OZEC_EMISMATCH, "Current position in stripe '" + std::to_string(c->pos) +
                                    "' after advancing by bytesPerCrc '" + std::to_string(bpc) +
                                    "' exceeds stripeLength '" + std::to_string(c->stripe_len) +
                                    "' without stripe alignment.");
  if (c->pos == c->stripe_len) {
    c->emit();
    c->cur = 0;
    c->pos = 0;
  }
  return OZEC_OK;
}

int ozec_crc_composer_update_bytes(ozec_crc_composer *c, const uint8_t *b, size_t len, int64_t bpc) {
  if (!c) return fail(OZEC_EINVAL, "null composer");
  if (len % 4 != 0)
    return fail(OZEC_EINVAL, "Trying to update CRC from byte array with length '" + std::to_string(len) +
                                 "' which is not a multiple of 4!");
  for (size_t i = 0; i < len; i += 4) {
    const uint32_t v = (uint32_t{b[i]} << 24) | (uint32_t{b[i + 1]} << 16) | (uint32_t{b[i + 2]} << 8) | b[i + 3];
    if (int rc = ozec_crc_composer_update(c, v, bpc)) return rc;
  }
  return OZEC_OK;
}

size_t ozec_crc_composer_pending(const ozec_crc_composer *c) {
  return c ? c->digest.size() + (c->pos > 0 ? 4 : 0) : 0;
}

int ozec_crc_composer_digest(ozec_crc_composer *c, uint8_t *out, size_t cap, size_t *len) {
  if (!c) return fail(OZEC_EINVAL, "null composer");
  const size_t need = ozec_crc_composer_pending(c);
  if (len) *len = need;
  if (need > cap || (need && !out)) return fail(OZEC_EINVAL, "digest buffer too small");
  if (c->pos > 0) {
    c->emit();
    c->cur = 0;
    c->pos = 0;
  }
  if (need) std::memcpy(out, c->digest.data(), need);
  c->digest.clear();
  return OZEC_OK;
}

void ozec_crc_composer_free(ozec_crc_composer *c) { delete c; }

int ozec_crc_compose_windows_batch(int checksum_type, const uint32_t *d_crcs, int64_t crc_cell_stride,
                                   size_t num_cells, size_t num_windows, size_t bpc, size_t last_len,
                                   int crcs_big_endian, uint32_t *d_out, int out_big_endian, void *stream) {
  CrcType t;
  if (int rc = crc_type_of(checksum_type, &t)) return rc;
  if (num_cells == 0) return OZEC_OK;
  if (!d_crcs || !d_out) return fail(OZEC_EINVAL, "null buffer");
  if (num_windows == 0 || bpc == 0 || last_len == 0 || last_len > bpc)
    return fail(OZEC_EINVAL, "need num_windows > 0 and 0 < last_len <= bpc");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  const CrcMath &cm = CrcMath::get(t);
  ozec::ComposeArgs a{};
  a.crcs = d_crcs;
  a.cell_stride = crc_cell_stride;
  a.ncells = static_cast<int64_t>(num_cells);
  a.nwin = static_cast<int64_t>(num_windows);
  a.bpc = static_cast<int64_t>(bpc);
  a.last_len = static_cast<int64_t>(last_len);
  a.poly = cm.poly();
  a.mono_bpc = cm.monomial(bpc);
  a.mono_last = cm.monomial(last_len);
  a.big_endian_in = crcs_big_endian;
  a.big_endian_out = out_big_endian;
  a.out = d_out;
  OZEC_HIP(ozec::launch_compose_windows(a, pick_stream(ctx, stream)));
  return OZEC_OK;
}

// ---- per-call counters -------------------------------------------------------------------------------

int ozec_stats(int op, ozec_op_stats *out) {
  if (op < 0 || op >= OZEC_NUM_OPS || !out) return fail(OZEC_EINVAL, "unknown op or null output");
  const ozec::OpCounters &c = ozec::g_stats[op];
  out->calls = c.calls.load(std::memory_order_relaxed);
  out->bytes = c.bytes.load(std::memory_order_relaxed);
  out->errors = c.errors.load(std::memory_order_relaxed);
  out->host_ns = c.host_ns.load(std::memory_order_relaxed);
  return OZEC_OK;
}

void ozec_stats_reset(void) {
  for (auto &c : ozec::g_stats) {
    c.calls.store(0);
    c.bytes.store(0);
    c.errors.store(0);
    c.host_ns.store(0);
  }
}

// ---- harness utilities ------------------------------------------------------------------------------

int ozec_fill_splitmix64_cells(uint8_t *d_base, int64_t cell_stride, size_t ncells, size_t n, uint64_t seed,
                               uint64_t first_stream, void *stream) {
  if (n == 0 || ncells == 0) return OZEC_OK;
  if (!d_base) return fail(OZEC_EINVAL, "null buffer");
  DevCtx *ctx;
  if (int rc = get_ctx(&ctx)) return rc;
  OZEC_HIP(ozec::launch_fill_splitmix64(d_base, cell_stride, static_cast<int64_t>(ncells), static_cast<int64_t>(n),
                                        seed, first_stream, pick_stream(ctx, stream)));
  return OZEC_OK;
}

int ozec_fill_splitmix64(uint8_t *d_dst, size_t n, uint64_t seed, uint64_t stream_id, void *stream) {
  return ozec_fill_splitmix64_cells(d_dst, 0, 1, n, seed, stream_id, stream);
}

}  // extern "C"
