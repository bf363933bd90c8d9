// Launch-side interface of the gfx950 kernels in kernels.hip (host code only sees these declarations).
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>

#include "../../include/ozec.h"

namespace ozec {

// One coding job: rows x k coefficient matrix applied to k input units of every stripe.
//   input j of stripe s  : in  + s * in_stripe_stride  + in_off[j]
//   output r of stripe s : out + s * out_stripe_stride + out_off[r]
// (base may be null with absolute addresses in the offsets; strides may be 0 for a single stripe).
struct CodeArgs {
  const uint8_t *in;
  uint8_t *out;
  int64_t in_stripe_stride;
  int64_t out_stripe_stride;
  int64_t nstripes;
  int64_t len;
  int32_t k;
  int32_t rows;
  int32_t all_ones;  // every coefficient is 1 (XOR codec): pure XOR kernel
  int32_t unit_map;  // block order: 0 XCD-contiguous (default, see xcd_remap), 1 plain blockIdx order
  int64_t in_off[OZEC_MAX_K];
  int64_t out_off[OZEC_MAX_ROWS];
  uint8_t coef[OZEC_MAX_ROWS * OZEC_MAX_K];  // row-major rows x k
  // block-group layout (0 = flat): stripe s lives in group s / grp_stripes at g * {in,out}_grp_stride, at
  // (s % grp_stripes) * {in,out}_stripe_stride within it (ozec_encode_crc_block_groups)
  int64_t grp_stripes;
  int64_t in_grp_stride;
  int64_t out_grp_stride;
};

// Per-window CRC job over equally sized cells: cell c at base + c * cell_stride, `len` bytes each.
struct CrcArgs {
  const uint8_t *base;
  int64_t cell_stride;
  int64_t ncells;
  int64_t len;
  int64_t bpc;
  int64_t nwin;            // ceil(len / bpc)
  uint32_t *out;           // out[c * out_cell_stride + w]
  int64_t out_cell_stride; // in uint32 elements
  const uint32_t *tables[3];  // device G5 table blobs for this CRC type, B = 1, 2, 4 blocks per lane per step
  const uint32_t *g26[6];     // device G26 table blobs for this CRC type, one per kG26Cfg entry
  const uint32_t *nib;        // device nibble table blob for this CRC type (kNib* layout)
  const uint32_t *xo;         // device XO table blob for this CRC type (kXo* layout)
  const uint32_t *cv;         // device CV table blob for this CRC type (kCv* layout)
  const uint32_t *bshift;     // register shift by bpc bytes (7 tables of 32; kBshift*), null for other bpc
  uint32_t init_full;      // shift(0xFFFFFFFF, bpc bytes)
  uint32_t init_last;      // shift(0xFFFFFFFF, last window bytes)
  int32_t big_endian;
  int32_t raw;             // emit the raw (init 0, no xorout) register instead of getValue()
  uint32_t poly;           // reflected polynomial (bytewise register update of a cell's last 1-15 bytes, fused_nb.hpp)
  // verify mode (expected != null): instead of storing, compare with expected[c * out_cell_stride + w]
  // (stored big-endian when expected_be) and atomicMin (mismatch_base + w) into mismatch[c]
  const uint32_t *expected;
  int32_t *mismatch;
  int32_t expected_be;
  int32_t mismatch_base;
  int32_t unit_map;        // as CodeArgs::unit_map
};

// Fused encode + CRC (bpc % 16 == 0; len % 16 == 0 and 16-B aligned units, or, on the nibble kernel's shapes with
// bpc % 4096 == 0, any length and byte offsets: encode_crc_nb_bytes_supported).
//   encode mode (verify == 0): crc.out = crcs[s][unit][w] for all K inputs and R outputs (out_cell_stride = nwin)
//   reconstruct mode (verify == 1): the K inputs are checked against crc.expected[s][in_unit[j]][w]
//     (exp_units units per stripe) with failures atomicMin'ed into crc.mismatch[s] as in_unit*nwin + w, and only
//     the R rebuilt units' CRCs are stored: crc.out[s][r][w]
struct EncCrcArgs {
  CodeArgs code;
  CrcArgs crc;
  int32_t verify;
  int32_t exp_units;
  int32_t in_unit[OZEC_MAX_K];
  int32_t *work;  // WorkQueue counter slot of a persistent kernel (set by its launcher, work_lease)
};

// Device CRC "G5" table blob (uint32 entries), built on the host (crc_host.cpp), one per (CRC type, B) where
// B = 16-B blocks a lane folds per step.  Every table has 32 entries indexed by a 5-bit group of its input
// and starts on a 128-B boundary, so a ds_read_b32 of random indices is bank-conflict-free.
//   [kG5Blk,  +26*32)   block -> raw CRC: table g holds the contribution of block bits [5g, 5g+5)
//   [kG5Step, +7*32)    register shift by (63*B)*16 bytes (jump to the lane's next chunk)
//   [kG5Tree, +6*7*32)  register shift by 16*B*2^m bytes, m = 0..5 (lane-combine tree)
//   [kG5T0,   +256)     classic byte table T0 (tails of windows not a multiple of 16 B)
constexpr int kG5Blk = 0;
constexpr int kG5Step = 832;
constexpr int kG5Tree = 1056;
constexpr int kG5T0 = 2400;
constexpr int kG5Words = 2656;
constexpr int g5_slot(int B) { return B == 1 ? 0 : B == 2 ? 1 : 2; }

// Device CRC "G26" table blob for the step-grouped kernels: a lane folds B blocks per step, D steps per
// group, and every block is looked up in a table set that already includes its distance to the end of the
// group, so the lane register is shifted once per group instead of once per step.  E = B*D sets:
//   [0, E*kG26Set)          set e = r*B + s: block -> raw CRC advanced by (r*64*B + s)*16 zero bytes, i.e.
//                           the block is s blocks before the end of its step and r steps before the end of
//                           its group.  26 tables of 32 entries; table g is indexed by the 5 (or 4) block bits
//                           g26 extraction g places at bits 2..6 of a byte (kernels.hip g26_block, host
//                           crc_host.cpp g26_bit) -- one SDWA byte-select AND per lookup for 16 of them
//   [g26_gshift(E), +224)   register shift by D*64*B*16 bytes (one group), 7 tables of 5-bit groups
//   [g26_tree(E), +1344)    lane-tree shifts by 16*B*2^m bytes, m = 0..5 (as kG5Tree)
//   [g26_t0(E), +256)       classic byte table T0
constexpr int kG26Set = 26 * 32;
constexpr int g26_gshift(int E) { return E * kG26Set; }
constexpr int g26_tree(int E) { return E * kG26Set + 224; }
constexpr int g26_t0(int E) { return E * kG26Set + 224 + 1344; }
constexpr int g26_words(int E) { return E * kG26Set + 224 + 1344 + 256; }
// (B, D) of each G26 blob slot
constexpr int kG26Slots = 6;
constexpr int kG26Cfg[kG26Slots][2] = {{1, 4}, {2, 2}, {1, 2}, {2, 4}, {1, 8}, {1, 1}};
constexpr int g26_slot(int B, int D) {
  return B == 1 && D == 4   ? 0
         : B == 2 && D == 2 ? 1
         : B == 1 && D == 2 ? 2
         : B == 2 && D == 4 ? 3
         : B == 1 && D == 1 ? 5
                            : 4;
}

// Device CRC "nibble" blob for the nibble-table fused kernel (fused.hip encode_crc_nb): entry
// [e * 512 + p * 16 + n] = raw-CRC contribution of a 16-B block whose only non-zero nibble is n at nibble position p
// (block bits 4p..4p+3, i.e. byte p / 2, low nibble for even p), advanced by e * 1024 zero bytes (the block is e
// steps of a 64-lane wave before the end of its step group).  Same map as the G26 set e of (B = 1, D > e).
constexpr int kNibSets = 4;
constexpr int kNibWords = kNibSets * 32 * 16;

// Device CRC "XO" blob of the nibble kernel's free register shift (fused_nb.hpp, XO variants).  A lane's output
// register U is XORed into the first dword of its next 16-B block before that block's lookups: the raw CRC of
// (block ^ U) is crc(block) advanced by 0 bytes plus U advanced by 16 bytes (the CRC register identity
// raw(U; B) = raw(0; B ^ U)).  With the block tables advanced by kXoAdvance = 1008 bytes, U therefore moves by
// 1008 + 16 = 1024 bytes -- one step of the wave, the shift the register needs -- at the cost of one XOR, and every
// block lands kXoAdvance bytes too far; the register is brought back once per window by the inverse shift.
//   [0, kG26Set)            G26 set: block -> raw CRC advanced by kXoAdvance zero bytes (g26_block extraction)
//   [kXoInv, +224)          register shift by -kXoAdvance bytes (inverse of the advance), 7 tables of 5-bit groups
constexpr int kXoAdvance = 1024 - 16;
constexpr int kXoInv = kG26Set;
constexpr int kXoWords = kG26Set + 224;

// Device CRC "CV" blob of the combined input verification (fused_nb.hpp, CV variants; round 5).  A reconstruction
// checks the window CRCs of the K units it reads; instead of K raw registers (K shifts per step, K lane trees) the CV
// kernel keeps ONE register: input j's nibble contributions are pre-multiplied by x^(8 w_j), w_j = j * kCvStride
// bytes, so the register ends as XOR_j x^(8 w_j) raw_j, and is compared with the same combination of the stored
// CRCs.  Distinct weights make any single-unit error, and two units with the same error pattern, change the
// combination (x^(8 w_a) + x^(8 w_b) is a unit mod P for every pair: tests/test_cv_weights.py); a stripe that fails
// is re-verified unit by unit (nb_reverify), so the first failing (unit, window) reported is the reference's.
//   [j * 512 + p * 16 + n]            nibble table of input j (as kNib* set 0), advanced by j * kCvStride bytes
//   [kCvShift + j * 224 + g * 32 + v] register shift by j * kCvStride bytes, 7 tables of 5-bit groups
constexpr int kCvMaxK = 16;
constexpr int kCvStride = 1024;
constexpr int kCvShift = kCvMaxK * 512;
constexpr int kCvWords = kCvShift + kCvMaxK * 224;
constexpr int32_t kMismatchSuspect = 0x7ffffffe;  // mismatch[s] while a stripe awaits its unit-by-unit re-verify

// Device "bshift" blob: the register shift by bpc bytes for bpc = 4 KiB << i, i < kBshiftN (7 tables of 32 each), used by
// the run check of the streaming verify kernel (kernels.hip crc_windows_g26s VR: the stored CRCs of a run of windows
// folded by Horner's rule into the CRC the run has as one message)
constexpr int kBshiftN = 9;  // 4 KiB .. 1 MiB

// Runtime tuning knobs (ozec_set_tuning): 0 = built-in default.  Process-wide harness knobs for A/B and profiling
// runs (bench.py --tune, scripts/ab.py): every field is an atomic, so setting one while other threads launch is not a
// data race, but a set knob applies to every caller's next launch -- a production process leaves them at 0.
struct TuneKnobs {
  std::atomic<int64_t> grid{0};       // blocks for the coding kernels
  std::atomic<int> gf_variant{0};     // coding-kernel alternate, one of kGfVariants (kernels.hip launch_kr)
  std::atomic<int> crc_variant{0};    // CRC / fused-kernel alternate, one of kCrcVariants
  std::atomic<int64_t> crc_grid{0};   // blocks for the CRC / fused kernels
  std::atomic<int64_t> crc_run{0};    // streaming CRC kernels: bytes of consecutive windows per wave (default 256 KiB)
  std::atomic<int> unit_map{0};       // CodeArgs::unit_map for the coding kernels
  std::atomic<int64_t> host_chunk{4 << 20};  // host-buffer calls: bytes per unit per pipelined chunk (per-chunk stream
                                             // latency ~20 us: 256 KiB chunks ran 16 MiB CRC updates at 2.7 GB/s, 4 MiB
                                             // at 18)
  std::atomic<int64_t> host_chunk_shared{512 << 10};  // the same while other host-buffer calls hold slots (0: host_chunk)
  std::atomic<int64_t> host_slots{8};        // host-buffer calls: staging slots (concurrent calls) per GPU
  std::atomic<int64_t> queue_batches{0};     // stripe queue: batches in the ring (0 = default), read at queue creation
  std::atomic<int64_t> e2e_chunk{32};        // host batches: stripes per pipelined chunk when the caller passes 0
  std::atomic<int> e2e_rect{1};              // host batches: one rectangular copy per chunk (0: one per stripe)
  std::atomic<int64_t> host_graph{256 << 10};  // host-buffer coding calls of one staged chunk up to this many bytes
                                               // per unit replay a cached hipGraph of H2D + kernel + D2H (0: off;
                                               // 64 KiB-cell rs-6-3 stripe from pageable cells 74 -> 64 us)
  std::atomic<int64_t> host_zero_copy{48};  // host-buffer coding calls (ozec_encode / ozec_decode): the coding kernel
                                           // reads the pinned caller buffers or libozec's pinned staging and writes
                                           // the outputs over PCIe itself, in place of H2D + kernel + D2H, on a grid
                                           // of this many blocks (0: off).  HIP's SDMA copies run at the link rate on
                                           // some streams and at a third of it on others (profiles/r06/engines/); a
                                           // 1 MiB-cell rs-6-3 stripe from pinned memory 190-400 -> 150 us
  std::atomic<int64_t> host_zc_chunks{2};  // a lone zero-copy call from pageable (or callback-fed) units runs in
                                           // this many column chunks of at least 256 KiB per unit, the staging
                                           // copies of one overlapping the kernel on another (1: no overlap)
  std::atomic<int64_t> host_zc_shared_max{64 << 10};  // host coding calls of at most this many bytes per unit take
                                                     // zero copy even beside other calls in flight (0: only a lone
                                                     // call does).  JNI 64 KiB cells, 16 threads: 238 -> 174-177 us
                                                     // per stripe; 256 KiB cells at 4 threads lose (145 -> 212-245
                                                     // us), profiles/r06/jni_forms/jnisweep_r6r.json
  std::atomic<int> stream_priority{0};  // libozec's streams made by hipStreamCreateWithFlags (0) or by
                                        // hipStreamCreateWithPriority at the default priority (1), read when a stream
                                        // is made.  In a probe the first plain stream's 1-D copies run at the link
                                        // rate and every later one's at half (H2D) to a third (D2H) of it, while
                                        // streams made with a priority all run at the link rate
                                        // (profiles/r06/engines/engines_how*.json); libozec's own copy patterns (2-D
                                        // rect copies, concurrent slots, the host-batch pipelines) measured the same
                                        // either way (profiles/r06/engines/ab_stream_priority/), so the default stays
  std::atomic<int64_t> host_duplex{0};  // pinned host-buffer coding calls of at least this many bytes per unit go
                                        // up, through the kernel and back in column chunks, the D2H of chunk c on a
                                        // second stream beside the H2D of chunk c+1 (0: off, the default: 512 KiB
                                        // lost in both A/Bs -- JNI 1 MiB cells 263-294 -> 317-343 us at 1 thread,
                                        // 492-501 -> 774-779 us at 4; pinned batches 28.1-29.6 -> 23.4-23.5 GB/s,
                                        // profiles/r05/duplex/)
  std::atomic<int> host_pitch16{0};  // host batches: device unit pitch = the cell length (0, default) or the length
                                     // rounded up to 16 B (1: every unit 16-B aligned, at the cost of a 2D copy per
                                     // stripe each way; one rs-6-3 stripe of 700,001-B cells 245 -> 190 us, of
                                     // 1,007-B cells 117 -> 68 us with 0, profiles/r05/bytes/)
  // Small fused batches (scripts/small_batch_ab.py, profiles/r05/small/: rs-6-3 encode + CRC32C of 1 MiB cells, us per
  // call for the persistent default / the 4-wave geometry 222 / the unfused kernels):
  //   1 stripe 161 / 57 / 14, 16 stripes 145 / 61 / 65, 128 stripes 306 / 235 / 424, 256 stripes 513 / 487 / 808;
  //   full C3r / C5dev size (2048 / 4096 stripes) 222 is 8 % slower than the default.  rs-10-4 reconstruction of 4
  //   units: 1 stripe 241 / 91 / 95, 64 stripes 366 / 226 / 400.
  std::atomic<int64_t> fused_min_units{1024};  // fused encode + CRC batches on 16-B aligned units with fewer
                                               // (stripe, window) units take the unfused kernels (coding, then one
                                               // CRC pass), which spread a small batch over many more waves (0: always
                                               // fused)
  std::atomic<int64_t> rec_min_units{0};       // the same for fused reconstructions (verify + decode + CRC): 0, the
                                               // 4-wave geometry is never slower than their k + 2 unfused launches
  std::atomic<int64_t> nb_small_units{16384};  // fused batches of fewer units take the 4-wave nibble geometry (variant
                                               // 222) when no variant is pinned (0: off)
};

// Kernel alternates the library holds besides the defaults, selectable with ozec_set_tuning for A/B (0 = default).
// Every id has a parity test (tests/variants.py lists them; tests/test_variants.py checks the lists agree with
// ozec_tuning_variants); ozec_set_tuning rejects any other id.
//   gf_variant (coding kernel gf_code_vec, kernels.hip launch_kr): 1, 5, 11
//   crc_variant, by kernel family:
//     streaming CRC (launch_crc_windows): 20, 22 -- D-step groups instead of the XO default; 24 -- verify without
//       the run check (round 4's default); 28 / 29 -- compute with one lane tree per window (round 4) / per 4 windows
//     fused XOR codec (launch_enc_crc_kr, R = 1 all-ones): 2 no register shortcut, 3 D = 4 with loads one step ahead
//       (the round-1 default), 4 / 5 XO with D = 4 / 2,
//       20 / 21 streaming kernel with a ring of 2 / 4 steps
//     fused RS (launch_encode_crc): 49 per-window kernel, 56 / 59 streamed-input kernel (fused.hip), 62 / 87 / 150 /
//       163 / 167 / 170-174 / 176 / 177 / 187 / 189-194 / 196 / 220-222 / 231 / 234 nibble-table kernel (fused_nb.hpp
//       launch_nb_kr)
constexpr int kGfVariants[] = {1, 5, 11};
constexpr int kCrcVariants[] = {2,   3,   4,   5,   20,  21,  22,  24,  28,  29,  49,  56,  59,  62,  87,  150, 163, 167, 170, 171,
                                 172, 173, 174, 176, 177, 187, 189, 190, 191, 192, 193, 194, 196, 220, 221, 222,
                                 231, 234};

extern TuneKnobs g_tune;

// a non-blocking stream for libozec's copies and launches (TuneKnobs::stream_priority)
inline hipError_t make_stream(hipStream_t *s) {
  if (g_tune.stream_priority.load(std::memory_order_relaxed) == 0) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) least = 0;
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, least);
}

// Per-thread cap on the coding kernels' grid (0: none), set around a zero-copy launch (capi.cpp staged_pipeline): a
// kernel streaming over PCIe does best with a few dozen blocks looping over the chunks, so the reads of one chunk
// overlap the writes of the previous one, rather than every block reading at once and writing at once.
extern thread_local int64_t t_grid_cap;
struct GridCap {
  int64_t prev;
  explicit GridCap(int64_t cap) : prev(t_grid_cap) { t_grid_cap = cap; }
  ~GridCap() { t_grid_cap = prev; }
};

hipError_t launch_code(const CodeArgs &a, hipStream_t stream);
hipError_t launch_crc_windows(const CrcArgs &a, hipStream_t stream);
hipError_t launch_encode_crc(const EncCrcArgs &a, hipStream_t stream);
// d_mismatch[i] == INT32_MAX (no failure recorded) -> -1
hipError_t launch_finish_mismatch(int32_t *d_mismatch, int64_t n, hipStream_t stream);

// CrcComposer over each cell's window CRCs: windows of bpc bytes, the last of last_len
struct ComposeArgs {
  const uint32_t *crcs;      // [cell][window], stored ints ((int)getValue()), optionally big-endian
  int64_t cell_stride;       // in CRCs
  int64_t ncells, nwin;
  int64_t bpc, last_len;
  uint32_t poly;             // reversed polynomial (CrcUtil.getCrcPolynomialForType)
  uint32_t mono_bpc, mono_last;  // x^(8*bpc), x^(8*last_len) mod poly (CrcUtil.getMonomial)
  int big_endian_in, big_endian_out;
  uint32_t *out;             // [cell]
};
hipError_t launch_compose_windows(const ComposeArgs &a, hipStream_t stream);
hipError_t launch_fill_splitmix64(uint8_t *base, int64_t cell_stride, int64_t ncells, int64_t n, uint64_t seed,
                                  uint64_t first_stream, hipStream_t stream);
// true when the fused kernel supports this (k, rows) pair with the given geometry
bool encode_crc_supported(const CodeArgs &a, int64_t bpc);
// whether a supported fused batch of nwin windows per stripe should run fused: at least min_units (stripe, window)
// units (TuneKnobs::fused_min_units / rec_min_units), whatever the units' alignment (unaligned units follow the same
// rule: their unfused kernels run at full rate too, kernels.hip encode_crc_fused_pays)
bool encode_crc_fused_pays(const CodeArgs &a, int64_t nwin, int64_t min_units);
// the streamed-input fused kernel (fused.hip): RS shapes with full windows, bpc % 4096 == 0; `e` already rebased
bool encode_crc_lv_supported(const EncCrcArgs &e);
// the nibble-table kernel (fused_nb.hpp): the same shapes, and a short last window of any whole number of 16-B blocks
bool encode_crc_nb_supported(const EncCrcArgs &e);
bool encode_crc_nb_bytes_supported(const CodeArgs &a, int64_t bpc);
// tail: cells of any length (nb_tail); wide: units 2 GiB or more apart (`e` NOT rebased; one descriptor per unit)
hipError_t launch_encode_crc_lv(const EncCrcArgs &e, hipStream_t stream, int variant, bool tail = false,
                                bool wide = false);

// WorkQueue counter slots of the persistent kernels (device.hpp WorkQueue; pool in work_slots.cpp).  work_lease gives a
// zeroed slot of the current device, not in use by any launch still running, or null (capturing stream, pool full,
// allocation failure: the caller takes a non-persistent form); work_return hands it back, `used` when a kernel that
// counts on it was enqueued on `st` (an event recorded behind it gates the next lease).
// counter slot layout (device.hpp WorkQueue)
constexpr int kWqStride = 16;                 // ints between counters (64 B: one counter per cache line)
constexpr int kWqDone = 8 * kWqStride;        // finished-wave counter
constexpr int kWqInts = kWqDone + kWqStride;  // ints per slot
struct WorkSlot {
  int device = -1;
  int32_t *ctr = nullptr;
  hipEvent_t done = nullptr;
  bool recorded = false;  // `done` marks the last launch that used the slot (or the slot's zeroing)
  bool leased = false;
};
WorkSlot *work_lease(hipStream_t st);
void work_return(WorkSlot *w, hipStream_t st, bool used);

}  // namespace ozec
