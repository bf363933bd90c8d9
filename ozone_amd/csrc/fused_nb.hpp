// Nibble-table fused kernel (encode_crc_nb) and its launcher, instantiated per (K, R) shape in its own translation
// unit (fused_nb_<K>_<R>.hip) so the variants of the nine shapes compile in parallel; fused.hip dispatches.
#pragma once
#include <algorithm>

#include "device.hpp"

namespace ozec {


#define OZEC_NB_SHAPES(X) X(6, 3) X(6, 2) X(6, 1) X(3, 2) X(3, 1) X(10, 4) X(10, 3) X(10, 2) X(10, 1)
#define OZEC_NB_DECL(K, R) \
  hipError_t launch_nb_##K##_##R(const EncCrcArgs &e, hipStream_t st, int v, bool tail, bool wide);
OZEC_NB_SHAPES(OZEC_NB_DECL)

namespace {

// ------------------------------------------------------------------------------------------------
// Nibble-table fused kernel: the GF products and the CRC of every input share their LDS lookups.
//
// encode_crc_lv spends ~23 VALU per input dword on the GF part (5 selector ops + 3 v_perm + 1.5 XOR per output)
// and ~12 per input dword on the CRC index math, and is VALU-issue bound.  Here every nibble n of
// every input byte is looked up ONCE, with one ds_read_b64, in a table whose 8-B entry holds
//   .x = the products c_rj * n (n shifted to its nibble half) for the R outputs, byte r = output r,
//   .y = the raw-CRC contribution of n at its nibble position in the 16-B block (kNib* tables, distance set d).
// Per input block: 32 index ops (one SDWA op each: (byte << 4) & 0xf0 and byte & 0xf0), 32 lookups, 16 XORs
// into per-byte-position GF accumulators A[i] and 16 into the unit's CRC register -- 64 VALU against ~141 for
// rs-10-4 in encode_crc_lv.  A[i] holds the R output bytes of byte position i; a 4x4 byte transpose (8 v_perm per
// dword for R = 4) turns them into the R output dwords, whose CRCs use the G26 lookups as before.
//
// Tables: for each distance set d (D of them), input j and nibble position p, 16 entries of 8 B at a 16-B stride
// with the tables of p and p ^ 1 interleaved (+0 / +8): under ds_read_b64 banking ((a/4) mod 64) the 16 entries
// of a table cover 32 distinct banks, so random nibbles never conflict.  K*D*4 KiB of LDS (40 KiB for rs-10-4 at
// D = 1), built once per workgroup; the grid is persistent (one resident set of workgroups).
// Windows are a whole number of D-step groups (bpc a multiple of 4 KiB); a cell's short last window is front-padded
// with virtual zero blocks to whole groups (below).
__device__ __forceinline__ uint32_t nib_lo_idx(uint32_t w, int q, uint32_t v4) {  // ((byte_q << 4) & 0xf0)
  uint32_t d;
  switch (q) {
    case 0: asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(d) : "v"(v4), "v"(w)); break;
    case 1: asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(d) : "v"(v4), "v"(w)); break;
    case 2: asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(d) : "v"(v4), "v"(w)); break;
    default: asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(d) : "v"(v4), "v"(w)); break;
  }
  return d;
}
__device__ __forceinline__ uint32_t nib_hi_idx(uint32_t w, int q, uint32_t vf0) {  // (byte_q & 0xf0)
  uint32_t d;
  switch (q) {
    case 0: asm("v_and_b32 %0, %1, %2" : "=v"(d) : "v"(vf0), "v"(w)); break;
    case 1: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD" : "=v"(d) : "v"(w), "v"(vf0)); break;
    case 2: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD" : "=v"(d) : "v"(w), "v"(vf0)); break;
    default: asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD" : "=v"(d) : "v"(w), "v"(vf0)); break;
  }
  return d;
}
__device__ __forceinline__ uint2 lds64(const void *base, uint32_t byte_off) {
  return *reinterpret_cast<const uint2 *>(reinterpret_cast<const char *>(base) + byte_off);
}

// byte offset of the entry region of (distance set d, input j, byte i): lo-nibble table at +0, hi at +8
template <int K>
constexpr uint32_t nb_region(int d, int j, int i) {
  return static_cast<uint32_t>(((d * K + j) * 16 + i) * 256);
}

// store (or, reconstructing, check) the finished window CRC of unit q (inputs 0..K-1, then the R outputs)
template <int K, int R>
__device__ __forceinline__ void nb_emit(const EncCrcArgs &e, int64_t s, int64_t w, int q, uint32_t v, uint32_t init) {
  const CrcArgs &cr = e.crc;
  const int64_t nwin = cr.nwin;
  if (!e.verify) {
    cr.out[(s * (K + R) + q) * nwin + w] = crc_finish(v, init, cr.raw, cr.big_endian);
  } else if (q >= K) {
    cr.out[(s * R + (q - K)) * nwin + w] = crc_finish(v, init, cr.raw, cr.big_endian);
  } else if (cr.expected) {
    const int64_t idx = (s * e.exp_units + e.in_unit[q]) * nwin + w;
    const uint32_t ex = cr.expected_be ? __builtin_bswap32(cr.expected[idx]) : cr.expected[idx];
    if (crc_finish(v, init, 0, 0) != ex) atomicMin(cr.mismatch + s, static_cast<int32_t>(e.in_unit[q] * nwin + w));
  }
}

// The same from every emitting lane at once (EM variants): `q` is the lane's unit (a VGPR), the address is computed
// in the VALU and one store (or one compare) serves all units, instead of K + R divergent blocks with scalar
// address math, one per unit.  The lane's input unit comes from a select chain over the kernarg array (static
// indices only, so the array stays in SGPRs).
template <int K, int R>
__device__ __forceinline__ void nb_emit_lane(const EncCrcArgs &e, int64_t s, int64_t w, int q, uint32_t v,
                                             uint32_t init) {
  const CrcArgs &cr = e.crc;
  const int64_t nwin = cr.nwin;
  if (!e.verify) {
    cr.out[(s * (K + R) + q) * nwin + w] = crc_finish(v, init, cr.raw, cr.big_endian);
  } else if (q >= K) {
    cr.out[(s * R + (q - K)) * nwin + w] = crc_finish(v, init, cr.raw, cr.big_endian);
  } else if (cr.expected) {
    int32_t unit = e.in_unit[0];
#pragma unroll
    for (int j = 1; j < K; ++j) unit = q == j ? e.in_unit[j] : unit;
    const int64_t idx = (s * e.exp_units + unit) * nwin + w;
    const uint32_t ex = cr.expected_be ? __builtin_bswap32(cr.expected[idx]) : cr.expected[idx];
    if (crc_finish(v, init, 0, 0) != ex) atomicMin(cr.mismatch + s, static_cast<int32_t>(unit * nwin + w));
  }
}

// A cell whose length is not a multiple of 16 B (round 5; every key's last stripe has one, ECKeyOutputStream.java:276):
// the window loop runs over the last window's whole 16-B blocks only, then the lane holding unit q's raw register
// after the lane tree extends it bytewise over the unit's last tb (1..15) bytes at window offset o0, and the lanes of
// the output units compute those bytes' GF products from the K inputs (s_gf: the R products of each input nibble,
// byte r = output r) and store them.  Once per cell, a few hundred VALU on at most K + R lanes.  Unit offsets of such
// cells are not 16-B (often not 4-B) aligned: gfx950 buffer accesses take any byte offset (the amdhsa ABI runs
// shaders in unaligned access mode; hipcc emits 16-B loads for align-1 data itself).
template <int K, int R>
__device__ __forceinline__ uint32_t nb_tail(const EncCrcArgs &e, __amdgpu_buffer_rsrc_t rin,
                                            __amdgpu_buffer_rsrc_t rout, const uint32_t *s_gf, int q, uint32_t v,
                                            uint32_t o0, int32_t tb) {
  const CodeArgs &a = e.code;
  const uint32_t poly = e.crc.poly;
  uint32_t uoff = static_cast<uint32_t>(a.in_off[0]);  // the lane's unit offset (select chain: kernarg arrays stay SGPR)
#pragma unroll
  for (int j = 1; j < K; ++j) uoff = q == j ? static_cast<uint32_t>(a.in_off[j]) : uoff;
#pragma unroll
  for (int r = 0; r < R; ++r) uoff = q == K + r ? static_cast<uint32_t>(a.out_off[r]) : uoff;
  for (int32_t b = 0; b < tb; ++b) {
    const uint32_t ob = o0 + static_cast<uint32_t>(b);
    uint32_t byte;
    if (q < K) {
      byte = __builtin_amdgcn_raw_buffer_load_b8(rin, ob + uoff, 0, 0);
    } else {
      uint32_t acc = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint32_t x = __builtin_amdgcn_raw_buffer_load_b8(rin, ob, static_cast<int>(a.in_off[j]), 0);
        acc ^= s_gf[j * 32 + (x & 15)] ^ s_gf[j * 32 + 16 + (x >> 4)];
      }
      byte = (acc >> (8 * (q - K))) & 0xffu;
      __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(byte), rout, ob + uoff, 0, 0);
    }
    v ^= byte;
#pragma unroll
    for (int i = 0; i < 8; ++i) v = (v >> 1) ^ (poly & (0u - (v & 1u)));
  }
  return v;
}

// nb_tail for units 2 GiB or more apart (WIDE): the unit's bytes through 64-bit pointers (its base is per lane, and a
// buffer descriptor must be uniform), ib / ob = the stripe's window bases
template <int K, int R>
__device__ __forceinline__ uint32_t nb_tail_wide(const EncCrcArgs &e, const uint8_t *ib, uint8_t *ob,
                                                 const uint32_t *s_gf, int q, uint32_t v, uint32_t o0, int32_t tb) {
  const CodeArgs &a = e.code;
  const uint32_t poly = e.crc.poly;
  int64_t uoff = a.in_off[0];
#pragma unroll
  for (int j = 1; j < K; ++j) uoff = q == j ? a.in_off[j] : uoff;
#pragma unroll
  for (int r = 0; r < R; ++r) uoff = q == K + r ? a.out_off[r] : uoff;
  for (int32_t b = 0; b < tb; ++b) {
    const int64_t o = static_cast<int64_t>(o0) + b;
    uint32_t byte;
    if (q < K) {
      byte = ib[uoff + o];
    } else {
      uint32_t acc = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint32_t x = ib[a.in_off[j] + o];
        acc ^= s_gf[j * 32 + (x & 15)] ^ s_gf[j * 32 + 16 + (x >> 4)];
      }
      byte = (acc >> (8 * (q - K))) & 0xffu;
      ob[uoff + o] = static_cast<uint8_t>(byte);
    }
    v ^= byte;
#pragma unroll
    for (int i = 0; i < 8; ++i) v = (v >> 1) ^ (poly & (0u - (v & 1u)));
  }
  return v;
}

// CV: the combined check of one window, by the whole wave.  `have` marks the lane holding the combined register's total
// v (XOR_j x^(8 w_j) raw_j after the lane tree); lanes 0..K-1 turn input j's stored CRC back into its raw register
// (crc_finish inverted: ~ex ^ init), weight it by x^(8 w_j) (table s_cvs + 224 j) and the 16-lane XOR gives the
// expected combination.  A difference marks the stripe for nb_reverify.
template <int K>
__device__ __forceinline__ void nb_check_combined(const EncCrcArgs &e, const uint32_t *s_cvs, int64_t s, int64_t w,
                                                  int lane, bool have, uint32_t v, uint32_t init) {
  const CrcArgs &cr = e.crc;
  const uint64_t holder = __ballot(have);
  const uint32_t got = static_cast<uint32_t>(__shfl(static_cast<int>(v), static_cast<int>(__builtin_ctzll(holder)), 64));
  uint32_t t = 0;
  if (lane < K) {
    int32_t unit = e.in_unit[0];
#pragma unroll
    for (int j = 1; j < K; ++j) unit = lane == j ? e.in_unit[j] : unit;
    const uint32_t ex0 = cr.expected[(s * e.exp_units + unit) * cr.nwin + w];
    const uint32_t ex = cr.expected_be ? __builtin_bswap32(ex0) : ex0;
    t = g5_shift(s_cvs + lane * 224, ~ex ^ init);
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) t ^= static_cast<uint32_t>(__shfl_xor(static_cast<int>(t), m, 64));
  if (lane == 0 && got != t) atomicMin(cr.mismatch + s, kMismatchSuspect);
}

// K inputs, R outputs, D steps per CRC group, NB input ring slots, WPB waves per block, WAVES min waves per SIMD,
// FENCE: dwords of a block whose lookups go between scheduling fences (2: halves, at most 16 results live; 1:
// quarters; 4: one fence per input block; 0: no fences, the compiler may overlap inputs); RS: reduce-scatter lane tree;
// DYN: 0 one wave per unit, no grid-stride; 1 persistent grid (one resident set of workgroups, tables built once per
// workgroup) fed by the WorkQueue, a claim per unit made one unit ahead
// XO: the output registers move by one step with no shift lookups (kernels.hpp kXo*): each is XORed into the first
// dword of its next output block, whose G26 lookups use the set advanced by kXoAdvance bytes; the advance is undone
// once per window.  Saves R x 7 lookups per step (the input registers keep their D-step shifts: their nibble lookups
// also yield the GF products, which must see the unmodified data)
// EM: the window CRCs leave through nb_emit_lane (one lane-parallel store / compare) instead of K + R unit blocks
// H (< K, XO with D = 2 only): only inputs 0..H-1 get the second distance set (K + H instead of 2K tables of 4 KiB, so
// rs-10-x two-step groups fit two workgroups per CU); inputs H..K-1 are looked up in set 0 and shifted by one step
// after every step (table at kSh1), inputs 0..H-1 by two at the group end
// TAIL: the last 1-15 bytes of cells of any length (nb_tail)
// CV (round 5; reconstructions that verify, 16-B cells): the K input registers are ONE, fed by nibble tables whose CRC
// halves are pre-multiplied by x^(8 w_j) per input (kernels.hpp kCv*), checked against the same combination of the
// stored CRCs; a failing stripe is marked kMismatchSuspect and re-verified unit by unit (nb_reverify).  Saves the
// shifts and lane trees of K - 1 registers: for rs-10-4 one shift per step instead of ~7.5 (H = 5, D = 2) and 5
// registers through the lane tree instead of 14.
// WIDE (round 6): units 2 GiB or more apart (no 32-bit unit offsets after rebase32): one buffer descriptor per unit
// (64-bit base, soffset 0) instead of one per stripe side, the byte tail through 64-bit pointers (nb_tail_wide)
// (Round-3 probes -- output-register groups, VALU / LDS pads, far-addressing without the index OR, late lane-tree
// tables, guided and static persistent orders -- are measured in DESIGN 2.3 and were taken out of the library.)
template <int K, int R, int D, int NB, int WPB, int WAVES, int FENCE = 2, bool RS = true, int DYN = 0, bool XO = false,
          bool EM = false, int H = K, bool TAIL = false, bool CV = false, bool WIDE = false>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(WAVES, 8))) void encode_crc_nb(
    const EncCrcArgs e) {
  static_assert(R >= 1 && R <= 4, "one GF byte per output in the entry dword");
  static_assert(D <= kNibSets, "distance sets of the nibble blob");
  static_assert((D * K) % NB == 0, "the ring must divide the unrolled group so ring indices are compile-time");
  static_assert(DYN == 0 || DYN == 1, "one wave per unit, or the persistent WorkQueue grid");
  static_assert(H == K || (XO && D == 2 && H >= 0 && H < K), "partial second distance set: XO, two-step groups");
  static_assert(!TAIL || (RS && EM), "byte tails leave through the lane-parallel emit");
  static_assert(!CV || (D == 1 && XO && EM && RS && H == K && !TAIL && K <= 16), "combined verify: one-step groups");
  constexpr int kInRegs = CV ? 1 : K;  // input registers
  constexpr int kSets = K + (D - 1) * H;  // (d, j) nibble tables of 4 KiB: all K inputs in set 0, inputs < H in sets >= 1
  // one LDS block: G26 blob of D sets, then the (d, j, p) nibble tables, then the GF dwords of the setup.  Table
  // regions past the 16-bit ds_read offset range are reached with bit 15 set in the index register (one v_or_b32).
  // XO: the input-register shift and the lane-tree shifts of the G26 blob, then the XO blob, instead of the G26 sets
  constexpr uint32_t kXoOff = 224 + 1344;  // XO: word offset of the XO blob
  constexpr uint32_t kShIn = XO ? 0 : g26_gshift(D);  // word offset of the input-register shift
  constexpr uint32_t kTree = XO ? 224 : g26_tree(D);  // and of the lane-tree shifts
  constexpr uint32_t kSh1 = kXoOff + kXoWords;  // H < K: one-step register shift (inputs H..K-1)
  constexpr uint32_t kTW = XO ? kXoOff + kXoWords + (H < K ? 224 : 0) : g26_words(D);
  constexpr uint32_t kTB = (kTW * 4 + 255) / 256 * 256;  // nibble tables
  constexpr uint32_t kLds = kTB + kSets * 4096 + K * 32 * 4 + (CV ? K * 224 * 4 : 0);
  static_assert(kLds <= 160 * 1024, "LDS per workgroup");
  __shared__ __attribute__((aligned(256))) uint8_t s_all[kLds];
  uint32_t *const s_t = reinterpret_cast<uint32_t *>(s_all);
  uint2 *const s_c = reinterpret_cast<uint2 *>(s_all + kTB);
  uint32_t *const s_gf = reinterpret_cast<uint32_t *>(s_all + kTB + kSets * 4096);
  uint32_t *const s_tree = s_t + kTree;  // lane-tree shifts
  uint32_t *const s_cvs = s_gf + K * 32;  // CV: input j's weight shift (x^(8 w_j)), 7 tables of 32
  const CodeArgs &a = e.code;
  const CrcArgs &cr = e.crc;
  for (int t = threadIdx.x; t < K * 32; t += blockDim.x) {
    const int j = t >> 5, h = (t >> 4) & 1, n = t & 15;
    uint32_t dw = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) dw |= gf_mul_byte(a.coef[r * K + j], static_cast<uint32_t>(n) << (4 * h)) << (8 * r);
    s_gf[t] = dw;
  }
  if constexpr (XO) {
    load_tables(s_t, cr.g26[g26_slot(1, D)] + g26_gshift(D), 224 + 1344);
    load_tables(s_t + kXoOff, cr.xo, kXoWords);
    if constexpr (H < K) load_tables(s_t + kSh1, cr.g26[g26_slot(1, 1)] + g26_gshift(1), 224);
    if constexpr (CV) load_tables(s_cvs, cr.cv + kCvShift, K * 224);
  } else {
    load_tables(s_t, cr.g26[g26_slot(1, D)], g26_words(D));
  }
  __syncthreads();
  for (int q = threadIdx.x; q < kSets * 512; q += blockDim.x) {
    const int t = q >> 4, n = q & 15, p = t & 31, dj = t >> 5, j = dj % K, d = dj / K;
    const uint32_t off = static_cast<uint32_t>((t >> 1) * 256 + n * 16 + (t & 1) * 8);
    s_c[off >> 3] = make_uint2(s_gf[j * 32 + (p & 1) * 16 + n],
                               CV ? cr.cv[(j * 32 + p) * 16 + n] : cr.nib[(d * 32 + p) * 16 + n]);
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwin = cr.nwin;
  const int64_t units = a.nstripes * nwin;
  const int32_t T = static_cast<int32_t>(cr.bpc >> 10);  // steps per window
  const uint32_t voff = static_cast<uint32_t>(lane) * 16u;
  uint32_t v4, vf0;  // index-op operands in VGPRs (VOP2/SDWA with no SGPR or literal operand issue fastest)
  asm volatile("v_mov_b32 %0, 4" : "=v"(v4));
  asm volatile("v_mov_b32 %0, 0xf0" : "=v"(vf0));
  int64_t off_max = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) off_max = a.in_off[j] > off_max ? a.in_off[j] : off_max;
  // descriptor ranges end with the last unit's window (rebase32: offset + cell length < 2^31)
  const int64_t wmax = cr.bpc < a.len ? cr.bpc : a.len;
  const uint32_t in_extent = static_cast<uint32_t>(off_max + wmax);
  int64_t out_max = 0;
#pragma unroll
  for (int r = 0; r < R; ++r) out_max = a.out_off[r] > out_max ? a.out_off[r] : out_max;
  const uint32_t out_extent = static_cast<uint32_t>(out_max + wmax);
  const int64_t bid = a.unit_map == 1 ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  WorkQueue wq{e.work, units, static_cast<int>(blockIdx.x & 7), 0};
  int64_t u = DYN == 1 ? wq.next(lane) : bid * WPB + wave;
  while (u < units) {
    // DYN 1: the next unit is claimed before this one is worked on, so the atomic's round trip overlaps the work
    const int64_t u_next = DYN == 1 ? wq.next(lane) : u + static_cast<int64_t>(gridDim.x) * WPB;
    // wave-uniform by construction; said explicitly so the descriptors below stay in SGPRs (the 64-bit division
    // runs in the VALU, and without this the buffer accesses were wrapped in waterfall loops)
    const int64_t s = uniform64(u / nwin);
    const int64_t w = uniform64(u - s * nwin);
    const uint8_t *const ib = a.in + in_off(a, s) + w * cr.bpc;
    uint8_t *const ob = a.out + out_off(a, s) + w * cr.bpc;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc_n(ib, in_extent);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc_n(ob, out_extent);
    // steps of this window: a cell's last window may be short (its whole 16-B blocks here, its last 1-15 bytes in
    // nb_tail).  It is run as whole D-step groups with Pb virtual zero blocks in front, as the per-window kernel
    // does: a zero block leaves a zero CRC register at zero and has zero GF products, and the blocks after it keep
    // their distance to the window end.  Virtual blocks and the look-ahead past the window are addressed outside
    // both descriptors: their loads return zeros without a memory access and their stores are dropped.
    int32_t Tu = T, Pb = 0;
    if (w == nwin - 1) {
      const int32_t mb = static_cast<int32_t>((a.len - w * cr.bpc) >> 4);
      Tu = (mb + 64 * D - 1) / (64 * D) * D;
      Pb = Tu * 64 - mb;
    }
    const int32_t Gu = Tu / D;
    const int32_t vbase = static_cast<int32_t>(voff) - Pb * 16;  // lane's byte offset at step 0 (< 0: virtual)
    auto vstep = [&](int32_t t) {
      const int32_t o = vbase + t * 1024;
      return t < Tu && o >= 0 ? static_cast<uint32_t>(o) : 0x80000000u;
    };
    auto load = [&](uint32_t vo, int j) {
      if constexpr (WIDE) {
        const auto d = __builtin_amdgcn_raw_buffer_load_b128(make_rsrc_n(ib + a.in_off[j], static_cast<uint32_t>(wmax)),
                                                             vo, 0, 2);
        return make_uint4(d[0], d[1], d[2], d[3]);
      } else {
        const auto d = __builtin_amdgcn_raw_buffer_load_b128(rin, vo, static_cast<int>(a.in_off[j]), 2);
        return make_uint4(d[0], d[1], d[2], d[3]);
      }
    };
    uint32_t S[K + R];
#pragma unroll
    for (int q = 0; q < K + R; ++q) S[q] = 0;
    uint4 ring[NB];
#pragma unroll
    for (int i = 0; i + 1 < NB; ++i) ring[i] = load(vstep(i / K), i % K);
    for (int32_t g = 0; g < Gu; ++g) {
#pragma unroll
      for (int rr = 0; rr < D; ++rr) {
        const int32_t t = g * D + rr;
        const int d = D - 1 - rr;  // distance set of this step's blocks
        const uint32_t vcur = vstep(t), vnext = vstep(t + 1);
        uint32_t A[16];
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int ii = rr * K + j;
          const int ahead = ii + NB - 1;
          static_assert(NB - 1 <= K, "look-ahead of at most one step");
          ring[ahead % NB] = load(ahead / K == rr ? vcur : vnext, ahead % K);
          const uint4 x = ring[ii % NB];
          const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
          XorChain ch;
          if constexpr (!CV) ch.push(S[j]);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (FENCE > 0 && c > 0 && c % (FENCE > 0 ? FENCE : 1) == 0) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int i = 4 * c + q;
              const uint32_t reg = kTB + nb_region<K>(j < H ? d : 0, j, i);
              uint2 lo, hi;
              if (reg + 256 <= 65536) {
                lo = lds64(s_all, reg + nib_lo_idx(xw[c], q, v4));
                hi = lds64(s_all, reg + 8 + nib_hi_idx(xw[c], q, vf0));
              } else {
                lo = lds64(s_all, (reg - 0x8000u) + (nib_lo_idx(xw[c], q, v4) | 0x8000u));
                hi = lds64(s_all, (reg + 8 - 0x8000u) + (nib_hi_idx(xw[c], q, vf0) | 0x8000u));
              }
              A[i] = j == 0 ? (lo.x ^ hi.x) : xor3(A[i], lo.x, hi.x);
              ch.push(lo.y);
              ch.push(hi.y);
            }
          }
          if constexpr (CV) S[0] ^= ch.get();  // the lookups' tree first, the running register last
          else S[j] = ch.get();
          if (FENCE > 0) __builtin_amdgcn_sched_barrier(0);
        }
        // 4x4 byte transposes: A[4c + q] byte r -> output r, dword c, byte q
        uint32_t o[4][4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const uint32_t a0 = A[4 * c], a1 = A[4 * c + 1], a2 = A[4 * c + 2], a3 = A[4 * c + 3];
          const uint32_t l01 = __builtin_amdgcn_perm(a1, a0, 0x05010400u), l23 = __builtin_amdgcn_perm(a3, a2, 0x05010400u);
          o[0][c] = __builtin_amdgcn_perm(l23, l01, 0x05040100u);
          if constexpr (R > 1) o[1][c] = __builtin_amdgcn_perm(l23, l01, 0x07060302u);
          if constexpr (R > 2) {
            const uint32_t h01 = __builtin_amdgcn_perm(a1, a0, 0x07030602u), h23 = __builtin_amdgcn_perm(a3, a2, 0x07030602u);
            o[2][c] = __builtin_amdgcn_perm(h23, h01, 0x05040100u);
            if constexpr (R > 3) o[3][c] = __builtin_amdgcn_perm(h23, h01, 0x07060302u);
          }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint4 p = make_uint4(o[r][0], o[r][1], o[r][2], o[r][3]);
          __attribute__((ext_vector_type(4))) unsigned int dv = {p.x, p.y, p.z, p.w};
          if constexpr (WIDE) {
            __builtin_amdgcn_raw_buffer_store_b128(dv, make_rsrc_n(ob + a.out_off[r], static_cast<uint32_t>(wmax)), vcur,
                                                   0, 2);
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(dv, rout, vcur, static_cast<int>(a.out_off[r]), 2);
          }
          store_data_hold(p);
          if constexpr (XO) {
            uint4 px = p;
            px.x ^= S[K + r];
            S[K + r] = g26_block<true>(s_t + kXoOff, px);
          } else {
            S[K + r] ^= g26_block<true>(s_t + d * kG26Set, p);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (H < K) {
          if (rr + 1 < D) {
#pragma unroll
            for (int q = H; q < K; ++q) S[q] = g5_shift(s_t + kSh1, S[q]);
          }
        }
      }
      if (g + 1 < Gu) {
#pragma unroll
        for (int q = 0; q < (XO ? kInRegs : K + R); ++q)
          S[q] = g5_shift(s_t + (q < H ? kShIn : q < K ? kSh1 : g26_gshift(D)), S[q]);
      }
    }
    const bool last = w == nwin - 1;
    const uint32_t init = last ? cr.init_last : cr.init_full;
    if constexpr (XO) {  // undo the advance of every output block
#pragma unroll
      for (int r = 0; r < R; ++r) S[K + r] = g5_shift(s_t + kXoOff + kXoInv, S[K + r]);
    }
    if constexpr (CV) {
      // registers through the tree: the combined input register, then the R outputs
      uint32_t Sc[1 + R];
      Sc[0] = S[0];
#pragma unroll
      for (int r = 0; r < R; ++r) Sc[1 + r] = S[K + r];
      int q = 0;
      const uint32_t v = g5_lane_tree_rs<1 + R>(s_tree - kG5Tree, Sc, lane, q);
      if (lane < tree_np(1 + R) && q >= 1 && q < 1 + R) nb_emit_lane<K, R>(e, s, w, K + q - 1, v, init);
      if (cr.expected) nb_check_combined<K>(e, s_cvs, s, w, lane, lane < tree_np(1 + R) && q == 0, v, init);
    } else if constexpr (RS) {
      int q = 0;
      const uint32_t v = g5_lane_tree_rs<K + R>(s_tree - kG5Tree, S, lane, q);
      if constexpr (EM) {
        uint32_t vt = v;
        if constexpr (TAIL) {  // the cell's last 1-15 bytes (nb_tail)
          const int32_t tb = last ? static_cast<int32_t>((a.len - w * cr.bpc) & 15) : 0;
          if (tb != 0 && lane < tree_np(K + R) && q < K + R) {
            const uint32_t o0 = static_cast<uint32_t>((a.len - w * cr.bpc) & ~int64_t{15});
            if constexpr (WIDE) vt = nb_tail_wide<K, R>(e, ib, ob, s_gf, q, v, o0, tb);
            else vt = nb_tail<K, R>(e, rin, rout, s_gf, q, v, o0, tb);
          }
        }
        if (lane < tree_np(K + R) && q < K + R) nb_emit_lane<K, R>(e, s, w, q, vt, init);
      } else if (lane < tree_np(K + R)) {  // each unit's total once; static unit index (kernarg arrays stay SGPR-indexed)
#pragma unroll
        for (int qq = 0; qq < K + R; ++qq)
          if (q == qq) nb_emit<K, R>(e, s, w, qq, v, init);
      }
    } else {
#pragma unroll
      for (int q = 0; q < K + R; ++q) {
        const uint32_t v = g5_lane_tree(s_tree - kG5Tree, S[q], lane);
        if (lane == q) nb_emit<K, R>(e, s, w, q, v, init);
      }
    }
    u = u_next;
  }
  if constexpr (DYN == 1) wq.finish(lane, static_cast<int32_t>(gridDim.x) * WPB);
}

template <int K, int R, int D, int NB, int WPB, int WAVES, int FENCE = 2, bool RS = true, int DYN = 0, bool XO = false,
          bool EM = false, int H = K, bool TAIL = false, bool CV = false, bool WIDE = false>
hipError_t launch_nb(const EncCrcArgs &e, hipStream_t st) {
  if constexpr ((D * K) % NB != 0) {  // the ring must divide the unrolled group: fall back to one that does
    // NB = 2 with an odd group once made this launcher call itself with the same arguments (a host stack overflow,
    // SIGSEGV in the caller: DESIGN 2.3); the fallback must differ from NB and divide the group
    constexpr int kNB = (D * K) % 2 == 0 ? 2 : (D * K <= K + 1 ? D * K : 1);
    static_assert(kNB != NB && (D * K) % kNB == 0 && kNB - 1 <= K, "fallback ring must differ and divide the group");
    return launch_nb<K, R, D, kNB, WPB, WAVES, FENCE, RS, DYN, XO, EM, H, TAIL, CV, WIDE>(e, st);
  } else {
    auto kern = encode_crc_nb<K, R, D, NB, WPB, WAVES, FENCE, RS, DYN, XO, EM, H, TAIL, CV, WIDE>;
    const int64_t units = e.code.nstripes * e.crc.nwin;
    const int64_t blocks = (units + WPB - 1) / WPB;
    int64_t g = blocks;
    if constexpr (DYN != 0) {
      // persistent: one resident set of workgroups (occupancy x CUs), each building its tables once; the caller has
      // leased the WorkQueue counter slot (e.work, fused.hip work_lease)
      if (e.work == nullptr || units > (int64_t{1} << 30)) return hipErrorInvalidValue;
      static std::atomic<int> resident{0};  // per instantiation and process (one device type)
      if (resident.load(std::memory_order_relaxed) == 0) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, WPB * 64, 0) != hipSuccess)
          return hipErrorInvalidValue;
        resident.store(std::max(1, cus * std::max(1, per_cu)), std::memory_order_relaxed);
      }
      g = std::min<int64_t>(resident.load(std::memory_order_relaxed), blocks);
    }
    // non-persistent: one wave per (stripe, window) unit, no grid-stride: every workgroup builds its K*D*4 KiB of
    // tables, and the dispatcher's refill of finished workgroups balances the CUs.  Measured on MI355X against a
    // static persistent grid (profiles/r02/nb/ab_grid_*.log): C3r 56.2 % -> 63.5 %, C5dev 60.1 % -> 65.7 %.
    const int64_t cg = g_tune.crc_grid;
    if (cg > 0) g = std::min<int64_t>(cg, blocks);
    (void)hipGetLastError();  // the error returned below must be this launch's, not a stale one (fused.hip work_return)
    hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(std::max<int64_t>(1, g))), dim3(WPB * 64), 0, st, e);
    return hipGetLastError();
  }
}

// whether variant v of the nibble kernel runs on the persistent WorkQueue grid (needs a leased counter slot)
constexpr bool nb_variant_persistent(int v) { return v == 150 || v == 163 || v == 167 || v == 170 || v == 171 ||
                                                     v == 172 || v == 176 || v == 177 || v == 187 || (v >= 189 && v <= 194) ||
                                                     v == 196 || v == 231 || v == 234; }
// whether variant v checks a reconstruction's inputs through one combined register (then nb_reverify follows it)
constexpr bool nb_variant_cv(int v) { return v == 231 || v == 234; }

// variant (g_tune.crc_variant, kernels.hpp kCrcVariants): the measured alternates of the nibble-table kernel
template <int K, int R>
hipError_t launch_nb_kr(const EncCrcArgs &e, hipStream_t st, int v) {
  constexpr int kD2 = K * 2 * 4096 + g26_words(2) * 4 <= 65536 ? 2 : 1;  // D = 2 where its tables fit
  constexpr int kNB = K % 2 == 0 && K > 2 ? K / 2 : K;                    // a deeper ring dividing the group
  constexpr int kHh = K / 2;
  switch (v) {
    // round-2 defaults, non-persistent (profiles/r02/nb/): rs-10-x one-step groups with a ring of K / 2 (62), rs-6-x /
    // rs-3-x two-step groups in 12-wave workgroups (87)
    case 62: return launch_nb<K, R, 1, kNB, 8, 4>(e, st);
    case 87: return launch_nb<K, R, kD2, 2, 12, 4>(e, st);
    // round 3, free output-register shifts (XO) on the persistent WorkQueue grid: 150 = 62's geometry, 163 = two-step
    // groups in 16-wave workgroups, 167 = 163 with a ring of K / 2
    case 150: return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 1, true>(e, st);
    case 163: return launch_nb<K, R, 2, 2, 16, 4, 2, true, 1, true>(e, st);
    case 167: return launch_nb<K, R, 2, kNB, 16, 4, 2, true, 1, true>(e, st);
    // the same with the lane-parallel emit (EM; the defaults, fused.hip): 170 = 150, 171 = 167, 172 = 163, and the
    // non-persistent fallbacks 173 = 151 (62 + XO), 174 = 152 (87 + XO)
    case 170: return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 1, true, true>(e, st);
    case 171: return launch_nb<K, R, 2, kNB, 16, 4, 2, true, 1, true, true>(e, st);
    case 172: return launch_nb<K, R, 2, 2, 16, 4, 2, true, 1, true, true>(e, st);
    case 173: return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 0, true, true>(e, st);
    case 174: return launch_nb<K, R, kD2, 2, 12, 4, 2, true, 0, true, true>(e, st);
    // two-step groups with the second distance set for the first K / 2 inputs only (H), the rest shifted every step:
    // 8-wave (176) and 16-wave (177, the rs-10-x default) workgroups
    case 176: return launch_nb<K, R, 2, kNB, 8, 4, 2, true, 1, true, true, kHh>(e, st);
    case 177: return launch_nb<K, R, 2, kNB, 16, 4, 2, true, 1, true, true, kHh>(e, st);
    // round 4, occupancy: the defaults are held to one 16-wave workgroup per CU by VGPRs (177: 119 -> 4 waves per SIMD;
    // 171: 73 -> 6, but a second 16-wave workgroup needs 8).  187: 177 with lookups fenced per dword (16 fewer results
    // live); 189: 171 in 12-wave workgroups (two per CU: 24 waves); 190: 171 held to 8 waves per SIMD (two 16-wave
    // workgroups per CU).  177 held to 5 waves per SIMD in 10-wave workgroups spills (22 VGPRs to scratch) and ran 21 %
    // slower (profiles/r04/a/ab_c3r.log, variants 186 / 188, since removed)
    case 187: return launch_nb<K, R, 2, kNB, 16, 4, 1, true, 1, true, true, kHh>(e, st);
    case 189: return launch_nb<K, R, 2, kNB, 12, 4, 2, true, 1, true, true>(e, st);
    case 190: return launch_nb<K, R, 2, kNB, 16, 8, 2, true, 1, true, true>(e, st);
    // 191: 170 (one-step groups, 87 VGPRs for rs-10-4: 5 waves per SIMD, but 8-wave workgroups fill only 16 wave slots
    // per CU) in 10-wave workgroups: two per CU, 20 waves; 192: 172 (ring of 2) in 12-wave workgroups
    case 191: return launch_nb<K, R, 1, kNB, 10, 5, 2, true, 1, true, true>(e, st);
    case 192: return launch_nb<K, R, 2, 2, 12, 4, 2, true, 1, true, true>(e, st);
    // 193: 171 in 14-wave workgroups held to 7 waves per SIMD (two per CU: 28 waves); 194: 171 with half the inputs'
    // second distance set (36 + 12 KiB of tables: three 9-wave workgroups per CU, 27 waves); 196: 177 with a ring of 2
    // and dword fences (fewer VGPRs) in 16-wave workgroups
    case 193: return launch_nb<K, R, 2, kNB, 14, 7, 2, true, 1, true, true>(e, st);
    case 194: return launch_nb<K, R, 2, kNB, 9, 7, 2, true, 1, true, true, kHh>(e, st);
    case 196: return launch_nb<K, R, 2, 2, 16, 4, 1, true, 1, true, true, kHh>(e, st);
    // round 5, small batches: 173 (one-step groups, one wave per (stripe, window) unit, no WorkQueue) in workgroups of
    // 1 / 2 / 4 waves, so a batch of a few hundred units spreads over as many CUs instead of 16-wave workgroups on a
    // handful (the LDS pipe of each CU serves all its waves)
    case 220: return launch_nb<K, R, 1, kNB, 1, 4, 2, true, 0, true, true>(e, st);
    case 221: return launch_nb<K, R, 1, kNB, 2, 4, 2, true, 0, true, true>(e, st);
    case 222: return launch_nb<K, R, 1, kNB, 4, 4, 2, true, 0, true, true>(e, st);
    // round 5, combined input verification (CV) for reconstructions that check stored CRCs: 231 = 170's one-step groups
    // in 16-wave workgroups (the default for rs-6-x / rs-10-x, fused.hip), 234 = 231 with a ring of 2 loads; for an
    // encode or without stored CRCs either runs 170 itself.  (230 = 8-wave workgroups, 232 = two 10-wave and 233 = two
    // 12-wave workgroups per CU measured 2-23 % slower than 231, profiles/r05/cv/, and were taken out.)
    case 231:
      if (!e.verify || !e.crc.expected) return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 1, true, true>(e, st);
      return launch_nb<K, R, 1, kNB, 16, 4, 2, true, 1, true, true, K, false, true>(e, st);
    case 234:
      if (!e.verify || !e.crc.expected) return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 1, true, true>(e, st);
      return launch_nb<K, R, 1, 2, 16, 4, 2, true, 1, true, true, K, false, true>(e, st);
    default: break;
  }
  return hipErrorInvalidValue;
}

// cells of any length at any byte offsets (encode_crc_nb_bytes_supported): the defaults and their alternates with the
// lane-parallel emit, instantiated a second time with the nb_tail epilogue (TAIL), so the kernels of 16-B cells keep
// their code (the epilogue in every instantiation cost C3r 1.3-2 %, profiles/r05/bytes/)
constexpr bool nb_variant_tail(int v) {
  return v == 170 || v == 171 || v == 172 || v == 173 || v == 174 || v == 177 || (v >= 220 && v <= 222);
}

template <int K, int R>
hipError_t launch_nb_tail_kr(const EncCrcArgs &e, hipStream_t st, int v) {
  constexpr int kD2 = K * 2 * 4096 + g26_words(2) * 4 <= 65536 ? 2 : 1;
  constexpr int kNB = K % 2 == 0 && K > 2 ? K / 2 : K;
  constexpr int kHh = K / 2;
  switch (v) {
    case 170: return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 1, true, true, K, true>(e, st);
    case 171: return launch_nb<K, R, 2, kNB, 16, 4, 2, true, 1, true, true, K, true>(e, st);
    case 172: return launch_nb<K, R, 2, 2, 16, 4, 2, true, 1, true, true, K, true>(e, st);
    case 173: return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 0, true, true, K, true>(e, st);
    case 174: return launch_nb<K, R, kD2, 2, 12, 4, 2, true, 0, true, true, K, true>(e, st);
    case 177: return launch_nb<K, R, 2, kNB, 16, 4, 2, true, 1, true, true, kHh, true>(e, st);
    case 220: return launch_nb<K, R, 1, kNB, 1, 4, 2, true, 0, true, true, K, true>(e, st);
    case 221: return launch_nb<K, R, 1, kNB, 2, 4, 2, true, 0, true, true, K, true>(e, st);
    case 222: return launch_nb<K, R, 1, kNB, 4, 4, 2, true, 0, true, true, K, true>(e, st);
    default: break;
  }
  return hipErrorInvalidValue;
}
// units 2 GiB or more apart (round 6): the one-step geometry of 173 with one descriptor per unit, for 16-B-multiple
// cells and (TAIL) any length; a rare layout (a caller's cells scattered over a large HBM pool), so one form only
template <int K, int R>
hipError_t launch_nb_wide_kr(const EncCrcArgs &e, hipStream_t st, bool tail) {
  constexpr int kNB = K % 2 == 0 && K > 2 ? K / 2 : K;
  if (tail) return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 0, true, true, K, true, false, true>(e, st);
  return launch_nb<K, R, 1, kNB, 8, 4, 2, true, 0, true, true, K, false, false, true>(e, st);
}
}  // namespace
}  // namespace ozec
