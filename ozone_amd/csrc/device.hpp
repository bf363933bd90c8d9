// Device helpers shared by the gfx950 kernel translation units (kernels.hip, fused.hip): GF(2^8) permute
// tables, CRC G5/G26 table lookups, buffer descriptors, XCD-aware block order, and the host-side argument
// helpers of the launchers.  Internal to libozec (everything sits in an anonymous namespace per TU).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "kernels.hpp"

namespace ozec {
namespace {

constexpr int kBlock = 256;
#ifndef OZEC_GF_WAVES
#define OZEC_GF_WAVES 4  // >= 4 waves per SIMD: <= 128 VGPRs for the coding kernels
#endif
constexpr int kMaxGrid = 256 * 8;  // 8 blocks of 256 threads per CU, grid-stride beyond

// ------------------------------------------------------------------------------------------------
// GF(2^8) helpers

__device__ __forceinline__ uint32_t gf_mul_byte(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    r ^= (b & 1u) ? a : 0u;
    b >>= 1;
    a = (a << 1) ^ ((a & 0x80u) ? 0x11du : 0u);
  }
  return r & 0xffu;
}

struct PermTab {
  uint32_t lo0, lo1, mid0, mid1, top;
};

__device__ __forceinline__ uint32_t pack4(uint32_t c, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
  return gf_mul_byte(c, m0) | (gf_mul_byte(c, m1) << 8) | (gf_mul_byte(c, m2) << 16) | (gf_mul_byte(c, m3) << 24);
}

__device__ __forceinline__ PermTab make_tab(uint32_t c) {
  PermTab t;
  t.lo0 = pack4(c, 0, 1, 2, 3);
  t.lo1 = pack4(c, 4, 5, 6, 7);
  t.mid0 = pack4(c, 0, 8, 16, 24);
  t.mid1 = pack4(c, 32, 40, 48, 56);
  t.top = pack4(c, 0, 64, 128, 192);
  return t;
}

struct Sel {
  uint32_t s0, s1, s2;
};

__device__ __forceinline__ Sel make_sel(uint32_t w) {
  Sel s;
  s.s0 = w & 0x07070707u;
  s.s1 = (w >> 3) & 0x07070707u;
  s.s2 = (w >> 6) & 0x03030303u;
  return s;
}

// c * w for the 4 bytes of w. v_perm_b32(S0, S1, sel): selector byte 0-3 picks a byte of S1, 4-7 of S0.
__device__ __forceinline__ uint32_t gf_mul4(const PermTab &t, const Sel &s) {
  return __builtin_amdgcn_perm(t.lo1, t.lo0, s.s0) ^ __builtin_amdgcn_perm(t.mid1, t.mid0, s.s1) ^
         __builtin_amdgcn_perm(t.top, t.top, s.s2);
}

// ---- register-resident tables: lo1/mid1/top are wave-uniform and live in SGPRs, lo0/mid0 in VGPRs, so
// each v_perm_b32 reads exactly one SGPR (the gfx9 constant-bus limit) and a coefficient costs 2 VGPRs.
__device__ __forceinline__ uint32_t perm_sv(uint32_t hi_s, uint32_t lo_v, uint32_t sel) {
  uint32_t d;
  asm("v_perm_b32 %0, %1, %2, %3" : "=v"(d) : "s"(hi_s), "v"(lo_v), "v"(sel));
  return d;
}
__device__ __forceinline__ uint32_t perm_top_s(uint32_t top_s, uint32_t sel) {
  uint32_t d;  // selectors 0..3 only read S1 (= the SGPR table); S0 is a don't-care VGPR
  asm("v_perm_b32 %0, %1, %2, %1" : "=v"(d) : "v"(sel), "s"(top_s));
  return d;
}
__device__ __forceinline__ uint32_t perm_vv(uint32_t hi, uint32_t lo, uint32_t sel) {
  uint32_t d;
  asm("v_perm_b32 %0, %1, %2, %3" : "=v"(d) : "v"(hi), "v"(lo), "v"(sel));
  return d;
}
// A VALU write to the data VGPRs of a 16-B VMEM store issued just before it can corrupt the stored bytes on
// MI355X: seen as a few wrong bytes per 16-lane group in the fused XOR kernels under load (scripts/diag_c4.py),
// while hipcc inserts no wait states for this case.  Call right after the store(s): the data registers stay
// allocated until two wait states after the store, so the next writer of those VGPRs cannot come sooner.
__device__ __forceinline__ void store_data_hold(const uint4 &v) {
#ifndef OZEC_NO_STORE_HOLD  // defined only to show tests/isa_scan.py the unguarded ISA
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 1" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
#endif
}

// Byte offset of stripe s: s * stripe_stride, or in the block-group layout (grp_stripes > 0, one block file per
// unit) group s / grp_stripes at grp_stride, stripe s % grp_stripes within it.  s is wave-uniform (SALU).
__device__ __forceinline__ int64_t grouped_off(int64_t s, int64_t stride, int64_t gs, int64_t gstride) {
  if (gs <= 0) return s * stride;
  const uint32_t g = static_cast<uint32_t>(s) / static_cast<uint32_t>(gs);
  return static_cast<int64_t>(g) * gstride + (s - static_cast<int64_t>(g) * gs) * stride;
}
__device__ __forceinline__ int64_t in_off(const CodeArgs &a, int64_t s) {
  return grouped_off(s, a.in_stripe_stride, a.grp_stripes, a.in_grp_stride);
}
__device__ __forceinline__ int64_t out_off(const CodeArgs &a, int64_t s) {
  return grouped_off(s, a.out_stripe_stride, a.grp_stripes, a.out_grp_stride);
}

// gfx950 3-input bitwise op; truth table 0x96 = a ^ b ^ c
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// XOR of a sequence of values with three-input XORs: (n-1)/2 ops for n values (every branch folds away
// once the pushing loops are unrolled)
struct XorChain {
  uint32_t acc = 0, spare = 0;
  int n = 0;
  bool has_spare = false;
  __device__ __forceinline__ void push(uint32_t v) {
    if (n++ == 0) {
      acc = v;
    } else if (!has_spare) {
      spare = v;
      has_spare = true;
    } else {
      acc = xor3(acc, spare, v);
      has_spare = false;
    }
  }
  __device__ __forceinline__ uint32_t get() const { return has_spare ? acc ^ spare : acc; }
};

struct RegTab {
  uint32_t lo0, mid0;      // VGPR
  uint32_t lo1, mid1, top; // SGPR (wave-uniform)
};

__device__ __forceinline__ uint32_t gf_mul4_reg(const RegTab &t, const Sel &s) {
  return xor3(perm_sv(t.lo1, t.lo0, s.s0), perm_sv(t.mid1, t.mid0, s.s1), perm_top_s(t.top, s.s2));
}
__device__ __forceinline__ uint32_t gf_mul4_lds(const PermTab &t, const Sel &s) {
  return xor3(perm_vv(t.lo1, t.lo0, s.s0), perm_vv(t.mid1, t.mid0, s.s1), perm_vv(t.top, t.top, s.s2));
}

__device__ __forceinline__ void build_tabs(PermTab *s_tab, const CodeArgs &a, int rows, int k) {
  for (int t = threadIdx.x; t < rows * k; t += blockDim.x) s_tab[t] = make_tab(a.coef[t]);
}

// ------------------------------------------------------------------------------------------------
// Coding kernels

// Host-built permute tables for the templated kernels, passed by value in the kernarg segment so they are
// s_load'ed straight into SGPRs (no LDS round trip, no readfirstlane).
template <int N>
struct TabArgs {
  uint32_t w[N][5];  // per coefficient: lo0, lo1, mid0, mid1, top
};

// XCD-aware block order: the dispatcher deals blocks round-robin over the 8 XCDs (b and b+8 share one), so map
// block b to work item (b % 8) * (n / 8) + b / 8: every XCD streams one contiguous eighth of the batch instead of
// all eight interleaving at 4 KiB granularity.  Bijective on [0, n) (the n % 8 tail keeps its own index).
// Measured on C2 (scripts/tune_map.py): 75.6 % -> 78.7 % of the HBM roofline.  Placement is a speed hint only.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t n) {
  const uint32_t q = n >> 3;
  return b < (q << 3) ? (b & 7) * q + (b >> 3) : b;
}

// byte range of a stripe-side descriptor over n units at offsets off[0..n), each reached for `span` bytes: an access
// past it returns zeros or is dropped instead of reaching other memory.  Every kernel bounds its indices itself; this
// is the second fence (rebase32 keeps offset + span < 2^31).
template <int N>
__device__ __forceinline__ uint32_t unit_extent(const int64_t *off, int64_t span) {
  int64_t mx = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) mx = off[i] > mx ? off[i] : mx;
  return static_cast<uint32_t>(mx + span);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base) {
  // raw buffer (stride 0), full 4 GiB range; bounds are checked explicitly by the kernels
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, 0xffffffff, 0x00020000);
}
// raw buffer of `nbytes` records: a load whose offset (voffset + soffset + instruction offset, all three are range
// checked on gfx950) is past the end returns zeros without touching memory
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_n(const void *base, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, static_cast<int>(nbytes), 0x00020000);
}

// ------------------------------------------------------------------------------------------------
// CRC helpers.  Every 32-bit-output linear map (block -> raw CRC, register shift by n bytes) is evaluated
// as an XOR of lookups in 32-entry tables indexed by 5-bit groups of its input.  A 32-entry table aligned
// to 128 B covers each of the 32 LDS banks exactly once, so a ds_read_b32 of 64 random lanes is
// conflict-free (2 LDS cycles) -- with 256-entry byte tables random indices cost ~3.5x that in bank
// conflicts, which is what bounded the first version.  Layout: kernels.hpp (kG5*).

__device__ __forceinline__ uint32_t g5_idx(uint32_t v) { return v & 31u; }

// raw CRC of one 16-B block (26 groups of 5 bits; group 25 holds bits 125..127)
__device__ __forceinline__ uint32_t g5_block(const uint32_t *T, const uint4 b) {
  const uint32_t w[4] = {b.x, b.y, b.z, b.w};
  uint32_t t[26];
#pragma unroll
  for (int g = 0; g < 26; ++g) {
    const int o = 5 * g, d = o >> 5, sh = o & 31;
    const uint32_t v = (sh <= 27 || d == 3) ? (w[d] >> sh) : __builtin_amdgcn_alignbit(w[d + 1], w[d], sh);
    t[g] = T[kG5Blk + g * 32 + g5_idx(v)];
  }
  uint32_t r = xor3(t[0], t[1], t[2]);
#pragma unroll
  for (int g = 3; g + 1 < 26; g += 2) r = xor3(r, t[g], t[g + 1]);
  return r ^ t[25];
}

// register shift by the byte distance the 7 x 32 table block at T encodes
__device__ __forceinline__ uint32_t g5_shift(const uint32_t *T, uint32_t s) {
  uint32_t t[7];
#pragma unroll
  for (int g = 0; g < 7; ++g) t[g] = T[g * 32 + g5_idx(s >> (5 * g))];
  return xor3(xor3(t[0], t[1], t[2]), xor3(t[3], t[4], t[5]), t[6]);
}

// merge the 64 lane registers of a wave (lane l's chunk precedes lane l+1's) -> every lane gets the total
__device__ __forceinline__ uint32_t g5_lane_tree(const uint32_t *T, uint32_t v, int lane) {
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), 1 << m, 64));
    const bool upper = (lane >> m) & 1;
    const uint32_t lower = upper ? other : v;
    const uint32_t hi = upper ? v : other;
    v = g5_shift(T + kG5Tree + m * 224, lower) ^ hi;
  }
  return v;
}

// a wave-uniform 64-bit value, said explicitly (kept in SGPRs)
__device__ __forceinline__ int64_t uniform64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32));
  return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}

// Dynamic work distribution of the persistent fused kernels (the nibble kernel and the XOR codec's per-window kernel
// with DYN = 1).  The (stripe, window) units are cut into 8 contiguous ranges, one per XCD (the dispatcher deals workgroups round-robin over the 8 XCDs, so workgroup b starts
// on range b % 8: each XCD streams one contiguous eighth of the batch), and a wave takes the next unit of its range
// with one atomicAdd (a vector-memory atomic issued by lane 0 and broadcast with readfirstlane), one unit ahead of
// the one it works on; a wave whose range is used up moves on to the next range, so every unit is taken exactly once
// whatever the grid size or placement.  The counters are a slot leased for the launch (fused.hip work_lease):
// the last wave of a launch to finish puts the slot back to zero, and the slot is reused only after an event recorded
// behind the launch has completed.
struct WorkQueue {
  int32_t *ctr;
  int64_t units;
  int q0, qi;
  __device__ __forceinline__ int64_t next(int lane) {
    while (qi < 8) {
      const int q = (q0 + qi) & 7;
      const int64_t lo = units * q / 8, hi = units * (q + 1) / 8;
      int32_t t = 0;
      if (lane == 0) t = atomicAdd(ctr + q * kWqStride, 1);
      t = __builtin_amdgcn_readfirstlane(t);
      if (lo + t < hi) return lo + t;
      ++qi;
    }
    return units;
  }
  // every wave calls this once after its last unit: the last of `waves` resets the slot
  __device__ __forceinline__ void finish(int lane, int32_t waves) {
    if (lane == 0 && atomicAdd(ctr + kWqDone, 1) == waves - 1) {
      for (int q = 0; q < 8; ++q) atomicExch(ctr + q * kWqStride, 0);
      atomicExch(ctr + kWqDone, 0);
    }
  }
};

__device__ __forceinline__ void load_tables(uint32_t *s_t, const uint32_t *g, int words) {
  const uint4 *src = reinterpret_cast<const uint4 *>(g);
  uint4 *dst = reinterpret_cast<uint4 *>(s_t);
  for (int i = threadIdx.x; i < words / 4; i += blockDim.x) dst[i] = src[i];
}

__device__ __forceinline__ uint32_t crc_finish(uint32_t raw, uint32_t init, int raw_out, int big_endian) {
  uint32_t v = raw_out ? raw : ~(raw ^ init);
  return big_endian ? __builtin_bswap32(v) : v;
}

// store the window CRC, or (verify mode) compare it with the expected value and record the first failure
__device__ __forceinline__ void crc_emit(const CrcArgs &a, int64_t cell, int64_t w, uint32_t raw, bool last) {
  const uint32_t init = last ? a.init_last : a.init_full;
  const int64_t idx = cell * a.out_cell_stride + w;
  if (a.expected) {
    const uint32_t v = crc_finish(raw, init, 0, 0);
    const uint32_t e = a.expected_be ? __builtin_bswap32(a.expected[idx]) : a.expected[idx];
    if (v != e) atomicMin(a.mismatch + cell, a.mismatch_base + static_cast<int32_t>(w));
  } else {
    a.out[idx] = crc_finish(raw, init, a.raw, a.big_endian);
  }
}

// ---- G26: step-grouped CRC with SDWA-friendly bit groups (table layout: kernels.hpp kG26*) ----------
// A table lookup needs its 5-bit index times 4 (the byte offset of a dword entry).  Bits 8b+2..8b+6 of a
// dword come out as exactly that with ONE op, `(w >> 8b) & 0x7c` (v_and_b32 with an SDWA byte select), so
// 16 of the 26 groups of a 16-B block are read straight from the data dwords.  The 48 bits left over (bits
// 8b+7..8b+9 of every byte boundary) are gathered by two rotate-and-merge registers (3 ops, 4 groups each)
// and one register of 4-bit groups (5 ops, 2 groups): 36 VALU for 26 lookups, against 52 for 5-bit groups
// cut at fixed offsets (shift + mask each).  Table g reads block bits crc_host.cpp g26_bit(g, *).

__device__ __forceinline__ uint32_t lds_at(const uint32_t *T, uint32_t byte_off) {
  return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(T) + byte_off);
}
__device__ __forceinline__ uint32_t rotr32(uint32_t w, int k) { return __builtin_amdgcn_alignbit(w, w, k); }
// (a & m) | (b & ~m) in one v_bitop3_b32 (truth table 0xca) with the mask in a VGPR: on gfx950 it issues at
// the rate of a plain v_and_b32, while v_bfi_b32 (and any VALU op with an SGPR or literal operand) takes
// ~1.7x as long per wave-instruction (scripts/valu_rate.hip, profiles/r01/session4/valu_rate.log)
__device__ __forceinline__ uint32_t bsel(uint32_t a, uint32_t b, uint32_t m) {
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xca" : "=v"(d) : "v"(m), "v"(a), "v"(b));
  return d;
}
// ((w >> 8q) & mask) in one op: v_and_b32 with an SDWA byte select (q = 0: plain AND; the compiler finds the
// WORD_1 / BYTE_3 forms itself but not BYTE_1)
template <int Q>
__device__ __forceinline__ uint32_t byte_and(uint32_t w, uint32_t mask) {
  if constexpr (Q == 1) {
    uint32_t d;
    asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
        : "=v"(d) : "v"(w), "s"(mask));
    return d;
  } else {
    return (w >> (8 * Q)) & mask;
  }
}

// as byte_and with the mask in a VGPR for every byte position: no SGPR or literal operand, which puts the AND in
// the fast VALU issue class (a v_perm or an SGPR / literal-operand op costs ~1.6x a plain VOP2 op per step,
// scripts/gpu_valu_pad.sh)
template <int Q>
__device__ __forceinline__ uint32_t byte_and_v(uint32_t w, uint32_t vmask) {
  uint32_t d;
  if constexpr (Q == 0) {
    asm("v_and_b32 %0, %1, %2" : "=v"(d) : "v"(vmask), "v"(w));
  } else if constexpr (Q == 1) {
    asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD"
        : "=v"(d) : "v"(w), "v"(vmask));
  } else if constexpr (Q == 2) {
    asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2 src1_sel:DWORD"
        : "=v"(d) : "v"(w), "v"(vmask));
  } else {
    asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3 src1_sel:DWORD"
        : "=v"(d) : "v"(w), "v"(vmask));
  }
  return d;
}

// Lane tree for U registers at once, as reduce-scatter: at level m the lanes whose bit m is set keep the upper
// half of their register list and the others the lower half, and each kept register is merged with the partner's
// copy of it (one exchange + one shift per kept register).  After log2(NP) levels (NP = U rounded up to a power of
// two) every lane holds one register, then the remaining levels merge it as g5_lane_tree does.  Shifts per lane:
// NP - 1 + (6 - log2 NP) instead of 6 U -- 17 instead of 84 for the 14 registers of rs-10-4.  Returns the merged
// register of unit `unit` = sum over m < log2 NP of bit m of the lane times NP >> (m + 1) (equal in all lanes that
// agree on those bits; unit >= U is padding).
constexpr int tree_np(int U) { return U <= 1 ? 1 : U <= 2 ? 2 : U <= 4 ? 4 : U <= 8 ? 8 : U <= 16 ? 16 : 32; }
template <int U>
__device__ __forceinline__ uint32_t g5_lane_tree_rs(const uint32_t *T, const uint32_t (&S)[U], int lane, int &unit) {
  static_assert(U <= 32, "at most 32 registers");
  constexpr int NP = tree_np(U);
  constexpr int L = NP == 1 ? 0 : NP == 2 ? 1 : NP == 4 ? 2 : NP == 8 ? 3 : NP == 16 ? 4 : 5;
  uint32_t r[NP];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < NP; ++i) r[i] = i < U ? S[i] : 0u;
  unit = 0;
#pragma unroll
  for (int m = 0; m < L; ++m) {
    const int h = (NP >> m) >> 1;
    const bool upper = (lane >> m) & 1;
    const uint32_t um = upper ? 0xffffffffu : 0u;  // selects below through a mask register (bitop3), so that the
                                                  // register list is never turned into a dynamically indexed array
    unit += upper ? h : 0;
#pragma unroll
    for (int i = 0; i < h; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t send = bsel(r[i], r[h + i], um);  // the half the partner keeps
      const uint32_t keep = bsel(r[h + i], r[i], um);
      const uint32_t recv = static_cast<uint32_t>(__shfl_xor(static_cast<int>(send), 1 << m, 64));
      r[i] = g5_shift(T + kG5Tree + m * 224, bsel(recv, keep, um)) ^ bsel(keep, recv, um);
    }
  }
  uint32_t v = r[0];
#pragma unroll
  for (int m = L; m < 6; ++m) {
    const uint32_t other = static_cast<uint32_t>(__shfl_xor(static_cast<int>(v), 1 << m, 64));
    const bool upper = (lane >> m) & 1;
    v = g5_shift(T + kG5Tree + m * 224, upper ? other : v) ^ (upper ? v : other);
  }
  return v;
}

// XOR of the 26 lookups of block b in the table set at T (26 x 32 words).  VMASK: byte_and_v with vm = 0x7c in
// a VGPR instead of the SGPR / literal mask.
template <bool HALVES = false, bool VMASK = false>
__device__ __forceinline__ uint32_t g26_block(const uint32_t *T, const uint4 b, uint32_t vm = 0x7cu) {
  const uint32_t w[4] = {b.x, b.y, b.z, b.w};
  uint32_t t[26];
  auto four = [&](uint32_t v, int g0) {
    if constexpr (VMASK) {
      t[g0] = lds_at(T, g0 * 128 + byte_and_v<0>(v, vm));
      t[g0 + 1] = lds_at(T, (g0 + 1) * 128 + byte_and_v<1>(v, vm));
      t[g0 + 2] = lds_at(T, (g0 + 2) * 128 + byte_and_v<2>(v, vm));
      t[g0 + 3] = lds_at(T, (g0 + 3) * 128 + byte_and_v<3>(v, vm));
    } else {
      t[g0] = lds_at(T, g0 * 128 + byte_and<0>(v, 0x7cu));
      t[g0 + 1] = lds_at(T, (g0 + 1) * 128 + byte_and<1>(v, 0x7cu));
      t[g0 + 2] = lds_at(T, (g0 + 2) * 128 + byte_and<2>(v, 0x7cu));
      t[g0 + 3] = lds_at(T, (g0 + 3) * 128 + byte_and<3>(v, 0x7cu));
    }
  };
  if constexpr (HALVES) {
    // two halves of 14 and 12 lookups with a scheduling fence between them: at most 14 lookup results are live
    four(w[0], 0);
    four(w[1], 4);
    four(bsel(rotr32(w[0], 5), rotr32(w[1], 2), 0x1c1c1c1cu), 16);
    uint32_t e = bsel(rotr32(w[1], 7), rotr32(w[3], 6), 0x04040404u) & 0x0c0c0c0cu;
    e |= e << 10;
    t[24] = lds_at(T, 24 * 128 + ((e >> 8) & 0x3cu));
    t[25] = lds_at(T, 25 * 128 + ((e >> 24) & 0x3cu));
    uint32_t r = xor3(t[0], t[1], t[2]);
    r = xor3(r, t[3], t[4]);
    r = xor3(r, t[5], t[6]);
    r = xor3(r, t[7], t[16]);
    r = xor3(r, t[17], t[18]);
    r = xor3(r, t[19], t[24]);
    r ^= t[25];
    __builtin_amdgcn_sched_barrier(0);
    four(w[2], 8);
    four(w[3], 12);
    four(bsel(rotr32(w[2], 5), rotr32(w[3], 2), 0x1c1c1c1cu), 20);
    r = xor3(r, t[8], t[9]);
#pragma unroll
    for (int g = 10; g < 16; g += 2) r = xor3(r, t[g], t[g + 1]);
    r = xor3(r, t[20], t[21]);
    return xor3(r, t[22], t[23]);
  }
#pragma unroll
  for (int d = 0; d < 4; ++d) four(w[d], 4 * d);
#pragma unroll
  for (int h = 0; h < 2; ++h) four(bsel(rotr32(w[2 * h], 5), rotr32(w[2 * h + 1], 2), 0x1c1c1c1cu), 16 + 4 * h);
  uint32_t e = bsel(rotr32(w[1], 7), rotr32(w[3], 6), 0x04040404u) & 0x0c0c0c0cu;
  e |= e << 10;
  t[24] = lds_at(T, 24 * 128 + ((e >> 8) & 0x3cu));
  t[25] = lds_at(T, 25 * 128 + ((e >> 24) & 0x3cu));
  uint32_t r = xor3(t[0], t[1], t[2]);
#pragma unroll
  for (int g = 3; g + 1 < 26; g += 2) r = xor3(r, t[g], t[g + 1]);
  return r ^ t[25];
}

// ------------------------------------------------------------------------------------------------
// launch helpers

inline unsigned grid_for(int64_t work_items, int per_block) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > kMaxGrid) g = kMaxGrid;
  return static_cast<unsigned>(g);
}

inline bool aligned16(int64_t v) { return (v & 15) == 0; }

inline bool vec_ok(const CodeArgs &a) {
  if (!aligned16(reinterpret_cast<intptr_t>(a.in)) || !aligned16(reinterpret_cast<intptr_t>(a.out))) return false;
  if (a.nstripes > 1 && (!aligned16(a.in_stripe_stride) || !aligned16(a.out_stripe_stride))) return false;
  if (a.grp_stripes > 0 && (!aligned16(a.in_grp_stride) || !aligned16(a.out_grp_stride))) return false;
  for (int j = 0; j < a.k; ++j)
    if (!aligned16(a.in_off[j])) return false;
  for (int r = 0; r < a.rows; ++r)
    if (!aligned16(a.out_off[r])) return false;
  return true;
}

inline uint32_t gf_mul_host(uint32_t a, uint32_t b) {
  uint32_t r = 0;
  for (int i = 0; i < 8; ++i) {
    if (b & 1) r ^= a;
    b >>= 1;
    a = (a << 1) ^ ((a & 0x80) ? 0x11d : 0);
  }
  return r & 0xff;
}

inline uint32_t pack4_host(uint32_t c, uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3) {
  return gf_mul_host(c, m0) | (gf_mul_host(c, m1) << 8) | (gf_mul_host(c, m2) << 16) | (gf_mul_host(c, m3) << 24);
}

template <int N>
TabArgs<N> host_tabs(const CodeArgs &a) {
  TabArgs<N> t;
  for (int i = 0; i < N; ++i) {
    const uint32_t c = a.coef[i];
    t.w[i][0] = pack4_host(c, 0, 1, 2, 3);
    t.w[i][1] = pack4_host(c, 4, 5, 6, 7);
    t.w[i][2] = pack4_host(c, 0, 8, 16, 24);
    t.w[i][3] = pack4_host(c, 32, 40, 48, 56);
    t.w[i][4] = pack4_host(c, 0, 64, 128, 192);
  }
  return t;
}

// Fold the smallest unit offset into the base pointers so every unit offset fits the 32-bit buffer soffset.
inline bool rebase32(CodeArgs &a) {
  const int64_t lim = (int64_t{1} << 31) - a.len - 16;
  int64_t mn = a.in_off[0], mx = a.in_off[0];
  for (int j = 1; j < a.k; ++j) {
    mn = a.in_off[j] < mn ? a.in_off[j] : mn;
    mx = a.in_off[j] > mx ? a.in_off[j] : mx;
  }
  if (mx - mn > lim) return false;
  a.in = reinterpret_cast<const uint8_t *>(reinterpret_cast<uintptr_t>(a.in) + mn);
  for (int j = 0; j < a.k; ++j) a.in_off[j] -= mn;
  mn = mx = a.out_off[0];
  for (int r = 1; r < a.rows; ++r) {
    mn = a.out_off[r] < mn ? a.out_off[r] : mn;
    mx = a.out_off[r] > mx ? a.out_off[r] : mx;
  }
  if (mx - mn > lim) return false;
  a.out = reinterpret_cast<uint8_t *>(reinterpret_cast<uintptr_t>(a.out) + mn);
  for (int r = 0; r < a.rows; ++r) a.out_off[r] -= mn;
  return true;
}

}  // namespace
}  // namespace ozec
