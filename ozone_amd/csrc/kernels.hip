// gfx950 (CDNA4) kernels for the Ozone EC + chunk-checksum hot path.
//
// GF(2^8) coding (RSUtil.encodeData, EC/rawcoder/util/RSUtil.java:87-133, and the XOR coders):
//   Each coefficient c becomes three byte-permute tables held in registers:
//     T_lo  = c*{0..7}              (2 dwords)   indexed by bits 0-2 of a data byte
//     T_mid = c*{0,8,..,56}         (2 dwords)   indexed by bits 3-5
//     T_top = c*{0,64,128,192}      (1 dword)    indexed by bits 6-7
//   so c*x = T_lo[x&7] ^ T_mid[(x>>3)&7] ^ T_top[x>>6] (GF multiplication is GF(2)-linear in x).  One
//   v_perm_b32 looks up 4 bytes at once, so a 4-byte word costs 3 perms + 2 xors per coefficient, and the
//   per-input selector extraction (5 ops) is shared by every output row.  This is the CDNA4 analogue of the
//   split-nibble pshufb tables GF256.gfVectMulInit builds (GF256.java:259-330): the lookup happens in the
//   VALU permute unit instead of LDS, so it costs no LDS bandwidth and has no bank conflicts.
//   Loads/stores are 16 B per lane (global_load_dwordx4), fully coalesced: lane i of a 256-thread block
//   owns bytes [16i, 16i+16) of a 4 KiB chunk of every unit of one stripe.
//
// CRC32 / CRC32C per bytesPerChecksum window (ChecksumByteBuffer.CrcIntTable, CM/ChecksumByteBuffer.java:51-121):
//   One wave per window.  Lane l owns 16-B blocks l, l+64, l+128, ... of the window (coalesced 1 KiB per
//   wave-instruction) and folds them with Horner's rule  S = S*x^(8*1024) ^ f16(block)  where f16 is the raw
//   CRC of one block (16 slice tables in LDS) and the 1 KiB shift is 4 table lookups.  A 6-level shuffle
//   tree then merges the 64 lane registers (shift by 16*2^m bytes at level m).  Windows whose length is
//   not a multiple of 1 KiB are front-padded with virtual zero blocks (leading zeros do not change a raw
//   CRC that starts from 0); the init value is added back as a precomputed shift(0xFFFFFFFF, N).
#include <algorithm>

#include "device.hpp"

namespace ozec {

TuneKnobs g_tune;
thread_local int64_t t_grid_cap = 0;

namespace {

// Fully unrolled K inputs x R outputs.  Addressing: one buffer descriptor per stripe side (SGPRs), the unit
// offset in soffset (SGPR) and the lane offset v*16 in a single VGPR, so a lane spends 1 VGPR on addresses.
// SREG: lo1/mid1/top are SGPR operands straight from the kernarg segment, lo0/mid0 live in VGPRs (loaded once
// from LDS as single dwords); K*R <= 18.  Otherwise all five dwords are re-read from LDS for every unit
// (uniform-address broadcasts), which keeps large schemas (rs-10-4 decode) inside 128 VGPRs.
// VPT vectors of 16 B per lane per unit (a unit = VPT x 4 KiB of every cell of one stripe); LAUX/SAUX are the
// cache-policy bits of the loads/stores (0 = default, 2 = nt).
// OPT bit 0: parity dwords in three-input XOR chains across the K inputs (1.5 VALU per coefficient and dword instead
// of 2); bit 1: selector masks held in VGPRs (plain VOP2 AND instead of the literal-operand form).
// WIDE (round 5): one buffer descriptor per unit (its own 64-bit base, soffset 0) instead of one per stripe side with
// 32-bit unit offsets -- for units 2 GiB or more apart (separately allocated cells, a stripe spread over a large HBM
// pool), which rebase32 cannot bring into 32 bits.  The descriptors take the SGPRs the register-table form keeps its
// tables in, so WIDE reads the tables from LDS.
template <int K, int R, bool SREG, int VPT, int LAUX, int SAUX, int OPT = 0, bool WIDE = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(OZEC_GF_WAVES, 8))) void gf_code_vec(
    const CodeArgs a, const TabArgs<K * R> tabs) {
  __shared__ __attribute__((aligned(16))) uint32_t s_w[5][K * R];
  for (int t = threadIdx.x; t < K * R; t += blockDim.x)
#pragma unroll
    for (int q = 0; q < 5; ++q) s_w[q][t] = tabs.w[t][q];
  __syncthreads();
  uint32_t vlo0[SREG ? K * R : 1], vmid0[SREG ? K * R : 1];
  if constexpr (SREG) {
#pragma unroll
    for (int t = 0; t < K * R; ++t) {
      vlo0[t] = s_w[0][t];
      vmid0[t] = s_w[2][t];
    }
  }

  uint32_t m7 = 0x07070707u, m3 = 0x03030303u;
  if constexpr (OPT & 2) {  // materialised once, live in VGPRs
    asm volatile("v_mov_b32 %0, 0x7070707" : "=v"(m7));
    asm volatile("v_mov_b32 %0, 0x3030303" : "=v"(m3));
  }
  const uint32_t nvec = static_cast<uint32_t>(a.len >> 4);
  constexpr uint32_t kChunk = kBlock * VPT;
  const uint32_t cpc = (nvec + kChunk - 1) / kChunk;  // units per cell
  const uint32_t units = static_cast<uint32_t>(a.nstripes) * cpc;
  const uint32_t bid = a.unit_map == 1 ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const uint32_t in_extent = unit_extent<K>(a.in_off, a.len), out_extent = unit_extent<R>(a.out_off, a.len);
  for (uint32_t u = bid; u < units; u += gridDim.x) {
    if constexpr (!SREG) asm volatile("" ::: "memory");  // keep the LDS table reads inside the loop
    const uint32_t s = u / cpc;
    const uint32_t c = u - s * cpc;
    const uint32_t v0 = c * kChunk + threadIdx.x;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc_n(a.in + in_off(a, s), in_extent);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc_n(a.out + out_off(a, s), out_extent);
    uint4 x[VPT][K];
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const uint32_t v = v0 + q * kBlock;
      if (v < nvec) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
          if constexpr (WIDE) {
            const auto d = __builtin_amdgcn_raw_buffer_load_b128(
                make_rsrc_n(a.in + in_off(a, s) + a.in_off[j], static_cast<uint32_t>(a.len)), v * 16u, 0, LAUX);
            x[q][j] = make_uint4(d[0], d[1], d[2], d[3]);
          } else {
            const auto d = __builtin_amdgcn_raw_buffer_load_b128(rin, v * 16u, static_cast<int>(a.in_off[j]), LAUX);
            x[q][j] = make_uint4(d[0], d[1], d[2], d[3]);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < VPT; ++q) {
      const uint32_t v = v0 + q * kBlock;
      if (v >= nvec) continue;
      uint4 acc[R];
      XorChain ch[R][4];
#pragma unroll
      for (int r = 0; r < R; ++r) acc[r] = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < K; ++j) {
        auto sel = [&](uint32_t w) {
          if constexpr (OPT & 2) {
            Sel s;
            asm("v_and_b32 %0, %1, %2" : "=v"(s.s0) : "v"(m7), "v"(w));
            asm("v_and_b32 %0, %1, %2" : "=v"(s.s1) : "v"(m7), "v"(w >> 3));
            asm("v_and_b32 %0, %1, %2" : "=v"(s.s2) : "v"(m3), "v"(w >> 6));
            return s;
          } else {
            return make_sel(w);
          }
        };
        const Sel sl[4] = {sel(x[q][j].x), sel(x[q][j].y), sel(x[q][j].z), sel(x[q][j].w)};
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int t = r * K + j;
          if constexpr (OPT & 1) {
            uint32_t lo0, lo1, mid0, mid1, top;
            if constexpr (SREG) {
              lo0 = vlo0[t], mid0 = vmid0[t], lo1 = tabs.w[t][1], mid1 = tabs.w[t][3], top = tabs.w[t][4];
            } else {
              lo0 = s_w[0][t], lo1 = s_w[1][t], mid0 = s_w[2][t], mid1 = s_w[3][t], top = s_w[4][t];
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              ch[r][c].push(SREG ? perm_sv(lo1, lo0, sl[c].s0) : perm_vv(lo1, lo0, sl[c].s0));
              ch[r][c].push(SREG ? perm_sv(mid1, mid0, sl[c].s1) : perm_vv(mid1, mid0, sl[c].s1));
              ch[r][c].push(SREG ? perm_top_s(top, sl[c].s2) : perm_vv(top, top, sl[c].s2));
            }
            continue;
          }
          uint4 m;
          if constexpr (SREG) {
            const RegTab tb{vlo0[t], vmid0[t], tabs.w[t][1], tabs.w[t][3], tabs.w[t][4]};
            m.x = gf_mul4_reg(tb, sl[0]);
            m.y = gf_mul4_reg(tb, sl[1]);
            m.z = gf_mul4_reg(tb, sl[2]);
            m.w = gf_mul4_reg(tb, sl[3]);
          } else {
            const PermTab tb{s_w[0][t], s_w[1][t], s_w[2][t], s_w[3][t], s_w[4][t]};
            m.x = gf_mul4_lds(tb, sl[0]);
            m.y = gf_mul4_lds(tb, sl[1]);
            m.z = gf_mul4_lds(tb, sl[2]);
            m.w = gf_mul4_lds(tb, sl[3]);
          }
          acc[r].x ^= m.x;
          acc[r].y ^= m.y;
          acc[r].z ^= m.z;
          acc[r].w ^= m.w;
        }
        // bound live ranges: input j's selectors (and, in LDS mode, its table reads) stay in this group
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (OPT & 1) {
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = make_uint4(ch[r][0].get(), ch[r][1].get(), ch[r][2].get(), ch[r][3].get());
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        __attribute__((ext_vector_type(4))) unsigned int d = {acc[r].x, acc[r].y, acc[r].z, acc[r].w};
        if constexpr (WIDE) {
          __builtin_amdgcn_raw_buffer_store_b128(
              d, make_rsrc_n(a.out + out_off(a, s) + a.out_off[r], static_cast<uint32_t>(a.len)), v * 16u, 0, SAUX);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(d, rout, v * 16u, static_cast<int>(a.out_off[r]), SAUX);
        }
      }
    }
  }
}

// Runtime k, R outputs (tables re-read from LDS per input). Used for schemas not instantiated above.
// BUF (round 5): cells at any byte offset -- raw buffer loads and stores (32-bit offsets from a rebased CodeArgs,
// rebase32) instead of typed 16-B pointer accesses, which need 16-B alignment.
template <int R, bool BUF = false>
__global__ __launch_bounds__(kBlock) void gf_code_vec_generic(const CodeArgs a, int row0) {
  __shared__ PermTab s_tab[OZEC_MAX_ROWS * OZEC_MAX_K];
  const int k = a.k;
  for (int t = threadIdx.x; t < R * k; t += blockDim.x) s_tab[t] = make_tab(a.coef[row0 * k + t]);
  __syncthreads();
  const uint32_t nvec = static_cast<uint32_t>(a.len >> 4);
  const uint32_t cpc = (nvec + kBlock - 1) / kBlock;
  const uint32_t units = static_cast<uint32_t>(a.nstripes) * cpc;
  for (uint32_t u = blockIdx.x; u < units; u += gridDim.x) {
    const uint32_t s = u / cpc;
    const uint32_t v = (u - s * cpc) * kBlock + threadIdx.x;
    if (v >= nvec) continue;
    const uint8_t *ib = a.in + in_off(a, s) + static_cast<int64_t>(v) * 16;
    uint8_t *ob = a.out + out_off(a, s) + static_cast<int64_t>(v) * 16;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in + in_off(a, s)), rout = make_rsrc(a.out + out_off(a, s));
    uint4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < k; ++j) {
      uint4 x;
      if constexpr (BUF) {
        const auto d = __builtin_amdgcn_raw_buffer_load_b128(rin, v * 16u, static_cast<int>(a.in_off[j]), 0);
        x = make_uint4(d[0], d[1], d[2], d[3]);
      } else {  // align-1 copy: global_load_dwordx4 at any byte address (gfx950 unaligned access mode)
        __builtin_memcpy(&x, ib + a.in_off[j], 16);
      }
      const Sel sx = make_sel(x.x), sy = make_sel(x.y), sz = make_sel(x.z), sw = make_sel(x.w);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const PermTab t = s_tab[r * k + j];
        acc[r].x ^= gf_mul4(t, sx);
        acc[r].y ^= gf_mul4(t, sy);
        acc[r].z ^= gf_mul4(t, sz);
        acc[r].w ^= gf_mul4(t, sw);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (BUF) {
        __attribute__((ext_vector_type(4))) unsigned int d = {acc[r].x, acc[r].y, acc[r].z, acc[r].w};
        __builtin_amdgcn_raw_buffer_store_b128(d, rout, v * 16u, static_cast<int>(a.out_off[row0 + r]), 0);
      } else {
        __builtin_memcpy(ob + a.out_off[row0 + r], &acc[r], 16);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) store_data_hold(acc[r]);
  }
}

// XOR of K inputs (XORRawEncoder / XORRawDecoder): one output.  BUF: any byte offset, as gf_code_vec_generic.
template <int K, bool BUF = false>
__global__ __launch_bounds__(kBlock) void xor_vec(const CodeArgs a) {
  const uint32_t nvec = static_cast<uint32_t>(a.len >> 4);
  const uint32_t cpc = (nvec + kBlock - 1) / kBlock;
  const uint32_t units = static_cast<uint32_t>(a.nstripes) * cpc;
  const int k = K > 0 ? K : a.k;
  for (uint32_t u = blockIdx.x; u < units; u += gridDim.x) {
    const uint32_t s = u / cpc;
    const uint32_t v = (u - s * cpc) * kBlock + threadIdx.x;
    if (v >= nvec) continue;
    const uint8_t *ib = a.in + in_off(a, s) + static_cast<int64_t>(v) * 16;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(a.in + in_off(a, s));
    uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < (K > 0 ? K : OZEC_MAX_K); ++j) {
      if (K == 0 && j >= k) break;
      uint4 x;
      if constexpr (BUF) {
        const auto d = __builtin_amdgcn_raw_buffer_load_b128(rin, v * 16u, static_cast<int>(a.in_off[j]), 0);
        x = make_uint4(d[0], d[1], d[2], d[3]);
      } else {  // align-1 copy: global_load_dwordx4 at any byte address (gfx950 unaligned access mode)
        __builtin_memcpy(&x, ib + a.in_off[j], 16);
      }
      acc.x ^= x.x;
      acc.y ^= x.y;
      acc.z ^= x.z;
      acc.w ^= x.w;
    }
    if constexpr (BUF) {
      __attribute__((ext_vector_type(4))) unsigned int d = {acc.x, acc.y, acc.z, acc.w};
      __builtin_amdgcn_raw_buffer_store_b128(d, make_rsrc(a.out + out_off(a, s)), v * 16u,
                                             static_cast<int>(a.out_off[0]), 0);
      store_data_hold(acc);
    } else {
      __builtin_memcpy(a.out + out_off(a, s) + a.out_off[0] + static_cast<int64_t>(v) * 16, &acc, 16);
    }
  }
}

// Byte-granular coding for lengths not a multiple of 16 (tail) and unaligned layouts.
__global__ __launch_bounds__(kBlock) void gf_code_bytes(const CodeArgs a, int64_t start) {
  __shared__ PermTab s_tab[OZEC_MAX_ROWS * OZEC_MAX_K];
  const int k = a.k, rows = a.rows;
  build_tabs(s_tab, a, rows, k);
  __syncthreads();
  const int64_t span = a.len - start;
  const int64_t total = span * a.nstripes;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t s = i / span;
    const int64_t x = start + (i - s * span);
    const uint8_t *ib = a.in + in_off(a, s) + x;
    uint8_t *ob = a.out + out_off(a, s) + x;
    for (int r = 0; r < rows; ++r) {
      uint32_t acc = 0;
      for (int j = 0; j < k; ++j) {
        const uint32_t b = ib[a.in_off[j]];
        acc ^= a.all_ones ? b : (gf_mul4(s_tab[r * k + j], make_sel(b)) & 0xffu);
      }
      ob[a.out_off[r]] = static_cast<uint8_t>(acc);
    }
  }
}

// One wave per (cell, window).  Lane l owns 16-B blocks l, l+64, ... of the window and folds every block of its group of D steps
// into its register through the table set of the block's distance to the group end (no per-step register
// shift): S = shift_group(S) ^ XOR_{steps r, blocks s} G26[r*B+s](block).  Windows are front-padded with
// virtual zero blocks to whole groups; virtual blocks are not loaded and add nothing.
// UA (round 5): cells at any byte offset -- 16-B loads through an align-1 copy (global_load_dwordx4 at the unaligned
// address, which gfx950 serves at full rate, profiles/r05/unaligned/) instead of the aligned non-temporal load.
template <int B, int D, int PD = 1, bool UA = false>
__global__ __launch_bounds__(kBlock) void crc_windows_g26(const CrcArgs a) {
  constexpr int E = B * D;
  static_assert(D % 2 == 0, "two register sets alternate across steps");
  __shared__ __attribute__((aligned(16))) uint32_t s_t[g26_words(E)];
  load_tables(s_t, a.g26[g26_slot(B, D)], g26_words(E));
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t units = a.ncells * a.nwin;
  const int64_t bid = a.unit_map == 1 ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  for (int64_t u = bid * (kBlock / 64) + wave; u < units; u += static_cast<int64_t>(gridDim.x) * (kBlock / 64)) {
    const int64_t c = u / a.nwin;
    const int64_t w = u - c * a.nwin;
    const bool last = w == a.nwin - 1;
    const int64_t N = last ? a.len - w * a.bpc : a.bpc;
    const int64_t m = N >> 4;
    const int64_t G = (m + 64 * E - 1) / (64 * E);  // groups
    const int64_t P = G * 64 * E - m;               // virtual zero blocks in front
    const uint8_t *win = a.base + c * a.cell_stride + w * a.bpc;
    uint32_t S = 0;
    auto load_step = [&](int64_t t, uint4 (&dst)[B]) {
      const bool pad = t * 64 * B < P;  // wave-uniform
#pragma unroll
      for (int q = 0; q < B; ++q) {
        const int64_t vb = t * 64 * B + lane * B + q - P;
        if (!pad || vb >= 0) {
          if constexpr (UA) {
            __builtin_memcpy(&dst[q], win + vb * 16, 16);
          } else {
            const u32x4 d = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(win + vb * 16));
            dst[q] = make_uint4(d[0], d[1], d[2], d[3]);
          }
        } else {
          dst[q] = make_uint4(0, 0, 0, 0);
        }
      }
    };
    if constexpr (PD == 1) {
      uint4 xa[B], xb[B];
      if (G > 0) load_step(0, xa);
      for (int64_t g = 0; g < G; ++g) {
#pragma unroll
        for (int rr = 0; rr < D; ++rr) {
          const int64_t t = g * D + rr;
          uint4(&cur)[B] = (rr & 1) ? xb : xa;
          uint4(&nxt)[B] = (rr & 1) ? xa : xb;
          if (rr + 1 < D || g + 1 < G) load_step(t + 1, nxt);
#pragma unroll
          for (int q = 0; q < B; ++q) S ^= g26_block(s_t + ((D - 1 - rr) * B + (B - 1 - q)) * kG26Set, cur[q]);
        }
        if (g + 1 < G) S = g5_shift(s_t + g26_gshift(E), S);
      }
    } else {  // two steps in flight: three register sets rotated by copies
      uint4 x0[B], x1[B], x2[B];
      const int64_t T = G * D;
      if (T > 0) load_step(0, x0);
      if (T > 1) load_step(1, x1);
      for (int64_t g = 0; g < G; ++g) {
#pragma unroll
        for (int rr = 0; rr < D; ++rr) {
          const int64_t t = g * D + rr;
          if (t + 2 < T) load_step(t + 2, x2);
#pragma unroll
          for (int q = 0; q < B; ++q) S ^= g26_block(s_t + ((D - 1 - rr) * B + (B - 1 - q)) * kG26Set, x0[q]);
#pragma unroll
          for (int q = 0; q < B; ++q) {
            x0[q] = x1[q];
            x1[q] = x2[q];
          }
        }
        if (g + 1 < G) S = g5_shift(s_t + g26_gshift(E), S);
      }
    }
    S = g5_lane_tree(s_t + g26_tree(E) - kG5Tree, S, lane);
    for (int64_t i = m * 16; i < N; ++i) S = (S >> 8) ^ s_t[g26_t0(E) + ((S ^ win[i]) & 0xff)];
    if (lane == 0) crc_emit(a, c, w, S, last);
  }
}

// Streaming form of crc_windows_g26 (B = 1) for full windows of bpc % (1024*D) == 0 bytes: each wave owns a
// contiguous run of `per_wave` windows (cell-major, so consecutive windows are consecutive in memory) and keeps
// NS - 1 steps of loads in flight ACROSS window boundaries -- the per-window kernel drains its load pipeline at
// the end of every window (16 steps of a 16 KiB window) and refills it at the start of the next.  At a window
// end the 64 lane registers are merged, the CRC is emitted, and the register restarts at 0; no virtual blocks.
// Window w of cell c is emitted as (c, w) with the full-window init (a short last window, if any, is left to
// crc_windows_g26).  Persistent grid: one resident set of waves, each streaming its own stretch of HBM.
// Code shape, from the ISA: the loads are unconditional (past the end of its run the cursor stays on the run's
// last step, so the NS - 1 surplus loads re-read it) and land in a ring of NS register sets indexed by the
// unrolled step (NS divides D), so no register copy or branch sits between a load and its use -- either makes
// the compiler wait for every load in flight (vmcnt(0)) at every step.  For the same reason verify mode reads
// the stored CRC with a scalar load (lgkmcnt), not a vector one.
// XO: the register moves by one step with no shift lookups (kernels.hpp kXo*): it is XORed into the first dword of
// its lane's next block, which is looked up in the XO set; the advance is undone once per window.  D then only sets
// the unroll (the load ring NS divides it); the LDS holds the lane-tree shifts and the XO blob instead of D sets.
// VR (round 5, verify with XO): the wave first checks its whole run of windows as ONE message -- the register is not
// reset and not merged at window ends, so the lane tree and the XO inverse run once per run instead of once per
// window -- against the stored window CRCs folded by Horner's rule (E = E x^(8 bpc) + raw_w, the shift by bpc from
// a.bshift).  A run that matches is done (16 windows of 16 KiB: one tree instead of 16, 7 lookups per window for E);
// one that does not is checked again window by window, so the first failing window recorded per cell is the
// reference's.  Two windows of a run with the same error pattern k windows apart cancel only if
// 1 + x^(8 bpc k) shares a factor with P beyond x + 1 (tests/test_cv_weights.py).
// TB (round 5, compute with XO): the registers of TB consecutive windows go through ONE reduce-scatter lane tree
// (g5_lane_tree_rs; TB - 1 + 6 - log2 TB shifts instead of 6 TB) and one XO inverse per lane, then lanes 0..TB-1 store
// one window each.
template <int D, int NS, bool XO = false, bool VR = false, int TB = 1>
__global__ __launch_bounds__(kBlock) void crc_windows_g26s(const CrcArgs a, int64_t nfull, int64_t per_wave) {
  static_assert(NS >= 2 && D % NS == 0, "the register ring must divide the unrolled group");
  static_assert(!VR || XO, "the run check folds through the XO blob");
  static_assert(TB == 1 || (XO && (TB == 2 || TB == 4 || TB == 8)), "batched trees: XO, a power of two");
  constexpr int kTree = XO ? 0 : g26_tree(D), kXoOff = 1344, kBsOff = 1344 + kXoWords;
  __shared__ __attribute__((aligned(16))) uint32_t s_t[XO ? 1344 + kXoWords + (VR ? 224 : 0) : g26_words(D)];
  if constexpr (XO) {
    load_tables(s_t, a.g26[g26_slot(1, D)] + g26_tree(D), 1344);
    load_tables(s_t + kXoOff, a.xo, kXoWords);
    if constexpr (VR) load_tables(s_t + kBsOff, a.bshift, 224);
  } else {
    load_tables(s_t, a.g26[g26_slot(1, D)], g26_words(D));
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t bid = a.unit_map == 1 ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int64_t total = a.ncells * nfull;
  const int64_t u0 = (bid * (kBlock / 64) + wave) * per_wave;
  if (u0 >= total) return;
  const int64_t u1 = u0 + per_wave < total ? u0 + per_wave : total;
  const int32_t G = static_cast<int32_t>(a.bpc >> 10) / D;  // groups of D steps per window (>= 1)
  const int32_t T = G * D;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  // load cursor (wave-uniform): window lu = (cell lc, window lw), step lt
  int64_t lu = u0, lc = u0 / nfull, lw = u0 - lc * nfull;
  int32_t lt = 0;
  const uint8_t *lbase = a.base + lc * a.cell_stride + lw * a.bpc + lane * 16;
  auto load_next = [&](uint4 &dst) {
    const u32x4 d = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(lbase + lt * 1024));
    dst = make_uint4(d[0], d[1], d[2], d[3]);
    if (lt + 1 < T) {
      ++lt;
    } else if (lu + 1 < u1) {
      lt = 0;
      ++lu;
      if (++lw == nfull) {
        lw = 0;
        ++lc;
      }
      lbase = a.base + lc * a.cell_stride + lw * a.bpc + lane * 16;
    }
  };
  uint4 x[NS];
  if constexpr (VR) {
    if (a.expected) {  // (VR is launched for verify only)
#pragma unroll
      for (int i = 0; i + 1 < NS; ++i) load_next(x[i]);
      int64_t cc = u0 / nfull, cw = u0 - cc * nfull;
      uint32_t S = 0, E = 0;
      for (int64_t u = u0; u < u1; ++u) {
        const uint32_t ex0 = *(cu32 *)(a.expected + cc * a.out_cell_stride + cw);
        E = g5_shift(s_t + kBsOff, E) ^ ~((a.expected_be ? __builtin_bswap32(ex0) : ex0) ^ a.init_full);
        int32_t g = 0;
        do {
#pragma unroll
          for (int rr = 0; rr < D; ++rr) {
            load_next(x[(rr + NS - 1) % NS]);
            uint4 xs = x[rr % NS];
            xs.x ^= S;
            S = g26_block(s_t + kXoOff, xs);
          }
        } while (++g < G);
        if (++cw == nfull) {
          cw = 0;
          ++cc;
        }
      }
      S = g5_lane_tree(s_t + kTree - kG5Tree, S, lane);
      S = g5_shift(s_t + kXoOff + kXoInv, S);
      if (S == E) return;  // wave-uniform: every lane holds the merged register
      // the rare path: this run window by window (the cursor back at its start)
      lu = u0, lc = u0 / nfull, lw = u0 - lc * nfull, lt = 0;
      lbase = a.base + lc * a.cell_stride + lw * a.bpc + lane * 16;
    }
  }
#pragma unroll
  for (int i = 0; i + 1 < NS; ++i) load_next(x[i]);
  if constexpr (TB > 1) {
    if (!a.expected) {
      for (int64_t ub = u0; ub < u1; ub += TB) {
        uint32_t Sw[TB];
#pragma unroll
        for (int q = 0; q < TB; ++q) {
          uint32_t S = 0;
          if (ub + q < u1) {  // wave-uniform
            int32_t g = 0;
            do {
#pragma unroll
              for (int rr = 0; rr < D; ++rr) {
                load_next(x[(rr + NS - 1) % NS]);
                uint4 xs = x[rr % NS];
                xs.x ^= S;
                S = g26_block(s_t + kXoOff, xs);
              }
            } while (++g < G);
          }
          Sw[q] = S;
        }
        int q = 0;
        uint32_t v = g5_lane_tree_rs<TB>(s_t + kTree - kG5Tree, Sw, lane, q);
        v = g5_shift(s_t + kXoOff + kXoInv, v);
        if (lane < TB && ub + q < u1) {
          const int64_t c = (ub + q) / nfull, w = ub + q - c * nfull;
          a.out[c * a.out_cell_stride + w] = crc_finish(v, a.init_full, a.raw, a.big_endian);
        }
      }
      return;
    }
  }
  int64_t cc = u0 / nfull, cw = u0 - cc * nfull;  // compute cursor: (cell, window) of u
  for (int64_t u = u0; u < u1; ++u) {
    uint32_t ex = 0;
    if (a.expected) ex = *(cu32 *)(a.expected + cc * a.out_cell_stride + cw);
    uint32_t S = 0;
    int32_t g = 0;
    do {
#pragma unroll
      for (int rr = 0; rr < D; ++rr) {
        load_next(x[(rr + NS - 1) % NS]);
        if constexpr (XO) {
          uint4 xs = x[rr % NS];
          xs.x ^= S;
          S = g26_block(s_t + kXoOff, xs);
        } else {
          S ^= g26_block(s_t + (D - 1 - rr) * kG26Set, x[rr % NS]);
        }
      }
      if (!XO && g + 1 < G) S = g5_shift(s_t + g26_gshift(D), S);
    } while (++g < G);
    S = g5_lane_tree(s_t + kTree - kG5Tree, S, lane);
    if constexpr (XO) S = g5_shift(s_t + kXoOff + kXoInv, S);
    if (lane == 0) {
      if (a.expected) {
        if (crc_finish(S, a.init_full, 0, 0) != (a.expected_be ? __builtin_bswap32(ex) : ex))
          atomicMin(a.mismatch + cc, a.mismatch_base + static_cast<int32_t>(cw));
      } else {
        a.out[cc * a.out_cell_stride + cw] = crc_finish(S, a.init_full, a.raw, a.big_endian);
      }
    }
    if (++cw == nfull) {
      cw = 0;
      ++cc;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Fused encode + CRC: one wave per (stripe, window); each step a lane takes the 16-B blocks of every data unit
// (lanes interleaved, 64 blocks per step), produces the parity blocks and folds all K+R units into their CRC
// registers while the bytes are in VGPRs.
// XORC (all-ones single row: the XOR codec): the output is the XOR of the inputs, and since the raw CRC
// register recursion is GF(2)-linear in (register, data), the output's register is the XOR of the inputs'
// registers at every step -- its CRC costs no table lookups.
// Fused encode + CRC on the G26 scheme (B = 1): one wave per (stripe, window), D steps per group, every
// unit's register updated with S ^= G26[D-1-rr](block) and shifted once per group.  GF coefficient tables
// (TM): 1 = {lo0, lo1, mid0, mid1} from LDS in one ds_read_b128 broadcast + top as an SGPR operand;
// 2 = lo1/mid1/top as SGPR operands, {lo0, mid0} from LDS in one ds_read_b64 broadcast; 3 = as 1 with top from
// LDS too (ds_read_b32 broadcast).
// XO (XOR codec only): the input registers move by one step with no shift lookups (kernels.hpp kXo*; as
// crc_windows_g26s), the parity's register is still the XOR of theirs, and the advance is undone once per window.
// TAIL (round 6, the XOR codec only): cells of any length at any byte offset.  The window loop takes the whole 16-B
// blocks of the last window (buffer accesses at any byte address); after the lane tree, the lane of unit q extends its
// register bytewise over the window's last 1-15 bytes, the parity lane XORing the K inputs' bytes and storing them
// (xor_tail).  The raw register update is GF(2)-linear in (register, byte), so the parity's register stays the XOR of
// the inputs' registers through the tail as well.
template <int K>
__device__ __forceinline__ uint32_t xor_tail(const EncCrcArgs &e, __amdgpu_buffer_rsrc_t rin,
                                             __amdgpu_buffer_rsrc_t rout, int q, uint32_t v, uint32_t o0, int32_t tb) {
  const CodeArgs &a = e.code;
  const uint32_t poly = e.crc.poly;
  for (int32_t b = 0; b < tb; ++b) {
    const uint32_t ob = o0 + static_cast<uint32_t>(b);
    uint32_t byte = 0;
    if (q < K) {
      byte = __builtin_amdgcn_raw_buffer_load_b8(rin, ob, static_cast<int>(a.in_off[q]), 0);
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) byte ^= __builtin_amdgcn_raw_buffer_load_b8(rin, ob, static_cast<int>(a.in_off[j]), 0);
      __builtin_amdgcn_raw_buffer_store_b8(static_cast<uint8_t>(byte), rout, ob, static_cast<int>(a.out_off[0]), 0);
    }
    v ^= byte;
#pragma unroll
    for (int i = 0; i < 8; ++i) v = (v >> 1) ^ (poly & (0u - (v & 1u)));
  }
  return v;
}

// WIDE (round 6, the XOR codec only): units 2 GiB or more apart -- one buffer descriptor per unit (64-bit base), the tail
// through 64-bit pointers (xor_tail_wide).
template <int K>
__device__ __forceinline__ uint32_t xor_tail_wide(const EncCrcArgs &e, const uint8_t *ib, uint8_t *ob, int q, uint32_t v,
                                                  uint32_t o0, int32_t tb) {
  const CodeArgs &a = e.code;
  const uint32_t poly = e.crc.poly;
  for (int32_t b = 0; b < tb; ++b) {
    const int64_t o = static_cast<int64_t>(o0) + b;
    uint32_t byte = 0;
    if (q < K) {
      byte = ib[a.in_off[q] + o];
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) byte ^= ib[a.in_off[j] + o];
      ob[a.out_off[0] + o] = static_cast<uint8_t>(byte);
    }
    v ^= byte;
#pragma unroll
    for (int i = 0; i < 8; ++i) v = (v >> 1) ^ (poly & (0u - (v & 1u)));
  }
  return v;
}

template <int K, int R, int D, bool XORC, int TM, int WAVES = 4, bool PF = false, bool HV = false, bool XO = false,
          bool TAIL = false, bool WIDE = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(WAVES, 8))) void encode_crc_g26(const EncCrcArgs e, const TabArgs<K * R> tabs) {
  constexpr int E = D;
  static_assert(D >= 1, "group of at least one step");
  static_assert(!XO || XORC, "XO only where every CRC register belongs to an input (the XOR codec)");
  static_assert(!TAIL || (XORC && R == 1 && !XO), "byte tails: the XOR codec's default form");
  static_assert(!WIDE || (XORC && R == 1 && !XO), "one descriptor per unit: the XOR codec's default form");
  constexpr int kXoOff = g26_words(E);  // XO: the XO blob after the G26 blob
  __shared__ __attribute__((aligned(16))) uint32_t s_t[g26_words(E) + (XO ? kXoWords : 0)];
  __shared__ __attribute__((aligned(16))) uint4 s_q[K * R];
  __shared__ __attribute__((aligned(16))) uint2 s_d[K * R];
  __shared__ uint32_t s_top[K * R];
  const CodeArgs &a = e.code;
  const CrcArgs &cr = e.crc;
  load_tables(s_t, cr.g26[g26_slot(1, D)], g26_words(E));
  if constexpr (XO) load_tables(s_t + kXoOff, cr.xo, kXoWords);
  for (int t = threadIdx.x; t < K * R; t += blockDim.x) {
    s_q[t] = make_uint4(tabs.w[t][0], tabs.w[t][1], tabs.w[t][2], tabs.w[t][3]);
    s_d[t] = make_uint2(tabs.w[t][0], tabs.w[t][2]);
    s_top[t] = tabs.w[t][4];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwin = cr.nwin;
  const int64_t units = a.nstripes * nwin;
  const int64_t bid = a.unit_map == 1 ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int64_t wmax = cr.bpc < a.len ? cr.bpc : a.len;  // bytes of a window
  const uint32_t in_extent = unit_extent<K>(a.in_off, wmax), out_extent = unit_extent<R>(a.out_off, wmax);
  for (int64_t u = bid * (kBlock / 64) + wave; u < units; u += static_cast<int64_t>(gridDim.x) * (kBlock / 64)) {
    const int64_t s = u / nwin;
    const int64_t w = u - s * nwin;
    const bool last = w == nwin - 1;
    const int64_t N = last ? a.len - w * cr.bpc : cr.bpc;
    const int64_t m = N >> 4;
    const int32_t G = static_cast<int32_t>((m + 64 * D - 1) / (64 * D));
    const int32_t P = G * 64 * D - static_cast<int32_t>(m);  // window <= 2 GiB: 32-bit block indices
    const uint8_t *const ib = a.in + in_off(a, s) + w * cr.bpc;
    uint8_t *const ob = a.out + out_off(a, s) + w * cr.bpc;
    const __amdgpu_buffer_rsrc_t rin = make_rsrc_n(ib, in_extent);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc_n(ob, out_extent);
    uint32_t S[K + R];
#pragma unroll
    for (int q = 0; q < K + R; ++q) S[q] = 0;
    auto load_x = [&](int32_t t, uint4 (&dst)[K]) {
      const int32_t vb = t * 64 + lane - P;
      auto ld = [&](int j) {
        if constexpr (WIDE) {
          const auto d = __builtin_amdgcn_raw_buffer_load_b128(make_rsrc_n(ib + a.in_off[j], static_cast<uint32_t>(wmax)),
                                                               static_cast<uint32_t>(vb) * 16u, 0, 2);
          return make_uint4(d[0], d[1], d[2], d[3]);
        } else {
          const auto d = __builtin_amdgcn_raw_buffer_load_b128(rin, static_cast<uint32_t>(vb) * 16u,
                                                               static_cast<int>(a.in_off[j]), 2);
          return make_uint4(d[0], d[1], d[2], d[3]);
        }
      };
      if (__builtin_expect(t * 64 >= P, 1)) {  // wave-uniform: only the first steps hold virtual blocks
#pragma unroll
        for (int j = 0; j < K; ++j) dst[j] = ld(j);
      } else {
#pragma unroll
        for (int j = 0; j < K; ++j) dst[j] = vb >= 0 ? ld(j) : make_uint4(0, 0, 0, 0);
      }
    };
    static_assert(!PF || D % 2 == 0, "prefetch alternates two register sets");
    uint4 xa[K], xb[K];
    const uint32_t vmask = 0x7cu;
    if (PF && G > 0) load_x(0, xa);
    for (int32_t g = 0; g < G; ++g) {
#pragma unroll
      for (int rr = 0; rr < D; ++rr) {
        asm volatile("" ::: "memory");  // keep the LDS coefficient reads inside the step
        const int32_t t = g * D + rr;
        const int32_t vb = t * 64 + lane - P;
        uint4(&x)[K] = (PF && (rr & 1)) ? xb : xa;
        if constexpr (PF) {
          if (rr + 1 < D || g + 1 < G) load_x(t + 1, (rr & 1) ? xa : xb);
        } else {
          load_x(t, x);
        }
        uint4 acc[R];
        if constexpr (XORC) {
          acc[0] = x[0];
#pragma unroll
          for (int j = 1; j < K; ++j) {
            acc[0].x ^= x[j].x;
            acc[0].y ^= x[j].y;
            acc[0].z ^= x[j].z;
            acc[0].w ^= x[j].w;
          }
        } else {
          // parity dword = XOR of 3K permute results, reduced by chained three-input XORs (1.5 ops per
          // coefficient instead of 2 for xor3-then-accumulate)
          XorChain ch[R][4];
#pragma unroll
          for (int j = 0; j < K; ++j) {
            const uint32_t xw[4] = {x[j].x, x[j].y, x[j].z, x[j].w};
            Sel sl[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) sl[c] = make_sel(xw[c]);
#pragma unroll
            for (int r = 0; r < R; ++r) {
              const int tt = r * K + j;
              uint32_t lo0, lo1, mid0, mid1, top;
              if constexpr (TM == 1 || TM == 3) {
                const uint4 q4 = s_q[tt];
                lo0 = q4.x, lo1 = q4.y, mid0 = q4.z, mid1 = q4.w;
                top = TM == 1 ? tabs.w[tt][4] : s_top[tt];
              } else {
                const uint2 d2 = s_d[tt];
                lo0 = d2.x, mid0 = d2.y, lo1 = tabs.w[tt][1], mid1 = tabs.w[tt][3], top = tabs.w[tt][4];
              }
#pragma unroll
              for (int c = 0; c < 4; ++c) {
                ch[r][c].push(TM == 2 ? perm_sv(lo1, lo0, sl[c].s0) : perm_vv(lo1, lo0, sl[c].s0));
                ch[r][c].push(TM == 2 ? perm_sv(mid1, mid0, sl[c].s1) : perm_vv(mid1, mid0, sl[c].s1));
                ch[r][c].push(TM == 3 ? perm_vv(top, top, sl[c].s2) : perm_top_s(top, sl[c].s2));
              }
            }
          }
#pragma unroll
          for (int r = 0; r < R; ++r)
            acc[r] = make_uint4(ch[r][0].get(), ch[r][1].get(), ch[r][2].get(), ch[r][3].get());
        }
        if (vb >= 0) {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            __attribute__((ext_vector_type(4))) unsigned int d = {acc[r].x, acc[r].y, acc[r].z, acc[r].w};
            if constexpr (WIDE) {
              __builtin_amdgcn_raw_buffer_store_b128(d, make_rsrc_n(ob + a.out_off[r], static_cast<uint32_t>(wmax)),
                                                     static_cast<uint32_t>(vb) * 16u, 0, 2);
            } else {
              __builtin_amdgcn_raw_buffer_store_b128(d, rout, static_cast<uint32_t>(vb) * 16u,
                                                     static_cast<int>(a.out_off[r]), 2);
            }
          }
        }
        if constexpr (XORC) store_data_hold(acc[0]);
#pragma unroll
        for (int j = 0; j < (XORC ? K : K + R); ++j) {
          if constexpr (XO) {
            uint4 xs = x[j];
            xs.x ^= S[j];
            S[j] = g26_block<HV, false>(s_t + kXoOff, xs, vmask);
          } else {
            S[j] ^= g26_block<HV, false>(s_t + (D - 1 - rr) * kG26Set, j < K ? x[j] : acc[j - K], vmask);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (!XO && g + 1 < G) {
#pragma unroll
        for (int j = 0; j < (XORC ? K : K + R); ++j) S[j] = g5_shift(s_t + g26_gshift(E), S[j]);
      }
    }
    if constexpr (XORC) {
      S[K] = 0;
#pragma unroll
      for (int j = 0; j < K; ++j) S[K] ^= S[j];
    }
    if constexpr (XO) {  // undo the advance (the parity register is linear in the inputs': the same once)
#pragma unroll
      for (int q = 0; q <= K; ++q) S[q] = g5_shift(s_t + kXoOff + kXoInv, S[q]);
    }
    const uint32_t init = last ? cr.init_last : cr.init_full;
    int32_t tb = 0;
    if constexpr (TAIL) tb = last ? static_cast<int32_t>(N & 15) : 0;
#pragma unroll
    for (int q = 0; q < K + R; ++q) {
      uint32_t v = g5_lane_tree(s_t + g26_tree(E) - kG5Tree, S[q], lane);
      if (lane == q) {
        if constexpr (TAIL) {
          if (tb != 0) {
            if constexpr (WIDE) v = xor_tail_wide<K>(e, ib, ob, q, v, static_cast<uint32_t>(m * 16), tb);
            else v = xor_tail<K>(e, rin, rout, q, v, static_cast<uint32_t>(m * 16), tb);
          }
        }
        if (!e.verify) {
          cr.out[(s * (K + R) + q) * nwin + w] = crc_finish(v, init, cr.raw, cr.big_endian);
        } else if (q >= K) {
          cr.out[(s * R + (q - K)) * nwin + w] = crc_finish(v, init, cr.raw, cr.big_endian);
        } else if (cr.expected) {
          const int64_t idx = (s * e.exp_units + e.in_unit[q]) * nwin + w;
          const uint32_t ex = cr.expected_be ? __builtin_bswap32(cr.expected[idx]) : cr.expected[idx];
          if (crc_finish(v, init, 0, 0) != ex)
            atomicMin(cr.mismatch + s, static_cast<int32_t>(e.in_unit[q] * nwin + w));
        }
      }
    }
  }
}

// Streaming fused XOR encode + CRC (the XOR codec: one all-ones row) for stripes whose windows are all full
// (len % bpc == 0, bpc % (1024*D) == 0).  As crc_windows_g26s: each wave owns a contiguous run of (stripe,
// window) units on a persistent grid and keeps NS - 1 steps of the K input loads in flight across window and
// stripe ends; loads and parity stores are unconditional (no virtual blocks in full windows; past the end of
// its run the load cursor stays on the run's last step), so no step waits for the whole pipeline.  The
// per-window kernel above masks its loads and stores per lane for virtual blocks, and the compiler then waits
// with vmcnt(0) at every step (ISA of encode_crc_g26<2, 1, 4, true, 1, 4, true>).  Encode mode only.
template <int K, int D, int NS>
__global__ __launch_bounds__(kBlock) void encode_xor_crc_g26s(const EncCrcArgs e, int64_t per_wave) {
  static_assert(NS >= 2 && D % NS == 0, "the register ring must divide the unrolled group");
  __shared__ __attribute__((aligned(16))) uint32_t s_t[g26_words(D)];
  const CodeArgs &a = e.code;
  const CrcArgs &cr = e.crc;
  load_tables(s_t, cr.g26[g26_slot(1, D)], g26_words(D));
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwin = cr.nwin;
  const int64_t total = a.nstripes * nwin;
  const int64_t bid = a.unit_map == 1 ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  const int64_t u0 = (bid * (kBlock / 64) + wave) * per_wave;
  if (u0 >= total) return;
  const int64_t u1 = u0 + per_wave < total ? u0 + per_wave : total;
  const int32_t G = static_cast<int32_t>(cr.bpc >> 10) / D;  // groups of D steps per window (>= 1)
  const int32_t T = G * D;
  const uint32_t voff = static_cast<uint32_t>(lane) * 16u;
  // load cursor (wave-uniform): unit lu = (stripe ls, window lw), step lt
  int64_t lu = u0, ls = u0 / nwin, lw = u0 - ls * nwin;
  int32_t lt = 0;
  const uint32_t in_extent = unit_extent<K>(a.in_off, cr.bpc), out_extent = unit_extent<1>(a.out_off, cr.bpc);
  __amdgpu_buffer_rsrc_t rin = make_rsrc_n(a.in + in_off(a, ls) + lw * cr.bpc, in_extent);
  auto load_next = [&](uint4 (&dst)[K]) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const auto d = __builtin_amdgcn_raw_buffer_load_b128(rin, voff, static_cast<int>(a.in_off[j]) + lt * 1024, 2);
      dst[j] = make_uint4(d[0], d[1], d[2], d[3]);
    }
    if (lt + 1 < T) {
      ++lt;
    } else if (lu + 1 < u1) {
      lt = 0;
      ++lu;
      if (++lw == nwin) {
        lw = 0;
        ++ls;
      }
      rin = make_rsrc_n(a.in + in_off(a, ls) + lw * cr.bpc, in_extent);
    }
  };
  uint4 x[NS][K];
#pragma unroll
  for (int i = 0; i + 1 < NS; ++i) load_next(x[i]);
  int64_t cs = u0 / nwin, cw = u0 - cs * nwin;  // compute cursor
  for (int64_t u = u0; u < u1; ++u) {
    const __amdgpu_buffer_rsrc_t rout = make_rsrc_n(a.out + out_off(a, cs) + cw * cr.bpc, out_extent);
    uint32_t S[K];
#pragma unroll
    for (int j = 0; j < K; ++j) S[j] = 0;
    int32_t g = 0;
    do {
#pragma unroll
      for (int rr = 0; rr < D; ++rr) {
        load_next(x[(rr + NS - 1) % NS]);
        const uint4(&cur)[K] = x[rr % NS];
        uint4 par = cur[0];
#pragma unroll
        for (int j = 1; j < K; ++j) {
          par.x ^= cur[j].x;
          par.y ^= cur[j].y;
          par.z ^= cur[j].z;
          par.w ^= cur[j].w;
        }
        __attribute__((ext_vector_type(4))) unsigned int pd = {par.x, par.y, par.z, par.w};
        __builtin_amdgcn_raw_buffer_store_b128(pd, rout, voff, static_cast<int>(a.out_off[0]) + (g * D + rr) * 1024,
                                               2);
        store_data_hold(par);
#pragma unroll
        for (int j = 0; j < K; ++j) S[j] ^= g26_block(s_t + (D - 1 - rr) * kG26Set, cur[j]);
      }
      if (g + 1 < G) {
#pragma unroll
        for (int j = 0; j < K; ++j) S[j] = g5_shift(s_t + g26_gshift(D), S[j]);
      }
    } while (++g < G);
    // the parity's register is the XOR of the inputs' registers (the raw CRC is GF(2)-linear)
    uint32_t Sp = S[0];
#pragma unroll
    for (int j = 1; j < K; ++j) Sp ^= S[j];
#pragma unroll
    for (int q = 0; q <= K; ++q) {
      const uint32_t v = g5_lane_tree(s_t + g26_tree(D) - kG5Tree, q < K ? S[q] : Sp, lane);
      if (lane == q) cr.out[(cs * (K + 1) + q) * nwin + cw] = crc_finish(v, cr.init_full, cr.raw, cr.big_endian);
    }
    if (++cw == nwin) {
      cw = 0;
      ++cs;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// COMPOSITE_CRC (CrcUtil / CrcComposer, hadoop-ozone/common/.../client/checksum/): CRC values in the reversed
// representation (bit 31 = x^0); composing A then B = A * x^(8|B|) mod P xor B.

// CrcUtil.galoisFieldMultiply (CrcUtil.java:249-270), branch-free
__device__ __forceinline__ uint32_t gf32_mul(uint32_t p, uint32_t q, uint32_t m) {
  uint32_t sum = 0, px = p;
#pragma unroll 8
  for (int i = 31; i >= 0; --i) {
    sum ^= px & (0u - ((q >> i) & 1u));
    px = (px >> 1) ^ (m & (0u - (px & 1u)));
  }
  return sum;
}

// CrcUtil.getMonomial (CrcUtil.java:74-98): x^(8*len) mod m, len >= 0
__device__ uint32_t gf32_monomial(int64_t len, uint32_t m) {
  uint32_t mult = 0x80000000u >> 8, prod = 0x80000000u;
  for (; len > 0; len >>= 1) {
    if (len & 1) prod = gf32_mul(prod, mult, m);
    mult = gf32_mul(mult, mult, m);
  }
  return prod;
}

// One wave per cell: lane l composes a contiguous run of windows, then a 6-level shuffle tree composes the
// 64 runs in order.  Equal to CrcComposer.update over the windows in order (its `cur == 0` shortcut gives the
// same value as composing onto 0), i.e. to the CRC of the whole cell.
__global__ __launch_bounds__(kBlock) void compose_windows(const ComposeArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t cell = static_cast<int64_t>(blockIdx.x) * (kBlock / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (cell >= a.ncells) return;
  const uint32_t *c = a.crcs + cell * a.cell_stride;
  const int64_t per = (a.nwin + 63) / 64;
  const int64_t w0 = lane * per, w1 = w0 + per < a.nwin ? w0 + per : a.nwin;
  uint32_t acc = 0;
  int64_t len = 0;
  for (int64_t w = w0; w < w1; ++w) {
    const bool last = w == a.nwin - 1;
    uint32_t v = c[w];
    if (a.big_endian_in) v = __builtin_bswap32(v);
    acc = gf32_mul(acc, last ? a.mono_last : a.mono_bpc, a.poly) ^ v;
    len += last ? a.last_len : a.bpc;
  }
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    const uint32_t oacc = static_cast<uint32_t>(__shfl_down(static_cast<int>(acc), 1 << m, 64));
    const int64_t olen = __shfl_down(len, 1 << m, 64);
    if ((lane & ((2 << m) - 1)) == 0 && olen > 0) {
      acc = gf32_mul(acc, gf32_monomial(olen, a.poly), a.poly) ^ oacc;
      len += olen;
    }
  }
  if (lane == 0) a.out[cell] = a.big_endian_out ? __builtin_bswap32(acc) : acc;
}

__global__ void finish_mismatch(int32_t *m, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n && m[i] == 0x7fffffff) m[i] = -1;
}

// ------------------------------------------------------------------------------------------------
// splitmix64 fill (bench / test data), twin of tests/golden/synth.py

__global__ __launch_bounds__(kBlock) void fill_splitmix64(uint8_t *base, int64_t cell_stride, int64_t ncells,
                                                          int64_t n, uint64_t seed, uint64_t first_stream) {
  const int64_t words = (n + 7) >> 3;
  const int64_t total = words * ncells;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t c = i / words;
    const int64_t wi = i - c * words;
    const uint64_t state0 = seed ^ ((first_stream + static_cast<uint64_t>(c)) * 0x9E3779B97F4A7C15ull);
    uint64_t z = state0 + static_cast<uint64_t>(wi + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    uint8_t *dst = base + c * cell_stride + wi * 8;
    const int64_t nb = n - wi * 8 < 8 ? n - wi * 8 : 8;
    if (nb == 8 && (reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
      *reinterpret_cast<uint64_t *>(dst) = z;
    } else {
      for (int b = 0; b < nb; ++b) dst[b] = static_cast<uint8_t>(z >> (8 * b));
    }
  }
}

// WIDE instantiations: up to 18 coefficients (rs-3-x, rs-6-x, rs-10-1); rs-10-2..4 spilled 16-97 VGPRs in that form
// and keep the typed-pointer kernel (aligned) or the byte kernel (odd offsets) for units 2 GiB apart
constexpr int kWideMaxKR = 18;

template <int K, int R, int VPT, int LAUX, int SAUX, int OPT = 0, bool WIDE = false>
hipError_t launch_krv(const CodeArgs &a, hipStream_t st, int64_t default_grid) {
  constexpr bool kSreg = K * R <= 18 && !WIDE;
  const uint32_t nvec = static_cast<uint32_t>(a.len >> 4);
  const int64_t units = a.nstripes * ((nvec + kBlock * VPT - 1) / (kBlock * VPT));
  const TabArgs<K * R> tabs = host_tabs<K * R>(a);
  const int64_t tg = g_tune.grid;
  int64_t grid = tg > 0 ? tg : t_grid_cap > 0 ? std::min(t_grid_cap, default_grid) : default_grid;
  grid = std::max<int64_t>(1, std::min<int64_t>(grid, units));
  hipLaunchKernelGGL((gf_code_vec<K, R, kSreg, VPT, LAUX, SAUX, OPT, WIDE>), dim3(static_cast<unsigned>(grid)), dim3(kBlock),
                     0, st, a, tabs);
  return hipGetLastError();
}

// Defaults measured on MI355X (scripts/tune.py, scripts/tune_all.py, profiles/r01/tune_*.log): one 4 KiB chunk
// per block on a non-persistent grid (XCD-contiguous block order, xcd_remap) with non-temporal loads and stores,
// for register-table and LDS-table kernels alike (C2 77.9 %, C3 77.9 % of the HBM roofline).
// ozec_set_tuning("gf_variant", v) pins an alternate for A/B (kernels.hpp kGfVariants): 1 plain (cached) loads and
// stores, 5 two 16-B vectors per lane per unit (8 KiB chunks, 8192 blocks), 11 parity in three-input XOR chains
// (-6.5 % VALU, no faster: profiles/r02/gf/ab_gf_variants.log).  (The other cache-policy and selector-mask variants of
// rounds 1-2 were taken out of the library.)
template <int K, int R>
hipError_t launch_kr(const CodeArgs &a, hipStream_t st) {
  constexpr int64_t kAll = int64_t{1} << 40;
  switch (g_tune.gf_variant.load(std::memory_order_relaxed)) {
    case 1: return launch_krv<K, R, 1, 0, 0>(a, st, kAll);
    case 5: return launch_krv<K, R, 2, 0, 0>(a, st, 8192);
    case 11: return launch_krv<K, R, 1, 2, 2, 1>(a, st, kAll);
    default: break;
  }
  return launch_krv<K, R, 1, 2, 2>(a, st, kAll);
}

// grid_for with the thread's zero-copy cap (t_grid_cap) applied
inline unsigned capped_grid(int64_t units) {
  const unsigned g = grid_for(units, 1);
  return t_grid_cap > 0 && static_cast<int64_t>(g) > t_grid_cap ? static_cast<unsigned>(t_grid_cap) : g;
}

template <int K>
hipError_t launch_xor(const CodeArgs &a, hipStream_t st, bool buf) {
  const uint32_t nvec = static_cast<uint32_t>(a.len >> 4);
  const int64_t units = a.nstripes * ((nvec + kBlock - 1) / kBlock);
  if (buf) {
    hipLaunchKernelGGL((xor_vec<K, true>), dim3(capped_grid(units)), dim3(kBlock), 0, st, a);
  } else {
    hipLaunchKernelGGL((xor_vec<K>), dim3(capped_grid(units)), dim3(kBlock), 0, st, a);
  }
  return hipGetLastError();
}

// aligned layouts keep the typed-pointer kernels measured in rounds 1-4; any other layout whose offsets fit a
// 32-bit buffer offset after rebase32 runs the BUF instantiations (launch_code checks which applies)
hipError_t launch_vec(const CodeArgs &a, hipStream_t st) {
  CodeArgs rb = a;
  const bool fits32 = rebase32(rb);
  const bool buf = fits32 && !vec_ok(a);  // BUF needs 32-bit offsets; the typed kernels (align-1 copies) take any
  const CodeArgs &x = buf ? rb : a;
  if (a.all_ones && a.rows == 1) {
    switch (a.k) {
      case 2: return launch_xor<2>(x, st, buf);
      case 3: return launch_xor<3>(x, st, buf);
      case 4: return launch_xor<4>(x, st, buf);
      case 6: return launch_xor<6>(x, st, buf);
      case 10: return launch_xor<10>(x, st, buf);
      default: return launch_xor<0>(x, st, buf);
    }
  }
#define OZEC_KR(KK, RR)                                                                                           \
  if (a.k == KK && a.rows == RR) {                                                                                  \
    if (fits32) return launch_kr<KK, RR>(rb, st);                                                                   \
    if constexpr (KK * RR <= kWideMaxKR)                                                                           \
      if (a.len < (int64_t{1} << 31)) return launch_krv<KK, RR, 1, 2, 2, 0, true>(a, st, int64_t{1} << 40);         \
  }
  OZEC_KR(3, 1) OZEC_KR(3, 2)
  OZEC_KR(6, 1) OZEC_KR(6, 2) OZEC_KR(6, 3)
  OZEC_KR(10, 1) OZEC_KR(10, 2) OZEC_KR(10, 3) OZEC_KR(10, 4)
#undef OZEC_KR
  const uint32_t nvec = static_cast<uint32_t>(a.len >> 4);
  const int64_t units = a.nstripes * ((nvec + kBlock - 1) / kBlock);
  const unsigned grid = capped_grid(units);
  for (int row0 = 0; row0 < a.rows; row0 += 4) {
    const int rr = a.rows - row0 < 4 ? a.rows - row0 : 4;
    if (buf) {
      switch (rr) {
        case 1: hipLaunchKernelGGL((gf_code_vec_generic<1, true>), dim3(grid), dim3(kBlock), 0, st, x, row0); break;
        case 2: hipLaunchKernelGGL((gf_code_vec_generic<2, true>), dim3(grid), dim3(kBlock), 0, st, x, row0); break;
        case 3: hipLaunchKernelGGL((gf_code_vec_generic<3, true>), dim3(grid), dim3(kBlock), 0, st, x, row0); break;
        default: hipLaunchKernelGGL((gf_code_vec_generic<4, true>), dim3(grid), dim3(kBlock), 0, st, x, row0); break;
      }
    } else {
      switch (rr) {
        case 1: hipLaunchKernelGGL(gf_code_vec_generic<1>, dim3(grid), dim3(kBlock), 0, st, a, row0); break;
        case 2: hipLaunchKernelGGL(gf_code_vec_generic<2>, dim3(grid), dim3(kBlock), 0, st, a, row0); break;
        case 3: hipLaunchKernelGGL(gf_code_vec_generic<3>, dim3(grid), dim3(kBlock), 0, st, a, row0); break;
        default: hipLaunchKernelGGL(gf_code_vec_generic<4>, dim3(grid), dim3(kBlock), 0, st, a, row0); break;
      }
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

}  // namespace

hipError_t launch_code(const CodeArgs &a, hipStream_t st) {
  if (a.len <= 0 || a.nstripes <= 0) return hipSuccess;
  int64_t start = 0;
  // every layout runs the 16-B vector kernels (round 5): buffer descriptors at any byte offset while the unit offsets
  // fit 32 bits, gf_code_vec's WIDE form or the typed kernels' align-1 copies beyond (a packed batch of odd-length
  // cells ran gf_code_bytes at ~5 GB/s, profiles/r05/small/); the byte kernel takes the last 1-15 bytes of a cell
  if (a.len >= 16) {
    hipError_t err = launch_vec(a, st);
    if (err != hipSuccess) return err;
    start = a.len & ~static_cast<int64_t>(15);
  }
  if (start < a.len) {
    const int64_t total = (a.len - start) * a.nstripes;
    hipLaunchKernelGGL(gf_code_bytes, dim3(grid_for(total, kBlock)), dim3(kBlock), 0, st, a, start);
    return hipGetLastError();
  }
  return hipSuccess;
}

namespace {

// Windows per wave of the streaming kernels: runs of about crc_run bytes (256 KiB: measured best against
// persistent grids and one-window runs, profiles/r01/session3/tune_grid.log), or an even split over crc_grid
// blocks when that knob is set.  The grid is not persistent: blocks start in order, so the waves in flight
// stream neighbouring stretches of HBM.
int64_t stream_per_wave(int64_t total, int64_t bpc) {
  const int64_t cg = g_tune.crc_grid, cr = g_tune.crc_run;
  if (cg > 0) {
    const int64_t waves = std::max<int64_t>(1, std::min<int64_t>(cg * (kBlock / 64), total));
    return (total + waves - 1) / waves;
  }
  const int64_t run = cr > 0 ? cr : int64_t{256} << 10;
  // a small batch (one stripe's cells through the unfused path: tens of windows) is spread over at least ~2048 waves
  // instead of a handful of 256 KiB runs; batches of 32 Ki windows and more keep the tuned run length
  return std::max<int64_t>(1, std::min(run / bpc, total / 2048));
}

int64_t stream_grid(int64_t total, int64_t per_wave) {
  return ((total + per_wave - 1) / per_wave + (kBlock / 64) - 1) / (kBlock / 64);
}

// Full windows of every cell through the streaming kernel, the short last window of each cell (len % bpc)
// through the per-window kernel.
template <int D, int NS, bool XO = false, bool VR = false, int TB = 1>
hipError_t launch_crc_stream(const CrcArgs &a, hipStream_t st) {
  const int64_t nfull = a.len / a.bpc;
  const int64_t total = a.ncells * nfull;
  if (total > 0) {
    const int64_t per_wave = stream_per_wave(total, a.bpc);
    hipLaunchKernelGGL((crc_windows_g26s<D, NS, XO, VR, TB>), dim3(static_cast<unsigned>(stream_grid(total, per_wave))),
                       dim3(kBlock), 0, st, a, nfull, per_wave);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
  }
  if (nfull < a.nwin) {
    CrcArgs t = a;
    const int64_t off = nfull * a.bpc;
    t.base = a.base + off;
    t.len = a.len - off;
    t.nwin = 1;
    if (a.out) t.out = a.out + nfull;
    if (a.expected) t.expected = a.expected + nfull;
    t.mismatch_base = a.mismatch_base + static_cast<int32_t>(nfull);
    const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(16384, (a.ncells + 3) / 4))));
    hipLaunchKernelGGL((crc_windows_g26<1, 4, 2>), grid, dim3(kBlock), 0, st, t);
    return hipGetLastError();
  }
  return hipSuccess;
}

}  // namespace

hipError_t launch_crc_windows(const CrcArgs &a, hipStream_t st) {
  const int64_t units = a.ncells * a.nwin;
  if (units <= 0) return hipSuccess;
  const bool vec = aligned16(reinterpret_cast<intptr_t>(a.base)) && (a.ncells == 1 || aligned16(a.cell_stride)) &&
                   aligned16(a.bpc);
  if (vec) {
    const int v = g_tune.crc_variant.load(std::memory_order_relaxed);
    // streaming kernel for windows of whole 4 KiB groups, (D, ring) = (4, 2) with free register shifts (XO): CRC32C
    // 78.5 -> 80.3 %, verify 77.8 -> 80.3 % in same-process A/Bs (profiles/r03/ab/crcxo_*.log) against the D-step
    // groups of rounds 1-2, which variants 20 (ring of 2) and 22 (ring of 4, the round-2 default) keep for A/B
    if (a.bpc % 4096 == 0) {
      if (v == 20) return launch_crc_stream<4, 2>(a, st);
      if (v == 22) return launch_crc_stream<4, 4>(a, st);
      // verify with bpc = 4 KiB << i: a run of windows checked as one message (VR), window by window only when it
      // fails; 24 pins the window-by-window check (round 4's default)
      if (a.expected && a.bshift && v != 24) return launch_crc_stream<4, 2, true, true>(a, st);
      // compute: the lane trees of 8 consecutive windows at once (CRC32C 1.361 -> 1.285 ms for 8 GiB, 78.9 -> 83.6 %;
      // 4 windows 1.293 ms, profiles/r05/crc/); 28 one tree per window (round 4), 29 four windows
      if (!a.expected && v == 29) return launch_crc_stream<4, 2, true, false, 4>(a, st);
      if (!a.expected && v != 28) return launch_crc_stream<4, 2, true, false, 8>(a, st);
      return launch_crc_stream<4, 2, true>(a, st);
    }
    // per-window kernel: G26 tables, B = 1 block per lane per step, groups of D = 4 steps, two steps of loads in
    // flight, 16384 blocks (scripts/tune_crc.py)
    const int64_t cg = g_tune.crc_grid;
    const int64_t g = cg > 0 ? cg : 16384;
    const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(g, (units + 3) / 4)))), block(kBlock);
    hipLaunchKernelGGL((crc_windows_g26<1, 4, 2>), grid, block, 0, st, a);
  } else {
    // cells at unaligned offsets (a packed batch of odd-length cells) and windows of any length (bpc not a multiple of
    // 16: every window starts at its own byte offset): the per-window kernel with align-1 loads, each window's last
    // 1-15 bytes folded bytewise after the lane tree.  (Until round 5 these ran a byte-at-a-time kernel, one thread
    // per window.)
    const int64_t cg = g_tune.crc_grid;
    const int64_t g = cg > 0 ? cg : 16384;
    const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(g, (units + 3) / 4)))), block(kBlock);
    hipLaunchKernelGGL((crc_windows_g26<1, 4, 2, true>), grid, block, 0, st, a);
  }
  return hipGetLastError();
}

namespace {

template <int K, int D, int NS>
hipError_t launch_xor_stream(const EncCrcArgs &e, hipStream_t st) {
  const int64_t total = e.code.nstripes * e.crc.nwin;
  const int64_t per_wave = stream_per_wave(total, e.crc.bpc);
  hipLaunchKernelGGL((encode_xor_crc_g26s<K, D, NS>), dim3(static_cast<unsigned>(stream_grid(total, per_wave))),
                     dim3(kBlock), 0, st, e, per_wave);
  return hipGetLastError();
}

template <int K, int R>
hipError_t launch_enc_crc_kr(const EncCrcArgs &e, hipStream_t st, bool wide = false) {
  const int64_t units = e.code.nstripes * e.crc.nwin;
  const TabArgs<K * R> tabs = host_tabs<K * R>(e.code);
  // defaults measured on MI355X (scripts/tune_crc.py, profiles/r01/session2/tune_g26*.log): one wave per window
  // with no grid-stride, G26 tables in groups of D = 2 steps, coefficient tables {lo0,lo1,mid0,mid1} by one
  // ds_read_b128 broadcast and `top` as an SGPR operand (all from LDS past 18 coefficients: SGPR budget)
  const int64_t cg = g_tune.crc_grid;
  const int64_t g = cg > 0 ? cg : (units + 3) / 4;
  const dim3 grid(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(g, (units + 3) / 4)))), block(kBlock);
  constexpr int kTM = K * R <= 18 ? 1 : 3;
  constexpr int kW = K + R >= 12 ? 3 : 4;  // rs-10-x: 14 unit registers and operands do not fit 128 VGPRs
  const int v = g_tune.crc_variant.load(std::memory_order_relaxed);
  if constexpr (R == 1 && K <= 6) {
    // XOR codec, every window full: the streaming kernel, for A/B only (variants 20 / 21: ring of 2 / 4 steps).
    // On C4 it reaches 62-71 % of the HBM roofline against 72-73 % for the per-window kernel below at every grid
    // and run length tried (profiles/r01/session3/tune_grid.log).
    if (e.code.all_ones && !e.verify && (v == 20 || v == 21) && e.code.len % e.crc.bpc == 0 &&
        e.crc.bpc % 4096 == 0) {
      if (v == 20) return launch_xor_stream<K, 4, 2>(e, st);
      return launch_xor_stream<K, 4, K <= 3 ? 4 : 2>(e, st);
    }
  }
  if constexpr (R == 1) {
    if (wide && e.code.all_ones) {  // units 2 GiB or more apart (WIDE; TAIL for any length)
      if (aligned16(e.code.len))
        hipLaunchKernelGGL((encode_crc_g26<K, R, 2, true, 1, 4, false, false, false, false, true>), grid, block, 0, st, e,
                           tabs);
      else
        hipLaunchKernelGGL((encode_crc_g26<K, R, 2, true, 1, 4, false, false, false, true, true>), grid, block, 0, st, e,
                           tabs);
      return hipGetLastError();
    }
    if (e.code.all_ones && (!aligned16(e.code.len) || !vec_ok(e.code))) {  // any length, any byte offset (TAIL)
      hipLaunchKernelGGL((encode_crc_g26<K, R, 2, true, 1, 4, false, false, false, true>), grid, block, 0, st, e, tabs);
      return hipGetLastError();
    }
    if (e.code.all_ones && v != 2) {
      // XOR codec: groups of D = 2 steps, loads issued at the step (45 VGPRs for xor-2-1, 8 waves per SIMD).  Round 1
      // chose D = 4 with the next step's loads in flight (67 VGPRs; variant 3 now): C4 77.9 % vs 75.8 % then
      // (profiles/r01/session2/ab_c4.log); on the round-4 build D = 2 is 1.0-1.8 % faster in 4 same-process A/Bs on
      // two boxes (profiles/r04/c4/ab_c4_*.log).  On a persistent WorkQueue grid either runs 10-12 % slower
      // (ab_c4_persistent_*.log; not kept)
      if (v == 3) hipLaunchKernelGGL((encode_crc_g26<K, R, 4, true, 1, 4, true>), grid, block, 0, st, e, tabs);
      else if (v == 4)  // free register shifts (XO)
        hipLaunchKernelGGL((encode_crc_g26<K, R, 4, true, 1, 4, true, false, true>), grid, block, 0, st, e, tabs);
      else if (v == 5)
        hipLaunchKernelGGL((encode_crc_g26<K, R, 2, true, 1, 4, true, false, true>), grid, block, 0, st, e, tabs);
      else hipLaunchKernelGGL((encode_crc_g26<K, R, 2, true, 1>), grid, block, 0, st, e, tabs);
      return hipGetLastError();
    }
  }
  // per-window kernel (variant 49 pins it for the RS shapes the nibble kernel also takes): CRC lookups of a block in
  // two fenced halves; groups of D = 4 steps for rs-6-3 (123 VGPRs, 0 spilled), D = 2 where 14 unit registers and
  // their operands must fit 128 VGPRs (profiles/r01/session4/ab_c5*.log; the other round-1 geometries, 11-17, were
  // slower and are gone)
  if constexpr (K == 6 && R == 3) hipLaunchKernelGGL((encode_crc_g26<K, R, 4, false, kTM, 4, false, true>), grid, block, 0, st, e, tabs);
  else hipLaunchKernelGGL((encode_crc_g26<K, R, 2, false, kTM, kW>), grid, block, 0, st, e, tabs);
  return hipGetLastError();
}

#define OZEC_FUSED_SHAPES(X) X(6, 3) X(6, 2) X(6, 1) X(3, 2) X(3, 1) X(10, 4) X(10, 3) X(10, 2) X(10, 1) X(2, 1)

}  // namespace

bool encode_crc_supported(const CodeArgs &a, int64_t bpc) {
  bool kr = false;
#define OZEC_SHAPE_OK(KK, RR) kr |= (a.k == KK && a.rows == RR);
  OZEC_FUSED_SHAPES(OZEC_SHAPE_OK)
#undef OZEC_SHAPE_OK
  CodeArgs rb = a;
  if (!kr || bpc <= 0 || !aligned16(bpc)) return false;
  if (!rebase32(rb))  // units 2 GiB or more apart: the WIDE forms, one buffer descriptor per unit (round 6)
    return a.len < (int64_t{1} << 31) && (encode_crc_nb_bytes_supported(a, bpc) || (a.all_ones && a.rows == 1));
  // the XOR codec's per-window kernel takes any length and byte offset (encode_crc_g26 TAIL, round 6)
  return (aligned16(a.len) && vec_ok(a)) || encode_crc_nb_bytes_supported(a, bpc) || (a.all_ones && a.rows == 1);
}

bool encode_crc_fused_pays(const CodeArgs &a, int64_t nwin, int64_t min_units) {
  // units at unaligned offsets: the unfused kernels of the nibble shapes take them at full rate too since round 5
  // (gf_code_vec through buffer descriptors, crc_windows_g26 with align-1 loads; before, their byte paths ran 7-8x
  // slower, profiles/r05/small/small_batch_ab_first.json)
  return a.nstripes * nwin >= min_units;
}

hipError_t launch_encode_crc(const EncCrcArgs &e0, hipStream_t st) {
  if (e0.code.nstripes * e0.crc.nwin <= 0) return hipSuccess;
  EncCrcArgs e = e0;
  if (!rebase32(e.code)) {  // units 2 GiB or more apart: one buffer descriptor per unit (WIDE, round 6)
    if (e0.code.len >= (int64_t{1} << 31)) return hipErrorInvalidValue;
    const int k = e0.code.k, r = e0.code.rows;
    if (e0.code.all_ones && r == 1) {
      if (k == 2) return launch_enc_crc_kr<2, 1>(e0, st, true);
      if (k == 3) return launch_enc_crc_kr<3, 1>(e0, st, true);
      if (k == 6) return launch_enc_crc_kr<6, 1>(e0, st, true);
      if (k == 10) return launch_enc_crc_kr<10, 1>(e0, st, true);
      return hipErrorInvalidValue;
    }
    if (!encode_crc_nb_bytes_supported(e0.code, e0.crc.bpc)) return hipErrorInvalidValue;
    return launch_encode_crc_lv(e0, st, 0, !aligned16(e0.code.len), true);
  }
  // the RS shapes with whole windows and a short last window of any whole number of blocks: the nibble-table kernel
  // (fused_nb.hpp); 56 / 59 the streamed-input kernel (full windows only); variant 49 pins the per-window kernel
  const int v = g_tune.crc_variant.load(std::memory_order_relaxed);
  if (!aligned16(e.code.len) || !vec_ok(e.code)) {
    // byte-granular cells (a key's last stripe, odd unit strides): the nibble kernel's TAIL instantiations (nb_tail);
    // a pinned variant without one falls back to the default.  The XOR codec: its per-window kernel's TAIL form
    if (!(e.code.all_ones && e.code.rows == 1)) {
      if (!encode_crc_nb_bytes_supported(e.code, e.crc.bpc)) return hipErrorInvalidValue;
      return launch_encode_crc_lv(e, st, v, true);
    }
  }
  if (v == 0 || (v >= 50 && v < 300)) {
    const bool lv = v == 56 || v == 59;
    if (lv ? encode_crc_lv_supported(e) : encode_crc_nb_supported(e)) return launch_encode_crc_lv(e, st, v);
  }
  const int k = e.code.k, r = e.code.rows;
#define OZEC_SHAPE_LAUNCH(KK, RR) \
  if (k == KK && r == RR) return launch_enc_crc_kr<KK, RR>(e, st);
  OZEC_FUSED_SHAPES(OZEC_SHAPE_LAUNCH)
#undef OZEC_SHAPE_LAUNCH
  return hipErrorInvalidValue;
}

hipError_t launch_compose_windows(const ComposeArgs &a, hipStream_t st) {
  if (a.ncells <= 0) return hipSuccess;
  hipLaunchKernelGGL(compose_windows, dim3(static_cast<unsigned>((a.ncells + kBlock / 64 - 1) / (kBlock / 64))),
                     dim3(kBlock), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_finish_mismatch(int32_t *d_mismatch, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(finish_mismatch, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, st, d_mismatch, n);
  return hipGetLastError();
}

hipError_t launch_fill_splitmix64(uint8_t *base, int64_t cell_stride, int64_t ncells, int64_t n, uint64_t seed,
                                  uint64_t first_stream, hipStream_t st) {
  const int64_t total = ((n + 7) >> 3) * ncells;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_splitmix64, dim3(grid_for(total, kBlock)), dim3(kBlock), 0, st, base, cell_stride, ncells,
                     n, seed, first_stream);
  return hipGetLastError();
}

}  // namespace ozec
