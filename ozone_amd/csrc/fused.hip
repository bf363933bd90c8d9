// Fused encode (or reconstruct) + CRC for full windows: encode_crc_nb (nibble tables, the default, further below) and
// encode_crc_lv ("streamed inputs", variants 50-59), described here first.
//
// The per-window fused kernel in kernels.hip (encode_crc_g26) loads all K input blocks of a step at once and
// keeps every input, every parity accumulator and the coefficient tables of the step live together: 123 VGPRs
// for rs-6-3 (4 waves per SIMD) and 160 for rs-10-4 reconstruction (3 waves).  Its time is VALU + LDS issue
// (DESIGN §2.3), and on gfx950 the VALU issue rate of a SIMD grows with the waves it can pick from (integer ops
// at 4 waves: 2.2-3.4 cycles per wave-instruction, at 8 waves 1.6-2.7; profiles/r01/session4/valu_rate.log).
//
// This kernel does the same arithmetic per 16-B block with a live set of about half that size, so the SIMDs get
// 5-8 waves:
//   * inputs stream through a ring of NB block registers: input j of step t is consumed (its CRC, then its GF
//     contributions to the R parity accumulators) while the loads of the next NB - 1 (step, input) slots are in
//     flight; one input block is live at a time, not K (the look-ahead past a window's end reads nothing: it is
//     addressed outside the input descriptor's range, and out-of-range buffer loads return zeros without a memory
//     access);
//   * the GF tables of a coefficient come from LDS as one ds_read_b128 broadcast ({lo0, lo1, mid0, mid1}) plus one
//     ds_read_b128 holding the `top` tables of input j for all R outputs -- nothing from the kernarg segment, so
//     no SGPR spills into VGPR lanes;
//   * parity dwords accumulate in three-input XOR chains (1.5 VALU per coefficient and dword) across the K inputs.
// Windows must be full (len % bpc == 0) and a whole number of D-step groups (bpc % (1024 D) == 0): no virtual
// blocks, so loads and stores are unconditional (a per-lane predicate makes the compiler wait for every load in
// flight at every step).  The load cursor runs NB - 1 slots ahead of the compute cursor.
//
// Same results as encode_crc_g26 bit for bit (same G26 tables, same per-lane folding, same lane tree); the
// launcher (launch_encode_crc) picks this kernel for the shapes and geometries above and falls back otherwise.
#include "fused_nb.hpp"

namespace ozec {
namespace {

__device__ __forceinline__ uint32_t and_v(uint32_t a, uint32_t m) {
  uint32_t d;
  asm("v_and_b32 %0, %1, %2" : "=v"(d) : "v"(m), "v"(a));
  return d;
}

// K inputs, R outputs, D steps per CRC group, NB ring slots, WPB waves per block, WAVES minimum waves per SIMD,
// ACC: parity dwords in plain accumulators (1 VGPR, 2 VALU per coefficient and dword) instead of XOR chains
// (2 VGPRs, 1.5 VALU); OPT bit 0: all 12 permutes of a coefficient before their XORs (no consumer right behind its
// producer: gfx950 pads v_perm -> v_bitop3 back-to-back with s_nop), bit 1: GF selector masks held in VGPRs
// (plain VOP2 AND instead of the literal-operand form)
template <int K, int R, int D, int NB, int WPB, int WAVES, bool ACC = false, int OPT = 0>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(WAVES, 8))) void encode_crc_lv(
    const EncCrcArgs e) {
  static_assert(R >= 1 && R <= 4, "the packed top tables hold up to 4 outputs");
  static_assert((D * K) % NB == 0, "the ring must divide the unrolled group so ring indices are compile-time");
  __shared__ __attribute__((aligned(16))) uint32_t s_t[g26_words(D)];
  __shared__ __attribute__((aligned(16))) uint4 s_q[K * R];  // {lo0, lo1, mid0, mid1} of coefficient r*K + j
  __shared__ __attribute__((aligned(16))) uint4 s_top[K];    // top tables of input j for outputs 0..3
  const CodeArgs &a = e.code;
  const CrcArgs &cr = e.crc;
  load_tables(s_t, cr.g26[g26_slot(1, D)], g26_words(D));
  for (int t = threadIdx.x; t < K * R; t += blockDim.x) {
    const PermTab p = make_tab(a.coef[t]);
    s_q[t] = make_uint4(p.lo0, p.lo1, p.mid0, p.mid1);
  }
  for (int j = threadIdx.x; j < K; j += blockDim.x) {
    uint32_t tp[4] = {0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < R; ++r) tp[r] = make_tab(a.coef[r * K + j]).top;
    s_top[j] = make_uint4(tp[0], tp[1], tp[2], tp[3]);
  }
  __syncthreads();

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t nwin = cr.nwin;
  const int64_t units = a.nstripes * nwin;
  const int32_t T = static_cast<int32_t>(cr.bpc >> 10);  // steps per window
  const int32_t G = T / D;                                // groups per window
  const uint32_t voff = static_cast<uint32_t>(lane) * 16u;
  uint32_t m7 = 0x07070707u, m3 = 0x03030303u;
  if constexpr (OPT & 2) {  // materialised once, live in VGPRs
    asm volatile("v_mov_b32 %0, 0x7070707" : "=v"(m7));
    asm volatile("v_mov_b32 %0, 0x3030303" : "=v"(m3));
  }
  int64_t off_max = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) off_max = a.in_off[j] > off_max ? a.in_off[j] : off_max;
  const uint32_t in_extent = static_cast<uint32_t>(off_max + cr.bpc);
  const uint32_t out_extent = unit_extent<R>(a.out_off, cr.bpc);
  const int64_t bid = a.unit_map == 1 ? blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
  for (int64_t u = bid * WPB + wave; u < units; u += static_cast<int64_t>(gridDim.x) * WPB) {
    const int64_t s = u / nwin;
    const int64_t w = u - s * nwin;
    // the input descriptor's range ends with the last unit's window (rebase32: in_off + bpc < 2^31); the look-ahead
    // loads past the window's last step get voffset + 2^31, outside the range: they return zeros and cost no
    // memory traffic (no 32-bit wrap: 2^31 + 1008 + in_off < 2^32)
    const __amdgpu_buffer_rsrc_t rin = make_rsrc_n(a.in + in_off(a, s) + w * cr.bpc, in_extent);
    const __amdgpu_buffer_rsrc_t rout = make_rsrc_n(a.out + out_off(a, s) + w * cr.bpc, out_extent);
    // step part of the address in a VGPR (one add per step), unit offset in soffset: K SGPRs in all, instead of
    // one SGPR per (step, unit) slot of the unrolled group
    auto vstep = [&](int32_t t) { return voff + (t < T ? static_cast<uint32_t>(t) * 1024u : 0x80000000u); };
    auto load = [&](uint32_t vo, int j) {
      const auto d = __builtin_amdgcn_raw_buffer_load_b128(rin, vo, static_cast<int>(a.in_off[j]), 2);
      return make_uint4(d[0], d[1], d[2], d[3]);
    };
    uint32_t S[K + R];
#pragma unroll
    for (int q = 0; q < K + R; ++q) S[q] = 0;
    uint4 ring[NB];
#pragma unroll
    for (int i = 0; i + 1 < NB; ++i) ring[i] = load(vstep(i / K), i % K);
    for (int32_t g = 0; g < G; ++g) {
#pragma unroll
      for (int rr = 0; rr < D; ++rr) {
        const int32_t t = g * D + rr;
        const uint32_t *tab = s_t + (D - 1 - rr) * kG26Set;
        const uint32_t vcur = vstep(t), vnext = vstep(t + 1);
        XorChain ch[R][4];
        uint32_t acc[R][4];
        if constexpr (ACC) {
#pragma unroll
          for (int r = 0; r < R; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[r][c] = 0;
        }
#pragma unroll
        for (int j = 0; j < K; ++j) {
          const int ii = rr * K + j;  // slot within the group
          const int ahead = ii + NB - 1;
          static_assert(NB - 1 <= K, "look-ahead of at most one step");
          ring[ahead % NB] = load(ahead / K == rr ? vcur : vnext, ahead % K);
          const uint4 x = ring[ii % NB];
          asm volatile("" ::: "memory");  // keep this input's LDS table reads here
          S[j] ^= g26_block<true>(tab, x);
          __builtin_amdgcn_sched_barrier(0);
          const uint32_t xw[4] = {x.x, x.y, x.z, x.w};
          Sel sl[4];
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if constexpr (OPT & 2) {
              sl[c].s0 = and_v(xw[c], m7);
              sl[c].s1 = and_v(xw[c] >> 3, m7);
              sl[c].s2 = and_v(xw[c] >> 6, m3);
            } else {
              sl[c] = make_sel(xw[c]);
            }
          }
          const uint4 tops = s_top[j];
          const uint32_t top[4] = {tops.x, tops.y, tops.z, tops.w};
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const uint4 q = s_q[r * K + j];
            if constexpr ((OPT & 1) && !ACC) {
              uint32_t pp[4][3];
#pragma unroll
              for (int c = 0; c < 4; ++c) {
                pp[c][0] = perm_vv(q.y, q.x, sl[c].s0);
                pp[c][1] = perm_vv(q.w, q.z, sl[c].s1);
                pp[c][2] = perm_vv(top[r], top[r], sl[c].s2);
              }
#pragma unroll
              for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int i = 0; i < 3; ++i) ch[r][c].push(pp[c][i]);
              continue;
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const uint32_t plo = perm_vv(q.y, q.x, sl[c].s0), pmid = perm_vv(q.w, q.z, sl[c].s1),
                             ptop = perm_vv(top[r], top[r], sl[c].s2);
              if constexpr (ACC) {
                acc[r][c] = xor3(acc[r][c], plo, pmid) ^ ptop;
              } else {
                ch[r][c].push(plo);
                ch[r][c].push(pmid);
                ch[r][c].push(ptop);
              }
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint4 p = ACC ? make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3])
                              : make_uint4(ch[r][0].get(), ch[r][1].get(), ch[r][2].get(), ch[r][3].get());
          __attribute__((ext_vector_type(4))) unsigned int d = {p.x, p.y, p.z, p.w};
          __builtin_amdgcn_raw_buffer_store_b128(d, rout, vcur, static_cast<int>(a.out_off[r]), 2);
          store_data_hold(p);
          S[K + r] ^= g26_block<true>(tab, p);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (g + 1 < G) {
#pragma unroll
        for (int q = 0; q < K + R; ++q) S[q] = g5_shift(s_t + g26_gshift(D), S[q]);
      }
    }
    const bool last = w == nwin - 1;
    const uint32_t init = last ? cr.init_last : cr.init_full;
#pragma unroll
    for (int q = 0; q < K + R; ++q) {
      const uint32_t v = g5_lane_tree(s_t + g26_tree(D) - kG5Tree, S[q], lane);
      if (lane == q) {
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
    }
  }
}

template <int K, int R, int D, int NB, int WPB, int WAVES, bool ACC = false, int OPT = 0>
hipError_t launch_lv(const EncCrcArgs &e, hipStream_t st) {
  if constexpr ((D * K) % NB != 0) {
    return launch_lv<K, R, D, 2, WPB, WAVES, ACC, OPT>(e, st);  // ring must divide the unrolled group
  } else {
    const int64_t units = e.code.nstripes * e.crc.nwin;
    const int64_t blocks = (units + WPB - 1) / WPB;
    const int64_t g = g_tune.crc_grid > 0 ? std::min<int64_t>(g_tune.crc_grid, blocks) : blocks;
    hipLaunchKernelGGL((encode_crc_lv<K, R, D, NB, WPB, WAVES, ACC, OPT>),
                       dim3(static_cast<unsigned>(std::max<int64_t>(1, g))), dim3(WPB * 64), 0, st, e);
    return hipGetLastError();
  }
}

// variant (g_tune.crc_variant): the streamed-input kernel's measured defaults, kept for A/B against the nibble kernel
// (profiles/r02/lv/ab_variants_lv3.log, ab_opt_lv5.log): 56 = groups of D = 4 steps, ring of 4 input blocks, 5 waves
// per SIMD (the rs-10-x form, 95 VGPRs), permutes before their XORs; 59 = ring of 2 at 6 waves (the rs-6-x form, 76
// VGPRs), permutes first and selector masks in VGPRs.  (Variants 50-58 were taken out of the library.)
template <int K, int R>
hipError_t launch_lv_kr(const EncCrcArgs &e, hipStream_t st, int v) {
  if (v == 56) return launch_lv<K, R, 4, 4, 4, 5, false, 1>(e, st);
  if (v == 59) return launch_lv<K, R, 4, 2, 4, 6, false, 3>(e, st);
  return hipErrorInvalidValue;
}

}  // namespace

namespace {
// nb: the nibble kernel's shapes (also rs-6-x / rs-3-x with one output: single-unit reconstruction); else the
// streamed-input kernel's
bool fused_shape(const CodeArgs &a, bool nb) {
  if (a.all_ones && a.rows == 1) return false;  // the XOR codec has its own register shortcut (encode_crc_g26 XORC)
  return (a.k == 6 && (a.rows == 3 || a.rows == 2 || (nb && a.rows == 1))) ||
         (a.k == 10 && a.rows >= 1 && a.rows <= 4) || (a.k == 3 && (a.rows == 2 || (nb && a.rows == 1)));
}
}  // namespace

// After a CV variant (fused_nb.hpp): every stripe whose combined input check failed (mismatch == kMismatchSuspect) is
// checked again unit by unit, window by window, and gets the reference's first failing (unit, window); other stripes
// leave at once.  One block per stripe, one wave per (input, window): lane l folds blocks l, l+64, ... of the window
// (register shifted by the 1008-B gap to its next block, then XORed into that block's first dword -- a register
// followed by a block has the raw CRC of the block with the register in its first 4 bytes), the G5 lane tree merges
// the lanes.  (Round 5's first form ran one thread per (input, window) bytewise: a batch whose every stripe failed
// took 316 ms for 2048 rs-10-4 stripes instead of 5.6 ms, profiles/r05/reverify/.)
__global__ __launch_bounds__(256) void nb_reverify(const EncCrcArgs e) {
  __shared__ __attribute__((aligned(16))) uint32_t s_t[kG5Words];
  const CodeArgs &a = e.code;
  const CrcArgs &cr = e.crc;
  bool any = false;  // the common case: no stripe of this block is suspect -- leave before loading the tables
  for (int64_t s = blockIdx.x; s < a.nstripes && !any; s += gridDim.x) any = cr.mismatch[s] == kMismatchSuspect;
  if (!any) return;
  load_tables(s_t, cr.tables[0], kG5Words);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int waves = blockDim.x >> 6;
  const int64_t nwin = cr.nwin;
  for (int64_t s = blockIdx.x; s < a.nstripes; s += gridDim.x) {
    // every wave reads the mark before any wave can lower it (atomicMin below): the barrier keeps a fast wave's first
    // report from making a slower one skip the stripe
    const bool suspect = cr.mismatch[s] == kMismatchSuspect;
    __syncthreads();
    if (!suspect) continue;
    for (int64_t t = wave; t < a.k * nwin; t += waves) {
      const int j = static_cast<int>(t / nwin);
      const int64_t w = t - j * nwin;
      const bool last = w == nwin - 1;
      const int64_t n = last ? a.len - w * cr.bpc : cr.bpc;  // a multiple of 16 B (CV runs without TAIL)
      const int64_t m = n >> 4, steps = (m + 63) >> 6, pad = steps * 64 - m;
      const uint8_t *p = a.in + in_off(a, s) + a.in_off[j] + w * cr.bpc;
      uint32_t S = 0;
      for (int64_t q = 0; q < steps; ++q) {
        const int64_t vb = q * 64 + lane - pad;  // < 0: a virtual zero block in front of the window
        uint4 b = make_uint4(0, 0, 0, 0);
        if (vb >= 0) __builtin_memcpy(&b, p + vb * 16, 16);
        if (q > 0) S = g5_shift(s_t + kG5Step, S);
        b.x ^= S;
        S = g5_block(s_t, b);
      }
      S = g5_lane_tree(s_t, S, lane);
      if (lane == 0) {
        const uint32_t ex0 = cr.expected[(s * e.exp_units + e.in_unit[j]) * nwin + w];
        const uint32_t ex = cr.expected_be ? __builtin_bswap32(ex0) : ex0;
        if (crc_finish(S, last ? cr.init_last : cr.init_full, 0, 0) != ex)
          atomicMin(cr.mismatch + s, static_cast<int32_t>(e.in_unit[j] * nwin + w));
      }
    }
  }
}

bool encode_crc_lv_supported(const EncCrcArgs &e) {
  return fused_shape(e.code, false) && e.crc.bpc > 0 && e.crc.bpc % 4096 == 0 && e.code.len % e.crc.bpc == 0;
}

// the nibble kernel also takes a short last window of any whole number of 16-B blocks, front-padded with virtual zero
// blocks to whole step groups (fused_nb.hpp): cells of rs-3-2-1524k with 16 KiB windows end in a 4 KiB window
// (ECBlockChecksumComputer.java:160-166), the last stripe of a block group in a cell of any length
bool encode_crc_nb_supported(const EncCrcArgs &e) {
  return fused_shape(e.code, true) && e.crc.bpc > 0 && e.crc.bpc % 4096 == 0 && e.code.len > 0 && e.code.len % 16 == 0;
}

// cells of any length at any byte offsets (round 5): the nibble kernel's EM variants run the whole 16-B blocks of the
// last window as above and the last 1-15 bytes in nb_tail; gfx950 buffer accesses take unaligned offsets (probe:
// profiles/r05/unaligned/, unaligned 16-B loads at full rate)
bool encode_crc_nb_bytes_supported(const CodeArgs &a, int64_t bpc) {
  return fused_shape(a, true) && bpc > 0 && bpc % 4096 == 0 && a.len > 0;
}

namespace {

hipError_t launch_nb_shape(const EncCrcArgs &e, hipStream_t st, int v, bool tail, bool wide) {
  const int k = e.code.k, r = e.code.rows;
  if (k == 6 && r == 3) return launch_nb_6_3(e, st, v, tail, wide);
  if (k == 6 && r == 2) return launch_nb_6_2(e, st, v, tail, wide);
  if (k == 6 && r == 1) return launch_nb_6_1(e, st, v, tail, wide);
  if (k == 3 && r == 2) return launch_nb_3_2(e, st, v, tail, wide);
  if (k == 3 && r == 1) return launch_nb_3_1(e, st, v, tail, wide);
  if (k == 10 && r == 4) return launch_nb_10_4(e, st, v, tail, wide);
  if (k == 10 && r == 3) return launch_nb_10_3(e, st, v, tail, wide);
  if (k == 10 && r == 2) return launch_nb_10_2(e, st, v, tail, wide);
  if (k == 10 && r == 1) return launch_nb_10_1(e, st, v, tail, wide);
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_encode_crc_lv(const EncCrcArgs &e, hipStream_t st, int v, bool tail, bool wide) {
  const int k = e.code.k, r = e.code.rows;
  if (wide) {  // units 2 GiB or more apart: one descriptor per unit, the one geometry instantiated for it (fused_nb.hpp)
    (void)hipGetLastError();
    return launch_nb_shape(e, st, 0, tail, true);
  }
  if (!tail && (v == 56 || v == 59)) {
    if (k == 6 && r == 3) return launch_lv_kr<6, 3>(e, st, v);
    if (k == 6 && r == 2) return launch_lv_kr<6, 2>(e, st, v);
    if (k == 3 && r == 2) return launch_lv_kr<3, 2>(e, st, v);
    if (k == 10 && r == 4) return launch_lv_kr<10, 4>(e, st, v);
    if (k == 10 && r == 3) return launch_lv_kr<10, 3>(e, st, v);
    if (k == 10 && r == 2) return launch_lv_kr<10, 2>(e, st, v);
    if (k == 10 && r == 1) return launch_lv_kr<10, 1>(e, st, v);
    return hipErrorInvalidValue;
  }
  // default: the nibble-table kernel (same-process A/Bs on MI355X).  Round 2 (profiles/r02/nb/): rs-10-x with a ring
  // of 5 input blocks and one-step groups (62: C3r 62.9 %; encode_crc_lv 52.5 %), rs-6-x / rs-3-x with two-step
  // groups in 12-wave workgroups (87: C5dev 66.9 %; encode_crc_lv 57.9 %).  Round 3 (profiles/r03/ab/): the output
  // registers shift for free (XO), and the grid is persistent, fed by the WorkQueue -- rs-10-x 150 (62's geometry;
  // C3r 64.8 % vs 63.7 % for 102, 62.5 % for 62), rs-3-x 163 (two-step groups in 16-wave workgroups), rs-6-x 167 (163
  // with a ring of 3 input blocks; C5dev 68.4 % for 163 vs 67.2 % for 87 on one box); without a counter slot the same
  // kernels on a one-wave-per-window grid (173 / 174).  The window CRCs leave through one lane-parallel store /
  // compare (EM: 170 = 150, 171 = 167, 172 = 163 with it; C3r 5.711 -> 5.582 ms, C5dev 6.956 -> 6.911 ms,
  // profiles/r03/em/ab_*.log); rs-10-x takes two-step groups with the second distance set for half the inputs (177,
  // 0.5-1.3 % faster than 170 in three same-process A/Bs, profiles/r03/h/)
  WorkSlot *ws = e.code.nstripes * e.crc.nwin <= (int64_t{1} << 30) ? work_lease(st) : nullptr;
  if (tail && !nb_variant_tail(v)) v = 0;  // byte-granular cells: the TAIL instantiations of the EM variants
  // a small batch: workgroups of 4 waves spread its units over many CUs (the 16-wave persistent workgroups put them on
  // a few, whose LDS pipes then serve all their waves; kernels.hpp TuneKnobs::nb_small_units)
  if (v == 0 && e.code.nstripes * e.crc.nwin < g_tune.nb_small_units.load(std::memory_order_relaxed)) v = 222;
  // reconstructions that check stored CRCs: one combined input register (231, CV; nb_reverify after it).  Same-process
  // A/Bs (profiles/r05/cv/): C3r 5.86-5.88 -> 5.70-5.71 ms on one box, 5.62 -> 5.34 ms on another; rs-6-3 lose 1 / lose
  // 3 -2.5 / -2.2 %; rs-3-2 lose 1 even, so it keeps 172
  if (v == 0 && ws && !tail && e.verify && e.crc.expected && k >= 6) v = 231;
  if (v == 0) v = k == 10 ? (ws ? 177 : 173) : !ws ? 174 : k == 6 ? 171 : 172;
  const bool used = ws && nb_variant_persistent(v);
  EncCrcArgs ed = e;
  ed.work = used ? ws->ctr : nullptr;
  hipError_t err = launch_nb_shape(ed, st, v, tail, false);
  if (err == hipSuccess && !tail && nb_variant_cv(v) && e.verify && e.crc.expected) {
    const int64_t g = std::min<int64_t>(e.code.nstripes, 4096);
    hipLaunchKernelGGL(nb_reverify, dim3(static_cast<unsigned>(g)), dim3(256), 0, st, e);
    err = hipGetLastError();
  }
  // the event goes behind the launch whatever `err` says: an event behind a launch that never ran costs nothing, a
  // kernel left running without one would share its counters with the slot's next lease
  if (ws) work_return(ws, st, used);
  return err;
}

}  // namespace ozec
