#include "crc_host.hpp"

#include "kernels.hpp"

#include <utility>

namespace ozec {

int g26_bit(int g, int i);

namespace {

uint32_t mat_times(const uint32_t *mat, uint32_t v) {
  uint32_t r = 0;
  for (int c = 0; v; ++c, v >>= 1)
    if (v & 1) r ^= mat[c];
  return r;
}

void mat_square(const uint32_t *m, uint32_t *out) {
  for (int c = 0; c < 32; ++c) out[c] = mat_times(m, m[c]);
}

// inverse of the 32x32 GF(2) matrix given by its columns (Gauss-Jordan on [A | I]); the shift operators are
// invertible because x is a unit mod P (P(0) = 1)
void mat_invert(const uint32_t *cols, uint32_t *inv) {
  uint32_t rows[32], id[32];  // row r of A as a bit mask over columns, and of the identity
  for (int r = 0; r < 32; ++r) {
    rows[r] = 0;
    for (int c = 0; c < 32; ++c) rows[r] |= ((cols[c] >> r) & 1u) << c;
    id[r] = 1u << r;
  }
  for (int c = 0; c < 32; ++c) {
    int piv = c;
    while (piv < 32 && !((rows[piv] >> c) & 1u)) ++piv;
    if (piv == 32) continue;  // singular (not for a shift: P(0) = 1); the CPU test checks inverse o advance = identity
    std::swap(rows[c], rows[piv]);
    std::swap(id[c], id[piv]);
    for (int r = 0; r < 32; ++r)
      if (r != c && ((rows[r] >> c) & 1u)) {
        rows[r] ^= rows[c];
        id[r] ^= id[c];
      }
  }
  for (int c = 0; c < 32; ++c) {  // column c of the inverse: bit r = id[r] bit c
    inv[c] = 0;
    for (int r = 0; r < 32; ++r) inv[c] |= ((id[r] >> c) & 1u) << r;
  }
}

}  // namespace

const CrcMath &CrcMath::get(CrcType t) {
  static const CrcMath crc32(0xEDB88320u);
  static const CrcMath crc32c(0x82F63B78u);
  return t == CrcType::kCrc32 ? crc32 : crc32c;
}

CrcMath::CrcMath(uint32_t poly) : poly_(poly) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int b = 0; b < 8; ++b) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
    t0_[i] = c;
  }
  // operator for one zero byte: reg -> (reg >> 8) ^ T0[reg & 0xff]
  for (int c = 0; c < 32; ++c) {
    const uint32_t reg = 1u << c;
    op_[0][c] = (reg >> 8) ^ t0_[reg & 0xff];
  }
  for (int i = 1; i < 64; ++i) mat_square(op_[i - 1], op_[i]);

  blob_b1_ = build_blob(1);
  blob_b2_ = build_blob(2);
  blob_b4_ = build_blob(4);
  for (int i = 0; i < kG26Slots; ++i) g26_[i] = build_g26(kG26Cfg[i][0], kG26Cfg[i][1]);
  // nibble tables: the G26 block map split into 32 nibble-indexed tables per distance set
  nib_.assign(kNibWords, 0);
  uint32_t bit[128];
  for (int p = 0; p < 128; ++p) bit[p] = shift(t0_[1u << (p & 7)], 15 - (p >> 3));
  for (int e = 0; e < kNibSets; ++e)
    for (int p = 0; p < 32; ++p)
      for (uint32_t n = 0; n < 16; ++n) {
        uint32_t acc = 0;
        for (int i = 0; i < 4; ++i)
          if ((n >> i) & 1) acc ^= bit[4 * p + i];
        nib_[(e * 32 + p) * 16 + n] = shift(acc, static_cast<uint64_t>(e) * 1024);
      }
  // XO blob: the G26 block set advanced by kXoAdvance bytes, then the inverse of that advance
  xo_.assign(kXoWords, 0);
  for (int g = 0; g < 26; ++g)
    for (uint32_t v = 0; v < 32; ++v) {
      uint32_t acc = 0;
      for (int i = 0; i < 5; ++i) {
        const int p = g26_bit(g, i);
        if (p >= 0 && ((v >> i) & 1)) acc ^= bit[p];
      }
      xo_[g * 32 + v] = shift(acc, kXoAdvance);
    }
  uint32_t adv[32], back[32];
  shift_matrix(kXoAdvance, adv);
  mat_invert(adv, back);
  for (int g = 0; g < 7; ++g)
    for (uint32_t v = 0; v < 32; ++v) xo_[kXoInv + g * 32 + v] = apply(back, static_cast<uint32_t>(uint64_t{v} << (5 * g)));
  // CV blob: input j's nibble tables and the register shift, both by w_j = j * kCvStride bytes
  cv_.assign(kCvWords, 0);
  for (int j = 0; j < kCvMaxK; ++j) {
    uint32_t wj[32];
    shift_matrix(static_cast<uint64_t>(j) * kCvStride, wj);
    for (int i = 0; i < 512; ++i) cv_[j * 512 + i] = apply(wj, nib_[i]);
    for (int g = 0; g < 7; ++g)
      for (uint32_t v = 0; v < 32; ++v)
        cv_[kCvShift + j * 224 + g * 32 + v] = apply(wj, static_cast<uint32_t>(uint64_t{v} << (5 * g)));
  }
  // bshift blob: register shift by 4 KiB << i bytes
  bshift_.assign(kBshiftN * 224, 0);
  for (int i = 0; i < kBshiftN; ++i) {
    uint32_t m[32];
    shift_matrix(uint64_t{4096} << i, m);
    for (int g = 0; g < 7; ++g)
      for (uint32_t v = 0; v < 32; ++v) bshift_[i * 224 + g * 32 + v] = apply(m, static_cast<uint32_t>(uint64_t{v} << (5 * g)));
  }
}

// Block bit (0..127; dword d bit k = 32d + k, i.e. byte p/8 bit p%8) that index bit i of G26 table g reads,
// -1 past the table's width.  Mirrors the extraction in kernels.hip g26_block:
//   g = 4d+b   (16 tables): w_d bits 8b+2..8b+6                       ((w_d >> 8b) & 0x7c)
//   g = 16+4h+b (8 tables): c_h = rotr(w_2h,5) on bits 2..4 of each byte, rotr(w_2h+1,2) on bits 5..6:
//                            w_2h bits 8b+7..8b+9, then w_2h+1 bits 8b+7..8b+8 (mod 32)
//   g = 24, 25  (4 bits)  : e = (rotr(w1,7) on bits 8b+2, rotr(w3,6) on bits 8b+3) & 0x0c0c0c0c, e |= e << 10;
//                            bits 10..13 and 26..29 of e: the w1/w3 bits 8b+9 left over
int g26_bit(int g, int i) {
  if (g < 16) return i < 5 ? 32 * (g >> 2) + 8 * (g & 3) + 2 + i : -1;
  if (g < 24) {
    const int h = (g - 16) >> 2, b = (g - 16) & 3;
    if (i < 3) return 64 * h + (8 * b + 7 + i) % 32;
    if (i < 5) return 64 * h + 32 + (8 * b + 7 + i - 3) % 32;
    return -1;
  }
  static const int k24[4] = {32 + 17, 96 + 17, 32 + 9, 96 + 9};
  static const int k25[4] = {32 + 1, 96 + 1, 32 + 25, 96 + 25};
  if (i >= 4) return -1;
  return g == 24 ? k24[i] : k25[i];
}

std::vector<uint32_t> CrcMath::build_g26(int B, int D) const {
  const int E = B * D;
  std::vector<uint32_t> blob(g26_words(E), 0);
  uint32_t bit[128];
  for (int p = 0; p < 128; ++p) bit[p] = shift(t0_[1u << (p & 7)], 15 - (p >> 3));
  for (int e = 0; e < E; ++e) {
    const int r = e / B, s = e % B;
    const uint64_t dist = (static_cast<uint64_t>(r) * 64 * B + s) * 16;
    uint32_t sb[128];
    for (int p = 0; p < 128; ++p) sb[p] = shift(bit[p], dist);
    for (int g = 0; g < 26; ++g)
      for (uint32_t v = 0; v < 32; ++v) {
        uint32_t acc = 0;
        for (int i = 0; i < 5; ++i) {
          const int p = g26_bit(g, i);
          if (p >= 0 && ((v >> i) & 1)) acc ^= sb[p];
        }
        blob[e * kG26Set + g * 32 + v] = acc;
      }
  }
  auto fill_shift = [&](int off, uint64_t n) {
    for (int g = 0; g < 7; ++g)
      for (uint32_t v = 0; v < 32; ++v) blob[off + g * 32 + v] = shift(static_cast<uint32_t>(uint64_t{v} << (5 * g)), n);
  };
  fill_shift(g26_gshift(E), static_cast<uint64_t>(D) * 64 * B * 16);
  for (int m = 0; m < 6; ++m) fill_shift(g26_tree(E) + m * 224, static_cast<uint64_t>(16) * B << m);
  for (int v = 0; v < 256; ++v) blob[g26_t0(E) + v] = t0_[v];
  return blob;
}

std::vector<uint32_t> CrcMath::build_blob(int B) const {
  std::vector<uint32_t> blob(kG5Words, 0);
  // contribution of block bit p (byte p/8, bit p%8) to the raw CRC of a 16-B block processed from 0
  uint32_t bit[128];
  for (int p = 0; p < 128; ++p) bit[p] = shift(t0_[1u << (p & 7)], 15 - (p >> 3));
  for (int g = 0; g < 26; ++g)
    for (uint32_t v = 0; v < 32; ++v) {
      uint32_t r = 0;
      for (int t = 0; t < 5; ++t)
        if (((v >> t) & 1) && 5 * g + t < 128) r ^= bit[5 * g + t];
      blob[kG5Blk + g * 32 + v] = r;
    }
  auto fill_shift = [&](int off, uint64_t n) {
    for (int g = 0; g < 7; ++g)
      for (uint32_t v = 0; v < 32; ++v) blob[off + g * 32 + v] = shift(static_cast<uint32_t>(uint64_t{v} << (5 * g)), n);
  };
  fill_shift(kG5Step, static_cast<uint64_t>(63) * B * 16);
  for (int m = 0; m < 6; ++m) fill_shift(kG5Tree + m * 224, static_cast<uint64_t>(16) * B << m);
  for (int v = 0; v < 256; ++v) blob[kG5T0 + v] = t0_[v];
  return blob;
}

uint32_t CrcMath::shift(uint32_t reg, uint64_t n) const {
  for (int i = 0; n && reg; ++i, n >>= 1)
    if (n & 1) reg = mat_times(op_[i], reg);
  return reg;
}

}  // namespace ozec
