#include "crc_host.hpp"

#include "kernels.hpp"

namespace ozec {
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

}  // namespace

const CrcMath &CrcMath::get(CrcType t) {
  static const CrcMath crc32(0xEDB88320u);
  static const CrcMath crc32c(0x82F63B78u);
  return t == CrcType::kCrc32 ? crc32 : crc32c;
}

CrcMath::CrcMath(uint32_t poly) {
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

  // device blob
  blob_.assign(kCrcTableWords, 0);
  // slice tables T_m[v] = shift(T0[v], m) for m = 0..15
  for (int m = 0; m < 16; ++m)
    for (int v = 0; v < 256; ++v) blob_[kCrcSliceOff + m * 256 + v] = shift(t0_[v], m);
  // Z_n[j][v] = shift(v << 8j, n)
  auto fill_z = [&](int off, uint64_t n) {
    for (int j = 0; j < 4; ++j)
      for (int v = 0; v < 256; ++v) blob_[off + j * 256 + v] = shift(static_cast<uint32_t>(v) << (8 * j), n);
  };
  fill_z(kCrcZ1024Off, 1024);
  for (int m = 1; m <= 5; ++m) fill_z(kCrcTreeOff + (m - 1) * 1024, 16ull << m);
}

uint32_t CrcMath::shift(uint32_t reg, uint64_t n) const {
  for (int i = 0; n && reg; ++i, n >>= 1)
    if (n & 1) reg = mat_times(op_[i], reg);
  return reg;
}

}  // namespace ozec
