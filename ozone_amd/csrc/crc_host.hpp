// Host-side CRC math: table construction for the GPU kernels and GF(2) shift/combine operators.
// Reflected CRC-32 (poly 0xEDB88320) and CRC-32C (poly 0x82F63B78), init/xorout 0xFFFFFFFF -- the
// arithmetic of ChecksumByteBuffer.CrcIntTable (CM/ChecksumByteBuffer.java:51-121) and the JDK
// java.util.zip.CRC32 / CRC32C that ChecksumByteBufferFactory hands out (ChecksumByteBufferFactory.java:74-89).
#pragma once
#include <cstdint>
#include <vector>

#include "kernels.hpp"

namespace ozec {

enum class CrcType { kCrc32 = 0, kCrc32c = 1 };

class CrcMath {
 public:
  static const CrcMath &get(CrcType t);
  // raw register after appending n zero bytes (multiplication by x^(8n) mod P)
  uint32_t shift(uint32_t reg, uint64_t n) const;
  // crc(A||B) from the finished values crc(A), crc(B) and |B| (zlib-style combine)
  uint32_t combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b) const { return shift(crc_a, len_b) ^ crc_b; }
  // the device G5 table blob (kernels.hpp kG5* layout) for B = 1 or 4 blocks per lane per step
  const std::vector<uint32_t> &device_tables(int B) const { return B == 1 ? blob_b1_ : B == 2 ? blob_b2_ : blob_b4_; }
  // the device G26 table blob (kernels.hpp kG26*) for slot `slot` of kG26Cfg
  const std::vector<uint32_t> &g26_tables(int slot) const { return g26_[slot]; }
  // the device nibble blob (kernels.hpp kNib*)
  const std::vector<uint32_t> &nib_tables() const { return nib_; }
  // the device XO blob (kernels.hpp kXo*)
  const std::vector<uint32_t> &xo_tables() const { return xo_; }
  // the device CV blob (kernels.hpp kCv*)
  const std::vector<uint32_t> &cv_tables() const { return cv_; }
  // the register shift by (4 KiB << i) bytes as 7 tables of 32 (the bshift blob of kernels.hpp), i < kBshiftN
  const std::vector<uint32_t> &bshift_tables() const { return bshift_; }
  uint32_t byte_table(int v) const { return t0_[v]; }
  uint32_t poly() const { return poly_; }
  // x^(8n) mod P in CrcUtil's reversed representation (CrcUtil.getMonomial)
  uint32_t monomial(uint64_t n) const { return shift(0x80000000u, n); }
  // the shift-by-n operator as 32 columns (column c = shift(1 << c, n)), for repeated use with apply()
  void shift_matrix(uint64_t n, uint32_t cols[32]) const {
    for (int c = 0; c < 32; ++c) cols[c] = shift(1u << c, n);
  }
  static uint32_t apply(const uint32_t cols[32], uint32_t v) {
    uint32_t r = 0;
    for (int c = 0; v; ++c, v >>= 1)
      if (v & 1) r ^= cols[c];
    return r;
  }

 private:
  explicit CrcMath(uint32_t poly);
  uint32_t poly_;
  uint32_t t0_[256];
  // op_[i] = operator for 2^i zero BYTES as a 32x32 GF(2) matrix (column c = image of bit c)
  uint32_t op_[64][32];
  std::vector<uint32_t> blob_b1_, blob_b2_, blob_b4_;
  std::vector<uint32_t> g26_[kG26Slots];
  std::vector<uint32_t> nib_;
  std::vector<uint32_t> xo_;
  std::vector<uint32_t> cv_;
  std::vector<uint32_t> bshift_;
  std::vector<uint32_t> build_blob(int B) const;
  std::vector<uint32_t> build_g26(int B, int D) const;
};

}  // namespace ozec
