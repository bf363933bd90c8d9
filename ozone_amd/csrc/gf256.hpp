// Host-side GF(2^8) coding math for the RS coder: the O(k^3) setup the reference runs once per schema or
// per erasure pattern.  The per-byte work runs on the GPU (kernels.hip).
#pragma once
#include <cstdint>
#include <vector>

namespace ozec {

// Field GF(2^8), primitive polynomial 0x11d, generator 2 (RSUtil.java:34-37, GF256.java:260).
class GF256 {
 public:
  static const GF256 &get();
  uint8_t mul(uint8_t a, uint8_t b) const { return mul_[a][b]; }
  // GF256.gfInv (GF256.java:178-184): 0 maps to 0.
  uint8_t inv(uint8_t a) const { return inv_[a]; }

 private:
  GF256();
  uint8_t mul_[256][256];
  uint8_t inv_[256];
};

// RSUtil.genCauchyMatrix (RSUtil.java:64-77): (k+p) x k, identity on top, a[i][j] = 1/(i ^ j) below.
std::vector<uint8_t> cauchy_matrix(int k, int p);

// GF256.gfInvertMatrix (GF256.java:191-250): Gauss-Jordan with the reference's pivot search order.
// `in` is clobbered.  Returns false when singular ("Not invertible").
bool invert_matrix(uint8_t *in, uint8_t *out, int n);

// RSRawDecoder.generateDecodeMatrix (RSRawDecoder.java:143-176).  `valid` holds the first k valid unit
// indexes (ascending), `erased` the erased units in caller order.  Row i of the result recovers erased[i].
// Reproduces the reference quirk for erased parity listed before erased data.
bool decode_matrix(int k, int p, const int *valid, const int *erased, int n_erased,
                   std::vector<uint8_t> &rows);

}  // namespace ozec
