#include "gf256.hpp"

#include <cstring>

namespace ozec {

const GF256 &GF256::get() {
  static const GF256 instance;
  return instance;
}

GF256::GF256() {
  // exp/log over generator 2; the product table is what GF256.gfMulTab() (GF256.java:141-162) holds.
  uint8_t exp[510];
  int log[256] = {0};
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    exp[i] = exp[i + 255] = static_cast<uint8_t>(x);
    log[x] = i;
    x = (x << 1) ^ ((x & 0x80) ? 0x11d : 0);
  }
  for (int a = 0; a < 256; ++a)
    for (int b = 0; b < 256; ++b)
      mul_[a][b] = (a && b) ? exp[log[a] + log[b]] : 0;
  inv_[0] = 0;
  for (int a = 1; a < 256; ++a) inv_[a] = exp[(255 - log[a]) % 255];
}

std::vector<uint8_t> cauchy_matrix(int k, int p) {
  const GF256 &gf = GF256::get();
  std::vector<uint8_t> a(static_cast<size_t>(k + p) * k, 0);
  for (int i = 0; i < k; ++i) a[static_cast<size_t>(i) * k + i] = 1;
  for (int i = k; i < k + p; ++i)
    for (int j = 0; j < k; ++j) a[static_cast<size_t>(i) * k + j] = gf.inv(static_cast<uint8_t>(i ^ j));
  return a;
}

bool invert_matrix(uint8_t *in, uint8_t *out, int n) {
  const GF256 &gf = GF256::get();
  std::memset(out, 0, static_cast<size_t>(n) * n);
  for (int i = 0; i < n; ++i) out[i * n + i] = 1;
  for (int i = 0; i < n; ++i) {
    uint8_t *ri = in + i * n, *oi = out + i * n;
    if (ri[i] == 0) {
      int j = i + 1;
      while (j < n && in[j * n + i] == 0) ++j;
      if (j == n) return false;
      for (int c = 0; c < n; ++c) {
        std::swap(ri[c], in[j * n + c]);
        std::swap(oi[c], out[j * n + c]);
      }
    }
    const uint8_t pivot_inv = gf.inv(ri[i]);
    for (int c = 0; c < n; ++c) {
      ri[c] = gf.mul(ri[c], pivot_inv);
      oi[c] = gf.mul(oi[c], pivot_inv);
    }
    for (int j = 0; j < n; ++j) {
      if (j == i) continue;
      const uint8_t f = in[j * n + i];
      for (int c = 0; c < n; ++c) {
        out[j * n + c] ^= gf.mul(f, oi[c]);
        in[j * n + c] ^= gf.mul(f, ri[c]);
      }
    }
  }
  return true;
}

bool decode_matrix(int k, int p, const int *valid, const int *erased, int n_erased,
                   std::vector<uint8_t> &rows) {
  const GF256 &gf = GF256::get();
  const int n_all = k + p;
  const std::vector<uint8_t> enc = cauchy_matrix(k, p);
  std::vector<uint8_t> tmp(static_cast<size_t>(k) * k);
  // invertMatrix is allocated (k+p) x k in the reference (RSRawDecoder.java:119); rows >= k stay zero.
  std::vector<uint8_t> inv(static_cast<size_t>(n_all) * k, 0);
  for (int i = 0; i < k; ++i)
    std::memcpy(&tmp[static_cast<size_t>(i) * k], &enc[static_cast<size_t>(valid[i]) * k], k);
  if (!invert_matrix(tmp.data(), inv.data(), k)) return false;

  int n_erased_data = 0;
  for (int i = 0; i < n_erased; ++i) n_erased_data += erased[i] < k;

  rows.assign(static_cast<size_t>(n_erased) * k, 0);
  for (int i = 0; i < n_erased_data; ++i)
    std::memcpy(&rows[static_cast<size_t>(i) * k], &inv[static_cast<size_t>(erased[i]) * k], k);
  for (int r = n_erased_data; r < n_erased; ++r) {
    const uint8_t *erow = &enc[static_cast<size_t>(erased[r]) * k];
    for (int i = 0; i < k; ++i) {
      uint8_t s = 0;
      for (int j = 0; j < k; ++j) s ^= gf.mul(inv[static_cast<size_t>(j) * k + i], erow[j]);
      rows[static_cast<size_t>(r) * k + i] = s;
    }
  }
  return true;
}

}  // namespace ozec
