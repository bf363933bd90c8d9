// Host emulation of the G26 CRC scheme (kernels.hip g26_block / crc_windows_g26): builds the device table blobs
// with the product's own builder (crc_host.cpp) and runs the device algorithm -- SDWA-style extraction, step
// groups, 64 lane registers, lane combine -- on the CPU, comparing every window with the byte-wise CRC.
// Checks the bit-group map (g26_bit) and the table-set distances without a GPU.  Exit 0 = all equal.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "crc_host.hpp"
#include "kernels.hpp"

using namespace ozec;

static uint32_t rotr(uint32_t w, int k) { return (w >> k) | (w << (32 - k)); }
static uint32_t bsel(uint32_t a, uint32_t b, uint32_t m) { return (a & m) | (b & ~m); }
static uint32_t at(const uint32_t *T, uint32_t byte_off) { return T[byte_off / 4]; }

static uint32_t g26_block(const uint32_t *T, const uint32_t w[4]) {
  uint32_t r = 0;
  auto four = [&](uint32_t v, int g0) {
    for (int q = 0; q < 4; ++q) r ^= at(T, (g0 + q) * 128 + ((v >> (8 * q)) & 0x7c));
  };
  for (int d = 0; d < 4; ++d) four(w[d], 4 * d);
  for (int h = 0; h < 2; ++h) four(bsel(rotr(w[2 * h], 5), rotr(w[2 * h + 1], 2), 0x1c1c1c1c), 16 + 4 * h);
  uint32_t e = bsel(rotr(w[1], 7), rotr(w[3], 6), 0x04040404) & 0x0c0c0c0c;
  e |= e << 10;
  r ^= at(T, 24 * 128 + ((e >> 8) & 0x3c));
  r ^= at(T, 25 * 128 + ((e >> 24) & 0x3c));
  return r;
}

static uint32_t shift7(const uint32_t *T, uint32_t s) {
  uint32_t r = 0;
  for (int g = 0; g < 7; ++g) r ^= T[g * 32 + ((s >> (5 * g)) & 31)];
  return r;
}

int main() {
  srand(12345);
  int checked = 0;
  for (int ty = 0; ty < 2; ++ty) {
    const CrcMath &cm = CrcMath::get(static_cast<CrcType>(ty));
    for (int slot = 0; slot < kG26Slots; ++slot) {
      const int B = kG26Cfg[slot][0], D = kG26Cfg[slot][1], E = B * D;
      const std::vector<uint32_t> &T = cm.g26_tables(slot);
      if (static_cast<int>(T.size()) != g26_words(E)) {
        printf("blob size mismatch slot %d\n", slot);
        return 1;
      }
      const int sizes[] = {1, 2, 37, 63, 64, 65, 64 * E - 1, 64 * E, 64 * E + 1, 1024, 3 * 64 * E + 5, 2000};
      for (int m : sizes) {
        std::vector<uint8_t> buf(static_cast<size_t>(m) * 16);
        for (auto &x : buf) x = static_cast<uint8_t>(rand());
        uint32_t ref = 0;  // raw register: init 0, no xorout
        for (uint8_t x : buf) ref = (ref >> 8) ^ cm.byte_table((ref ^ x) & 0xff);
        const long G = (m + 64L * E - 1) / (64L * E), P = G * 64L * E - m;
        uint32_t total = 0;
        for (int l = 0; l < 64; ++l) {
          uint32_t S = 0;
          for (long g = 0; g < G; ++g) {
            for (int rr = 0; rr < D; ++rr) {
              const long t = g * D + rr;
              for (int q = 0; q < B; ++q) {
                const long vb = t * 64 * B + l * B + q - P;
                uint32_t w[4] = {0, 0, 0, 0};
                if (vb >= 0) memcpy(w, &buf[vb * 16], 16);
                S ^= g26_block(T.data() + ((D - 1 - rr) * B + (B - 1 - q)) * kG26Set, w);
              }
            }
            if (g + 1 < G) S = shift7(T.data() + g26_gshift(E), S);
          }
          total = cm.shift(total, 16 * B) ^ S;  // lane l's chunk precedes lane l+1's by B blocks
        }
        if (total != ref) {
          printf("FAIL crc type %d slot %d (B=%d D=%d) blocks %d: %08x vs %08x\n", ty, slot, B, D, m, total, ref);
          return 1;
        }
        ++checked;
      }
    }
  }
  // nibble tables of the nibble-table fused kernel (fused.hip encode_crc_nb): the XOR over a block's 32 nibbles of
  // nib[e][p][nibble] must be the block's raw CRC advanced by e KiB
  int nib_checked = 0;
  for (int ty = 0; ty < 2; ++ty) {
    const CrcMath &cm = CrcMath::get(static_cast<CrcType>(ty));
    const std::vector<uint32_t> &N = cm.nib_tables();
    if (static_cast<int>(N.size()) != kNibWords) {
      printf("nibble blob size mismatch\n");
      return 1;
    }
    for (int e = 0; e < kNibSets; ++e)
      for (int it = 0; it < 2000; ++it) {
        uint8_t b[16];
        for (auto &x : b) x = static_cast<uint8_t>(rand());
        if (it == 0) memset(b, 0, 16);
        if (it == 1) memset(b, 0xff, 16);
        uint32_t reg = 0;
        for (uint8_t x : b) reg = (reg >> 8) ^ cm.byte_table((reg ^ x) & 0xff);
        const uint32_t ref = cm.shift(reg, static_cast<uint64_t>(e) * 1024);
        uint32_t got = 0;
        for (int p = 0; p < 32; ++p) got ^= N[(e * 32 + p) * 16 + ((b[p >> 1] >> (4 * (p & 1))) & 15)];
        if (got != ref) {
          printf("FAIL nibble tables crc type %d set %d: %08x vs %08x\n", ty, e, got, ref);
          return 1;
        }
        ++nib_checked;
      }
  }
  // XO scheme of the nibble kernel's output registers (fused_nb.hpp, XO variants): per step every lane XORs its
  // register into the first dword of its next block and looks the block up in the XO set (advanced by kXoAdvance
  // bytes), so the register moves by one 1 KiB step with no shift lookups; the inverse table undoes the advance
  int xo_checked = 0;
  for (int ty = 0; ty < 2; ++ty) {
    const CrcMath &cm = CrcMath::get(static_cast<CrcType>(ty));
    const std::vector<uint32_t> &X = cm.xo_tables();
    if (static_cast<int>(X.size()) != kXoWords) {
      printf("XO blob size mismatch\n");
      return 1;
    }
    for (int it = 0; it < 200; ++it) {  // the inverse really inverts the advance
      const uint32_t v = static_cast<uint32_t>(rand()) * 2654435761u + static_cast<uint32_t>(it);
      if (shift7(X.data() + kXoInv, cm.shift(v, kXoAdvance)) != v) {
        printf("FAIL XO inverse crc type %d\n", ty);
        return 1;
      }
    }
    for (int T : {1, 2, 3, 4, 16}) {  // steps per window (bpc = T KiB)
      std::vector<uint8_t> buf(static_cast<size_t>(T) * 1024);
      for (auto &x : buf) x = static_cast<uint8_t>(rand());
      uint32_t ref = 0;
      for (uint8_t x : buf) ref = (ref >> 8) ^ cm.byte_table((ref ^ x) & 0xff);
      uint32_t total = 0;
      for (int l = 0; l < 64; ++l) {
        uint32_t U = 0;
        for (int t = 0; t < T; ++t) {
          uint32_t w[4];
          memcpy(w, &buf[static_cast<size_t>(t) * 1024 + 16 * l], 16);
          w[0] ^= U;
          U = g26_block(X.data(), w);
        }
        total = cm.shift(total, 16) ^ shift7(X.data() + kXoInv, U);
      }
      if (total != ref) {
        printf("FAIL XO window crc type %d T=%d: %08x vs %08x\n", ty, T, total, ref);
        return 1;
      }
      ++xo_checked;
    }
  }
  // G5 scheme of the combined-verify re-check (fused.hip nb_reverify): lane l folds blocks l, l+64, ... -- register
  // shifted by the 1008-B gap (kG5Step), XORed into the block's first dword, block looked up in the kG5Blk tables --
  // and the lane tree (kG5Tree, shifts by 16 * 2^m) merges the lanes; windows front-padded with zero blocks
  int g5_checked = 0;
  for (int ty = 0; ty < 2; ++ty) {
    const CrcMath &cm = CrcMath::get(static_cast<CrcType>(ty));
    const std::vector<uint32_t> &G = cm.device_tables(1);
    if (static_cast<int>(G.size()) != kG5Words) {
      printf("G5 blob size mismatch\n");
      return 1;
    }
    auto g5_block = [&](const uint32_t w[4]) {
      uint32_t r = 0;
      for (int g = 0; g < 26; ++g) {
        const int o = 5 * g, d = o >> 5, sh = o & 31;
        const uint32_t v = (sh <= 27 || d == 3) ? (w[d] >> sh) : ((w[d] >> sh) | (w[d + 1] << (32 - sh)));
        r ^= G[kG5Blk + g * 32 + (v & 31)];
      }
      return r;
    };
    for (int m : {1, 5, 63, 64, 65, 256, 257, 1024}) {  // 16-B blocks per window
      std::vector<uint8_t> buf(static_cast<size_t>(m) * 16);
      for (auto &x : buf) x = static_cast<uint8_t>(rand());
      uint32_t ref = 0;
      for (uint8_t x : buf) ref = (ref >> 8) ^ cm.byte_table((ref ^ x) & 0xff);
      const long steps = (m + 63) / 64, pad = steps * 64 - m;
      uint32_t S[64];
      for (int l = 0; l < 64; ++l) {
        S[l] = 0;
        for (long q = 0; q < steps; ++q) {
          const long vb = q * 64 + l - pad;
          uint32_t w[4] = {0, 0, 0, 0};
          if (vb >= 0) memcpy(w, &buf[vb * 16], 16);
          if (q > 0) S[l] = shift7(G.data() + kG5Step, S[l]);
          w[0] ^= S[l];
          S[l] = g5_block(w);
        }
      }
      for (int lv = 0; lv < 6; ++lv) {  // g5_lane_tree: lane l's registers precede lane l + 2^lv's
        uint32_t nS[64];
        for (int l = 0; l < 64; ++l) {
          const int o = l ^ (1 << lv);
          const bool upper = (l >> lv) & 1;
          nS[l] = shift7(G.data() + kG5Tree + lv * 224, upper ? S[o] : S[l]) ^ (upper ? S[l] : S[o]);
        }
        memcpy(S, nS, sizeof(S));
      }
      for (int l = 0; l < 64; ++l)
        if (S[l] != ref) {
          printf("FAIL G5 re-check window crc type %d blocks %d lane %d: %08x vs %08x\n", ty, m, l, S[l], ref);
          return 1;
        }
      ++g5_checked;
    }
  }
  printf("g26 emulation: %d windows bit-exact; nibble tables: %d blocks bit-exact; XO: %d windows bit-exact; "
         "G5 re-check: %d windows bit-exact\n", checked, nib_checked, xo_checked, g5_checked);
  return 0;
}
