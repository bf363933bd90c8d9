// Host-side code of libozec under AddressSanitizer + UndefinedBehaviorSanitizer (and ThreadSanitizer for the copy
// pool): the O(k^3) GF(2^8) setup (gf256.cpp), the CRC table / shift / combine math (crc_host.cpp) and the parallel
// staging copy (copy_pool.cpp), checked against the C oracle where it has a counterpart.  SURVEY.md §5 "race
// detection / sanitizers": host ASan/TSan on the C ABI's host code and the oracle; the kernels are checked by
// bit-exact comparison on the GPU instead.  Built and run by tests/test_host_sanitize.py (CPU only).
//
//   main modes: "math" (ASan/UBSan build)  -- every erasure pattern of rs-3-2 / rs-6-3 / rs-10-4 (and a few wider
//                                             schemas) through decode_matrix vs oracle_rs_decode_matrix, Cauchy
//                                             matrices and inverses, CRC shift/combine vs the byte-wise oracle,
//                                             the device table blobs built end to end;
//               "copy" (TSan or ASan build) -- parallel_copy from several caller threads at once with pool
//                                             resizes in between, every byte checked.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "copy_pool.hpp"
#include "crc_host.hpp"
#include "gf256.hpp"

extern "C" {
int oracle_rs_decode_matrix(int k, int p, const int *valid, const int *erased, int n_erased, uint8_t *out);
void oracle_gen_cauchy_matrix(uint8_t *a, int m, int k);
int oracle_gf_invert_matrix(uint8_t *in, uint8_t *out, int n);
uint8_t oracle_gf_mul(uint8_t a, uint8_t b);
uint32_t oracle_crc(int type, const uint8_t *b, size_t n);
}

static int g_fail = 0;
#define CHECK(cond, ...)                       \
  do {                                         \
    if (!(cond)) {                             \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);       \
      std::fprintf(stderr, "\n");              \
      if (++g_fail > 20) std::exit(1);         \
    }                                          \
  } while (0)

// every subset of {0..n-1} of size 1..maxe, in increasing order (also fed reversed: caller order matters)
static void subsets(int n, int maxe, std::vector<std::vector<int>> &out) {
  for (uint32_t m = 1; m < (1u << n); ++m) {
    const int c = __builtin_popcount(m);
    if (c > maxe) continue;
    std::vector<int> s;
    for (int i = 0; i < n; ++i)
      if (m & (1u << i)) s.push_back(i);
    out.push_back(s);
  }
}

static long check_decode(int k, int p) {
  std::vector<std::vector<int>> pats;
  subsets(k + p, p, pats);
  long n = 0;
  for (auto erased : pats) {
    for (int order = 0; order < 2; ++order) {
      if (order) std::reverse(erased.begin(), erased.end());
      std::vector<int> valid;
      for (int u = 0; u < k + p && static_cast<int>(valid.size()) < k; ++u)
        if (std::find(erased.begin(), erased.end(), u) == erased.end()) valid.push_back(u);
      std::vector<uint8_t> rows;
      const bool ok = ozec::decode_matrix(k, p, valid.data(), erased.data(), static_cast<int>(erased.size()), rows);
      std::vector<uint8_t> ref(static_cast<size_t>(erased.size()) * k);
      const int rc = oracle_rs_decode_matrix(k, p, valid.data(), erased.data(), static_cast<int>(erased.size()),
                                             ref.data());
      CHECK(ok == (rc == 0), "rs-%d-%d decode_matrix status %d vs oracle %d", k, p, ok, rc);
      if (ok && rc == 0) CHECK(rows == ref, "rs-%d-%d decode matrix differs from the oracle", k, p);
      ++n;
    }
  }
  return n;
}

static void check_cauchy_and_inverse() {
  for (int k = 1; k <= 16; ++k)
    for (int p = 1; p <= 8; ++p) {
      const std::vector<uint8_t> a = ozec::cauchy_matrix(k, p);
      std::vector<uint8_t> ref(static_cast<size_t>(k + p) * k);
      oracle_gen_cauchy_matrix(ref.data(), k + p, k);
      CHECK(a == ref, "cauchy %d+%d", k, p);
      // the k x k submatrix of rows p..p+k-1 (mixed identity/parity rows) is invertible; both inverses agree
      std::vector<uint8_t> m(a.begin() + static_cast<long>(p) * k, a.begin() + static_cast<long>(p + k) * k);
      std::vector<uint8_t> m2 = m, inv(m.size()), inv2(m.size());
      const bool ok = ozec::invert_matrix(m.data(), inv.data(), k);
      const int rc = oracle_gf_invert_matrix(m2.data(), inv2.data(), k);
      CHECK(ok == (rc == 0), "invert status %d vs %d (k=%d p=%d)", ok, rc, k, p);
      if (ok) CHECK(inv == inv2, "inverse differs (k=%d p=%d)", k, p);
    }
  // a singular matrix is reported, not inverted
  std::vector<uint8_t> sing = {1, 2, 2, 4}, out(4);
  CHECK(!ozec::invert_matrix(sing.data(), out.data(), 2), "singular matrix inverted");
  const ozec::GF256 &gf = ozec::GF256::get();
  for (int a = 0; a < 256; ++a)
    for (int b = 0; b < 256; ++b)
      CHECK(gf.mul(static_cast<uint8_t>(a), static_cast<uint8_t>(b)) ==
                oracle_gf_mul(static_cast<uint8_t>(a), static_cast<uint8_t>(b)), "gf mul %d %d", a, b);
}

static void check_crc() {
  std::mt19937_64 rng(0x00EC5EED);
  std::vector<uint8_t> buf(1 << 16);
  for (auto &b : buf) b = static_cast<uint8_t>(rng());
  for (int t = 0; t < 2; ++t) {
    const ozec::CrcMath &m = ozec::CrcMath::get(t ? ozec::CrcType::kCrc32c : ozec::CrcType::kCrc32);
    for (int i = 0; i < 300; ++i) {
      const size_t a = rng() % 4097, b = rng() % 30000;
      const uint32_t ca = oracle_crc(t, buf.data(), a), cb = oracle_crc(t, buf.data() + a, b);
      CHECK(m.combine(ca, cb, b) == oracle_crc(t, buf.data(), a + b), "crc%d combine a=%zu b=%zu", t, a, b);
    }
    // the device blobs: built end to end (ASan sees any write outside them), sizes as kernels.hpp lays them out
    for (int B : {1, 2, 4}) CHECK(!m.device_tables(B).empty(), "G5 blob B=%d empty", B);
    for (int s = 0; s < 5; ++s) CHECK(!m.g26_tables(s).empty(), "G26 blob %d empty", s);
    uint32_t cols[32];
    m.shift_matrix(12345, cols);
    for (int i = 0; i < 100; ++i) {
      const uint32_t v = static_cast<uint32_t>(rng());
      CHECK(ozec::CrcMath::apply(cols, v) == m.shift(v, 12345), "shift matrix");
    }
  }
}

static void check_copy() {
  std::atomic<int> bad{0};
  auto caller = [&](int id) {
    std::mt19937_64 rng(1000 + id);
    for (int it = 0; it < 6; ++it) {
      std::vector<ozec::CopyTask> tasks;
      std::vector<std::vector<uint8_t>> src, dst;
      const int ntask = 1 + static_cast<int>(rng() % 5);
      std::vector<size_t> so, dof;  // misaligned starts: the streaming copy's head / body / tail split
      for (int i = 0; i < ntask; ++i) {
        const size_t n = 1 + rng() % (3u << 20);
        so.push_back(rng() % 64);
        dof.push_back(rng() % 64);
        src.emplace_back(n + so.back());
        dst.emplace_back(n + dof.back() + 64, 0);
        for (size_t j = 0; j < src.back().size(); j += 97) src.back()[j] = static_cast<uint8_t>(rng());
        src.back()[so.back() + n - 1] = static_cast<uint8_t>(id + it);
      }
      for (int i = 0; i < ntask; ++i)
        tasks.push_back({dst[i].data() + dof[i], src[i].data() + so[i], src[i].size() - so[i]});
      ozec::parallel_copy(tasks, (it & 1) ? ozec::CopyDir::kToStaging : ozec::CopyDir::kFromStaging);
      for (int i = 0; i < ntask; ++i) {
        const size_t n = src[i].size() - so[i];
        if (std::memcmp(dst[i].data() + dof[i], src[i].data() + so[i], n) != 0) ++bad;
        for (size_t j = 0; j < dof[i]; ++j) bad += dst[i][j] != 0;                   // nothing written before
        for (size_t j = dof[i] + n; j < dst[i].size(); ++j) bad += dst[i][j] != 0;  // or after the range
      }
    }
  };
  for (int stream : {1, 2, 3, 0})  // streaming stores both ways / into staging only / when shared, plain memcpy
    for (int threads : {4, 0, 2}) {
      ozec::set_copy_stream(stream);
      ozec::set_copy_spin_us(stream == 2 ? 50 : 0);  // workers and callers polling before they sleep, or not
      ozec::set_copy_threads(threads);  // resize the pool between rounds of concurrent callers
      std::vector<std::thread> ts;
      for (int c = 0; c < 4; ++c) ts.emplace_back(caller, c);
      for (auto &t : ts) t.join();
    }
  ozec::set_copy_stream(-1);
  ozec::set_copy_spin_us(0);
  CHECK(bad.load() == 0, "%d parallel copies differ", bad.load());
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "math";
  if (!std::strcmp(mode, "math")) {
    check_cauchy_and_inverse();
    long n = 0;
    for (auto kp : {std::pair<int, int>{3, 2}, {6, 3}, {10, 4}, {2, 1}, {6, 2}, {12, 4}, {4, 7}}) n += check_decode(kp.first, kp.second);
    check_crc();
    std::printf("math: %ld decode patterns, cauchy/inverse 16x8 schemas, GF table, CRC combine -- %s\n", n,
                g_fail ? "FAILED" : "ok");
  } else {
    check_copy();
    std::printf("copy: 4 store modes x 3 pool sizes x 4 concurrent callers, misaligned -- %s\n", g_fail ? "FAILED" : "ok");
  }
  return g_fail ? 1 : 0;
}
