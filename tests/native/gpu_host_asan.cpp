// The host-buffer paths of the C ABI on a real GPU, with libozec's host code built under AddressSanitizer + UBSan
// (make -C ozone_amd/csrc asan-host; the kernels are the regular objects, nothing on the device is instrumented).
// Every caller buffer is its own heap allocation of exactly the bytes the call may touch, often misaligned, so an
// out-of-bounds read or write by the staging pipelines, the rectangular copies of the C5 host batch or the stripe
// queue's ring is reported.  Results are checked against the C oracle.  Built by scripts/build_gpu_host_asan.sh,
// run on the GPU box by scripts/gpu_host_asan.sh.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/ozec.h"

extern "C" {
int oracle_rs_encode(int k, int p, int len, const uint8_t *const *in, uint8_t *const *out);
void oracle_xor_encode(int k, int len, const uint8_t *const *in, uint8_t *out);
uint32_t oracle_crc(int type, const uint8_t *b, size_t n);
size_t oracle_crc_windows(int type, const uint8_t *data, size_t n, size_t bpc, uint32_t *out);
}

static int g_fail = 0;
#define CHECK(cond, ...)                                        \
  do {                                                          \
    if (!(cond)) {                                              \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);                        \
      std::fprintf(stderr, " [%s]\n", ozec_last_error());      \
      if (++g_fail > 20) std::exit(1);                          \
    }                                                           \
  } while (0)

static std::mt19937_64 rng(0x00EC5EED);

// a heap buffer of exactly n bytes starting `mis` bytes into its allocation (misaligned on purpose)
struct Buf {
  uint8_t *base = nullptr, *p = nullptr;
  size_t n = 0;
  Buf(size_t n_, size_t mis = 0) : n(n_) {
    base = static_cast<uint8_t *>(std::malloc(n_ + mis + 1));
    p = base + mis;
  }
  ~Buf() { std::free(base); }
  Buf(const Buf &) = delete;
  void fill() {
    for (size_t i = 0; i < n; ++i) p[i] = static_cast<uint8_t>(rng());
  }
};

static void encode_decode(int codec, int k, int p, size_t len, size_t mis) {
  ozec_coder *enc = nullptr, *dec = nullptr;
  CHECK(ozec_encoder_create(codec, k, p, &enc) == OZEC_OK, "encoder");
  CHECK(ozec_decoder_create(codec, k, p, &dec) == OZEC_OK, "decoder");
  std::vector<Buf *> in, out, ref;
  std::vector<const uint8_t *> ip;
  std::vector<uint8_t *> op, rp;
  for (int j = 0; j < k; ++j) {
    in.push_back(new Buf(len, (mis + j) % 16));
    in.back()->fill();
    ip.push_back(in.back()->p);
  }
  for (int r = 0; r < p; ++r) {
    out.push_back(new Buf(len, (mis + 3 * r) % 16));
    ref.push_back(new Buf(len));
    std::memset(out.back()->p, 0xA5, len);
    op.push_back(out.back()->p);
    rp.push_back(ref.back()->p);
  }
  CHECK(ozec_encode(enc, ip.data(), op.data(), len) == OZEC_OK, "encode k=%d p=%d len=%zu", k, p, len);
  if (codec == OZEC_CODEC_RS) {
    oracle_rs_encode(k, p, static_cast<int>(len), ip.data(), rp.data());
  } else {
    oracle_xor_encode(k, static_cast<int>(len), ip.data(), rp[0]);
    for (int r = 1; r < p; ++r) std::memset(rp[r], 0, len);
  }
  for (int r = 0; r < p; ++r) CHECK(!std::memcmp(op[r], rp[r], len), "parity %d k=%d p=%d len=%zu", r, k, p, len);
  // decode: erase data unit 0 and the last unit (RS), or unit 0 (XOR)
  std::vector<const uint8_t *> units(k + p, nullptr);
  for (int j = 0; j < k; ++j) units[j] = ip[j];
  for (int r = 0; r < p; ++r) units[k + r] = op[r];
  std::vector<int> erased = codec == OZEC_CODEC_RS && p > 1 ? std::vector<int>{0, k + p - 1} : std::vector<int>{0};
  for (int e : erased) units[e] = nullptr;
  std::vector<Buf *> dout;
  std::vector<uint8_t *> dp;
  for (size_t i = 0; i < erased.size(); ++i) {
    dout.push_back(new Buf(len, (mis + 5) % 16));
    dp.push_back(dout.back()->p);
  }
  CHECK(ozec_decode(dec, units.data(), erased.data(), static_cast<int>(erased.size()), dp.data(), len) == OZEC_OK,
        "decode");
  for (size_t i = 0; i < erased.size(); ++i) {
    const uint8_t *want = erased[i] < k ? ip[erased[i]] : op[erased[i] - k];
    CHECK(!std::memcmp(dp[i], want, len), "decoded unit %d len=%zu", erased[i], len);
  }
  for (auto *b : in) delete b;
  for (auto *b : out) delete b;
  for (auto *b : ref) delete b;
  for (auto *b : dout) delete b;
  ozec_coder_free(enc);
  ozec_coder_free(dec);
}

static void checksums(size_t len, size_t bpc, size_t mis) {
  for (int t : {OZEC_CHECKSUM_CRC32, OZEC_CHECKSUM_CRC32C}) {
    const int ot = t == OZEC_CHECKSUM_CRC32 ? 0 : 1;
    Buf d(len, mis);
    d.fill();
    const size_t nwin = (len + bpc - 1) / bpc;
    std::vector<uint32_t> got(nwin + 1, 0xdeadbeef), want(nwin + 1);
    uint32_t *gp = static_cast<uint32_t *>(std::malloc(sizeof(uint32_t) * (nwin ? nwin : 1)));
    CHECK(ozec_checksum_windows(t, d.p, len, bpc, gp, 0) == OZEC_OK, "windows len=%zu bpc=%zu", len, bpc);
    oracle_crc_windows(ot, d.p, len, bpc, want.data());
    for (size_t w = 0; w < nwin; ++w) CHECK(gp[w] == want[w], "crc%d window %zu len=%zu bpc=%zu", ot, w, len, bpc);
    int64_t bad = -2;
    if (nwin > 2) {
      d.p[bpc + 1] ^= 0x40;  // window 1 corrupted
      CHECK(ozec_checksum_verify(t, d.p, len, bpc, gp, nwin, 0, &bad) == OZEC_EMISMATCH && bad == 1,
            "verify reported %lld", static_cast<long long>(bad));
      d.p[bpc + 1] ^= 0x40;
    }
    std::free(gp);
    // streaming update in random pieces == one CRC of the whole buffer
    uint32_t st = ozec_crc_reset(t);
    for (size_t off = 0; off < len;) {
      const size_t piece = std::min<size_t>(len - off, 1 + rng() % (len / 3 + 1));
      Buf pb(piece, rng() % 16);
      std::memcpy(pb.p, d.p + off, piece);
      CHECK(ozec_crc_update(t, &st, pb.p, piece) == OZEC_OK, "update");
      off += piece;
    }
    CHECK(ozec_crc_value(t, st) == oracle_crc(ot, d.p, len), "streaming crc%d len=%zu", ot, len);
  }
}

// C5 host batch: S stripes in one pageable (or registered) allocation with padded strides
static void host_batch(bool registered) {
  ozec_coder *enc = nullptr;
  CHECK(ozec_encoder_create(OZEC_CODEC_RS, 6, 3, &enc) == OZEC_OK, "encoder");
  const int k = 6, p = 3;
  const size_t len = 65536, bpc = 16384, S = 37, nwin = len / bpc;
  const int64_t unit = len + 48, stripe = (k + p) * unit + 16;
  const size_t total = S * stripe;
  Buf batch(total, 0);
  batch.fill();
  const size_t ncrc = S * (k + p) * nwin;
  uint32_t *crcs = static_cast<uint32_t *>(std::malloc(ncrc * 4));
  if (registered) CHECK(ozec_host_register(batch.p, total, 0) == OZEC_OK, "register");
  CHECK(ozec_encode_crc_host_batch(enc, batch.p, stripe, unit, batch.p + k * unit, stripe, unit, S, len,
                                   OZEC_CHECKSUM_CRC32C, bpc, crcs, 0, 4) == OZEC_OK,
        "host batch");
  if (registered) CHECK(ozec_host_unregister(batch.p) == OZEC_OK, "unregister");
  for (size_t s = 0; s < S; ++s) {
    const uint8_t *in[6];
    std::vector<std::vector<uint8_t>> ref(p, std::vector<uint8_t>(len));
    uint8_t *rp[3] = {ref[0].data(), ref[1].data(), ref[2].data()};
    for (int j = 0; j < k; ++j) in[j] = batch.p + s * stripe + j * unit;
    oracle_rs_encode(k, p, static_cast<int>(len), in, rp);
    for (int r = 0; r < p; ++r)
      CHECK(!std::memcmp(batch.p + s * stripe + (k + r) * unit, rp[r], len), "stripe %zu parity %d", s, r);
    for (int u = 0; u < k + p; ++u) {
      uint32_t w[4];
      oracle_crc_windows(1, batch.p + s * stripe + u * unit, len, bpc, w);
      for (size_t i = 0; i < nwin; ++i) CHECK(crcs[(s * (k + p) + u) * nwin + i] == w[i], "stripe %zu unit %d crc", s, u);
    }
  }
  std::free(crcs);
  ozec_coder_free(enc);
}

// stripe queue: pageable cells of two lengths (a length change rotates the batch), waits out of order, free with
// stripes still pending
static void stripe_queue() {
  ozec_coder *enc = nullptr;
  CHECK(ozec_encoder_create(OZEC_CODEC_RS, 3, 2, &enc) == OZEC_OK, "encoder");
  const int k = 3, p = 2;
  const size_t cell = 1 << 16, bpc = 4096;
  ozec_stripe_queue *q = nullptr;
  CHECK(ozec_stripe_queue_create(enc, cell, 4, OZEC_CHECKSUM_CRC32, bpc, 1, &q) == OZEC_OK, "queue");
  struct Stripe {
    size_t len;
    std::vector<Buf *> d, par;
    uint32_t *crc;
    uint64_t ticket;
  };
  std::vector<Stripe> st(23);
  for (size_t i = 0; i < st.size(); ++i) {
    Stripe &s = st[i];
    s.len = i < 10 ? cell : cell - 4096 - 16 * (i % 3 == 0);
    const uint8_t *dp[3];
    uint8_t *pp[2];
    for (int j = 0; j < k; ++j) {
      s.d.push_back(new Buf(s.len, (i + j) % 7));
      s.d.back()->fill();
      dp[j] = s.d.back()->p;
    }
    for (int r = 0; r < p; ++r) {
      s.par.push_back(new Buf(s.len, r));
      pp[r] = s.par.back()->p;
    }
    const size_t nw = (s.len + bpc - 1) / bpc;
    s.crc = static_cast<uint32_t *>(std::malloc((k + p) * nw * 4));
    CHECK(ozec_stripe_queue_submit(q, dp, pp, s.len, s.crc, &s.ticket) == OZEC_OK, "submit %zu", i);
    if (i == 12) CHECK(ozec_stripe_queue_wait(q, st[5].ticket) == OZEC_OK, "wait");
  }
  CHECK(ozec_stripe_queue_wait(q, st[19].ticket) == OZEC_OK, "wait");
  CHECK(ozec_stripe_queue_free(q) == OZEC_OK, "free with pending stripes");  // completes 20..22
  for (size_t i = 0; i < st.size(); ++i) {
    Stripe &s = st[i];
    const uint8_t *dp[3] = {s.d[0]->p, s.d[1]->p, s.d[2]->p};
    std::vector<std::vector<uint8_t>> ref(p, std::vector<uint8_t>(s.len));
    uint8_t *rp[2] = {ref[0].data(), ref[1].data()};
    oracle_rs_encode(k, p, static_cast<int>(s.len), dp, rp);
    const size_t nw = (s.len + bpc - 1) / bpc;
    for (int r = 0; r < p; ++r) CHECK(!std::memcmp(s.par[r]->p, rp[r], s.len), "queued stripe %zu parity %d", i, r);
    for (int u = 0; u < k + p; ++u) {
      std::vector<uint32_t> w(nw);
      oracle_crc_windows(0, u < k ? dp[u] : rp[u - k], s.len, bpc, w.data());
      for (size_t x = 0; x < nw; ++x)
        CHECK(s.crc[u * nw + x] == __builtin_bswap32(w[x]), "queued stripe %zu unit %d crc", i, u);
    }
    for (auto *b : s.d) delete b;
    for (auto *b : s.par) delete b;
    std::free(s.crc);
  }
  ozec_coder_free(enc);
}

// reconstruction host batch (the new pipeline): pageable exact-size buffers, mixed erasures (several runs)
static void recon_batch(bool register_in) {
  ozec_coder *enc = nullptr, *dec = nullptr;
  const int k = 10, p = 4;
  CHECK(ozec_encoder_create(OZEC_CODEC_RS, k, p, &enc) == OZEC_OK, "encoder");
  CHECK(ozec_decoder_create(OZEC_CODEC_RS, k, p, &dec) == OZEC_OK, "decoder");
  const size_t len = 1 << 15, bpc = 4096, S = 11, nwin = len / bpc;
  const int64_t unit = len, stripe = (k + p) * unit;
  Buf batch(S * stripe, 0);
  batch.fill();
  for (size_t s = 0; s < S; ++s) {  // parity of every stripe from the oracle: the stored stripes are consistent
    const uint8_t *in[10];
    uint8_t *out[4];
    for (int j = 0; j < k; ++j) in[j] = batch.p + s * stripe + j * unit;
    for (int r = 0; r < p; ++r) out[r] = batch.p + s * stripe + (k + r) * unit;
    oracle_rs_encode(k, p, static_cast<int>(len), in, out);
  }
  std::vector<uint32_t> stored(S * (k + p) * nwin);
  for (size_t s = 0; s < S; ++s)
    for (int u = 0; u < k + p; ++u) oracle_crc_windows(1, batch.p + s * stripe + u * unit, len, bpc, &stored[(s * (k + p) + u) * nwin]);
  std::vector<uint8_t> orig(batch.p, batch.p + S * stripe);
  const int erased[4] = {1, 4, 10, 13};
  int present[10], np_ = 0;
  for (int u = 0; u < k + p; ++u)
    if (u != 1 && u != 4 && u != 10 && u != 13) present[np_++] = u;
  for (size_t s = 0; s < S; ++s)
    for (int e : erased) std::memset(batch.p + s * stripe + e * unit, 0xEE, len);
  Buf exp(S * (k + p) * nwin * 4, 1), out(S * 4 * len, 2), ocrc(S * 4 * nwin * 4, 3), mism(S * 4, 1);
  std::memcpy(exp.p, stored.data(), exp.n);
  if (register_in) CHECK(ozec_host_register(batch.p, batch.n, 0) == OZEC_OK, "register");
  CHECK(ozec_reconstruct_crc_host_batch(dec, batch.p, stripe, unit, present, np_, erased, 4, out.p, 4 * len, len, S, len,
                                        OZEC_CHECKSUM_CRC32C, bpc, reinterpret_cast<uint32_t *>(exp.p), 0,
                                        reinterpret_cast<uint32_t *>(ocrc.p), 0, reinterpret_cast<int32_t *>(mism.p),
                                        3) == OZEC_OK,
        "reconstruct host batch");
  if (register_in) CHECK(ozec_host_unregister(batch.p) == OZEC_OK, "unregister");
  for (size_t s = 0; s < S; ++s) {
    int32_t m;
    std::memcpy(&m, mism.p + 4 * s, 4);  // the caller's buffer is misaligned on purpose
    CHECK(m == -1, "stripe %zu mismatch %d", s, m);
    for (int i = 0; i < 4; ++i) {
      CHECK(!std::memcmp(out.p + (s * 4 + i) * len, orig.data() + s * stripe + erased[i] * unit, len), "rebuilt %zu/%d", s, i);
      CHECK(!std::memcmp(ocrc.p + (s * 4 + i) * nwin * 4, &stored[(s * (k + p) + erased[i]) * nwin], nwin * 4), "crc %zu/%d", s, i);
    }
  }
  ozec_coder_free(enc);
  ozec_coder_free(dec);
}

int main() {
  if (ozec_device_count() < 1) {
    std::printf("no GPU\n");
    return 2;
  }
  for (size_t len : {size_t{1}, size_t{15}, size_t{16}, size_t{4097}, size_t{(1 << 20) + 7}, size_t{5 << 20}})
    for (size_t mis : {size_t{0}, size_t{3}}) {
      encode_decode(OZEC_CODEC_RS, 6, 3, len, mis);
      encode_decode(OZEC_CODEC_RS, 10, 4, len, mis + 1);
      encode_decode(OZEC_CODEC_XOR, 2, 1, len, mis + 2);
    }
  for (size_t len : {size_t{1}, size_t{100}, size_t{16384}, size_t{50000}, size_t{(3 << 20) + 5}})
    for (size_t bpc : {size_t{512}, size_t{1000}, size_t{16384}}) checksums(len, bpc, len % 7);
  host_batch(false);
  host_batch(true);
  stripe_queue();
  recon_batch(false);
  recon_batch(true);
  std::printf("gpu host paths under ASan+UBSan: %s\n", g_fail ? "FAILED" : "ok");
  return g_fail ? 1 : 0;
}
