/*
 * ozec_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference (Apache Ozone @ 2024-10-08) CPU algorithms for the
 * erasure-coding + chunk-checksum hot path.  It is the CHECKER for the HIP product path and the
 * `cpu_baseline` leg of bench.py ("kind": "port"); nothing in ozone_amd/ links, loads or calls it.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use it.
 *
 * Parity pinning (see tests/golden/make_golden.py and DESIGN.md "Oracle"):
 *   - GF(2^8) exp/log tables are generated from poly 0x11d and checked byte-for-byte against the literal
 *     tables in GF256.java:31-139 (sha256 recorded in tests/golden/ref_pins.json);
 *   - CRC slice-by-8 tables are generated from the reflected polys and checked against the literal
 *     tables of PureJavaCrc32ByteBuffer.java / PureJavaCrc32CByteBuffer.java (sha256 recorded);
 *   - Cauchy parity rows are checked against SURVEY.md Appendix B (derived from the reference tables);
 *   - CRC check values "123456789" -> CRC-32 0xCBF43926 / CRC-32C 0xE3069283; CRC-32 vs zlib.crc32.
 *   - a second, independent pure-Python restatement (tests/golden/pyref.py) produced the committed
 *     golden vectors; this C oracle must agree with them byte-for-byte.
 *
 * Reference paths below are relative to /root/reference/:
 *   EC/ = hadoop-hdds/erasurecode/src/main/java/org/apache/ozone/erasurecode/
 *   CM/ = hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- GF(2^8) -------------------- */

static uint8_t GF_BASE[256];     /* EC/rawcoder/util/GF256.java:31-84   2^i mod 0x11d, [255] = 1   */
static uint8_t GF_LOG_BASE[256]; /* EC/rawcoder/util/GF256.java:86-139  log, with [0]=0, [1]=0xff    */
static uint8_t GF_MUL_TAB[256][256]; /* EC/rawcoder/util/GF256.java:141-154 theGfMulTab              */
static int gf_ready = 0;

static uint8_t gf_mul_raw(uint8_t a, uint8_t b) {
  /* GF256.gfMul, EC/rawcoder/util/GF256.java:164-176 */
  if (a == 0 || b == 0) return 0;
  int tmp = GF_LOG_BASE[a] + GF_LOG_BASE[b];
  if (tmp > 254) tmp -= 255;
  return GF_BASE[tmp];
}

static void gf_init(void) {
  if (gf_ready) return;
  unsigned x = 1;
  for (int i = 0; i < 255; i++) {
    GF_BASE[i] = (uint8_t)x;
    x <<= 1;
    if (x & 0x100) x ^= 0x11d; /* primitive polynomial 285, RSUtil.java:34-37 */
  }
  GF_BASE[255] = 1;
  memset(GF_LOG_BASE, 0, sizeof GF_LOG_BASE);
  for (int i = 1; i < 255; i++) GF_LOG_BASE[GF_BASE[i]] = (uint8_t)i;
  GF_LOG_BASE[1] = 0xff; /* the reference table stores log(1) as 255 (GF256.java:87) */
  for (int i = 0; i < 256; i++)
    for (int j = 0; j < 256; j++) GF_MUL_TAB[i][j] = gf_mul_raw((uint8_t)i, (uint8_t)j);
  gf_ready = 1;
}

void oracle_gf_tables(uint8_t *base, uint8_t *logb) {
  gf_init();
  memcpy(base, GF_BASE, 256);
  memcpy(logb, GF_LOG_BASE, 256);
}

uint8_t oracle_gf_mul(uint8_t a, uint8_t b) { gf_init(); return gf_mul_raw(a, b); }

uint8_t oracle_gf_inv(uint8_t a) {
  /* GF256.gfInv, GF256.java:178-184: GF_BASE[255 - GF_LOG_BASE[a & 0xff] & 0xff]; Java precedence is
   * (255 - log) & 0xff with log a SIGNED byte, i.e. (255 - (int8_t)log) & 0xff. */
  gf_init();
  if (a == 0) return 0;
  int lg = (int8_t)GF_LOG_BASE[a];
  return GF_BASE[(255 - lg) & 0xff];
}

/* GF256.gfInvertMatrix, GF256.java:191-250. Mutates `in`. Returns 0, or -1 ("Not invertible"). */
int oracle_gf_invert_matrix(uint8_t *in, uint8_t *out, int n) {
  gf_init();
  for (int i = 0; i < n * n; i++) out[i] = 0;
  for (int i = 0; i < n; i++) out[i * n + i] = 1;
  for (int i = 0; i < n; i++) {
    if (in[i * n + i] == 0) {
      int j;
      for (j = i + 1; j < n; j++)
        if (in[j * n + i] != 0) break;
      if (j == n) return -1;
      for (int k = 0; k < n; k++) {
        uint8_t t = in[i * n + k]; in[i * n + k] = in[j * n + k]; in[j * n + k] = t;
        t = out[i * n + k]; out[i * n + k] = out[j * n + k]; out[j * n + k] = t;
      }
    }
    uint8_t piv = oracle_gf_inv(in[i * n + i]);
    for (int j = 0; j < n; j++) {
      in[i * n + j] = gf_mul_raw(in[i * n + j], piv);
      out[i * n + j] = gf_mul_raw(out[i * n + j], piv);
    }
    for (int j = 0; j < n; j++) {
      if (j == i) continue;
      uint8_t t = in[j * n + i];
      for (int k = 0; k < n; k++) {
        out[j * n + k] ^= gf_mul_raw(t, out[i * n + k]);
        in[j * n + k] ^= gf_mul_raw(t, in[i * n + k]);
      }
    }
  }
  return 0;
}

/* GF256.gfVectMulInit, GF256.java:259-330: tbl[0..15] = c*{0..15}, tbl[16..31] = c*{0x00,0x10..0xf0} */
void oracle_gf_vect_mul_init(uint8_t c, uint8_t *tbl) {
  gf_init();
  for (int i = 0; i < 16; i++) {
    tbl[i] = gf_mul_raw(c, (uint8_t)i);
    tbl[16 + i] = gf_mul_raw(c, (uint8_t)(i << 4));
  }
}

/* RSUtil.genCauchyMatrix, EC/rawcoder/util/RSUtil.java:64-77; a is m x k, zero-initialised here. */
void oracle_gen_cauchy_matrix(uint8_t *a, int m, int k) {
  gf_init();
  memset(a, 0, (size_t)m * k);
  for (int i = 0; i < k; i++) a[k * i + i] = 1;
  int pos = k * k;
  for (int i = k; i < m; i++)
    for (int j = 0; j < k; j++) a[pos++] = oracle_gf_inv((uint8_t)(i ^ j));
}

/* RSUtil.initTables, RSUtil.java:48-59 */
void oracle_init_tables(int k, int rows, const uint8_t *matrix, int offset, uint8_t *gftables) {
  int idx = offset, off = 0;
  for (int i = 0; i < rows; i++)
    for (int j = 0; j < k; j++) {
      oracle_gf_vect_mul_init(matrix[idx++], gftables + off);
      off += 32;
    }
}

/* RSUtil.encodeData(byte[] gfTables, int dataLen, byte[][] inputs, int[] inOff, byte[][] outputs, int[] outOff)
 * RSUtil.java:87-133.  out[l][x] ^= MulTab[gfTables[j*32 + l*numInputs*32 + 1]][in[j][x]].  Outputs are
 * accumulated into (the caller zero-fills, CoderUtil.resetOutputBuffers, CoderUtil.java:84-98). */
void oracle_encode_data(const uint8_t *gftables, int len, int num_in, const uint8_t *const *in,
                        int num_out, uint8_t *const *out) {
  gf_init();
  for (int l = 0; l < num_out; l++) {
    uint8_t *o = out[l];
    for (int j = 0; j < num_in; j++) {
      const uint8_t *x = in[j];
      const uint8_t *line = GF_MUL_TAB[gftables[j * 32 + l * num_in * 32 + 1]];
      int times = len / 8, i = 0;
      for (int t = 0; t < times; t++, i += 8) {
        o[i + 0] ^= line[x[i + 0]]; o[i + 1] ^= line[x[i + 1]];
        o[i + 2] ^= line[x[i + 2]]; o[i + 3] ^= line[x[i + 3]];
        o[i + 4] ^= line[x[i + 4]]; o[i + 5] ^= line[x[i + 5]];
        o[i + 6] ^= line[x[i + 6]]; o[i + 7] ^= line[x[i + 7]];
      }
      for (; i < len; i++) o[i] ^= line[x[i]];
    }
  }
}

/* RSRawEncoder ctor + doEncode, EC/rawcoder/RSRawEncoder.java:39-76.  Returns -1 if k+p >= 256. */
int oracle_rs_encode(int k, int p, int len, const uint8_t *const *in, uint8_t *const *out) {
  if (k + p >= 256) return -1;
  uint8_t *mat = (uint8_t *)malloc((size_t)(k + p) * k);
  uint8_t *tabs = (uint8_t *)malloc((size_t)(k + p) * k * 32);
  oracle_gen_cauchy_matrix(mat, k + p, k);
  oracle_init_tables(k, p, mat, k * k, tabs);
  for (int l = 0; l < p; l++) memset(out[l], 0, (size_t)len);
  oracle_encode_data(tabs, len, k, in, p, out);
  free(mat);
  free(tabs);
  return 0;
}

/* RSRawDecoder.generateDecodeMatrix + processErasures, EC/rawcoder/RSRawDecoder.java:117-176.
 * valid[0..k-1] = first k non-null input indexes (CoderUtil.getValidIndexes, CoderUtil.java:163-173).
 * decode_matrix receives n_erased x k rows. Reproduces the reference's ordering quirk: rows for slots
 * i < numErasedDataUnits read invertMatrix[k*erased[i]...], which lies in the zero tail of the (k+p)*k
 * array when erased[i] >= k.  Returns 0 / -1 (not invertible). */
int oracle_rs_decode_matrix(int k, int p, const int *valid, const int *erased, int n_erased,
                            uint8_t *decode_matrix) {
  gf_init();
  int n_all = k + p;
  uint8_t *enc = (uint8_t *)calloc((size_t)n_all * k, 1);
  uint8_t *tmp = (uint8_t *)calloc((size_t)n_all * k, 1);
  uint8_t *inv = (uint8_t *)calloc((size_t)n_all * k, 1);
  uint8_t *dec = (uint8_t *)calloc((size_t)n_all * k, 1);
  oracle_gen_cauchy_matrix(enc, n_all, k);
  int n_erased_data = 0;
  for (int i = 0; i < n_erased; i++)
    if (erased[i] < k) n_erased_data++;
  for (int i = 0; i < k; i++) {
    int r = valid[i];
    for (int j = 0; j < k; j++) tmp[k * i + j] = enc[k * r + j];
  }
  int rc = oracle_gf_invert_matrix(tmp, inv, k);
  if (rc == 0) {
    for (int i = 0; i < n_erased_data; i++)
      for (int j = 0; j < k; j++) {
        int idx = k * erased[i] + j; /* may index the zero tail, as in the reference */
        dec[k * i + j] = idx < n_all * k ? inv[idx] : 0;
      }
    for (int pp = n_erased_data; pp < n_erased; pp++)
      for (int i = 0; i < k; i++) {
        uint8_t s = 0;
        for (int j = 0; j < k; j++) s ^= gf_mul_raw(inv[j * k + i], enc[k * erased[pp] + j]);
        dec[k * pp + i] = s;
      }
    memcpy(decode_matrix, dec, (size_t)n_erased * k);
  }
  free(enc); free(tmp); free(inv); free(dec);
  return rc;
}

/* RSRawDecoder.doDecode(ByteArrayDecodingState), RSRawDecoder.java:87-101.
 * inputs: k+p slots, NULL = erased / not read.  Returns 0, -1 not invertible, -2 too few inputs. */
int oracle_rs_decode(int k, int p, int len, const uint8_t *const *inputs, const int *erased,
                     int n_erased, uint8_t *const *outputs) {
  int valid[256], nv = 0;
  for (int i = 0; i < k + p; i++)
    if (inputs[i]) valid[nv++] = i;
  if (nv < k) return -2;
  uint8_t *dm = (uint8_t *)calloc((size_t)(n_erased ? n_erased : 1) * k, 1);
  int rc = oracle_rs_decode_matrix(k, p, valid, erased, n_erased, dm);
  if (rc == 0) {
    uint8_t *tabs = (uint8_t *)malloc((size_t)(n_erased ? n_erased : 1) * k * 32);
    oracle_init_tables(k, n_erased, dm, 0, tabs);
    const uint8_t *real[256];
    for (int i = 0; i < k; i++) real[i] = inputs[valid[i]];
    for (int l = 0; l < n_erased; l++) memset(outputs[l], 0, (size_t)len);
    oracle_encode_data(tabs, len, k, real, n_erased, outputs);
    free(tabs);
  }
  free(dm);
  return rc;
}

/* XORRawEncoder.doEncode, EC/rawcoder/XORRawEncoder.java:65-85 */
void oracle_xor_encode(int k, int len, const uint8_t *const *in, uint8_t *out) {
  memcpy(out, in[0], (size_t)len);
  for (int i = 1; i < k; i++)
    for (int x = 0; x < len; x++) out[x] ^= in[i][x];
}

/* XORRawDecoder.doDecode, EC/rawcoder/XORRawDecoder.java:65-86: XOR every input except erased[0].
 * Returns -2 if a non-erased slot is NULL (the reference would NPE). */
int oracle_xor_decode(int n_units, int len, const uint8_t *const *inputs, int erased0, uint8_t *out) {
  memset(out, 0, (size_t)len);
  for (int i = 0; i < n_units; i++) {
    if (i == erased0) continue;
    if (!inputs[i]) return -2;
    for (int x = 0; x < len; x++) out[x] ^= inputs[i][x];
  }
  return 0;
}

/* ---------------------------------------------------------------- CRC ------------------------ */
/* ChecksumByteBuffer.CrcIntTable, CM/ChecksumByteBuffer.java:51-121; tables T8_0..T8_7 laid out as
 * T[0x000..0x7FF] exactly like PureJavaCrc32ByteBuffer.java (poly 0xEDB88320) and
 * PureJavaCrc32CByteBuffer.java (poly 0x82F63B78). type 0 = CRC32, 1 = CRC32C. */
static uint32_t CRC_T[2][0x800];
static int crc_ready = 0;

static void crc_init(void) {
  if (crc_ready) return;
  const uint32_t polys[2] = {0xEDB88320u, 0x82F63B78u};
  for (int t = 0; t < 2; t++) {
    for (uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for (int b = 0; b < 8; b++) c = (c & 1) ? (c >> 1) ^ polys[t] : (c >> 1);
      CRC_T[t][i] = c;
    }
    for (int s = 1; s < 8; s++)
      for (int i = 0; i < 256; i++) {
        uint32_t prev = CRC_T[t][(s - 1) * 256 + i];
        CRC_T[t][s * 256 + i] = (prev >> 8) ^ CRC_T[t][prev & 0xff];
      }
  }
  crc_ready = 1;
}

void oracle_crc_table(int type, uint32_t *out2048) {
  crc_init();
  memcpy(out2048, CRC_T[type], sizeof(uint32_t) * 0x800);
}

/* CrcIntTable.update(int crc, ByteBuffer b, int[] table), ChecksumByteBuffer.java:82-120: raw state update */
uint32_t oracle_crc_update(int type, uint32_t crc, const uint8_t *b, size_t n) {
  crc_init();
  const uint32_t *T = CRC_T[type];
  size_t i = 0;
  for (; n - i > 7; i += 8) {
    uint32_t c0 = (b[i + 0] ^ crc) & 0xff;
    uint32_t c1 = (b[i + 1] ^ (crc >>= 8)) & 0xff;
    uint32_t c2 = (b[i + 2] ^ (crc >>= 8)) & 0xff;
    uint32_t c3 = (b[i + 3] ^ (crc >> 8)) & 0xff;
    crc = (T[0x700 + c0] ^ T[0x600 + c1]) ^ (T[0x500 + c2] ^ T[0x400 + c3]);
    uint32_t c4 = b[i + 4], c5 = b[i + 5], c6 = b[i + 6], c7 = b[i + 7];
    crc ^= (T[0x300 + c4] ^ T[0x200 + c5]) ^ (T[0x100 + c6] ^ T[c7]);
  }
  for (; i < n; i++) crc = (crc >> 8) ^ T[(crc ^ b[i]) & 0xff];
  return crc;
}

/* reset(); update(window); getValue()  -- CrcIntTable.reset/getValue, ChecksumByteBuffer.java:66-75 */
uint32_t oracle_crc(int type, const uint8_t *b, size_t n) {
  return ~oracle_crc_update(type, 0xffffffffu, b, n);
}

/* Checksum.computeChecksum(ChunkBuffer), CM/Checksum.java:157-200 with ChunkBufferImplWithByteBuffer.iterate
 * (CM/ChunkBufferImplWithByteBuffer.java:78-98): one CRC per bpc window from offset 0, last window short.
 * Writes ceil(n/bpc) values (the (int)getValue() ints; Checksum.int2ByteString stores them big-endian). */
size_t oracle_crc_windows(int type, const uint8_t *data, size_t n, size_t bpc, uint32_t *out) {
  size_t w = 0;
  for (size_t off = 0; off < n; off += bpc) {
    size_t len = n - off < bpc ? n - off : bpc;
    out[w++] = oracle_crc(type, data + off, len);
  }
  return w;
}

/* ---------------------------------------------------------------- COMPOSITE_CRC ---------------- */
/* OC/ = hadoop-ozone/common/src/main/java/org/apache/hadoop/ozone/client/checksum/
 * CRC values here are the stored ints ((int)getValue()), in the reference's "reversed" representation:
 * bit 31 is the x^0 coefficient, bit 0 the x^31 one; MULTIPLICATIVE_IDENTITY = 0x80000000 (OC/CrcUtil.java:34). */

/* CrcUtil.getCrcPolynomialForType, OC/CrcUtil.java:53-64 */
uint32_t oracle_crc_poly(int type) { return type == 0 ? 0xEDB88320u : 0x82F63B78u; }

/* CrcUtil.galoisFieldMultiply, OC/CrcUtil.java:249-270: p * q mod m, bit-serial */
uint32_t oracle_gf32_multiply(uint32_t p, uint32_t q, uint32_t m) {
  uint32_t summation = 0, cur_term = 0x80000000u, px = p;
  while (cur_term != 0) {
    if (q & cur_term) summation ^= px;
    int has_max_degree = (px & 1) != 0;
    px >>= 1;
    if (has_max_degree) px ^= m;
    cur_term >>= 1;
  }
  return summation;
}

/* CrcUtil.getMonomial, OC/CrcUtil.java:74-98: x^(8*len) mod m by square-and-multiply from x^8.
 * Returns -1 (IllegalArgumentException) for len < 0. */
int oracle_crc_monomial(int64_t len, uint32_t m, uint32_t *out) {
  if (len == 0) { *out = 0x80000000u; return 0; }
  if (len < 0) return -1;
  uint32_t multiplier = 0x80000000u >> 8, product = 0x80000000u;
  int64_t degree = len;
  while (degree > 0) {
    if (degree & 1) product = product == 0x80000000u ? multiplier : oracle_gf32_multiply(product, multiplier, m);
    multiplier = oracle_gf32_multiply(multiplier, multiplier, m);
    degree >>= 1;
  }
  *out = product;
  return 0;
}

/* CrcUtil.compose / composeWithMonomial, OC/CrcUtil.java:110-127 */
int oracle_crc_compose(uint32_t crc_a, uint32_t crc_b, int64_t len_b, uint32_t m, uint32_t *out) {
  uint32_t mono;
  if (oracle_crc_monomial(len_b, m, &mono)) return -1;
  *out = oracle_gf32_multiply(crc_a, mono, m) ^ crc_b;
  return 0;
}

/* CrcComposer, OC/CrcComposer.java:44-215 */
typedef struct {
  uint32_t poly, mono_hint;
  int64_t hint, stripe_len, pos;
  uint32_t cur;
  uint8_t *digest;
  size_t dlen, dcap;
} oracle_composer;

static void composer_emit(oracle_composer *c) {
  if (c->dlen + 4 > c->dcap) {
    c->dcap = c->dcap ? 2 * c->dcap : 64;
    c->digest = (uint8_t *)realloc(c->digest, c->dcap);
  }
  /* CrcUtil.intToBytes / writeInt, OC/CrcUtil.java:135-175: big-endian */
  c->digest[c->dlen++] = (uint8_t)(c->cur >> 24);
  c->digest[c->dlen++] = (uint8_t)(c->cur >> 16);
  c->digest[c->dlen++] = (uint8_t)(c->cur >> 8);
  c->digest[c->dlen++] = (uint8_t)c->cur;
}

/* newStripedCrcComposer, OC/CrcComposer.java:84-95 (newCrcComposer = stripe length Long.MAX_VALUE, :61-66) */
oracle_composer *oracle_composer_new(int type, int64_t bytes_per_crc_hint, int64_t stripe_length) {
  oracle_composer *c = (oracle_composer *)calloc(1, sizeof(oracle_composer));
  c->poly = oracle_crc_poly(type);
  if (oracle_crc_monomial(bytes_per_crc_hint, c->poly, &c->mono_hint)) { free(c); return NULL; }
  c->hint = bytes_per_crc_hint;
  c->stripe_len = stripe_length;
  return c;
}

/* update(int crcB, long bytesPerCrc), OC/CrcComposer.java:168-199.
 * 0 ok, -1 negative length (IllegalArgumentException), -2 stripe overrun (IOException). */
int oracle_composer_update(oracle_composer *c, uint32_t crc_b, int64_t bytes_per_crc) {
  if (c->cur == 0) {
    c->cur = crc_b;
  } else if (bytes_per_crc == c->hint) {
    c->cur = oracle_gf32_multiply(c->cur, c->mono_hint, c->poly) ^ crc_b;
  } else {
    if (oracle_crc_compose(c->cur, crc_b, bytes_per_crc, c->poly, &c->cur)) return -1;
  }
  c->pos += bytes_per_crc;
  if (c->pos > c->stripe_len) return -2;
  if (c->pos == c->stripe_len) {
    composer_emit(c);
    c->cur = 0;
    c->pos = 0;
  }
  return 0;
}

/* digest(), OC/CrcComposer.java:205-214: flush a partial stripe, return and reset the digest */
size_t oracle_composer_digest(oracle_composer *c, uint8_t *out, size_t cap) {
  if (c->pos > 0) {
    composer_emit(c);
    c->cur = 0;
    c->pos = 0;
  }
  size_t n = c->dlen < cap ? c->dlen : cap;
  if (out && n) memcpy(out, c->digest, n);
  size_t all = c->dlen;
  c->dlen = 0;
  return all;
}

void oracle_composer_free(oracle_composer *c) {
  if (!c) return;
  free(c->digest);
  free(c);
}

/* bytes the next digest() returns (test helper) */
size_t oracle_composer_pending(const oracle_composer *c) { return c->dlen + (c->pos > 0 ? 4 : 0); }
