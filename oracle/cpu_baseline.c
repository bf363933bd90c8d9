/*
 * cpu_baseline.c -- TEST / BENCHMARK INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * Times the reference's CPU path on the host cores on a bounded sample of a bench workload, the way
 * RawErasureCoderBenchmark.performBench does (ECT/rawcoder/RawErasureCoderBenchmark.java:182-236; ECT =
 * hadoop-hdds/erasurecode/src/test/java/org/apache/ozone/erasurecode/): T threads share one coder (its tables
 * are built once, as in the RSRawEncoder constructor, EC/rawcoder/RSRawEncoder.java:39-58), every thread has its
 * own cells and repeats one unit of work until the wall budget is spent; throughput counts data bytes.
 *
 *   coding    : the oracle's restatement of RSUtil.encodeData / RSRawDecoder / XORRaw* (ozec_oracle.c), i.e. the
 *               rs_java coder's table loop (EC/rawcoder/util/RSUtil.java:87-133)
 *   CRC32C    : what the JDK's java.util.zip.CRC32C intrinsic does on x86 (ChecksumByteBufferFactory.java:74-89
 *               picks it at run time): the SSE4.2 crc32 instruction over three interleaved streams, the streams
 *               joined with zero-extension operators (no table-driven CrcIntTable)
 *   CRC32     : zlib's crc32 (the JDK's java.util.zip.CRC32 is zlib's algorithm)
 *
 * usage: cpu_baseline <workload> <threads> <seconds>    workload: c1 c2 c3 c3r c4 c5 crc verify crc32
 * prints one JSON object: units, seconds, data_bytes_per_unit, GB/s.
 */
#define _GNU_SOURCE
#include <nmmintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <zlib.h>

/* ozec_oracle.c (linked) */
void oracle_gen_cauchy_matrix(uint8_t *a, int m, int k);
void oracle_init_tables(int k, int rows, const uint8_t *matrix, int offset, uint8_t *gftables);
void oracle_encode_data(const uint8_t *gftables, int len, int num_in, const uint8_t *const *in, int num_out,
                        uint8_t *const *out);
int oracle_rs_decode_matrix(int k, int p, const int *valid, const int *erased, int n_erased, uint8_t *decode_matrix);
void oracle_xor_encode(int k, int len, const uint8_t *const *in, uint8_t *out);
uint32_t oracle_crc(int type, const uint8_t *b, size_t n);

#define MIB (1u << 20)
#define BPC 16384u

/* ------------------------------------------------------------------ CRC32C, hardware, 3 streams ---------- */
/* A raw CRC register followed by n zero bytes is a GF(2)-linear map of the register; tabulated per byte of the
 * register it costs 4 lookups.  Streams of SHORT bytes are joined with it. */
#define SHORT 256u
static uint32_t zeros_short[4][256];

static uint32_t gf2_times(const uint32_t *mat, uint32_t vec) {
  uint32_t sum = 0;
  for (int i = 0; vec; i++, vec >>= 1)
    if (vec & 1) sum ^= mat[i];
  return sum;
}

static void gf2_square(uint32_t *sq, const uint32_t *mat) {
  for (int n = 0; n < 32; n++) sq[n] = gf2_times(mat, mat[n]);
}

/* operator for `len` zero bytes (len a power of two times 1) */
static void zeros_op(uint32_t *even, size_t len) {
  uint32_t odd[32];
  odd[0] = 0x82F63B78u; /* one zero bit */
  uint32_t row = 1;
  for (int n = 1; n < 32; n++, row <<= 1) odd[n] = row;
  gf2_square(even, odd); /* 2 bits */
  gf2_square(odd, even); /* 4 bits */
  do {                   /* 8, 16, ... bits: len bytes */
    gf2_square(even, odd);
    len >>= 1;
    if (len == 0) return;
    gf2_square(odd, even);
    len >>= 1;
  } while (len);
  memcpy(even, odd, sizeof(odd));
}

static void zeros_table(uint32_t zeros[][256], size_t len) {
  uint32_t op[32];
  zeros_op(op, len);
  for (uint32_t n = 0; n < 256; n++) {
    zeros[0][n] = gf2_times(op, n);
    zeros[1][n] = gf2_times(op, n << 8);
    zeros[2][n] = gf2_times(op, n << 16);
    zeros[3][n] = gf2_times(op, n << 24);
  }
}

static inline uint32_t shift_crc(uint32_t zeros[][256], uint32_t crc) {
  return zeros[0][crc & 0xff] ^ zeros[1][(crc >> 8) & 0xff] ^ zeros[2][(crc >> 16) & 0xff] ^ zeros[3][crc >> 24];
}

static uint32_t crc32c_hw(const uint8_t *p, size_t n) {
  uint64_t c0 = 0xffffffffu;
  while (n >= 3 * SHORT) {
    uint64_t c1 = 0, c2 = 0;
    const uint8_t *end = p + SHORT;
    do {
      uint64_t a, b, c;
      memcpy(&a, p, 8);
      memcpy(&b, p + SHORT, 8);
      memcpy(&c, p + 2 * SHORT, 8);
      c0 = _mm_crc32_u64(c0, a);
      c1 = _mm_crc32_u64(c1, b);
      c2 = _mm_crc32_u64(c2, c);
      p += 8;
    } while (p < end);
    c0 = shift_crc(zeros_short, (uint32_t)c0) ^ (uint32_t)c1;
    c0 = shift_crc(zeros_short, (uint32_t)c0) ^ (uint32_t)c2;
    p += 2 * SHORT;
    n -= 3 * SHORT;
  }
  for (; n >= 8; n -= 8, p += 8) {
    uint64_t a;
    memcpy(&a, p, 8);
    c0 = _mm_crc32_u64(c0, a);
  }
  for (; n; n--) c0 = _mm_crc32_u8((uint32_t)c0, *p++);
  return ~(uint32_t)c0;
}

static void crc_windows(int crc32c, const uint8_t *d, size_t n, uint32_t *out) {
  for (size_t off = 0, w = 0; off < n; off += BPC, w++) {
    size_t l = n - off < BPC ? n - off : BPC;
    out[w] = crc32c ? crc32c_hw(d + off, l) : (uint32_t)crc32(0L, d + off, (uInt)l);
  }
}

/* ------------------------------------------------------------------ workloads ---------------------------- */
struct coder {
  int k, p;
  uint8_t enc_tabs[16 * 64 * 32];
  uint8_t dec_tabs[16 * 64 * 32];
  int erased[16], ne, valid[64];
};

static struct coder g_coder;
static const char *g_workload;
static double g_seconds;
static size_t g_data_bytes;

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void fill(uint8_t *d, size_t n, uint64_t seed) {
  uint64_t x = seed;
  for (size_t i = 0; i < n; i += 8) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    memcpy(d + i, &z, n - i < 8 ? n - i : 8);
  }
}

struct job {
  uint8_t *cells[32];
  uint32_t crcs[32][MIB / BPC];
  uint32_t stored[32][MIB / BPC];
  long units;
  int id;
};

static void encode(struct job *j, int k, int p) {
  for (int r = 0; r < p; r++) memset(j->cells[k + r], 0, MIB); /* CoderUtil.resetOutputBuffers */
  oracle_encode_data(g_coder.enc_tabs, MIB, k, (const uint8_t *const *)j->cells, p, j->cells + k);
}

static int run_unit(struct job *j) {
  const char *w = g_workload;
  struct coder *c = &g_coder;
  if (!strcmp(w, "c1") || !strcmp(w, "c2")) {
    encode(j, c->k, c->p);
  } else if (!strcmp(w, "c3") || !strcmp(w, "c3r")) {
    const uint8_t *in[16];
    for (int i = 0; i < c->k; i++) in[i] = j->cells[c->valid[i]];
    uint8_t *out[4] = {j->cells[14], j->cells[15], j->cells[16], j->cells[17]};
    if (!strcmp(w, "c3r"))  /* ChunkInputStream verify of the units read */
      for (int i = 0; i < c->k; i++) {
        crc_windows(1, in[i], MIB, j->crcs[i]);
        if (memcmp(j->crcs[i], j->stored[c->valid[i]], sizeof(j->crcs[i]))) return -1;
      }
    for (int r = 0; r < c->ne; r++) memset(out[r], 0, MIB);
    oracle_encode_data(c->dec_tabs, MIB, c->k, in, c->ne, out);
    if (!strcmp(w, "c3r"))  /* BlockOutputStream CRC of the rebuilt units */
      for (int r = 0; r < c->ne; r++) crc_windows(1, out[r], MIB, j->crcs[16 + r]);
  } else if (!strcmp(w, "c4")) {
    oracle_xor_encode(2, MIB, (const uint8_t *const *)j->cells, j->cells[2]); /* XORRawEncoder.doEncode */
    for (int u = 0; u < 3; u++) crc_windows(1, j->cells[u], MIB, j->crcs[u]);
  } else if (!strcmp(w, "c5")) {
    encode(j, 6, 3);
    for (int u = 0; u < 9; u++) crc_windows(1, j->cells[u], MIB, j->crcs[u]);
  } else if (!strcmp(w, "crc") || !strcmp(w, "crc32")) {
    crc_windows(!strcmp(w, "crc"), j->cells[0], MIB, j->crcs[0]);
  } else if (!strcmp(w, "verify")) {
    crc_windows(1, j->cells[0], MIB, j->crcs[0]);
    if (memcmp(j->crcs[0], j->stored[0], sizeof(j->crcs[0]))) return -1;
  }
  return 0;
}

static double g_stop;

/* one percall_windows thread: its own buffer, every 16 KiB window CRC32C'd, until `secs` have passed */
static void *percall_windows_thread(void *arg) {
  struct pw { size_t n; double secs; long calls; double t; uint32_t sink; } *j = arg;
  uint8_t *buf = aligned_alloc(4096, (j->n + 4095) / 4096 * 4096);
  fill(buf, j->n, 31);
  const double t0 = now();
  double t = t0;
  uint32_t sink = 0;
  do {
    for (size_t off = 0; off < j->n; off += BPC) sink ^= crc32c_hw(buf + off, j->n - off < BPC ? j->n - off : BPC);
    j->calls++;
    t = now();
  } while (t - t0 < j->secs);
  j->t = t - t0;
  j->sink = sink;
  free(buf);
  return NULL;
}

static void *worker(void *arg) {
  struct job *j = arg;
  while (now() < g_stop) {
    if (run_unit(j)) {
      j->units = -1;
      return NULL;
    }
    j->units++;
  }
  return NULL;
}

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s <workload> <threads> <seconds>\n", argv[0]);
    return 2;
  }
  g_workload = argv[1];
  if (!strcmp(g_workload, "percall_windows")) {
    /* Checksum.computeChecksum of one n-byte buffer: CRC32C of every 16 KiB window (the JDK-class SSE4.2 CRC per
     * window), from T threads at once, each on its own buffer: usage percall_windows <bytes> <seconds> [threads] */
    const size_t n = (size_t)atol(argv[2]);
    const double secs = atof(argv[3]);
    const int T = argc > 4 && atoi(argv[4]) > 0 ? atoi(argv[4]) : 1;
    pthread_t th[256];
    struct pw { size_t n; double secs; long calls; double t; uint32_t sink; } jobs[256];
    void *(*run)(void *) = percall_windows_thread;
    for (int i = 0; i < T && i < 256; i++) {
      jobs[i] = (struct pw){n, secs, 0, 0, 0};
      pthread_create(&th[i], NULL, run, &jobs[i]);
    }
    long calls = 0;
    double tmax = 0;
    uint32_t sink = 0;
    for (int i = 0; i < T && i < 256; i++) {
      pthread_join(th[i], NULL);
      calls += jobs[i].calls;
      tmax = jobs[i].t > tmax ? jobs[i].t : tmax;
      sink ^= jobs[i].sink;
    }
    printf("{\"workload\": \"%s\", \"bytes\": %zu, \"threads\": %d, \"calls\": %ld, \"us_per_call\": %.3f, "
           "\"GBps\": %.3f, \"sink\": %u}\n", g_workload, n, T, calls, tmax / ((double)calls / T) * 1e6,
           (double)calls * n / tmax / 1e9, sink);
    return 0;
  }
  if (!strcmp(g_workload, "percall_crc32c") || !strcmp(g_workload, "percall_encode")) {
    /* per-call cost of one ChecksumByteBuffer.update(n bytes) / one rs-6-3 stripe encode of n-byte cells,
     * single thread (the JDK intrinsic / rs_java call a Java writer makes): usage percall_* <bytes> <seconds> */
    const size_t n = (size_t)atol(argv[2]);
    const double secs = atof(argv[3]);
    zeros_table(zeros_short, SHORT);
    const int enc = !strcmp(g_workload, "percall_encode");
    uint8_t *cells[9];
    for (int u = 0; u < 9; u++) {
      cells[u] = aligned_alloc(4096, (n + 4095) / 4096 * 4096);
      fill(cells[u], n, 77 + u);
    }
    if (enc) {
      uint8_t mat[9 * 6];
      oracle_gen_cauchy_matrix(mat, 9, 6);
      oracle_init_tables(6, 3, mat, 36, g_coder.enc_tabs);
    }
    volatile uint32_t sink = 0;
    long calls = 0;
    const double t0 = now();
    double t = t0;
    do {
      for (int r = 0; r < 16; r++, calls++) {
        if (enc) {
          for (int q = 0; q < 3; q++) memset(cells[6 + q], 0, n);
          oracle_encode_data(g_coder.enc_tabs, (int)n, 6, (const uint8_t *const *)cells, 3, cells + 6);
          sink ^= cells[6][0];
        } else {
          sink ^= crc32c_hw(cells[0], n);
        }
      }
      t = now();
    } while (t - t0 < secs);
    printf("{\"workload\": \"%s\", \"bytes\": %zu, \"calls\": %ld, \"us_per_call\": %.3f, \"sink\": %u}\n",
           g_workload, n, calls, (t - t0) / calls * 1e6, sink);
    return 0;
  }
  int T = atoi(argv[2]);
  g_seconds = atof(argv[3]);
  if (T < 1) T = 1;
  zeros_table(zeros_short, SHORT);
  { /* the fast CRCs must equal the oracle's CrcIntTable restatement before they are timed */
    static uint8_t buf[3 * BPC];
    fill(buf, sizeof(buf), 99);
    const size_t lens[] = {0, 1, 7, 8, 255, 767, 768, 769, 4096, BPC - 1, BPC, BPC + 3, 3 * BPC};
    for (size_t i = 0; i < sizeof(lens) / sizeof(lens[0]); i++)
      if (crc32c_hw(buf + 1, lens[i] - (lens[i] == 3 * BPC)) != oracle_crc(1, buf + 1, lens[i] - (lens[i] == 3 * BPC)) ||
          (uint32_t)crc32(0L, buf, (uInt)lens[i]) != oracle_crc(0, buf, lens[i])) {
        fprintf(stderr, "CRC self-check failed at length %zu\n", lens[i]);
        return 4;
      }
  }
  struct coder *c = &g_coder;
  const char *w = g_workload;
  int ncells = 1;
  if (!strcmp(w, "c1")) c->k = 3, c->p = 2, ncells = 5, g_data_bytes = 3ull * MIB;
  else if (!strcmp(w, "c2") || !strcmp(w, "c5")) c->k = 6, c->p = 3, ncells = 9, g_data_bytes = 6ull * MIB;
  else if (!strcmp(w, "c3") || !strcmp(w, "c3r")) c->k = 10, c->p = 4, ncells = 18, g_data_bytes = 10ull * MIB;
  else if (!strcmp(w, "c4")) c->k = 2, c->p = 1, ncells = 3, g_data_bytes = 2ull * MIB;
  else if (!strcmp(w, "crc") || !strcmp(w, "verify") || !strcmp(w, "crc32")) ncells = 1, g_data_bytes = MIB;
  else {
    fprintf(stderr, "unknown workload %s\n", w);
    return 2;
  }
  if (c->k) {
    uint8_t mat[64 * 64];
    oracle_gen_cauchy_matrix(mat, c->k + c->p, c->k);
    oracle_init_tables(c->k, c->p, mat, c->k * c->k, c->enc_tabs);
  }
  if (c->k == 10) { /* decode erasing {0,1,2,3}: the first 10 valid are 4..13 (RSRawDecoder.java:79-82) */
    c->ne = 4;
    for (int i = 0; i < 4; i++) c->erased[i] = i;
    for (int i = 0; i < 10; i++) c->valid[i] = 4 + i;
    uint8_t dm[4 * 10];
    if (oracle_rs_decode_matrix(10, 4, c->valid, c->erased, 4, dm)) return 3;
    oracle_init_tables(10, 4, dm, 0, c->dec_tabs);
  }
  struct job *jobs = calloc((size_t)T, sizeof(struct job));
  pthread_t *th = calloc((size_t)T, sizeof(pthread_t));
  for (int t = 0; t < T; t++) {
    jobs[t].id = t;
    for (int u = 0; u < ncells; u++) {
      jobs[t].cells[u] = aligned_alloc(4096, MIB);
      fill(jobs[t].cells[u], MIB, 0x00EC5EEDull * 1000003ull + (uint64_t)t * 64 + u);
    }
    if (c->k == 10) { /* a valid stripe, its stored CRCs for the verify step */
      encode(&jobs[t], 10, 4);
      for (int u = 0; u < 14; u++) crc_windows(1, jobs[t].cells[u], MIB, jobs[t].stored[u]);
    }
    if (!strcmp(w, "verify")) crc_windows(1, jobs[t].cells[0], MIB, jobs[t].stored[0]);
    if (run_unit(&jobs[t])) { /* warm: tables and pages */
      fprintf(stderr, "self-check failed\n");
      return 4;
    }
  }
  double t0 = now();
  g_stop = t0 + g_seconds;
  for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, worker, &jobs[t]);
  long units = 0;
  for (int t = 0; t < T; t++) {
    pthread_join(th[t], NULL);
    if (jobs[t].units < 0) return 5;
    units += jobs[t].units;
  }
  double el = now() - t0;
  printf("{\"workload\": \"%s\", \"threads\": %d, \"units\": %ld, \"seconds\": %.4f, \"data_bytes_per_unit\": %zu, "
         "\"GBps\": %.4f}\n",
         w, T, units, el, g_data_bytes, units * (double)g_data_bytes / el / 1e9);
  return 0;
}
