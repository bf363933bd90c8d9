/*
 * Per-call timing of the Java drop-in's production path: jni/ozec_jni.c's encodeArrays /
 * decodeArrays on heap byte[] cells, driven through the JNI test double (tests/native/mockjni) exactly as
 * OzecNative's natives are called by AbstractHipRawEncoder/Decoder -- one stripe per call
 * (ECKeyOutputStream.java:304, heap buffers :701; ECReconstructionCoordinator.java:283), T threads sharing one coder
 * (RawErasureCoderBenchmark.java:201-206).  Each call runs the glue's GetByteArrayRegion into a pooled pinned arena,
 * libozec's in-place DMA + kernel, and SetByteArrayRegion back.
 *
 *   jni_percall SECONDS SPEC...        SPEC = encode|decode:K:P:CELL_BYTES:THREADS
 *
 * SPEC modes encodedirect / decodedirect call encodeDirect / decodeDirect on pinned direct buffers instead (every
 * cell in one ozec_host_alloc block, what OzecNative.allocatePinned hands a writer's buffer pool).
 * prints one JSON object per SPEC: calls, seconds, us per stripe (wall / calls per thread), GB/s of data bytes.  Before
 * timing, one encode + decode round trip of every thread's stripe is checked (the decoded units equal the originals).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "jni.h"
#include "../../include/ozec.h"

#define P(name) Java_org_apache_ozone_erasurecode_rawcoder_OzecNative_##name
jlong P(coderCreate)(JNIEnv *, jclass, jboolean, jint, jint, jint);
void P(coderRelease)(JNIEnv *, jclass, jlong);
void P(encodeArrays)(JNIEnv *, jclass, jlong, jobjectArray, jintArray, jint, jobjectArray, jintArray);
void P(decodeArrays)(JNIEnv *, jclass, jlong, jobjectArray, jintArray, jint, jintArray, jobjectArray, jintArray);
void P(encodeDirect)(JNIEnv *, jclass, jlong, jobjectArray, jintArray, jint, jobjectArray, jintArray);
void P(decodeDirect)(JNIEnv *, jclass, jlong, jobjectArray, jintArray, jint, jintArray, jobjectArray, jintArray);
int ozec_jni_heap_mode(int mode, unsigned long *cb_calls, unsigned long *arena_calls);

JNIEnv *mock_env(void);
struct mock_object *mock_bytes(void *p, int64_t len);
struct mock_object *mock_direct(void *p, int64_t cap);
struct mock_object *mock_ints(int32_t *p, int64_t n);
struct mock_object *mock_objects(int64_t n);
void mock_set(struct mock_object *arr, int64_t i, struct mock_object *v);
int mock_take_exception(char *cls, int cls_cap, char *msg, int msg_cap);

enum { MAXU = 32 };
static int K, R, CELL, DECODE, DIRECT;
static double SECONDS;
static jlong g_enc, g_dec;
static int g_erased[4] = {0, 1, 2, 3}; /* rs-6-3 decode: 3 erased {0, 1, 2}; rs-10-4: {0, 1, 2, 3} */
static int g_ne;

typedef struct {
  uint8_t *unit[MAXU]; /* k data + p parity cells, each a byte[] (DIRECT: cells of one pinned block) */
  uint8_t *block;      /* DIRECT: the ozec_host_alloc block holding every cell and the decode outputs */
  uint8_t *rec[4];     /* decode outputs */
  struct mock_object *enc_in, *enc_out, *dec_in, *dec_out, *zeros_in, *zeros_out, *zeros_dec, *erased;
  int32_t zeros[MAXU], er[4];
  long calls;
  double start, stop;
} worker_t;

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

static void fail_if_exception(const char *what) {
  char c[128], m[512];
  if (mock_take_exception(c, sizeof c, m, sizeof m)) {
    fprintf(stderr, "%s: %s: %s\n", what, c, m);
    exit(2);
  }
}

static void setup(worker_t *w, unsigned seed) {
  JNIEnv *env = mock_env();
  (void)env;
  w->block = NULL;
  if (DIRECT && ozec_host_alloc((size_t)(K + R + g_ne) * (size_t)CELL, (void **)&w->block) != 0) {
    fprintf(stderr, "ozec_host_alloc failed: %s\n", ozec_last_error());
    exit(2);
  }
  struct mock_object *(*wrap)(void *, int64_t) = DIRECT ? mock_direct : mock_bytes;
  for (int u = 0; u < K + R; ++u) {
    w->unit[u] = DIRECT ? w->block + (size_t)u * (size_t)CELL : malloc((size_t)CELL);
    if (u < K)
      for (int i = 0; i < CELL; ++i) w->unit[u][i] = (uint8_t)((seed = seed * 1103515245u + 12345u) >> 16);
    else
      memset(w->unit[u], 0xA5, (size_t)CELL);
  }
  w->enc_in = mock_objects(K);
  w->enc_out = mock_objects(R);
  for (int u = 0; u < K; ++u) mock_set(w->enc_in, u, wrap(w->unit[u], CELL));
  for (int r = 0; r < R; ++r) mock_set(w->enc_out, r, wrap(w->unit[K + r], CELL));
  memset(w->zeros, 0, sizeof w->zeros);
  w->zeros_in = mock_ints(w->zeros, K + R);
  w->zeros_out = mock_ints(w->zeros, R);
  w->dec_in = mock_objects(K + R);
  for (int u = 0; u < K + R; ++u) {
    int gone = 0;
    for (int e = 0; e < g_ne; ++e) gone |= g_erased[e] == u;
    mock_set(w->dec_in, u, gone ? NULL : wrap(w->unit[u], CELL));
  }
  w->dec_out = mock_objects(g_ne);
  for (int e = 0; e < g_ne; ++e) {
    w->rec[e] = DIRECT ? w->block + (size_t)(K + R + e) * (size_t)CELL : calloc(1, (size_t)CELL);
    mock_set(w->dec_out, e, wrap(w->rec[e], CELL));
    w->er[e] = g_erased[e];
  }
  w->zeros_dec = mock_ints(w->zeros, g_ne);
  w->erased = mock_ints(w->er, g_ne);
}

static void call(worker_t *w) {
  JNIEnv *env = mock_env();
  if (DECODE)
    (DIRECT ? P(decodeDirect) : P(decodeArrays))(env, NULL, g_dec, (jobjectArray)w->dec_in, (jintArray)w->zeros_in,
                                                 CELL, (jintArray)w->erased, (jobjectArray)w->dec_out,
                                                 (jintArray)w->zeros_dec);
  else
    (DIRECT ? P(encodeDirect) : P(encodeArrays))(env, NULL, g_enc, (jobjectArray)w->enc_in, (jintArray)w->zeros_in,
                                                 CELL, (jobjectArray)w->enc_out, (jintArray)w->zeros_out);
}

static pthread_barrier_t g_bar;

static void *run(void *arg) {
  worker_t *w = arg;
  pthread_barrier_wait(&g_bar);
  w->start = now();
  const double end = w->start + SECONDS;
  long c = 0;
  do {
    call(w);
    ++c;
  } while (now() < end);
  w->stop = now();
  w->calls = c;
  return NULL;
}

static int run_spec(const char *spec) {
  char mode[16] = {0};
  int T = 0;
  if (sscanf(spec, "%15[a-z]:%d:%d:%d:%d", mode, &K, &R, &CELL, &T) != 5 || K <= 0 || R <= 0 || K + R > MAXU ||
      CELL <= 0 || T <= 0 || T > 256) {
    fprintf(stderr, "bad spec %s\n", spec);
    return 1;
  }
  DECODE = !strncmp(mode, "decode", 6);
  DIRECT = strstr(mode, "direct") != NULL;  /* encodedirect / decodedirect: pinned direct buffers (allocatePinned) */
  g_ne = R < 4 ? R : 4;
  JNIEnv *env = mock_env();
  g_enc = P(coderCreate)(env, NULL, 0, 0, K, R);
  g_dec = P(coderCreate)(env, NULL, 1, 0, K, R);
  fail_if_exception("coderCreate");
  worker_t *ws = calloc((size_t)T, sizeof *ws);
  for (int t = 0; t < T; ++t) setup(&ws[t], 0x9E3779B9u * (unsigned)(t + 1));
  /* round trip of every worker's stripe: encode into the parity byte[], decode the erased units, compare */
  int ok = 1;
  const int mode_decode = DECODE;
  for (int t = 0; t < T; ++t) {
    DECODE = 0;
    call(&ws[t]);
    fail_if_exception("encodeArrays");
    DECODE = 1;
    call(&ws[t]);
    fail_if_exception("decodeArrays");
    for (int e = 0; e < g_ne; ++e) ok &= !memcmp(ws[t].rec[e], ws[t].unit[g_erased[e]], (size_t)CELL);
  }
  DECODE = mode_decode;
  for (int t = 0; t < T; ++t) call(&ws[t]); /* warm: arenas grown, graphs cached */
  fail_if_exception("warm-up");
  unsigned long cb0, ar0, cb1, ar1;
  (void)ozec_jni_heap_mode(-1, &cb0, &ar0);
  pthread_barrier_init(&g_bar, NULL, (unsigned)T);
  pthread_t *th = calloc((size_t)T, sizeof *th);
  for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, run, &ws[t]);
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  pthread_barrier_destroy(&g_bar);
  fail_if_exception("timed calls");
  (void)ozec_jni_heap_mode(-1, &cb1, &ar1);
  long calls = 0;
  double t0 = ws[0].start, t1 = ws[0].stop;
  for (int t = 0; t < T; ++t) {
    calls += ws[t].calls;
    if (ws[t].start < t0) t0 = ws[t].start;
    if (ws[t].stop > t1) t1 = ws[t].stop;
  }
  const double el = t1 - t0;
  const double data = (double)calls * K * (double)CELL; /* data bytes, as RawErasureCoderBenchmark counts them */
  printf("{\"mode\": \"%s\", \"k\": %d, \"p\": %d, \"erased\": %d, \"cell_bytes\": %d, \"threads\": %d, \"calls\": %ld, "
         "\"seconds\": %.4f, \"us_per_stripe\": %.2f, \"GBps\": %.3f, \"round_trip_ok\": %s, "
         "\"callback_form_calls\": %lu, \"arena_form_calls\": %lu}\n",
         DECODE ? (DIRECT ? "decodedirect" : "decode") : (DIRECT ? "encodedirect" : "encode"), K, R, DECODE ? g_ne : 0,
         CELL, T, calls, el, el / ((double)calls / T) * 1e6,
         data / el / 1e9, ok ? "true" : "false", cb1 - cb0, ar1 - ar0);
  fflush(stdout);
  P(coderRelease)(env, NULL, g_enc);
  P(coderRelease)(env, NULL, g_dec);
  for (int t = 0; t < T; ++t) {
    if (DIRECT) {
      (void)ozec_host_free(ws[t].block);
      continue;
    }
    for (int u = 0; u < K + R; ++u) free(ws[t].unit[u]);
    for (int e = 0; e < g_ne; ++e) free(ws[t].rec[e]);
  }
  free(ws);
  free(th);
  return ok ? 0 : 3;
}

/* OZEC_TUNE="key=value,key=value": ozec_set_tuning knobs for A/B runs of the harness (bench.py --tune) */
static int apply_tuning(void) {
  const char *e = getenv("OZEC_TUNE");
  if (!e || !*e) return 0;
  char buf[512];
  snprintf(buf, sizeof buf, "%s", e);
  for (char *kv = strtok(buf, ","); kv; kv = strtok(NULL, ",")) {
    char *eq = strchr(kv, '=');
    if (!eq) return 1;
    *eq = 0;
    if (ozec_set_tuning(kv, atoll(eq + 1)) != 0) {
      fprintf(stderr, "unknown tuning knob %s\n", kv);
      return 1;
    }
  }
  return 0;
}

int main(int argc, char **argv) {
  if (apply_tuning()) return 1;
  if (argc < 3) {
    fprintf(stderr, "usage: %s SECONDS encode|decode:K:P:CELL_BYTES:THREADS...\n", argv[0]);
    return 1;
  }
  SECONDS = atof(argv[1]);
  int rc = 0;
  for (int i = 2; i < argc && !rc; ++i) rc = run_spec(argv[i]);
  return rc;
}
