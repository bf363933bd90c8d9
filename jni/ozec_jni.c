/*
 * ozec_jni.c -- JNI glue of the Java drop-in (java/.../OzecNative.java): resolves Java buffers to addresses and
 * hands them to the JNI-free marshaling core (ozec_marshal.c), which validates, calls libozec and picks the Java
 * exception.  Build on a host with a JDK:
 *   cc -O2 -fPIC -shared -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude jni/ozec_jni.c jni/ozec_marshal.c \
 *      -Lozone_amd/lib -lozec -Wl,-rpath,'$ORIGIN' -o libozec_jni.so
 * (tests/test_jni_glue.py compiles this same file against a test double of the JNI interface, tests/native/mockjni).
 *
 * Reference counterparts (EC/ = hadoop-hdds/erasurecode/src/main/java/org/apache/ozone/erasurecode/):
 *   encodeDirect / decodeDirect   <- AbstractNativeRawEncoder.doEncode :49-73 / AbstractNativeRawDecoder.doDecode :49-75
 *                                    -> hadoop's performEncodeImpl / performDecodeImpl (HadoopNativeECAccessorUtil :32-58)
 *   encodeArrays / decodeArrays   <- doEncode(ByteArrayEncodingState) / doDecode(ByteArrayDecodingState); the reference
 *                                    copies heap arrays into direct buffers (:80-93), here into a pooled pinned
 *                                    arena (arrays held critical for the parallel copy only, never across device
 *                                    work: heap_* below)
 *   coderCreate / coderRelease    <- NativeRSRawEncoder ctor / release (EC/rawcoder/NativeRSRawEncoder.java:39-62)
 *   crcUpdate* / checksumWindows* <- ChecksumByteBuffer.update (CM/ChecksumByteBuffer.java:32-44) and
 *                                    Checksum.computeChecksum (CM/Checksum.java:157-200)
 *   queue*                        <- the stripe queue of ECKeyOutputStream (hadoop-ozone/client/.../ECKeyOutputStream.java:501-543)
 */
#include <jni.h>
#include <pthread.h>
#include <stdatomic.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ozec.h"
#include "ozec_marshal.h"

#define JNI_FN(name) Java_org_apache_ozone_erasurecode_rawcoder_OzecNative_##name
#define MAX_BUFS 256

static void throw_status(JNIEnv *env, const ozm_status *st) {
  if ((*env)->ExceptionCheck(env)) return;  /* the pending one (e.g. a refused array pin's OutOfMemoryError) stands */
  jclass c = (*env)->FindClass(env, st->exception_class);
  if (!c) { /* e.g. HadoopIllegalArgumentException absent from the class path: its superclass */
    (*env)->ExceptionClear(env);
    c = (*env)->FindClass(env, st->code == OZEC_EINVAL ? "java/lang/IllegalArgumentException"
                                                       : "java/lang/RuntimeException");
  }
  if (c) (*env)->ThrowNew(env, c, st->message);
}

static void throw_rc(JNIEnv *env, int rc) {
  ozm_status st;
  ozm_fail(rc, NULL, &st);
  throw_status(env, &st);
}

/* Java array of direct ByteBuffers (+ int[] positions) -> ozm_buf[]; null elements stay absent. */
static int collect_direct(JNIEnv *env, jobjectArray arr, jintArray offs, ozm_buf *bufs, int *n, ozm_status *st) {
  if (!arr || !offs) return ozm_fail(OZEC_EINVAL, "Invalid buffer array, null", st);
  const jsize len = (*env)->GetArrayLength(env, arr);
  if (len > MAX_BUFS || (*env)->GetArrayLength(env, offs) < len)
    return ozm_fail(OZEC_EINVAL, "Invalid buffer / offset arrays", st);
  jint o[MAX_BUFS];
  (*env)->GetIntArrayRegion(env, offs, 0, len, o);
  for (jsize i = 0; i < len; ++i) {
    jobject b = (*env)->GetObjectArrayElement(env, arr, i);
    memset(&bufs[i], 0, sizeof(bufs[i]));
    if (b) {
      bufs[i].present = 1;
      bufs[i].base = (*env)->GetDirectBufferAddress(env, b); /* NULL for a heap buffer: rejected by ozm_resolve */
      bufs[i].capacity = (int64_t)(*env)->GetDirectBufferCapacity(env, b);
      bufs[i].offset = o[i];
      (*env)->DeleteLocalRef(env, b);
    }
  }
  *n = (int)len;
  return 0;
}

/* Java byte[][] (+ int[] offsets) -> the arrays' local references, lengths and offsets (no address: heap arrays are
 * copied, see heap_* below); refs_free() deletes the references. */
typedef struct {
  jbyteArray arr[MAX_BUFS];
  int n;
} array_set;

static int collect_arrays(JNIEnv *env, jobjectArray arr, jintArray offs, ozm_buf *bufs, array_set *as,
                          ozm_status *st) {
  as->n = 0;
  if (!arr || !offs) return ozm_fail(OZEC_EINVAL, "Invalid buffer array, null", st);
  const jsize len = (*env)->GetArrayLength(env, arr);
  if (len > MAX_BUFS || (*env)->GetArrayLength(env, offs) < len)
    return ozm_fail(OZEC_EINVAL, "Invalid buffer / offset arrays", st);
  jint o[MAX_BUFS];
  (*env)->GetIntArrayRegion(env, offs, 0, len, o);
  for (jsize i = 0; i < len; ++i) {
    as->arr[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, arr, i);
    memset(&bufs[i], 0, sizeof(bufs[i]));
    if (as->arr[i]) {
      bufs[i].present = 1;
      bufs[i].capacity = (*env)->GetArrayLength(env, as->arr[i]);
      bufs[i].offset = o[i];
    }
  }
  as->n = (int)len;
  return 0;
}

static void refs_free(JNIEnv *env, array_set *as) {
  for (int i = 0; i < as->n; ++i)
    if (as->arr[i]) (*env)->DeleteLocalRef(env, as->arr[i]);
  as->n = 0;
}

/* ---------------------------------------------------------------- heap arrays: copied, never pinned across the GPU
 * A byte[] pinned with GetPrimitiveArrayCritical for the whole call would hold the VM's GC locker through staging, the
 * PCIe transfers and the kernel (~0.2 ms per rs-6-3 stripe of 1 MiB cells; every ECKeyOutputStream writer passes heap
 * buffers, ECKeyOutputStream.java:701).  Instead the regions a call reads are copied into pinned memory and its outputs
 * back, the arrays held critical for each copy only, as the reference's bridge copies heap arrays into direct buffers
 * (AbstractNativeRawEncoder.java:80-93).  Coder calls (round 6) copy into libozec's own pinned staging through the
 * ozec_encode_cb / ozec_decode_cb callbacks, chunk by chunk while the GPU works on the previous chunk (heap_code);
 * checksum calls copy into a pinned arena leased for the call.  Calls are cut in column pieces of HEAP_CHUNK bytes per
 * cell (coding and window CRCs are position-wise), so a call's staging is at most (k + p) x 4 MiB.
 * Arenas come from a process-wide pool of ARENA_POOL, leased for one call: pinned memory stays bounded however many
 * Java threads call at once; a call that finds every arena leased gets a pageable one of its own (libozec then stages
 * it through its pinned slots), so no call waits for another. */
#define HEAP_CHUNK ((int64_t)4 << 20)
#define ARENA_ALIGN 256
#define ARENA_POOL 32
/* Pinned arena memory is bounded: at most ARENA_BYTES_MAX bytes over the whole pool (env
 * OZEC_JNI_ARENA_MB, default 1024), a lease that would pass it runs on a pageable arena instead; an arena left unleased
 * for ARENA_IDLE_S seconds is given back at the next lease.  Each arena remembers the NUMA node its pages were placed
 * on, and a lease prefers a free arena on the calling thread's node, so a datanode's threads on both sockets DMA from
 * local memory.  Worst case pinned by the JNI layer: ARENA_BYTES_MAX ("Pinned memory"). */
#define ARENA_IDLE_S 30

typedef struct {
  uint8_t *p;
  size_t cap;
  int node;          /* NUMA node of the arena's pages, -1 unknown */
  struct timespec t; /* when it was last handed back */
} arena_t;

typedef struct {
  int slot;    /* index into g_arenas, or -1: `own` (pool exhausted, or the pinned bound reached) */
  arena_t own; /* pageable, freed at release */
} arena_lease;

static pthread_mutex_t g_arena_mu = PTHREAD_MUTEX_INITIALIZER;
static arena_t g_arenas[ARENA_POOL];
static int g_arena_leased[ARENA_POOL];
static size_t g_arena_bytes; /* pinned bytes held by the pool, guarded by g_arena_mu */

static size_t arena_bytes_max(void) {
  static size_t v;
  if (!v) {
    const char *e = getenv("OZEC_JNI_ARENA_MB");
    const long mb = e && *e ? atol(e) : 1024;
    v = (size_t)(mb > 0 ? mb : 1024) << 20;
  }
  return v;
}

static int caller_node(void) {
  unsigned cpu = 0, node = 0;
  return syscall(SYS_getcpu, &cpu, &node, NULL) == 0 ? (int)node : -1;
}

/* a free pooled arena -- on the caller's NUMA node if one is free, the largest among the candidates (to spare
 * reallocations) -- or a call-owned pageable one; pooled arenas idle for ARENA_IDLE_S are freed on the way */
static void arena_lease_begin(arena_lease *l) {
  l->slot = -1;
  memset(&l->own, 0, sizeof(l->own));
  const int node = caller_node();
  struct timespec now;
  clock_gettime(CLOCK_MONOTONIC, &now);
  uint8_t *idle[ARENA_POOL];
  int nidle = 0;
  pthread_mutex_lock(&g_arena_mu);
  int near = -1, any = -1;
  for (int i = 0; i < ARENA_POOL; ++i) {
    if (g_arena_leased[i]) continue;
    arena_t *a = &g_arenas[i];
    if (a->p && now.tv_sec - a->t.tv_sec > ARENA_IDLE_S) {
      idle[nidle++] = a->p;
      g_arena_bytes -= a->cap;
      a->p = NULL;
      a->cap = 0;
    }
    if (any < 0 || a->cap > g_arenas[any].cap) any = i;
    if (a->p && a->node == node && (near < 0 || a->cap > g_arenas[near].cap)) near = i;
  }
  l->slot = near >= 0 ? near : any;
  if (l->slot >= 0) g_arena_leased[l->slot] = 1;
  pthread_mutex_unlock(&g_arena_mu);
  for (int i = 0; i < nidle; ++i) (void)ozec_host_free(idle[i]);
}

static void arena_lease_end(arena_lease *l) {
  if (l->slot < 0) {
    free(l->own.p);
    return;
  }
  pthread_mutex_lock(&g_arena_mu);
  clock_gettime(CLOCK_MONOTONIC, &g_arenas[l->slot].t);
  g_arena_leased[l->slot] = 0;
  pthread_mutex_unlock(&g_arena_mu);
}

/* the leased arena, grown to at least `bytes`; NULL (status set) when it cannot be had */
static uint8_t *arena(arena_lease *l, size_t bytes, ozm_status *st) {
  arena_t *a = l->slot >= 0 ? &g_arenas[l->slot] : &l->own;
  if (a->cap >= bytes) return a->p;
  const size_t cap = (bytes + ((size_t)1 << 20) - 1) >> 20 << 20;
  if (l->slot >= 0) {
    uint8_t *old = a->p;
    pthread_mutex_lock(&g_arena_mu);
    const int fits = g_arena_bytes - a->cap + cap <= arena_bytes_max();
    g_arena_bytes -= a->cap;
    a->p = NULL;
    a->cap = 0;
    if (fits) g_arena_bytes += cap; /* reserved before the allocation, so concurrent growths stay under the bound */
    else g_arena_leased[l->slot] = 0; /* over the bound: this call goes pageable (libozec stages it) */
    pthread_mutex_unlock(&g_arena_mu);
    if (old) (void)ozec_host_free(old);
    if (!fits) {
      l->slot = -1;
      a = &l->own;
    } else {
      int rc = ozec_host_alloc(cap, (void **)&a->p);
      if (rc) {
        a->p = NULL;
        pthread_mutex_lock(&g_arena_mu);
        g_arena_bytes -= cap;
        pthread_mutex_unlock(&g_arena_mu);
        ozm_fail(rc, NULL, st);
        return NULL;
      }
      a->cap = cap;
      a->node = -1;
      (void)ozec_host_page_node(a->p, &a->node);
      return a->p;
    }
  }
  free(a->p);
  a->p = (uint8_t *)aligned_alloc(ARENA_ALIGN, cap);
  a->cap = a->p ? cap : 0;
  if (!a->p) ozm_fail(OZEC_ENOMEM, "out of memory", st);
  return a->p;
}

static int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

/* The array copies: every array of the set held with GetPrimitiveArrayCritical for the copy ONLY (released before
 * libozec does any device work), and the regions moved by ozec_host_copy -- libozec's parallel copy pool on the GPU's
 * NUMA node, as its own staging copies are -- instead of one GetByteArrayRegion after another on the calling thread:
 * one rs-6-3 stripe of 1 MiB heap cells spends ~150 us in that single-threaded copy-in (bench.py jni rows).  Nothing
 * in a critical section calls JNI or waits for a Java thread (the pool's workers are native threads).  An array the VM
 * will not hand out (NULL) ends the pinning: the arrays already held are released, and with no exception pending every
 * region is moved by Get/SetByteArrayRegion instead.  Returns 0, or -1 with a Java exception pending (typically the
 * OutOfMemoryError of a refused pin): the caller then makes no further JNI call but returns to Java. */
static int copy_regions(JNIEnv *env, const array_set *as, const ozm_buf *bufs, int64_t off, int64_t cl,
                        const ozm_buf *stage, int in) {
  void *pin[MAX_BUFS] = {0};
  void *dst[MAX_BUFS];
  const void *src[MAX_BUFS];
  size_t nb[MAX_BUFS];
  int n = 0, refused = 0;
  for (int i = 0; i < as->n && !refused; ++i) {
    if (!as->arr[i] || !stage[i].present) continue;
    pin[i] = (*env)->GetPrimitiveArrayCritical(env, as->arr[i], NULL);
    if (!pin[i]) {
      refused = 1;
      break;
    }
    uint8_t *arr = (uint8_t *)pin[i] + bufs[i].offset + off;
    dst[n] = in ? (void *)stage[i].base : (void *)arr;
    src[n] = in ? (const void *)arr : (const void *)stage[i].base;
    nb[n] = (size_t)cl;
    ++n;
  }
  const int rc = n && !refused ? ozec_host_copy(dst, src, nb, n, in) : 0;
  for (int i = 0; i < as->n; ++i)  /* nothing was copied when a pin was refused: release without write-back */
    if (pin[i]) (*env)->ReleasePrimitiveArrayCritical(env, as->arr[i], pin[i], in || refused ? JNI_ABORT : 0);
  if (!refused && !rc) return 0;
  if ((*env)->ExceptionCheck(env)) return -1;  /* no JNI call but the few allowed with an exception pending */
  for (int i = 0; i < as->n; ++i) {  /* every array region, one JNI copy each */
    if (!as->arr[i] || !stage[i].present) continue;
    if (in)
      (*env)->GetByteArrayRegion(env, as->arr[i], (jsize)(bufs[i].offset + off), (jsize)cl, (jbyte *)stage[i].base);
    else
      (*env)->SetByteArrayRegion(env, as->arr[i], (jsize)(bufs[i].offset + off), (jsize)cl,
                                 (const jbyte *)stage[i].base);
    if ((*env)->ExceptionCheck(env)) return -1;
  }
  return 0;
}

/* encode (erased == NULL) or decode of heap arrays already validated by ozm_*_check (round 6): libozec's staged
 * pipeline with the glue moving the bytes (ozec_encode_cb / ozec_decode_cb).  libozec cuts each HEAP_CHUNK piece of the
 * call into column chunks and asks for chunk c's inputs (heap_fill: the arrays held critical for that copy only,
 * copy_regions) while its kernel works on chunk c - 1 straight from its pinned staging, and hands back each chunk's
 * outputs (heap_drain) -- the copies overlap the GPU instead of preceding and following it.  No array is pinned while
 * libozec waits for the device: the callbacks run between its device operations and release every pin before they
 * return. */
typedef struct {
  JNIEnv *env;
  const array_set *ai, *ao;
  const ozm_buf *ib, *ob;
  int64_t base; /* this piece's offset within the call */
} heap_job;

static void staging_bufs(const array_set *as, const void *const *p, size_t len, ozm_buf *stage) {
  for (int i = 0; i < as->n; ++i) {
    memset(&stage[i], 0, sizeof(stage[i]));
    stage[i].present = p[i] != NULL;
    stage[i].base = p[i];
    stage[i].capacity = (int64_t)len;
  }
}

static int heap_fill(void *user, size_t off, size_t len, uint8_t *const *dst) {
  heap_job *j = (heap_job *)user;
  ozm_buf stage[MAX_BUFS];
  staging_bufs(j->ai, (const void *const *)dst, len, stage);
  return copy_regions(j->env, j->ai, j->ib, j->base + (int64_t)off, (int64_t)len, stage, 1) ? -1 : 0;
}

static int heap_drain(void *user, size_t off, size_t len, const uint8_t *const *src) {
  heap_job *j = (heap_job *)user;
  ozm_buf stage[MAX_BUFS];
  staging_bufs(j->ao, (const void *const *)src, len, stage);
  return copy_regions(j->env, j->ao, j->ob, j->base + (int64_t)off, (int64_t)len, stage, 0) ? -1 : 0;
}

static int heap_code_cb(JNIEnv *env, ozec_coder *h, const array_set *ai, const ozm_buf *ib, const array_set *ao,
                        const ozm_buf *ob, const int *erased, int ne, int64_t len, ozm_status *st) {
  heap_job j = {env, ai, ao, ib, ob, 0};
  uint8_t present[MAX_BUFS];
  for (int i = 0; i < ai->n; ++i) present[i] = ai->arr[i] != NULL;
  for (int64_t off = 0; off < len; off += HEAP_CHUNK) {
    const int64_t cl = len - off < HEAP_CHUNK ? len - off : HEAP_CHUNK;
    j.base = off;
    const int rc = erased ? ozec_decode_cb(h, present, erased, ne, (size_t)cl, heap_fill, heap_drain, &j)
                          : ozec_encode_cb(h, (size_t)cl, heap_fill, heap_drain, &j);
    if (rc) {
      if ((*env)->ExceptionCheck(env)) return ozm_fail(OZEC_ENOMEM, "a Java array could not be copied", st);
      return ozm_fail(rc, NULL, st);
    }
  }
  return 0;
}

/* The arena form: the inputs copied into a leased pinned arena, libozec's in-place DMA + kernel on it, the outputs
 * copied back -- the copies outside libozec's slot, so concurrent callers' copies and device work interleave freely */
static int heap_code_arena(JNIEnv *env, ozec_coder *h, const array_set *ai, const ozm_buf *ib, const array_set *ao,
                           const ozm_buf *ob, const int *erased, int ne, int64_t len, ozm_status *st) {
  ozm_buf si[MAX_BUFS], so[MAX_BUFS];
  int nin = 0;
  for (int i = 0; i < ai->n; ++i) nin += ai->arr[i] != NULL;
  arena_lease l;
  arena_lease_begin(&l);
  int rc = 0;
  for (int64_t off = 0; off < len && !rc; off += HEAP_CHUNK) {
    const int64_t cl = len - off < HEAP_CHUNK ? len - off : HEAP_CHUNK;
    const int64_t stride = round_up(cl, ARENA_ALIGN);
    uint8_t *a = arena(&l, (size_t)((int64_t)(nin + ao->n) * stride), st);
    if (!a) {
      rc = st->code;
      break;
    }
    int slot = 0;
    for (int i = 0; i < ai->n; ++i) {  /* present inputs in consecutive arena slots, outputs after them */
      memset(&si[i], 0, sizeof(si[i]));
      if (!ai->arr[i]) continue;
      si[i].present = 1;
      si[i].base = a + (int64_t)slot++ * stride;
      si[i].capacity = cl;
    }
    for (int r = 0; r < ao->n; ++r) {
      memset(&so[r], 0, sizeof(so[r]));
      so[r].present = ao->arr[r] != NULL;
      so[r].base = a + (int64_t)(nin + r) * stride;
      so[r].capacity = cl;
    }
    if (copy_regions(env, ai, ib, off, cl, si, 1)) {
      rc = ozm_fail(OZEC_ENOMEM, "a Java array could not be read", st);  /* its exception is pending */
      break;
    }
    rc = erased ? ozm_decode(h, si, ai->n, erased, ne, so, ao->n, cl, st)
                : ozm_encode(h, si, ai->n, so, ao->n, cl, st);
    if (!rc && copy_regions(env, ao, ob, off, cl, so, 0))
      rc = ozm_fail(OZEC_ENOMEM, "a Java array could not be written", st);
  }
  arena_lease_end(&l);
  return rc;
}

/* Which form a call takes (env OZEC_JNI_HEAP: "cb", "arena", default "auto"): a call alone in the process takes the
 * callback form (its copies overlap its own device work: rs-6-3 1 MiB cells, one thread, 260 -> ~224 us per stripe);
 * a call made while another coder call is in flight takes the arena form, whose copies run outside libozec's slots
 * (4 / 16 threads: the callback form held slots through its copies and lost ~20% aggregate, profiles/r06/zero_copy/) */
enum { HEAP_AUTO, HEAP_CB, HEAP_ARENA };
static _Atomic int g_heap_inflight, g_heap_mode = -1;
static _Atomic unsigned long g_heap_forms[2]; /* calls taken by the callback form, by the arena form */

static int heap_mode(void) {
  int m = atomic_load(&g_heap_mode);
  if (m < 0) {
    const char *e = getenv("OZEC_JNI_HEAP");
    m = e && !strcmp(e, "cb") ? HEAP_CB : e && !strcmp(e, "arena") ? HEAP_ARENA : HEAP_AUTO;
    atomic_store(&g_heap_mode, m);
  }
  return m;
}

/* not a native method: the tests' switch between the forms (mode 0 auto, 1 callback, 2 arena; -1 leaves it) and the
 * count of calls each form took; returns the previous mode */
JNIEXPORT int ozec_jni_heap_mode(int mode, unsigned long *cb_calls, unsigned long *arena_calls) {
  const int prev = heap_mode();
  if (mode >= HEAP_AUTO && mode <= HEAP_ARENA) atomic_store(&g_heap_mode, mode);
  if (cb_calls) *cb_calls = atomic_load(&g_heap_forms[0]);
  if (arena_calls) *arena_calls = atomic_load(&g_heap_forms[1]);
  return prev;
}

static int heap_code(JNIEnv *env, ozec_coder *h, const array_set *ai, const ozm_buf *ib, const array_set *ao,
                     const ozm_buf *ob, const int *erased, int ne, int64_t len, ozm_status *st) {
  const int mode = heap_mode();
  const int others = atomic_fetch_add(&g_heap_inflight, 1);
  const int cb = mode == HEAP_CB || (mode == HEAP_AUTO && others == 0);
  atomic_fetch_add(&g_heap_forms[cb ? 0 : 1], 1);
  const int rc = cb ? heap_code_cb(env, h, ai, ib, ao, ob, erased, ne, len, st)
                    : heap_code_arena(env, h, ai, ib, ao, ob, erased, ne, len, st);
  atomic_fetch_sub(&g_heap_inflight, 1);
  return rc;
}

static int int_array(JNIEnv *env, jintArray a, int *out, int max, int *n, ozm_status *st) {
  *n = 0;
  if (!a) return ozm_fail(OZEC_EINVAL, "null index array", st);
  const jsize len = (*env)->GetArrayLength(env, a);
  if (len > max) return ozm_fail(OZEC_EINVAL, "Too many erased, not recoverable", st);
  jint v[MAX_BUFS];
  (*env)->GetIntArrayRegion(env, a, 0, len, v);
  for (jsize i = 0; i < len; ++i) out[i] = v[i];
  *n = (int)len;
  return 0;
}

/* ---------------------------------------------------------------- library / coder lifecycle */

JNIEXPORT jint JNICALL JNI_OnLoad(JavaVM *vm, void *reserved) {
  (void)vm;
  (void)reserved;
  return JNI_VERSION_1_8;
}

JNIEXPORT jint JNICALL JNI_FN(deviceCount)(JNIEnv *env, jclass cls) {
  (void)env;
  (void)cls;
  return ozec_device_count();
}

/* ---- the GPUs of this JVM (ozec_set_devices; OzecNative reads ozone.ec.hip.devices / ozone.ec.hip.device.policy) */
JNIEXPORT void JNICALL JNI_FN(setDevices)(JNIEnv *env, jclass cls, jintArray devices) {
  (void)cls;
  int d[MAX_BUFS], n = 0;
  ozm_status st;
  if (devices && int_array(env, devices, d, MAX_BUFS, &n, &st)) {
    throw_status(env, &st);
    return;
  }
  int rc = ozec_set_devices(d, n);
  if (rc) throw_rc(env, rc);
}

JNIEXPORT jintArray JNICALL JNI_FN(getDevices)(JNIEnv *env, jclass cls) {
  (void)cls;
  int d[MAX_BUFS];
  int n = ozec_get_devices(d, MAX_BUFS);
  if (n > MAX_BUFS) n = MAX_BUFS;
  jintArray a = (*env)->NewIntArray(env, n);
  if (a) (*env)->SetIntArrayRegion(env, a, 0, n, (const jint *)d);
  return a;
}

JNIEXPORT void JNICALL JNI_FN(setDevicePolicy)(JNIEnv *env, jclass cls, jint policy) {
  (void)cls;
  int rc = ozec_set_device_policy(policy);
  if (rc) throw_rc(env, rc);
}

JNIEXPORT jint JNICALL JNI_FN(coderDevice)(JNIEnv *env, jclass cls, jlong h) {
  (void)cls;
  if (!h) {
    throw_rc(env, OZEC_ECLOSED);
    return -1;
  }
  return ozec_coder_device((ozec_coder *)(intptr_t)h);
}

/* RawErasureCoderFactory.createEncoder/createDecoder: throws when no GPU is usable, so CodecUtil falls back
 * (CodecUtil.createRawEncoderWithFallback, EC/rawcoder/util/CodecUtil.java:62-78) */
JNIEXPORT jlong JNICALL JNI_FN(coderCreate)(JNIEnv *env, jclass cls, jboolean decoder, jint codec, jint k, jint p) {
  (void)cls;
  ozec_coder *h = NULL;
  int rc = decoder ? ozec_decoder_create(codec, k, p, &h) : ozec_encoder_create(codec, k, p, &h);
  if (rc) {
    throw_rc(env, rc);
    return 0;
  }
  return (jlong)(intptr_t)h;
}

/* release(): the Java side zeroes its handle under its write lock, so every later call sees "closed" */
JNIEXPORT void JNICALL JNI_FN(coderRelease)(JNIEnv *env, jclass cls, jlong h) {
  (void)env;
  (void)cls;
  if (!h) return;
  ozec_coder_release((ozec_coder *)(intptr_t)h);
  ozec_coder_free((ozec_coder *)(intptr_t)h);
}

/* ---------------------------------------------------------------- encode / decode */

JNIEXPORT void JNICALL JNI_FN(encodeDirect)(JNIEnv *env, jclass cls, jlong h, jobjectArray in, jintArray inOff, jint len,
                                            jobjectArray out, jintArray outOff) {
  (void)cls;
  ozm_buf ib[MAX_BUFS], ob[MAX_BUFS];
  int ni = 0, no = 0;
  ozm_status st;
  if (collect_direct(env, in, inOff, ib, &ni, &st) || collect_direct(env, out, outOff, ob, &no, &st) ||
      ozm_encode((ozec_coder *)(intptr_t)h, ib, ni, ob, no, len, &st))
    throw_status(env, &st);
}

JNIEXPORT void JNICALL JNI_FN(encodeArrays)(JNIEnv *env, jclass cls, jlong h, jobjectArray in, jintArray inOff, jint len,
                                            jobjectArray out, jintArray outOff) {
  (void)cls;
  ozm_buf ib[MAX_BUFS], ob[MAX_BUFS];
  array_set ai, ao;
  ozm_status st;
  ai.n = ao.n = 0;
  int rc = collect_arrays(env, in, inOff, ib, &ai, &st);
  if (!rc) rc = collect_arrays(env, out, outOff, ob, &ao, &st);
  if (!rc) rc = ozm_encode_check((ozec_coder *)(intptr_t)h, ib, ai.n, ob, ao.n, len, &st);
  if (!rc) rc = heap_code(env, (ozec_coder *)(intptr_t)h, &ai, ib, &ao, ob, NULL, 0, len, &st);
  refs_free(env, &ao);
  refs_free(env, &ai);
  if (rc) throw_status(env, &st);
}

JNIEXPORT void JNICALL JNI_FN(decodeDirect)(JNIEnv *env, jclass cls, jlong h, jobjectArray in, jintArray inOff, jint len,
                                            jintArray erased, jobjectArray out, jintArray outOff) {
  (void)cls;
  ozm_buf ib[MAX_BUFS], ob[MAX_BUFS];
  int er[MAX_BUFS];
  int ni = 0, no = 0, ne = 0;
  ozm_status st;
  if (collect_direct(env, in, inOff, ib, &ni, &st) || collect_direct(env, out, outOff, ob, &no, &st) ||
      int_array(env, erased, er, MAX_BUFS, &ne, &st) ||
      ozm_decode((ozec_coder *)(intptr_t)h, ib, ni, er, ne, ob, no, len, &st))
    throw_status(env, &st);
}

JNIEXPORT void JNICALL JNI_FN(decodeArrays)(JNIEnv *env, jclass cls, jlong h, jobjectArray in, jintArray inOff, jint len,
                                            jintArray erased, jobjectArray out, jintArray outOff) {
  (void)cls;
  ozm_buf ib[MAX_BUFS], ob[MAX_BUFS];
  int er[MAX_BUFS];
  int ne = 0;
  array_set ai, ao;
  ozm_status st;
  ai.n = ao.n = 0;
  int rc = int_array(env, erased, er, MAX_BUFS, &ne, &st);
  if (!rc) rc = collect_arrays(env, in, inOff, ib, &ai, &st);
  if (!rc) rc = collect_arrays(env, out, outOff, ob, &ao, &st);
  if (!rc) rc = ozm_decode_check((ozec_coder *)(intptr_t)h, ib, ai.n, er, ne, ob, ao.n, len, &st);
  if (!rc) rc = heap_code(env, (ozec_coder *)(intptr_t)h, &ai, ib, &ao, ob, er, ne, len, &st);
  refs_free(env, &ao);
  refs_free(env, &ai);
  if (rc) throw_status(env, &st);
}

/* ---------------------------------------------------------------- checksums */

/* ChecksumByteBuffer.update(ByteBuffer) on a direct buffer: returns the new register */
JNIEXPORT jint JNICALL JNI_FN(crcUpdateDirect)(JNIEnv *env, jclass cls, jint type, jint state, jobject buf, jint off,
                                               jint len) {
  (void)cls;
  ozm_buf b = {0};
  ozm_status st;
  uint32_t s = (uint32_t)state;
  b.present = buf != NULL;
  if (buf) {
    b.base = (*env)->GetDirectBufferAddress(env, buf);
    b.capacity = (int64_t)(*env)->GetDirectBufferCapacity(env, buf);
    b.offset = off;
  }
  if (ozm_crc_update(type, &s, &b, len, &st)) throw_status(env, &st);
  return (jint)s;
}

/* update(byte[] b, int off, int len) */
JNIEXPORT jint JNICALL JNI_FN(crcUpdateArray)(JNIEnv *env, jclass cls, jint type, jint state, jbyteArray arr, jint off,
                                              jint len) {
  (void)cls;
  ozm_buf b = {0};
  ozm_status st;
  uint32_t s = (uint32_t)state;
  int rc;
  if (!arr) {
    rc = ozm_crc_update(type, &s, &b, len, &st);
  } else {
    /* bounds first (no address read), then the region in arena chunks: the register carries across them */
    b.present = 1;
    b.capacity = (*env)->GetArrayLength(env, arr);
    b.offset = off;
    b.base = (void *)arr; /* a placeholder address for the check: never read */
    const uint8_t *unused;
    rc = len == 0 ? 0 : ozm_resolve(&b, 1, 0, len, &unused, &st);
    arena_lease l;
    arena_lease_begin(&l);
    for (int64_t o = 0; !rc && o < len; o += HEAP_CHUNK) {
      const int64_t cl = len - o < HEAP_CHUNK ? len - o : HEAP_CHUNK;
      uint8_t *a = arena(&l, (size_t)cl, &st);
      if (!a) {
        rc = st.code;
        break;
      }
      (*env)->GetByteArrayRegion(env, arr, (jsize)(off + o), (jsize)cl, (jbyte *)a);
      ozm_buf c = {a, 0, cl, 1};
      rc = ozm_crc_update(type, &s, &c, cl, &st);
    }
    arena_lease_end(&l);
  }
  if (rc) throw_status(env, &st);
  return (jint)s;
}

/* Checksum.computeChecksum of one buffer region (data: a direct buffer, or a byte[] copied into the arena in chunks
 * of whole windows): big-endian CRC bytes of every window into out (SetByteArrayRegion, no pin across the GPU call);
 * returns the number of bytes written (4 per window) */
static jint checksum_windows(JNIEnv *env, jint type, jobject direct, jbyteArray data, jint off, jint len, jint bpc,
                             jbyteArray out) {
  ozm_status st;
  if (!out) {
    ozm_fail(OZEC_EINVAL, "null checksum output", &st);
    throw_status(env, &st);
    return 0;
  }
  ozm_buf b = {0};
  b.present = direct != NULL || data != NULL;
  if (direct) {
    b.base = (*env)->GetDirectBufferAddress(env, direct);
    b.capacity = (int64_t)(*env)->GetDirectBufferCapacity(env, direct);
  } else if (data) {
    b.base = (void *)data; /* a placeholder address for the bounds check: never read */
    b.capacity = (*env)->GetArrayLength(env, data);
  }
  b.offset = off;
  const jsize cap = (*env)->GetArrayLength(env, out);
  int rc = 0;
  int64_t total = 0;
  const uint8_t *unused;
  if (bpc <= 0) rc = ozm_fail(OZEC_EINVAL, "bytesPerChecksum must be positive", &st);
  else if (len != 0 && (rc = ozm_resolve(&b, 1, 0, len, &unused, &st)) == 0 &&
           (int64_t)cap < 4 * (((int64_t)len + bpc - 1) / bpc))
    rc = ozm_fail(OZEC_EINVAL, "checksum output too small", &st);
  /* whole windows per round trip (at least one): the arena holds the chunk's data (byte[] only) and its CRCs */
  const int64_t chunk = bpc <= 0 ? 1 : HEAP_CHUNK < bpc ? bpc : HEAP_CHUNK / bpc * bpc;
  arena_lease l;
  arena_lease_begin(&l);
  for (int64_t o = 0; !rc && o < len; o += chunk) {
    const int64_t cl = len - o < chunk ? len - o : chunk;
    const int64_t nw = (cl + bpc - 1) / bpc, dbytes = direct ? 0 : round_up(cl, ARENA_ALIGN);
    uint8_t *a = arena(&l, (size_t)(dbytes + 4 * nw), &st);
    if (!a) {
      rc = st.code;
      break;
    }
    ozm_buf c = b;
    if (!direct) {
      (*env)->GetByteArrayRegion(env, data, (jsize)(off + o), (jsize)cl, (jbyte *)a);
      c.base = a;
      c.offset = 0;
      c.capacity = cl;
    } else {
      c.offset = off + o;
    }
    int64_t written = 0;
    rc = ozm_checksum_windows(type, &c, cl, bpc, a + dbytes, 4 * nw, &written, &st);
    if (!rc) {
      (*env)->SetByteArrayRegion(env, out, (jsize)total, (jsize)written, (const jbyte *)(a + dbytes));
      total += written;
    }
  }
  arena_lease_end(&l);
  if (rc) throw_status(env, &st);
  return (jint)total;
}

JNIEXPORT jint JNICALL JNI_FN(checksumWindowsDirect)(JNIEnv *env, jclass cls, jint type, jobject buf, jint off, jint len,
                                                     jint bpc, jbyteArray out) {
  (void)cls;
  return checksum_windows(env, type, buf, NULL, off, len, bpc, out);
}

JNIEXPORT jint JNICALL JNI_FN(checksumWindowsArray)(JNIEnv *env, jclass cls, jint type, jbyteArray data, jint off,
                                                    jint len, jint bpc, jbyteArray out) {
  (void)cls;
  return checksum_windows(env, type, NULL, data, off, len, bpc, out);
}

/* ---------------------------------------------------------------- pinned memory + stripe queue (§8(f) row 3) */

/* a direct ByteBuffer over pinned host memory on the current GPU's NUMA node (ozec_host_alloc): cells DMA'd in place */
JNIEXPORT jobject JNICALL JNI_FN(allocatePinned)(JNIEnv *env, jclass cls, jint bytes) {
  (void)cls;
  void *p = NULL;
  int rc = bytes < 0 ? OZEC_EINVAL : ozec_host_alloc((size_t)bytes, &p);
  if (rc) {
    throw_rc(env, rc);
    return NULL;
  }
  return (*env)->NewDirectByteBuffer(env, p, (jlong)bytes);
}

JNIEXPORT void JNICALL JNI_FN(freePinned)(JNIEnv *env, jclass cls, jobject buf) {
  (void)cls;
  if (!buf) return;
  int rc = ozec_host_free((*env)->GetDirectBufferAddress(env, buf));
  if (rc) throw_rc(env, rc);
}

JNIEXPORT jlong JNICALL JNI_FN(queueCreate)(JNIEnv *env, jclass cls, jlong enc, jint cellLen, jint stripesPerBatch,
                                            jint type, jint bpc) {
  (void)cls;
  ozec_stripe_queue *q = NULL;
  int rc = cellLen <= 0 || stripesPerBatch <= 0 || bpc < 0
               ? OZEC_EINVAL
               : ozec_stripe_queue_create((ozec_coder *)(intptr_t)enc, (size_t)cellLen, (size_t)stripesPerBatch, type,
                                          (size_t)bpc, 1, &q);
  if (rc) {
    throw_rc(env, rc);
    return 0;
  }
  return (jlong)(intptr_t)q;
}

/* submit(data cells, parity cells, len, crcs): direct buffers at their positions; returns the stripe's ticket.
 * The Java side keeps the buffers referenced until waitFor(ticket) returns (HipStripeQueue).  Cell counts, lengths
 * and the CRC buffer's room from crcsOffset are checked against the queue by ozm_queue_submit. */
JNIEXPORT jlong JNICALL JNI_FN(queueSubmit)(JNIEnv *env, jclass cls, jlong q, jobjectArray data, jintArray dataOff,
                                            jobjectArray parity, jintArray parityOff, jint len, jobject crcs,
                                            jint crcsOffset) {
  (void)cls;
  ozm_buf db[MAX_BUFS], pb[MAX_BUFS], cb = {0};
  int nd = 0, np = 0;
  ozm_status st;
  uint64_t ticket = 0;
  if (collect_direct(env, data, dataOff, db, &nd, &st) || collect_direct(env, parity, parityOff, pb, &np, &st)) {
    throw_status(env, &st);
    return 0;
  }
  if (crcs) {
    cb.present = 1;
    cb.base = (*env)->GetDirectBufferAddress(env, crcs);
    cb.capacity = (int64_t)(*env)->GetDirectBufferCapacity(env, crcs);
    cb.offset = crcsOffset;
    if (!cb.base) {
      ozm_fail(OZEC_EINVAL, "crcs must be a direct buffer", &st);
      throw_status(env, &st);
      return 0;
    }
  }
  if (ozm_queue_submit((ozec_stripe_queue *)(intptr_t)q, db, nd, pb, np, len, &cb, &ticket, &st)) {
    throw_status(env, &st);
    return 0;
  }
  return (jlong)ticket;
}

JNIEXPORT void JNICALL JNI_FN(queueWait)(JNIEnv *env, jclass cls, jlong q, jlong ticket) {
  (void)cls;
  int rc = ozec_stripe_queue_wait((ozec_stripe_queue *)(intptr_t)q, (uint64_t)ticket);
  if (rc) throw_rc(env, rc);
}

JNIEXPORT void JNICALL JNI_FN(queueFree)(JNIEnv *env, jclass cls, jlong q) {
  (void)cls;
  int rc = ozec_stripe_queue_free((ozec_stripe_queue *)(intptr_t)q);
  if (rc) throw_rc(env, rc);
}

/* ---------------------------------------------------------------- batch reconstruction (§8(f) row 1 on host buffers) */

/* a direct buffer as an ozm_buf from its start (the Java side slices it; no buffer position is read here) */
static ozm_buf direct_buf(JNIEnv *env, jobject b) {
  ozm_buf r = {NULL, 0, -1, 0};
  if (!b) return r;
  r.base = (*env)->GetDirectBufferAddress(env, b);
  r.capacity = (*env)->GetDirectBufferCapacity(env, b);
  r.present = 1;
  return r;
}

/* reconstructHostBatch(decoder, stripes, stripeStride, unitStride, present[], erased[], out, numStripes, cellLen,
 * checksumType, bytesPerChecksum, expected, outCrcs, mismatch): every buffer direct (allocatePinned for DMA in
 * place); CRC buffers hold big-endian ints as ChecksumData's ByteStrings do. */
JNIEXPORT void JNICALL JNI_FN(reconstructHostBatch)(JNIEnv *env, jclass cls, jlong dec, jobject stripes,
                                                    jlong stripeStride, jlong unitStride, jintArray present,
                                                    jintArray erased, jobject out, jint numStripes, jint cellLen,
                                                    jint type, jint bpc, jobject expected, jobject outCrcs,
                                                    jobject mismatch) {
  (void)cls;
  ozm_status st;
  int pr[MAX_BUFS], er[MAX_BUFS], npr = 0, ner = 0;
  if (int_array(env, present, pr, MAX_BUFS, &npr, &st) || int_array(env, erased, er, MAX_BUFS, &ner, &st)) {
    throw_status(env, &st);
    return;
  }
  const ozm_buf sb = direct_buf(env, stripes), ob = direct_buf(env, out), eb = direct_buf(env, expected),
                cb = direct_buf(env, outCrcs), mb = direct_buf(env, mismatch);
  if ((stripes && !sb.base) || (out && !ob.base) || (expected && !eb.base) || (outCrcs && !cb.base) ||
      (mismatch && !mb.base)) {
    ozm_fail(OZEC_EINVAL, "reconstructHostBatch needs direct buffers", &st);
    throw_status(env, &st);
    return;
  }
  if (ozm_reconstruct_host_batch((ozec_coder *)(intptr_t)dec, &sb, stripeStride, unitStride, pr, npr, er, ner, &ob,
                                 numStripes, cellLen, type, bpc, &eb, &cb, &mb, &st))
    throw_status(env, &st);
}

/* ---------------------------------------------------------------- COMPOSITE_CRC (§8(f) row 4) */
/* CrcUtil.getMonomial / CrcUtil.compose (OC/CrcUtil.java:74-127) and CrcComposer (OC/CrcComposer.java:44-215) over
 * ozec_crc_monomial / ozec_crc_compose / ozec_crc_composer_*; OC/ = hadoop-ozone/common/src/main/java/org/apache/
 * hadoop/ozone/client/checksum/.  HipCrcUtil / HipCrcComposer (java/.../ozone/client/checksum/) are the callers. */

JNIEXPORT jint JNICALL JNI_FN(crcMonomial)(JNIEnv *env, jclass cls, jint type, jlong lengthBytes) {
  (void)cls;
  ozm_status st;
  uint32_t v = 0;
  if (ozm_crc_monomial(type, lengthBytes, &v, &st)) throw_status(env, &st);
  return (jint)v;
}

JNIEXPORT jint JNICALL JNI_FN(crcCompose)(JNIEnv *env, jclass cls, jint type, jint crcA, jint crcB, jlong lengthB) {
  (void)cls;
  ozm_status st;
  uint32_t v = 0;
  if (ozm_crc_compose(type, (uint32_t)crcA, (uint32_t)crcB, lengthB, &v, &st)) throw_status(env, &st);
  return (jint)v;
}

JNIEXPORT jlong JNICALL JNI_FN(composerCreate)(JNIEnv *env, jclass cls, jint type, jlong bytesPerCrcHint,
                                               jlong stripeLength) {
  (void)cls;
  ozm_status st;
  ozec_crc_composer *c = NULL;
  if (ozm_composer_create(type, bytesPerCrcHint, stripeLength, &c, &st)) {
    throw_status(env, &st);
    return 0;
  }
  return (jlong)(intptr_t)c;
}

JNIEXPORT void JNICALL JNI_FN(composerUpdate)(JNIEnv *env, jclass cls, jlong c, jint crc, jlong bytesPerCrc) {
  (void)cls;
  ozm_status st;
  if (ozm_composer_update((ozec_crc_composer *)(intptr_t)c, (uint32_t)crc, bytesPerCrc, &st)) throw_status(env, &st);
}

/* update(byte[] crcBuffer, int offset, int length, long bytesPerCrc): big-endian CRCs read in place */
JNIEXPORT void JNICALL JNI_FN(composerUpdateBytes)(JNIEnv *env, jclass cls, jlong c, jbyteArray buf, jint offset,
                                                   jint length, jlong bytesPerCrc) {
  (void)cls;
  ozm_status st;
  const jsize cap = buf ? (*env)->GetArrayLength(env, buf) : 0;
  const uint8_t *b = buf ? (const uint8_t *)(*env)->GetPrimitiveArrayCritical(env, buf, NULL) : NULL;
  int rc = ozm_composer_update_bytes((ozec_crc_composer *)(intptr_t)c, b, cap, offset, length, bytesPerCrc, &st);
  if (b) (*env)->ReleasePrimitiveArrayCritical(env, buf, (void *)b, JNI_ABORT);
  if (rc) throw_status(env, &st);
}

/* bytes the next digest returns (the Java side sizes its array with it) */
JNIEXPORT jint JNICALL JNI_FN(composerPending)(JNIEnv *env, jclass cls, jlong c) {
  (void)env;
  (void)cls;
  return (jint)ozec_crc_composer_pending((const ozec_crc_composer *)(intptr_t)c);
}

/* digest() into out; returns its length */
JNIEXPORT jint JNICALL JNI_FN(composerDigest)(JNIEnv *env, jclass cls, jlong c, jbyteArray out) {
  (void)cls;
  ozm_status st;
  int64_t written = 0;
  const jsize cap = out ? (*env)->GetArrayLength(env, out) : 0;
  uint8_t *o = out ? (uint8_t *)(*env)->GetPrimitiveArrayCritical(env, out, NULL) : NULL;
  int rc = ozm_composer_digest((ozec_crc_composer *)(intptr_t)c, o, cap, &written, &st);
  if (o) (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
  if (rc) throw_status(env, &st);
  return (jint)written;
}

JNIEXPORT void JNICALL JNI_FN(composerFree)(JNIEnv *env, jclass cls, jlong c) {
  (void)env;
  (void)cls;
  ozec_crc_composer_free((ozec_crc_composer *)(intptr_t)c);
}

/* ozec_crc_compose_windows_batch for a caller that holds device pointers (a GPU pipeline's window CRCs): the
 * composite CRC of every cell from its window CRCs, on `stream` (0 = the default stream), asynchronous */
JNIEXPORT void JNICALL JNI_FN(composeWindowsBatch)(JNIEnv *env, jclass cls, jint type, jlong dCrcs, jlong crcCellStride,
                                                   jlong numCells, jlong numWindows, jlong bpc, jlong lastLen,
                                                   jboolean crcsBigEndian, jlong dOut, jboolean outBigEndian,
                                                   jlong stream) {
  (void)cls;
  int rc = numCells < 0 || numWindows < 0 || bpc < 0 || lastLen < 0
               ? OZEC_EINVAL
               : ozec_crc_compose_windows_batch(type, (const uint32_t *)(intptr_t)dCrcs, crcCellStride, (size_t)numCells,
                                                (size_t)numWindows, (size_t)bpc, (size_t)lastLen, crcsBigEndian ? 1 : 0,
                                                (uint32_t *)(intptr_t)dOut, outBigEndian ? 1 : 0,
                                                (void *)(intptr_t)stream);
  if (rc) throw_rc(env, rc);
}
