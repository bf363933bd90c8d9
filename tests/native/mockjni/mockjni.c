/*
 * TEST DOUBLE: fake Java objects and the JNI functions of tests/native/mockjni/jni.h, driven from Python (ctypes) by
 * tests/test_jni_glue.py to call the real jni/ozec_jni.c entry points.  Direct buffers and byte[] wrap caller memory;
 * GetPrimitiveArrayCritical hands out the array memory itself (as HotSpot does) and counts pins so the test can
 * check that every pin is released; ThrowNew records the pending exception.  The counters are atomic, so the glue can
 * be driven from several threads (tests/native/jni_percall.c, bench.py --workload jni).
 */
#include "jni.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { K_DIRECT = 1, K_BYTES = 2, K_INTS = 3, K_OBJS = 4, K_CLASS = 5 };

struct mock_object {
  int kind;
  void *data;
  int64_t len;
  struct mock_object **elems;
  char name[96];
  int owns;  /* data allocated by the mock (NewIntArray) */
};

static int g_pins, g_local_refs;
static char g_exc_class[96], g_exc_msg[512];
static int g_exc_pending;
static int g_calls_with_pending;  /* JNI calls other than the exception-safe ones made while an exception was pending */
static char g_missing[96];

static jclass find_class(JNIEnv *env, const char *name) {
  (void)env;
  if (g_exc_pending) __atomic_add_fetch(&g_calls_with_pending, 1, __ATOMIC_RELAXED);
  if (g_missing[0] && !strcmp(name, g_missing)) {
    g_exc_pending = 1;
    snprintf(g_exc_class, sizeof g_exc_class, "java/lang/NoClassDefFoundError");
    snprintf(g_exc_msg, sizeof g_exc_msg, "%s", name);
    return NULL;
  }
  struct mock_object *c = calloc(1, sizeof *c);
  c->kind = K_CLASS;
  snprintf(c->name, sizeof c->name, "%s", name);
  return c; /* leaked: a test process makes few */
}

static jint throw_new(JNIEnv *env, jclass c, const char *msg) {
  (void)env;
  g_exc_pending = 1;
  snprintf(g_exc_class, sizeof g_exc_class, "%s", c->name);
  snprintf(g_exc_msg, sizeof g_exc_msg, "%s", msg ? msg : "");
  return 0;
}

static void exception_clear(JNIEnv *env) {
  (void)env;
  g_exc_pending = 0;
}

static void delete_local_ref(JNIEnv *env, jobject o) {
  (void)env;
  if (o) __atomic_sub_fetch(&g_local_refs, 1, __ATOMIC_RELAXED);
}

static jsize array_length(JNIEnv *env, jarray a) {
  (void)env;
  return (jsize)a->len;
}

static jobject object_array_element(JNIEnv *env, jobjectArray a, jsize i) {
  (void)env;
  if (a->kind != K_OBJS || i < 0 || i >= a->len) return NULL;
  if (a->elems[i]) __atomic_add_fetch(&g_local_refs, 1, __ATOMIC_RELAXED);
  return a->elems[i];
}

static void int_array_region(JNIEnv *env, jintArray a, jsize start, jsize n, jint *buf) {
  (void)env;
  memcpy(buf, (jint *)a->data + start, sizeof(jint) * (size_t)n);
}

/* test hook: the next `g_refuse_after` pins succeed, then GetPrimitiveArrayCritical returns NULL with an
 * OutOfMemoryError pending (a JVM that cannot pin); -1 = never refuse */
static int g_refuse_after = -1;

static void *array_critical(JNIEnv *env, jarray a, jboolean *is_copy) {
  (void)env;
  if (g_exc_pending) __atomic_add_fetch(&g_calls_with_pending, 1, __ATOMIC_RELAXED);
  if (g_refuse_after == 0) {
    g_refuse_after = -1;
    g_exc_pending = 1;
    snprintf(g_exc_class, sizeof g_exc_class, "java/lang/OutOfMemoryError");
    snprintf(g_exc_msg, sizeof g_exc_msg, "could not pin the array");
    return NULL;
  }
  if (g_refuse_after > 0) --g_refuse_after;
  if (is_copy) *is_copy = 0;
  __atomic_add_fetch(&g_pins, 1, __ATOMIC_RELAXED);
  return a->data;
}

static void release_array_critical(JNIEnv *env, jarray a, void *p, jint mode) {
  (void)env;
  (void)a;
  (void)p;
  (void)mode;
  __atomic_sub_fetch(&g_pins, 1, __ATOMIC_RELAXED);
}

static jobject new_direct(JNIEnv *env, void *p, jlong cap) {
  (void)env;
  struct mock_object *o = calloc(1, sizeof *o);
  o->kind = K_DIRECT;
  o->data = p;
  o->len = cap;
  return o;
}

static void *direct_address(JNIEnv *env, jobject o) {
  (void)env;
  return o && o->kind == K_DIRECT ? o->data : NULL;
}

static jlong direct_capacity(JNIEnv *env, jobject o) {
  (void)env;
  return o && o->kind == K_DIRECT ? o->len : -1;
}

/* Get/SetByteArrayRegion: the JVM's bounds check (ArrayIndexOutOfBoundsException pending, nothing copied) */
static int region_ok(jarray a, jsize start, jsize n) {
  if (a->kind == K_BYTES && start >= 0 && n >= 0 && (int64_t)start + n <= a->len) return 1;
  snprintf(g_exc_class, sizeof g_exc_class, "java/lang/ArrayIndexOutOfBoundsException");
  snprintf(g_exc_msg, sizeof g_exc_msg, "Array region %d..%lld out of bounds for length %lld", start,
           (long long)start + n, (long long)a->len);
  g_exc_pending = 1;
  return 0;
}

static int g_region_copies;

static jboolean exception_check(JNIEnv *env) {
  (void)env;
  return (jboolean)(g_exc_pending != 0);
}

static void get_byte_region(JNIEnv *env, jbyteArray a, jsize start, jsize n, jbyte *buf) {
  (void)env;
  if (g_exc_pending) __atomic_add_fetch(&g_calls_with_pending, 1, __ATOMIC_RELAXED);
  if (!region_ok(a, start, n)) return;
  memcpy(buf, (jbyte *)a->data + start, (size_t)n);
  __atomic_add_fetch(&g_region_copies, 1, __ATOMIC_RELAXED);
}

static void set_byte_region(JNIEnv *env, jbyteArray a, jsize start, jsize n, const jbyte *buf) {
  (void)env;
  if (g_exc_pending) __atomic_add_fetch(&g_calls_with_pending, 1, __ATOMIC_RELAXED);
  if (!region_ok(a, start, n)) return;
  memcpy((jbyte *)a->data + start, buf, (size_t)n);
  __atomic_add_fetch(&g_region_copies, 1, __ATOMIC_RELAXED);
}

/* a new int[] owns its memory (freed with mock_free) */
static jintArray new_int_array(JNIEnv *env, jsize n) {
  (void)env;
  struct mock_object *o = calloc(1, sizeof *o);
  o->kind = K_INTS;
  o->data = calloc((size_t)(n ? n : 1), sizeof(jint));
  o->len = n;
  o->owns = 1;  /* handed to the Java caller: not a local reference the glue must delete */
  return o;
}

static void set_int_region(JNIEnv *env, jintArray a, jsize start, jsize n, const jint *buf) {
  (void)env;
  memcpy((jint *)a->data + start, buf, sizeof(jint) * (size_t)n);
}

static const struct JNINativeInterface_ g_table = {
    find_class,           throw_new,      exception_clear,       delete_local_ref, array_length,
    object_array_element, int_array_region, array_critical,      release_array_critical,
    new_direct,           direct_address, direct_capacity,       get_byte_region,  set_byte_region,
    new_int_array,        set_int_region, exception_check,
};
static JNIEnv g_env = &g_table;

/* ---- driver API (ctypes) */
JNIEnv *mock_env(void) { return &g_env; }
void mock_refuse_pin_after(int n) { g_refuse_after = n; }
int mock_calls_with_pending(void) { return __atomic_load_n(&g_calls_with_pending, __ATOMIC_RELAXED); }

static struct mock_object *obj(int kind, void *data, int64_t len) {
  struct mock_object *o = calloc(1, sizeof *o);
  o->kind = kind;
  o->data = data;
  o->len = len;
  return o;
}

struct mock_object *mock_direct(void *p, int64_t cap) { return obj(K_DIRECT, p, cap); }
/* a heap ByteBuffer: a Java object that is not direct (GetDirectBufferAddress -> NULL) */
struct mock_object *mock_heap_buffer(void *p, int64_t cap) { return obj(K_BYTES, p, cap); }
struct mock_object *mock_bytes(void *p, int64_t len) { return obj(K_BYTES, p, len); }
struct mock_object *mock_ints(int32_t *p, int64_t n) { return obj(K_INTS, p, n); }

struct mock_object *mock_objects(int64_t n) {
  struct mock_object *o = obj(K_OBJS, NULL, n);
  o->elems = calloc((size_t)(n ? n : 1), sizeof(struct mock_object *));
  return o;
}

void mock_set(struct mock_object *arr, int64_t i, struct mock_object *v) { arr->elems[i] = v; }
void *mock_data(struct mock_object *o) { return o ? o->data : NULL; }
int64_t mock_len(struct mock_object *o) { return o ? o->len : -1; }

void mock_free(struct mock_object *o) {
  if (!o) return;
  free(o->elems);
  if (o->owns) free(o->data);
  free(o);
}

int mock_pins(void) { return __atomic_load_n(&g_pins, __ATOMIC_RELAXED); }
int mock_region_copies(void) { return __atomic_load_n(&g_region_copies, __ATOMIC_RELAXED); }

/* libozec entry points that do device work, wrapped at link time (-Wl,--wrap=...): the most array pins outstanding
 * when the glue called any of them -- VERDICT r3: heap arrays must not stay pinned across device work */
static int g_pins_at_device_call = 0, g_device_calls = 0;
static void at_device_call(void) {
  __atomic_add_fetch(&g_device_calls, 1, __ATOMIC_RELAXED);
  const int pins = __atomic_load_n(&g_pins, __ATOMIC_RELAXED);
  int seen = __atomic_load_n(&g_pins_at_device_call, __ATOMIC_RELAXED);
  while (pins > seen &&
         !__atomic_compare_exchange_n(&g_pins_at_device_call, &seen, pins, 0, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
}
int mock_pins_at_device_call(void) { return g_pins_at_device_call; }
int mock_device_calls(void) { return g_device_calls; }
void mock_reset_device_calls(void) { g_pins_at_device_call = g_device_calls = 0; }

#include "../../../include/ozec.h"
int __real_ozec_encode(ozec_coder *, const uint8_t *const *, uint8_t *const *, size_t);
int __wrap_ozec_encode(ozec_coder *c, const uint8_t *const *in, uint8_t *const *out, size_t len) {
  at_device_call();
  return __real_ozec_encode(c, in, out, len);
}
int __real_ozec_decode(ozec_coder *, const uint8_t *const *, const int *, int, uint8_t *const *, size_t);
int __wrap_ozec_decode(ozec_coder *c, const uint8_t *const *in, const int *e, int ne, uint8_t *const *out,
                       size_t len) {
  at_device_call();
  return __real_ozec_decode(c, in, e, ne, out, len);
}
/* the callback forms (round 6): pins outstanding at entry, and -- through trampolines around the glue's fill / drain --
 * pins still outstanding when a callback hands control back to libozec (which then launches or waits on the device) */
static int g_pins_after_callback;
int mock_pins_after_callback(void) { return g_pins_after_callback; }
typedef struct {
  ozec_fill_fn fill;
  ozec_drain_fn drain;
  void *user;
} cb_tramp;
static int tramp_fill(void *u, size_t off, size_t len, uint8_t *const *dst) {
  cb_tramp *t = (cb_tramp *)u;
  int rc = t->fill(t->user, off, len, dst);
  if (__atomic_load_n(&g_pins, __ATOMIC_RELAXED) > 0) __atomic_add_fetch(&g_pins_after_callback, 1, __ATOMIC_RELAXED);
  return rc;
}
static int tramp_drain(void *u, size_t off, size_t len, const uint8_t *const *src) {
  cb_tramp *t = (cb_tramp *)u;
  int rc = t->drain(t->user, off, len, src);
  if (__atomic_load_n(&g_pins, __ATOMIC_RELAXED) > 0) __atomic_add_fetch(&g_pins_after_callback, 1, __ATOMIC_RELAXED);
  return rc;
}
int __real_ozec_encode_cb(ozec_coder *, size_t, ozec_fill_fn, ozec_drain_fn, void *);
int __wrap_ozec_encode_cb(ozec_coder *c, size_t len, ozec_fill_fn fill, ozec_drain_fn drain, void *user) {
  at_device_call();
  cb_tramp t = {fill, drain, user};
  return __real_ozec_encode_cb(c, len, tramp_fill, tramp_drain, &t);
}
int __real_ozec_decode_cb(ozec_coder *, const uint8_t *, const int *, int, size_t, ozec_fill_fn, ozec_drain_fn, void *);
int __wrap_ozec_decode_cb(ozec_coder *c, const uint8_t *present, const int *e, int ne, size_t len, ozec_fill_fn fill,
                          ozec_drain_fn drain, void *user) {
  at_device_call();
  cb_tramp t = {fill, drain, user};
  return __real_ozec_decode_cb(c, present, e, ne, len, tramp_fill, tramp_drain, &t);
}
int __real_ozec_crc_update(int, uint32_t *, const uint8_t *, size_t);
int __wrap_ozec_crc_update(int t, uint32_t *s, const uint8_t *d, size_t len) {
  at_device_call();
  return __real_ozec_crc_update(t, s, d, len);
}
int __real_ozec_checksum_windows(int, const uint8_t *, size_t, size_t, uint32_t *, int);
int __wrap_ozec_checksum_windows(int t, const uint8_t *d, size_t len, size_t bpc, uint32_t *out, int be) {
  at_device_call();
  return __real_ozec_checksum_windows(t, d, len, bpc, out, be);
}
/* pinned allocations of the glue's arenas (ozec_host_alloc / ozec_host_free, wrapped): calls and live count */
static int g_host_allocs = 0, g_host_live = 0;
int __real_ozec_host_alloc(size_t, void **);
int __wrap_ozec_host_alloc(size_t bytes, void **out) {
  int rc = __real_ozec_host_alloc(bytes, out);
  if (rc == 0) {
    __atomic_add_fetch(&g_host_allocs, 1, __ATOMIC_RELAXED);
    __atomic_add_fetch(&g_host_live, 1, __ATOMIC_RELAXED);
  }
  return rc;
}
int __real_ozec_host_free(void *);
int __wrap_ozec_host_free(void *p) {
  if (p) __atomic_sub_fetch(&g_host_live, 1, __ATOMIC_RELAXED);
  return __real_ozec_host_free(p);
}
int mock_host_allocs(void) { return __atomic_load_n(&g_host_allocs, __ATOMIC_RELAXED); }
int mock_host_live(void) { return __atomic_load_n(&g_host_live, __ATOMIC_RELAXED); }
int mock_local_refs(void) { return __atomic_load_n(&g_local_refs, __ATOMIC_RELAXED); }
void mock_set_missing_class(const char *name) { snprintf(g_missing, sizeof g_missing, "%s", name ? name : ""); }

/* 1 and the exception if one is pending (then cleared), else 0 */
int mock_take_exception(char *cls, int cls_cap, char *msg, int msg_cap) {
  if (!g_exc_pending) return 0;
  snprintf(cls, (size_t)cls_cap, "%s", g_exc_class);
  snprintf(msg, (size_t)msg_cap, "%s", g_exc_msg);
  g_exc_pending = 0;
  return 1;
}
