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
 *                                    copies heap arrays into direct buffers (:75-86), here they are pinned in place
 *   coderCreate / coderRelease    <- NativeRSRawEncoder ctor / release (EC/rawcoder/NativeRSRawEncoder.java:39-62)
 *   crcUpdate* / checksumWindows* <- ChecksumByteBuffer.update (CM/ChecksumByteBuffer.java:32-44) and
 *                                    Checksum.computeChecksum (CM/Checksum.java:157-200)
 *   queue*                        <- the stripe queue of ECKeyOutputStream (hadoop-ozone/client/.../ECKeyOutputStream.java:501-543)
 */
#include <jni.h>
#include <stdint.h>
#include <string.h>

#include "../include/ozec.h"
#include "ozec_marshal.h"

#define JNI_FN(name) Java_org_apache_ozone_erasurecode_rawcoder_OzecNative_##name
#define MAX_BUFS 256

static void throw_status(JNIEnv *env, const ozm_status *st) {
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

/* Java byte[][] (+ int[] offsets): references first (JNI calls are not allowed inside a critical region), then
 * every array pinned with GetPrimitiveArrayCritical; unpin() releases them. */
typedef struct {
  jbyteArray arr[MAX_BUFS];
  int n;
} pinned_set;

static int collect_arrays(JNIEnv *env, jobjectArray arr, jintArray offs, ozm_buf *bufs, pinned_set *ps,
                          ozm_status *st) {
  ps->n = 0;
  if (!arr || !offs) return ozm_fail(OZEC_EINVAL, "Invalid buffer array, null", st);
  const jsize len = (*env)->GetArrayLength(env, arr);
  if (len > MAX_BUFS || (*env)->GetArrayLength(env, offs) < len)
    return ozm_fail(OZEC_EINVAL, "Invalid buffer / offset arrays", st);
  jint o[MAX_BUFS];
  (*env)->GetIntArrayRegion(env, offs, 0, len, o);
  for (jsize i = 0; i < len; ++i) {
    ps->arr[i] = (jbyteArray)(*env)->GetObjectArrayElement(env, arr, i);
    memset(&bufs[i], 0, sizeof(bufs[i]));
    if (ps->arr[i]) {
      bufs[i].present = 1;
      bufs[i].capacity = (*env)->GetArrayLength(env, ps->arr[i]);
      bufs[i].offset = o[i];
    }
  }
  ps->n = (int)len;
  return 0;
}

static void pin(JNIEnv *env, pinned_set *ps, ozm_buf *bufs) {
  for (int i = 0; i < ps->n; ++i)
    if (ps->arr[i]) bufs[i].base = (*env)->GetPrimitiveArrayCritical(env, ps->arr[i], NULL);
}

/* mode 0 copies back (outputs) if the VM handed out a copy; JNI_ABORT for inputs, which are never modified */
static void unpin(JNIEnv *env, pinned_set *ps, ozm_buf *bufs, jint mode) {
  for (int i = 0; i < ps->n; ++i)
    if (ps->arr[i]) {
      if (bufs[i].base) (*env)->ReleasePrimitiveArrayCritical(env, ps->arr[i], (void *)bufs[i].base, mode);
      (*env)->DeleteLocalRef(env, ps->arr[i]);
    }
  ps->n = 0;
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
  pinned_set pi, po;
  ozm_status st;
  pi.n = po.n = 0;
  int rc = collect_arrays(env, in, inOff, ib, &pi, &st);
  if (!rc) rc = collect_arrays(env, out, outOff, ob, &po, &st);
  if (!rc) {
    pin(env, &pi, ib);
    pin(env, &po, ob);
    rc = ozm_encode((ozec_coder *)(intptr_t)h, ib, pi.n, ob, po.n, len, &st); /* no JNI call in between */
  }
  unpin(env, &po, ob, 0);
  unpin(env, &pi, ib, JNI_ABORT);
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
  pinned_set pi, po;
  ozm_status st;
  pi.n = po.n = 0;
  int rc = int_array(env, erased, er, MAX_BUFS, &ne, &st);
  if (!rc) rc = collect_arrays(env, in, inOff, ib, &pi, &st);
  if (!rc) rc = collect_arrays(env, out, outOff, ob, &po, &st);
  if (!rc) {
    pin(env, &pi, ib);
    pin(env, &po, ob);
    rc = ozm_decode((ozec_coder *)(intptr_t)h, ib, pi.n, er, ne, ob, po.n, len, &st);
  }
  unpin(env, &po, ob, 0);
  unpin(env, &pi, ib, JNI_ABORT);
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
    b.present = 1;
    b.capacity = (*env)->GetArrayLength(env, arr);
    b.offset = off;
    b.base = (*env)->GetPrimitiveArrayCritical(env, arr, NULL);
    rc = ozm_crc_update(type, &s, &b, len, &st);
    if (b.base) (*env)->ReleasePrimitiveArrayCritical(env, arr, (void *)b.base, JNI_ABORT);
  }
  if (rc) throw_status(env, &st);
  return (jint)s;
}

/* Checksum.computeChecksum of one direct buffer region: big-endian CRC bytes of every window into out; returns the
 * number of bytes written (4 per window) */
JNIEXPORT jint JNICALL JNI_FN(checksumWindowsDirect)(JNIEnv *env, jclass cls, jint type, jobject buf, jint off, jint len,
                                                     jint bpc, jbyteArray out) {
  (void)cls;
  ozm_buf b = {0};
  ozm_status st;
  int64_t written = 0;
  if (!out) {
    ozm_fail(OZEC_EINVAL, "null checksum output", &st);
    throw_status(env, &st);
    return 0;
  }
  b.present = buf != NULL;
  if (buf) {
    b.base = (*env)->GetDirectBufferAddress(env, buf);
    b.capacity = (int64_t)(*env)->GetDirectBufferCapacity(env, buf);
    b.offset = off;
  }
  const jsize cap = (*env)->GetArrayLength(env, out);
  uint8_t *o = (uint8_t *)(*env)->GetPrimitiveArrayCritical(env, out, NULL);
  int rc = ozm_checksum_windows(type, &b, len, bpc, o, cap, &written, &st);
  if (o) (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
  if (rc) throw_status(env, &st);
  return (jint)written;
}

JNIEXPORT jint JNICALL JNI_FN(checksumWindowsArray)(JNIEnv *env, jclass cls, jint type, jbyteArray data, jint off,
                                                    jint len, jint bpc, jbyteArray out) {
  (void)cls;
  ozm_buf b = {0};
  ozm_status st;
  int64_t written = 0;
  if (!out) {
    ozm_fail(OZEC_EINVAL, "null checksum output", &st);
    throw_status(env, &st);
    return 0;
  }
  const jsize cap = (*env)->GetArrayLength(env, out);
  if (data) {
    b.present = 1;
    b.capacity = (*env)->GetArrayLength(env, data);
    b.offset = off;
    b.base = (*env)->GetPrimitiveArrayCritical(env, data, NULL);
  }
  uint8_t *o = (uint8_t *)(*env)->GetPrimitiveArrayCritical(env, out, NULL);
  int rc = ozm_checksum_windows(type, &b, len, bpc, o, cap, &written, &st);
  if (o) (*env)->ReleasePrimitiveArrayCritical(env, out, o, 0);
  if (data && b.base) (*env)->ReleasePrimitiveArrayCritical(env, data, (void *)b.base, JNI_ABORT);
  if (rc) throw_status(env, &st);
  return (jint)written;
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
