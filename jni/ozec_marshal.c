/* ozec_marshal.c -- see ozec_marshal.h.  Plain C over the libozec C ABI; no JNI, no JVM. */
#include "ozec_marshal.h"

#include <stdio.h>
#include <string.h>

const char *ozm_exception_class(int rc) {
  switch (rc) {
    case OZEC_OK: return NULL;
    case OZEC_ECLOSED:
    case OZEC_EDEVICE: return "java/io/IOException";
    case OZEC_ENOTINVERTIBLE: return "java/lang/RuntimeException";
    case OZEC_ENOMEM: return "java/lang/OutOfMemoryError";
    case OZEC_EUNSUPPORTED: return "java/lang/UnsupportedOperationException";
    case OZEC_EMISMATCH: return "org/apache/hadoop/ozone/common/OzoneChecksumException";
    case OZEC_EINVAL:
    default: return "org/apache/hadoop/HadoopIllegalArgumentException";
  }
}

int ozm_fail(int rc, const char *msg, ozm_status *st) {
  if (!st) return rc;
  st->code = rc;
  const char *cls = ozm_exception_class(rc);
  snprintf(st->exception_class, sizeof(st->exception_class), "%s", cls ? cls : "");
  snprintf(st->message, sizeof(st->message), "%s", msg ? msg : (rc ? ozec_last_error() : ""));
  return rc;
}

static int ok(ozm_status *st) { return ozm_fail(OZEC_OK, "", st); }

int ozm_resolve(const ozm_buf *bufs, int n, int allow_absent, int64_t len, const uint8_t **out, ozm_status *st) {
  char msg[160];
  if (n < 0 || (n > 0 && (!bufs || !out))) return ozm_fail(OZEC_EINVAL, "Invalid buffer array", st);
  if (len < 0) return ozm_fail(OZEC_EINVAL, "Invalid data length, negative", st);
  for (int i = 0; i < n; ++i) {
    const ozm_buf *b = &bufs[i];
    if (!b->present) {
      if (!allow_absent) return ozm_fail(OZEC_EINVAL, "Invalid buffer found, not allowing null", st);
      out[i] = NULL;
      continue;
    }
    if (!b->base) { /* GetDirectBufferAddress of a heap buffer, or a failed pin */
      snprintf(msg, sizeof(msg), "Invalid buffer [%d]: no native address (not a direct buffer)", i);
      return ozm_fail(OZEC_EINVAL, msg, st);
    }
    if (b->offset < 0 || (b->capacity >= 0 && b->offset + len > b->capacity)) {
      snprintf(msg, sizeof(msg), "Invalid buffer [%d]: offset %lld + length %lld exceeds capacity %lld", i,
               (long long)b->offset, (long long)len, (long long)b->capacity);
      return ozm_fail(OZEC_EINVAL, msg, st);
    }
    out[i] = (const uint8_t *)b->base + b->offset;
  }
  return ok(st);
}

static int coder_shape(ozec_coder *c, int want_decoder, int *k, int *p, ozm_status *st) {
  int codec = 0, is_dec = 0;
  if (!c) return ozm_fail(OZEC_ECLOSED, "coder is closed", st); /* the Java handle is 0 after release() */
  int rc = ozec_coder_info(c, &codec, k, p, &is_dec);
  if (rc) return ozm_fail(rc, NULL, st);
  if (is_dec != want_decoder) return ozm_fail(OZEC_EINVAL, want_decoder ? "not a decoder" : "not an encoder", st);
  return ok(st);
}

int ozm_encode(ozec_coder *enc, const ozm_buf *in, int nin, const ozm_buf *out, int nout, int64_t len,
               ozm_status *st) {
  int k = 0, p = 0;
  char msg[96];
  if (coder_shape(enc, 0, &k, &p, st)) return st ? st->code : OZEC_EINVAL;
  if (nin != k) {
    snprintf(msg, sizeof(msg), "Invalid inputs length %d !=%d", nin, k); /* EncodingState.java:37-46 */
    return ozm_fail(OZEC_EINVAL, msg, st);
  }
  if (nout != p) {
    snprintf(msg, sizeof(msg), "Invalid outputs length %d !=%d", nout, p);
    return ozm_fail(OZEC_EINVAL, msg, st);
  }
  const uint8_t *ip[OZEC_MAX_K];
  const uint8_t *op[OZEC_MAX_ROWS];
  if (k > OZEC_MAX_K || p > OZEC_MAX_ROWS) return ozm_fail(OZEC_EUNSUPPORTED, "schema exceeds the kernel limits", st);
  if (ozm_resolve(in, nin, 0, len, ip, st) || ozm_resolve(out, nout, 0, len, op, st)) return st ? st->code : OZEC_EINVAL;
  int rc = ozec_encode(enc, ip, (uint8_t *const *)op, (size_t)len);
  return rc ? ozm_fail(rc, NULL, st) : ok(st);
}

int ozm_decode(ozec_coder *dec, const ozm_buf *in, int nin, const int *erased, int nerased, const ozm_buf *out,
               int nout, int64_t len, ozm_status *st) {
  int k = 0, p = 0;
  if (coder_shape(dec, 1, &k, &p, st)) return st ? st->code : OZEC_EINVAL;
  if (nin != k + p) return ozm_fail(OZEC_EINVAL, "Invalid inputs length", st); /* DecodingState.java:35-51 */
  if (nerased != nout || (nerased > 0 && !erased))
    return ozm_fail(OZEC_EINVAL, "erasedIndexes and outputs mismatch in length", st);
  if (nerased > p) return ozm_fail(OZEC_EINVAL, "Too many erased, not recoverable", st);
  const uint8_t *ip[256];
  const uint8_t *op[OZEC_MAX_ROWS];
  if (nin > 256 || nout > OZEC_MAX_ROWS) return ozm_fail(OZEC_EUNSUPPORTED, "schema exceeds the kernel limits", st);
  if (ozm_resolve(in, nin, 1, len, ip, st) || ozm_resolve(out, nout, 0, len, op, st)) return st ? st->code : OZEC_EINVAL;
  int rc = ozec_decode(dec, ip, erased, nerased, (uint8_t *const *)op, (size_t)len);
  return rc ? ozm_fail(rc, NULL, st) : ok(st);
}

int ozm_crc_update(int checksum_type, uint32_t *state, const ozm_buf *buf, int64_t len, ozm_status *st) {
  const uint8_t *p = NULL;
  if (!state) return ozm_fail(OZEC_EINVAL, "null state", st);
  if (len == 0) return ok(st);
  if (ozm_resolve(buf, 1, 0, len, &p, st)) return st ? st->code : OZEC_EINVAL;
  int rc = ozec_crc_update(checksum_type, state, p, (size_t)len);
  return rc ? ozm_fail(rc, NULL, st) : ok(st);
}

int ozm_checksum_windows(int checksum_type, const ozm_buf *buf, int64_t len, int64_t bpc, uint8_t *out,
                         int64_t out_cap, int64_t *written, ozm_status *st) {
  const uint8_t *p = NULL;
  if (written) *written = 0;
  if (bpc <= 0) return ozm_fail(OZEC_EINVAL, "bytesPerChecksum must be positive", st);
  if (len == 0) return ok(st); /* empty data: an empty checksum list (Checksum.java:171-178) */
  const int64_t nwin = (len + bpc - 1) / bpc;
  if (!out || out_cap < 4 * nwin) return ozm_fail(OZEC_EINVAL, "checksum output too small", st);
  if (ozm_resolve(buf, 1, 0, len, &p, st)) return st ? st->code : OZEC_EINVAL;
  /* big-endian 4-byte values are exactly Ints.toByteArray((int) getValue()) (Checksum.java:59-70) */
  int rc = ozec_checksum_windows(checksum_type, p, (size_t)len, (size_t)bpc, (uint32_t *)out, 1);
  if (rc) return ozm_fail(rc, NULL, st);
  if (written) *written = 4 * nwin;
  return ok(st);
}

/* bytes a buffer must hold from its offset, or fail */
static int need(const ozm_buf *b, int64_t bytes, const char *what, const uint8_t **out, ozm_status *st) {
  char msg[128];
  if (!b || !b->present || !b->base) {
    snprintf(msg, sizeof(msg), "%s buffer missing", what);
    return ozm_fail(OZEC_EINVAL, msg, st);
  }
  if (b->offset < 0 || (b->capacity >= 0 && b->offset + bytes > b->capacity)) {
    snprintf(msg, sizeof(msg), "%s buffer too small: %lld bytes needed", what, (long long)bytes);
    return ozm_fail(OZEC_EINVAL, msg, st);
  }
  *out = (const uint8_t *)b->base + b->offset;
  return ok(st);
}

int ozm_reconstruct_host_batch(ozec_coder *dec, const ozm_buf *stripes, int64_t stripe_stride, int64_t unit_stride,
                               const int *present, int npresent, const int *erased, int nerased, const ozm_buf *out,
                               int64_t num_stripes, int64_t cell_len, int checksum_type, int64_t bpc,
                               const ozm_buf *expected, const ozm_buf *out_crcs, const ozm_buf *mismatch,
                               ozm_status *st) {
  int k = 0, p = 0;
  if (coder_shape(dec, 1, &k, &p, st)) return st ? st->code : OZEC_EINVAL;
  if (num_stripes < 0 || cell_len < 0 || stripe_stride < 0 || unit_stride < 0)
    return ozm_fail(OZEC_EINVAL, "negative size or stride", st);
  if (bpc <= 0) return ozm_fail(OZEC_EINVAL, "bytesPerChecksum must be positive", st);
  if (nerased < 0 || (nerased > 0 && !erased) || npresent < 0 || (npresent > 0 && !present))
    return ozm_fail(OZEC_EINVAL, "erasedIndexes and outputs mismatch in length", st);
  if (nerased > p) return ozm_fail(OZEC_EINVAL, "Too many erased, not recoverable", st);
  if (num_stripes == 0 || cell_len == 0) return ok(st);
  const int64_t nwin = (cell_len + bpc - 1) / bpc, S = num_stripes;
  const uint8_t *in = NULL, *o = NULL, *oc = NULL, *ex = NULL, *mm = NULL;
  if (need(stripes, (S - 1) * stripe_stride + (int64_t)(k + p - 1) * unit_stride + cell_len, "stripe", &in, st))
    return st ? st->code : OZEC_EINVAL;
  if (nerased && (need(out, S * nerased * cell_len, "output", &o, st) ||
                  need(out_crcs, S * nerased * nwin * 4, "checksum output", &oc, st)))
    return st ? st->code : OZEC_EINVAL;
  if (expected && expected->present) {
    if (need(expected, S * (k + p) * nwin * 4, "expected checksum", &ex, st) ||
        need(mismatch, S * 4, "mismatch", &mm, st))
      return st ? st->code : OZEC_EINVAL;
  }
  int rc = ozec_reconstruct_crc_host_batch(dec, in, stripe_stride, unit_stride, present, npresent, erased, nerased,
                                           (uint8_t *)o, nerased * cell_len, cell_len, (size_t)S, (size_t)cell_len,
                                           checksum_type, (size_t)bpc, (const uint32_t *)ex, 1, (uint32_t *)oc, 1,
                                           (int32_t *)mm, 0);
  return rc ? ozm_fail(rc, NULL, st) : ok(st);
}
