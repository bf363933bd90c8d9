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

/* presence, offsets and capacities of n buffers for `len` bytes each; with need_base, their addresses too */
static int check_bufs(const ozm_buf *bufs, int n, int allow_absent, int64_t len, int need_base, ozm_status *st) {
  char msg[160];
  if (n < 0 || (n > 0 && !bufs)) return ozm_fail(OZEC_EINVAL, "Invalid buffer array", st);
  if (len < 0) return ozm_fail(OZEC_EINVAL, "Invalid data length, negative", st);
  for (int i = 0; i < n; ++i) {
    const ozm_buf *b = &bufs[i];
    if (!b->present) {
      if (!allow_absent) return ozm_fail(OZEC_EINVAL, "Invalid buffer found, not allowing null", st);
      continue;
    }
    if (need_base && !b->base) { /* GetDirectBufferAddress of a heap buffer */
      snprintf(msg, sizeof(msg), "Invalid buffer [%d]: no native address (not a direct buffer)", i);
      return ozm_fail(OZEC_EINVAL, msg, st);
    }
    if (b->offset < 0 || (b->capacity >= 0 && b->offset + len > b->capacity)) {
      snprintf(msg, sizeof(msg), "Invalid buffer [%d]: offset %lld + length %lld exceeds capacity %lld", i,
               (long long)b->offset, (long long)len, (long long)b->capacity);
      return ozm_fail(OZEC_EINVAL, msg, st);
    }
  }
  return ok(st);
}

int ozm_resolve(const ozm_buf *bufs, int n, int allow_absent, int64_t len, const uint8_t **out, ozm_status *st) {
  if (n > 0 && !out) return ozm_fail(OZEC_EINVAL, "Invalid buffer array", st);
  if (check_bufs(bufs, n, allow_absent, len, 1, st)) return st ? st->code : OZEC_EINVAL;
  for (int i = 0; i < n; ++i) out[i] = bufs[i].present ? (const uint8_t *)bufs[i].base + bufs[i].offset : NULL;
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

int ozm_encode_check(ozec_coder *enc, const ozm_buf *in, int nin, const ozm_buf *out, int nout, int64_t len,
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
  if (k > OZEC_MAX_K || p > OZEC_MAX_ROWS) return ozm_fail(OZEC_EUNSUPPORTED, "schema exceeds the kernel limits", st);
  if (check_bufs(in, nin, 0, len, 0, st) || check_bufs(out, nout, 0, len, 0, st)) return st ? st->code : OZEC_EINVAL;
  return ok(st);
}

int ozm_encode(ozec_coder *enc, const ozm_buf *in, int nin, const ozm_buf *out, int nout, int64_t len,
               ozm_status *st) {
  if (ozm_encode_check(enc, in, nin, out, nout, len, st)) return st ? st->code : OZEC_EINVAL;
  const uint8_t *ip[OZEC_MAX_K];
  const uint8_t *op[OZEC_MAX_ROWS];
  if (ozm_resolve(in, nin, 0, len, ip, st) || ozm_resolve(out, nout, 0, len, op, st)) return st ? st->code : OZEC_EINVAL;
  int rc = ozec_encode(enc, ip, (uint8_t *const *)op, (size_t)len);
  return rc ? ozm_fail(rc, NULL, st) : ok(st);
}

int ozm_decode_check(ozec_coder *dec, const ozm_buf *in, int nin, const int *erased, int nerased, const ozm_buf *out,
                     int nout, int64_t len, ozm_status *st) {
  int k = 0, p = 0;
  if (coder_shape(dec, 1, &k, &p, st)) return st ? st->code : OZEC_EINVAL;
  if (nin != k + p) return ozm_fail(OZEC_EINVAL, "Invalid inputs length", st); /* DecodingState.java:35-51 */
  if (nerased != nout || (nerased > 0 && !erased))
    return ozm_fail(OZEC_EINVAL, "erasedIndexes and outputs mismatch in length", st);
  if (nerased > p) return ozm_fail(OZEC_EINVAL, "Too many erased, not recoverable", st);
  if (nin > 256 || nout > OZEC_MAX_ROWS) return ozm_fail(OZEC_EUNSUPPORTED, "schema exceeds the kernel limits", st);
  if (check_bufs(in, nin, 1, len, 0, st) || check_bufs(out, nout, 0, len, 0, st)) return st ? st->code : OZEC_EINVAL;
  return ok(st);
}

int ozm_decode(ozec_coder *dec, const ozm_buf *in, int nin, const int *erased, int nerased, const ozm_buf *out,
               int nout, int64_t len, ozm_status *st) {
  if (ozm_decode_check(dec, in, nin, erased, nerased, out, nout, len, st)) return st ? st->code : OZEC_EINVAL;
  const uint8_t *ip[256];
  const uint8_t *op[OZEC_MAX_ROWS];
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

/* a * b + c in int64 without wrapping; 0 on overflow or a negative term */
static int span(int64_t a, int64_t b, int64_t c, int64_t *out) {
  int64_t m;
  if (a < 0 || b < 0 || c < 0 || __builtin_mul_overflow(a, b, &m) || __builtin_add_overflow(m, c, out)) return 0;
  return 1;
}

int ozm_queue_submit(ozec_stripe_queue *q, const ozm_buf *data, int nd, const ozm_buf *parity, int np, int64_t len,
                     const ozm_buf *crcs, uint64_t *ticket, ozm_status *st) {
  int k = 0, p = 0, rows = 0, ctype = 0;
  size_t cell = 0, bpc = 0;
  char msg[128];
  if (!q) return ozm_fail(OZEC_ECLOSED, "HipStripeQueue closed", st);
  int rc = ozec_stripe_queue_info(q, &k, &p, &rows, &cell, &ctype, &bpc);
  if (rc) return ozm_fail(rc, NULL, st);
  if (nd != k || np != p) {
    snprintf(msg, sizeof(msg), "Invalid inputs/outputs length %d/%d != %d/%d", nd, np, k, p);
    return ozm_fail(OZEC_EINVAL, msg, st);
  }
  if (len <= 0 || (uint64_t)len > cell) {
    snprintf(msg, sizeof(msg), "stripe length %lld not in [1, %zu]", (long long)len, cell);
    return ozm_fail(OZEC_EINVAL, msg, st);
  }
  const uint8_t *dp[OZEC_MAX_K], *pp[256], *cp = NULL;
  if (k > OZEC_MAX_K || p > 256) return ozm_fail(OZEC_EUNSUPPORTED, "schema exceeds the kernel limits", st);
  if (ozm_resolve(data, nd, 0, len, dp, st) || ozm_resolve(parity, np, 0, len, pp, st)) return st ? st->code : OZEC_EINVAL;
  if (ctype != OZEC_CHECKSUM_NONE && crcs && crcs->present) {
    const int64_t nwin = ((int64_t)len + (int64_t)bpc - 1) / (int64_t)bpc;
    int64_t bytes;
    if (!span((int64_t)(k + rows) * nwin, 4, 0, &bytes)) return ozm_fail(OZEC_EINVAL, "checksum size overflows", st);
    if (need(crcs, bytes, "checksum", &cp, st)) return st ? st->code : OZEC_EINVAL;
  }
  rc = ozec_stripe_queue_submit(q, dp, (uint8_t *const *)pp, (size_t)len, (uint32_t *)cp, ticket);
  return rc ? ozm_fail(rc, NULL, st) : ok(st);
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
  /* every layout size in checked arithmetic: a huge Java stride must not wrap past the capacity check */
  int64_t last_unit, in_bytes, out_bytes, crc_bytes, exp_bytes, ner_cells, ner_crcs, units_crcs, out_stride;
  if (!span((int64_t)(k + p - 1), unit_stride, cell_len, &last_unit) ||
      !span(S - 1, stripe_stride, last_unit, &in_bytes) || !span(S, nerased, 0, &ner_cells) ||
      !span(ner_cells, cell_len, 0, &out_bytes) || !span(ner_cells, nwin, 0, &ner_crcs) ||
      !span(ner_crcs, 4, 0, &crc_bytes) || !span(S, (int64_t)(k + p) * nwin, 0, &units_crcs) ||
      !span(units_crcs, 4, 0, &exp_bytes) || !span(nerased, cell_len, 0, &out_stride))
    return ozm_fail(OZEC_EINVAL, "buffer layout size overflows", st);
  if (need(stripes, in_bytes, "stripe", &in, st)) return st ? st->code : OZEC_EINVAL;
  if (nerased && (need(out, out_bytes, "output", &o, st) || need(out_crcs, crc_bytes, "checksum output", &oc, st)))
    return st ? st->code : OZEC_EINVAL;
  if (expected && expected->present) {
    if (need(expected, exp_bytes, "expected checksum", &ex, st) || need(mismatch, S * 4, "mismatch", &mm, st))
      return st ? st->code : OZEC_EINVAL;
  }
  int rc = ozec_reconstruct_crc_host_batch(dec, in, stripe_stride, unit_stride, present, npresent, erased, nerased,
                                           (uint8_t *)o, out_stride, cell_len, (size_t)S, (size_t)cell_len,
                                           checksum_type, (size_t)bpc, (const uint32_t *)ex, 1, (uint32_t *)oc, 1,
                                           (int32_t *)mm, 0);
  return rc ? ozm_fail(rc, NULL, st) : ok(st);
}

/* ---------------------------------------------------------------- COMPOSITE_CRC */

/* like ozm_fail, with the reference's exception class instead of the status's default */
static int fail_as(int rc, const char *cls, const char *msg, ozm_status *st) {
  ozm_fail(rc, msg, st);
  if (st) snprintf(st->exception_class, sizeof(st->exception_class), "%s", cls);
  return rc;
}

static int crc_type_ok(int checksum_type, ozm_status *st) {
  char msg[96];
  if (checksum_type == OZEC_CHECKSUM_CRC32 || checksum_type == OZEC_CHECKSUM_CRC32C) return ok(st);
  snprintf(msg, sizeof(msg), "No CRC polynomial could be associated with type: %d", checksum_type);
  return fail_as(OZEC_EINVAL, "java/io/IOException", msg, st);
}

int ozm_crc_monomial(int checksum_type, int64_t len_bytes, uint32_t *out, ozm_status *st) {
  if (crc_type_ok(checksum_type, st)) return st ? st->code : OZEC_EINVAL;
  int rc = ozec_crc_monomial(checksum_type, len_bytes, out);
  return rc ? fail_as(rc, "java/lang/IllegalArgumentException", NULL, st) : ok(st);
}

int ozm_crc_compose(int checksum_type, uint32_t crc_a, uint32_t crc_b, int64_t len_b, uint32_t *out, ozm_status *st) {
  if (crc_type_ok(checksum_type, st)) return st ? st->code : OZEC_EINVAL;
  int rc = ozec_crc_compose(checksum_type, crc_a, crc_b, len_b, out);
  return rc ? fail_as(rc, "java/lang/IllegalArgumentException", NULL, st) : ok(st);
}

int ozm_composer_create(int checksum_type, int64_t bytes_per_crc_hint, int64_t stripe_length,
                        ozec_crc_composer **out, ozm_status *st) {
  if (crc_type_ok(checksum_type, st)) return st ? st->code : OZEC_EINVAL;
  /* newStripedCrcComposer's getMonomial(bytesPerCrcHint) rejects a negative hint */
  if (bytes_per_crc_hint < 0) {
    char msg[96];
    snprintf(msg, sizeof(msg), "lengthBytes must be positive, got %lld", (long long)bytes_per_crc_hint);
    return fail_as(OZEC_EINVAL, "java/lang/IllegalArgumentException", msg, st);
  }
  int rc = ozec_crc_composer_create(checksum_type, bytes_per_crc_hint, stripe_length, out);
  return rc ? ozm_fail(rc, NULL, st) : ok(st);
}

int ozm_composer_update(ozec_crc_composer *c, uint32_t crc, int64_t bytes_per_crc, ozm_status *st) {
  if (!c) return fail_as(OZEC_ECLOSED, "java/io/IOException", "CrcComposer closed", st);
  int rc = ozec_crc_composer_update(c, crc, bytes_per_crc);
  if (rc == OZEC_EMISMATCH) return fail_as(rc, "java/io/IOException", NULL, st);
  return rc ? fail_as(rc, "java/lang/IllegalArgumentException", NULL, st) : ok(st);
}

int ozm_composer_update_bytes(ozec_crc_composer *c, const uint8_t *buf, int64_t cap, int64_t offset, int64_t length,
                              int64_t bytes_per_crc, ozm_status *st) {
  char msg[160];
  if (!c) return fail_as(OZEC_ECLOSED, "java/io/IOException", "CrcComposer closed", st);
  if (length % 4 != 0) {
    snprintf(msg, sizeof(msg),
             "Trying to update CRC from byte array with length '%lld' at offset '%lld' which is not a multiple of 4!",
             (long long)length, (long long)offset);
    return fail_as(OZEC_EINVAL, "java/io/IOException", msg, st);
  }
  if (length <= 0) return ok(st);
  if (!buf) return fail_as(OZEC_EINVAL, "java/lang/NullPointerException", "crcBuffer is null", st);
  /* CrcComposer.update(byte[], int, int, long) (OC/CrcComposer.java:124-139): one CrcUtil.readInt (OC/CrcUtil.java:
   * 181-193) and one update per CRC, so the CRCs before a failing read are composed, as in the reference */
  for (int64_t o = offset; o < offset + length; o += 4) {
    if (o + 4 > cap) { /* readInt's bounds check */
      snprintf(msg, sizeof(msg), "readInt out of bounds: buf.length=%lld, offset=%lld", (long long)cap, (long long)o);
      return fail_as(OZEC_EINVAL, "java/io/IOException", msg, st);
    }
    if (o < 0) { /* buf[offset + 0] of a negative offset: the JVM's array bounds check */
      snprintf(msg, sizeof(msg), "Index %lld out of bounds for length %lld", (long long)o, (long long)cap);
      return fail_as(OZEC_EINVAL, "java/lang/ArrayIndexOutOfBoundsException", msg, st);
    }
    const uint8_t *b = buf + o;
    const uint32_t v = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
    if (ozm_composer_update(c, v, bytes_per_crc, st)) return st ? st->code : OZEC_EINVAL;
  }
  return ok(st);
}

int ozm_composer_digest(ozec_crc_composer *c, uint8_t *out, int64_t cap, int64_t *written, ozm_status *st) {
  size_t len = 0;
  if (written) *written = 0;
  if (!c) return fail_as(OZEC_ECLOSED, "java/io/IOException", "CrcComposer closed", st);
  int rc = ozec_crc_composer_digest(c, out, cap < 0 ? 0 : (size_t)cap, &len);
  if (rc) return ozm_fail(rc, NULL, st);
  if (written) *written = (int64_t)len;
  return ok(st);
}
