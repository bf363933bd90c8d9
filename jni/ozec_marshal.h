/*
 * ozec_marshal.h -- the JNI-free half of the Java drop-in (jni/ozec_jni.c is the other half).
 *
 * What the reference's ISA-L bridge does between Java buffers and the native coder, stated over plain C:
 *   AbstractNativeRawEncoder.doEncode (EC/rawcoder/AbstractNativeRawEncoder.java:49-73) turns every direct
 *   ByteBuffer into (buffer, position) and calls performEncodeImpl(inputs, inputOffsets, dataLen, outputs,
 *   outputOffsets); AbstractNativeRawDecoder.doDecode (:49-75) does the same with null inputs kept and the
 *   erasedIndexes passed through.  Heap arrays arrive as (byte[], offset) (ByteArrayEncodingState.inputOffsets).
 * The JNI layer only resolves each Java object to an ozm_buf (address of element 0 + byte offset + capacity); this
 * file validates the resolved arguments, calls libozec and maps its status to the Java exception the reference
 * throws, so all of that is testable on CPU without a JVM (tests/test_jni_marshal.py).
 * EC/ = hadoop-hdds/erasurecode/src/main/java/org/apache/ozone/erasurecode/
 */
#ifndef OZEC_MARSHAL_H
#define OZEC_MARSHAL_H

#include <stdint.h>

#include "../include/ozec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One Java buffer argument, resolved:
 *   direct ByteBuffer : base = GetDirectBufferAddress(b), offset = b.position(), capacity = b.capacity()
 *   byte[] + offset   : base = GetPrimitiveArrayCritical(a), offset = the state's offset, capacity = a.length
 *   null slot         : present = 0 (decode inputs only; Java null)
 * capacity < 0 means unknown (no bounds check). */
typedef struct {
  const void *base;
  int64_t offset;
  int64_t capacity;
  int present;
} ozm_buf;

/* A failed call: the Java exception to throw (JNI class name, e.g. "java/io/IOException") and its message. */
typedef struct {
  int code; /* OZEC_* status */
  char exception_class[64];
  char message[256];
} ozm_status;

/* JNI class of the exception the reference throws for a libozec status (NULL for OZEC_OK):
 *   OZEC_EINVAL         -> org/apache/hadoop/HadoopIllegalArgumentException (EncodingState/DecodingState checks)
 *   OZEC_ECLOSED        -> java/io/IOException ("... closed", TestRawCoderBase.java:118-134)
 *   OZEC_ENOTINVERTIBLE -> java/lang/RuntimeException ("Not invertible", GF256.java:214-217)
 *   OZEC_EDEVICE        -> java/io/IOException
 *   OZEC_ENOMEM         -> java/lang/OutOfMemoryError
 *   OZEC_EUNSUPPORTED   -> java/lang/UnsupportedOperationException
 *   OZEC_EMISMATCH      -> org/apache/hadoop/ozone/common/OzoneChecksumException (ChecksumData.java:118-150) */
const char *ozm_exception_class(int rc);
/* fill *st from rc and a message (NULL message: ozec_last_error()); returns rc */
int ozm_fail(int rc, const char *msg, ozm_status *st);

/* Resolve n buffers to addresses base + offset; absent slots become NULL when allow_absent, else an error.
 * Every present buffer must hold len bytes from its offset (offset >= 0, offset + len <= capacity). */
int ozm_resolve(const ozm_buf *bufs, int n, int allow_absent, int64_t len, const uint8_t **out, ozm_status *st);

/* ozm_encode / ozm_decode's validation alone (coder shape, counts, every present buffer's offset + len within its
 * capacity) without reading any address: the JNI glue checks heap arrays with it before it copies their regions */
int ozm_encode_check(ozec_coder *enc, const ozm_buf *in, int nin, const ozm_buf *out, int nout, int64_t len,
                     ozm_status *st);
int ozm_decode_check(ozec_coder *dec, const ozm_buf *in, int nin, const int *erased, int nerased, const ozm_buf *out,
                     int nout, int64_t len, ozm_status *st);
/* performEncodeImpl(inputs, inputOffsets, dataLen, outputs, outputOffsets): nin == k, nout == p */
int ozm_encode(ozec_coder *enc, const ozm_buf *in, int nin, const ozm_buf *out, int nout, int64_t len,
               ozm_status *st);
/* performDecodeImpl(inputs, inputOffsets, dataLen, erased, outputs, outputOffsets): nin == k + p (absent = null),
 * nout == nerased */
int ozm_decode(ozec_coder *dec, const ozm_buf *in, int nin, const int *erased, int nerased, const ozm_buf *out,
               int nout, int64_t len, ozm_status *st);

/* ChecksumByteBuffer.update(ByteBuffer / byte[], off, len) over a running register (CM/ChecksumByteBuffer.java:32-44) */
int ozm_crc_update(int checksum_type, uint32_t *state, const ozm_buf *buf, int64_t len, ozm_status *st);
/* Checksum.computeChecksum over one buffer (CM/Checksum.java:157-200): the 4-byte big-endian CRC of every
 * bytes_per_checksum window into out (out_cap bytes, >= 4 * ceil(len / bpc)); *written = bytes stored */
int ozm_checksum_windows(int checksum_type, const ozm_buf *buf, int64_t len, int64_t bytes_per_checksum,
                         uint8_t *out, int64_t out_cap, int64_t *written, ozm_status *st);

/* Batch reconstruction of stripes held in direct buffers (ECReconstructionCoordinator's read buffers; libozec
 * ozec_reconstruct_crc_host_batch).  stripes: [S][k+p][cell_len] at stripe_stride / unit_stride (absent and erased
 * units are never read); out: [S][nerased][cell_len]; out_crcs: [S][nerased][nwin] and expected: [S][k+p][nwin]
 * 4-byte big-endian values (Ints.toByteArray, Checksum.java:59-70); mismatch: [S] native-order ints, -1 or the first
 * failing unit * nwin + window.  expected (and mismatch) may be absent: no verification.  Every buffer's capacity is
 * checked against its layout before anything runs. */
int ozm_reconstruct_host_batch(ozec_coder *dec, const ozm_buf *stripes, int64_t stripe_stride, int64_t unit_stride,
                               const int *present, int npresent, const int *erased, int nerased, const ozm_buf *out,
                               int64_t num_stripes, int64_t cell_len, int checksum_type, int64_t bytes_per_checksum,
                               const ozm_buf *expected, const ozm_buf *out_crcs, const ozm_buf *mismatch,
                               ozm_status *st);

/* HipStripeQueue.submit (ozec_stripe_queue_submit): nd == k data cells and np == p parity cells of len bytes from
 * their offsets; crcs (absent = no CRCs wanted) must hold (k + coded rows) * ceil(len / bpc) 4-byte values from its
 * offset when the queue computes checksums.  *ticket identifies the stripe. */
int ozm_queue_submit(ozec_stripe_queue *q, const ozm_buf *data, int nd, const ozm_buf *parity, int np, int64_t len,
                     const ozm_buf *crcs, uint64_t *ticket, ozm_status *st);

/* ---- COMPOSITE_CRC: CrcUtil / CrcComposer (OC/CrcUtil.java:74-127, OC/CrcComposer.java:44-215; OC/ =
 * hadoop-ozone/common/src/main/java/org/apache/hadoop/ozone/client/checksum/) with the reference's exceptions:
 * a negative length -> java.lang.IllegalArgumentException (CrcUtil.getMonomial), an unsupported type or a composer
 * position past its stripe -> java.io.IOException (CrcUtil.getCrcPolynomialForType, CrcComposer.update), a CRC
 * byte run whose length is not a multiple of 4 -> java.io.IOException, a CRC read past the array -> java.io.IOException
 * "readInt out of bounds: ..." after the CRCs before it were composed (CrcUtil.readInt, OC/CrcUtil.java:181-193), a
 * negative offset -> java.lang.ArrayIndexOutOfBoundsException (the array access). */
int ozm_crc_monomial(int checksum_type, int64_t len_bytes, uint32_t *out, ozm_status *st);
int ozm_crc_compose(int checksum_type, uint32_t crc_a, uint32_t crc_b, int64_t len_b, uint32_t *out, ozm_status *st);
int ozm_composer_create(int checksum_type, int64_t bytes_per_crc_hint, int64_t stripe_length,
                        ozec_crc_composer **out, ozm_status *st);
int ozm_composer_update(ozec_crc_composer *c, uint32_t crc, int64_t bytes_per_crc, ozm_status *st);
/* update(byte[] crcBuffer, int offset, int length, long bytesPerCrc): buf is the array, cap its length */
int ozm_composer_update_bytes(ozec_crc_composer *c, const uint8_t *buf, int64_t cap, int64_t offset, int64_t length,
                              int64_t bytes_per_crc, ozm_status *st);
/* digest() into out (cap bytes; at least ozec_crc_composer_pending()); *written = digest length */
int ozm_composer_digest(ozec_crc_composer *c, uint8_t *out, int64_t cap, int64_t *written, ozm_status *st);

#ifdef __cplusplus
}
#endif
#endif /* OZEC_MARSHAL_H */
