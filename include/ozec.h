/*
 * ozec.h -- C ABI of libozec.so, the MI355X (gfx950) erasure-coding + chunk-checksum engine.
 *
 * This is the drop-in boundary for Ozone's EC raw-coder and chunk-checksum hot path.  Every entry point
 * takes plain pointers and sizes (no Java, Python or torch types) so a JNI shim, ctypes or any C caller can
 * bind it.  Each block below cites the reference interface it replaces (paths relative to the reference
 * checkout, EC/ = hadoop-hdds/erasurecode/src/main/java/org/apache/ozone/erasurecode/,
 * CM/ = hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/).  INTEGRATION.md shows the JNI
 * binding a maintainer would add on the Java side.
 *
 * Conventions
 *   - Return codes: 0 = OK, negative = error (OZEC_E*). ozec_last_error() returns a thread-local message
 *     mirroring the reference's exception text ("Not invertible", "... closed", "Invalid inputs length").
 *   - "host" entry points take host pointers (any alignment, pageable or pinned) and are synchronous, like
 *     RawErasureEncoder.encode (EC/rawcoder/RawErasureEncoder.java:66-97).  They stage through a
 *     process-global, per-GPU pinned buffer pool.
 *   - "_device" / "_batch" entry points take device pointers and a hipStream_t (NULL = the default stream
 *     of the current device) and are asynchronous on that stream.
 *   - Outputs are fully overwritten (the reference zero-fills, then accumulates: CoderUtil.java:84-98).
 *   - Inputs are never modified (TestRawCoderBase.java:180-220).
 */
#ifndef OZEC_H
#define OZEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes --------------------------------------------------------------------------- */
#define OZEC_OK 0
#define OZEC_EINVAL (-1)          /* HadoopIllegalArgumentException / IllegalArgumentException          */
#define OZEC_ENOTINVERTIBLE (-2)  /* RuntimeException("Not invertible"), GF256.java:214-217              */
#define OZEC_EDEVICE (-3)         /* HIP runtime error / no device                                       */
#define OZEC_ECLOSED (-4)         /* IOException("... closed") after release(), TestRawCoderBase.java:118-134 */
#define OZEC_ENOMEM (-5)
#define OZEC_EUNSUPPORTED (-6)    /* schema outside the compiled limits (k > OZEC_MAX_K, rows > OZEC_MAX_ROWS) */
#define OZEC_EMISMATCH (-7)       /* OzoneChecksumException: checksum mismatch, ChecksumData.java:118-150 */

/* ---- codecs and checksum types ------------------------------------------------------------ */
#define OZEC_CODEC_RS 0           /* ECReplicationConfig.EcCodec.RS  (hdds/client/ECReplicationConfig.java:44) */
#define OZEC_CODEC_XOR 1          /* ECReplicationConfig.EcCodec.XOR                                  */
/* numeric values follow ChecksumType in DatanodeClientProtocol.proto:422-434 */
#define OZEC_CHECKSUM_NONE 1
#define OZEC_CHECKSUM_CRC32 2
#define OZEC_CHECKSUM_CRC32C 3

#define OZEC_MAX_K 64             /* data units handled by the GPU kernels      */
#define OZEC_MAX_ROWS 16          /* parity rows / erased units per call        */

typedef struct ozec_coder ozec_coder; /* opaque encoder or decoder handle */

/* ---- library / device ------------------------------------------------------------------------ */
const char *ozec_last_error(void);
int ozec_version(void);
/* number of visible GPUs; 0 when none (the factory then throws, so CodecUtil falls back to rs_java:
 * CodecUtil.createRawEncoderWithFallback, EC/rawcoder/util/CodecUtil.java:55-82) */
int ozec_device_count(void);
/* hipSetDevice for the calling thread: the device of its device-pointer calls, and under OZEC_DEVICE_POLICY_CURRENT of
 * the coders it creates and its host calls.  In a process that chose no device list or policy (ozec_set_devices,
 * ozec_set_device_policy, OZEC_DEVICES, OZEC_DEVICE_POLICY), the first call also switches the PROCESS-WIDE policy to
 * OZEC_DEVICE_POLICY_CURRENT (the one-process-per-GPU model): from then on every thread's new coders go to that
 * thread's current device.  A device list or policy chosen later replaces that implicit policy. */
int ozec_set_device(int device);
/* ---- the GPUs of one drop-in process (one JVM per datanode / client drives every GPU of the node):
 * the device list is every visible GPU, or the OZEC_DEVICES environment variable ("0,2,5" / "all"), or this call
 * (n = 0 restores the default; duplicates allowed).  A coder is bound to one listed GPU when it is created (the
 * policy below); its host-buffer calls and stripe queues run there.  ozec_encode_crc_host_batch and
 * ozec_reconstruct_crc_host_batch split one batch into contiguous stripe ranges over the whole list, one pipeline per
 * GPU, run at once.  Coder-less host calls (CRCs of host buffers, ozec_host_alloc placement) run on a listed GPU each
 * thread is given on first use.  Device-pointer entry points run on the caller's current device. */
int ozec_set_devices(const int *devices, int n);
/* the device list: writes up to cap ordinals, returns how many there are */
int ozec_get_devices(int *devices, int cap);
#define OZEC_DEVICE_POLICY_ROUND_ROBIN 0 /* coders take the listed GPUs in turn (the default)                   */
#define OZEC_DEVICE_POLICY_NUMA 1        /* in turn among the listed GPUs on the creating thread's NUMA node      */
#define OZEC_DEVICE_POLICY_CURRENT 2     /* the creating thread's current device (one process per GPU)           */
/* also OZEC_DEVICE_POLICY=round_robin|numa|current in the environment */
int ozec_set_device_policy(int policy);
int ozec_device_policy(void);
/* wait for all work queued on the calling thread's current device (host-buffer calls are already synchronous) */
int ozec_synchronize(void);
/* give back the host-batch pipeline's chunk buffers (4 device + 4 pinned buffers of one chunk each: about 1.1 GiB
 * of HBM and, for pageable callers, of pinned memory with rs-6-3 1 MiB cells and 32-stripe chunks) and the staging
 * buffers of the idle host-call slots, on every GPU the process has used; the next call allocates again.  Device
 * memory goes back to HIP; pinned blocks are unregistered and their pages returned, their address ranges retired as
 * ozec_host_free does ("GPU faults") */
int ozec_release_staging(void);

/* ---- coder lifecycle: RawErasureCoderFactory.createEncoder/createDecoder
 *      (EC/rawcoder/RawErasureCoderFactory.java:29-56), RSRawEncoder/RSRawDecoder ctors
 *      (EC/rawcoder/RSRawEncoder.java:39-58, RSRawDecoder.java:57-71), XORRawEncoder/Decoder ctors,
 *      and the ISA-L bridge's initImpl (EC/rawcoder/NativeRSRawEncoder.java:39-51). ------------- */
int ozec_encoder_create(int codec, int num_data, int num_parity, ozec_coder **out);
int ozec_decoder_create(int codec, int num_data, int num_parity, ozec_coder **out);
/* RawErasureEncoder.release / RawErasureDecoder.release: idempotent; later calls return OZEC_ECLOSED */
int ozec_coder_release(ozec_coder *coder);
/* drop the caller's ownership of the handle (the Java object's cleaner / Python __del__); the memory goes with
 * the last owner: a stripe queue created on an encoder owns it too until ozec_stripe_queue_free, so releasing and
 * freeing the encoder first leaves the queue's calls failing with OZEC_ECLOSED, never touching freed memory */
void ozec_coder_free(ozec_coder *coder);
/* one more owner of the handle, to be dropped with one more ozec_coder_free */
int ozec_coder_retain(ozec_coder *coder);
/* 1 after ozec_coder_release, else 0 */
int ozec_coder_is_closed(const ozec_coder *coder);
/* the GPU the coder's host-buffer calls run on (negative: error) */
int ozec_coder_device(const ozec_coder *coder);
int ozec_coder_info(const ozec_coder *coder, int *codec, int *num_data, int *num_parity, int *is_decoder);

/* ---- encode: RawErasureEncoder.doEncode -> RSUtil.encodeData (EC/rawcoder/util/RSUtil.java:87-133),
 *      XORRawEncoder.doEncode (EC/rawcoder/XORRawEncoder.java:39-85); the JNI counterpart of
 *      hadoop's NativeRSRawEncoder.performEncodeImpl(inputs, inputOffsets, dataLen, outputs, outputOffsets)
 *      called from AbstractNativeRawEncoder.doEncode (EC/rawcoder/AbstractNativeRawEncoder.java:49-73).
 *      inputs[num_data], outputs[num_parity]: host pointers already advanced to position/offset. -------- */
int ozec_encode(ozec_coder *enc, const uint8_t *const *inputs, uint8_t *const *outputs, size_t len);

/* ---- decode: RawErasureDecoder.decode -> RSRawDecoder.doDecode (EC/rawcoder/RSRawDecoder.java:73-115),
 *      XORRawDecoder.doDecode (EC/rawcoder/XORRawDecoder.java:40-86); JNI counterpart of
 *      performDecodeImpl(inputs, inOffsets, dataLen, erased, outputs, outOffsets)
 *      (EC/rawcoder/AbstractNativeRawDecoder.java:49-75).
 *      inputs[num_data + num_parity]: NULL = erased or not read; the first num_data non-NULL inputs in
 *      ascending index order are used (RSRawDecoder.java:79-82).  erased[i] <-> outputs[i]. ----------- */
int ozec_decode(ozec_coder *dec, const uint8_t *const *inputs, const int *erased, int num_erased,
                uint8_t *const *outputs, size_t len);
/* The same two calls with the caller moving the bytes (round 6; the JNI glue's byte[] arrays, which it may hold
 * pinned only while it copies, AbstractNativeRawEncoder.java:75-86 copying them likewise): libozec runs its staged
 * pipeline in column chunks and calls fill(user, off, len, dst) to copy bytes [off, off + len) of every input into
 * dst[i] (its pinned staging; encode: the k inputs in order; decode: one slot per unit, k + p of them, NULL for the
 * units the decoder does not read) and drain(user, off, len, src) to copy the outputs' bytes [off, off + len) out of
 * src[r] (encode: the p outputs; decode: the n_erased outputs in erasedIndexes order; XOR outputs past the coded one
 * are zero) -- so the caller's copies of one chunk overlap the GPU's work on the other.  Both run on the calling
 * thread, never while a device call of this thread is being made; a nonzero return ends the call with that value.
 * present_units[u] != 0: the caller has unit u (ozec_decode's non-null inputs). */
typedef int (*ozec_fill_fn)(void *user, size_t off, size_t len, uint8_t *const *dst);
typedef int (*ozec_drain_fn)(void *user, size_t off, size_t len, const uint8_t *const *src);
int ozec_encode_cb(ozec_coder *encoder, size_t len, ozec_fill_fn fill, ozec_drain_fn drain, void *user);
int ozec_decode_cb(ozec_coder *decoder, const uint8_t *present_units, const int *erased, int n_erased, size_t len,
                   ozec_fill_fn fill, ozec_drain_fn drain, void *user);

/* ---- device-resident forms (same semantics, device pointers, async on `stream`) ---------------------- */
int ozec_encode_device(ozec_coder *enc, const uint8_t *const *d_inputs, uint8_t *const *d_outputs,
                       size_t len, void *stream);
int ozec_decode_device(ozec_coder *dec, const uint8_t *const *d_inputs, const int *erased,
                       int num_erased, uint8_t *const *d_outputs, size_t len, void *stream);

/* Batched stripes, the layout the datanode/bench keeps in HBM: unit u (0 <= u < k+p) of stripe s lives at
 *   base + s * stripe_stride + u * unit_stride            (bytes; any strides and lengths.  Every schema and
 *   the XOR codec run their 16-B vector kernels at any byte offset and unit spacing; the last
 *   1-15 bytes of a cell go bytewise)
 * encode reads units 0..k-1 of `d_in` and writes parity unit j to d_out + s*out_stripe_stride + j*out_unit_stride.
 * This is the batch entry SURVEY.md §7 "One stripe per call" asks for; the per-stripe semantics are exactly
 * RSUtil.encodeData's. */
int ozec_encode_batch(ozec_coder *enc, const uint8_t *d_in, int64_t in_stripe_stride,
                      int64_t in_unit_stride, uint8_t *d_out, int64_t out_stripe_stride,
                      int64_t out_unit_stride, size_t num_stripes, size_t len, void *stream);
/* decode a batch: `present` lists which of the k+p units are readable (ascending or not; the decoder uses
 * the first num_data in ascending order, as the reference does); erased[i] is written to
 * d_out + s*out_stripe_stride + i*out_unit_stride. */
int ozec_decode_batch(ozec_coder *dec, const uint8_t *d_in, int64_t in_stripe_stride,
                      int64_t in_unit_stride, const int *present, int num_present, const int *erased,
                      int num_erased, uint8_t *d_out, int64_t out_stripe_stride,
                      int64_t out_unit_stride, size_t num_stripes, size_t len, void *stream);

/* Fused encode + per-window checksum (north_star: "fused with encode, so each cell is read from HBM only
 * once").  crcs[s][u][w] (uint32, value of (int)getValue(), Checksum.java:59-70) for u in 0..k+p-1
 * (data then parity) and w in 0..ceil(len/bpc)-1.  big_endian != 0 stores each CRC byte-swapped, i.e.
 * exactly the 4 bytes Ints.toByteArray / Checksum.int2ByteString would produce. */
int ozec_encode_crc_batch(ozec_coder *enc, const uint8_t *d_in, int64_t in_stripe_stride,
                          int64_t in_unit_stride, uint8_t *d_out, int64_t out_stripe_stride,
                          int64_t out_unit_stride, size_t num_stripes, size_t len, int checksum_type,
                          size_t bytes_per_checksum, uint32_t *d_crcs, int big_endian, void *stream);

/* Fused encode + CRC over the datanode's block-group layout (BASELINE configs[3] / SURVEY §8(d) C4: one block
 * file per unit, 256 MiB blocks): unit u of stripe t of block group g at
 *   d_base + g * group_stride + u * unit_stride + t * len          (u < k: data blocks, k <= u < k+p: parity blocks)
 * All groups go in ONE launch (stripe g*stripes_per_group + t).  CRCs: d_crcs[g][t][unit][window] as in
 * ozec_encode_crc_batch (units = k data + the coded parity rows). */
int ozec_encode_crc_block_groups(ozec_coder *enc, uint8_t *d_base, int64_t group_stride, int64_t unit_stride,
                                 size_t num_groups, size_t stripes_per_group, size_t len, int checksum_type,
                                 size_t bytes_per_checksum, uint32_t *d_crcs, int big_endian, void *stream);

/* End-to-end fused encode (+ CRC) of stripes held in HOST memory (BASELINE configs[4] / SURVEY §8(d) C5: the
 * stripe batch a writer or datanode holds, one contiguous stripe range per GPU, §8(e)).  Same layouts and
 * semantics as ozec_encode_crc_batch with host pointers; checksum_type OZEC_CHECKSUM_NONE encodes only (h_crcs
 * may then be NULL).  Chunks of stripes_per_chunk stripes (0 = 32, tuning knob "e2e_chunk") are pipelined on the calling thread's device:
 * the H2D copies of chunk c+1, the kernel of chunk c and the D2H copies of chunk c-1 run at once on three streams.
 * Registered / pinned buffers (ozec_host_register, ozec_host_alloc) are DMA'd in place; pageable ones are staged
 * through NUMA-local pinned memory.  Synchronous: returns when parity and CRCs are in the caller's buffers. */
int ozec_encode_crc_host_batch(ozec_coder *enc, const uint8_t *h_in, int64_t in_stripe_stride,
                               int64_t in_unit_stride, uint8_t *h_out, int64_t out_stripe_stride,
                               int64_t out_unit_stride, size_t num_stripes, size_t len, int checksum_type,
                               size_t bytes_per_checksum, uint32_t *h_crcs, int big_endian, size_t stripes_per_chunk);

/* ---- chunk checksums: Checksum.computeChecksum(ByteBuffer / ChunkBuffer) (CM/Checksum.java:132-200) with
 *      ChunkBufferImplWithByteBuffer.iterate(bytesPerChecksum) (CM/ChunkBufferImplWithByteBuffer.java:78-98)
 *      and ChecksumByteBufferImpl/CrcIntTable per window (CM/ChecksumByteBuffer.java:51-121).
 *      One uint32 per window: ceil(len / bpc) values (0 for len == 0). ---------------------------------- */
int ozec_checksum_windows(int checksum_type, const uint8_t *data, size_t len, size_t bytes_per_checksum,
                          uint32_t *out, int big_endian);
int ozec_checksum_windows_device(int checksum_type, const uint8_t *d_data, size_t len,
                                 size_t bytes_per_checksum, uint32_t *d_out, int big_endian, void *stream);
/* many equally sized cells: cell c at d_base + c*cell_stride; out[c][w] */
int ozec_checksum_windows_batch(int checksum_type, const uint8_t *d_base, int64_t cell_stride,
                                size_t num_cells, size_t len, size_t bytes_per_checksum, uint32_t *d_out,
                                int big_endian, void *stream);
/* Checksum.verifyChecksum + ChecksumData.verifyChecksumDataMatches (CM/Checksum.java:241-297,
 * CM/ChecksumData.java:118-150): recompute and compare against expected[start_index ...].  Returns 0 when all
 * match, OZEC_EMISMATCH with *mismatch_index set to the first bad window otherwise. */
int ozec_checksum_verify(int checksum_type, const uint8_t *data, size_t len, size_t bytes_per_checksum,
                         const uint32_t *expected, size_t num_expected, size_t start_index,
                         int64_t *mismatch_index);

/* ---- batched checksum verify for the datanode scanner
 *      (KeyValueContainerCheck.verifyChecksum, hadoop-hdds/container-service/.../KeyValueContainerCheck.java:378-430)
 *      and Checksum.verifyChecksum over many chunks: recompute every window of num_cells cells and compare with
 *      d_expected[c][w] (stored big-endian when expected_big_endian, i.e. the raw ByteString bytes).
 *      d_mismatch[c] = -1 when every window matches, else the first failing window index. ------------------ */
int ozec_checksum_verify_batch(int checksum_type, const uint8_t *d_base, int64_t cell_stride, size_t num_cells,
                               size_t len, size_t bytes_per_checksum, const uint32_t *d_expected,
                               int expected_big_endian, int32_t *d_mismatch, void *stream);

/* ---- fused reconstruction, one pass over HBM for what
 *      ECReconstructionCoordinator.reconstructECBlockGroup (ECReconstructionCoordinator.java:240-352) does in three:
 *      verify the stored CRCs of the units read (ChunkInputStream.java:493-506), decode the erased units
 *      (RSRawDecoder / XORRawDecoder, same semantics as ozec_decode_batch), and compute the CRCs of the rebuilt units
 *      (BlockOutputStream.java:835).
 *      d_expected: [stripe][k+p][window] stored CRCs (NULL = skip verification; only the k units read are checked);
 *      d_out_crcs: [stripe][num_erased][window]; d_mismatch[s] = -1, or the smallest (unit * nwin + window) whose
 *      CRC did not verify. ---------------------------------------------------------------------------------- */
int ozec_reconstruct_crc_batch(ozec_coder *dec, const uint8_t *d_in, int64_t in_stripe_stride,
                               int64_t in_unit_stride, const int *present, int num_present, const int *erased,
                               int num_erased, uint8_t *d_out, int64_t out_stripe_stride, int64_t out_unit_stride,
                               size_t num_stripes, size_t len, int checksum_type, size_t bytes_per_checksum,
                               const uint32_t *d_expected, int expected_big_endian, uint32_t *d_out_crcs,
                               int out_big_endian, int32_t *d_mismatch, void *stream);
/* The same reconstruction for stripes held in HOST memory (the reconstruction coordinator's read buffers,
 * ECReconstructionCoordinator.java:240-352): same layouts and semantics with host pointers (h_expected
 * [stripe][k+p][window], h_out_crcs [stripe][num_erased][window], h_mismatch[stripe]; checksum_type CRC32 / CRC32C).
 * Only the k units the decoder reads are copied to the GPU, one rectangular copy per run of consecutive unit
 * indexes and chunk of stripes_per_chunk stripes (0 = the "e2e_chunk" knob); chunks are pipelined as in
 * ozec_encode_crc_host_batch (registered / pinned buffers DMA'd in place, pageable ones staged).  Synchronous. */
int ozec_reconstruct_crc_host_batch(ozec_coder *dec, const uint8_t *h_in, int64_t in_stripe_stride,
                                    int64_t in_unit_stride, const int *present, int num_present, const int *erased,
                                    int num_erased, uint8_t *h_out, int64_t out_stripe_stride, int64_t out_unit_stride,
                                    size_t num_stripes, size_t len, int checksum_type, size_t bytes_per_checksum,
                                    const uint32_t *h_expected, int expected_big_endian, uint32_t *h_out_crcs,
                                    int out_big_endian, int32_t *h_mismatch, size_t stripes_per_chunk);

/* ---- streaming ChecksumByteBuffer (CM/ChecksumByteBuffer.java:32-44): update(ByteBuffer) / getValue /
 *      reset over an opaque 32-bit state.  The GPU computes the raw CRC of the buffer and the host combines
 *      it with the running state (x^(8n) mod P shift), so results equal the sequential CrcIntTable. ---- */
uint32_t ozec_crc_reset(int checksum_type);
int ozec_crc_update(int checksum_type, uint32_t *state, const uint8_t *data, size_t len);
uint32_t ozec_crc_value(int checksum_type, uint32_t state); /* getValue() = ~state */

/* ---- host-side coding math (no GPU needed; exported for parity tests and for a Java-side cache) -------- */
/* RSUtil.genCauchyMatrix (EC/rawcoder/util/RSUtil.java:64-77): (k+p) x k, row-major */
int ozec_rs_encode_matrix(int num_data, int num_parity, uint8_t *matrix);
/* RSRawDecoder.generateDecodeMatrix (EC/rawcoder/RSRawDecoder.java:143-176) incl. its erased-order quirk */
int ozec_rs_decode_matrix(int num_data, int num_parity, const int *valid_indexes, const int *erased,
                          int num_erased, uint8_t *decode_matrix);
/* GF256.gfInvertMatrix (EC/rawcoder/util/GF256.java:191-250); `in` is clobbered like the reference's */
int ozec_gf_invert_matrix(uint8_t *in, uint8_t *out, int n);
uint8_t ozec_gf_mul(uint8_t a, uint8_t b);
/* ECReplicationConfig(String) parser (hdds/client/ECReplicationConfig.java:96-130): "rs-6-3-1024k" */
int ozec_parse_replication(const char *s, int *codec, int *num_data, int *num_parity, int *chunk_size);
/* crc(A||B) from crc(A), crc(B), |B| -- the combine primitive behind streaming update and stripe checksums */
uint32_t ozec_crc_combine(int checksum_type, uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* ---- writer-side stripe batching -------------------------------------------------------
 * ECKeyOutputStream encodes one stripe per RawErasureEncoder.encode call (ECKeyOutputStream.java:304; its stripe
 * queue :114, :501-543).  A stripe queue accepts stripes as they fill and encodes them in batches of
 * stripes_per_batch on the GPU (one fused encode (+ CRC) launch per batch, three batches in rotation).  Cells are
 * DMA'd straight from / into the caller's buffers when those are pinned (ozec_host_alloc, or any pinned host
 * memory), else through pinned staging.  The buffers given to submit must stay valid and unmodified until wait()
 * has returned for that ticket (or until ozec_stripe_queue_free). */
/* pinned host memory for cell buffers (the JNI side wraps it with NewDirectByteBuffer).  Its pages are placed on
 * the host NUMA node closest to the GPU (ozec_host_alloc: the calling thread's GPU, see ozec_set_devices), so DMA
 * never crosses the inter-socket fabric; every staging buffer libozec allocates itself is placed the same way. */
int ozec_host_alloc(size_t bytes, void **out);
int ozec_host_alloc_on(size_t bytes, int device, void **out);
/* unregister the block and retire its address range: its pages go back to the kernel, but the range is never used for
 * a later block ("GPU faults").  OZEC_EINVAL for a pointer ozec_host_alloc did not return; OZEC_EDEVICE
 * when the HIP runtime refuses to unregister it -- the block is then left mapped and registered (a leak, counted by
 * ozec_host_free_failures) rather than changed under a registration HIP still holds. */
int ozec_host_free(void *p);
uint64_t ozec_host_free_failures(void);
/* host NUMA node closest to `device` (-1: unknown / not a NUMA host) */
int ozec_device_numa_node(int device, int *node);
/* NUMA node holding the (touched) page at p, -1 if unknown -- placement diagnostics */
int ozec_host_page_node(const void *p, int *node);
/* copy `count` host regions (dst[i] <- src[i], bytes[i]) with libozec's parallel copy pool -- the workers of the NUMA
 * node of the calling thread's GPU, the caller taking part -- and return when all are done.  For glue layers that move
 * caller memory to and from pinned buffers themselves: the JNI drop-in copies Java byte[] regions (held with
 * GetPrimitiveArrayCritical for the copy only) into its pinned arena, as AbstractNativeRawEncoder.java:80-93 copies
 * heap arrays into direct buffers.  to_pinned: the destinations are pinned buffers a DMA reads next (streaming stores
 * where the CPU has them). */
int ozec_host_copy(void *const *dst, const void *const *src, const size_t *bytes, int count, int to_pinned);
/* pin caller-owned memory for DMA (e.g. one rank's stripe range of a batch shared between processes), placing
 * its pages on `device`'s NUMA node first (device < 0: no placement; only pages wholly inside the range move).
 * Placement is best effort: where the kernel refuses it the memory is pinned where it lies, and
 * ozec_host_placement_failures() counts such calls.  ozec_host_unregister undoes the pinning.
 * After ozec_host_unregister the caller may free or reuse the memory.  (Rounds 4-5 asked callers to keep such ranges
 * mapped until exit, after hipErrorIllegalAddress aborts in HIP's own pageable copies of a test process; round 6 found
 * no stale lock or registration left behind by either call -- ROCr's pointer info reports the range unknown right
 * after the unregister and after every pageable copy -- and the GPU suites run green with their ranges unregistered
 * and freed: DESIGN.md 4, "GPU faults".)  Memory that comes and goes often is cheaper from ozec_host_alloc /
 * ozec_host_free, which keep the registration cost off the hot path. */
int ozec_host_register(void *p, size_t bytes, int device);
uint64_t ozec_host_placement_failures(void);
int ozec_host_unregister(void *p);
typedef struct ozec_stripe_queue ozec_stripe_queue;
/* checksum_type OZEC_CHECKSUM_NONE: parity only; CRC32 / CRC32C: also the bpc-window CRCs of all k+p units,
 * written per stripe as crcs[unit][window] (window count from the stripe's length), big-endian if asked */
int ozec_stripe_queue_create(ozec_coder *encoder, size_t cell_len, size_t stripes_per_batch, int checksum_type,
                             size_t bpc, int big_endian, ozec_stripe_queue **out);
/* queue one stripe (k data cells of len <= cell_len bytes -> p parity cells, optional CRCs); a batch holds one
 * length, so a stripe of another length first launches the pending batch.  *ticket identifies the stripe. */
int ozec_stripe_queue_submit(ozec_stripe_queue *q, const uint8_t *const *data, uint8_t *const *parity, size_t len,
                             uint32_t *crcs, uint64_t *ticket);
/* launch the partly filled batch now */
int ozec_stripe_queue_flush(ozec_stripe_queue *q);
/* block until every stripe up to and including `ticket` has its parity (and CRCs) in the caller's buffers */
int ozec_stripe_queue_wait(ozec_stripe_queue *q, uint64_t ticket);
/* the queue's shape: data / parity units, coded parity rows (XOR: 1), cell length, checksum type and bpc (any may
 * be NULL) -- what a binding checks a submit's buffers against */
int ozec_stripe_queue_info(const ozec_stripe_queue *q, int *num_data, int *num_parity, int *rows, size_t *cell_len,
                           int *checksum_type, size_t *bytes_per_checksum);
/* introspection: batches in flight, first ticket of the oldest one (UINT64_MAX if none), stripes in filling batches */
int ozec_stripe_queue_state(ozec_stripe_queue *q, size_t *in_flight, uint64_t *oldest_in_flight_ticket,
                            size_t *filling);
/* complete every stripe not yet waited for (its parity / CRCs land in the caller's buffers), then destroy */
int ozec_stripe_queue_free(ozec_stripe_queue *q);

/* ---- COMPOSITE_CRC: CrcUtil / CrcComposer ------------------------------------------
 * OC/ = hadoop-ozone/common/src/main/java/org/apache/hadoop/ozone/client/checksum/.  CRC values are the stored
 * ints ((int)getValue()) in CrcUtil's reversed representation; checksum_type is OZEC_CHECKSUM_CRC32/CRC32C
 * (CrcUtil.getCrcPolynomialForType, OC/CrcUtil.java:53-64). */
/* CrcUtil.getMonomial (OC/CrcUtil.java:74-98): x^(8*len) mod P; OZEC_EINVAL for len < 0 */
int ozec_crc_monomial(int checksum_type, int64_t len_bytes, uint32_t *out);
/* CrcUtil.compose (OC/CrcUtil.java:124-127): crc_a * x^(8*len_b) xor crc_b; OZEC_EINVAL for len_b < 0 */
int ozec_crc_compose(int checksum_type, uint32_t crc_a, uint32_t crc_b, int64_t len_b, uint32_t *out);
/* CrcComposer (OC/CrcComposer.java:44-215).  stripe_length <= 0 means unstriped (newCrcComposer, :61-66);
 * otherwise newStripedCrcComposer (:84-95): one 4-byte big-endian CRC is emitted per stripe_length bytes. */
typedef struct ozec_crc_composer ozec_crc_composer;
int ozec_crc_composer_create(int checksum_type, int64_t bytes_per_crc_hint, int64_t stripe_length,
                             ozec_crc_composer **out);
/* update(int crcB, long bytesPerCrc) (:168-199): OZEC_EINVAL for a negative length, OZEC_EMISMATCH when the
 * position passes stripe_length without landing on it (the reference's IOException) */
int ozec_crc_composer_update(ozec_crc_composer *c, uint32_t crc, int64_t bytes_per_crc);
/* update(byte[] crcBuffer, int offset, int length, long bytesPerCrc) (:124-139): big-endian 4-byte CRCs,
 * OZEC_EINVAL unless len % 4 == 0 */
int ozec_crc_composer_update_bytes(ozec_crc_composer *c, const uint8_t *crc_bytes, size_t len, int64_t bytes_per_crc);
/* bytes the next digest returns */
size_t ozec_crc_composer_pending(const ozec_crc_composer *c);
/* digest() (:205-214): flush a partial stripe, copy the digest into out (OZEC_EINVAL if cap is too small,
 * nothing is consumed then), reset */
int ozec_crc_composer_digest(ozec_crc_composer *c, uint8_t *out, size_t cap, size_t *len);
void ozec_crc_composer_free(ozec_crc_composer *c);
/* Device batch: CrcComposer over each cell's window CRCs, in order: d_crcs[cell * crc_cell_stride + w] for
 * w < num_windows, every window bpc bytes long except the last (last_len bytes) -> d_out[cell].  This is the
 * chunk/block composite CRC of ECBlockChecksumComputer.computeCompositeCrc (client/checksum/
 * ECBlockChecksumComputer.java:105-195) over GPU-produced window CRCs; it equals the CRC of the whole cell. */
int ozec_crc_compose_windows_batch(int checksum_type, const uint32_t *d_crcs, int64_t crc_cell_stride,
                                   size_t num_cells, size_t num_windows, size_t bpc, size_t last_len,
                                   int crcs_big_endian, uint32_t *d_out, int out_big_endian, void *stream);

/* ---- per-call counters (SURVEY §5 metrics: the reference's ECReconstructionMetrics.java:34-41 and
 *      ContainerClientMetrics.java:41-42 count operations; a metrics2 source for the GPU coder publishes these).
 *      Process-wide, per entry-point family: calls, data bytes of successful calls, failed calls and host time
 *      spent inside the calls (for the asynchronous device entry points that is the enqueue time). --------- */
#define OZEC_OP_ENCODE 0          /* ozec_encode (the JNI drop-in's encode)                                 */
#define OZEC_OP_DECODE 1          /* ozec_decode                                                            */
#define OZEC_OP_ENCODE_DEVICE 2   /* ozec_encode_device / ozec_encode_batch                                 */
#define OZEC_OP_DECODE_DEVICE 3   /* ozec_decode_device / ozec_decode_batch                                 */
#define OZEC_OP_FUSED 4           /* ozec_encode_crc_batch / _block_groups / ozec_reconstruct_crc_batch      */
#define OZEC_OP_HOST_BATCH 5      /* ozec_encode_crc_host_batch / ozec_reconstruct_crc_host_batch           */
#define OZEC_OP_CHECKSUM 6        /* ozec_checksum_windows / _verify / ozec_crc_update (host buffers)       */
#define OZEC_OP_CHECKSUM_DEVICE 7 /* ozec_checksum_windows_batch / _device / ozec_checksum_verify_batch     */
#define OZEC_OP_QUEUE 8           /* ozec_stripe_queue_submit / _flush / _wait                              */
#define OZEC_NUM_OPS 9
typedef struct {
  uint64_t calls;
  uint64_t bytes;   /* data bytes: k * len per stripe coded, the bytes checksummed */
  uint64_t errors;
  uint64_t host_ns;
} ozec_op_stats;
int ozec_stats(int op, ozec_op_stats *out);
void ozec_stats_reset(void);
/* fused batch calls (ozec_encode_crc_batch, ozec_reconstruct_crc_batch) since the process started, by the route they
 * took: one fused kernel, or the unfused kernels (coding, then CRC passes) -- which kernels a workload reaches */
int ozec_fused_routes(uint64_t *fused, uint64_t *unfused);

/* ---- harness utilities ------------------------------------------------------------------------------- */
/* process-wide tuning knobs for A/B and profiling runs (a production process leaves them at their defaults; a set
 * knob applies to every caller's next call): kernels ("grid", "gf_variant", "crc_variant", "crc_grid", "crc_run",
 * "unit_map"; 0 = default) and host-buffer staging ("host_chunk" bytes per unit per chunk, "host_chunk_shared" the
 * same while other host-buffer calls are in flight (0: always host_chunk), "host_slots", "copy_threads" = helper
 * threads for pageable <-> pinned copies, 0 = copy on the calling thread, "copy_stream" -1..3, "queue_batches",
 * "e2e_chunk", "e2e_rect", "host_graph" = bytes per unit up to which a one-chunk staged encode / decode replays a
 * cached hipGraph of its H2D + kernel + D2H, default 256 KiB, 0 = off).  OZEC_EINVAL for an unknown key, a value out of range, or a kernel variant the library
 * does not hold. */
int ozec_set_tuning(const char *key, int64_t value);
/* the current value of a knob ozec_set_tuning sets (every key but "copy_threads" / "copy_stream"); OZEC_EINVAL for
 * any other key */
int ozec_get_tuning(const char *key, int64_t *value);
/* the kernel variants "gf_variant" / "crc_variant" accept besides 0: writes up to cap ids, returns how many exist */
int ozec_tuning_variants(const char *key, int *ids, int cap);
/* fill n bytes with splitmix64 stream `stream_id` of `seed` (tests/golden/synth.py is the CPU twin) */
int ozec_fill_splitmix64(uint8_t *d_dst, size_t n, uint64_t seed, uint64_t stream_id, void *stream);
/* same, many cells: cell c (stream first_stream + c) at d_base + c*cell_stride */
int ozec_fill_splitmix64_cells(uint8_t *d_base, int64_t cell_stride, size_t num_cells, size_t n,
                               uint64_t seed, uint64_t first_stream, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* OZEC_H */
