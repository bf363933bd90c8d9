package org.apache.ozone.erasurecode.rawcoder;

import java.io.IOException;
import java.nio.ByteBuffer;

/**
 * JNI entry points of libozec_jni (jni/ozec_jni.c) over the libozec C ABI (include/ozec.h).  Loaded once per
 * JVM; {@link #checkAvailable()} throws when the library or a GPU is missing, which makes the HIP coder
 * constructors throw and CodecUtil fall back to the next coder (CodecUtil.java:62-78).
 * System property {@code ozone.ec.hip.library} may name the library file; otherwise java.library.path is searched.
 *
 * <p>One JVM drives every GPU of its node (a datanode or client is one process): {@code ozone.ec.hip.devices} (e.g.
 * {@code 0,1,2,3}; default: every visible GPU) lists them and {@code ozone.ec.hip.device.policy}
 * ({@code round_robin}, the default; {@code numa}; {@code current}) says how coders are bound to them -- each coder
 * (one per ECKeyOutputStream, ECKeyOutputStream.java:117, and per reconstruction, ECBlockReconstructedStripeInputStream
 * .java:232) runs its calls and stripe queues on its own GPU, and a host batch is split over all listed GPUs
 * (ozec_set_devices, include/ozec.h).
 */
public final class OzecNative {
  public static final int CODEC_RS = 0;
  public static final int CODEC_XOR = 1;
  /** ChecksumType numbers of DatanodeClientProtocol.proto:422-434. */
  public static final int CHECKSUM_NONE = 1;
  public static final int CHECKSUM_CRC32 = 2;
  public static final int CHECKSUM_CRC32C = 3;

  private static final Throwable LOAD_FAILURE;

  static {
    Throwable failure = null;
    try {
      String path = System.getProperty("ozone.ec.hip.library");
      if (path != null) {
        System.load(path);
      } else {
        System.loadLibrary("ozec_jni");
      }
    } catch (Throwable t) {
      failure = t;
    }
    LOAD_FAILURE = failure;
    if (failure == null) {
      configureDevices(System.getProperty("ozone.ec.hip.devices"), System.getProperty("ozone.ec.hip.device.policy"));
    }
  }

  /** Apply the device properties; a bad value leaves the library's default (every visible GPU, round robin). */
  static void configureDevices(String devices, String policy) {
    try {
      if (devices != null && !devices.trim().isEmpty() && !"all".equals(devices.trim())) {
        final String[] parts = devices.split(",");
        final int[] list = new int[parts.length];
        for (int i = 0; i < parts.length; ++i) {
          list[i] = Integer.parseInt(parts[i].trim());
        }
        setDevices(list);
      }
      if (policy != null) {
        setDevicePolicy("numa".equals(policy) ? DEVICE_POLICY_NUMA
            : "current".equals(policy) ? DEVICE_POLICY_CURRENT : DEVICE_POLICY_ROUND_ROBIN);
      }
    } catch (IOException | RuntimeException e) {
      // a device the node does not have (IOException) or a malformed value: keep the default
    }
  }

  private OzecNative() {
  }

  /** True when the JNI library loaded and at least one GPU is visible. */
  public static boolean isAvailable() {
    return LOAD_FAILURE == null && deviceCount() > 0;
  }

  public static void checkAvailable() {
    if (LOAD_FAILURE != null) {
      throw new UnsupportedOperationException("libozec_jni is not loadable", LOAD_FAILURE);
    }
    if (deviceCount() <= 0) {
      throw new UnsupportedOperationException("no HIP device is visible");
    }
  }

  public static native int deviceCount();

  public static final int DEVICE_POLICY_ROUND_ROBIN = 0;
  public static final int DEVICE_POLICY_NUMA = 1;
  public static final int DEVICE_POLICY_CURRENT = 2;

  // ---- the GPUs of this process (ozec_set_devices / ozec_get_devices / ozec_set_device_policy / ozec_coder_device)
  /**
   * The GPUs coders and host batches use from now on; an empty array restores every visible GPU.
   * @throws IOException a listed ordinal is not a GPU of this node (the list is left unchanged)
   */
  public static native void setDevices(int[] devices) throws IOException;

  public static native int[] getDevices();

  public static native void setDevicePolicy(int policy);

  /** The GPU a coder handle's calls run on; IOException for a null handle. */
  static native int coderDevice(long handle) throws IOException;

  // ---- coders (ozec_encoder_create / ozec_decoder_create / ozec_coder_release + ozec_coder_free)
  static native long coderCreate(boolean decoder, int codec, int numData, int numParity);

  static native void coderRelease(long handle);

  // ---- AbstractNativeRawEncoder.performEncodeImpl / AbstractNativeRawDecoder.performDecodeImpl
  static native void encodeDirect(long handle, ByteBuffer[] inputs, int[] inputOffsets, int dataLen,
      ByteBuffer[] outputs, int[] outputOffsets);

  static native void encodeArrays(long handle, byte[][] inputs, int[] inputOffsets, int dataLen,
      byte[][] outputs, int[] outputOffsets);

  static native void decodeDirect(long handle, ByteBuffer[] inputs, int[] inputOffsets, int dataLen,
      int[] erasedIndexes, ByteBuffer[] outputs, int[] outputOffsets);

  static native void decodeArrays(long handle, byte[][] inputs, int[] inputOffsets, int dataLen,
      int[] erasedIndexes, byte[][] outputs, int[] outputOffsets);

  // ---- checksums (ozec_crc_update, ozec_checksum_windows)
  public static native int crcUpdateDirect(int type, int state, ByteBuffer buffer, int offset, int length);

  public static native int crcUpdateArray(int type, int state, byte[] array, int offset, int length);

  /** Big-endian CRC of every bytesPerChecksum window into out; returns the bytes written (4 per window). */
  public static native int checksumWindowsDirect(int type, ByteBuffer data, int offset, int length,
      int bytesPerChecksum, byte[] out);

  public static native int checksumWindowsArray(int type, byte[] data, int offset, int length,
      int bytesPerChecksum, byte[] out);

  // ---- pinned host memory + stripe queue (ozec_host_alloc, ozec_stripe_queue_*)
  public static native ByteBuffer allocatePinned(int bytes);

  public static native void freePinned(ByteBuffer buffer);

  static native long queueCreate(long encoder, int cellLen, int stripesPerBatch, int checksumType,
      int bytesPerChecksum);

  static native long queueSubmit(long queue, ByteBuffer[] data, int[] dataOffsets, ByteBuffer[] parity,
      int[] parityOffsets, int length, ByteBuffer crcs, int crcsOffset);

  static native void queueWait(long queue, long ticket);

  static native void queueFree(long queue);

  // ---- batch reconstruction from host buffers (ozec_reconstruct_crc_host_batch, SURVEY §8(f) row 1)
  static native void reconstructHostBatch(long decoder, ByteBuffer stripes, long stripeStride, long unitStride,
      int[] presentUnits, int[] erasedIndexes, ByteBuffer out, int numStripes, int cellLength, int checksumType,
      int bytesPerChecksum, ByteBuffer expectedChecksums, ByteBuffer outChecksums, ByteBuffer mismatch);

  // ---- COMPOSITE_CRC (ozec_crc_monomial / ozec_crc_compose / ozec_crc_composer_* / ozec_crc_compose_windows_batch;
  //      CrcUtil.java:74-127, CrcComposer.java:44-215 under hadoop-ozone/common/.../ozone/client/checksum/)
  public static native int crcMonomial(int type, long lengthBytes);

  public static native int crcCompose(int type, int crcA, int crcB, long lengthB);

  public static native long composerCreate(int type, long bytesPerCrcHint, long stripeLength) throws IOException;

  public static native void composerUpdate(long composer, int crc, long bytesPerCrc) throws IOException;

  public static native void composerUpdateBytes(long composer, byte[] crcBuffer, int offset, int length,
      long bytesPerCrc) throws IOException;

  public static native int composerPending(long composer);

  public static native int composerDigest(long composer, byte[] out);

  public static native void composerFree(long composer);

  /** Device pointers and stream as longs: for callers that keep the window CRCs in HBM. */
  public static native void composeWindowsBatch(int type, long deviceCrcs, long crcCellStride, long numCells,
      long numWindows, long bytesPerCrc, long lastLength, boolean crcsBigEndian, long deviceOut,
      boolean outBigEndian, long stream);
}
