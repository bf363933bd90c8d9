package org.apache.hadoop.ozone.common;

import java.nio.ByteBuffer;

import org.apache.ozone.erasurecode.rawcoder.OzecNative;

/**
 * ChecksumByteBuffer (CM/ChecksumByteBuffer.java:32-44) whose updates run on the GPU through libozec
 * (ozec_crc_update: the raw CRC of the buffer is computed per 16 KiB window in parallel and combined with the
 * running register on the host, so every value equals CrcIntTable's / java.util.zip's).  Only updates of at least
 * {@code ozone.checksum.hip.min.bytes} bytes go to the GPU, and by default none do: for a buffer in host memory one
 * GPU round trip (staging copy, H2D, kernel, D2H) never beat one core's SSE4.2 CRC32C on MI355X at any size from
 * 1 B to 16 MiB (bench.py --workload stream, profiles/r02/bench/stream_*.json).  The GPU's CRC pays where the
 * bytes are on the device anyway: fused with encode (HipStripeQueue, ozec_encode_crc_*), in reconstruction and in
 * the scanner's batched verify.  Smaller updates use the reflected byte table below.
 * CM/ = hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/
 */
public final class HipChecksumByteBuffer implements ChecksumByteBuffer {
  private static final int MIN_GPU_BYTES = Integer.getInteger("ozone.checksum.hip.min.bytes", Integer.MAX_VALUE);
  private static final int[] CRC32_TABLE = table(0xEDB88320);
  private static final int[] CRC32C_TABLE = table(0x82F63B78);

  private final int type;
  private final int[] table;
  private int crc;

  /** @param type OzecNative.CHECKSUM_CRC32 or OzecNative.CHECKSUM_CRC32C */
  public HipChecksumByteBuffer(int type) {
    if (type != OzecNative.CHECKSUM_CRC32 && type != OzecNative.CHECKSUM_CRC32C) {
      throw new IllegalArgumentException("unsupported checksum type " + type);
    }
    this.type = type;
    this.table = type == OzecNative.CHECKSUM_CRC32 ? CRC32_TABLE : CRC32C_TABLE;
    reset();
  }

  private static int[] table(int poly) {
    int[] t = new int[256];
    for (int i = 0; i < 256; i++) {
      int c = i;
      for (int b = 0; b < 8; b++) {
        c = (c & 1) != 0 ? (c >>> 1) ^ poly : c >>> 1;
      }
      t[i] = c;
    }
    return t;
  }

  @Override
  public void update(ByteBuffer buffer) {
    final int n = buffer.remaining();
    if (n == 0) {
      return;
    }
    final int pos = buffer.position();
    if (n >= MIN_GPU_BYTES && buffer.isDirect()) {
      crc = OzecNative.crcUpdateDirect(type, crc, buffer, pos, n);
    } else if (n >= MIN_GPU_BYTES && buffer.hasArray()) {
      crc = OzecNative.crcUpdateArray(type, crc, buffer.array(), buffer.arrayOffset() + pos, n);
    } else {
      for (int i = 0; i < n; i++) {
        crc = (crc >>> 8) ^ table[(crc ^ buffer.get(pos + i)) & 0xff];
      }
    }
    buffer.position(pos + n);
  }

  /** Overrides the interface default, which wraps the array in a read-only buffer that has no accessible array. */
  @Override
  public void update(byte[] b, int off, int len) {
    if (len >= MIN_GPU_BYTES) {
      crc = OzecNative.crcUpdateArray(type, crc, b, off, len);
      return;
    }
    for (int i = 0; i < len; i++) {
      crc = (crc >>> 8) ^ table[(crc ^ b[off + i]) & 0xff];
    }
  }

  @Override
  public void update(int b) {
    crc = (crc >>> 8) ^ table[(crc ^ b) & 0xff];
  }

  @Override
  public long getValue() {
    return (~crc) & 0xffffffffL;
  }

  @Override
  public void reset() {
    crc = 0xffffffff;
  }
}
