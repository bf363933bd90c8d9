package org.apache.hadoop.ozone.common;

import java.nio.ByteBuffer;

import org.apache.ozone.erasurecode.rawcoder.OzecNative;

/**
 * ChecksumByteBuffer (CM/ChecksumByteBuffer.java:32-44) over the runtime's own CRC -- the ChecksumByteBufferImpl the
 * reference's factory builds on java.util.zip.CRC32 / CRC32C (CM/ChecksumByteBufferFactory.java:74-89,
 * CM/ChecksumByteBufferImpl.java:77-106) -- that can hand large updates of host buffers to the GPU.
 *
 * <p>Every update goes to that host CRC unless it is at least {@code ozone.checksum.hip.min.bytes} bytes long, and by
 * default none is: for a buffer in host memory one GPU round trip (staging copy, H2D, kernel, D2H) never beat one
 * core's JDK-class CRC32C on MI355X from 1 B to 64 MiB (bench.py --workload stream: crc_update_* and
 * checksum_windows_* rows, profiles/r03/).  So installed with its default this class costs one extra virtual call per
 * update and nothing else.  The GPU's CRC pays where the bytes are on the device anyway: fused with encode
 * (HipStripeQueue, ozec_encode_crc_*), in reconstruction and in the scanner's batched verify (INTEGRATION.md §2).
 *
 * <p>After a GPU update the value is the host segment's CRC combined with the register before it
 * (update(P, E) = update(INIT, E) ^ shift(P ^ INIT, |E|), the CRC recursion being affine), so any mix of host and GPU
 * updates returns exactly what the host CRC alone returns.
 * CM/ = hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/
 */
public final class HipChecksumByteBuffer implements ChecksumByteBuffer {
  /** Updates of at least this many bytes go to the GPU (default: none). */
  static final int MIN_GPU_BYTES = Integer.getInteger("ozone.checksum.hip.min.bytes", Integer.MAX_VALUE);
  private static final int INIT = 0xffffffff;

  private final int type;
  private final int poly;
  private final ChecksumByteBuffer host;
  private int prefix = INIT;  // register of everything before the host segment
  private long hostLen;       // bytes the host CRC has seen since its last reset
  private boolean split;      // a GPU update happened since reset()

  /** True when the GPU threshold is set and libozec_jni is usable; HipChecksumAccelerator.wrap (the provider of the
   * hdds-common ChecksumAccelerator seam, java/patches/hdds-common-checksum-hook.patch) installs this class only then. */
  public static boolean enabled() {
    return MIN_GPU_BYTES != Integer.MAX_VALUE && OzecNative.isAvailable();
  }

  /**
   * @param type OzecNative.CHECKSUM_CRC32 or OzecNative.CHECKSUM_CRC32C
   * @param host the runtime's CRC of that type (ChecksumByteBufferFactory's JDK-backed impl)
   */
  public HipChecksumByteBuffer(int type, ChecksumByteBuffer host) {
    if (type != OzecNative.CHECKSUM_CRC32 && type != OzecNative.CHECKSUM_CRC32C) {
      throw new IllegalArgumentException("unsupported checksum type " + type);
    }
    this.type = type;
    this.poly = type == OzecNative.CHECKSUM_CRC32 ? 0xEDB88320 : 0x82F63B78;
    this.host = host;
    reset();
  }

  @Override
  public void update(ByteBuffer buffer) {
    final int n = buffer.remaining();
    if (n >= MIN_GPU_BYTES && (buffer.isDirect() || buffer.hasArray())) {
      final int pos = buffer.position();
      final int reg = register();
      prefix = buffer.isDirect() ? OzecNative.crcUpdateDirect(type, reg, buffer, pos, n)
          : OzecNative.crcUpdateArray(type, reg, buffer.array(), buffer.arrayOffset() + pos, n);
      buffer.position(pos + n);
      restartHostSegment();
      return;
    }
    host.update(buffer);
    hostLen += n;
  }

  @Override
  public void update(byte[] b, int off, int len) {
    if (len >= MIN_GPU_BYTES) {
      prefix = OzecNative.crcUpdateArray(type, register(), b, off, len);
      restartHostSegment();
      return;
    }
    host.update(b, off, len);
    hostLen += len;
  }

  @Override
  public void update(int b) {
    host.update(b);
    hostLen++;
  }

  @Override
  public long getValue() {
    return split ? (~register()) & 0xffffffffL : host.getValue();
  }

  @Override
  public void reset() {
    host.reset();
    prefix = INIT;
    hostLen = 0;
    split = false;
  }

  private void restartHostSegment() {
    host.reset();
    hostLen = 0;
    split = true;
  }

  /** The CRC register (before the final inversion) of everything updated since reset(). */
  private int register() {
    final int h = ~(int) host.getValue();
    return split ? h ^ shift(prefix ^ INIT, hostLen) : h;
  }

  /** v * x^(8n) mod P in the reflected domain: the register after n zero bytes with no init (zlib's
   * crc32_combine operator squaring: O(log n) 32x32 GF(2) matrix products). */
  private int shift(int v, long n) {
    if (n == 0 || v == 0) {
      return v;
    }
    int[] odd = new int[32];
    int[] even = new int[32];
    odd[0] = poly;  // operator of one zero bit
    for (int i = 1, row = 1; i < 32; i++, row <<= 1) {
      odd[i] = row;
    }
    square(even, odd);  // two zero bits
    square(odd, even);  // four zero bits
    do {
      square(even, odd);  // one zero byte on the first pass, then 2^k bytes
      if ((n & 1) != 0) {
        v = times(even, v);
      }
      n >>>= 1;
      if (n == 0) {
        break;
      }
      square(odd, even);
      if ((n & 1) != 0) {
        v = times(odd, v);
      }
      n >>>= 1;
    } while (n != 0);
    return v;
  }

  private static int times(int[] mat, int vec) {
    int sum = 0;
    for (int i = 0; vec != 0; i++, vec >>>= 1) {
      if ((vec & 1) != 0) {
        sum ^= mat[i];
      }
    }
    return sum;
  }

  private static void square(int[] square, int[] mat) {
    for (int i = 0; i < 32; i++) {
      square[i] = times(mat, mat[i]);
    }
  }
}
