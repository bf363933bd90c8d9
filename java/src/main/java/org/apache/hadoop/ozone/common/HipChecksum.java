package org.apache.hadoop.ozone.common;

import java.nio.ByteBuffer;

import org.apache.ozone.erasurecode.rawcoder.OzecNative;

/**
 * Batch hook of Checksum.computeChecksum (CM/Checksum.java:157-200): every bytesPerChecksum window of one buffer
 * checksummed in one libozec call (ozec_checksum_windows).  Returns the concatenated 4-byte big-endian CRCs, i.e.
 * exactly the bytes of the ByteString list Checksum builds with int2ByteString((int) getValue())
 * (Checksum.java:59-70), last window short.  The buffer's position is not moved.
 */
public final class HipChecksum {
  private HipChecksum() {
  }

  /** True when libozec_jni and a GPU are usable (the hook falls back to the JDK CRCs otherwise). */
  public static boolean isAvailable() {
    return OzecNative.isAvailable();
  }

  /** @param type OzecNative.CHECKSUM_CRC32 or OzecNative.CHECKSUM_CRC32C */
  public static byte[] computeChecksumBytes(int type, ByteBuffer data, int bytesPerChecksum) {
    final int n = data.remaining();
    final int windows = n == 0 ? 0 : (int) ((n + (long) bytesPerChecksum - 1) / bytesPerChecksum);
    final byte[] out = new byte[4 * windows];
    if (n == 0) {
      return out;
    }
    if (data.isDirect()) {
      OzecNative.checksumWindowsDirect(type, data, data.position(), n, bytesPerChecksum, out);
    } else if (data.hasArray()) {
      OzecNative.checksumWindowsArray(type, data.array(), data.arrayOffset() + data.position(), n, bytesPerChecksum,
          out);
    } else {
      byte[] copy = new byte[n];
      data.duplicate().get(copy);
      OzecNative.checksumWindowsArray(type, copy, 0, n, bytesPerChecksum, out);
    }
    return out;
  }
}
