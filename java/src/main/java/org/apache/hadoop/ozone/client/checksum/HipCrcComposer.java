package org.apache.hadoop.ozone.client.checksum;

import java.io.DataInputStream;
import java.io.IOException;

import org.apache.hadoop.util.DataChecksum;
import org.apache.ozone.erasurecode.rawcoder.OzecNative;

/**
 * CrcComposer (OC/CrcComposer.java:44-215) over libozec's native composer (ozec_crc_composer_*): the same factories,
 * updates, digest layout (one 4-byte big-endian CRC per stripe, or one in all when unstriped) and exceptions --
 * IOException for an unsupported type, a stripe overrun ("Current position in stripe ... without stripe alignment.")
 * and a CRC byte run that is not a multiple of 4; IllegalArgumentException for a negative length.  The composition
 * itself (CrcUtil.compose / composeWithMonomial, x^(8n) mod P) runs natively, so ECBlockChecksumComputer and
 * ReplicatedBlockChecksumComputer can swap this in for CrcComposer.  The native state is freed by close().
 * OC/ = hadoop-ozone/common/src/main/java/org/apache/hadoop/ozone/client/checksum/
 */
public final class HipCrcComposer implements AutoCloseable {
  private long handle;

  private HipCrcComposer(long handle) {
    this.handle = handle;
  }

  /** CrcComposer.newCrcComposer (:61-66): all CRCs collapse into one value. */
  public static HipCrcComposer newCrcComposer(DataChecksum.Type type, long bytesPerCrcHint) throws IOException {
    return newStripedCrcComposer(type, bytesPerCrcHint, Long.MAX_VALUE);
  }

  /** CrcComposer.newStripedCrcComposer (:84-95): one CRC per stripeLength bytes of underlying data. */
  public static HipCrcComposer newStripedCrcComposer(DataChecksum.Type type, long bytesPerCrcHint, long stripeLength)
      throws IOException {
    return new HipCrcComposer(OzecNative.composerCreate(HipCrcUtil.checksumType(type), bytesPerCrcHint, stripeLength));
  }

  /** update(byte[] crcBuffer, int offset, int length, long bytesPerCrc) (:124-139). */
  public void update(byte[] crcBuffer, int offset, int length, long bytesPerCrc) throws IOException {
    OzecNative.composerUpdateBytes(handle(), crcBuffer, offset, length, bytesPerCrc);
  }

  /** update(DataInputStream, long numChecksumsToRead, long bytesPerCrc) (:151-158). */
  public void update(DataInputStream checksumIn, long numChecksumsToRead, long bytesPerCrc) throws IOException {
    for (long i = 0; i < numChecksumsToRead; ++i) {
      update(checksumIn.readInt(), bytesPerCrc);
    }
  }

  /** update(int crcB, long bytesPerCrc) (:168-199). */
  public void update(int crcB, long bytesPerCrc) throws IOException {
    OzecNative.composerUpdate(handle(), crcB, bytesPerCrc);
  }

  /** digest() (:205-214): flushes a partial stripe, returns the composed CRCs and resets. */
  public byte[] digest() {
    final long h = handle;
    if (h == 0) {
      throw new IllegalStateException("CrcComposer closed");
    }
    final byte[] out = new byte[OzecNative.composerPending(h)];
    OzecNative.composerDigest(h, out);
    return out;
  }

  @Override
  public void close() {
    if (handle != 0) {
      OzecNative.composerFree(handle);
      handle = 0;
    }
  }

  private long handle() throws IOException {
    if (handle == 0) {
      throw new IOException("CrcComposer closed");
    }
    return handle;
  }
}
