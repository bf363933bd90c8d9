package org.apache.hadoop.ozone.common;

import java.nio.ByteBuffer;
import java.util.ArrayList;
import java.util.List;

import org.apache.hadoop.hdds.protocol.datanode.proto.ContainerProtos.ChecksumType;
import org.apache.ozone.erasurecode.rawcoder.OzecNative;
import org.apache.ratis.thirdparty.com.google.protobuf.ByteString;
import org.apache.ratis.thirdparty.com.google.protobuf.UnsafeByteOperations;

/**
 * Batch hook of Checksum.computeChecksum(ChunkBuffer) (CM/Checksum.java:157-179): every bytesPerChecksum window of one
 * host buffer checksummed in one libozec call (ozec_checksum_windows), giving the same ChecksumData the reference's
 * window loop builds -- 4-byte big-endian int2ByteString((int) getValue()) per window, last window short
 * (Checksum.java:59-70).
 *
 * <p>{@link HipChecksumAccelerator} (the provider of hdds-common's ChecksumAccelerator seam,
 * java/patches/hdds-common-checksum-hook.patch) takes this path only when {@link #useGpu} says so: CRC32/CRC32C, a
 * single-buffer ChunkBuffer, libozec usable, and at least {@code ozone.checksum.hip.batch.min.bytes} bytes.
 * That threshold defaults to never: a host buffer crosses PCIe twice (staging copy, H2D, kernel, D2H) and on MI355X
 * that lost to one core's JDK-class CRC32C at every size measured, 16 KiB to 64 MiB, from 1 and from 16 threads
 * (bench.py --workload stream, checksum_windows_* rows, profiles/r03/).  Every other call runs the reference's own
 * loop unchanged, so the hook never makes Checksum slower.  The GPU CRC is used where the bytes are already on the
 * device (INTEGRATION.md §2).
 * CM/ = hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/
 */
public final class HipChecksum {
  /** Host buffers of at least this many bytes are checksummed on the GPU (default: none, see above). */
  static final long MIN_GPU_BYTES = Long.getLong("ozone.checksum.hip.batch.min.bytes", Long.MAX_VALUE);

  private HipChecksum() {
  }

  /** True when libozec_jni and a GPU are usable. */
  public static boolean isAvailable() {
    return OzecNative.isAvailable();
  }

  /**
   * Whether Checksum.computeChecksum(ChunkBuffer) should take the GPU batch path for this call: only the single-buffer
   * ChunkBuffer (ChunkBufferImplWithByteBuffer, CM/ChunkBufferImplWithByteBuffer.java:78-98), whose iterate() the
   * batch reproduces including the position it leaves; the buffer-list and incremental forms (whose iterate copies
   * across buffers, or rejects a bytesPerChecksum other than its increment) keep the reference's loop.
   */
  public static boolean useGpu(ChecksumType type, ChunkBuffer data) {
    if (MIN_GPU_BYTES == Long.MAX_VALUE || data.remaining() < MIN_GPU_BYTES) {
      return false;
    }
    if (type != ChecksumType.CRC32 && type != ChecksumType.CRC32C) {
      return false;
    }
    return data instanceof ChunkBufferImplWithByteBuffer && isAvailable();
  }

  /**
   * The ChecksumData of {@code data} (a single-buffer ChunkBuffer, see {@link #useGpu}).  Like the reference's
   * {@code data.iterate(bytesPerChecksum)} loop, it consumes the buffer: its position ends at its limit.
   */
  public static ChecksumData computeChecksum(ChecksumType type, ChunkBuffer data, int bytesPerChecksum) {
    final ByteBuffer b = data.asByteBufferList().get(0);
    final byte[] crcs = computeChecksumBytes(type == ChecksumType.CRC32 ? OzecNative.CHECKSUM_CRC32
        : OzecNative.CHECKSUM_CRC32C, b, bytesPerChecksum);
    b.position(b.limit());
    final List<ByteString> list = new ArrayList<>(crcs.length / 4);
    for (int i = 0; i < crcs.length; i += 4) {
      list.add(UnsafeByteOperations.unsafeWrap(crcs, i, 4));
    }
    return new ChecksumData(type, bytesPerChecksum, list);
  }

  /**
   * The concatenated 4-byte big-endian window CRCs of {@code data} from its position (ozec_checksum_windows).
   * @param type OzecNative.CHECKSUM_CRC32 or OzecNative.CHECKSUM_CRC32C
   */
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
