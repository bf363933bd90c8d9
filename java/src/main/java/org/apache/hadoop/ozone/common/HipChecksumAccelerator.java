package org.apache.hadoop.ozone.common;

import org.apache.hadoop.hdds.protocol.datanode.proto.ContainerProtos.ChecksumType;
import org.apache.ozone.erasurecode.rawcoder.OzecNative;

/**
 * The MI355X {@link ChecksumAccelerator}: the provider the hdds-common checksum seam
 * (java/patches/hdds-common-checksum-hook.patch: ChecksumAccelerator / ChecksumAccelerators, looked up with
 * ServiceLoader) finds in this jar through META-INF/services/org.apache.hadoop.ozone.common.ChecksumAccelerator.
 *
 * <p>hdds-common never names this class or anything else in this jar: without the jar on the class path, or with
 * libozec_jni unusable, or with neither opt-in threshold set ({@code ozone.checksum.hip.min.bytes} for the streaming
 * CRC, {@code ozone.checksum.hip.batch.min.bytes} for the batch), {@link #isAvailable} is false or the provider is never
 * found, and Checksum / ChecksumByteBufferFactory run the reference's code unchanged.
 */
public final class HipChecksumAccelerator implements ChecksumAccelerator {

  /** ServiceLoader's no-argument constructor. */
  public HipChecksumAccelerator() {
  }

  @Override
  public boolean isAvailable() {
    return (HipChecksumByteBuffer.MIN_GPU_BYTES != Integer.MAX_VALUE || HipChecksum.MIN_GPU_BYTES != Long.MAX_VALUE)
        && OzecNative.isAvailable();
  }

  @Override
  public ChecksumByteBuffer wrap(boolean crc32c, ChecksumByteBuffer host) {
    if (!HipChecksumByteBuffer.enabled()) {
      return host;
    }
    return new HipChecksumByteBuffer(crc32c ? OzecNative.CHECKSUM_CRC32C : OzecNative.CHECKSUM_CRC32, host);
  }

  @Override
  public ChecksumData computeChecksum(ChecksumType type, ChunkBuffer data, int bytesPerChecksum) {
    return HipChecksum.useGpu(type, data) ? HipChecksum.computeChecksum(type, data, bytesPerChecksum) : null;
  }
}
