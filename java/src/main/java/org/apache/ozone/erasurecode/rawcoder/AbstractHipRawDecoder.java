package org.apache.ozone.erasurecode.rawcoder;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.util.concurrent.locks.ReentrantReadWriteLock;

import org.apache.hadoop.hdds.client.ECReplicationConfig;

/**
 * Base of the MI355X (HIP) raw decoders, in the shape of AbstractNativeRawDecoder
 * (EC/rawcoder/AbstractNativeRawDecoder.java:35-102).  decode() stays synchronized in the base class
 * (RawErasureDecoder.java:82); the first-k-valid input selection and the decode-matrix cache keyed on
 * (erasedIndexes, validIndexes) live in libozec and follow RSRawDecoder.prepareDecoding (RSRawDecoder.java:103-115).
 */
abstract class AbstractHipRawDecoder extends RawErasureDecoder {
  private final ReentrantReadWriteLock lock = new ReentrantReadWriteLock();
  private long handle;

  AbstractHipRawDecoder(ECReplicationConfig config, int codec) {
    super(config);
    OzecNative.checkAvailable();
    handle = OzecNative.coderCreate(true, codec, getNumDataUnits(), getNumParityUnits());
  }

  private long handleOrThrow() throws IOException {
    if (handle == 0) {
      throw new IOException(getClass().getSimpleName() + " closed");
    }
    return handle;
  }

  @Override
  protected void doDecode(ByteBufferDecodingState state) throws IOException {
    lock.readLock().lock();
    try {
      int[] inputOffsets = new int[state.inputs.length];
      int[] outputOffsets = new int[state.outputs.length];
      for (int i = 0; i < state.inputs.length; ++i) {
        if (state.inputs[i] != null) {
          inputOffsets[i] = state.inputs[i].position();
        }
      }
      for (int i = 0; i < state.outputs.length; ++i) {
        outputOffsets[i] = state.outputs[i].position();
      }
      OzecNative.decodeDirect(handleOrThrow(), state.inputs, inputOffsets, state.decodeLength, state.erasedIndexes,
          state.outputs, outputOffsets);
    } finally {
      lock.readLock().unlock();
    }
  }

  @Override
  protected void doDecode(ByteArrayDecodingState state) throws IOException {
    lock.readLock().lock();
    try {
      OzecNative.decodeArrays(handleOrThrow(), state.inputs, state.inputOffsets, state.decodeLength,
          state.erasedIndexes, state.outputs, state.outputOffsets);
    } finally {
      lock.readLock().unlock();
    }
  }

  /**
   * Reconstruct many stripes in one call (ECReconstructionCoordinator's read buffers): verify the stored checksums of
   * the units read, rebuild the erased units and checksum them, pipelined over PCIe (ozec_reconstruct_crc_host_batch).
   * All buffers are direct (OzecNative.allocatePinned for DMA in place) and read from their start:
   * stripes [numStripes][k+p][cellLength] at stripeStride / unitStride; out [numStripes][erased][cellLength];
   * outChecksums [numStripes][erased][windows] and expectedChecksums [numStripes][k+p][windows] as 4-byte big-endian
   * values (the ByteStrings of ChecksumData); mismatch [numStripes] native-order ints, -1 or the first failing
   * unit * windows + window.  expectedChecksums and mismatch may be null (no verification).
   */
  public void reconstructBatch(ByteBuffer stripes, long stripeStride, long unitStride, int[] presentUnits,
      int[] erasedIndexes, ByteBuffer out, int numStripes, int cellLength, int checksumType, int bytesPerChecksum,
      ByteBuffer expectedChecksums, ByteBuffer outChecksums, ByteBuffer mismatch) throws IOException {
    lock.readLock().lock();
    try {
      OzecNative.reconstructHostBatch(handleOrThrow(), stripes, stripeStride, unitStride, presentUnits, erasedIndexes,
          out, numStripes, cellLength, checksumType, bytesPerChecksum, expectedChecksums, outChecksums, mismatch);
    } finally {
      lock.readLock().unlock();
    }
  }

  @Override
  public boolean preferDirectBuffer() {
    return true;
  }

  @Override
  public void release() {
    lock.writeLock().lock();
    try {
      if (handle != 0) {
        OzecNative.coderRelease(handle);
        handle = 0;
      }
    } finally {
      lock.writeLock().unlock();
    }
  }
}
