package org.apache.ozone.erasurecode.rawcoder;

import java.io.IOException;
import java.util.concurrent.locks.ReentrantReadWriteLock;

import org.apache.hadoop.hdds.client.ECReplicationConfig;

/**
 * Base of the MI355X (HIP) raw encoders, in the shape of AbstractNativeRawEncoder
 * (EC/rawcoder/AbstractNativeRawEncoder.java:35-99): the state checks stay in the inherited encode(), the coding
 * runs in libozec.  Unlike the ISA-L bridge, heap arrays are not copied into direct buffers first
 * (AbstractNativeRawEncoder.java:75-86): they are pinned for the synchronous call.  The native handle is a cheap
 * host object (coding matrix); device state is per process and per GPU inside libozec.
 */
abstract class AbstractHipRawEncoder extends RawErasureEncoder {
  // guards the handle against release() while a call is in flight (AbstractNativeRawEncoder.java:41-43)
  private final ReentrantReadWriteLock lock = new ReentrantReadWriteLock();
  private long handle;

  AbstractHipRawEncoder(ECReplicationConfig config, int codec) {
    super(config);
    OzecNative.checkAvailable();
    handle = OzecNative.coderCreate(false, codec, getNumDataUnits(), getNumParityUnits());
  }

  private long handleOrThrow() throws IOException {
    if (handle == 0) {
      throw new IOException(getClass().getSimpleName() + " closed");
    }
    return handle;
  }

  @Override
  protected void doEncode(ByteBufferEncodingState state) throws IOException {
    lock.readLock().lock();
    try {
      int[] inputOffsets = new int[state.inputs.length];
      int[] outputOffsets = new int[state.outputs.length];
      for (int i = 0; i < state.inputs.length; ++i) {
        inputOffsets[i] = state.inputs[i].position();
      }
      for (int i = 0; i < state.outputs.length; ++i) {
        outputOffsets[i] = state.outputs[i].position();
      }
      OzecNative.encodeDirect(handleOrThrow(), state.inputs, inputOffsets, state.encodeLength, state.outputs,
          outputOffsets);
    } finally {
      lock.readLock().unlock();
    }
  }

  @Override
  protected void doEncode(ByteArrayEncodingState state) throws IOException {
    // every production caller passes heap buffers (ECKeyOutputStream.java:701): pinned in place, no Java copy
    lock.readLock().lock();
    try {
      OzecNative.encodeArrays(handleOrThrow(), state.inputs, state.inputOffsets, state.encodeLength, state.outputs,
          state.outputOffsets);
    } finally {
      lock.readLock().unlock();
    }
  }

  /** The GPU coder reads heap arrays in place too; direct buffers skip the pinning. */
  @Override
  public boolean preferDirectBuffer() {
    return true;
  }

  /** Idempotent; later encode calls throw IOException("... closed") (TestRawCoderBase.java:118-150). */
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

  long nativeHandle() {
    return handle;
  }
}
