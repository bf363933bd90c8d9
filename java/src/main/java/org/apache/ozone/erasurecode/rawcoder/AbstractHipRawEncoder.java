package org.apache.ozone.erasurecode.rawcoder;

import java.io.IOException;
import java.util.concurrent.locks.ReentrantReadWriteLock;

import org.apache.hadoop.hdds.client.ECReplicationConfig;

/**
 * Base of the MI355X (HIP) raw encoders, in the shape of AbstractNativeRawEncoder
 * (EC/rawcoder/AbstractNativeRawEncoder.java:35-99): the state checks stay in the inherited encode(), the coding
 * runs in libozec.  As the ISA-L bridge copies heap arrays into direct buffers (AbstractNativeRawEncoder.java:75-86),
 * the JNI glue copies the arrays' regions into pinned memory and the outputs back (each array held with
 * GetPrimitiveArrayCritical for that copy only, the regions moved by libozec's parallel copy pool, ozec_host_copy): a
 * call alone fills libozec's own staging through the ozec_encode_cb callbacks, chunk by chunk, and the kernel codes it
 * in place over PCIe; a call beside others copies through a pooled pinned arena.  No array stays pinned while the GPU
 * works.  The native handle is a cheap host object (coding matrix); device state is per process and per GPU inside
 * libozec.
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
    // every production caller passes heap buffers (ECKeyOutputStream.java:701): the glue copies their regions into
    // pinned memory and back (jni/ozec_jni.c heap_code: libozec's staging when the call is alone, a pooled arena beside
    // other calls), in parallel, with no array pinned across the device work
    lock.readLock().lock();
    try {
      OzecNative.encodeArrays(handleOrThrow(), state.inputs, state.inputOffsets, state.encodeLength, state.outputs,
          state.outputOffsets);
    } finally {
      lock.readLock().unlock();
    }
  }

  /** Direct buffers are coded from where they lie (pinned ones, OzecNative.allocatePinned, with no staging copy);
   *  heap arrays take the glue's copy. */
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
