package org.apache.ozone.erasurecode.rawcoder;

import java.io.IOException;
import java.nio.ByteBuffer;
import java.util.ArrayDeque;

/**
 * Writer-side stripe batching (SURVEY §8(f) row 3) over ozec_stripe_queue_*: ECKeyOutputStream encodes one stripe
 * per RawErasureEncoder.encode call (hadoop-ozone/client/.../ECKeyOutputStream.java:304, stripe queue :501-543);
 * with this queue the writer hands a full stripe over and keeps filling the next one, and the GPU encodes
 * stripesPerBatch stripes (+ their window CRCs) per fused launch with the copies of three batches overlapped.
 * Cells and CRC buffers must be direct buffers; the ones from {@link OzecNative#allocatePinned} are DMA'd without
 * staging.  Buffers stay referenced (and must stay unmodified) until waitFor returns for their ticket.  The native
 * queue co-owns the encoder's native handle (ozec_coder_retain), so releasing the encoder first only makes later
 * submits fail with "closed"; the handle's memory goes with close().
 */
public final class HipStripeQueue implements AutoCloseable {
  private final int numData;
  private final int numParity;
  private final ArrayDeque<Object[]> held = new ArrayDeque<>();
  private long queue;

  /**
   * @param checksumType OzecNative.CHECKSUM_NONE / CHECKSUM_CRC32 / CHECKSUM_CRC32C; CRCs are written big-endian,
   *                     i.e. the bytes Checksum.int2ByteString stores (Checksum.java:59-70)
   */
  public HipStripeQueue(RawErasureEncoder encoder, int cellSize, int stripesPerBatch, int checksumType,
      int bytesPerChecksum) {
    if (!(encoder instanceof AbstractHipRawEncoder)) {
      throw new IllegalArgumentException("the stripe queue needs a GPU encoder (rs_hip / xor_hip)");
    }
    numData = encoder.getNumDataUnits();
    numParity = encoder.getNumParityUnits();
    queue = OzecNative.queueCreate(((AbstractHipRawEncoder) encoder).nativeHandle(), cellSize, stripesPerBatch,
        checksumType, bytesPerChecksum);
  }

  /** Queue one stripe; returns its ticket.  crcs (direct, may be null) receives (k + coded parity) x windows CRCs. */
  public synchronized long submit(ByteBuffer[] dataCells, ByteBuffer[] parityCells, int length, ByteBuffer crcs)
      throws IOException {
    if (queue == 0) {
      throw new IOException("HipStripeQueue closed");
    }
    if (dataCells.length != numData || parityCells.length != numParity) {
      throw new IllegalArgumentException("Invalid inputs/outputs length");
    }
    int[] dataOffsets = new int[numData];
    int[] parityOffsets = new int[numParity];
    for (int i = 0; i < numData; i++) {
      dataOffsets[i] = dataCells[i].position();
    }
    for (int i = 0; i < numParity; i++) {
      parityOffsets[i] = parityCells[i].position();
    }
    long ticket = OzecNative.queueSubmit(queue, dataCells, dataOffsets, parityCells, parityOffsets, length, crcs,
        crcs == null ? 0 : crcs.position());
    held.addLast(new Object[] {ticket, dataCells, parityCells, crcs});
    return ticket;
  }

  /** Block until parity and CRCs of every stripe up to and including ticket are in their buffers. */
  public synchronized void waitFor(long ticket) throws IOException {
    if (queue == 0) {
      throw new IOException("HipStripeQueue closed");
    }
    OzecNative.queueWait(queue, ticket);
    while (!held.isEmpty() && (Long) held.peekFirst()[0] <= ticket) {
      held.removeFirst();
    }
  }

  /** Completes every stripe not yet waited for, then frees the queue. */
  @Override
  public synchronized void close() {
    if (queue != 0) {
      long q = queue;
      queue = 0;
      OzecNative.queueFree(q);
      held.clear();
    }
  }
}
