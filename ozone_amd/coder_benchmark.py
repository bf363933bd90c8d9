"""RawErasureCoderBenchmark (ECT/rawcoder/RawErasureCoderBenchmark.java:45-411) for the GPU coder.

Same definitions as the reference harness:
  * rs-6-3; one shared coder for all threads (`:201-206`); decode erases all parity {6, 7, 8} (`:315`);
  * a random test buffer of ~126 MB rounded to a multiple of k x chunk (`:320-335`), re-sliced by every
    thread into k chunk-size inputs per call (`:380-392`);
  * throughput = data bytes of all threads / wall time (`:219-224`), MB = 2^20 B.
Coders: 0 = DummyRawErasureCoderFactory (framework floor, no GPU), 1 = HipRSRawErasureCoderFactory (the
host-buffer ABI, `ozec_encode` / `ozec_decode`, i.e. what the JNI drop-in calls per stripe).

  python -m ozone_amd.coder_benchmark <encode|decode> <coderIndex> [numThreads] [dataSize-in-MB] [chunkSize-in-KB]
"""
import enum
import math
import sys
import threading
import time

import numpy as np

from .bytebuffer import ByteBuffer
from .rawcoder import DummyRawErasureCoderFactory, ECReplicationConfig, HipRSRawErasureCoderFactory

TARGET_BUFFER_SIZE_MB = 126
OPTIONS = ECReplicationConfig(6, 3)
NUM_DATA_UNITS = OPTIONS.get_data()
NUM_PARITY_UNITS = OPTIONS.get_parity()
NUM_ALL_UNITS = NUM_DATA_UNITS + NUM_PARITY_UNITS
ERASED_INDEXES = [6, 7, 8]
MAX_CHUNK_SIZE = TARGET_BUFFER_SIZE_MB // NUM_DATA_UNITS * 1024  # KB


class CODER(enum.Enum):
    DUMMY_CODER = "Dummy coder"
    RS_CODER = "Reed-Solomon HIP coder"

    def __str__(self):
        return self.value


CODER_MAKERS = [DummyRawErasureCoderFactory(), HipRSRawErasureCoderFactory()]


class BenchData:
    """BenchData (`:299-353`): one instance per thread, outputs allocated once."""
    chunk_size = 0
    total_data_size_kb = 0
    buffer_size_kb = 0

    @classmethod
    def configure(cls, data_size_mb, chunk_size_kb):
        cls.chunk_size = chunk_size_kb * 1024
        # buffer size must be a multiple of numDataUnits * chunkSize (Java Math.round = floor(x + 0.5))
        rnd = int(math.floor(TARGET_BUFFER_SIZE_MB * 1024.0 / NUM_DATA_UNITS / chunk_size_kb + 0.5))
        if rnd <= 0:
            raise ValueError("chunk size too large")
        cls.buffer_size_kb = NUM_DATA_UNITS * chunk_size_kb * rnd
        rnd = int(math.floor(data_size_mb * 1024.0 / cls.buffer_size_kb + 0.5)) or 1
        cls.total_data_size_kb = rnd * cls.buffer_size_kb

    def __init__(self, direct):
        alloc = ByteBuffer.allocate_direct if direct else ByteBuffer.allocate
        self.inputs = [None] * NUM_DATA_UNITS
        self.outputs = [alloc(self.chunk_size) for _ in range(NUM_PARITY_UNITS)]
        self.decode_inputs = [None] * NUM_ALL_UNITS

    def prepare_dec_input(self):
        self.decode_inputs[:NUM_DATA_UNITS] = self.inputs

    def encode(self, encoder):
        encoder.encode(self.inputs, self.outputs)

    def decode(self, decoder):
        decoder.decode(self.decode_inputs, ERASED_INDEXES, self.outputs)


def _gen_test_data(direct, size_kb, seed=0):
    n = size_kb * 1024
    data = (ByteBuffer.allocate_direct if direct else ByteBuffer.allocate)(n)
    data.put(np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8))
    data.flip()
    return data


def _init_buffers(num, direct):
    return [(ByteBuffer.allocate_direct if direct else ByteBuffer.allocate)(1) for _ in range(num)]


def _bench_thread(is_encode, coder, test_data, out):
    bd = BenchData(coder.prefer_direct_buffer())
    rounds = BenchData.total_data_size_kb // BenchData.buffer_size_kb
    t0 = time.perf_counter()
    for _ in range(rounds):
        while test_data.remaining() > 0:
            for o in bd.outputs:
                o.clear()
            for j in range(NUM_DATA_UNITS):
                b = test_data.duplicate()
                b.limit(test_data.position() + BenchData.chunk_size)
                bd.inputs[j] = b.slice()
                test_data.position(test_data.position() + BenchData.chunk_size)
            if is_encode:
                bd.encode(coder)
            else:
                bd.prepare_dec_input()
                bd.decode(coder)
        test_data.clear()
    out.append(time.perf_counter() - t0)


def perform_bench(op_type, coder, num_threads, data_size_mb, chunk_size_kb, log=print):
    """performBench (`:182-236`). Returns the total throughput in MB/s."""
    if op_type not in ("encode", "decode"):
        raise ValueError("Invalid type: should be either 'encode' or 'decode'")
    if chunk_size_kb <= 0 or chunk_size_kb > MAX_CHUNK_SIZE:
        raise ValueError(f"Chunk size should be positive and no larger than {MAX_CHUNK_SIZE}")
    BenchData.configure(data_size_mb, chunk_size_kb)
    log(f"Using {BenchData.buffer_size_kb // 1024}MB buffer.")
    factory = CODER_MAKERS[list(CODER).index(coder)]
    is_encode = op_type == "encode"
    if is_encode:  # getRawEncoder (`:238-246`): one warm-up call on 1-byte buffers
        c = factory.create_encoder(OPTIONS)
        d = c.prefer_direct_buffer()
        c.encode(_init_buffers(NUM_DATA_UNITS, d), _init_buffers(NUM_PARITY_UNITS, d))
    else:  # getRawDecoder (`:248-260`)
        c = factory.create_decoder(OPTIONS)
        d = c.prefer_direct_buffer()
        ins = _init_buffers(NUM_ALL_UNITS, d)
        for e in ERASED_INDEXES:
            ins[e] = None
        c.decode(ins, ERASED_INDEXES, _init_buffers(len(ERASED_INDEXES), d))
    test_data = _gen_test_data(d, BenchData.buffer_size_kb)
    durations = []
    threads = [threading.Thread(target=_bench_thread, args=(is_encode, c, test_data.duplicate(), durations))
               for _ in range(num_threads)]
    t0 = time.perf_counter()
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    duration = time.perf_counter() - t0
    c.release()
    if len(durations) != num_threads:
        raise RuntimeError("Error waiting for thread to finish.")
    total_mb = BenchData.total_data_size_kb * num_threads / 1024.0
    mbps = total_mb / duration
    log(f"{coder} {op_type} {total_mb:.2f}MB data, with chunk size {BenchData.chunk_size // 1024}KB")
    log(f"Total time: {duration:.2f} s.")
    log(f"Total throughput: {mbps:.2f} MB/s")
    ds = sorted(durations)
    pct = ds[int(math.ceil(len(ds) * 0.9)) - 1]
    log("Threads statistics: ")
    log(f"{len(ds)} threads in total.")
    log(f"Min: {ds[0]:.2f} s, Max: {ds[-1]:.2f} s, Avg: {sum(ds) / len(ds):.2f} s, 90th Percentile: {pct:.2f} s.")
    return mbps


def main(argv):
    usage = ("Usage: python -m ozone_amd.coder_benchmark <encode/decode> <coderIndex> "
             "[numThreads] [dataSize-in-MB] [chunkSize-in-KB]\nAvailable coders with coderIndex:\n" +
             "".join(f"{i}:{c}\n" for i, c in enumerate(CODER)))
    if len(argv) < 2:
        print(usage)
        return 1
    op, idx = argv[0], int(argv[1])
    if op not in ("encode", "decode") or not 0 <= idx < len(CODER):
        print(usage)
        return 1
    threads = int(argv[2]) if len(argv) > 2 else 1
    size_mb = int(argv[3]) if len(argv) > 3 else 10240
    chunk_kb = int(argv[4]) if len(argv) > 4 else 1024
    perform_bench(op, list(CODER)[idx], threads, size_mb, chunk_kb)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
