"""TestRawErasureCoderBenchmark.java and TestDummyRawCoder.java, mirrored.

The dummy coder runs host-only (no GPU), so its tests are CPU tests; the RS benchmark drives the GPU host-buffer
ABI and is marked gpu."""
import numpy as np
import pytest

from ozone_amd import coder_benchmark as cb
from ozone_amd.bytebuffer import ByteBuffer, ECChunk
from ozone_amd.rawcoder import (DummyRawErasureCoderFactory, ECReplicationConfig, HadoopIllegalArgumentException,
                                IllegalArgumentException)


def test_benchmark_dummy_coder():
    """TestRawErasureCoderBenchmark.testDummyCoder (:26-33)."""
    lines = []
    assert cb.perform_bench("encode", cb.CODER.DUMMY_CODER, 2, 100, 1024, log=lines.append) > 0
    assert lines[0] == "Using 126MB buffer." and lines[1].startswith("Dummy coder encode 252.00MB data")
    assert cb.perform_bench("decode", cb.CODER.DUMMY_CODER, 5, 150, 100, log=lines.append) > 0


def test_benchmark_definitions_match_reference():
    """BenchData.configure (RawErasureCoderBenchmark.java:320-335): buffer = k * chunk * round(126 MiB / k / chunk),
    total = buffer * max(1, round(dataSize / buffer))."""
    cb.BenchData.configure(10240, 1024)
    assert cb.BenchData.buffer_size_kb == 6 * 1024 * 21 and cb.BenchData.total_data_size_kb == 129024 * 81
    cb.BenchData.configure(135, 20)
    assert cb.BenchData.buffer_size_kb == 6 * 20 * 1075 and cb.BenchData.total_data_size_kb == 129000
    with pytest.raises(ValueError):
        cb.perform_bench("encode", cb.CODER.DUMMY_CODER, 1, 10, cb.MAX_CHUNK_SIZE + 1)
    assert cb.main([]) == 1 and cb.main(["bogus", "0"]) == 1


@pytest.mark.parametrize("erased", [[0, 2], [0, 6]])
def test_dummy_coder_leaves_outputs_untouched(erased):
    """TestDummyRawCoder (:27-78): encode/decode succeed and outputs stay all-zero."""
    f = DummyRawErasureCoderFactory()
    assert (f.get_coder_name(), f.get_codec_name()) == ("dummy_dummy", "dummy")
    conf = ECReplicationConfig(6, 3)
    enc, dec = f.create_encoder(conf), f.create_decoder(conf)
    n = 1024
    data = [ByteBuffer.wrap(np.random.default_rng(i).integers(0, 256, n, dtype=np.uint8)) for i in range(6)]
    par = [ByteBuffer.allocate(n) for _ in range(3)]
    enc.encode([ECChunk(b) for b in data], [ECChunk(b) for b in par])
    assert all(not b.array().any() for b in par)
    assert all(b.position() == n for b in data)  # inputs consumed exactly as by a real coder
    ins = [ByteBuffer.allocate(n) for _ in range(9)]
    for e in erased:
        ins[e] = None
    outs = [ByteBuffer.allocate(n) for _ in erased]
    dec.decode(ins, erased, outs)
    assert all(not b.array().any() for b in outs)
    # the inherited validation still applies
    with pytest.raises(HadoopIllegalArgumentException):
        enc.encode(data[:5], par)
    with pytest.raises(IllegalArgumentException):
        dec.decode(ins, [0, 1, 2, 3], [ByteBuffer.allocate(n)] * 4)
    enc.release()
    enc.release()  # no-op, and the coder stays usable (RawErasureEncoder.release: "Nothing to do here.")
    enc.encode([ByteBuffer.allocate(8) for _ in range(6)], [ByteBuffer.allocate(8) for _ in range(3)])


@pytest.mark.gpu
def test_benchmark_rs_coder():
    """TestRawErasureCoderBenchmark.testRSCoder (:35-42) on the GPU coder."""
    assert cb.perform_bench("encode", cb.CODER.RS_CODER, 3, 200, 200, log=lambda *_: None) > 0
    assert cb.perform_bench("decode", cb.CODER.RS_CODER, 4, 135, 20, log=lambda *_: None) > 0
