"""ozone_amd -- MI355X (gfx950) erasure-coding + chunk-checksum engine for Apache Ozone's hot path.

The compute lives in libozec.so (HIP kernels + C ABI, include/ozec.h).  This package is the host-side
mirror of the reference's plugin interfaces:
  ozone_amd.rawcoder  -- RawErasureCoderFactory / RawErasureEncoder / RawErasureDecoder / CodecRegistry
  ozone_amd.checksum  -- Checksum / ChecksumData / ChecksumByteBuffer (CRC32, CRC32C)
"""
from . import _lib  # noqa: F401
from .bytebuffer import ByteBuffer, ECChunk  # noqa: F401
from .checksum import Checksum, ChecksumByteBuffer, ChecksumData, ChecksumType, OzoneChecksumException  # noqa: F401
from .rawcoder import (CodecRegistry, CodecUtil, DummyRawDecoder, DummyRawEncoder,  # noqa: F401
                       DummyRawErasureCoderFactory, ECReplicationConfig, HadoopIllegalArgumentException,
                       HipRSRawErasureCoderFactory, HipXORRawErasureCoderFactory, IllegalArgumentException,
                       IOException, RawErasureDecoder, RawErasureEncoder)

__version__ = "0.1.0"
