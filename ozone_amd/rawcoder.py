"""MI355X raw erasure coders behind the reference's plugin interface.

Mirrors hadoop-hdds/erasurecode (EC/ = .../org/apache/ozone/erasurecode/):
  RawErasureCoderFactory      EC/rawcoder/RawErasureCoderFactory.java:29-56
  RawErasureEncoder.encode    EC/rawcoder/RawErasureEncoder.java:66-145   (+ EncodingState checks)
  RawErasureDecoder.decode    EC/rawcoder/RawErasureDecoder.java:82-169   (+ DecodingState checks)
  CodecRegistry / CodecUtil   EC/CodecRegistry.java:43-170, EC/rawcoder/util/CodecUtil.java:55-110
  ECReplicationConfig         hadoop-hdds/common/.../hdds/client/ECReplicationConfig.java:42-130
The arithmetic runs on the GPU through libozec.so (include/ozec.h); this module only validates arguments
exactly like the reference base classes, resolves buffer addresses and maps status codes to the
reference's exceptions.  Device-resident batch entry points (encode_batch / decode_batch /
encode_crc_batch) take torch tensors or raw device addresses.
"""
import ctypes
import threading

import numpy as np

from . import _lib as L
from .bytebuffer import ByteBuffer, ECChunk

# ---------------------------------------------------------------- exceptions -------------------------


class HadoopIllegalArgumentException(ValueError):
    pass


class IllegalArgumentException(ValueError):
    pass


class IOException(OSError):
    pass


class NotInvertibleException(RuntimeError):
    """RuntimeException("Not invertible") from GF256.gfInvertMatrix (GF256.java:214-217)."""


def _raise_for(rc, default=IllegalArgumentException):
    msg = L.last_error()
    if rc == L.OZEC_ECLOSED:
        raise IOException(msg)
    if rc == L.OZEC_ENOTINVERTIBLE:
        raise NotInvertibleException(msg)
    if rc in (L.OZEC_EDEVICE, L.OZEC_ENOMEM):
        raise RuntimeError(msg)
    if rc == L.OZEC_EUNSUPPORTED:
        raise NotImplementedError(msg)
    raise default(msg)


# ---------------------------------------------------------------- config --------------------------------

class ECReplicationConfig:
    RS = "rs"
    XOR = "xor"

    def __init__(self, data, parity=None, codec=RS, ec_chunk_size=1024 * 1024):
        if isinstance(data, str):  # ECReplicationConfig(String), ECReplicationConfig.java:96-130
            c, k, p, cs = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
            rc = L.lib().ozec_parse_replication(data.encode(), ctypes.byref(c), ctypes.byref(k), ctypes.byref(p),
                                                ctypes.byref(cs))
            if rc != L.OZEC_OK:
                raise IllegalArgumentException(L.last_error())
            self.codec = self.RS if c.value == L.OZEC_CODEC_RS else self.XOR
            self.data, self.parity, self.ec_chunk_size = k.value, p.value, cs.value
        else:
            self.data, self.parity, self.codec, self.ec_chunk_size = data, parity, codec.lower(), ec_chunk_size

    def get_data(self):
        return self.data

    def get_parity(self):
        return self.parity

    def get_codec(self):
        return self.codec

    def get_ec_chunk_size(self):
        return self.ec_chunk_size

    def get_required_nodes(self):
        return self.data + self.parity

    def __repr__(self):
        return f"{self.codec.upper()}-{self.data}-{self.parity}-{self.ec_chunk_size // 1024}k"


def _codec_id(name):
    return {"rs": L.OZEC_CODEC_RS, "xor": L.OZEC_CODEC_XOR}[name]


# ---------------------------------------------------------------- helpers ------------------------------

def _in_array(x):
    """A byte[] input: any uint8 buffer; strided views are copied into one contiguous run (the library reads
    `len` bytes from the address).  Other dtypes are rejected rather than reinterpreted."""
    if x is None:
        return None
    a = x if isinstance(x, np.ndarray) else np.frombuffer(x, np.uint8)
    if a.dtype != np.uint8 or a.ndim != 1:
        raise IllegalArgumentException(f"Invalid buffer: a 1-D uint8 array is required, got {a.dtype} {a.shape}")
    return np.ascontiguousarray(a)


def _out_array(x):
    """A byte[] output is written in place, so it must be one writeable contiguous run of uint8 (a strided view
    would be written past its elements; `bytes` is immutable)."""
    if x is None:
        return None
    a = x if isinstance(x, np.ndarray) else np.frombuffer(x, np.uint8)
    if a.dtype != np.uint8 or a.ndim != 1 or not a.flags.c_contiguous or not a.flags.writeable:
        raise IllegalArgumentException("Invalid output buffer: a writeable 1-D C-contiguous uint8 array is required")
    return a


def _as_buffers(items, outputs=False):
    """Accept ByteBuffer, ECChunk, numpy uint8 arrays, bytearray or None for each slot."""
    out = []
    for x in items:
        if x is None or isinstance(x, ByteBuffer):
            out.append(x)
        elif isinstance(x, ECChunk):
            out.append(ECChunk.to_buffers([x])[0])
        else:
            out.append(ByteBuffer.wrap(_out_array(x) if outputs else _in_array(x)))
    return out


def _first_valid(buffers):
    for b in buffers:
        if b is not None:
            return b
    raise IllegalArgumentException("Invalid inputs are found, all being null")


def _dev_ptr(t):
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def _stream_ptr(stream):
    if stream is None:
        try:
            import torch
            if torch.cuda.is_available():
                return torch.cuda.current_stream().cuda_stream
        except Exception:  # pragma: no cover
            pass
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


class _Coder:
    def __init__(self, config, decoder):
        self._config = config
        self._handle = ctypes.c_void_p()
        create = L.lib().ozec_decoder_create if decoder else L.lib().ozec_encoder_create
        rc = create(_codec_id(config.get_codec()), config.get_data(), config.get_parity(), ctypes.byref(self._handle))
        if rc != L.OZEC_OK:
            _raise_for(rc, HadoopIllegalArgumentException)

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and h.value:
            try:
                L.lib().ozec_coder_free(h)
            except Exception:  # pragma: no cover - interpreter shutdown
                pass
            self._handle = None

    def get_num_data_units(self):
        return self._config.get_data()

    def get_num_parity_units(self):
        return self._config.get_parity()

    def get_num_all_units(self):
        return self._config.get_data() + self._config.get_parity()

    def prefer_direct_buffer(self):
        return True  # the GPU path stages from any host address; direct buffers skip the heap copy in JNI

    def allow_change_inputs(self):
        return False

    def allow_verbose_dump(self):
        return False

    def release(self):
        """Idempotent; later encode/decode raise IOException("... closed") (TestRawCoderBase.java:118-150)."""
        L.lib().ozec_coder_release(self._handle)

    @property
    def device(self):
        """The GPU this coder's host-buffer calls and stripe queues run on (chosen at creation: set_devices)."""
        return int(L.lib().ozec_coder_device(self._handle))


# ---------------------------------------------------------------- encoder --------------------------------

class RawErasureEncoder(_Coder):
    """RawErasureEncoder (EC/rawcoder/RawErasureEncoder.java:42-193) running on the GPU."""

    def __init__(self, config):
        super().__init__(config, decoder=False)

    def encode(self, inputs, outputs):
        """encode(ByteBuffer[]/ECChunk[]) or encode(byte[][]) -- numpy arrays / bytearrays are the byte[] form."""
        if not any(isinstance(x, (ByteBuffer, ECChunk)) for x in list(inputs) + list(outputs)):
            return self._encode_arrays(inputs, outputs)
        ins = _as_buffers(inputs)
        outs = _as_buffers(outputs, outputs=True)
        # ByteBufferEncodingState (ByteBufferEncodingState.java:36-48) + EncodingState.checkParameters
        valid = _first_valid(ins)
        n = valid.remaining()
        direct = valid.is_direct()
        self._check_parameters(ins, outs)
        for group in (ins, outs):
            for b in group:
                if b is None:
                    raise HadoopIllegalArgumentException("Invalid buffer found, not allowing null")
                if b.remaining() != n:
                    raise HadoopIllegalArgumentException(
                        f"Invalid buffer remaining {b.remaining()}, not of length {n}")
                if b.is_direct() != direct:
                    raise HadoopIllegalArgumentException(f"Invalid buffer, isDirect should be {direct}")
        if n == 0:
            return
        self._run([b.address() for b in ins], [b.address() for b in outs], n)
        for b in ins:  # dataLen bytes consumed (RawErasureEncoder.java:91-96)
            b.position(b.position() + n)

    def _encode_arrays(self, inputs, outputs):
        """encode(byte[][] inputs, byte[][] outputs) (RawErasureEncoder.java:114-125)."""
        ins = [_in_array(x) for x in inputs]
        outs = list(outputs)
        n = _first_valid(ins).size
        self._check_parameters(ins, outs)
        for group in (ins, outs):
            for b in group:
                if b is None:
                    raise HadoopIllegalArgumentException("Invalid buffer found, not allowing null")
                if len(b) != n:
                    raise HadoopIllegalArgumentException(f"Invalid buffer not of length {n}")
        if n == 0:
            return
        outs = [_out_array(o) for o in outs]
        self._run([x.ctypes.data for x in ins], [o.ctypes.data for o in outs], n)

    def _check_parameters(self, ins, outs):
        if len(ins) != self.get_num_data_units():
            raise HadoopIllegalArgumentException(
                f"Invalid inputs length {len(ins)} !={self.get_num_data_units()}")
        if len(outs) != self.get_num_parity_units():
            raise HadoopIllegalArgumentException(
                f"Invalid outputs length {len(outs)} !={self.get_num_parity_units()}")

    def _run(self, in_addrs, out_addrs, n):
        rc = L.lib().ozec_encode(self._handle, L.ptr_array(in_addrs), L.ptr_array(out_addrs), n)
        if rc != L.OZEC_OK:
            _raise_for(rc, HadoopIllegalArgumentException)

    # ---- device-resident forms ---------------------------------------------------------------------
    def encode_device(self, d_inputs, d_outputs, length, stream=None):
        rc = L.lib().ozec_encode_device(self._handle, L.ptr_array([_dev_ptr(x) for x in d_inputs]),
                                        L.ptr_array([_dev_ptr(x) for x in d_outputs]), length, _stream_ptr(stream))
        if rc != L.OZEC_OK:
            _raise_for(rc)

    def encode_batch(self, d_in, in_stripe_stride, in_unit_stride, d_out, out_stripe_stride, out_unit_stride,
                     num_stripes, length, stream=None):
        rc = L.lib().ozec_encode_batch(self._handle, _dev_ptr(d_in), in_stripe_stride, in_unit_stride,
                                       _dev_ptr(d_out), out_stripe_stride, out_unit_stride, num_stripes, length,
                                       _stream_ptr(stream))
        if rc != L.OZEC_OK:
            _raise_for(rc)

    def encode_stripes(self, data, parity=None, stream=None):
        """data: uint8 CUDA tensor [S, k, L] -> parity [S, p, L] (allocated when not given)."""
        import torch
        S, k, n = data.shape
        assert k == self.get_num_data_units() and data.is_contiguous()
        if parity is None:
            parity = torch.empty((S, self.get_num_parity_units(), n), dtype=torch.uint8, device=data.device)
        self.encode_batch(data, k * n, n, parity, parity.shape[1] * n, n, S, n, stream)
        return parity

    def encode_crc_batch(self, d_in, in_stripe_stride, in_unit_stride, d_out, out_stripe_stride, out_unit_stride,
                         num_stripes, length, checksum_type, bytes_per_checksum, d_crcs, big_endian=False,
                         stream=None):
        rc = L.lib().ozec_encode_crc_batch(self._handle, _dev_ptr(d_in), in_stripe_stride, in_unit_stride,
                                           _dev_ptr(d_out), out_stripe_stride, out_unit_stride, num_stripes, length,
                                           int(checksum_type), bytes_per_checksum, _dev_ptr(d_crcs),
                                           1 if big_endian else 0, _stream_ptr(stream))
        if rc != L.OZEC_OK:
            _raise_for(rc)


    def encode_crc_block_groups(self, d_base, group_stride, unit_stride, num_groups, stripes_per_group, length,
                                checksum_type, bytes_per_checksum, d_crcs, big_endian=False, stream=None):
        """Fused encode + CRC over block groups (one block per unit; ozec_encode_crc_block_groups): unit u of stripe
        t of group g at d_base + g*group_stride + u*unit_stride + t*length; CRCs [g][t][unit][window]."""
        rc_ = L.lib().ozec_encode_crc_block_groups(self._handle, _dev_ptr(d_base), group_stride, unit_stride, num_groups,
                                                   stripes_per_group, length, int(checksum_type), bytes_per_checksum,
                                                   _dev_ptr(d_crcs), 1 if big_endian else 0, _stream_ptr(stream))
        if rc_ != L.OZEC_OK:
            _raise_for(rc_)

    def encode_crc_host_batch(self, h_in, in_stripe_stride, in_unit_stride, h_out, out_stripe_stride,
                              out_unit_stride, num_stripes, length, checksum_type, bytes_per_checksum, h_crcs=None,
                              big_endian=False, stripes_per_chunk=0):
        """End-to-end encode (+ CRC) of stripes in host memory (ozec_encode_crc_host_batch): host
        addresses (ints) or numpy arrays; registered / pinned memory is DMA'd in place.  Synchronous."""
        def addr(x):
            return None if x is None else x if isinstance(x, int) else x.ctypes.data
        rc = L.lib().ozec_encode_crc_host_batch(self._handle, addr(h_in), in_stripe_stride, in_unit_stride, addr(h_out),
                                                out_stripe_stride, out_unit_stride, num_stripes, length,
                                                int(checksum_type), bytes_per_checksum, addr(h_crcs),
                                                1 if big_endian else 0, stripes_per_chunk)
        if rc != L.OZEC_OK:
            _raise_for(rc)


# ---------------------------------------------------------------- decoder --------------------------------

class RawErasureDecoder(_Coder):
    """RawErasureDecoder (EC/rawcoder/RawErasureDecoder.java:42-217) running on the GPU."""

    def __init__(self, config):
        super().__init__(config, decoder=True)
        self._lock = threading.Lock()  # decode() is synchronized in the reference (RawErasureDecoder.java:82)

    def decode(self, inputs, erased_indexes, outputs):
        with self._lock:
            if not any(isinstance(x, (ByteBuffer, ECChunk)) for x in list(inputs) + list(outputs)):
                return self._decode_arrays(inputs, erased_indexes, outputs)
            ins = _as_buffers(inputs)
            outs = _as_buffers(outputs, outputs=True)
            valid = _first_valid(ins)
            n = valid.remaining()
            direct = valid.is_direct()
            self._check_parameters(ins, erased_indexes, outs)
            count = 0
            for i, b in enumerate(ins):  # ByteBufferDecodingState.checkInputBuffers (:103-130)
                if b is None:
                    continue
                if b.remaining() != n:
                    raise IllegalArgumentException(f"Invalid buffer [{i}], not of length {n}")
                if b.is_direct() != direct:
                    raise IllegalArgumentException(f"Invalid buffer [{i}], isDirect should be {direct}")
                count += 1
            if count < self.get_num_data_units():
                raise IllegalArgumentException(
                    f"No enough valid inputs are provided ({count} vs. {self.get_num_data_units()}), not recoverable")
            for b in outs:  # checkOutputBuffers (:132-145)
                if b is None:
                    raise IllegalArgumentException("Invalid buffer found, not allowing null")
                if b.remaining() != n:
                    raise IllegalArgumentException(f"Invalid buffer, not of length {n}")
                if b.is_direct() != direct:
                    raise IllegalArgumentException(f"Invalid buffer, isDirect should be {direct}")
            if n == 0:
                return
            self._run([None if b is None else b.address() for b in ins], erased_indexes,
                      [b.address() for b in outs], n)
            for b in ins:
                if b is not None:
                    b.position(b.position() + n)

    def _decode_arrays(self, inputs, erased_indexes, outputs):
        ins = [_in_array(x) for x in inputs]
        n = _first_valid(ins).size
        self._check_parameters(ins, erased_indexes, outputs)
        count = 0
        for b in ins:
            if b is None:
                continue
            if b.size != n:
                raise IllegalArgumentException(f"Invalid buffer, not of length {n}")
            count += 1
        if count < self.get_num_data_units():
            raise IllegalArgumentException("No enough valid inputs are provided, not recoverable")
        for b in outputs:
            if b is None:
                raise IllegalArgumentException("Invalid buffer found, not allowing null")
            if len(b) != n:
                raise IllegalArgumentException(f"Invalid buffer not of length {n}")
        if n == 0:
            return
        outs = [_out_array(o) for o in outputs]
        self._run([None if b is None else b.ctypes.data for b in ins], erased_indexes,
                  [o.ctypes.data for o in outs], n)

    def _check_parameters(self, ins, erased, outs):
        # DecodingState.checkParameters (DecodingState.java:35-51)
        if len(ins) != self.get_num_all_units():
            raise IllegalArgumentException("Invalid inputs length")
        if len(erased) != len(outs):
            raise IllegalArgumentException("erasedIndexes and outputs mismatch in length")
        if len(erased) > self.get_num_parity_units():
            raise IllegalArgumentException("Too many erased, not recoverable")

    def _run(self, in_addrs, erased, out_addrs, n):
        rc = L.lib().ozec_decode(self._handle, L.ptr_array(in_addrs), L.int_array(list(erased)), len(erased),
                                 L.ptr_array(out_addrs), n)
        if rc != L.OZEC_OK:
            _raise_for(rc)

    # ---- device-resident forms ---------------------------------------------------------------------
    def decode_device(self, d_inputs, erased_indexes, d_outputs, length, stream=None):
        rc = L.lib().ozec_decode_device(self._handle, L.ptr_array([_dev_ptr(x) for x in d_inputs]),
                                        L.int_array(list(erased_indexes)), len(erased_indexes),
                                        L.ptr_array([_dev_ptr(x) for x in d_outputs]), length, _stream_ptr(stream))
        if rc != L.OZEC_OK:
            _raise_for(rc)

    def decode_batch(self, d_in, in_stripe_stride, in_unit_stride, present_units, erased_indexes, d_out,
                     out_stripe_stride, out_unit_stride, num_stripes, length, stream=None):
        rc = L.lib().ozec_decode_batch(self._handle, _dev_ptr(d_in), in_stripe_stride, in_unit_stride,
                                       L.int_array(list(present_units)), len(present_units),
                                       L.int_array(list(erased_indexes)), len(erased_indexes), _dev_ptr(d_out),
                                       out_stripe_stride, out_unit_stride, num_stripes, length, _stream_ptr(stream))
        if rc != L.OZEC_OK:
            _raise_for(rc)


    def reconstruct_crc_batch(self, d_in, in_stripe_stride, in_unit_stride, present_units, erased_indexes, d_out,
                              out_stripe_stride, out_unit_stride, num_stripes, length, checksum_type,
                              bytes_per_checksum, d_out_crcs, d_expected=None, d_mismatch=None,
                              expected_big_endian=False, out_big_endian=False, stream=None):
        """Fused reconstruction: verify the read units' stored CRCs, decode, CRC the rebuilt
        units.  d_mismatch[s] = -1 or the smallest unit*nwin + window that failed verification."""
        rc = L.lib().ozec_reconstruct_crc_batch(
            self._handle, _dev_ptr(d_in), in_stripe_stride, in_unit_stride, L.int_array(list(present_units)),
            len(present_units), L.int_array(list(erased_indexes)), len(erased_indexes), _dev_ptr(d_out),
            out_stripe_stride, out_unit_stride, num_stripes, length, int(checksum_type), bytes_per_checksum,
            _dev_ptr(d_expected), 1 if expected_big_endian else 0, _dev_ptr(d_out_crcs), 1 if out_big_endian else 0,
            _dev_ptr(d_mismatch), _stream_ptr(stream))
        if rc != L.OZEC_OK:
            _raise_for(rc)

    def reconstruct_crc_host_batch(self, h_in, in_stripe_stride, in_unit_stride, present_units, erased_indexes, h_out,
                                   out_stripe_stride, out_unit_stride, num_stripes, length, checksum_type,
                                   bytes_per_checksum, h_out_crcs, h_expected=None, h_mismatch=None,
                                   expected_big_endian=False, out_big_endian=False, stripes_per_chunk=0):
        """reconstruct_crc_batch for stripes in HOST memory (ozec_reconstruct_crc_host_batch): the reconstruction
        coordinator's read buffers, pipelined over PCIe.  Host addresses (ints) or numpy arrays; a numpy array must be
        C-contiguous and large enough for the layout it is given as.  Synchronous."""
        k, p = self._config.data, self._config.parity
        e = len(erased_indexes)
        nwin = -(-length // bytes_per_checksum) if bytes_per_checksum > 0 else 0
        S = num_stripes

        def addr(x, what, need, dtype):
            if x is None or isinstance(x, int):
                return x
            if not isinstance(x, np.ndarray) or not x.flags.c_contiguous or x.dtype != dtype or x.nbytes < need:
                raise IllegalArgumentException(f"Invalid {what} buffer: a C-contiguous {np.dtype(dtype).name} array of "
                                               f">= {need} bytes is required")
            if what != "input" and what != "expected" and not x.flags.writeable:
                raise IllegalArgumentException(f"Invalid {what} buffer: not writeable")
            return x.ctypes.data
        umax = max(present_units) if present_units else 0
        in_need = (S - 1) * in_stripe_stride + umax * in_unit_stride + length if S else 0
        out_need = (S - 1) * out_stripe_stride + (e - 1) * out_unit_stride + length if S and e else 0
        rc = L.lib().ozec_reconstruct_crc_host_batch(
            self._handle, addr(h_in, "input", in_need, np.uint8), in_stripe_stride, in_unit_stride,
            L.int_array(list(present_units)), len(present_units), L.int_array(list(erased_indexes)), e,
            addr(h_out, "output", out_need, np.uint8), out_stripe_stride, out_unit_stride, num_stripes, length,
            int(checksum_type), bytes_per_checksum,
            addr(h_expected, "expected", S * (k + p) * nwin * 4, np.uint32), 1 if expected_big_endian else 0,
            addr(h_out_crcs, "rebuilt CRC", S * e * nwin * 4, np.uint32), 1 if out_big_endian else 0,
            addr(h_mismatch, "mismatch", S * 4, np.int32), stripes_per_chunk)
        if rc != L.OZEC_OK:
            _raise_for(rc)


# ---------------------------------------------------------------- dummy coder ----------------------------

class DummyRawEncoder(RawErasureEncoder):
    """DummyRawEncoder (EC/rawcoder/DummyRawEncoder.java:30-45): the inherited validation and position
    bookkeeping run, the coding step does nothing -- the framework-overhead floor of the benchmark.
    Host-only: it never touches the GPU library."""

    def __init__(self, config):  # no native handle
        self._config = config
        self._handle = None

    def _run(self, in_addrs, out_addrs, n):
        pass  # "Nothing to do. Output buffers have already been reset"

    def release(self):
        pass  # RawErasureEncoder.release: "Nothing to do here."


class DummyRawDecoder(RawErasureDecoder):
    """DummyRawDecoder (EC/rawcoder/DummyRawDecoder.java): validation only, no decoding."""

    def __init__(self, config):
        self._config = config
        self._handle = None
        self._lock = threading.Lock()

    def _run(self, in_addrs, erased, out_addrs, n):
        pass

    def release(self):
        pass


# ---------------------------------------------------------------- factories / registry -------------------

class RawErasureCoderFactory:
    """RawErasureCoderFactory (EC/rawcoder/RawErasureCoderFactory.java:29-56)."""

    coder_name = None
    codec_name = None

    def create_encoder(self, config):
        return RawErasureEncoder(config)

    def create_decoder(self, config):
        return RawErasureDecoder(config)

    def get_coder_name(self):
        return self.coder_name

    def get_codec_name(self):
        return self.codec_name


class DummyRawErasureCoderFactory(RawErasureCoderFactory):
    """DummyRawErasureCoderFactory (EC/rawcoder/DummyRawErasureCoderFactory.java:27-52)."""
    coder_name = "dummy_dummy"
    codec_name = "dummy"

    def create_encoder(self, config):
        return DummyRawEncoder(config)

    def create_decoder(self, config):
        return DummyRawDecoder(config)


class HipRSRawErasureCoderFactory(RawErasureCoderFactory):
    coder_name = "rs_hip"
    codec_name = "rs"


class HipXORRawErasureCoderFactory(RawErasureCoderFactory):
    coder_name = "xor_hip"
    codec_name = "xor"


class CodecRegistry:
    """CodecRegistry (EC/CodecRegistry.java:43-170) for the GPU factories of this package."""

    _instance = None

    def __init__(self, factories=None):
        self._by_codec = {}
        self.update_coders(factories or [HipRSRawErasureCoderFactory(), HipXORRawErasureCoderFactory()])

    @classmethod
    def get_instance(cls):
        if cls._instance is None:
            cls._instance = cls()
        return cls._instance

    def update_coders(self, factories):
        for f in factories:
            lst = self._by_codec.setdefault(f.get_codec_name(), [])
            if any(x.get_coder_name() == f.get_coder_name() for x in lst):  # CodecRegistry.java:80-90
                continue
            lst.append(f)

    def get_coder_names(self, codec):
        return [f.get_coder_name() for f in self._by_codec.get(codec, [])]

    def get_coders(self, codec):
        return list(self._by_codec.get(codec, []))

    def get_codec_names(self):
        return sorted(self._by_codec)

    def get_coder_by_name(self, codec, coder_name):
        for f in self._by_codec.get(codec, []):
            if f.get_coder_name() == coder_name:
                return f
        return None


class CodecUtil:
    """CodecUtil.createRaw{En,De}coderWithFallback (EC/rawcoder/util/CodecUtil.java:55-110)."""

    @staticmethod
    def _create(config, decoder):
        reg = CodecRegistry.get_instance()
        errors = []
        for f in reg.get_coders(config.get_codec()):
            try:
                return f.create_decoder(config) if decoder else f.create_encoder(config)
            except Exception as e:  # skipped, like LinkageError/Exception in CodecUtil.java:62-78
                errors.append(f"{f.get_coder_name()}: {e}")
        raise IllegalArgumentException(
            f"Fail to create raw erasure {'decoder' if decoder else 'encoder'} with given codec: "
            f"{config.get_codec()} ({'; '.join(errors)})")

    @staticmethod
    def create_raw_encoder_with_fallback(config):
        return CodecUtil._create(config, False)

    @staticmethod
    def create_raw_decoder_with_fallback(config):
        return CodecUtil._create(config, True)


# ---------------------------------------------------------------- host-side math ---------------------------

def rs_encode_matrix(k, p):
    """RSUtil.genCauchyMatrix (RSUtil.java:64-77) as computed by libozec."""
    m = np.zeros((k + p) * k, np.uint8)
    rc = L.lib().ozec_rs_encode_matrix(k, p, m.ctypes.data)
    if rc != L.OZEC_OK:
        _raise_for(rc, HadoopIllegalArgumentException)
    return m.reshape(k + p, k)


def rs_decode_matrix(k, p, valid_indexes, erased_indexes):
    """RSRawDecoder.generateDecodeMatrix (RSRawDecoder.java:143-176) as computed by libozec."""
    out = np.zeros(max(1, len(erased_indexes)) * k, np.uint8)
    rc = L.lib().ozec_rs_decode_matrix(k, p, L.int_array(list(valid_indexes)), L.int_array(list(erased_indexes)),
                                       len(erased_indexes), out.ctypes.data)
    if rc != L.OZEC_OK:
        _raise_for(rc)
    return out[:len(erased_indexes) * k].reshape(len(erased_indexes), k)


def gf_invert_matrix(mat):
    a = np.ascontiguousarray(mat, np.uint8).copy()
    n = a.shape[0]
    out = np.zeros((n, n), np.uint8)
    rc = L.lib().ozec_gf_invert_matrix(a.ctypes.data, out.ctypes.data, n)
    if rc != L.OZEC_OK:
        _raise_for(rc)
    return out


def gf_mul(a, b):
    return int(L.lib().ozec_gf_mul(a, b))


def device_count():
    return int(L.lib().ozec_device_count())


DEVICE_POLICY = {"round_robin": 0, "numa": 1, "current": 2}


def set_devices(devices=None):
    """The GPUs this process's coders and host batches use (ozec_set_devices): None / [] restores every visible GPU
    (or OZEC_DEVICES).  Coders created afterwards take them in turn; host batches split over all of them."""
    devs = list(devices or [])
    arr = (ctypes.c_int * max(1, len(devs)))(*devs)
    rc = L.lib().ozec_set_devices(arr, len(devs))
    if rc != L.OZEC_OK:
        _raise_for(rc)


def get_devices():
    n = L.lib().ozec_get_devices(None, 0)
    arr = (ctypes.c_int * max(1, n))()
    L.lib().ozec_get_devices(arr, n)
    return list(arr)[:n]


def set_device_policy(policy):
    rc = L.lib().ozec_set_device_policy(DEVICE_POLICY[policy] if isinstance(policy, str) else int(policy))
    if rc != L.OZEC_OK:
        _raise_for(rc)


def fill_splitmix64_cells(d_base, cell_stride, num_cells, length, seed, first_stream, stream=None):
    rc = L.lib().ozec_fill_splitmix64_cells(_dev_ptr(d_base), cell_stride, num_cells, length, seed, first_stream,
                                            _stream_ptr(stream))
    if rc != L.OZEC_OK:
        _raise_for(rc)
