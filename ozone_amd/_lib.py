"""ctypes binding of libozec.so (include/ozec.h) -- the only way the Python host layer reaches the GPU.

There is no Python or CPU fallback: if the in-tree library is missing or fails to load, every entry point
raises OzecLibraryError.  Build it with `python -c "import __graft_entry__ as g; g.build()"` or
`make -C ozone_amd/csrc`.
"""
import ctypes
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
# OZEC_LIB_OVERRIDE: another build of the same library (the sanitizer build of tests/test_host_abi_asan.py)
LIB_PATH = os.environ.get("OZEC_LIB_OVERRIDE") or os.path.join(_HERE, "lib", "libozec.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "ozec.h")

OZEC_OK = 0
OZEC_EINVAL = -1
OZEC_ENOTINVERTIBLE = -2
OZEC_EDEVICE = -3
OZEC_ECLOSED = -4
OZEC_ENOMEM = -5
OZEC_EUNSUPPORTED = -6
OZEC_EMISMATCH = -7

OZEC_CODEC_RS = 0
OZEC_CODEC_XOR = 1
OZEC_CHECKSUM_NONE = 1
OZEC_CHECKSUM_CRC32 = 2
OZEC_CHECKSUM_CRC32C = 3
OZEC_MAX_K = 64
OZEC_MAX_ROWS = 16
OP_NAMES = ["encode", "decode", "encode_device", "decode_device", "fused", "host_batch", "checksum",
            "checksum_device", "queue"]  # OZEC_OP_* order


class OpStats(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_uint64), ("bytes", ctypes.c_uint64), ("errors", ctypes.c_uint64),
                ("host_ns", ctypes.c_uint64)]


class OzecLibraryError(RuntimeError):
    """libozec.so is missing or broken: the GPU path cannot run (there is deliberately no fallback)."""


class OzecError(Exception):
    def __init__(self, code, message):
        super().__init__(message)
        self.code = code


_lib = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_voidp = ctypes.c_void_p
c_ptrs = ctypes.POINTER(ctypes.c_void_p)
c_intp = ctypes.POINTER(ctypes.c_int)
c_i64 = ctypes.c_int64
c_size = ctypes.c_size_t

# ozec_fill_fn / ozec_drain_fn (include/ozec.h): (user, off, len, unit pointers) -> status
FILL_FN = ctypes.CFUNCTYPE(ctypes.c_int, c_voidp, c_size, c_size, ctypes.POINTER(ctypes.c_void_p))
DRAIN_FN = ctypes.CFUNCTYPE(ctypes.c_int, c_voidp, c_size, c_size, ctypes.POINTER(ctypes.c_void_p))

_SIGS = {
    "ozec_encode_cb": (ctypes.c_int, [c_voidp, c_size, FILL_FN, DRAIN_FN, c_voidp]),
    "ozec_decode_cb": (ctypes.c_int, [c_voidp, ctypes.POINTER(ctypes.c_uint8), c_intp, ctypes.c_int, c_size, FILL_FN,
                                      DRAIN_FN, c_voidp]),
    "ozec_last_error": (ctypes.c_char_p, []),
    "ozec_version": (ctypes.c_int, []),
    "ozec_device_count": (ctypes.c_int, []),
    "ozec_set_device": (ctypes.c_int, [ctypes.c_int]),
    "ozec_synchronize": (ctypes.c_int, []),
    "ozec_encoder_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(c_voidp)]),
    "ozec_decoder_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(c_voidp)]),
    "ozec_coder_release": (ctypes.c_int, [c_voidp]),
    "ozec_coder_free": (None, [c_voidp]),
    "ozec_coder_retain": (ctypes.c_int, [c_voidp]),
    "ozec_release_staging": (ctypes.c_int, []),
    "ozec_coder_is_closed": (ctypes.c_int, [c_voidp]),
    "ozec_coder_info": (ctypes.c_int, [c_voidp, c_intp, c_intp, c_intp, c_intp]),
    "ozec_encode": (ctypes.c_int, [c_voidp, c_ptrs, c_ptrs, c_size]),
    "ozec_decode": (ctypes.c_int, [c_voidp, c_ptrs, c_intp, ctypes.c_int, c_ptrs, c_size]),
    "ozec_encode_device": (ctypes.c_int, [c_voidp, c_ptrs, c_ptrs, c_size, c_voidp]),
    "ozec_decode_device": (ctypes.c_int, [c_voidp, c_ptrs, c_intp, ctypes.c_int, c_ptrs, c_size, c_voidp]),
    "ozec_encode_batch": (ctypes.c_int, [c_voidp, c_voidp, c_i64, c_i64, c_voidp, c_i64, c_i64, c_size, c_size,
                                         c_voidp]),
    "ozec_decode_batch": (ctypes.c_int, [c_voidp, c_voidp, c_i64, c_i64, c_intp, ctypes.c_int, c_intp, ctypes.c_int,
                                         c_voidp, c_i64, c_i64, c_size, c_size, c_voidp]),
    "ozec_encode_crc_batch": (ctypes.c_int, [c_voidp, c_voidp, c_i64, c_i64, c_voidp, c_i64, c_i64, c_size, c_size,
                                             ctypes.c_int, c_size, c_voidp, ctypes.c_int, c_voidp]),
    "ozec_checksum_windows": (ctypes.c_int, [ctypes.c_int, c_voidp, c_size, c_size, c_voidp, ctypes.c_int]),
    "ozec_checksum_windows_device": (ctypes.c_int, [ctypes.c_int, c_voidp, c_size, c_size, c_voidp, ctypes.c_int,
                                                    c_voidp]),
    "ozec_checksum_windows_batch": (ctypes.c_int, [ctypes.c_int, c_voidp, c_i64, c_size, c_size, c_size, c_voidp,
                                                   ctypes.c_int, c_voidp]),
    "ozec_checksum_verify": (ctypes.c_int, [ctypes.c_int, c_voidp, c_size, c_size, c_voidp, c_size, c_size,
                                            ctypes.POINTER(c_i64)]),
    "ozec_checksum_verify_batch": (ctypes.c_int, [ctypes.c_int, c_voidp, c_i64, c_size, c_size, c_size, c_voidp,
                                                  ctypes.c_int, c_voidp, c_voidp]),
    "ozec_reconstruct_crc_batch": (ctypes.c_int, [c_voidp, c_voidp, c_i64, c_i64, c_intp, ctypes.c_int, c_intp,
                                                  ctypes.c_int, c_voidp, c_i64, c_i64, c_size, c_size, ctypes.c_int,
                                                  c_size, c_voidp, ctypes.c_int, c_voidp, ctypes.c_int, c_voidp,
                                                  c_voidp]),
    "ozec_reconstruct_crc_host_batch": (ctypes.c_int, [c_voidp, c_voidp, c_i64, c_i64, c_intp, ctypes.c_int, c_intp,
                                                       ctypes.c_int, c_voidp, c_i64, c_i64, c_size, c_size, ctypes.c_int,
                                                       c_size, c_voidp, ctypes.c_int, c_voidp, ctypes.c_int, c_voidp,
                                                       c_size]),
    "ozec_crc_reset": (ctypes.c_uint32, [ctypes.c_int]),
    "ozec_crc_update": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), c_voidp, c_size]),
    "ozec_crc_value": (ctypes.c_uint32, [ctypes.c_int, ctypes.c_uint32]),
    "ozec_rs_encode_matrix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_voidp]),
    "ozec_rs_decode_matrix": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, c_intp, c_intp, ctypes.c_int, c_voidp]),
    "ozec_gf_invert_matrix": (ctypes.c_int, [c_voidp, c_voidp, ctypes.c_int]),
    "ozec_gf_mul": (ctypes.c_uint8, [ctypes.c_uint8, ctypes.c_uint8]),
    "ozec_parse_replication": (ctypes.c_int, [ctypes.c_char_p, c_intp, c_intp, c_intp, c_intp]),
    "ozec_crc_combine": (ctypes.c_uint32, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    "ozec_host_alloc": (ctypes.c_int, [c_size, ctypes.POINTER(c_voidp)]),
    "ozec_host_alloc_on": (ctypes.c_int, [c_size, ctypes.c_int, ctypes.POINTER(c_voidp)]),
    "ozec_host_free": (ctypes.c_int, [c_voidp]),
    "ozec_host_free_failures": (ctypes.c_uint64, []),
    "ozec_device_numa_node": (ctypes.c_int, [ctypes.c_int, c_intp]),
    "ozec_host_page_node": (ctypes.c_int, [c_voidp, c_intp]),
    "ozec_host_copy": (ctypes.c_int, [c_voidp, c_voidp, c_voidp, ctypes.c_int, ctypes.c_int]),
    "ozec_host_register": (ctypes.c_int, [c_voidp, c_size, ctypes.c_int]),
    "ozec_host_placement_failures": (ctypes.c_uint64, []),
    "ozec_host_unregister": (ctypes.c_int, [c_voidp]),
    "ozec_encode_crc_block_groups": (ctypes.c_int, [c_voidp, c_voidp, c_i64, c_i64, c_size, c_size, c_size,
                                                    ctypes.c_int, c_size, c_voidp, ctypes.c_int, c_voidp]),
    "ozec_encode_crc_host_batch": (ctypes.c_int, [c_voidp, c_voidp, c_i64, c_i64, c_voidp, c_i64, c_i64, c_size,
                                                  c_size, ctypes.c_int, c_size, c_voidp, ctypes.c_int, c_size]),
    "ozec_stripe_queue_info": (ctypes.c_int, [c_voidp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                              ctypes.POINTER(ctypes.c_int), ctypes.POINTER(c_size),
                                              ctypes.POINTER(ctypes.c_int), ctypes.POINTER(c_size)]),
    "ozec_stripe_queue_state": (ctypes.c_int, [c_voidp, ctypes.POINTER(c_size), ctypes.POINTER(ctypes.c_uint64),
                                               ctypes.POINTER(c_size)]),
    "ozec_stripe_queue_create": (ctypes.c_int, [c_voidp, c_size, c_size, ctypes.c_int, c_size, ctypes.c_int,
                                                ctypes.POINTER(c_voidp)]),
    "ozec_stripe_queue_submit": (ctypes.c_int, [c_voidp, c_ptrs, c_ptrs, c_size, c_voidp,
                                                ctypes.POINTER(ctypes.c_uint64)]),
    "ozec_stripe_queue_flush": (ctypes.c_int, [c_voidp]),
    "ozec_stripe_queue_wait": (ctypes.c_int, [c_voidp, ctypes.c_uint64]),
    "ozec_stripe_queue_free": (ctypes.c_int, [c_voidp]),
    "ozec_crc_monomial": (ctypes.c_int, [ctypes.c_int, c_i64, ctypes.POINTER(ctypes.c_uint32)]),
    "ozec_crc_compose": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, c_i64,
                                        ctypes.POINTER(ctypes.c_uint32)]),
    "ozec_crc_composer_create": (ctypes.c_int, [ctypes.c_int, c_i64, c_i64, ctypes.POINTER(c_voidp)]),
    "ozec_crc_composer_update": (ctypes.c_int, [c_voidp, ctypes.c_uint32, c_i64]),
    "ozec_crc_composer_update_bytes": (ctypes.c_int, [c_voidp, c_voidp, c_size, c_i64]),
    "ozec_crc_composer_pending": (c_size, [c_voidp]),
    "ozec_crc_composer_digest": (ctypes.c_int, [c_voidp, c_voidp, c_size, ctypes.POINTER(c_size)]),
    "ozec_crc_composer_free": (None, [c_voidp]),
    "ozec_crc_compose_windows_batch": (ctypes.c_int, [ctypes.c_int, c_voidp, c_i64, c_size, c_size, c_size, c_size,
                                                      ctypes.c_int, c_voidp, ctypes.c_int, c_voidp]),
    "ozec_stats": (ctypes.c_int, [ctypes.c_int, c_voidp]),
    "ozec_stats_reset": (None, []),
    "ozec_fused_routes": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    "ozec_set_tuning": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int64]),
    "ozec_get_tuning": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]),
    "ozec_tuning_variants": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "ozec_set_devices": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "ozec_get_devices": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "ozec_set_device_policy": (ctypes.c_int, [ctypes.c_int]),
    "ozec_device_policy": (ctypes.c_int, []),
    "ozec_coder_device": (ctypes.c_int, [ctypes.c_void_p]),
    "ozec_fill_splitmix64": (ctypes.c_int, [c_voidp, c_size, ctypes.c_uint64, ctypes.c_uint64, c_voidp]),
    "ozec_fill_splitmix64_cells": (ctypes.c_int, [c_voidp, c_i64, c_size, c_size, ctypes.c_uint64, ctypes.c_uint64,
                                                  c_voidp]),
}


def lib():
    """Load the in-tree libozec.so (once)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OzecLibraryError(
                f"{LIB_PATH} not found: build the HIP extension first (make -C ozone_amd/csrc); "
                "ozone_amd has no CPU fallback")
        try:
            L = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover - environment specific
            raise OzecLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def header_symbols():
    """Function names declared in include/ozec.h."""
    text = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\s*\*?\s*(ozec_[a-z0-9_]+)\s*\(", text, re.M)))


def last_error():
    return lib().ozec_last_error().decode("utf-8", "replace")


def check(rc):
    """Raise OzecError for a negative status."""
    if rc != OZEC_OK:
        raise OzecError(rc, last_error())
    return rc


def ptr_array(addrs):
    arr = (c_voidp * max(1, len(addrs)))()
    for i, a in enumerate(addrs):
        arr[i] = a if a else None
    return arr


def int_array(vals):
    return (ctypes.c_int * max(1, len(vals)))(*vals)


def stats():
    """{op name: {calls, bytes, errors, host_ns}} from ozec_stats (per-call counters of the C ABI)."""
    out = {}
    for i, name in enumerate(OP_NAMES):
        st = OpStats()
        check(lib().ozec_stats(i, ctypes.byref(st)))
        out[name] = {"calls": st.calls, "bytes": st.bytes, "errors": st.errors, "host_ns": st.host_ns}
    return out


def stats_reset():
    lib().ozec_stats_reset()
