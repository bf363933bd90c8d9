#!/usr/bin/env python3
"""Non-faulting probe of host-memory lock lifetimes (round 6, DESIGN §4 "GPU faults").

Every recorded hipErrorIllegalAddress (rounds 4-5, five runs) surfaced in a torch PAGEABLE copy of exactly 1,310,720 B
(a (4, 5, 65536) uint8 tensor; `.cpu()` three times, `.to("cuda")` of a numpy array once).  HIP carries out such a
copy by locking the caller's pages (ROCr hsa_amd_memory_lock_to_pool, "Locking to pool" in its log).  This probe asks
ROCr directly -- hsa_amd_pointer_info, which reports HSA_EXT_POINTER_TYPE_LOCKED for a locked host range with its
base and size -- how long such a lock lives:

  phase copy : after a pageable D2H / H2D of that size, is the host range still locked?  after the tensor is freed?
               after N further pageable copies of other sizes (how many locks does HIP keep)?
  phase free : the same question for libozec's own pinned blocks (ozec_host_alloc / ozec_host_free) and for caller
               memory registered with ozec_host_register then unregistered.

Nothing here forces a fault: the probe reads ROCr's bookkeeping and never touches a range it suspects.
Usage: python scripts/lock_probe.py
"""
import ctypes
import gc
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ozone_amd.stripe_queue import host_alloc, host_register, host_unregister  # noqa: E402

TYPES = {0: "UNKNOWN", 1: "HSA", 2: "LOCKED", 3: "GRAPHICS", 4: "IPC", 5: "RESERVED_ADDR", 6: "HSA_VMEM"}


class PtrInfo(ctypes.Structure):
    _fields_ = [("size", ctypes.c_uint32), ("type", ctypes.c_int), ("agentBaseAddress", ctypes.c_void_p),
                ("hostBaseAddress", ctypes.c_void_p), ("sizeInBytes", ctypes.c_size_t), ("userData", ctypes.c_void_p),
                ("agentOwner", ctypes.c_uint64), ("global_flags", ctypes.c_uint32), ("registered", ctypes.c_bool)]


hsa = None
hip = None
COPY = 4 * 5 * 65536


def loaded(stem):
    """path of the copy of a shared library this process has mapped (torch may bundle its own ROCm runtime)"""
    with open("/proc/self/maps") as f:
        for line in f:
            if stem in line and line.rstrip().endswith((".so", ".so.1", ".so.2", ".so.6", ".so.7")) or \
                    (stem in line and ".so." in line):
                return line.split()[-1]
    return None


def bind():
    global hsa, hip
    hp, ap = loaded("libhsa-runtime64"), loaded("libamdhip64")
    say(f"loaded ROCr {hp}, HIP {ap}")
    hsa = ctypes.CDLL(hp)
    hsa.hsa_amd_pointer_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(PtrInfo), ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p]
    hip = ctypes.CDLL(ap)
    hip.hipPointerGetAttribute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]


def hipinfo(p):
    """HIP's own view: HIP_POINTER_ATTRIBUTE_MEMORY_TYPE (2) and RANGE_START_ADDR (11) / RANGE_SIZE (12)"""
    mt, start, size = ctypes.c_uint(0), ctypes.c_void_p(0), ctypes.c_size_t(0)
    e1 = hip.hipPointerGetAttribute(ctypes.byref(mt), 2, ctypes.c_void_p(p))
    e2 = hip.hipPointerGetAttribute(ctypes.byref(start), 11, ctypes.c_void_p(p))
    e3 = hip.hipPointerGetAttribute(ctypes.byref(size), 12, ctypes.c_void_p(p))
    hip.hipGetLastError()
    return f"hip(err {e1}/{e2}/{e3} type={mt.value} start={hex(start.value or 0)} size={size.value:#x})"


def info(p):
    i = PtrInfo()
    i.size = ctypes.sizeof(PtrInfo)
    st = hsa.hsa_amd_pointer_info(ctypes.c_void_p(p), ctypes.byref(i), None, None, None)
    t = TYPES.get(i.type, str(i.type))
    if t == "UNKNOWN":
        return f"st={st} {t}; {hipinfo(p)}"
    return (f"st={st} {t} host_base={hex(i.hostBaseAddress or 0)} size={i.sizeInBytes:#x} registered={i.registered}; "
            f"{hipinfo(p)}")


def say(msg):
    print(msg, flush=True)


def phase_copy(dev):
    g = torch.full((4, 5, 65536), 7, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    y = g.cpu()
    a = y.data_ptr()
    say(f"[copy] D2H .cpu() of {COPY} B into host {hex(a)}: {info(a)}")
    del y
    gc.collect()
    say(f"[copy] after the host tensor is freed: {info(a)}")
    x = np.full((4, 5, 65536), 3, np.uint8)
    b = x.ctypes.data
    d = torch.from_numpy(x).to(dev)
    torch.cuda.synchronize()
    say(f"[copy] H2D .to() of {COPY} B from numpy {hex(b)}: {info(b)}")
    del x, d
    gc.collect()
    say(f"[copy] after the numpy array is freed: {info(b)}")
    keep = []
    for i in range(12):
        n = (1 << 20) + (i + 1) * 65536 * 3
        t = torch.empty(n, dtype=torch.uint8, device=dev)
        h = t.cpu()
        keep.append(h)
        say(f"[copy] after {i + 1} further pageable copies ({n} B into {hex(h.data_ptr())}): first range {info(a)}; "
            f"this one {info(h.data_ptr())}")
    del keep
    gc.collect()
    say(f"[copy] end: first range {info(a)}, numpy range {info(b)}")


def phase_free(dev):
    pb = host_alloc(8 << 20)
    p = pb.array.ctypes.data
    say(f"[free] ozec_host_alloc 8 MiB at {hex(p)}: {info(p)}")
    d = torch.empty(8 << 20, dtype=torch.uint8, device=dev)
    d.copy_(torch.from_numpy(pb.array))  # DMA from the pinned block
    torch.cuda.synchronize()
    pb.free()
    say(f"[free] after ozec_host_free: {info(p)}")
    buf = np.zeros(4 << 20, np.uint8)
    q = buf.ctypes.data + (-buf.ctypes.data) % 4096
    host_register(q, 2 << 20, -1)
    say(f"[free] ozec_host_register 2 MiB at {hex(q)}: {info(q)}")
    host_unregister(q)
    say(f"[free] after ozec_host_unregister: {info(q)}")
    del buf


def main():
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    bind()
    say(f"GPU_PINNED_MIN_XFER_SIZE={os.environ.get('GPU_PINNED_MIN_XFER_SIZE')}")
    phase_copy(dev)
    phase_free(dev)
    say("probe done")


if __name__ == "__main__":
    main()
