"""BASELINE configs[4] (C5) path and its host memory: ozec_encode_crc_host_batch against the oracle (pinned and
pageable batches, several chunkings), NUMA-local pinned allocations, and one host batch split by stripe range
between two rank processes on one device (the multi-GPU partition of SURVEY §8(e), rehearsed on one GPU)."""
import ctypes
import mmap
import os
import socket

import numpy as np
import pytest

import oracle
from synth import SEED, cells

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from ozone_amd import _lib as L  # noqa: E402
from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402
from ozone_amd.shard import stripe_range  # noqa: E402
from ozone_amd.stripe_queue import device_numa_node, host_alloc, host_register, host_unregister, page_node  # noqa

OTYPE = {ck.ChecksumType.CRC32C: oracle.CRC32C, ck.ChecksumType.CRC32: oracle.CRC32}


def _batch(S, k, p, n, first, extra_unit_gap=0):
    """[S][k+p][n] host batch (data from the oracle's generator, parity slots 0xA5) with optional gap per unit."""
    us = n + extra_unit_gap
    buf = np.full(S * (k + p) * us, 0xA5, np.uint8)
    v = buf.reshape(S, k + p, us)
    for s in range(S):
        for j, x in enumerate(cells(SEED, first + s * k, k, n)):
            v[s, j, :n] = x
    return buf, v, us


def _check(v, crcs, codec, k, p, n, S, ctype, bpc, big_endian=False):
    nwin = (n + bpc - 1) // bpc if ctype != ck.ChecksumType.NONE else 0
    units = k + (1 if codec == "xor" else p)
    for s in range(S):
        d = [np.array(v[s, j, :n]) for j in range(k)]
        ref = oracle.rs_encode(k, p, d) if codec == "rs" else [oracle.xor_encode(d)] + [np.zeros(n, np.uint8)] * (p - 1)
        for r in range(p):
            assert (v[s, k + r, :n] == ref[r]).all(), (s, r)
        if nwin:
            got = crcs.reshape(S, units, nwin)[s]
            if big_endian:
                got = got.byteswap()
            for u, cell in enumerate(d + ref[:units - k]):
                assert (got[u] == oracle.crc_windows(OTYPE[ctype], cell, bpc)).all(), (s, u)


@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("codec,k,p,n,S,chunk,ctype,bpc", [
    ("rs", 6, 3, 1 << 16, 37, 8, ck.ChecksumType.CRC32C, 16384),   # 5 chunks through a ring of 3
    ("rs", 6, 3, 1 << 20, 5, 0, ck.ChecksumType.CRC32C, 16384),    # C5 cells, default chunking
    ("rs", 10, 4, 50000, 7, 2, ck.ChecksumType.CRC32, 4096),       # unfused fallback shape (len % 16 != 0)
    ("rs", 3, 2, 1 << 15, 9, 4, ck.ChecksumType.NONE, 0),          # encode only
    ("xor", 2, 1, 1 << 16, 11, 3, ck.ChecksumType.CRC32C, 8192),
    ("xor", 3, 2, 1 << 14, 6, 4, ck.ChecksumType.CRC32C, 4096),    # XOR p > 1: extra parity zero-filled
])
def test_host_batch_vs_oracle(pinned, codec, k, p, n, S, chunk, ctype, bpc):
    buf, v, us = _batch(S, k, p, n, 800000 + 1000 * k)
    units = k + (1 if codec == "xor" else p)
    nwin = (n + bpc - 1) // bpc if bpc else 0
    crcs = np.zeros(max(1, S * units * nwin), np.uint32)
    keep = []
    if pinned:  # the whole batch and the CRC area registered, as bench.py's C5 batch is
        pb = host_alloc(buf.nbytes)
        pb.array[:] = buf
        pc = host_alloc(crcs.nbytes)
        pc.array[:] = 0
        keep += [pb, pc]
        v = pb.array.reshape(S, k + p, us)
        crcs = pc.array.view(np.uint32)
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p, codec))
    base = v.ctypes.data
    e.encode_crc_host_batch(base, (k + p) * us, us, base + k * us, (k + p) * us, us, S, n, ctype, bpc,
                            crcs if ctype != ck.ChecksumType.NONE else None, False, chunk)
    _check(v, crcs, codec, k, p, n, S, ctype, bpc)


def test_host_batch_strided_units_and_big_endian():
    """Units not back to back (a gap after every cell): the per-cell copy path; CRCs stored big-endian."""
    k, p, n, S, bpc = 6, 3, 1 << 15, 6, 4096
    buf, v, us = _batch(S, k, p, n, 810000, extra_unit_gap=4096)
    pb = host_alloc(buf.nbytes)
    pb.array[:] = buf
    v = pb.array.reshape(S, k + p, us)
    crcs = np.zeros(S * (k + p) * (n // bpc), np.uint32)
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    base = v.ctypes.data
    e.encode_crc_host_batch(base, (k + p) * us, us, base + k * us, (k + p) * us, us, S, n, ck.ChecksumType.CRC32C,
                            bpc, crcs, True, 4)
    _check(v, crcs, "rs", k, p, n, S, ck.ChecksumType.CRC32C, bpc, big_endian=True)
    assert (v[:, :, n:] == 0xA5).all()  # the gaps are untouched


def test_release_staging_between_host_batches():
    """ozec_release_staging gives the host-batch ring (device chunk buffers, pinned staging) and the idle slots'
    buffers back (they only ever grew); the next calls allocate again and stay bit-exact."""
    from ozone_amd import _lib as L
    k, p, n, S, bpc = 6, 3, 1 << 16, 9, 16384
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    for rep in range(3):
        buf, v, us = _batch(S, k, p, n, 815000 + rep * 100)
        crcs = np.zeros(S * (k + p) * (n // bpc), np.uint32)
        base = v.ctypes.data
        e.encode_crc_host_batch(base, (k + p) * us, us, base + k * us, (k + p) * us, us, S, n, ck.ChecksumType.CRC32C,
                                bpc, crcs, False, 4)  # pageable: staged through the ring's pinned buffers
        _check(v, crcs, "rs", k, p, n, S, ck.ChecksumType.CRC32C, bpc)
        d = cells(SEED, 815500 + rep, k, 5000)
        par = [np.zeros(5000, np.uint8) for _ in range(p)]
        e.encode(d, par)  # a host-buffer call through a staging slot
        assert all((a == b).all() for a, b in zip(par, oracle.rs_encode(k, p, d)))
        assert L.lib().ozec_release_staging() == 0


def test_host_register_pins_when_placement_is_refused(tmp_path):
    """ozec_host_register places pages best effort (it used to fail outright when mbind was refused, as
    under a seccomp profile without CAP_SYS_NICE): with mbind failing (test hook) the memory is still pinned, a host
    batch over it is bit-exact, and the refusal is counted."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = f"""
import sys; sys.path[:0] = [{root!r}, {os.path.join(root, 'tests')!r}, {os.path.join(root, 'tests', 'golden')!r}]
import numpy as np, torch
torch.cuda.set_device(0)
from ozone_amd import _lib as L, checksum as ck, rawcoder as rc
from ozone_amd.stripe_queue import host_register, host_unregister
import test_gpu_e2e as t
k, p, n, S, bpc = 6, 3, 1 << 15, 5, 8192
buf, v, us = t._batch(S, k, p, n, 816000)
crcs = np.zeros(S * (k + p) * (n // bpc), np.uint32)
before = L.lib().ozec_host_placement_failures()
host_register(buf.ctypes.data, buf.nbytes, 0)
host_register(crcs.ctypes.data, crcs.nbytes, 0)
assert L.lib().ozec_host_placement_failures() == before + 2
e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
base = v.ctypes.data
e.encode_crc_host_batch(base, (k + p) * us, us, base + k * us, (k + p) * us, us, S, n, ck.ChecksumType.CRC32C, bpc,
                        crcs, False, 2)
t._check(v, crcs, "rs", k, p, n, S, ck.ChecksumType.CRC32C, bpc)
host_unregister(buf.ctypes.data); host_unregister(crcs.ctypes.data)
print("ok")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, OZEC_TEST_FAIL_MBIND="1"))
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_host_batch_errors():
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(6, 3))
    buf = np.zeros(9 * 4096, np.uint8)
    with pytest.raises(rc.IllegalArgumentException):
        e.encode_crc_host_batch(buf, 9 * 4096, 4096, None, 9 * 4096, 4096, 1, 4096, ck.ChecksumType.CRC32C, 4096,
                                np.zeros(9, np.uint32))
    with pytest.raises(rc.IllegalArgumentException):  # CRC requested without a CRC buffer
        e.encode_crc_host_batch(buf, 9 * 4096, 4096, buf.ctypes.data + 6 * 4096, 9 * 4096, 4096, 1, 4096,
                                ck.ChecksumType.CRC32C, 4096, None)
    e.release()
    with pytest.raises(rc.IOException):
        e.encode_crc_host_batch(buf, 9 * 4096, 4096, buf.ctypes.data + 6 * 4096, 9 * 4096, 4096, 1, 4096,
                                ck.ChecksumType.NONE, 0, None)


def _recon_batch(codec, k, p, n, S, first, gap=0):
    """[S][k+p][n + gap] host stripes, every unit present (parity from the oracle)."""
    us = n + gap
    buf = np.full(S * (k + p) * us, 0xA5, np.uint8)
    v = buf.reshape(S, k + p, us)
    for s in range(S):
        d = cells(SEED, first + s * k, k, n)
        par = oracle.rs_encode(k, p, d) if codec == "rs" else [oracle.xor_encode(d)] + [np.zeros(n, np.uint8)] * (p - 1)
        for u, x in enumerate(d + par):
            v[s, u, :n] = x
    return buf, v, us


@pytest.mark.parametrize("pinned", [True, False])
@pytest.mark.parametrize("codec,k,p,erased,n,S,chunk,bpc,gap", [
    ("rs", 10, 4, [0, 1, 2, 3], 1 << 16, 13, 4, 16384, 0),      # one run of read units {4..13}, 4 chunks
    ("rs", 10, 4, [1, 4, 10, 13], 1 << 15, 7, 3, 4096, 0),      # four runs {0},{2,3},{5..9},{11,12}
    ("rs", 6, 3, [0, 2, 7], 1 << 16, 9, 0, 16384, 4096),        # gaps between units: per-cell copies
    ("rs", 6, 3, [8], 50000, 5, 2, 1000, 0),                    # unfused fallback (len, bpc not 16-aligned)
    ("xor", 2, 1, [1], 1 << 15, 6, 4, 8192, 0),
])
def test_reconstruct_host_batch_vs_oracle(pinned, codec, k, p, erased, n, S, chunk, bpc, gap):
    """ozec_reconstruct_crc_host_batch: rebuilt units equal the originals, their CRCs equal the stored ones, and a
    corrupted window of a read unit is reported for its stripe only."""
    buf, v, us = _recon_batch(codec, k, p, n, S, 830000 + 100 * k, gap)
    nwin = (n + bpc - 1) // bpc
    ctype, otype = ck.ChecksumType.CRC32C, oracle.CRC32C
    stored = np.stack([np.stack([oracle.crc_windows(otype, np.array(v[s, u, :n]), bpc) for u in range(k + p)])
                       for s in range(S)]).astype(np.uint32).reshape(-1)
    present = [u for u in range(k + p) if u not in erased]
    read = present[:k]
    orig = np.array(v[:, :, :n])
    v[:, erased, :] = 0xEE                       # erased units hold garbage in the caller's buffers
    v[2, read[-1], 2 * bpc + 5] ^= 0x01          # stripe 2: silent corruption in the last unit read
    e = len(erased)
    out = np.zeros(S * e * n, np.uint8)
    ocrc = np.zeros(S * e * nwin, np.uint32)
    mism = np.zeros(S, np.int32)
    keep = []
    if pinned:
        pb, po, pc, pe, pm = (host_alloc(x.nbytes) for x in (buf, out, ocrc, stored, mism))
        pb.array[:] = buf
        pe.array[:] = stored.view(np.uint8)
        keep += [pb, po, pc, pe, pm]
        v = pb.array.reshape(S, k + p, us)
        out, ocrc, stored, mism = po.array, pc.array.view(np.uint32), pe.array.view(np.uint32), pm.array.view(np.int32)
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p, codec))
    dec.reconstruct_crc_host_batch(v.reshape(-1), (k + p) * us, us, present, erased, out, e * n, n, S, n, ctype, bpc,
                                   ocrc, h_expected=stored, h_mismatch=mism, stripes_per_chunk=chunk)
    got = out.reshape(S, e, n)
    oc = ocrc.reshape(S, e, nwin)
    st = stored.reshape(S, k + p, nwin)
    assert mism[2] == read[-1] * nwin + 2 and all(mism[s] == -1 for s in range(S) if s != 2), list(mism)
    for s in range(S):
        for i, u in enumerate(erased):
            if s != 2:  # stripe 2's rebuilt units are decoded from the corrupted input
                assert (got[s, i] == orig[s, u]).all(), (s, u)
                assert (oc[s, i] == st[s, u]).all(), (s, u)
            assert (oc[s, i] == oracle.crc_windows(otype, got[s, i], bpc)).all(), (s, u)


def test_reconstruct_host_batch_errors():
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(6, 3))
    buf = np.zeros(9 * 4096, np.uint8)
    out = np.zeros(4096, np.uint8)
    crc = np.zeros(1, np.uint32)
    with pytest.raises(rc.IllegalArgumentException):  # output array too small for the layout
        dec.reconstruct_crc_host_batch(buf, 9 * 4096, 4096, list(range(1, 9)), [0], np.zeros(100, np.uint8), 4096,
                                       4096, 1, 4096, ck.ChecksumType.CRC32C, 4096, crc)
    with pytest.raises(rc.IllegalArgumentException):  # verification without a mismatch buffer
        dec.reconstruct_crc_host_batch(buf, 9 * 4096, 4096, list(range(1, 9)), [0], out, 4096, 4096, 1, 4096,
                                       ck.ChecksumType.CRC32C, 4096, crc, h_expected=np.zeros(9, np.uint32))
    with pytest.raises(rc.IllegalArgumentException):  # too many erased
        dec.reconstruct_crc_host_batch(buf, 9 * 4096, 4096, [4, 5, 6, 7, 8, 3], [0, 1, 2, 3], np.zeros(4 * 4096, np.uint8),
                                       4 * 4096, 4096, 1, 4096, ck.ChecksumType.CRC32C, 4096, np.zeros(4, np.uint32))


_REGISTERED_KEEP = []  # OZEC_TEST_KEEP_REGISTERED=1: the round 4-5 workaround, registered ranges mapped until exit


def test_pinned_memory_is_numa_local():
    """ozec_host_alloc places its pages on the GPU's NUMA node (mbind before the pinning touch)."""
    node = device_numa_node(0)
    pb = host_alloc(64 << 20)
    pb.array[::4096] = 1
    got = {page_node(pb.array.ctypes.data + off) for off in (0, 32 << 20, (64 << 20) - 1)}
    if node < 0:
        pytest.skip("host reports no NUMA node for the GPU")
    assert got == {node}, (node, got)
    pb.free()
    # ozec_host_register places a caller's (untouched) mapping the same way and pins it
    mm = mmap.mmap(-1, 16 << 20)
    anchor = ctypes.c_char.from_buffer(mm)
    addr = ctypes.addressof(anchor)
    host_register(addr, 16 << 20, 0)
    assert page_node(addr) == node and page_node(addr + (16 << 20) - 1) == node
    host_unregister(addr)
    if os.environ.get("OZEC_TEST_KEEP_REGISTERED") == "1":
        _REGISTERED_KEEP.append((mm, anchor))
    else:
        del anchor
        mm.close()  # unmapped after the unregistration, as a caller would


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank(rank, world, port, path, S, n, bpc, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)  # both "GPUs" are device 0 here
        from ozone_amd import checksum as ck_
        from ozone_amd import rawcoder as rc_
        k, p = 6, 3
        sb = (k + p) * n
        total = os.path.getsize(path)
        fd = os.open(path, os.O_RDWR)
        mm = mmap.mmap(fd, total, mmap.MAP_SHARED)
        os.close(fd)
        anchor = ctypes.c_char.from_buffer(mm)
        base = ctypes.addressof(anchor)
        lo, hi = stripe_range(S, rank, world)
        nwin = n // bpc
        crc_off = S * sb
        host_register(base + lo * sb, (hi - lo) * sb, 0)
        e = rc_.RawErasureEncoder(rc_.ECReplicationConfig(k, p))
        e.encode_crc_host_batch(base + lo * sb, sb, n, base + lo * sb + k * n, sb, n, hi - lo, n,
                                ck_.ChecksumType.CRC32C, bpc, base + crc_off + lo * (k + p) * nwin * 4, False, 2)
        host_unregister(base + lo * sb)
        dist.barrier()
        dist.destroy_process_group()
        del anchor
        mm.close()
        q.put((rank, "ok"))
    except Exception as ex:  # pragma: no cover - reported to the parent
        q.put((rank, repr(ex)))


def test_two_ranks_split_one_host_batch_on_one_device():
    """Two rank processes (gloo) each take their contiguous stripe range of ONE shared host batch, register it and
    run ozec_encode_crc_host_batch on the same GPU; the union is bit-exact against the oracle.  This is the N > 1
    partition of bench.py's C5 leg (ranks own disjoint ranges, no collective on the data path)."""
    import torch.multiprocessing as mp
    S, n, bpc, k, p = 9, 1 << 16, 16384, 6, 3
    nwin = n // bpc
    buf, v, us = _batch(S, k, p, n, 820000)
    # shared memory (tmpfs), as bench.py's batch: long-term pinning of file-backed pages is refused by the kernel
    path = f"/dev/shm/ozec_test_batch_{os.getpid()}"
    with open(path, "wb") as f:
        f.write(buf.tobytes())
        f.write(np.zeros(S * (k + p) * nwin, np.uint32).tobytes())
    try:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_rank, args=(r, 2, port, path, S, n, bpc, q)) for r in range(2)]
        for pr in procs:
            pr.start()
        res = dict(q.get(timeout=120) for _ in range(2))
        for pr in procs:
            pr.join(timeout=60)
        assert res == {0: "ok", 1: "ok"}, res
        raw = np.fromfile(path, np.uint8)
    finally:
        os.unlink(path)
    v = raw[:S * (k + p) * n].reshape(S, k + p, n)
    crcs = raw[S * (k + p) * n:].view(np.uint32)
    _check(v, crcs, "rs", k, p, n, S, ck.ChecksumType.CRC32C, bpc)


def test_per_call_counters_on_the_gpu_paths():
    from ozone_amd import _lib
    _lib.stats_reset()
    k, p, n, S = 6, 3, 1 << 16, 5
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    d = cells(SEED, 830000, k, n)
    out = [np.zeros(n, np.uint8) for _ in range(p)]
    for _ in range(3):
        e.encode(d, out)
    buf, v, us = _batch(S, k, p, n, 831000)
    crcs = np.zeros(S * (k + p) * (n // 16384), np.uint32)
    e.encode_crc_host_batch(v.ctypes.data, (k + p) * us, us, v.ctypes.data + k * us, (k + p) * us, us, S, n,
                            ck.ChecksumType.CRC32C, 16384, crcs, False, 2)
    st = _lib.stats()
    assert st["encode"]["calls"] == 3 and st["encode"]["bytes"] == 3 * k * n and st["encode"]["errors"] == 0
    # the e2e batch counts once, as a host batch, not again for the fused launches it makes
    assert st["host_batch"]["calls"] == 1 and st["host_batch"]["bytes"] == S * k * n
    assert st["fused"]["calls"] == 0


# ------------------------------------------------------------------------------ several GPUs in one process (N2)


@pytest.fixture
def device_list():
    """ozec_set_devices for the test, the default list restored afterwards."""
    yield rc.set_devices
    rc.set_devices(None)


@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0]])
def test_host_batches_split_over_the_device_list(device_list, devs):
    """one process drives every GPU of its list.  On the one-GPU box the list [0, 0] ([0, 0, 0])
    stands for two (three) GPUs: a host batch is cut into that many stripe ranges, each run by its own pipeline thread
    on its listed device, and the union equals the oracle -- encode + CRC (pinned and pageable) and the fused
    reconstruction with a corrupted window reported for its own stripe.  Coders take the listed devices in turn."""
    device_list(devs)
    assert rc.get_devices() == devs
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(6, 3))
    assert e.device == 0
    k, p, n, S, chunk, bpc = 6, 3, 1 << 16, 23, 4, 16384
    for pinned in (True, False):
        buf, v, us = _batch(S, k, p, n, 890000 + 100 * len(devs) + pinned)
        crcs = np.zeros(S * (k + p) * (n // bpc), np.uint32)
        keep = []
        if pinned:
            pb, pc = host_alloc(buf.nbytes), host_alloc(crcs.nbytes)
            pb.array[:] = buf
            keep += [pb, pc]
            v, crcs = pb.array.reshape(S, k + p, us), pc.array.view(np.uint32)
        base = v.ctypes.data
        e.encode_crc_host_batch(base, (k + p) * us, us, base + k * us, (k + p) * us, us, S, n, ck.ChecksumType.CRC32C,
                                bpc, crcs, False, chunk)
        _check(v, crcs, "rs", k, p, n, S, ck.ChecksumType.CRC32C, bpc)
    # reconstruction, split the same way
    k, p, erased = 10, 4, [1, 4, 10, 13]
    buf, v, us = _recon_batch("rs", k, p, n, S, 895000, 0)
    nwin = n // bpc
    stored = np.stack([np.stack([oracle.crc_windows(oracle.CRC32C, np.array(v[s, u, :n]), bpc) for u in range(k + p)])
                       for s in range(S)]).astype(np.uint32).reshape(-1)
    present = [u for u in range(k + p) if u not in erased]
    orig = np.array(v[:, :, :n])
    bad = S - 2  # a stripe of the last part
    v[bad, present[0], 7] ^= 0x40
    out = np.zeros(S * 4 * n, np.uint8)
    ocrc = np.zeros(S * 4 * nwin, np.uint32)
    mism = np.zeros(S, np.int32)
    dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
    dec.reconstruct_crc_host_batch(v.reshape(-1), (k + p) * us, us, present, erased, out, 4 * n, n, S, n,
                                   ck.ChecksumType.CRC32C, bpc, ocrc, h_expected=stored, h_mismatch=mism,
                                   stripes_per_chunk=chunk)
    assert mism[bad] == present[0] * nwin and all(mism[s] == -1 for s in range(S) if s != bad), list(mism)
    got, oc, st = out.reshape(S, 4, n), ocrc.reshape(S, 4, nwin), stored.reshape(S, k + p, nwin)
    for s in range(S):
        if s == bad:
            continue
        for i, u in enumerate(erased):
            assert (got[s, i] == orig[s, u]).all() and (oc[s, i] == st[s, u]).all(), (s, u)


def test_device_list_errors_and_default(device_list):
    n = rc.device_count()
    with pytest.raises(RuntimeError):  # no such device (OZEC_EDEVICE)
        rc.set_devices([n])
    device_list([0])
    assert rc.get_devices() == [0]
    rc.set_devices(None)
    assert rc.get_devices() == list(range(n)) or os.environ.get("OZEC_DEVICES")
    for name in ("round_robin", "numa", "current"):
        rc.set_device_policy(name)
        assert rc.RawErasureEncoder(rc.ECReplicationConfig(3, 2)).device in range(n)
    rc.set_device_policy("round_robin")


@pytest.mark.parametrize("n", [1007, 50001, 700001])
@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("pitch16", [0, 1])
def test_host_batches_of_odd_cells_vs_oracle(n, pinned, pitch16):
    """A key's last, partial stripe has cells of any length (parityCellSize = dataBuffers[0].position(),
    ECKeyOutputStream.java:276).  The host batches lay such cells out on the device at a unit pitch of the length
    (units at odd offsets: the kernels take any byte offset) or, with host_pitch16 = 1, of the length rounded up to
    16 B (capi.cpp dunit); contiguous odd cells (unit stride = length) and a gapped layout, encode + CRC32C and the
    fused reconstruction, vs the oracle."""
    lib = L.lib()
    assert lib.ozec_set_tuning(b"host_pitch16", pitch16) == 0
    try:
        _odd_host_batches(n, pinned)
    finally:
        lib.ozec_set_tuning(b"host_pitch16", 0)


def _odd_host_batches(n, pinned):
    k, p, S, bpc = 6, 3, 5, 16384
    for gap in (0, 3):
        buf, v, us = _batch(S, k, p, n, 4100 + n % 97 + gap, gap)
        keep = None
        if pinned:
            keep = host_alloc(buf.nbytes)
            keep.array[:] = buf
            buf = keep.array
            v = buf.reshape(S, k + p, us)
        nwin = -(-n // bpc)
        crcs = np.zeros(S * (k + p) * nwin, np.uint32)
        enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
        enc.encode_crc_host_batch(buf.ctypes.data, (k + p) * us, us, buf.ctypes.data + k * us, (k + p) * us, us, S, n,
                                  ck.ChecksumType.CRC32C, bpc, crcs, False, 2)
        _check(v, crcs, "rs", k, p, n, S, ck.ChecksumType.CRC32C, bpc)
        erased = [0, 4, 7]
        present = [u for u in range(k + p) if u not in erased]
        stored = crcs.reshape(S, k + p, nwin).copy()
        truth = [[np.array(v[s, u, :n]) for u in erased] for s in range(S)]
        out = np.zeros(S * 3 * n, np.uint8)
        ocrc = np.zeros(S * 3 * nwin, np.uint32)
        mism = np.zeros(S, np.int32)
        dec = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
        dec.reconstruct_crc_host_batch(buf, (k + p) * us, us, present, erased, out, 3 * n, n, S, n,
                                       ck.ChecksumType.CRC32C, bpc, ocrc, h_expected=stored.reshape(-1),
                                       h_mismatch=mism, stripes_per_chunk=2)
        got, oc = out.reshape(S, 3, n), ocrc.reshape(S, 3, nwin)
        assert (mism == -1).all(), (n, pinned, gap)
        for s in range(S):
            for q, u in enumerate(erased):
                assert (got[s, q] == truth[s][q]).all() and (oc[s, q] == stored[s, u]).all(), (n, pinned, gap, s, u)
        if keep is not None:
            del v, buf
            keep.free()
