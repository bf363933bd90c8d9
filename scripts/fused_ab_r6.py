"""Same-process A/B of the round-6 fused forms against the unfused route they replace:
  WIDE  units 768 MiB apart (a stripe spans > 2 GiB): rs-6-3 and xor-2-1 encode + CRC32C, rs-10-4 reconstruction of 4
        erased units + CRC32C; aligned and at an odd base
  TAIL  XOR encode + CRC32C of packed cells whose length is not a multiple of 16 B (xor-2-1, xor-6-1, xor-10-1)
Per case the route is forced through libozec's own routing knobs (fused: fused_min_units = rec_min_units = 0;
unfused: both 2^62), checked with ozec_fused_routes, the outputs of the two routes compared byte for byte, and the
call timed with HIP events on the launch stream (median of 5 rounds of 10 calls, the routes interleaved).  One JSON
line per case.  `full`: the WIDE form against the compact layout at a full 1,024-stripe batch instead.
usage: python scripts/fused_ab_r6.py [full]"""
import ctypes
import json
import os
import statistics
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from ozone_amd import _lib as L  # noqa: E402
from ozone_amd import checksum as ck  # noqa: E402
from ozone_amd import rawcoder as rc  # noqa: E402

torch.cuda.set_device(0)
lib = L.lib()
US = 768 << 20
BPC = 16384


def routes():
    f, u = ctypes.c_uint64(), ctypes.c_uint64()
    assert lib.ozec_fused_routes(ctypes.byref(f), ctypes.byref(u)) == 0
    return f.value, u.value


def set_route(fused):
    v = 0 if fused else 1 << 62
    for key in (b"fused_min_units", b"rec_min_units"):
        assert lib.ozec_set_tuning(key, v) == 0


def timed(call, reps=10):
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        call()
    b.record(st)
    b.synchronize()
    return a.elapsed_time(b) / reps


def ab(name, call, outputs, moved, extra):
    res = {}
    snaps = {}
    for fused in (True, False):
        set_route(fused)
        r0 = routes()
        for o in outputs:
            o.zero_()
        call()
        torch.cuda.synchronize()
        r1 = routes()
        took = "fused" if r1[0] > r0[0] else "unfused" if r1[1] > r0[1] else "none"
        assert took == ("fused" if fused else "unfused"), (name, fused, r0, r1)
        snaps[fused] = [o.clone() for o in outputs]
    same = all(torch.equal(x, y) for x, y in zip(snaps[True], snaps[False]))
    del snaps
    times = {True: [], False: []}
    for _ in range(5):
        for fused in (True, False):
            set_route(fused)
            times[fused].append(timed(call))
    for fused in (True, False):
        ms = statistics.median(times[fused])
        res["fused" if fused else "unfused"] = {"ms": round(ms, 4), "GB/s": round(moved / ms / 1e6, 1)}
    res.update(extra)
    res.update({"case": name, "outputs_identical": same,
                "speedup": round(res["unfused"]["ms"] / res["fused"]["ms"], 3)})
    print(json.dumps(res), flush=True)
    set_route(True)


def wide_cases():
    n, S = 1 << 20, 64
    ss = n
    for mode, codec, k, p in (("encode", "rs", 6, 3), ("encode", "xor", 2, 1), ("reconstruct", "rs", 10, 4)):
        for shift in (0, 3):
            units = k + p
            buf = torch.empty(shift + (units - 1) * US + S * ss + 64, dtype=torch.uint8, device="cuda")
            base = buf[shift:]
            for u in range(units):
                base[u * US:u * US + S * ss].random_(0, 256)
            conf = rc.ECReplicationConfig(k, p, codec)
            nwin = -(-n // BPC)
            if mode == "encode":
                enc = rc.RawErasureEncoder(conf)
                crcs = torch.zeros((S, k + p, nwin), dtype=torch.int32, device="cuda")

                def call(enc=enc, base=base, crcs=crcs, k=k):
                    enc.encode_crc_batch(base, ss, US, base[k * US:], ss, US, S, n, ck.ChecksumType.CRC32C, BPC, crcs)
                outs = [crcs]  # the parity lands in the pool itself, rewritten identically by both routes
                moved = (k + p) * n * S + (k + p) * nwin * 4 * S
            else:
                dec = rc.RawErasureDecoder(conf)
                erased = [0, 1, 2, 3]
                present = [u for u in range(units) if u not in erased][:k]
                out = torch.empty((S, len(erased), n), dtype=torch.uint8, device="cuda")
                ocrc = torch.zeros((S, len(erased), nwin), dtype=torch.int32, device="cuda")

                def call(dec=dec, base=base, present=present, erased=erased, out=out, ocrc=ocrc):
                    dec.reconstruct_crc_batch(base, ss, US, present, erased, out, len(erased) * n, n, S, n,
                                              ck.ChecksumType.CRC32C, BPC, ocrc)
                outs = [out, ocrc]
                moved = (k + len(erased)) * n * S + len(erased) * nwin * 4 * S
            ab(f"WIDE {mode} {codec}-{k}-{p}", call, outs, moved,
               {"offset": shift, "unit_stride": US, "stripes": S, "cell": n})
            del buf, base
            torch.cuda.empty_cache()


def tail_cases():
    S = 512
    for k in (2, 6, 10):
        for n in (1 << 20, (1 << 20) + 5, 700001):
            conf = rc.ECReplicationConfig(k, 1, "xor")
            enc = rc.RawErasureEncoder(conf)
            ss = (k + 1) * n  # packed: stripes back to back, units back to back (odd offsets when n is odd)
            buf = torch.empty(S * ss + 64, dtype=torch.uint8, device="cuda").random_(0, 256)
            nwin = -(-n // BPC)
            crcs = torch.zeros((S, k + 1, nwin), dtype=torch.int32, device="cuda")

            def call(enc=enc, buf=buf, crcs=crcs, k=k, n=n, ss=ss):
                enc.encode_crc_batch(buf, ss, n, buf[k * n:], ss, n, S, n, ck.ChecksumType.CRC32C, BPC, crcs)
            moved = (k + 1) * n * S + (k + 1) * nwin * 4 * S
            ab(f"TAIL encode xor-{k}-1", call, [crcs], moved, {"cell": n, "stripes": S, "packed": True})
            del buf
            torch.cuda.empty_cache()


def wide_vs_compact(S=1024):
    """The WIDE form's own cost at a full batch: rs-6-3 encode + CRC32C of S stripes of 1 MiB cells with units 1.25 GiB
    apart (WIDE: one buffer descriptor per unit) against the same stripes with units 1 MiB apart inside each stripe
    (the C5dev layout), both on the fused route, median of 5 rounds of 10 calls, routes interleaved."""
    k, p, n = 6, 3, 1 << 20
    set_route(True)
    us_wide = (5 << 30) // 4
    nwin = n // BPC
    res = {}
    for name, unit_stride, stripe_stride, span in (("wide", us_wide, n, (k + p - 1) * us_wide + S * n),
                                                   ("compact", n, (k + p) * n, S * (k + p) * n)):
        buf = torch.empty(span + 64, dtype=torch.uint8, device="cuda")
        buf.random_(0, 256)
        enc = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
        crcs = torch.zeros((S, k + p, nwin), dtype=torch.int32, device="cuda")

        def call(enc=enc, buf=buf, crcs=crcs, us=unit_stride, ss=stripe_stride):
            enc.encode_crc_batch(buf, ss, us, buf[k * us:], ss, us, S, n, ck.ChecksumType.CRC32C, BPC, crcs)
        r0 = routes()
        call()
        torch.cuda.synchronize()
        assert routes()[0] > r0[0], name
        res[name] = (call, buf, crcs)
    times = {"wide": [], "compact": []}
    for _ in range(5):
        for name in ("wide", "compact"):
            times[name].append(timed(res[name][0]))
    moved = S * ((k + p) * n + (k + p) * nwin * 4)
    out = {"case": f"WIDE vs compact, rs-6-3 encode + CRC32C, {S} stripes of 1 MiB, fused"}
    for name in ("wide", "compact"):
        ms = statistics.median(times[name])
        out[name] = {"ms": round(ms, 4), "frac_of_8TBps": round(moved / (ms * 1e-3) / 8e12, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "full":
        wide_vs_compact()
    else:
        wide_cases()
        tail_cases()
