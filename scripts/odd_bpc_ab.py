"""CRC32C of windows whose length is not a multiple of 16 B (bytes.per.checksum of any value >= 8 KiB is legal,
OzoneClientConfig.java:284-290) and of cells at odd offsets, for the library given by OZEC_LIB_OVERRIDE (or the
in-tree one): ozec_checksum_windows_batch over 1 GiB of cells, HIP-event timed, one JSON line per case.  Run once
per library to compare the round-5 per-window kernel with the byte-at-a-time kernel it replaced.
usage: python scripts/odd_bpc_ab.py [TAG]"""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from ozone_amd import checksum as ck  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "cur"
torch.cuda.set_device(0)
n = 1 << 20
for bpc, shift in ((10000, 0), (10001, 0), (8200, 0), (16384, 3), (16384, 0)):
    cells = 1024
    buf = torch.randint(0, 256, (cells * n + 64,), dtype=torch.uint8, device="cuda")
    base = buf[shift:]
    nwin = -(-n // bpc)
    out = torch.empty((cells, nwin), dtype=torch.int32, device="cuda")

    def call():
        ck.checksum_windows_batch(ck.ChecksumType.CRC32C, base, n, cells, n, bpc, out)
    for _ in range(2):
        call()
    torch.cuda.synchronize()
    reps = 5
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(reps):
        call()
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / reps
    print(json.dumps({"lib": tag, "bpc": bpc, "offset": shift, "bytes": cells * n, "ms": round(ms, 3),
                      "GB/s": round(cells * n / ms / 1e6, 1)}), flush=True)
    del buf, out
