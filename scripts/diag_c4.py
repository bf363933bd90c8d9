"""Fused XOR encode + CRC (C4 shapes) on the GPU, checked against torch's XOR of the inputs, repeated runs per
kernel variant: counts 16-KiB windows whose stored parity differs (diagnosed the 16-B store-data hazard that
kernels.hip store_data_hold guards against)."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
from ozone_amd import _lib as L
from ozone_amd import checksum as ck
from ozone_amd import rawcoder as rc
torch.cuda.set_device(0)
lib = L.lib()
n, bpc = 1 << 20, 16384
bad_total = 0
for S in (1024, 4096):
    X = torch.empty((S, 3, n), dtype=torch.uint8, device="cuda")
    for u in range(2):
        rc.fill_splitmix64_cells(X[:, u], 3 * n, S, n, 2, u * S)
    ref = torch.bitwise_xor(X[:, 0], X[:, 1])
    ex = rc.RawErasureEncoder(rc.ECReplicationConfig(2, 1, "xor"))
    crc_ref = None
    for v in [int(x) for x in os.environ.get("VARIANTS", "13,0,20").split(",")]:
        lib.ozec_set_tuning(b"crc_variant", v)
        for run in range(int(os.environ.get("RUNS", "3"))):
            X[:, 2].fill_(0x5A)
            c = torch.full((S, 3, n // bpc), 7, dtype=torch.int32, device="cuda")
            ex.encode_crc_batch(X, 3 * n, n, X[:, 2:], 3 * n, n, S, n, ck.ChecksumType.CRC32C, bpc, c)
            torch.cuda.synchronize()
            dp = (X[:, 2] != ref).view(S, n // bpc, bpc).any(dim=2)
            if crc_ref is None:
                crc_ref = c.clone()
            dc = int((c != crc_ref).sum())
            bad_total += int(dp.sum()) + dc
            print(f"S={S} variant={v} run={run}: parity windows wrong={int(dp.sum())} crc entries differing={dc}",
                  flush=True)
    lib.ozec_set_tuning(b"crc_variant", 0)
    del X, ref
    torch.cuda.empty_cache()
print("ALL EXACT" if bad_total == 0 else f"MISMATCHES {bad_total}")
sys.exit(0 if bad_total == 0 else 3)
