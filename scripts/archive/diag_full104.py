import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, "tests/golden")
import numpy as np, torch
import oracle
from ozone_amd import rawcoder as rc
torch.cuda.set_device(0)
k, p, n, S = 10, 4, 1 << 20, int(sys.argv[1]) if len(sys.argv) > 1 else 2048
SEED = 0x00EC5EED
units = torch.empty((S, k + p, n), dtype=torch.uint8, device="cuda")
for u in range(k):
    rc.fill_splitmix64_cells(units[:, u], (k + p) * n, S, n, SEED, 200000 * (u + 1))
rc.RawErasureEncoder(rc.ECReplicationConfig(k, p)).encode_batch(units, (k + p) * n, n, units[:, k:], (k + p) * n, n, S, n)
torch.cuda.synchronize()
for s in [0, 1, 100, S // 2, S - 1]:
    h = units[s].cpu().numpy()
    ref = oracle.rs_encode(k, p, list(h[:k]))
    print("enc stripe", s, [bool((h[k + r] == ref[r]).all()) for r in range(p)], flush=True)
d = rc.RawErasureDecoder(rc.ECReplicationConfig(k, p))
out = torch.empty((S, 4, n), dtype=torch.uint8, device="cuda")
erased = [0, 1, 2, 3]
present = [u for u in range(k + p) if u not in erased]
d.decode_batch(units, (k + p) * n, n, present, erased, out, 4 * n, n, S, n)
torch.cuda.synchronize()
for i, u in enumerate(erased):
    eq = (out[:, i] == units[:, u]).all(dim=1).cpu().numpy()
    bad = np.nonzero(~eq)[0]
    print("dec unit", u, "bad stripes", len(bad), bad[:10], flush=True)
    if len(bad):
        s = int(bad[0])
        diff = (out[s, i] != units[s, u]).cpu().numpy()
        idx = np.nonzero(diff)[0]
        print("  stripe", s, "nbad bytes", len(idx), "first", idx[:8], flush=True)
