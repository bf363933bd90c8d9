"""Diagnostic: templated coding kernels across grid-stride iterations vs the oracle."""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, "tests/golden")
import numpy as np, torch
import oracle
from ozone_amd import rawcoder as rc
from synth import cells
torch.cuda.set_device(0)
n = 1 << 16
for (k, p, S) in [(6, 3, 64), (10, 4, 64), (10, 2, 64), (10, 1, 64), (3, 2, 200), (10, 4, 2200)]:
    data = torch.empty((S, k, n), dtype=torch.uint8, device="cuda")
    rc.fill_splitmix64_cells(data, n, S * k, n, 7, 0)
    e = rc.RawErasureEncoder(rc.ECReplicationConfig(k, p))
    par = e.encode_stripes(data)
    torch.cuda.synchronize()
    dh = data.cpu().numpy(); ph = par.cpu().numpy()
    bad = []
    for s in list(range(min(S, 40))) + [S - 1]:
        ref = oracle.rs_encode(k, p, list(dh[s]))
        for r in range(p):
            if not (ph[s, r] == ref[r]).all():
                idx = np.nonzero(ph[s, r] != ref[r])[0]
                bad.append((s, r, int(idx[0]), len(idx)))
    print(k, p, S, "bad:", bad[:10], len(bad), flush=True)
