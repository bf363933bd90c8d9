"""Host <-> device copies for the GPU tests through pinned staging (round 6, DESIGN §4 "GPU faults").

The tests never hand HIP a pageable host buffer to DMA: every recorded hipErrorIllegalAddress (rounds 4-5) surfaced in
a torch pageable copy (`.cpu()`, `.to("cuda")`) of a recurring size, which HIP performs by locking the caller's heap
pages for the transfer (ROCr hsa_amd_memory_lock_to_pool).  Here the bytes go through one pinned torch buffer
(hipHostMalloc memory from torch's caching host allocator, never returned to the OS while the process lives), so no
test transfer depends on a transient lock of memory that glibc may trim and hand out again.  `to_dev` / `to_host`
replace `torch.from_numpy(a).to(DEV)` / `x.cpu().numpy()` one for one and are synchronous.
"""
import numpy as np
import torch

DEV = "cuda:0"
_stage = None


def _pinned(nbytes):
    global _stage
    if _stage is None or _stage.numel() < nbytes:
        cap = max(nbytes, 8 << 20)
        _stage = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
    return _stage


def to_dev(a, dev=DEV):
    """numpy array -> new device tensor of the same dtype and shape, copied from pinned memory."""
    a = np.ascontiguousarray(a)
    dtype = torch.from_numpy(a[:0] if a.ndim else a.reshape(1)[:0]).dtype
    nb = a.nbytes
    d = torch.empty(nb, dtype=torch.uint8, device=dev)
    if nb:
        st = _pinned(nb)
        st[:nb].numpy()[:] = a.reshape(-1).view(np.uint8)
        d.copy_(st[:nb])
        torch.cuda.synchronize()
    return d.view(dtype).reshape(a.shape)


def to_host(x):
    """device tensor (any layout) -> numpy array (a copy) of the same dtype and shape, through pinned memory."""
    torch.cuda.synchronize()
    x = x.contiguous()
    npdt = torch.empty(0, dtype=x.dtype).numpy().dtype
    nb = x.numel() * x.element_size()
    if nb == 0:
        return np.empty(tuple(x.shape), npdt)
    st = _pinned(nb)
    st[:nb].copy_(x.reshape(-1).view(torch.uint8))
    torch.cuda.synchronize()
    return st[:nb].numpy().copy().view(npdt).reshape(tuple(x.shape))
