"""Deterministic synthetic cell data: splitmix64 byte streams.

The same generator runs on the GPU (ozec_fill_splitmix64 in the product library, used by bench.py to
fill HBM) and here (numpy), so tests can regenerate any fixture input from (seed, stream, length).
Each 64-bit output is emitted little-endian; stream `s` of seed `seed` starts from state
seed ^ (s * 0x9E3779B97F4A7C15)  -- one disjoint stream per cell, as SURVEY.md §8(d) asks.
"""
import numpy as np

GOLDEN = 0x9E3779B97F4A7C15
SEED = 0x00EC5EED
_M64 = (1 << 64) - 1


def splitmix64_bytes(seed: int, stream: int, n: int) -> np.ndarray:
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        state0 = np.uint64((seed ^ ((stream * GOLDEN) & _M64)) & _M64)
        idx = np.arange(1, words + 1, dtype=np.uint64)
        z = state0 + idx * np.uint64(GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def cells(seed: int, first_stream: int, count: int, n: int):
    return [splitmix64_bytes(seed, first_stream + i, n) for i in range(count)]
