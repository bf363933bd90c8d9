"""Independent pure-Python restatement of the reference EC + CRC arithmetic (TEST INFRASTRUCTURE).

Written from the reference's published algorithm, deliberately NOT sharing code or table-building
strategy with oracle/ozec_oracle.c, so that the two restatements cross-check each other:
  * GF(2^8) products by shift-and-add (Russian peasant) modulo 0x11d, inverses by search -- the
    reference's GF256.gfMul/gfInv (GF256.java:164-184) compute exactly these field operations;
  * matrix inverse by Gauss-Jordan on Python lists (the inverse of an invertible matrix is unique, so it
    agrees with GF256.gfInvertMatrix, GF256.java:191-250, whenever that one succeeds);
  * decode-matrix rows follow RSRawDecoder.generateDecodeMatrix (RSRawDecoder.java:143-176) including the
    erased-parity-before-data quirk;
  * CRC by the bit-at-a-time reflected definition (init/xorout 0xFFFFFFFF), i.e. what
    ChecksumByteBuffer.CrcIntTable (ChecksumByteBuffer.java:51-121) computes with its slice-by-8 tables.
Used by make_golden.py to produce tests/golden/*.json.
"""
import numpy as np

POLY = 0x11D


def gf_mul(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= POLY
        b >>= 1
    return r


MUL = np.array([[gf_mul(a, b) for b in range(256)] for a in range(256)], dtype=np.uint8)
INV = [0] + [next(b for b in range(1, 256) if MUL[a, b] == 1) for a in range(1, 256)]


def cauchy(k: int, p: int):
    """RSUtil.genCauchyMatrix (RSUtil.java:64-77): identity on top, then 1/(i ^ j)."""
    m = [[1 if i == j else 0 for j in range(k)] for i in range(k)]
    for i in range(k, k + p):
        m.append([INV[i ^ j] for j in range(k)])
    return m


def invert(mat):
    n = len(mat)
    a = [row[:] + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(mat)]
    for col in range(n):
        piv = next((r for r in range(col, n) if a[r][col]), None)
        if piv is None:
            raise RuntimeError("Not invertible")
        a[col], a[piv] = a[piv], a[col]
        s = INV[a[col][col]]
        a[col] = [int(MUL[s, v]) for v in a[col]]
        for r in range(n):
            if r != col and a[r][col]:
                f = a[r][col]
                a[r] = [v ^ int(MUL[f, w]) for v, w in zip(a[r], a[col])]
    return [row[n:] for row in a]


def apply(matrix_rows, inputs):
    """out[l] = XOR_j rows[l][j] * inputs[j] over GF(2^8) -- RSUtil.encodeData semantics."""
    n = len(inputs[0])
    outs = []
    for row in matrix_rows:
        acc = np.zeros(n, np.uint8)
        for c, x in zip(row, inputs):
            acc ^= MUL[c][x]
        outs.append(acc)
    return outs


def rs_encode(k, p, data):
    return apply(cauchy(k, p)[k:], data)


def decode_matrix(k, p, valid, erased):
    """RSRawDecoder.generateDecodeMatrix (RSRawDecoder.java:143-176), row per erased slot."""
    enc = cauchy(k, p)
    inv = invert([enc[r] for r in valid[:k]])
    n_data_erased = sum(1 for e in erased if e < k)
    rows = []
    for i, e in enumerate(erased):
        if i < n_data_erased:
            # invertMatrix is (k+p) x k with a zero tail below row k (RSRawDecoder.java:119)
            rows.append(inv[e][:] if e < k else [0] * k)
        else:
            rows.append([
                int(np.bitwise_xor.reduce([MUL[inv[j][i2], enc[e][j]] for j in range(k)]))
                for i2 in range(k)
            ])
    return rows


def rs_decode(k, p, inputs, erased):
    valid = [i for i, x in enumerate(inputs) if x is not None]
    if len(valid) < k:
        raise ValueError("No enough valid inputs")
    rows = decode_matrix(k, p, valid, erased)
    return apply(rows, [inputs[v] for v in valid[:k]])


def xor_encode(data):
    acc = data[0].copy()
    for d in data[1:]:
        acc ^= d
    return acc


def xor_decode(inputs, erased0):
    acc = np.zeros(len(next(x for x in inputs if x is not None)), np.uint8)
    for i, x in enumerate(inputs):
        if i != erased0:
            acc ^= x
    return acc


CRC_POLYS = {0: 0xEDB88320, 1: 0x82F63B78}  # 0 = CRC32, 1 = CRC32C


def _byte_table(poly):
    t = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        t.append(c)
    return t


_TABLES = {k: _byte_table(v) for k, v in CRC_POLYS.items()}


def crc_bitwise(ctype, data: bytes) -> int:
    poly, c = CRC_POLYS[ctype], 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
    return c ^ 0xFFFFFFFF


def crc(ctype, data) -> int:
    t, c = _TABLES[ctype], 0xFFFFFFFF
    for b in bytes(data):
        c = (c >> 8) ^ t[(c ^ b) & 0xFF]
    return c ^ 0xFFFFFFFF


def crc_windows(ctype, data, bpc):
    data = bytes(data)
    return [crc(ctype, data[o:o + bpc]) for o in range(0, len(data), bpc)]
