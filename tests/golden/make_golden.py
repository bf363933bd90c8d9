#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run from the repo root, CPU only).

  python tests/golden/make_golden.py            # regenerate *.json
  python tests/golden/make_golden.py --check    # regenerate in memory and diff against the committed files

What pins what (the reference is Java and cannot run here: no JDK):
  ref_pins.json   -- sha256 of the literal tables in the reference sources, read as TEXT when
                     /root/reference is mounted: GF256.java GF_BASE/GF_LOG_BASE (GF256.java:31-139) and the
                     2048-entry T tables of PureJavaCrc32ByteBuffer.java / PureJavaCrc32CByteBuffer.java.
                     Only hashes and a match flag are stored -- no reference source text is copied.
                     The C oracle's generated tables must hash to these values (tests/test_oracle_golden.py).
  ec_vectors.json -- encode/decode vectors produced by the independent pure-Python restatement
                     (pyref.py) on splitmix64 inputs (synth.py); the C oracle and the HIP path must match.
  crc_vectors.json-- CRC32/CRC32C window vectors from pyref.py (bit-/table-wise definition, zlib cross-check).
Erasure patterns follow TestRSRawCoderBase.java:33-115 / TestXORRawCoderBase.java:33-55, chunk lengths follow
TestRawCoderBase.java:84-86 (1024, 1024-17, 1024+16) plus the odd/edge sizes of SURVEY.md §7.
"""
import hashlib
import json
import os
import re
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import pyref  # noqa: E402
from synth import SEED, cells  # noqa: E402

REF = "/root/reference"
GF_JAVA = "hadoop-hdds/erasurecode/src/main/java/org/apache/ozone/erasurecode/rawcoder/util/GF256.java"
CRC32_JAVA = "hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/PureJavaCrc32ByteBuffer.java"
CRC32C_JAVA = "hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/PureJavaCrc32CByteBuffer.java"

INLINE_MAX = 1040  # store bytes inline (hex) up to this length, sha256 above


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint8).tobytes()).hexdigest()


def blob(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a.tobytes().hex() if a.size <= INLINE_MAX else "sha256:" + sha(a)


def _java_byte_array(text, name):
    body = re.search(name + r"\s*=\s*new byte\[\]\s*\{(.*?)\};", text, re.S).group(1)
    return np.array([int(h, 16) for h in re.findall(r"0x([0-9a-fA-F]{2})", body)], np.uint8)


def _java_int_table(text):
    body = re.search(r"int\[\]\s+T\s*=\s*\{(.*?)\};", text, re.S).group(1)
    vals = [int(h, 16) for h in re.findall(r"0x([0-9a-fA-F]{8})", body)]
    return np.array(vals, np.uint32)


def ref_pins():
    """Hash the reference's literal tables; cross-check them against our generated tables."""
    import oracle
    gf_text = open(os.path.join(REF, GF_JAVA)).read()
    base = _java_byte_array(gf_text, "GF_BASE")
    logb = _java_byte_array(gf_text, "GF_LOG_BASE")
    obase, olog = oracle.gf_tables()
    pins = {
        "source": "z-bb/ozone @ 2024-10-08 (/root/reference), literal tables read as text",
        "gf_base": {"file": GF_JAVA + ":31-84", "n": int(base.size), "sha256": sha(base),
                    "oracle_match": bool((base == obase).all())},
        "gf_log_base": {"file": GF_JAVA + ":86-139", "n": int(logb.size), "sha256": sha(logb),
                        "oracle_match": bool((logb == olog).all())},
    }
    # the field product implied by the reference tables == pyref's shift-and-add product (all 65,536 pairs)
    def mul_tab(a, b):
        if a == 0 or b == 0:
            return 0
        t = int(logb[a]) + int(logb[b])
        return int(base[t - 255 if t > 254 else t])
    ref_mul = np.array([[mul_tab(a, b) for b in range(256)] for a in range(256)], np.uint8)
    pins["gf_mul_table_matches_bitwise"] = bool((ref_mul == pyref.MUL).all())
    for key, path, ctype in (("crc32", CRC32_JAVA, 0), ("crc32c", CRC32C_JAVA, 1)):
        t = _java_int_table(open(os.path.join(REF, path)).read())
        ot = oracle.crc_table(ctype)
        pins[key + "_table"] = {"file": path, "n": int(t.size),
                                "sha256": hashlib.sha256(t.astype("<u4").tobytes()).hexdigest(),
                                "oracle_match": bool(t.size == ot.size and (t == ot).all())}
    return pins


def erasure_sets(k, p, data_idx, parity_idx):
    """TestCoderBase.getErasedIndexesForDecoding (TestCoderBase.java:172-187): data first, then k+parity."""
    return list(data_idx) + [k + i for i in parity_idx]


def present_units(k, p, erased):
    """Inputs left after erasing, then TestRawCoderBase.ensureOnlyLeastRequiredChunks
    (TestRawCoderBase.java:243-254) nulls the first redundant non-null inputs."""
    alive = [u for u in range(k + p) if u not in erased]
    return alive[len(alive) - k:]


def ec_vectors():
    cases = []
    stream = 0
    configs = [("rs", 3, 2), ("rs", 6, 3), ("rs", 10, 4), ("xor", 2, 1), ("xor", 4, 1)]
    lengths = [1, 7, 16, 1007, 1024, 1040, 4096 + 48, 16384 + 3, 1 << 20]
    for codec, k, p in configs:
        for n in lengths:
            data = cells(SEED, stream, k, n)
            par = pyref.rs_encode(k, p, data) if codec == "rs" else [pyref.xor_encode(data)]
            cases.append({"op": "encode", "codec": codec, "k": k, "p": p, "len": n, "seed": SEED,
                          "first_stream": stream, "parity": [blob(x) for x in par]})
            stream += k
    # decode: every pattern of TestRSRawCoderBase (rs-6-3 / rs-10-4) and every recoverable rs-3-2 set
    pats = [(6, 3, [0, 1, 2], []), (6, 3, [0, 2], []), (6, 3, [0], []), (6, 3, [2], []),
            (6, 3, [0], [0]), (6, 3, [], [0, 1, 2]), (6, 3, [], [0]), (6, 3, [], [2]),
            (6, 3, [], [0, 2]), (6, 3, [0], [0, 1]), (6, 3, [0, 2], [2]), (6, 3, [2, 4], []),
            (10, 4, [0], [0]), (10, 4, [0, 1, 2, 3], []), (10, 4, [1, 4], [0, 3])]
    import itertools
    for e in range(1, 3):
        for comb in itertools.combinations(range(5), e):
            pats.append((3, 2, [c for c in comb if c < 3], [c - 3 for c in comb if c >= 3]))
    for k, p, de, pe in pats:
        erased = erasure_sets(k, p, de, pe)
        for n in (1007, 1040, 16384 + 3):
            data = cells(SEED, stream, k, n)
            stream += k
            units = data + pyref.rs_encode(k, p, data)
            present = present_units(k, p, erased)
            inputs = [units[u] if u in present else None for u in range(k + p)]
            rows = pyref.decode_matrix(k, p, present, erased)
            out = pyref.rs_decode(k, p, inputs, erased)
            for e_idx, o in zip(erased, out):
                assert (o == units[e_idx]).all(), (k, p, erased)
            cases.append({"op": "decode", "codec": "rs", "k": k, "p": p, "len": n, "seed": SEED,
                          "first_stream": stream - k, "erased": erased, "present": present,
                          "decode_matrix": [bytes(r).hex() for r in rows],
                          "outputs": [blob(x) for x in out]})
    # the reference's erased-order quirk: parity listed before data -> zero output
    k, p, erased, n = 6, 3, [7, 0], 1024
    data = cells(SEED, stream, k, n)
    stream += k
    units = data + pyref.rs_encode(k, p, data)
    present = present_units(k, p, erased)
    inputs = [units[u] if u in present else None for u in range(k + p)]
    out = pyref.rs_decode(k, p, inputs, erased)
    assert not out[0].any() and (out[1] == units[0]).all()
    cases.append({"op": "decode", "codec": "rs", "k": k, "p": p, "len": n, "seed": SEED,
                  "first_stream": stream - k, "erased": erased, "present": present,
                  "decode_matrix": [bytes(r).hex() for r in pyref.decode_matrix(k, p, present, erased)],
                  "outputs": [blob(x) for x in out], "note": "erased-order quirk: output 0 all zero"})
    # XOR decode (TestXORRawCoderBase.java:33-55): every single erasure of xor-2-1 / xor-4-1
    for k in (2, 4):
        for er in range(k + 1):
            for n in (1007, 1040):
                data = cells(SEED, stream, k, n)
                stream += k
                units = data + [pyref.xor_encode(data)]
                inputs = [None if u == er else units[u] for u in range(k + 1)]
                out = pyref.xor_decode(inputs, er)
                assert (out == units[er]).all()
                cases.append({"op": "decode", "codec": "xor", "k": k, "p": 1, "len": n, "seed": SEED,
                              "first_stream": stream - k, "erased": [er],
                              "present": [u for u in range(k + 1) if u != er],
                              "outputs": [blob(out)]})
    return {"generator": "tests/golden/make_golden.py (pyref.py restatement)", "cases": cases}


def crc_vectors():
    out = {"check_123456789": {"crc32": pyref.crc_bitwise(0, b"123456789"),
                               "crc32c": pyref.crc_bitwise(1, b"123456789")},
           "cases": []}
    assert out["check_123456789"]["crc32"] == 0xCBF43926
    assert out["check_123456789"]["crc32c"] == 0xE3069283
    stream = 10_000
    specs = [(55, 10), (0, 16384), (1, 16384), (1000, 512), (4096, 1024), (65536 + 7, 2048),
             (1 << 18, 4096), (300000, 16384), (1 << 18, 32768), (1 << 20, 1 << 20), (1 << 20, 16384),
             (16384 * 3 + 5, 16384), (33, 32), (4095, 4096)]
    for n, bpc in specs:
        data = cells(SEED, stream, 1, n)[0]
        stream += 1
        for ctype, name in ((0, "crc32"), (1, "crc32c")):
            vals = pyref.crc_windows(ctype, data, bpc)
            if ctype == 0:  # independent implementation cross-check
                assert vals == [zlib.crc32(data[o:o + bpc].tobytes()) for o in range(0, n, bpc)]
            out["cases"].append({"type": name, "len": n, "bpc": bpc, "seed": SEED, "stream": stream - 1,
                                 "crcs": vals})
    return out


def main():
    files = {"ec_vectors.json": ec_vectors(), "crc_vectors.json": crc_vectors()}
    if os.path.isdir(REF):
        files["ref_pins.json"] = ref_pins()
    check = "--check" in sys.argv
    bad = 0
    for name, obj in files.items():
        path = os.path.join(HERE, name)
        text = json.dumps(obj, indent=1, sort_keys=True) + "\n"
        if check:
            same = os.path.exists(path) and open(path).read() == text
            print(f"{name}: {'OK' if same else 'DIFFERS'}")
            bad += not same
        else:
            with open(path, "w") as f:
                f.write(text)
            print(f"wrote {path} ({len(text)} bytes)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
