"""Helpers to read the committed golden fixtures (tests/golden/*.json)."""
import hashlib
import json
import os

import numpy as np

from synth import cells

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def matches(blob, arr):
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    if blob.startswith("sha256:"):
        return hashlib.sha256(arr.tobytes()).hexdigest() == blob[7:]
    return arr.tobytes().hex() == blob


def case_inputs(case):
    """Regenerate the data units of a golden case (k streams of splitmix64)."""
    return cells(case["seed"], case["first_stream"], case["k"], case["len"])


def ec_cases(op=None, max_len=None):
    out = []
    for c in load("ec_vectors.json")["cases"]:
        if op and c["op"] != op:
            continue
        if max_len and c["len"] > max_len:
            continue
        out.append(c)
    return out


def case_id(c):
    extra = f"-e{'_'.join(map(str, c['erased']))}" if c["op"] == "decode" else ""
    return f"{c['op']}-{c['codec']}{c['k']}-{c['p']}-n{c['len']}{extra}"
