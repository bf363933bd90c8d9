"""Every global name a function of the GPU test modules, bench.py or the scripts reads is bound at module level or
a builtin (CPU test).  The GPU tests are skipped here, so a missing import in one of them would otherwise surface
only on the GPU box."""
import builtins
import glob
import os
import symtable

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = sorted(glob.glob(os.path.join(ROOT, "tests", "test_gpu*.py")) + [os.path.join(ROOT, "bench.py")] +
               glob.glob(os.path.join(ROOT, "scripts", "*.py")))


def _unbound_globals(path):
    src = open(path).read()
    top = symtable.symtable(src, path, "exec")
    bound = {s.get_name() for s in top.get_symbols() if s.is_assigned() or s.is_imported()}
    bound |= set(dir(builtins)) | {"__file__", "__name__", "__doc__"}
    missing = []

    def walk(t):
        for s in t.get_symbols():
            if t.get_type() != "module" and s.is_global() and not s.is_declared_global() and s.is_referenced() \
                    and s.get_name() not in bound:
                missing.append(f"{t.get_name()}:{t.get_lineno()} {s.get_name()}")
        for c in t.get_children():
            walk(c)
    walk(top)
    return missing


@pytest.mark.parametrize("path", FILES, ids=[os.path.relpath(f, ROOT) for f in FILES])
def test_no_unbound_global_names(path):
    assert _unbound_globals(path) == []
