"""ISA scan for the store-data hazard of wide VMEM stores.

A `buffer_store_dwordx4` / `global_store_dwordx4` (or x3) reads its data VGPRs after issue; an instruction that
writes one of those VGPRs fewer than 2 wait states later corrupted stored bytes at full C4 size on MI355X
(profiles/r01/session3/diag_c4_store_hold.log), and hipcc (ROCm 7.2, gfx950) did not pad it.  The kernels guard
every such store with `store_data_hold` (kernels.hip).  This module finds the pattern in the device code that is
actually shipped: it unbundles the gfx950 code object from libozec.so, disassembles it and walks every wide
store's next instructions, counting `s_nop N` as N + 1 wait states.
"""
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
REQUIRED_WAIT_STATES = 2

_WIDE_STORE = re.compile(r"^\s*(global|buffer|flat|scratch)_store_dwordx([34])\s+(.*?)(\s+//.*)?$")
_INSTR = re.compile(r"^\s+([a-z_0-9]+)(?:\s+(.*?))?(\s+//.*)?$")
_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_FUNC = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def _regs(op):
    """VGPR numbers named by one operand string (v7, v[4:7])."""
    out = set()
    for m in _VREG.finditer(op):
        if m.group(1) is not None:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def _operands(text):
    return [o.strip() for o in text.split(",")] if text else []


def _writes(mnemonic, ops):
    """VGPRs a VALU instruction writes (its first operand).  Loads into the store's data registers are not
    counted: their data returns after the memory latency, long after the store has read its operands (the
    register spills of gf_code_vec<10,4> do exactly that, a scratch store then a buffer load into the same VGPRs)."""
    if ops and mnemonic.startswith("v_"):
        return _regs(ops[0])
    return set()


BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def disassemble_shared_object(so_path):
    """llvm-objdump text of every gfx950 code object bundled into a HIP shared library: the .hip_fatbin section holds
    one offload bundle per translation unit (kernels, fused, each fused_nb_<K>_<R>), back to back at aligned offsets."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", so_path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        blob = open(fat, "rb").read()
        starts = []
        i = blob.find(BUNDLE_MAGIC)
        while i >= 0:
            starts.append(i)
            i = blob.find(BUNDLE_MAGIC, i + 1)
        out = []
        for n, a in enumerate(starts):
            part, co = os.path.join(d, f"b{n}.bin"), os.path.join(d, f"k{n}.co")
            open(part, "wb").write(blob[a:starts[n + 1] if n + 1 < len(starts) else len(blob)])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--targets={TARGET}",
                            f"--input={part}", f"--output={co}"], check=True, capture_output=True)
            out.append(disassemble_code_object(co))
        return "\n".join(out)


def disassemble_code_object(co_path):
    return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co_path], check=True, capture_output=True,
                          text=True).stdout


def scan(text):
    """[(function, store line, offending line, wait states before it)] for every wide store whose data VGPRs are
    rewritten before REQUIRED_WAIT_STATES wait states have passed."""
    lines = text.splitlines()
    func = "?"
    bad = []
    for i, line in enumerate(lines):
        f = _FUNC.match(line)
        if f:
            func = f.group(1)
            continue
        m = _WIDE_STORE.match(line)
        if not m:
            continue
        ops = _operands(m.group(3))
        data = ops[1] if m.group(1) in ("global", "flat", "scratch") else ops[0]
        dregs = _regs(data)
        ws = 0
        for nxt in lines[i + 1:i + 12]:
            if _FUNC.match(nxt) or not nxt.strip():
                break
            im = _INSTR.match(nxt)
            if not im:
                continue
            mn, rest = im.group(1), im.group(2) or ""
            if _writes(mn, _operands(rest)) & dregs:
                bad.append((func, line.strip(), nxt.strip(), ws))
                break
            if mn == "s_nop":
                ws += int(rest.split()[0], 0) + 1
            else:
                ws += 1
            if ws >= REQUIRED_WAIT_STATES:
                break
    return bad
