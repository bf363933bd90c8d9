"""Resource usage (VGPRs, SGPRs, scratch, LDS, spills) of the gfx950 kernels shipped in libozec.so, from the code
objects' metadata notes: usage python scripts/kernel_resources.py [name-fragment ...]"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
KEYS = ("vgpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size", "vgpr_spill_count",
        "sgpr_spill_count")


def kernels(so_path):
    out = []
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section", f".hip_fatbin={fat}", so_path, os.path.join(d, "x")],
                       check=True, capture_output=True)
        blob = open(fat, "rb").read()
        offs = [m.start() for m in re.finditer(re.escape(MAGIC), blob)]
        for i, o in enumerate(offs):
            part = os.path.join(d, f"b{i}.bin")
            open(part, "wb").write(blob[o:offs[i + 1] if i + 1 < len(offs) else len(blob)])
            co = os.path.join(d, f"b{i}.co")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={part}", f"--output={co}"],
                               capture_output=True)
            if r.returncode or not os.path.getsize(co):
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readobj", "--notes", co], capture_output=True, text=True).stdout
            # the metadata keys of a kernel are sorted: .group_segment_fixed_size comes before its .name (and the
            # .args entries carry .name keys of their own), so values seen before a kernel's name are held for it
            cur, pending = None, {}
            for ln in notes.splitlines():
                m = re.search(r"\.(name|" + "|".join(KEYS) + r"):\s+(\S+)", ln)
                if not m:
                    continue
                k, v = m.groups()
                if k == "name":
                    if v.startswith("_Z"):
                        cur = {"name": v, **pending}
                        pending = {}
                        out.append(cur)
                elif k == "group_segment_fixed_size":
                    pending[k] = int(v)
                elif cur is not None:
                    cur[k] = int(v)
    return out


if __name__ == "__main__":
    so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ozone_amd", "lib", "libozec.so")
    pats = sys.argv[1:]
    for k in kernels(so):
        if not pats or any(p in k["name"] for p in pats):
            print(k["name"], " ".join(f"{x.split('_')[0]}{'_spill' if 'spill' in x else ''}={k.get(x)}"
                                      for x in KEYS))
