"""The Java drop-in (java/) against the reference's plugin surface, with no JDK: no javac exists in this image
(SURVEY §8(c)), so a rename in the reference or a typo here would otherwise only show on a JDK host.

tests/java_api/reference_api.json holds the declarations of the reference classes the drop-in extends, implements,
patches or mirrors (made by tests/java_api/make_java_api.py from the reference checkout, read as text).  Checked here:
overrides match the reference's abstract methods (names, parameter types, throws), every package-private state field
the coders read exists with that type, the factories implement RawErasureCoderFactory, the checksum classes implement
ChecksumByteBuffer, the CRC composer mirrors CrcComposer's public API, every Java native has its JNI_FN in
jni/ozec_jni.c with the matching arity, the services file is the reference's, and the checksum hook patch names
methods that exist (and applies, where the reference checkout is present)."""
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests", "java_api"))
import javasig  # noqa: E402

JAVA = os.path.join(ROOT, "java", "src", "main", "java")
REF = json.load(open(os.path.join(ROOT, "tests", "java_api", "reference_api.json")))["classes"]
REF_CHECKOUT = "/root/reference"
# java.util.zip.Checksum (JDK 8), the super-interface of ChecksumByteBuffer
JDK_CHECKSUM = {"update(int)", "update(byte[],int,int)", "getValue()", "reset()"}


def _ours():
    out = {}
    for dp, _, fs in os.walk(JAVA):
        for f in fs:
            if f.endswith(".java"):
                path = os.path.join(dp, f)
                src = open(path).read()
                pkg = re.search(r"^package\s+([\w.]+);", src, re.M).group(1)
                for name, info in javasig.classes(src).items():
                    info["package"], info["path"], info["src"] = pkg, path, src
                    out[name] = info
    return out


OURS = _ours()


def _sigs(info, public_only=False):
    return {javasig.sig_key(m): m for m in info["methods"] if not m["ctor"] and (not public_only or "public" in m["mods"])}


def _lineage(name):
    """our class and its superclasses, ours first, then the reference's"""
    chain = []
    while name:
        if name in OURS:
            chain.append(("ours", OURS[name]))
            name = OURS[name]["extends"]
        elif name in REF:
            chain.append(("ref", REF[name]))
            name = REF[name]["extends"]
        else:
            break
    return chain


def test_every_java_file_sits_in_its_package_directory():
    assert len(OURS) >= 14
    for name, info in OURS.items():
        rel = os.path.relpath(os.path.dirname(info["path"]), JAVA).replace(os.sep, ".")
        assert rel == info["package"], (name, rel, info["package"])


@pytest.mark.parametrize("base", ["RawErasureEncoder", "RawErasureDecoder"])
def test_coders_implement_the_reference_abstract_methods(base):
    coders = [n for n in OURS if base in [c[1].get("extends") for c in _lineage(n)] or OURS[n]["extends"] == base]
    concrete = [n for n in coders if "abstract" not in OURS[n]["mods"]]
    assert len(concrete) >= 2, coders  # RS and XOR
    ref = _sigs(REF[base])
    abstract = {k for k, m in ref.items() if "abstract" in m["mods"]}
    assert len(abstract) == 2  # doEncode / doDecode for ByteBuffer and byte[] states
    for n in concrete:
        have = set()
        for who, info in _lineage(n):
            if who == "ours":
                for k, m in _sigs(info).items():
                    have.add(k)
                    if k in ref:  # an override: same visibility or wider, no new checked exceptions
                        assert set(m["throws"]) <= set(ref[k]["throws"]), (n, k)
                        assert not ("private" in m["mods"]), (n, k)
        assert abstract <= have, (n, abstract - have)
        # every package-private state field the coders read exists on that state class (or its base)
        for who, info in _lineage(n):
            if who != "ours":
                continue
            for m in re.finditer(r"void\s+do(?:En|De)code\s*\(\s*(\w+)\s+(\w+)\s*\)\s*(?:throws[\w\s,]*)?\{",
                                 info["src"]):
                cls, var = m.group(1), m.group(2)
                fields = dict(REF[REF[cls]["extends"]]["fields"], **REF[cls]["fields"])
                body = info["src"][m.end():info["src"].find("\n  }\n", m.end())]
                used = set(re.findall(rf"\b{var}\.(\w+)\b(?!\s*\()", body))
                assert used and used <= set(fields), (n, cls, used - set(fields))
                # the arrays are what the JNI natives take
                for f in used & {"inputs", "outputs"}:
                    assert fields[f] in ("ByteBuffer[]", "byte[][]"), (cls, f, fields[f])


def test_factories_implement_raw_erasure_coder_factory():
    iface = set(_sigs(REF["RawErasureCoderFactory"]))
    facts = [n for n, i in OURS.items() if "RawErasureCoderFactory" in i["implements"]]
    assert sorted(facts) == ["HipRSRawErasureCoderFactory", "HipXORRawErasureCoderFactory"]
    for n in facts:
        mine = _sigs(OURS[n])
        assert iface <= set(mine), (n, iface - set(mine))
        for k in iface:
            assert mine[k]["ret"] == next(m["ret"] for m in REF["RawErasureCoderFactory"]["methods"]
                                          if javasig.sig_key(m) == k)
            assert "public" in mine[k]["mods"]


SVC_DIR = os.path.join(ROOT, "java", "src", "main", "resources", "META-INF", "services")
ACCEL_SVC = "org.apache.hadoop.ozone.common.ChecksumAccelerator"


def _listed(name):
    return [ln.strip() for ln in open(os.path.join(SVC_DIR, name)) if ln.strip() and not ln.startswith("#")]


def test_services_file_is_the_reference_plugin_seam():
    ref_services = json.load(open(os.path.join(ROOT, "tests", "java_api", "reference_api.json")))["services"]
    # the reference's coder seam, plus the checksum seam the hook patch adds to hdds-common
    assert sorted(os.listdir(SVC_DIR)) == sorted(ref_services + [ACCEL_SVC])
    listed = _listed(ref_services[0])
    for fq in listed:
        pkg, _, cls = fq.rpartition(".")
        assert cls in OURS and OURS[cls]["package"] == pkg, fq
    assert {fq.rpartition(".")[2] for fq in listed} == {"HipRSRawErasureCoderFactory", "HipXORRawErasureCoderFactory"}


def test_checksum_byte_buffer_implementation():
    info = OURS["HipChecksumByteBuffer"]
    assert "ChecksumByteBuffer" in info["implements"] and info["package"] == "org.apache.hadoop.ozone.common"
    need = set(_sigs(REF["ChecksumByteBuffer"])) | JDK_CHECKSUM
    mine = _sigs(info, public_only=True)
    assert need <= set(mine), need - set(mine)
    # the factory hook (java/patches) builds it from (type, the JDK-backed impl) and asks enabled() first
    ctors = [m["params"] for m in info["methods"] if m["ctor"]]
    assert ["int", "ChecksumByteBuffer"] in ctors
    assert "enabled()" in mine and "static" in mine["enabled()"]["mods"]
    # below its threshold every update is the host CRC's: no byte loop left in the class
    body = javasig.strip(info["src"])
    assert "host.update(buffer)" in body and "host.update(b, off, len)" in body and "host.update(b)" in body
    assert not re.search(r"table\[", body)


def test_checksum_batch_hook_signatures():
    info = OURS["HipChecksum"]
    mine = _sigs(info, public_only=True)
    assert "useGpu(ChecksumType,ChunkBuffer)" in mine and mine["useGpu(ChecksumType,ChunkBuffer)"]["ret"] == "boolean"
    assert mine["computeChecksum(ChecksumType,ChunkBuffer,int)"]["ret"] == "ChecksumData"
    # what it builds and calls exists in the reference with these shapes
    assert ["ChecksumType", "int", "List<ByteString>"] in [m["params"] for m in REF["ChecksumData"]["methods"]
                                                            if m["ctor"]]
    chunk = _sigs(REF["ChunkBuffer"])
    assert chunk["asByteBufferList()"]["ret"] == "List<ByteBuffer>" and chunk["remaining()"]["ret"] == "int"


def _patch():
    return open(os.path.join(ROOT, "java", "patches", "hdds-common-checksum-hook.patch")).read()


CM = "hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/"


def _patch_files():
    """{path: (added source lines, new file?)} of the hook patch"""
    out, cur = {}, None
    lines = _patch().splitlines()
    for i, ln in enumerate(lines):
        if ln.startswith("+++ b/"):
            cur = ln[6:]
            out[cur] = ([], i + 1 < len(lines) and lines[i + 1].startswith("@@ -0,0 "))
        elif cur and ln.startswith("+"):
            out[cur][0].append(ln[1:])
    return out


def _added_code(lines):
    """added lines without comments and string literals"""
    return javasig.strip("\n".join(lines))


def test_checksum_hook_patch_targets_exist():
    files = _patch_files()
    assert sorted(files) == sorted(CM + f for f in ("Checksum.java", "ChecksumAccelerator.java",
                                                    "ChecksumAccelerators.java", "ChecksumByteBufferFactory.java"))
    assert files[CM + "ChecksumAccelerator.java"][1] and files[CM + "ChecksumAccelerators.java"][1]  # new files
    assert "computeChecksum(ChunkBuffer)" in _sigs(REF["Checksum"])
    fac = _sigs(REF["ChecksumByteBufferFactory"])
    assert fac["crc32Impl()"]["ret"] == fac["crc32CImpl()"]["ret"] == "ChecksumByteBuffer"
    chk = _added_code(files[CM + "Checksum.java"][0])
    assert "ChecksumAccelerators.computeChecksum(checksumType, data, bytesPerChecksum)" in chk
    assert "if (accelerated != null)" in chk and "return accelerated;" in chk
    f = _added_code(files[CM + "ChecksumByteBufferFactory.java"][0])
    assert "ChecksumAccelerators.wrap(false, new ChecksumByteBufferImpl(new CRC32()))" in f
    assert "ChecksumAccelerators.wrap(true, crc32CHostImpl())" in f
    # the patched computeChecksum(ChunkBuffer) keeps the reference's variable names
    assert set(REF["Checksum"]["fields"]) >= {"checksumType", "bytesPerChecksum"}


# what the hook patch may name: the JDK, hdds-common's own package (the reference's classes and the two the patch adds)
# and the imports the patched files already have (the proto ChecksumType, slf4j)
_ALLOWED_IMPORTS = re.compile(r"^(java\.|org\.apache\.hadoop\.ozone\.common\.[A-Z]|org\.slf4j\."
                              r"|org\.apache\.hadoop\.hdds\.protocol\.datanode\.proto\.ContainerProtos\.ChecksumType$)")


def test_checksum_hook_patch_names_nothing_outside_hdds_common():
    """hdds-common must not depend on the HIP jar (the reactor would have a module cycle, and every Ozone
    process without the jar would fail on its first CRC).  Every import the patch adds is the JDK, hdds-common's package
    or an import the patched file already had; no added line names a class of this repo's jar or its packages."""
    ref_src = {}
    for path, (added, new) in _patch_files().items():
        code = _added_code(added)
        for imp in re.findall(r"^\s*import\s+(?:static\s+)?([\w.]+)\s*;", code, re.M):
            assert _ALLOWED_IMPORTS.match(imp), (path, imp)
        for ours in list(OURS) + ["OzecNative", "ozec", "erasurecode", "Hip"]:
            assert not re.search(r"\b" + ours, code), (path, ours)
        body = re.sub(r"^\s*(import|package)\s+[\w.]+\s*;", "", code, flags=re.M)
        names = set(re.findall(r"\b([A-Z]\w*)\b", body))
        # every class named is in hdds-common's package, imported, the JDK's java.lang, or declared by the patch
        declared = {"ChecksumAccelerator", "ChecksumAccelerators"}
        imported = {i.rpartition(".")[2] for i in re.findall(r"import\s+([\w.]+);", code)}
        if not new and os.path.isdir(REF_CHECKOUT):
            ref_src[path] = open(os.path.join(REF_CHECKOUT, path)).read()
            imported |= {i.rpartition(".")[2] for i in re.findall(r"import\s+([\w.]+);", ref_src[path])}
        java_lang = {"Exception", "RuntimeException", "LinkageError", "Throwable", "Override", "Class", "String"}
        hdds_common = set(REF) | {"ChunkBuffer", "ChecksumData", "ChecksumByteBuffer", "ChecksumByteBufferImpl",
                                  "OzoneChecksumException", "Checksum"}
        unknown = {n for n in names if not n.isupper()} - declared - imported - java_lang - hdds_common - {"CRC32"}
        assert not unknown, (path, unknown)


def test_checksum_seam_without_a_provider_is_the_reference():
    """No JVM here, so the no-provider behaviour is checked on the patched source: the accelerator is looked up once
    with ServiceLoader and every failure to load is caught; with no provider (INSTANCE null) wrap() returns the
    runtime's CRC unchanged and computeChecksum() returns null, which the patched Checksum answers with the
    reference's own window loop."""
    acc = "\n".join(_patch_files()[CM + "ChecksumAccelerators.java"][0])
    code = javasig.strip(acc)
    assert "ServiceLoader.load(" in code and "ChecksumAccelerator.class" in code
    assert "catch (ServiceConfigurationError | LinkageError | RuntimeException e)" in code
    assert "return INSTANCE == null ? host : INSTANCE.wrap(crc32c, host);" in code
    assert re.search(r"return INSTANCE == null \? null\s*: INSTANCE\.computeChecksum\(type, data, bytesPerChecksum\);", code)
    assert "private static final ChecksumAccelerator INSTANCE = load();" in code
    iface = javasig.classes("\n".join(_patch_files()[CM + "ChecksumAccelerator.java"][0]))["ChecksumAccelerator"]
    assert {javasig.sig_key(m) for m in iface["methods"]} == {
        "isAvailable()", "wrap(boolean,ChecksumByteBuffer)", "computeChecksum(ChecksumType,ChunkBuffer,int)"}


def test_hip_checksum_accelerator_is_the_registered_provider():
    assert _listed(ACCEL_SVC) == ["org.apache.hadoop.ozone.common.HipChecksumAccelerator"]
    info = OURS["HipChecksumAccelerator"]
    assert info["package"] == "org.apache.hadoop.ozone.common" and "ChecksumAccelerator" in info["implements"]
    iface = javasig.classes("\n".join(_patch_files()[CM + "ChecksumAccelerator.java"][0]))["ChecksumAccelerator"]
    mine = _sigs(info, public_only=True)
    for m in iface["methods"]:
        k = javasig.sig_key(m)
        assert k in mine and mine[k]["ret"] == m["ret"], k
    assert ["public"] == [x for x in ([m["mods"] for m in info["methods"] if m["ctor"] and not m["params"]] or [[]])[0]
                          if x == "public"]  # ServiceLoader needs a public no-argument constructor
    # the batch path leaves the ChunkBuffer consumed, as data.iterate(bytesPerChecksum) does
    hc = javasig.strip(OURS["HipChecksum"]["src"])
    assert "b.position(b.limit());" in hc and "data instanceof ChunkBufferImplWithByteBuffer" in hc


@pytest.mark.skipif(not os.path.isdir(REF_CHECKOUT), reason="reference checkout absent")
def test_checksum_hook_patch_applies_to_the_reference(tmp_path):
    for rel, (_, new) in _patch_files().items():
        dst = tmp_path / rel
        dst.parent.mkdir(parents=True, exist_ok=True)
        if new:  # the two files the patch adds to hdds-common
            assert not os.path.exists(os.path.join(REF_CHECKOUT, rel)), rel
        else:
            dst.write_text(open(os.path.join(REF_CHECKOUT, rel)).read())
    r = subprocess.run(["patch", "-p1", "--dry-run", "-i", os.path.join(ROOT, "java", "patches",
                                                                       "hdds-common-checksum-hook.patch")],
                       cwd=tmp_path, capture_output=True, text=True)
    assert r.returncode == 0 and "FAILED" not in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(not os.path.isdir(REF_CHECKOUT), reason="reference checkout absent")
def test_reference_api_fixture_is_current(tmp_path):
    import importlib
    mk = importlib.import_module("make_java_api")
    got = {}
    for name, rel in mk.FILES.items():
        got[name] = javasig.classes(open(os.path.join(REF_CHECKOUT, rel)).read())[name]
    assert json.loads(json.dumps(got)) == REF


def test_crc_composer_mirrors_the_reference_api():
    ref = {k: m for k, m in _sigs(REF["CrcComposer"], public_only=True).items()}
    mine = _sigs(OURS["HipCrcComposer"], public_only=True)
    assert OURS["HipCrcComposer"]["package"] == "org.apache.hadoop.ozone.client.checksum"
    for k, m in ref.items():
        assert k in mine, k
        assert mine[k]["ret"] == m["ret"].replace("CrcComposer", "HipCrcComposer"), k
        assert set(mine[k]["throws"]) == set(m["throws"]), k
        assert ("static" in mine[k]["mods"]) == ("static" in m["mods"]), k
    util = _sigs(REF["CrcUtil"])
    for k in ("getMonomial(long,int)", "compose(int,int,long,int)"):
        assert _sigs(OURS["HipCrcUtil"])[k]["ret"] == util[k]["ret"]
    assert set(REF["CrcUtil"]["fields"]) >= {"GZIP_POLYNOMIAL", "CASTAGNOLI_POLYNOMIAL"}


def test_every_native_has_its_jni_entry():
    natives = {m["name"]: m for m in OURS["OzecNative"]["methods"] if "native" in m["mods"]}
    jni = open(os.path.join(ROOT, "jni", "ozec_jni.c")).read()
    entries = {}
    for m in re.finditer(r"JNI_FN\((\w+)\)\s*\(([^)]*)\)", jni):
        entries[m.group(1)] = [p.strip() for p in m.group(2).split(",")]
    assert set(natives) == set(entries), (set(natives) ^ set(entries))
    jtype = {"int": "jint", "long": "jlong", "boolean": "jboolean", "byte[]": "jbyteArray", "int[]": "jintArray",
             "ByteBuffer": "jobject", "ByteBuffer[]": "jobjectArray", "byte[][]": "jobjectArray"}
    jret = {"int": "jint", "long": "jlong", "void": "void", "ByteBuffer": "jobject", "int[]": "jintArray"}
    for name, m in natives.items():
        params = entries[name]
        assert params[0].startswith("JNIEnv") and params[1].startswith("jclass"), name
        assert [p.split()[0] for p in params[2:]] == [jtype[t] for t in m["params"]], name
        decl = re.search(rf"JNIEXPORT\s+(\w+)\s+JNICALL\s+JNI_FN\({name}\)", jni).group(1)
        assert decl == jret[m["ret"]], (name, decl, m["ret"])
