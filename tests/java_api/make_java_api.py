"""Writes tests/java_api/reference_api.json: the declarations of the reference classes the Java drop-in extends,
implements, patches or mirrors (fields of the package-private state classes, abstract / overridable methods,
interfaces, factory methods), read from the reference checkout as text.  The file is data for
tests/test_java_conformance.py, which checks the committed java/ sources against it with no JDK and no reference
checkout at hand.  Regenerate: python tests/java_api/make_java_api.py /root/reference"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import javasig  # noqa: E402

EC = "hadoop-hdds/erasurecode/src/main/java/org/apache/ozone/erasurecode/rawcoder/"
CM = "hadoop-hdds/common/src/main/java/org/apache/hadoop/ozone/common/"
OC = "hadoop-ozone/common/src/main/java/org/apache/hadoop/ozone/client/checksum/"
FILES = {
    "RawErasureEncoder": EC + "RawErasureEncoder.java", "RawErasureDecoder": EC + "RawErasureDecoder.java",
    "RawErasureCoderFactory": EC + "RawErasureCoderFactory.java", "EncodingState": EC + "EncodingState.java",
    "ByteBufferEncodingState": EC + "ByteBufferEncodingState.java",
    "ByteArrayEncodingState": EC + "ByteArrayEncodingState.java", "DecodingState": EC + "DecodingState.java",
    "ByteBufferDecodingState": EC + "ByteBufferDecodingState.java",
    "ByteArrayDecodingState": EC + "ByteArrayDecodingState.java",
    "ChecksumByteBuffer": CM + "ChecksumByteBuffer.java", "ChecksumByteBufferFactory": CM + "ChecksumByteBufferFactory.java",
    "Checksum": CM + "Checksum.java", "ChecksumData": CM + "ChecksumData.java", "ChunkBuffer": CM + "ChunkBuffer.java",
    "CrcComposer": OC + "CrcComposer.java", "CrcUtil": OC + "CrcUtil.java",
}
SERVICES = "hadoop-hdds/erasurecode/src/main/resources/META-INF/services/"


def main(ref):
    out = {"source": "z-bb/ozone reference checkout, read as text", "classes": {}, "files": {}}
    for name, rel in FILES.items():
        src = open(os.path.join(ref, rel), encoding="utf-8").read()
        out["classes"][name] = javasig.classes(src)[name]
        out["files"][name] = rel
    out["services"] = sorted(os.listdir(os.path.join(ref, SERVICES)))
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_api.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
