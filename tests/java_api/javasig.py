"""A small Java declaration reader for the drop-in conformance check (tests/test_java_conformance.py): fields, method
and constructor signatures of one class body, with comments, strings and method bodies skipped.  Enough for the
reference's plugin classes and the committed drop-in sources; not a Java parser."""
import re

_MODS = {"public", "protected", "private", "static", "final", "abstract", "synchronized", "native", "transient",
         "volatile", "default", "strictfp"}


def strip(src):
    """Source without comments, string / char literals and annotations."""
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    src = re.sub(r"//[^\n]*", " ", src)
    src = re.sub(r'"(?:\\.|[^"\\])*"', '""', src)
    src = re.sub(r"'(?:\\.|[^'\\])'", "''", src)
    src = re.sub(r"@\w+(\.\w+)*(\([^)]*\))?", " ", src)
    return src


def _type_of_param(p):
    toks = [t for t in re.split(r"\s+", p.strip()) if t and t != "final"]
    if not toks:
        return None
    t = " ".join(toks[:-1])
    if toks[-1].endswith("[]"):
        t += "[]" * toks[-1].count("[]")
    return re.sub(r"\s+", "", t.replace("...", "[]"))


def _top_level(body):
    """Declarations at depth 0 of a class body: text with every {...} block reduced to {}."""
    out, depth = [], 0
    for ch in body:
        if ch == "{":
            if depth == 0:
                out.append("{")
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 0:
                out.append("}")
        elif depth == 0:
            out.append(ch)
    return "".join(out)


def classes(src):
    """{class name: {"kind", "extends", "implements", "mods", "fields": {name: type}, "methods": [sig...]}} of the
    top-level and nested types in one source file.  sig = {"name", "params", "mods", "ret", "throws"}."""
    s = strip(src)
    res = {}
    for m in re.finditer(r"((?:\b(?:public|protected|private|static|final|abstract)\s+)*)\b(class|interface|enum)\s+"
                         r"(\w+)(?:\s*<[^>{]*>)?\s*(?:extends\s+([\w.<>, ]+?))?\s*(?:implements\s+([\w.<>, ]+?))?\s*\{", s):
        start = m.end()
        depth, i = 1, start
        while depth and i < len(s):
            depth += s[i] == "{"
            depth -= s[i] == "}"
            i += 1
        body = _top_level(s[start:i - 1])
        info = {"kind": m.group(2), "extends": (m.group(4) or "").strip(), "mods": m.group(1).split(),
                "implements": [x.strip() for x in (m.group(5) or "").split(",") if x.strip()],
                "fields": {}, "methods": []}
        for d in re.split(r"[;}]", body):
            d = d.strip().rstrip("{").strip()
            if not d or re.search(r"\b(class|interface|enum)\b", d) or d.startswith(("static", "{")) and "(" not in d:
                continue
            eq, par = d.find("="), d.find("(")
            mm = None if 0 <= eq < par or par < 0 else \
                re.match(r"^(.*?)\b(\w+)\s*\(([^)]*)\)\s*(?:throws\s+([\w., ]+))?$", d, flags=re.S)
            if mm:
                mods, ret = _mods_and_type(mm.group(1))
                name = mm.group(2)
                if name in ("if", "for", "while", "switch", "catch", "return", "new", "synchronized", "super", "this"):
                    continue
                params = [t for t in (_type_of_param(p) for p in _split_params(mm.group(3))) if t]
                info["methods"].append({"name": name, "params": params, "mods": mods, "ret": ret,
                                        "throws": sorted(x.strip() for x in (mm.group(4) or "").split(",") if x.strip()),
                                        "ctor": not ret})
                continue
            fm = re.match(r"^([^=(]*?)\b(\w+)\s*(=.*)?$", d, flags=re.S)
            if fm:
                mods, typ = _mods_and_type(fm.group(1))
                if typ:
                    info["fields"][fm.group(2)] = typ
        res[m.group(3)] = info
    return res


def _mods_and_type(prefix):
    """('public static final int ') -> (['public', 'static', 'final'], 'int'); generics and arrays kept in the type"""
    prefix = re.sub(r"^\s*<[^>]*>\s*", "", prefix.strip())
    toks = prefix.split()
    mods = []
    while toks and toks[0] in _MODS:
        mods.append(toks.pop(0))
    if toks and toks[0].startswith("<"):  # generic method: <T> void f(...)
        while toks and not toks[0].endswith(">"):
            toks.pop(0)
        toks = toks[1:]
    return mods, re.sub(r"\s+", "", " ".join(toks))


def _split_params(p):
    out, depth, cur = [], 0, ""
    for ch in p:
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return out


def sig_key(m):
    return f"{m['name']}({','.join(m['params'])})"
