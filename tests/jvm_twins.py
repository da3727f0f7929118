"""Static checks of the JVM side of the drop-in boundary against the C ABI.

There is no JDK in this image, so src/java/causal/gpu/CauseWeave.java and
src/clj/causal/collections/list_gpu.clj are never compiled here.  Their
contract with the library is still plain text that can be read:

* the constants CauseWeave.java copies from include/causeweave.h (KIND_*,
  STATUS_*, CW_NIL, CW_MEM_HOST);
* its StructLayouts: field names, order and carrier types against the C
  structs, and every offset it reads or writes through a segment allocated
  with one of them, against the x86-64 natural-alignment offsets;
* its downcall handles: every symbol is declared in the header with the same
  arity and carrier types;
* list_gpu.clj: every CauseWeave static, nested class, method and field it
  names exists in CauseWeave.java.

check_twins() returns the list of problems (empty = in line); the tests feed
it the committed sources and deliberately drifted copies.
"""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "causeweave.h")
JAVA = os.path.join(ROOT, "src", "java", "causal", "gpu", "CauseWeave.java")
CLJ = os.path.join(ROOT, "src", "clj", "causal", "collections", "list_gpu.clj")

# Java StructLayout constant -> C typedef it mirrors
LAYOUTS = {"LIST_BATCH": "cw_list_batch", "LIST_BATCH_K128": "cw_list_batch_k128",
           "LIST_RESULT": "cw_list_result", "MAP_BATCH": "cw_map_batch",
           "MAP_RESULT": "cw_map_result"}
# C scalar type -> (Panama carrier, size)
CARRIER = {"uint64_t": ("JAVA_LONG", 8), "int64_t": ("JAVA_LONG", 8), "size_t": ("JAVA_LONG", 8),
           "uint32_t": ("JAVA_INT", 4), "int32_t": ("JAVA_INT", 4), "int": ("JAVA_INT", 4),
           "uint8_t": ("JAVA_BYTE", 1), "char": ("JAVA_BYTE", 1)}


def _strip_c_comments(src: str) -> str:
    return re.sub(r"/\*.*?\*/", " ", src, flags=re.S)


def header_constants(src: str) -> dict:
    """CW_KIND_* / CW_STATUS_* / CW_MEM_* enum values and the CW_NIL define."""
    s = _strip_c_comments(src)
    out = {}
    for body in re.findall(r"enum\s*\{(.*?)\}", s, flags=re.S):
        for name, expr in re.findall(r"(CW_\w+)\s*=\s*([^,]+)", body):
            e = expr.strip().replace("1u", "1")
            m = re.fullmatch(r"1\s*<<\s*(\d+)", e)
            out[name] = 1 << int(m.group(1)) if m else int(e, 0)
    if re.search(r"#define\s+CW_NIL\s+UINT64_MAX", s):
        out["CW_NIL"] = (1 << 64) - 1
    return out


def _c_field(decl: str):
    m = re.fullmatch(r"\s*(?:const\s+)?(\w+)\s*(\*?)\s*(\w+)\s*", decl)
    if not m:
        return None
    typ, ptr, name = m.groups()
    if ptr:
        return name, "ADDRESS", 8
    if typ not in CARRIER:
        return name, None, None  # a nested struct: not mirrored by the Java layouts
    return (name,) + CARRIER[typ]


def header_structs(src: str) -> dict:
    """typedef name -> [(field, carrier, size, offset)] with natural alignment."""
    s = _strip_c_comments(src)
    out = {}
    for body, name in re.findall(r"typedef\s+struct\s*\{(.*?)\}\s*(\w+)\s*;", s, flags=re.S):
        fields, off, ok = [], 0, True
        for decl in body.split(";"):
            if not decl.strip():
                continue
            f = _c_field(decl)
            if f is None or f[1] is None:
                ok = False
                break
            fname, car, size = f
            off = (off + size - 1) // size * size
            fields.append((fname, car, size, off))
            off += size
        if ok:
            out[name] = fields
    return out


def header_functions(src: str) -> dict:
    """cw_* prototype -> (return carrier or 'void', [parameter carriers])."""
    s = re.sub(r"(?m)^\s*#.*$", ";", _strip_c_comments(src))  # preprocessor lines end a statement
    s = " ".join(s.split())
    out = {}
    for ret, name, params in re.findall(r"(?:(?<=[;}{])|^)\s*([\w\s\*]+?)\s*\b(cw_\w+)\s*\(([^)]*)\)\s*;", s):
        ret = ret.strip()
        rc = "void" if ret == "void" else ("ADDRESS" if "*" in ret else CARRIER.get(ret.split()[-1], (None,))[0])
        ps = []
        for p in params.split(","):
            p = p.strip()
            if not p or p == "void":
                continue
            if "*" in p:
                ps.append("ADDRESS")
            else:
                ps.append(CARRIER.get(p.replace("const ", "").split()[0], (None,))[0])
        out[name] = (rc, ps)
    return out


def java_constants(src: str) -> dict:
    """public static final int/long constants of CauseWeave.java (several per line)."""
    out = {}
    for decl in re.findall(r"static\s+final\s+(?:int|long)\s+([^;]+);", src):
        for name, val in re.findall(r"(\w+)\s*=\s*(-?\d+)L?", decl):
            out[name] = int(val)
    return out


def java_layouts(src: str) -> dict:
    """StructLayout name -> [(carrier, field name)]."""
    out = {}
    for name, body in re.findall(r"StructLayout\s+(\w+)\s*=\s*MemoryLayout\.structLayout\((.*?)\);",
                                 src, flags=re.S):
        out[name] = re.findall(r"(JAVA_\w+|ADDRESS)\.withName\(\"(\w+)\"\)", body)
    return out


def java_handles(src: str) -> dict:
    """cw_* symbol -> (return carrier or 'void', [parameter carriers])."""
    out = {}
    for sym, kind, args in re.findall(
            r"h\(\"(cw_\w+)\",\s*FunctionDescriptor\.(of|ofVoid)\(([^)]*)\)\)", src):
        a = [x.strip() for x in args.split(",") if x.strip()]
        out[sym] = ("void", a) if kind == "ofVoid" else (a[0], a[1:])
    return out


def java_segment_accesses(src: str):
    """(layout, carrier, offset, line) for every get/set at a constant offset on
    a segment allocated with one of the StructLayouts (tracked in source order)."""
    seg_layout, out = {}, []
    for ln, line in enumerate(src.splitlines(), 1):
        m = re.search(r"MemorySegment\s+(\w+)\s*=\s*\w+\.allocate\((\w+)\)", line)
        if m:
            if m.group(2) in LAYOUTS:
                seg_layout[m.group(1)] = m.group(2)
            else:
                seg_layout.pop(m.group(1), None)
        for var, car, off in re.findall(r"\b(\w+)\.(?:set|get)\((JAVA_\w+|ADDRESS),\s*(\d+)\b", line):
            if var in seg_layout:
                out.append((seg_layout[var], car, int(off), ln))
    return out


def java_members(src: str):
    """Public names CauseWeave.java defines: static fields, methods, nested
    classes, and the fields of the nested classes."""
    statics = set(java_constants(src))
    methods = set(re.findall(r"public\s+(?:static\s+)?[\w\[\]<>]+\s+(\w+)\s*\(", src))
    classes = set(re.findall(r"class\s+(\w+)", src))
    fields = set()
    for decl in re.findall(r"public\s+(?:final\s+)?[\w\[\]]+(?:\[\])*\s+([\w\s,]+);", src):
        fields.update(x.strip() for x in decl.split(",") if x.strip())
    return statics, methods, classes, fields


def check_twins(header_src: str, java_src: str, clj_src: str) -> list:
    problems = []
    hc, jc = header_constants(header_src), java_constants(java_src)
    pairs = {"KIND_NORMAL": "CW_KIND_NORMAL", "KIND_HIDE": "CW_KIND_HIDE",
             "KIND_HHIDE": "CW_KIND_HHIDE", "KIND_HSHOW": "CW_KIND_HSHOW",
             "KIND_ROOT": "CW_KIND_ROOT", "CW_MEM_HOST": "CW_MEM_HOST"}
    for j in jc:
        if j.startswith("STATUS_"):
            pairs[j] = "CW_" + j
    for j, c in pairs.items():
        if j not in jc:
            problems.append(f"CauseWeave.java lacks {j}")
        elif c not in hc:
            problems.append(f"CauseWeave.java's {j} has no {c} in the header")
        elif jc[j] != hc[c]:
            problems.append(f"{j} = {jc[j]} in CauseWeave.java, {c} = {hc[c]} in the header")
    for c in hc:
        if c.startswith("CW_STATUS_") and c != "CW_STATUS_UNWOVEN" and c[3:] not in jc:
            problems.append(f"the header's {c} is missing from CauseWeave.java")
    if jc.get("CW_NIL", 0) % (1 << 64) != hc.get("CW_NIL"):
        problems.append("CW_NIL differs")
    hs, jl = header_structs(header_src), java_layouts(java_src)
    for jname, cname in LAYOUTS.items():
        if jname not in jl:
            problems.append(f"CauseWeave.java lacks the layout {jname}")
            continue
        cf = hs.get(cname)
        if cf is None:
            problems.append(f"the header lacks struct {cname}")
            continue
        want = [(car, f) for f, car, _, _ in cf]
        if jl[jname] != want:
            problems.append(f"{jname} = {jl[jname]} but {cname} = {want}")
    for lay, car, off, ln in java_segment_accesses(java_src):
        cf = {o: (f, c) for f, c, _, o in hs.get(LAYOUTS[lay], [])}
        if off not in cf:
            problems.append(f"CauseWeave.java:{ln}: offset {off} is no field of {LAYOUTS[lay]}")
        elif cf[off][1] != car:
            problems.append(f"CauseWeave.java:{ln}: {car} at offset {off} of {LAYOUTS[lay]}, "
                            f"field {cf[off][0]} is {cf[off][1]}")
    hf, jh = header_functions(header_src), java_handles(java_src)
    for sym, sig in jh.items():
        if sym not in hf:
            problems.append(f"CauseWeave.java binds {sym}, which the header does not declare")
        elif hf[sym] != sig:
            problems.append(f"{sym}: CauseWeave.java {sig}, header {hf[sym]}")
    statics, methods, classes, fields = java_members(java_src)
    for name in set(re.findall(r"CauseWeave/(\w+)", clj_src)):
        if name not in statics:
            problems.append(f"list_gpu.clj reads CauseWeave/{name}, which CauseWeave.java lacks")
    for name in set(re.findall(r"CauseWeave\$(\w+)", clj_src)):
        if name not in classes:
            problems.append(f"list_gpu.clj names CauseWeave${name}, which CauseWeave.java lacks")
    # interop calls on CauseWeave objects: (.method ^CauseWeave ...) and field reads (.field r)
    for name in set(re.findall(r"\(\.(\w+)\s+\^?CauseWeave\b", clj_src)):
        if name not in methods:
            problems.append(f"list_gpu.clj calls .{name}, which CauseWeave.java lacks")
    for name in set(re.findall(r"\(\.(\w+)\s+r\)", clj_src)):
        if name not in fields:
            problems.append(f"list_gpu.clj reads .{name} of a result, which CauseWeave.java lacks")
    return problems


def read_sources():
    return (open(HEADER).read(), open(JAVA).read(), open(CLJ).read())
