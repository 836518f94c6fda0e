#!/usr/bin/env python3
"""Extracts the declarations the KP:52 drop-in depends on from the reference's KProcessor.java into
tests/golden/kprocessor_api.json (data: names and types, no source text):

* the Order class (KP:448-475): top-level or nested, its package and modifiers, its public fields
  and the parameter types of its constructors;
* the type arguments of MatchingEngine's Processor (KP:63) and the package of that interface.

tests/test_java_processor.py checks integration/jni/GpuMatchingEngine.java against it (and against
KProcessor.java itself when /root/reference is present).

    python tools/gen_kprocessor_api.py [/root/reference/src/main/java/KProcessor.java]
"""
from __future__ import annotations

import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT_SRC = "/root/reference/src/main/java/KProcessor.java"
OUT = os.path.join(ROOT, "tests", "golden", "kprocessor_api.json")


def strip_comments(src: str) -> str:
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    return re.sub(r"//[^\n]*", " ", src)


def class_body(src: str, start: int) -> tuple[int, int]:
    """(index of '{', index of the matching '}') of the class declared at `start`."""
    i = src.index("{", start)
    depth = 0
    for j in range(i, len(src)):
        if src[j] == "{":
            depth += 1
        elif src[j] == "}":
            depth -= 1
            if depth == 0:
                return i, j
    raise ValueError("unbalanced class body")


def extract(src_text: str) -> dict:
    src = strip_comments(src_text)
    pkg = re.search(r"^\s*package\s+([\w.]+)\s*;", src, flags=re.M)
    # top-level classes: declared at brace depth 0
    depth, tops = 0, []
    for m in re.finditer(r"[{}]|\b(?:(public|final|abstract)\s+)*class\s+(\w+)", src):
        t = m.group(0)
        if t == "{":
            depth += 1
        elif t == "}":
            depth -= 1
        elif depth == 0:
            tops.append((m.group(2), m.start(), t))
    order = next((t for t in tops if t[0] == "Order"), None)
    nested = re.search(r"\bstatic\s+class\s+Order\b", src) is not None
    api: dict = {"package": pkg.group(1) if pkg else "", "order": None, "processor": None}
    if order:
        name, start, decl = order
        b0, b1 = class_body(src, start)
        body = src[b0 + 1:b1]
        fields = {}
        for fm in re.finditer(r"\bpublic\s+([\w<>]+)\s+(\w+)\s*;", body):
            fields[fm.group(2)] = fm.group(1)
        ctors = []
        for cm in re.finditer(r"\bpublic\s+Order\s*\(", body):
            j, depth = cm.end(), 1             # the parameter list, parentheses balanced
            while depth:
                depth += {"(": 1, ")": -1}.get(body[j], 0)
                j += 1
            plist = re.sub(r"@\w+\s*(\([^)]*\))?", " ", body[cm.end():j - 1])   # annotations out
            ctors.append([p.split()[0] for p in plist.split(",") if p.strip()])
        api["order"] = {"top_level": True, "nested": nested, "public": "public" in decl.split(),
                        "implements": [x.strip() for x in re.findall(r"implements\s+([\w, ]+)", src[start:b0])[0].split(",")]
                        if "implements" in src[start:b0] else [],
                        "fields": fields, "constructors": ctors}
    pm = re.search(r"class\s+MatchingEngine\s+implements\s+Processor\s*<\s*(\w+)\s*,\s*(\w+)\s*>", src)
    imp = re.search(r"import\s+([\w.]+\.Processor)\s*;", src)
    if pm:
        api["processor"] = {"key": pm.group(1), "value": pm.group(2), "interface": imp.group(1) if imp else None}
    return api


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else DEFAULT_SRC
    with open(path) as f:
        api = extract(f.read())
    with open(OUT, "w") as f:
        json.dump(api, f, indent=1, sort_keys=True)
        f.write("\n")
    print(json.dumps(api))


if __name__ == "__main__":
    main()
