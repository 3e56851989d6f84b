#!/usr/bin/env python3
"""oracle/split_ref.py -- TEST INFRASTRUCTURE ONLY.

Builds the reference's own two-rail split -- `APipeAllreduceOptions::calculateElements_AG`
(`gloo/gloo/pipeallreduce-a.h:137-294`) and `calculateElements_AA` (`:296-376`) -- into
`oracle/_ref/libsplit_ref.so`, so that the split table is pinned to the
reference's compiled code rather than to hand-evaluated rows.

Why not through oracle/Makefile: the header cannot be compiled as a whole here -- it includes
`gloo/sharp_allreduce.h` and `sharp/api/sharp.h` (`pipeallreduce-a.h:24-25`), which the image
lacks, and no stand-in for them is written.  The two methods themselves use nothing from those
headers: they read `this->context->size` and do integer arithmetic.  So this script locates the
two method definitions in the header where it lies (by their signatures, brace-matched), and
hands that text -- unmodified -- to `g++` on stdin inside a harness class whose `context` member
has a `size` field.  No reference text is written to disk or committed; only the compiled
`.so` lands in `oracle/_ref/` (git-ignored, like `libgloo_ref.so`).  Flags follow the
reference's Release build (`-O3 -DNDEBUG`, no `-march`, `gloo/CMakeLists.txt:92`).

    python3 oracle/split_ref.py            # builds _ref/libsplit_ref.so (needs /root/reference)

The exported entry point is `ref_split(table, P, n, &e1, &e2)` with table 0 = _AA, 1 = _AG
(HYDRA_SPLIT_AA / HYDRA_SPLIT_AG in include/hydra_hip.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF_HEADER = os.environ.get("HYDRA_REF_PIPE_HEADER",
                            "/root/reference/gloo/gloo/pipeallreduce-a.h")
OUT = os.path.join(HERE, "_ref", "libsplit_ref.so")

METHODS = ("calculateElements_AG", "calculateElements_AA")


def method_text(src: str, name: str) -> str:
    """The definition `void <name>(size_t elements, ...) { ... }` from the header text."""
    sig = "void %s(" % name
    start = src.find(sig)
    if start < 0:
        raise RuntimeError("%s not found in %s" % (name, REF_HEADER))
    if src.find(sig, start + 1) >= 0:
        raise RuntimeError("%s defined twice in %s" % (name, REF_HEADER))
    i = src.index("{", start)
    depth = 0
    j = i
    while True:  # the method bodies hold no braces inside strings or character literals
        c = src[j]
        if c == "{":
            depth += 1
        elif c == "}":
            depth -= 1
            if depth == 0:
                return src[start:j + 1]
        j += 1


def translation_unit(src: str) -> str:
    bodies = "\n".join(method_text(src, m) for m in METHODS)
    return (
        "#include <cstddef>\n"
        "namespace {\n"
        "struct SplitContext { int size; };\n"
        "struct SplitHarness {\n"
        "  SplitContext* context;\n"
        "#line 1 \"pipeallreduce-a.h (methods)\"\n"
        + bodies +
        "\n};\n"
        "}  // namespace\n"
        "extern \"C\" void ref_split(int table, int P, size_t n, size_t* e1, size_t* e2) {\n"
        "  SplitContext c{P};\n"
        "  SplitHarness h{&c};\n"
        "  if (table == 1) h.calculateElements_AG(n, e1, e2);\n"
        "  else h.calculateElements_AA(n, e1, e2);\n"
        "}\n")


def build(out: str = OUT) -> str:
    with open(REF_HEADER) as f:
        src = f.read()
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["g++", "-std=c++14", "-O3", "-DNDEBUG", "-fPIC", "-shared", "-w",
                    "-x", "c++", "-", "-o", out],
                   input=translation_unit(src).encode(), check=True)
    return out


def load(path: str = OUT):
    lib = ctypes.CDLL(path)
    sz = ctypes.c_size_t
    lib.ref_split.argtypes = [ctypes.c_int, ctypes.c_int, sz, ctypes.POINTER(sz),
                              ctypes.POINTER(sz)]
    lib.ref_split.restype = None
    return lib


def ref_split(lib, table: int, P: int, n: int):
    e1, e2 = ctypes.c_size_t(), ctypes.c_size_t()
    lib.ref_split(table, P, n, ctypes.byref(e1), ctypes.byref(e2))
    return e1.value, e2.value


if __name__ == "__main__":
    print(build(sys.argv[1] if len(sys.argv) > 1 else OUT))
