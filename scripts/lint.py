#!/usr/bin/env python3
"""Repository lint gate (reference: scripts/lint.py = cpplint + pylint summary,
run as a CI gate by scripts/travis/travis_script.sh:4-9).

cpplint / pylint are not installed in this image, so this is a self-contained
checker with the rules that matter for this code base:

C++ / HIP (include/, src/, tools/, tests/cpp/, examples/):
  * line length <= 110, no tabs, no trailing whitespace, file ends in '\\n'
  * headers carry an include guard (#ifndef X_H_ / #define X_H_) or #pragma once
  * no CUDA compatibility layers: no `__HIP_PLATFORM_NVIDIA__` / `__CUDACC__`
    dual paths, no `cuda*` runtime calls, no hipify markers
  * device code never writes through the scalar data cache: no scalar-memory
    instruction that stores or is atomic, and no scalar data-cache operation
    other than the invalidate. Checked on the sources AND on the disassembly of
    every built gfx950 code object under build/obj/gpu (llvm-objdump), so
    compiler-emitted code is covered too.
  * `using namespace` only in .cc files
Python (dmlc_core_amd/, tests/, scripts/, top level):
  * every file compiles; no tabs; line length <= 110
  * no bare `except:`; no unsafe deserialisation (pickle.load(s), yaml.load without SafeLoader)

Usage: python scripts/lint.py [--quiet]   (exit 1 on any finding)
"""
from __future__ import annotations

import ast
import os
import re
import sys
from typing import List, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP_DIRS = ["include", "src", "tools", "tests/cpp", "examples"]
PY_DIRS = ["dmlc_core_amd", "tests", "scripts", "examples"]
CPP_EXT = (".h", ".cc", ".hip", ".cpp")
SKIP_DIRS = {"__pycache__", "build", ".git", "gpurun_out"}

CUDA_COMPAT = re.compile(r"__HIP_PLATFORM_NVIDIA__|__CUDACC__|\bcuda[A-Z]\w*\(|HIPIFY|hipify")
# Structural rule: any scalar-prefixed mnemonic containing "store" or "atomic",
# and any scalar cache operation that is not the invalidate.
SCALAR_STORE = re.compile(r"\bs_\w*(?:store|atomic)\w*|\bs_\w*cache_(?!inv)\w+")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
OBJCOPY = "/opt/rocm/lib/llvm/bin/llvm-objcopy"

Finding = Tuple[str, int, str]


def _walk(dirs, exts):
    for d in dirs:
        base = os.path.join(ROOT, d)
        if not os.path.isdir(base):
            continue
        for dp, dn, fn in os.walk(base):
            dn[:] = [x for x in dn if x not in SKIP_DIRS]
            for f in sorted(fn):
                if f.endswith(exts):
                    yield os.path.join(dp, f)


def lint_cpp(path: str) -> List[Finding]:
    out: List[Finding] = []
    rel = os.path.relpath(path, ROOT)
    with open(path, encoding="utf-8") as f:
        text = f.read()
    if text and not text.endswith("\n"):
        out.append((rel, text.count("\n") + 1, "file does not end with a newline"))
    for i, line in enumerate(text.split("\n"), 1):
        if len(line) > 110:
            out.append((rel, i, f"line longer than 110 ({len(line)})"))
        if "\t" in line:
            out.append((rel, i, "tab character"))
        if line.rstrip() != line:
            out.append((rel, i, "trailing whitespace"))
        code = line.split("//", 1)[0]
        if CUDA_COMPAT.search(code):
            out.append((rel, i, "CUDA compatibility construct"))
        if SCALAR_STORE.search(line):
            out.append((rel, i, "scalar-cache store / atomic in device code"))
        if path.endswith(".h") and re.match(r"\s*using namespace\b", code):
            out.append((rel, i, "`using namespace` in a header"))
    if path.endswith(".h"):
        if "#pragma once" not in text and not re.search(r"#ifndef (\w+_H_)\s*\n#define \1", text):
            out.append((rel, 1, "missing include guard"))
    return out


def lint_code_objects() -> List[Finding]:
    """Disassemble every built gfx950 code object and apply SCALAR_STORE to the
    instruction stream (the sources may be clean while the compiler is not)."""
    import glob
    import subprocess
    import tempfile
    out: List[Finding] = []
    objs = sorted(glob.glob(os.path.join(ROOT, "build", "obj", "gpu", "*.hip.o")))
    if not objs or not all(os.path.exists(t) for t in (OBJDUMP, BUNDLER, OBJCOPY)):
        return out
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            rel = os.path.relpath(obj, ROOT)
            dev = os.path.join(tmp, os.path.basename(obj) + ".gfx950")
            fatbin = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
            # hipcc -c embeds the offload bundle in the host object's .hip_fatbin section.
            subprocess.run([OBJCOPY, "--dump-section", ".hip_fatbin=" + fatbin, obj,
                            os.path.join(tmp, "host.o")], capture_output=True)
            if not os.path.exists(fatbin):
                out.append((rel, 1, "no .hip_fatbin section to disassemble"))
                continue
            r = subprocess.run([BUNDLER, "--type=o", "--input=" + fatbin, "--output=" + dev,
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--unbundle"],
                               capture_output=True, text=True)
            if r.returncode != 0 or not os.path.exists(dev):
                out.append((rel, 1, "no gfx950 code object in the offload bundle"))
                continue
            d = subprocess.run([OBJDUMP, "-d", dev], capture_output=True, text=True)
            for i, line in enumerate(d.stdout.split("\n"), 1):
                if SCALAR_STORE.search(line):
                    out.append((rel, i, "scalar-cache store / atomic in disassembly"))
    return out


def lint_py(path: str) -> List[Finding]:
    out: List[Finding] = []
    rel = os.path.relpath(path, ROOT)
    with open(path, encoding="utf-8") as f:
        text = f.read()
    try:
        tree = ast.parse(text, filename=rel)
    except SyntaxError as e:
        return [(rel, e.lineno or 0, f"syntax error: {e.msg}")]
    for i, line in enumerate(text.split("\n"), 1):
        if len(line) > 110:
            out.append((rel, i, f"line longer than 110 ({len(line)})"))
        if "\t" in line:
            out.append((rel, i, "tab character"))
    for node in ast.walk(tree):
        if isinstance(node, ast.ExceptHandler) and node.type is None:
            out.append((rel, node.lineno, "bare except"))
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Attribute):
            owner = getattr(node.func.value, "id", "")
            if owner == "pickle" and node.func.attr in ("load", "loads"):
                out.append((rel, node.lineno, "pickle deserialisation"))
            if owner == "yaml" and node.func.attr == "load":
                kw = {k.arg for k in node.keywords}
                if "Loader" not in kw and len(node.args) < 2:
                    out.append((rel, node.lineno, "yaml.load without a SafeLoader"))
    return out


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    findings: List[Finding] = []
    ncpp = npy = 0
    for p in _walk(CPP_DIRS, CPP_EXT):
        ncpp += 1
        findings += lint_cpp(p)
    findings += lint_code_objects()
    py_files = list(_walk(PY_DIRS, (".py",)))
    py_files += [os.path.join(ROOT, f) for f in os.listdir(ROOT) if f.endswith(".py")]
    for p in py_files:
        npy += 1
        findings += lint_py(p)
    for rel, line, msg in findings:
        print(f"{rel}:{line}: {msg}")
    if "--quiet" not in argv:
        print(f"lint: {ncpp} C++/HIP files, {npy} Python files, {len(findings)} finding(s)")
    return 1 if findings else 0


if __name__ == "__main__":
    sys.exit(main())
