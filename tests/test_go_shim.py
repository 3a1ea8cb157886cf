"""CPU: a static check of the Go cgo shim (noise-erasurecode-plugin_amd/go/
infectious/fec.go) against the C ABI it binds.

The image has no Go toolchain, so the shim -- the package `main.go:24` would
import instead of github.com/vivint/infectious -- is never compiled here
("missing" #3).  What can be checked without Go: every C
function the shim calls is declared in include/rsmi.h or include/rsmi_wire.h
and exported by lib/librsmi.so, each call passes as many arguments as the
prototype has parameters, every C type and constant it names is declared,
and the exported Go API keeps infectious's names (NewFEC, Encode, Decode,
Share, DeepCopy, Required, Total).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "noise-erasurecode-plugin_amd", "go", "infectious", "fec.go")
HEADERS = [os.path.join(ROOT, "include", "rsmi.h"), os.path.join(ROOT, "include", "rsmi_wire.h")]
LIB = os.path.join(ROOT, "noise-erasurecode-plugin_amd", "lib", "librsmi.so")


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", " ", re.sub(r"//[^\n]*", " ", s), flags=re.S)


def _split_args(s):
    """Top-level comma split of an argument list (parentheses, brackets and
    braces nest)."""
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        if ch == "," and depth == 0:
            out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur)
    return [a.strip() for a in out]


def _c_prototypes():
    protos = {}
    for h in HEADERS:
        text = _strip_c_comments(open(h).read())
        for m in re.finditer(r"\b(rs_\w+)\s*\(([^;{}]*?)\)\s*;", text):
            params = _split_args(m.group(2))
            protos[m.group(1)] = 0 if params in ([], ["void"]) else len(params)
    return protos


def _c_names():
    text = "".join(_strip_c_comments(open(h).read()) for h in HEADERS)
    return set(re.findall(r"\b(rs_\w+|RS_\w+)\b", text))


def _go_calls():
    """(name, argument count) of every C.rs_*(...) call in the shim."""
    src = open(GO).read()
    calls = []
    for m in re.finditer(r"\bC\.(rs_\w+)\(", src):
        i, depth = m.end(), 1
        while depth:
            depth += {"(": 1, ")": -1}.get(src[i], 0)
            i += 1
        calls.append((m.group(1), len(_split_args(src[m.end():i - 1]))))
    return calls


def test_go_shim_calls_match_c_prototypes():
    protos = _c_prototypes()
    calls = _go_calls()
    assert len(calls) >= 10
    for name, nargs in calls:
        assert name in protos, f"fec.go calls C.{name}, not declared in include/"
        assert nargs == protos[name], f"C.{name}: {nargs} arguments in fec.go, {protos[name]} in the header"


def test_go_shim_names_declared_c_types_and_constants():
    names = _c_names()
    used = set(re.findall(r"\bC\.((?:rs|RS)_\w+)\b", open(GO).read()))
    missing = sorted(used - names)
    assert not missing, missing


def test_go_shim_symbols_exported_by_the_engine():
    if not os.path.exists(LIB):
        pytest.skip("lib/librsmi.so not built")
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rs_\w+)", out))
    for name, _ in _go_calls():
        assert name in exported, f"C.{name} is not exported by librsmi.so"


def test_go_shim_keeps_infectious_api_names():
    """The names main.go uses (main.go:57-69, 73, 77, 248, 254-262)."""
    src = open(GO).read()
    assert re.search(r"^package infectious\b", src, flags=re.M)
    for pat in (r"func NewFEC\(k, n int\) \(\*FEC, error\)",
                r"func \(f \*FEC\) Encode\(input \[\]byte, output func\(Share\)\) error",
                r"func \(f \*FEC\) Decode\(dst \[\]byte, shares \[\]Share\) \(\[\]byte, error\)",
                r"type Share struct", r"func \(s \*?Share\) DeepCopy\(\)",
                r"func \(f \*FEC\) Required\(\) int", r"func \(f \*FEC\) Total\(\) int"):
        assert re.search(pat, src), pat


def test_go_shim_exposes_device_sets():
    """NewFECOnDevices: the plugin process spans several
    GPUs through one device-set context; NewFEC honours RSMI_DEVICES so the
    unchanged plugin can too."""
    src = open(GO).read()
    assert re.search(r"func NewFECOnDevices\(k, n int, devices \[\]int\) \(\*FEC, error\)", src)
    assert "C.rs_new_devices(" in src and "RSMI_DEVICES" in src
    assert re.search(r"func \(f \*FEC\) Close\(\)", src)

