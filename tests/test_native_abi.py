"""The ctypes signatures in ops/_lib.py must match the C ABI of csrc/*.hip (arity), so a GPU run
never dies on an argument-count mismatch."""
import glob
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c_arity():
    out = {}
    for path in glob.glob(os.path.join(ROOT, "csrc", "*.hip")):
        src = open(path).read()
        for m in re.finditer(r"TDL_API\s+(?:\w+\s+)+?(tdl_\w+)\s*\(([^)]*)\)", src):
            args = [a for a in m.group(2).split(",") if a.strip()]
            out[m.group(1)] = len(args)
    return out


def test_signatures_match_c_sources():
    from trustworthy_dl.ops._lib import _SIGNATURES
    arity = _c_arity()
    assert arity, "no TDL_API entry points found"
    for name, argtypes in _SIGNATURES.items():
        assert name in arity, f"{name} declared in _lib but not exported by csrc"
        assert len(argtypes) == arity[name], f"{name}: python {len(argtypes)} args vs C {arity[name]}"
