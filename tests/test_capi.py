"""C-ABI checks that need no GPU: the library loads, exports every symbol the header
declares, and the ctypes signature table matches the header prototypes."""
import ctypes
import os
import re

import pytest

import pcms_amd  # noqa: F401  (registers the package)
from pcms_amd import _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "pcms_hip.h")


def _prototypes():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"\bint\s+(pcms_\w+)\s*\(([^)]*)\)\s*;", src):
        protos[m.group(1)] = [a.strip() for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
    return protos


def _code(arg: str) -> str:
    if arg == "hipStream_t s":
        return "s"
    if "*" in arg:
        return "p"
    t = arg.rsplit(" ", 1)[0].replace("const ", "").strip()
    return {"int": "i", "long": "l", "double": "d", "float": "f"}[t]


def test_header_matches_ctypes_table():
    protos = _prototypes()
    assert set(protos) == set(_lib.SIGNATURES), set(protos) ^ set(_lib.SIGNATURES)
    for name, args in protos.items():
        assert "".join(_code(a) for a in args) == _lib.SIGNATURES[name], name


def test_library_loads_and_exports_every_symbol():
    lib = _lib.load()
    for name in _prototypes():
        assert isinstance(getattr(lib, name), ctypes._CFuncPtr), name


def test_host_queries_without_gpu():
    assert _lib.query("pcms_conv3_chunk", _lib.BF16) == 32
    assert _lib.query("pcms_conv3_chunk", _lib.F32) == 8      # bf16x6: 8 fp32 channels per chunk
    assert _lib.query("pcms_conv3_chunk", _lib.F32X3) == 16
    # pack elements (activation dtype): bf16 32 per (chunk, tap, row); fp32 x6: 48 bf16 per
    # 8 channels = 24 floats; x3: 32 bf16 per 16 channels = 16 floats
    assert _lib.query("pcms_conv3_pack_elems", _lib.BF16, 64, 64) == 2 * 27 * 64 * 32
    assert _lib.query("pcms_conv3_pack_elems", _lib.F32, 64, 64) == 8 * 27 * 64 * 24
    assert _lib.query("pcms_conv3_pack_elems", _lib.F32X3, 64, 5) == 1 * 27 * 64 * 16
    assert _lib.query("pcms_conv3_mblocks", 2, 128, 128, 64) == 2 * 16 * 16 * 8
    assert _lib.query("pcms_loss_rows", 1 << 20) > 0
