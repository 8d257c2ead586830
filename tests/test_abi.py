"""The C-ABI library loads and exports every function include/*.h declares
(no compute calls: runs without a GPU)."""
import ctypes as C
import os
import re

import ccsx_amd as cx
from ccsx_amd.native import EXPORTS, LIB_PATH

INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")


def _declared(header: str) -> set[str]:
    text = open(os.path.join(INC, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\([^;{]*\)\s*;", text, flags=re.M))
    return {n for n in names if n not in ("if", "while", "for", "return", "sizeof")}


def test_library_loads():
    assert os.path.exists(LIB_PATH)
    cx.lib()


def test_headers_match_export_table():
    for h, names in EXPORTS.items():
        assert _declared(h) == set(names), h


def test_every_declared_symbol_exported():
    dll = C.CDLL(LIB_PATH)
    for h in sorted(os.listdir(INC)):
        if not h.endswith(".h"):
            continue
        for name in _declared(h):
            assert hasattr(dll, name), f"{h}: {name} not exported"


def test_no_oracle_symbols_in_product():
    dll = C.CDLL(LIB_PATH)
    for name in ("opoa_init", "ocsx_zmw", "ocsx_batch"):
        assert not hasattr(dll, name)
