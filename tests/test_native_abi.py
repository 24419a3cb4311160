"""CPU-side checks of the C-ABI library: it builds, loads, exports every declared symbol, and
its host-only helpers agree with the reference's fixtures.  No GPU compute here."""
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "zeroclone.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"\b(zc_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def L():
    from zeroclone_amd import _native
    return _native.lib()


def test_every_declared_symbol_is_exported(L):
    from zeroclone_amd import _native
    syms = declared_symbols()
    assert len(syms) >= 15
    bound = {name for name, _, _ in _native.SIGNATURES}
    for s in syms:
        assert hasattr(L, s), s
        assert s in bound, f"{s} declared in zeroclone.h but not bound in _native.SIGNATURES"


def test_version(L):
    assert b"gfx950" in L.zc_version()


def test_legal_order_table_matches_cpython(golden):
    from zeroclone_amd import _native
    order = golden("c4_set_order.json")["order"]
    for mask in range(128):
        assert _native.c4_legal_order(mask) == order[str(mask)]
        live = [m[0] for m in list({(i, 0) for i in range(7) if (mask >> i) & 1})]
        assert _native.c4_legal_order(mask) == live


def test_rows_roundtrip(golden):
    from zeroclone_amd import _native
    import ctypes
    for c in golden("c4_backend.json")["cases"][:100]:
        st = _native.c4_from_rows(c["board"], c["turn"])
        s = _native.C4State()
        s.stones[0] = int(st["stones"][0])
        s.stones[1] = int(st["stones"][1])
        s.turn = int(st["turn"])
        buf = ctypes.create_string_buffer(42)
        assert _native.lib().zc_c4_to_rows(ctypes.byref(s), buf) == 0
        back = buf.raw.decode().replace(" ", ".")
        assert back == c["board"]
        # bitboard legal mask == reference legal set
        occ = int(st["stones"][0]) | int(st["stones"][1])
        mask = sum(1 << col for col in range(7) if not (occ >> (7 * col + 5)) & 1)
        assert _native.c4_legal_order(mask) == c["legal"]


def test_invalid_arguments_fail_loudly(L):
    from zeroclone_amd import _native
    with pytest.raises(ValueError):
        _native.c4_from_rows("." * 42, 2)
    with pytest.raises(ValueError):
        _native.c4_legal_order(128)
