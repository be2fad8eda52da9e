"""CPU checks of the C-ABI library: it loads, exports every function include/blokus_engine.h
declares, and its host-side action tables equal the oracle's (no device calls)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from oracle.oracle import Oracle


def header_functions():
    with open(os.path.join(ROOT, "include", "blokus_engine.h"), encoding="utf-8") as f:
        txt = f.read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(bk_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_header():
    from blokus_rl_amd import engine
    lib = engine.load_library()
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n
    # and the binding declares exactly the header's functions
    assert sorted(engine.exported_symbols()) == names


@pytest.mark.parametrize("preset", [(20, 4, 5), (7, 2, 4), (7, 2, 5)])
def test_host_tables_equal_oracle(preset):
    from blokus_rl_amd.engine import host_tables
    tab, cells = host_tables(*preset)
    o = Oracle(*preset)
    assert (tab == o.action_table()).all()
    assert (cells == o.action_cells()).all()


def test_device_calls_fail_loudly_on_host_only_context():
    from blokus_rl_amd import engine
    lib = engine.load_library()
    h = ctypes.c_void_p()
    assert lib.bk_ctx_create(20, 4, 5, -1, ctypes.byref(h)) == 0
    rc = lib.bk_init_states(h, ctypes.c_void_p(0x1000), 1, None)
    assert rc == -1 and b"host-only" in lib.bk_last_error()
    assert lib.bk_ctx_create(21, 4, 5, -1, ctypes.byref(h)) == -1
    lib.bk_ctx_destroy(h)


def test_engine_refuses_without_gpu():
    import torch
    from blokus_rl_amd.engine import Engine, EngineError
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(EngineError):
        Engine(20, 4, 5)
