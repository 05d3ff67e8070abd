"""The C ABI (include/phx.h): the gfx950 library and the test emulation export every symbol."""
import os
import re
import subprocess

import pytest

import mpisppy_amd  # noqa: F401
from mpisppy_amd import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "phx.h")).read()
    return sorted(set(re.findall(r"\b(phx_[a-z_0-9]+)\s*\(", src)))


def exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_header_lists_symbols():
    fns = header_functions()
    assert set("phx_" + s for s in _native.SYMBOLS) == set(fns)


def test_gfx950_library_exports_header():
    from mpisppy_amd import build
    path = build.build_phx(verbose=False)
    syms = exported(path)
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing


def test_gfx950_code_object():
    """libphx.so carries a gfx950 code object (cross-compiled here)."""
    path = _native.LIB_PATH
    data = open(path, "rb").read()
    assert b"gfx950" in data


def test_emulation_exports_header(emu):
    syms = exported(emu.path)
    missing = ["emu_" + f for f in header_functions() if "emu_" + f not in syms]
    assert not missing, missing


def test_product_has_no_cpu_fallback(monkeypatch):
    """Without a GPU the engine refuses to run (no silent CPU path)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    opts = {"solver_name": "phx", "PHIterLimit": 1, "defaultPHrho": 1, "convthresh": 0, "verbose": False,
            "display_progress": False, "iter0_solver_options": {}, "iterk_solver_options": {}}
    with pytest.raises(_native.NativeError):
        PH(opts, ["scen0", "scen1"], farmer.scenario_creator)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_native.NativeError):
        _native.Lib(str(tmp_path / "nope.so"))
