"""CPU: the C-ABI library loads, exports every entry point include/saln.h
declares, and refuses to compute without a gfx950 device (no CPU path)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "saln.h")).read()
    return sorted(set(re.findall(r"\b(saln_[a-z0-9_]+)\s*\(", src)))


def test_header_matches_exports(saln):
    from sequencealigning_amd import _lib
    names = _declared()
    assert set(names) == set(_lib.EXPORTS)
    L = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(L, n), n


def test_nm_exports_are_extern_c(saln):
    from sequencealigning_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for n in _declared():
        assert n in syms, n


def test_abi_version(saln):
    from sequencealigning_amd import _lib
    assert _lib.lib().saln_abi_version() == 1


def test_no_cpu_fallback(saln):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from sequencealigning_amd import _lib
    with pytest.raises(_lib.SalnError, match="E_NO_DEVICE"):
        saln.n_w_align(b"AC", b"AC")


def test_struct_sizes(saln):
    from sequencealigning_amd import _lib
    assert ctypes.sizeof(_lib.NwResult) == 16
    assert ctypes.sizeof(_lib.NwScoring) == 16
    assert ctypes.sizeof(_lib.WfaResult) == 32


def test_cli_help():
    cli = os.path.join(ROOT, "sequencealigning_amd", "saln")
    r = subprocess.run([cli, "--help"], capture_output=True, text=True)
    assert r.returncode == 0
    assert "--query-file" in r.stdout and "--algo" in r.stdout


def test_avsa_launch_geometry_fits_32bit_grid(saln):
    """Every packed all-vs-all class launches at most a 32-bit work-item
    count per chunk (nw_avsa.cpp: the chunk derives from the class's pairs
    per block); pure host logic, no device needed."""
    from sequencealigning_amd import _lib
    L = _lib.lib()
    for v in (4, 5, 6, 7, 8):
        chunk, blocks = ctypes.c_uint64(), ctypes.c_uint64()
        assert L.saln_nw_avsa_launch_geometry(v, ctypes.byref(chunk), ctypes.byref(blocks)) == 0
        assert blocks.value * 256 <= 0xFFFFFFFF, v
        assert chunk.value >= 1 << 24 and chunk.value <= 1 << 31, v
    for v in (-1, 0, 3, 9):
        assert L.saln_nw_avsa_launch_geometry(v, None, None) == _lib.E_INVALID


def test_status_codes_match_header():
    src = open(os.path.join(ROOT, "include", "saln.h")).read()
    from sequencealigning_amd import _lib
    assert re.search(r"SALN_E_DEVICE_WAIT = (-\d+)", src).group(1) == str(_lib.E_DEVICE_WAIT)
    assert re.search(r"SALN_FLAG_WAIT_TIMEOUT (\d+)u", src).group(1) == str(_lib.FLAG_WAIT_TIMEOUT)
