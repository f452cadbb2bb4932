"""CPU: the engine's tuning options (saln_option_set, include/saln.h) — the
only way to change what it runs (it reads no environment variable).  Loading
the library needs no GPU; these calls touch no device.  (Per-context
overrides need a context, i.e. a device: tests/test_nw_gpu.py.)"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_options_table_matches_header(saln):
    from sequencealigning_amd import _lib
    names = _lib.option_names()
    hdr = open(os.path.join(ROOT, "include", "saln.h")).read()
    block = hdr[hdr.index("Tuning knobs (kernel geometry"):hdr.index("int saln_option_set")]
    assert sorted(re.findall(r'"([a-z0-9_.]+)"', block)) == sorted(names)
    assert len(names) == len(set(names)) >= 15


def test_option_set_get_reset(saln):
    from sequencealigning_amd import _lib
    for nm in _lib.option_names():
        v, d = _lib.get_option(nm)
        assert v == d, nm  # defaults at start (no other test leaves one set)
    _lib.set_option("nw.spec_passes", 5)
    assert _lib.get_option("nw.spec_passes") == (5, 3)
    assert _lib.non_default_options() == {"nw.spec_passes": 5}
    with _lib.options(**{"nw.spec_passes": 7, "nw.pk_tab": 0}):
        assert _lib.get_option("nw.spec_passes")[0] == 7 and _lib.get_option("nw.pk_tab")[0] == 0
    assert _lib.get_option("nw.spec_passes")[0] == 5 and _lib.get_option("nw.pk_tab")[0] == 3
    assert _lib.lib().saln_options_reset() == 0
    assert _lib.non_default_options() == {}


def test_option_errors(saln):
    from sequencealigning_amd import _lib
    with pytest.raises(_lib.SalnError):
        _lib.set_option("nw.no_such_option", 1)
    with pytest.raises(_lib.SalnError):
        _lib.set_option("nw.rows_k", 9)  # out of range
    assert _lib.get_option("nw.rows_k")[0] == 0


def test_engine_reads_no_environment():
    """No getenv in the engine's sources (the product path)."""
    csrc = os.path.join(ROOT, "sequencealigning_amd", "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".cpp", ".hpp", ".hip", ".h")):
            assert "getenv" not in open(os.path.join(csrc, f)).read(), f


def test_pruned_options_are_gone(saln):
    """Round 5 removed the A/B switches that lost or changed nothing
    (VERDICT r4 #5): they are unknown names now."""
    from sequencealigning_amd import _lib
    for nm in ("nw.pk_steady", "nw.tb_chunks", "nw.fill_lds_min", "nw.nib_codes",
               "nw.narrow_walk", "nw.rows_wpg", "nw.walk_prio"):
        with pytest.raises(_lib.SalnError):
            _lib.set_option(nm, 1)


def test_no_experiment_macros_in_product():
    """No SALN_* preprocessor switches in the kernels (A/B builds belong in
    tools/)."""
    src = open(os.path.join(ROOT, "sequencealigning_amd", "csrc", "nw_kernels.hip")).read()
    assert not re.findall(r"#\s*(?:ifndef|ifdef|if)\s+SALN_", src)

