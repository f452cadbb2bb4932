"""CPU: deterministic generators, CSR packing, mask geometry."""
import numpy as np

from sequencealigning_amd import synth
from sequencealigning_amd.nw import alignment_rows, pack_csr


def test_splitmix64_matches_oracle(oracle):
    import ctypes
    L = oracle.lib()
    L.ref_splitmix64.restype = ctypes.c_uint64
    st = ctypes.c_uint64(0x5EED0002)
    ref = [L.ref_splitmix64(ctypes.byref(st)) for _ in range(16)]
    assert synth.splitmix64(0x5EED0002, 16).tolist() == ref


def test_iid_pairs_shape_and_determinism():
    a = synth.iid_pairs(10, 150, 150, seed=1)
    b = synth.iid_pairs(10, 150, 150, seed=1)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    q, qo, d, do = a
    assert len(q) == 1500 and qo[-1] == 1500 and set(q.tobytes()) <= set(b"ACGT")


def test_mutate_rate():
    q, d = synth.mut_pair(20000, 0.05, 7)
    assert len(q) == 20000
    assert abs(len(d) - len(q)) < 400
    assert set(d) <= set(b"ACGT")


def test_pack_csr():
    buf, off = pack_csr([b"AC", b"", b"GGT"])
    assert off.tolist() == [0, 2, 2, 5]
    assert buf.tobytes() == b"ACGGT"


def test_alignment_rows():
    assert alignment_rows(b"AAA", b"AA", [(1, "="), (1, "I"), (1, "=")]) == ("AAA", "| |", "A-A")
